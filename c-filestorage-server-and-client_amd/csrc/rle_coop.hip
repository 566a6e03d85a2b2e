// rle_coop.hip — cooperative batch kernels for small buffers: one workgroup per buffer, one wave
// per tile, the cross-tile state exchanged through LDS.
//
// The one-wave-per-buffer kernels (rle_kernels.hip) walk a buffer's tiles in sequence, so a batch
// of few small buffers (configs[1]: 4096 x 4 KiB, 4-5 tiles each) gives each SIMD only 4 waves
// whose tile steps are long dependent chains, and the SIMDs sit idle much of the time (DESIGN.md
// §4, "Cooperative small-buffer kernels").  Here every tile of a buffer is its own wave, and the
// sequential state of the reference's scan (src/rleCompression.c:9-62) crosses tiles in two
// barrier-separated exchanges:
//   decode  1. each wave: its tile's token-phase map                -> LDS; barrier
//           2. entry phase = composition of the earlier tiles' maps; decoded length -> LDS; barrier
//           3. scatter into one staging for the whole buffer at the prefix offset; barrier
//           4. all waves fill and store the buffer's 16-byte output chunks
//   encode  1. each wave: the last run boundary of its tile          -> LDS; barrier
//           2. entry run start = max over the earlier tiles; token masks; compressed size -> LDS;
//              barrier
//           3. passes 1 and 2 into one staging at the prefix offset; barrier; all waves store it.
// The tile steps are the one-wave kernels' (rle_device.h: enc_analyze_bounds / enc_tokens /
// enc_pass1, dec_prepare / dec_lengths / dec_scatter / dec_fill_*), so the output is the same
// bytes.  A buffer with more tiles than the workgroup has waves (or, decode, more decoded bytes
// than its staging) is walked by wave 0 alone with the one-wave tile loop; streams the tiled path
// declines take the exact serial decoder, as there.
#include "rle_coop_limits.h"
#include "rle_device.h"
#include "rle_service.h"

#include <stdlib.h>
#include <string.h>

#include <atomic>


namespace rle {

static_assert(kCoopMaxWaves * kEncStep * kCoopEncRounds == kCoopEncMaxBytes &&
              kCoopMaxWaves * kTileStep * kCoopDecRounds == kCoopDecMaxIn, "rle_coop_limits.h");

__device__ __forceinline__ u32 coop_wave() { return uniform(threadIdx.x / kWave); }

// Completion-flag launches (put_status): every wave waits for its stores' acknowledgements (they
// are in the XCD's L2, or past it) before the barrier behind which thread 0 releases them all at
// system scope (one L2 write-back, in put_status) and stores the status.  All waves still running
// reach the barrier (the waves without a tile ended before the first one).
__device__ __forceinline__ void coop_release(u32 flags) {
    if (flags & kLaunchFlag) {
        vm_drain();
        __syncthreads();
    }
}

// ================================================================ ENCODE
// kW waves; 1024-byte tiles (enc_tile<true> form), so buffers of up to 1024 kW kR bytes are coop:
// kR rounds of kW tiles, round r + 1's tiles loading (into the slots round r has read) while round
// r writes its staging; the run start and output offset entering a round are carried from the last.
// One buffer (b: its index in out_len / status).  kU (the resident small-call service,
// rle_service.hip, whose workgroup serves one buffer after another): no wave ends before the last
// barrier -- the waves without a tile idle through the barriers -- and all of them share the stores.
template <u32 kW, bool kU, u32 kR = 1>
__device__ __forceinline__ void enc_coop_body(const uint8_t* src, uint8_t* dst, uint64_t U64,
                                              uint64_t* __restrict__ out_len, uint32_t* __restrict__ status, u32 b,
                                              u32 wt) {
    static_assert(kR == 1u || !kU, "the service serves one round");
    constexpr u32 kUmax = kEncStep * kW * kR;
    // output position r at byte 16 + r (chunk 0: guard of the non-starts' back-writes); +32: the
    // writes of positions past U land at the output end
    constexpr u32 kStageC = 16u + kUmax + kUmax / 2u + 32u;
    constexpr u32 kStage = ((kStageC > kEncStage ? kStageC : kEncStage) + 127u) & ~127u;
    __shared__ __attribute__((aligned(16))) uint8_t slots[kW * kEncSlot];
    __shared__ __attribute__((aligned(128))) uint8_t stage[kStage];
    __shared__ u32 xch[2 * kW];   // [0, kW) last run boundary per tile, [kW, 2kW) compressed size
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = coop_wave();
    u32 bad = (((uintptr_t)src | (uintptr_t)dst) & 15u) ? RLE_STATUS_MISALIGNED : 0u;
    if (U64 > kMaxBufferBytes) bad |= RLE_STATUS_TOOLARGE;
    if (bad) {
        if (threadIdx.x == 0) {
            out_len[b] = 0;
            put_status(status, b, bad, wt);
        }
        return;
    }
    const u32 U = (u32)U64;
    const u32x4 rsi = make_rsrc(src, (U + 15u) & ~15u);
    const u32x4 rso = make_rsrc(dst, U + U / 2u);
    const EncK kc = enc_k();
    const u32 ntiles = enc_ntiles_for(U);
    if (ntiles > kW * kR) {   // too long for the rounds: wave 0 walks it like encode_kernel
        if (wid != 0u) return;
        EncState st{0u, 0u, 0u, 0u, 0u, (wt & kLaunchWt) != 0u, {}};
        if (U <= 16384u)   // rle_kernels.hip kEncSmall
            walk_tiles<kEncStep, true>(rsi, 0u, enc_ntiles_for(U), lane, slots, [&](u32 t, const uint8_t* cs, const Refill& nx) {
                return enc_tile<true>(cs, nx, t * kEncStep, U, U, lane, stage, dst, rso, st, kc);
            });
        else
            walk_tiles(rsi, 0u, ntiles_for(U), lane, slots, [&](u32 t, const uint8_t* cs, const Refill& nx) {
                return enc_tile<false>(cs, nx, t * kTileStep, U, U, lane, stage, dst, rso, st, kc);
            });
        if (lane < st.out_pos - st.flushed) dst[st.flushed + lane] = stage[16u + lane];
        if (lane == 0) {
            out_len[b] = st.out_pos;
            put_status(status, b, RLE_STATUS_OK, wt);
        }
        return;
    }
    // waves with a tile in the first round (wave 0 also for U = 0)
    const u32 nact = ntiles == 0u ? 1u : (ntiles < kW ? ntiles : kW);
    if (!kU && wid >= nact) return;   // ended waves do not hold up s_barrier
    const u32 nrounds = kR == 1u || ntiles == 0u ? 1u : (ntiles + kW - 1u) / kW;
    const uint8_t* slot = slots + wid * kEncSlot;
    asm volatile("s_nop 4" ::: "memory");   // descriptor words may be fresh (walk_prime)
    if (wid < ntiles) Refill{rsi, kEncStep * wid + 16u * lane, uniform(lds_addr(slot)), true, lane == 0u}();
    u32 rs_c = 0u, O_c = 0u, top_c = 0u;   // carried into the round: run start, output offset, last byte
    for (u32 r = 0; r < nrounds; ++r) {
        const u32 t = r * kW + wid;
        const bool act = t < ntiles;
        const u32 rtiles = ntiles - r * kW < kW ? ntiles - r * kW : kW;   // tiles of this round
        vm_drain();
        __syncthreads();   // the round's tiles have landed (and the last round's staging is written)
        EncAn an{};
        if (act) {
            const u32x4 cur = *reinterpret_cast<const u32x4*>(slot + 16u * lane);
            const uint2 look = *reinterpret_cast<const uint2*>(slot + kSlot);
            // the input byte before the tile: the previous tile's last byte
            const u32 prev_top = wid ? *reinterpret_cast<const u32*>(slot - kEncSlot + kSlot - 4u) & 0xFF000000u : top_c;
            an = enc_analyze_bounds<true>(cur, look, kEncStep * t, U, U, lane, prev_top, kc);
            const u32 ilast = readlane(an.incl, kWave - 1u);   // last run boundary in the tile (0: none)
            if (lane == 0) xch[wid] = ilast;
        }
        if (kR > 1u && r + 1u < nrounds)   // (the round is full: slot kW - 1 holds its last tile)
            top_c = *reinterpret_cast<const u32*>(slots + (kW - 1u) * kEncSlot + kSlot - 4u) & 0xFF000000u;
        __syncthreads();   // every slot read: the next round's tiles may land
        if (kR > 1u && t + kW < ntiles) Refill{rsi, kEncStep * (t + kW) + 16u * lane, uniform(lds_addr(slot)), true, lane == 0u}();
        u32 nout = 0u, oincl = 0u;
        if (act) {
            u32 rs = rs_c;   // start of the run holding the byte before the tile
            for (u32 s = 0; s < wid; ++s) rs = xch[s] > rs ? xch[s] : rs;
            enc_tokens(an, rs);
            nout = bcnt(an.P, bcnt(an.P, bcnt(an.T, 0u)));
            oincl = wave_scan_incl(nout, 0u, OpAdd());
            if (lane == 0) xch[kW + wid] = readlane(oincl, kWave - 1u);
        }
        __syncthreads();
        u32 O = O_c, rtot = 0u, rmax = rs_c;
        for (u32 s = 0; s < rtiles; ++s) {
            const u32 c = xch[kW + s];
            O += s < wid ? c : 0u;
            rtot += c;
            rmax = xch[s] > rmax ? xch[s] : rmax;
        }
        if (act) {
            const u32* w = an.w;
            const u32 T = an.T, P = an.P, B24 = an.B24, validm = an.validm;
            const u32 NS = validm & ~T;
            const u32 e0 = lds_addr(stage) + 16u + O + oincl - nout;
            if (kEncStep * t + kEncStep <= U) enc_pass1<true>(w, T, P, NS, e0, kc.V01);
            else enc_pass1<false>(w, T, P, NS, e0, 0u);
            // pass 2 (enc_tile): count digits, and second bytes whose position is the buffer's end
            const u32 obase = 16u + O + oincl - nout;
            u32 prem = P;
            while (__builtin_amdgcn_ballot_w64(prem != 0u)) {
                if (prem) {
                    const u32 j = (u32)__builtin_ctz(prem);
                    prem &= prem - 1u;
                    const u32 mj = lowmask(j);
                    const u32 oj = bcnt(P & mj, bcnt(P & mj, bcnt(T & mj, obase)));
                    stage[oj + 2u] = (uint8_t)('1' + (u32)__builtin_ctz((B24 >> (j + 1u)) | 0x100u));
                }
            }
            const u32 vnext = (validm >> 1) | ((from_next_lane(validm, 0u) & 1u) << 15);
            const u32 PX = P & ~vnext;
            if (__builtin_amdgcn_ballot_w64(PX != 0u)) {
                if (PX) {
                    const u32 j = (u32)__builtin_ctz(PX);
                    const u32 mj = lowmask(j);
                    const u32 oj = bcnt(P & mj, bcnt(P & mj, bcnt(T & mj, obase)));
                    const u32 wj = j < 4u ? w[0] : j < 8u ? w[1] : j < 12u ? w[2] : w[3];
                    stage[oj + 1u] = (uint8_t)(wj >> (8u * (j & 3u)));
                }
            }
        }
        O_c += rtot;
        rs_c = rmax;
    }
    __syncthreads();
    // store: whole 16-byte chunks, then the final partial chunk byte by byte (nothing past C)
    const u32 total = O_c;
    const u32 nthr = kWave * (kU ? kW : nact), t = threadIdx.x, nfull = total >> 4;
    for (u32 c = t; c < nfull; c += nthr)
        vstore(rso, 16u * c, *reinterpret_cast<const u32x4*>(stage + 16u + 16u * c), (wt & kLaunchWt) != 0u);
    if (t < (total & 15u)) dst[16u * nfull + t] = stage[16u + 16u * nfull + t];
    coop_release(wt);
    if (t == 0) {
        out_len[b] = total;
        put_status(status, b, RLE_STATUS_OK, wt);
    }
}
template <u32 kW, u32 kR = 1>
__global__ __launch_bounds__(kWave* kW) void enc_coop_kernel(const uint8_t* __restrict__ in,
                                                             const uint64_t* __restrict__ in_off,
                                                             const uint64_t* __restrict__ in_len,
                                                             uint8_t* __restrict__ out,
                                                             const uint64_t* __restrict__ out_off,
                                                             uint64_t* __restrict__ out_len,
                                                             uint32_t* __restrict__ status, uint32_t n, uint32_t wt) {
    const u32 b = blockIdx.x;
    if (b >= n) return;
    enc_coop_body<kW, false, kR>(in + in_off[b], out + out_off[b], in_len[b], out_len, status, b, wt);
}

// ---------------------------------------------------------------- encode, any size, one pass
// (round 5, measured no faster than the segmented encode on 1 MiB buffers and slower on zero-filled
// ones, DESIGN.md §4: in the RLE_VARIANTS test library only)
#if RLE_VARIANTS
// One workgroup of kW waves walks a whole buffer in rounds of kW tiles (enc_coop_body's rounds),
// reading each input byte once: a round's output is staged, its whole 16-byte chunks stored, and
// the partial chunk carried to the staging's front for the next round.  The staging holds one
// round's output (at most 1.5 x 1024 kW bytes) past the carried chunk, so any buffer size fits.
// Thread 0 stores chunk 0 and then moves the partial chunk onto it (no other thread reads chunk 0
// or writes the partial chunk in that phase), so a round has four barriers.
template <u32 kW>
__device__ __forceinline__ void enc_stream_body(const uint8_t* src, uint8_t* dst, uint64_t U64,
                                                uint64_t* __restrict__ out_len, uint32_t* __restrict__ status, u32 b,
                                                u32 wt) {
    constexpr u32 kRoundOut = kEncStep * kW + kEncStep * kW / 2u;
    constexpr u32 kStage = (16u + 16u + kRoundOut + 32u + 127u) & ~127u;
    __shared__ __attribute__((aligned(16))) uint8_t slots[kW * kEncSlot];
    __shared__ __attribute__((aligned(128))) uint8_t stage[kStage];
    __shared__ u32 xch[2 * kW];
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = coop_wave();
    u32 bad = (((uintptr_t)src | (uintptr_t)dst) & 15u) ? RLE_STATUS_MISALIGNED : 0u;
    if (U64 > kMaxBufferBytes) bad |= RLE_STATUS_TOOLARGE;
    if (bad) {
        if (threadIdx.x == 0) {
            out_len[b] = 0;
            put_status(status, b, bad, wt);
        }
        return;
    }
    const u32 U = (u32)U64;
    const u32x4 rsi = make_rsrc(src, (U + 15u) & ~15u);
    const u32x4 rso = make_rsrc(dst, U + U / 2u);
    const EncK kc = enc_k();
    const bool wtb = (wt & kLaunchWt) != 0u;
    const u32 ntiles = enc_ntiles_for(U);
    const u32 nact = ntiles == 0u ? 1u : (ntiles < kW ? ntiles : kW);
    if (wid >= nact) return;   // ended waves do not hold up s_barrier
    const u32 nthr = kWave * nact;
    const u32 nrounds = ntiles == 0u ? 1u : (ntiles + kW - 1u) / kW;
    const uint8_t* slot = slots + wid * kEncSlot;
    asm volatile("s_nop 4" ::: "memory");   // descriptor words may be fresh (walk_prime)
    if (wid < ntiles) Refill{rsi, kEncStep * wid + 16u * lane, uniform(lds_addr(slot)), true, lane == 0u}();
    // carried: run start, output offset, last input byte; base = output offset of staging byte 16
    u32 rs_c = 0u, O_c = 0u, top_c = 0u, base = 0u;
    u32 nst = 0u;   // store instructions this wave issued after the round's tile loads (the last round)
    for (u32 r = 0; r < nrounds; ++r) {
        const u32 t = r * kW + wid;
        const bool act = t < ntiles;
        const u32 rtiles = ntiles - r * kW < kW ? ntiles - r * kW : kW;
        vm_wait_deep(nst);   // the tile loads, not the stores issued after them (vmcnt is in order)
        __syncthreads();   // the round's tiles have landed; the carried chunk is in place
        EncAn an{};
        if (act) {
            const u32x4 cur = *reinterpret_cast<const u32x4*>(slot + 16u * lane);
            const uint2 look = *reinterpret_cast<const uint2*>(slot + kSlot);
            const u32 prev_top = wid ? *reinterpret_cast<const u32*>(slot - kEncSlot + kSlot - 4u) & 0xFF000000u : top_c;
            an = enc_analyze_bounds<true>(cur, look, kEncStep * t, U, U, lane, prev_top, kc);
            if (lane == 0) xch[wid] = readlane(an.incl, kWave - 1u);
        }
        if (r + 1u < nrounds)
            top_c = *reinterpret_cast<const u32*>(slots + (kW - 1u) * kEncSlot + kSlot - 4u) & 0xFF000000u;
        __syncthreads();   // every slot read: the next round's tiles may land
        if (t + kW < ntiles) Refill{rsi, kEncStep * (t + kW) + 16u * lane, uniform(lds_addr(slot)), true, lane == 0u}();
        u32 nout = 0u, oincl = 0u;
        if (act) {
            u32 rs = rs_c;
            for (u32 s = 0; s < wid; ++s) rs = xch[s] > rs ? xch[s] : rs;
            enc_tokens(an, rs);
            nout = bcnt(an.P, bcnt(an.P, bcnt(an.T, 0u)));
            oincl = wave_scan_incl(nout, 0u, OpAdd());
            if (lane == 0) xch[kW + wid] = readlane(oincl, kWave - 1u);
        }
        __syncthreads();
        u32 O = O_c, rtot = 0u, rmax = rs_c;
        for (u32 s = 0; s < rtiles; ++s) {
            const u32 c = xch[kW + s];
            O += s < wid ? c : 0u;
            rtot += c;
            rmax = xch[s] > rmax ? xch[s] : rmax;
        }
        if (act) {
            const u32* w = an.w;
            const u32 T = an.T, P = an.P, B24 = an.B24, validm = an.validm;
            const u32 NS = validm & ~T;
            const u32 obase = 16u + (O - base) + oincl - nout;
            const u32 e0 = lds_addr(stage) + obase;
            if (kEncStep * t + kEncStep <= U) enc_pass1<true>(w, T, P, NS, e0, kc.V01);
            else enc_pass1<false>(w, T, P, NS, e0, 0u);
            u32 prem = P;
            while (__builtin_amdgcn_ballot_w64(prem != 0u)) {
                if (prem) {
                    const u32 j = (u32)__builtin_ctz(prem);
                    prem &= prem - 1u;
                    const u32 mj = lowmask(j);
                    const u32 oj = bcnt(P & mj, bcnt(P & mj, bcnt(T & mj, obase)));
                    stage[oj + 2u] = (uint8_t)('1' + (u32)__builtin_ctz((B24 >> (j + 1u)) | 0x100u));
                }
            }
            const u32 vnext = (validm >> 1) | ((from_next_lane(validm, 0u) & 1u) << 15);
            const u32 PX = P & ~vnext;
            if (__builtin_amdgcn_ballot_w64(PX != 0u)) {
                if (PX) {
                    const u32 j = (u32)__builtin_ctz(PX);
                    const u32 mj = lowmask(j);
                    const u32 oj = bcnt(P & mj, bcnt(P & mj, bcnt(T & mj, obase)));
                    const u32 wj = j < 4u ? w[0] : j < 8u ? w[1] : j < 12u ? w[2] : w[3];
                    stage[oj + 1u] = (uint8_t)(wj >> (8u * (j & 3u)));
                }
            }
        }
        O_c += rtot;
        rs_c = rmax;
        __syncthreads();   // the round's output is staged
        // whole chunks of [base, O_c) out; the partial one to the front (thread 0, after chunk 0)
        const u32 nfull = (O_c - base) >> 4;
        for (u32 c = threadIdx.x; c < nfull; c += nthr)
            vstore(rso, base + 16u * c, *reinterpret_cast<const u32x4*>(stage + 16u + 16u * c), wtb);
        if (threadIdx.x == 0u && nfull)
            *reinterpret_cast<u32x4*>(stage + 16u) = *reinterpret_cast<const u32x4*>(stage + 16u + 16u * nfull);
        base += 16u * nfull;
        const u32 w0 = kWave * wid;
        nst = uniform(nfull > w0 ? (nfull - w0 + nthr - 1u) / nthr : 0u);
    }
    __syncthreads();
    const u32 total = O_c;
    if (threadIdx.x < total - base) dst[base + threadIdx.x] = stage[16u + threadIdx.x];
    coop_release(wt);
    if (threadIdx.x == 0) {
        out_len[b] = total;
        put_status(status, b, RLE_STATUS_OK, wt);
    }
}
template <u32 kW>
__global__ __launch_bounds__(kWave* kW) void enc_stream_kernel(const uint8_t* __restrict__ in,
                                                               const uint64_t* __restrict__ in_off,
                                                               const uint64_t* __restrict__ in_len,
                                                               uint8_t* __restrict__ out,
                                                               const uint64_t* __restrict__ out_off,
                                                               uint64_t* __restrict__ out_len,
                                                               uint32_t* __restrict__ status, uint32_t n, uint32_t wt) {
    const u32 b = blockIdx.x;
    if (b >= n) return;
    enc_stream_body<kW>(in + in_off[b], out + out_off[b], in_len[b], out_len, status, b, wt);
}
#endif  // RLE_VARIANTS (one-pass encode)

// ================================================================ DECODE
// kW waves (tiles of 1008 bytes: dec_tile's geometry); buffers decoding to at most kUmax bytes from
// at most kR kW tiles: kR rounds of kW tiles as in enc_coop_body, the token phase and output offset
// carried across rounds, every round scattering into the one staging; then the fill and the stores.
// One buffer (b: its index in status; kU as enc_coop_body).
template <u32 kW, u32 kUmax, bool kU, u32 kR = 1>
__device__ __forceinline__ void dec_coop_body(const uint8_t* src, uint8_t* dst, uint64_t C64, uint64_t U64,
                                              uint64_t cap, uint32_t* __restrict__ status, u32 b, u32 wt) {
    // decoded position r at u16 16 + r (dec_tile's staging, one for the whole buffer); the one-wave
    // fallback needs kDecStage
    constexpr u32 kStageC = 2u * (16u + kUmax + 32u);
    constexpr u32 kStage = ((kStageC > kDecStage ? kStageC : kDecStage) + 127u) & ~127u;
    static_assert(kR == 1u || !kU, "the service serves one round");
    constexpr u32 kChunks = (kUmax + 15u) / 16u;
    constexpr u32 kSlotsB = (kW > 2u ? kW : 2u) * kSlot;
    // the fill's chunk-to-chunk bytes: in the slots (free by then) when they fit, which keeps the
    // 64 KiB staging within the CU's LDS
    constexpr bool kLastInSlots = 4u * kChunks <= kSlotsB && kUmax > 32768u;
    __shared__ __attribute__((aligned(16))) uint8_t slots[kSlotsB];
    __shared__ __attribute__((aligned(128))) uint8_t stage[kStage];
    __shared__ DecEntry tbl[256];
    __shared__ u32 xch[4 * kW];   // per tile: phase map, decoded length, serial, tail byte
    __shared__ u32 lastb_own[kLastInSlots ? 1u : kChunks + 1u];
    u32* const lastb = kLastInSlots ? reinterpret_cast<u32*>(slots) : lastb_own;
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = coop_wave();
    for (u32 i = threadIdx.x; i < 256u; i += kWave * kW) tbl[i] = dec_entry_from(kDecTable.e[i]);
    u32 bad = ((((uintptr_t)src | (uintptr_t)dst) & 15u) || cap < U64) ? RLE_STATUS_MISALIGNED : 0u;
    if (C64 > kMaxBufferBytes || U64 > kMaxBufferBytes) bad |= RLE_STATUS_TOOLARGE;
    if (bad) {
        if (threadIdx.x == 0) put_status(status, b, bad, wt);
        return;
    }
    const u32 C = (u32)C64, U = (u32)U64;
    const u32x4 rsi = make_rsrc(src, (C + 15u) & ~15u);
    const u32x4 rso = make_rsrc(dst, U);
    const u32 ntiles = ntiles_for(C);
    const DecK kc = dec_k();
    __syncthreads();   // the phase table is complete
    if (ntiles > kW * kR || U > kUmax) {   // wave 0 walks it like decode_kernel
        if (wid != 0u) return;
        walk_prime(rsi, 0u, ntiles, lane, slots);
        for (u32 k = lane; k < kDecStage / 16u; k += kWave) reinterpret_cast<u32x4*>(stage)[k] = u32x4{0u, 0u, 0u, 0u};
        wave_lds_sync();
        DecState st{0u, 0u, 0u, 0u, 0u, 0u, 0u, (wt & kLaunchWt) != 0u, {}};
        const bool serial = walk_tiles(
            rsi, 0u, ntiles, lane, slots,
            [&](u32 t, const uint8_t* cs, const Refill& nx) { return dec_tile(cs, nx, t * kTileStep, C, C, U, lane, tbl, stage, dst, rso, st, kc); },
            true);
        u32 stat;
        if (serial) stat = dec_serial(src, C, U, cap, dst, lane, stage);
        else {
            dec_finish(st, U, lane, stage, rso, dst);
            stat = dec_tiled_status(st, U);
        }
        if (lane == 0) put_status(status, b, stat, wt);
        return;
    }
    // waves with a tile in the first round (wave 0 also for C = 0)
    const u32 nact = ntiles == 0u ? 1u : (ntiles < kW ? ntiles : kW);
    if (!kU && wid >= nact) return;   // ended waves do not hold up s_barrier
    const u32 nthr = kWave * (kU ? kW : nact);   // threads zeroing, filling and storing
    const u32 nrounds = kR == 1u || ntiles == 0u ? 1u : (ntiles + kW - 1u) / kW;
    const uint8_t* slot = slots + wid * kSlot;
    asm volatile("s_nop 4" ::: "memory");   // descriptor words may be fresh (walk_prime)
    if (wid < ntiles) dma_tile(rsi, kTileStep * wid + 16u * lane, uniform(lds_addr(slot)));
    // the staging positions this buffer can reach: [0, 16 + U + 17) u16
    const u32 nz = (2u * (16u + U + 17u) + 15u) / 16u;
    for (u32 k = threadIdx.x; k < nz; k += nthr) reinterpret_cast<u32x4*>(stage)[k] = u32x4{0u, 0u, 0u, 0u};
    u32 d_c = 0u, O_c = 0u, tail = 0u;   // carried into the round: token phase, output offset, tail byte
    for (u32 r = 0; r < nrounds; ++r) {
        const u32 t = r * kW + wid;
        const bool act = t < ntiles;
        const u32 rtiles = ntiles - r * kW < kW ? ntiles - r * kW : kW;   // tiles of this round
        vm_drain();
        __syncthreads();   // tiles landed; table and zeroed staging visible; the last round scattered
        DecPrep pr{};
        if (act) {
            const u32x4 cur = *reinterpret_cast<const u32x4*>(slot + 16u * lane);
            pr = dec_prepare(cur, kTileStep * t, C, C, lane, tbl, kc);
            if (lane == 0) xch[wid] = readlane(pr.incl, kOwnLanes - 1u);   // the tile's phase map
        }
        __syncthreads();   // every slot read: the next round's tiles may land
        if (kR > 1u && t + kW < ntiles) dma_tile(rsi, kTileStep * (t + kW) + 16u * lane, uniform(lds_addr(slot)));
        DecLen ln{};
        u32 oincl = 0u;
        if (act) {
            u32 d = d_c;   // token phase entering the tile
            for (u32 s = 0; s < wid; ++s) d = bfe(xch[s], 8u * d, 8);
            ln = dec_lengths(pr, d);
            oincl = wave_scan_incl(ln.nout, 0u, OpAdd());
            constexpr uint64_t kOwned = (1ull << kOwnLanes) - 1ull;
            const bool serial = (__builtin_amdgcn_ballot_w64(ln.serial_lane) & kOwned) != 0ull;
            u32 tailv = 0u;
            if (pr.tail) {
                const uint64_t pfb = __builtin_amdgcn_ballot_w64(ln.PF != 0u) & kOwned;
                if (pfb) {   // the final token's byte extends to U
                    const u32 jf = (u32)__builtin_ctz(ln.PF | 0x10000u) & 15u;
                    const u32* w = pr.w;
                    const u32 wf = jf < 4u ? w[0] : jf < 8u ? w[1] : jf < 12u ? w[2] : w[3];
                    tailv = 0x100u | readlane(bfe(wf, 8u * (jf & 3u), 8), (u32)__builtin_ctzll(pfb));
                }
            }
            if (lane == 0) {
                xch[kW + wid] = readlane(oincl, kOwnLanes - 1u);
                xch[2 * kW + wid] = serial ? 1u : 0u;
                xch[3 * kW + wid] = tailv;
            }
        }
        __syncthreads();
        u32 O = O_c, rtot = 0u, serial = 0u, d_next = d_c;
        for (u32 s = 0; s < rtiles; ++s) {
            const u32 c = xch[kW + s];
            O += s < wid ? c : 0u;
            rtot += c;
            serial |= xch[2 * kW + s];
            tail |= xch[3 * kW + s];
            d_next = bfe(xch[s], 8u * d_next, 8);
        }
        if (serial || O_c + rtot > U) {   // not encoder output: the exact serial decoder (dec_tile declines)
            vm_drain();   // (the next round's tiles: nothing lands in the LDS after the workgroup)
            if (wid == 0u) {
                const u32 stat = dec_serial(src, C, U, cap, dst, lane, stage);
                if (lane == 0) put_status(status, b, stat, wt);
            }
            return;
        }
        if (act && lane < kOwnLanes && !(RLE_ABL & 2)) dec_scatter(ln, pr.w, lds_addr(stage) + 2u * (16u + O + oincl - ln.nout));
        O_c += rtot;
        d_c = d_next;
    }
    const u32 total = O_c;
    __syncthreads();
    // output chunk q (bytes [16q, 16q + 16)) = staging chunk q + 1: decoded positions below total,
    // then the tail byte (zero unless the stream ends in an unbounded token); every chunk holds a
    // key, so the byte entering chunk q is chunk q - 1's last key (lastb, through LDS across waves)
    const u32 nq = (U + 15u) >> 4, tv = rep4(tail & 0xFFu);
    for (u32 q0 = 0; q0 < nq; q0 += nthr) {
        const u32 q = q0 + threadIdx.x;
        u32x4 a, c;
        dec_read_chunk(reinterpret_cast<const u32x4*>(stage + 32u * (q + 1u)), a, c);
        u32 L[8];
        dec_fill_scan(a, c, L);
        if (q < nq) lastb[q] = (L[7] >> 16) & 0xFFu;
        __syncthreads();
        if (q < nq) {
            const u32x4 f = dec_fill_out(L, q ? lastb[q - 1u] : 0u);
            const u32 fv[4] = {f.x, f.y, f.z, f.w};
            const u32 rel = 16u * q < total ? total - 16u * q : 0u;
            u32 ob[4];
#pragma unroll
            for (u32 k = 0; k < 4; ++k) {
                const u32 nb = rel > 4u * k ? (rel - 4u * k < 4u ? rel - 4u * k : 4u) : 0u;
                const u32 m = lowmask(8u * nb);
                ob[k] = (fv[k] & m) | (tv & ~m);
            }
            if (16u * q + 16u <= U) {
                vstore(rso, 16u * q, u32x4{ob[0], ob[1], ob[2], ob[3]}, (wt & kLaunchWt) != 0u);
            } else {
                for (u32 j = 0; 16u * q + j < U; ++j) dst[16u * q + j] = (uint8_t)(ob[j >> 2] >> (8u * (j & 3u)));
            }
        }
    }
    coop_release(wt);
    if (threadIdx.x == 0) put_status(status, b, total < U ? RLE_STATUS_SHORT : RLE_STATUS_OK, wt);
}
template <u32 kW, u32 kUmax, u32 kR = 1>
__global__ __launch_bounds__(kWave* kW) void dec_coop_kernel(const uint8_t* __restrict__ in,
                                                             const uint64_t* __restrict__ in_off,
                                                             const uint64_t* __restrict__ in_len,
                                                             uint8_t* __restrict__ out,
                                                             const uint64_t* __restrict__ out_off,
                                                             const uint64_t* __restrict__ out_len,
                                                             const uint64_t* __restrict__ out_cap,
                                                             uint32_t* __restrict__ status, uint32_t n, uint32_t wt) {
    const u32 b = blockIdx.x;
    if (b >= n) return;
    const uint64_t* capp = out_cap ? out_cap : out_len;
    dec_coop_body<kW, kUmax, false, kR>(in + in_off[b], out + out_off[b], in_len[b], out_len[b], capp[b], status, b, wt);
}

// One buffer whose sizes the host knows (the drop-in's zero-copy calls, round 6): the same bodies
// with the sizes and addresses as kernel arguments, so that the first tiles' loads do not wait for a
// read of the launch words over PCIe.
template <u32 kW, u32 kR = 1>
__global__ __launch_bounds__(kWave* kW) void enc_coop_one_kernel(const uint8_t* __restrict__ src,
                                                                 uint8_t* __restrict__ dst, uint64_t U,
                                                                 uint64_t* __restrict__ out_len,
                                                                 uint32_t* __restrict__ status, uint32_t wt) {
    enc_coop_body<kW, false, kR>(src, dst, U, out_len, status, 0u, wt);
}
template <u32 kW, u32 kUmax, u32 kR = 1>
__global__ __launch_bounds__(kWave* kW) void dec_coop_one_kernel(const uint8_t* __restrict__ src,
                                                                 uint8_t* __restrict__ dst, uint64_t C, uint64_t U,
                                                                 uint64_t cap, uint32_t* __restrict__ status,
                                                                 uint32_t wt) {
    dec_coop_body<kW, kUmax, false, kR>(src, dst, C, U, cap, status, 0u, wt);
}

#if RLE_VARIANTS   // the resident service is built into the test library only (round 5)
// ================================================================ resident small-call service
// (rle_service.h): one workgroup per drop-in thread context.  Wave 0 polls the context's mailbox
// line (lanes 0..15: one 64-byte read over PCIe with system-scope loads; an acquire fence once a
// request is seen);
// a new complete request (req != done, tail == req) is broadcast through LDS and served by all
// kSvcWaves waves with the barrier-uniform codec bodies on the context's mapped buffer; every wave
// waits for its stores, and after a barrier thread 0 releases them at system scope and stores the
// acknowledgement.  kSvcIdleUs after the last request, kSvcLifeUs after the launch, on the stop
// word, or after kSvcMaxPolls polls, thread 0 marks `gone` with the launch's generation and the
// workgroup ends.  Mailbox words are read only with vector loads (never the scalar cache).
constexpr u32 kSvcUmax = 16384;
constexpr u32 kSvcMaxPolls = 1u << 24;
__global__ __launch_bounds__(kWave* kSvcWaves) void svc_kernel(SvcMail* mb, const uint8_t* src, uint8_t* dst,
                                                              uint32_t gen, uint32_t done, uint64_t idle_ticks,
                                                              uint64_t life_ticks) {
    __shared__ u32 sh[8];   // 0: action (0 none, 1 serve, 2 exit); 1..7: words 1..7 of the line (7: tail = req)
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = coop_wave();
    const uint64_t t0 = wall_clock64();
    uint64_t last = t0;
    const uint32_t* line = reinterpret_cast<const uint32_t*>(&mb->r);
    for (u32 polls = 0;; ++polls) {
        if (wid == 0u) {
            const u32 w = lane < 16u ? __hip_atomic_load(line + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
            const u32 req = readlane(w, 0), tail = readlane(w, 7), stop = readlane(w, 6);
            const uint64_t now = wall_clock64();
            u32 act = 0u;
            u32 wl = w;
            if (req != done && tail == req) {
                // acquire once per request, not per poll (a system-scope acquire invalidates the
                // XCD's L2: per poll, 8 resident workgroups slowed every other's request, r4f)
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                act = 1u;
                last = now;
                // the line again, ordered after seeing its new sequence number: the host writes the
                // fields before `tail` and `req`, but the lanes' loads of one poll are not ordered
                // among themselves, so a field read by another lane may predate them
                wl = lane < 8u ? __hip_atomic_load(line + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
            } else if (stop || now - last > idle_ticks || now - t0 > life_ticks || polls > kSvcMaxPolls) {
                act = 2u;
            }
            if (lane < 8u) sh[lane] = lane == 0u ? act : wl;
            if (act == 1u) done = req;
        }
        __syncthreads();
        const u32 act = uniform(sh[0]);
        if (act == 2u) {
            if (threadIdx.x == 0) __hip_atomic_store(&mb->a.gone, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        if (act == 1u) {
            const u32 seq = uniform(sh[7]), op = uniform(sh[1]), in_len = uniform(sh[2]);
            const u32 out_len = uniform(sh[3]), cap = uniform(sh[4]), wt = uniform(sh[5]) & kLaunchWt;
            if (op == kSvcEncode) {
                enc_coop_body<kSvcWaves, true>(src, dst, in_len, &mb->a.res_len, &mb->a.status, 0u, wt);
            } else {
                dec_coop_body<kSvcWaves, kSvcUmax, true>(src, dst, in_len, out_len, cap, &mb->a.status, 0u, wt);
            }
            vm_drain();   // this wave's stores acknowledged (in the L2 or past it) ...
            __syncthreads();
            if (threadIdx.x == 0) {   // ... then one system-scope release of them all and the acknowledgement
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                __hip_atomic_store(&mb->a.ack, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else {
            __syncthreads();   // (wave 0 rewrites sh at the next poll)
            __builtin_amdgcn_s_sleep(2);
        }
    }
}
#endif  // RLE_VARIANTS

}  // namespace rle

// ================================================================ C-ABI launchers
namespace {
uint32_t coop_store_policy(uint32_t n) {
    // write-through for launches whose output fits in the L2s (rle_kernels.hip store_policy)
    static const int force = [] {
        const char* e = getenv("RLE_MI355X_STORE");
        return !e ? -1 : !strcmp(e, "wt") ? 1 : !strcmp(e, "wb") ? 0 : -1;
    }();
    return force >= 0 ? (uint32_t)force : (n <= 4096u ? 1u : 0u);
}
// Cooperative mode: 0 never, 1 always (when the sizes qualify), -1 (default) when the whole launch is
// resident at once.  Past one residency round the cooperative workgroups run in rounds, each paying
// a whole buffer's setup chain, and the one-wave kernels are faster (configs[1], 4096 x 4 KiB:
// decode 21.5 us cooperative vs 13.3 us one-wave; encode 11.9 vs 11.2).  The mode is read once from
// RLE_MI355X_COOP; tests switch it in-process with rle_mi355x_set_coop_mode (no setenv while other
// threads may read the environment).
std::atomic<int> g_coop_mode{[] {
    const char* e = getenv("RLE_MI355X_COOP");
    return e ? atoi(e) : -1;
}()};

// Residency of one cooperative instantiation: workgroups per CU from the occupancy API (its LDS,
// e.g. ~40-48 KB for dec_coop_kernel<W, 16384>, limits it well below the wave count), times the CUs
// of the current device.  Each (kernel, device) pair is queried once and kept in a per-instantiation
// atomic slot (value + 1; 0 = not queried yet), so the sized entry points -- every drop-in call of
// every server worker thread -- read it without a lock (round 4: the round-3 form took one
// process-wide mutex per launch).  Two threads racing on the first query both ask the API and store
// the same value.
constexpr int kResDevices = 64;
template <auto Kern>
uint64_t resident_blocks(uint32_t threads) {
    static std::atomic<uint64_t> slot[kResDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kResDevices) return 0;
    const uint64_t v = slot[dev].load(std::memory_order_relaxed);
    if (v) return v - 1u;
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)Kern, (int)threads, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
        (void)hipGetLastError();
        per_cu = cus = 0;
    }
    const uint64_t r = (uint64_t)(per_cu > 0 ? per_cu : 0) * (uint64_t)(cus > 0 ? cus : 0);
    slot[dev].store(r + 1u, std::memory_order_relaxed);
    return r;
}
template <auto Kern>
bool coop_admits(uint32_t threads, uint32_t n) {
    const int mode = g_coop_mode.load(std::memory_order_relaxed);
    return mode == 0 ? false : mode == 1 ? true : (uint64_t)n <= resident_blocks<Kern>(threads);
}
}  // namespace

// Cooperative launches (include/rle_mi355x.h *_sized): 1 if launched, 0 if the batch does not
// qualify (the caller then uses the one-wave kernels), < 0 on a launch error.
extern "C" int rle_encode_coop_launch(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len, void* d_out,
                                      const uint64_t* d_out_off, uint64_t* d_out_len, uint32_t* d_status, uint32_t n,
                                      uint64_t max_len, uint32_t flags, void* stream) {
    if (max_len > rle::kEncStep * rle::kCoopMaxWaves * rle::kCoopEncRounds || max_len <= rle::kEncStep) return 0;
    const uint32_t tiles = (uint32_t)((max_len + rle::kEncStep - 1) / rle::kEncStep);
    if (g_coop_mode.load(std::memory_order_relaxed) == 0) return 0;
    const hipStream_t s = (hipStream_t)stream;
    const uint32_t wt = coop_store_policy(n) | flags;
    const dim3 g(n);
#define RLE_ENC_COOP(W, R)                                                                                      \
    do {                                                                                                        \
        if (!coop_admits<rle::enc_coop_kernel<W, R>>(64 * W, n)) return 0;                                      \
        hipLaunchKernelGGL((rle::enc_coop_kernel<W, R>), g, dim3(64 * W), 0, s, (const uint8_t*)d_in, d_in_off, \
                           d_in_len, (uint8_t*)d_out, d_out_off, d_out_len, d_status, n, wt);                   \
    } while (0)
    if (tiles <= 2) RLE_ENC_COOP(2, 1);
    else if (tiles <= 3) RLE_ENC_COOP(3, 1);
    else if (tiles <= 4) RLE_ENC_COOP(4, 1);
    else if (tiles <= 6) RLE_ENC_COOP(6, 1);
    else if (tiles <= 8) RLE_ENC_COOP(8, 1);
    else if (tiles <= 12) RLE_ENC_COOP(12, 1);
    else if (tiles <= 16) RLE_ENC_COOP(16, 1);
    else if (tiles <= 32) RLE_ENC_COOP(16, 2);
    else RLE_ENC_COOP(16, 4);
#undef RLE_ENC_COOP
    return hipGetLastError() == hipSuccess ? 1 : RLE_E_HIP;
}

extern "C" int rle_decode_coop_launch(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len, void* d_out,
                                      const uint64_t* d_out_off, const uint64_t* d_out_len, const uint64_t* d_out_cap,
                                      uint32_t* d_status, uint32_t n, uint64_t max_in_len, uint64_t max_out_len,
                                      uint32_t flags, void* stream) {
    if (max_in_len > (uint64_t)rle::kTileStep * rle::kCoopMaxWaves * rle::kCoopDecRounds ||
        max_in_len <= rle::kTileStep || max_out_len > rle::kCoopDecUmax)
        return 0;
    const uint32_t tiles = (uint32_t)((max_in_len + rle::kTileStep - 1) / rle::kTileStep);
    if (g_coop_mode.load(std::memory_order_relaxed) == 0) return 0;
    const hipStream_t s = (hipStream_t)stream;
    const uint32_t wt = coop_store_policy(n) | flags;
    const dim3 g(n);
#define RLE_DEC_COOP_R(W, UM, R)                                                                                    \
    do {                                                                                                            \
        if (!coop_admits<rle::dec_coop_kernel<W, UM, R>>(64 * W, n)) return 0;                                      \
        hipLaunchKernelGGL((rle::dec_coop_kernel<W, UM, R>), g, dim3(64 * W), 0, s, (const uint8_t*)d_in, d_in_off, \
                           d_in_len, (uint8_t*)d_out, d_out_off, d_out_len, d_out_cap, d_status, n, wt);            \
    } while (0)
#define RLE_DEC_COOP(W, UM) RLE_DEC_COOP_R(W, UM, 1)
    if (max_out_len > 32768u) {   // 32-64 KiB: rounds of 16 tiles
        RLE_DEC_COOP_R(16, 65536, 5);
    } else if (max_out_len > 16384u) {
        if (tiles <= 4) RLE_DEC_COOP(4, 32768);
        else if (tiles <= 8) RLE_DEC_COOP(8, 32768);
        else if (tiles <= 16) RLE_DEC_COOP(16, 32768);
        else if (tiles <= 48) RLE_DEC_COOP_R(16, 32768, 3);
        else RLE_DEC_COOP_R(16, 32768, 4);   // (a worst-case 32 KiB stream: up to 49 tiles)
    } else if (tiles > 16) {   // (random 16 KiB: 17 tiles)
        RLE_DEC_COOP_R(16, 16384, 2);
    } else if (max_out_len <= 4096u) {
        if (tiles <= 2) RLE_DEC_COOP(2, 4096);
        else if (tiles <= 3) RLE_DEC_COOP(3, 4096);
        else if (tiles <= 5) RLE_DEC_COOP(5, 4096);
        else RLE_DEC_COOP(8, 4096);
    } else {
        if (tiles <= 2) RLE_DEC_COOP(2, 16384);
        else if (tiles <= 3) RLE_DEC_COOP(3, 16384);
        else if (tiles <= 5) RLE_DEC_COOP(5, 16384);
        else if (tiles <= 8) RLE_DEC_COOP(8, 16384);
        else if (tiles <= 12) RLE_DEC_COOP(12, 16384);
        else RLE_DEC_COOP(16, 16384);
    }
#undef RLE_DEC_COOP
#undef RLE_DEC_COOP_R
    return hipGetLastError() == hipSuccess ? 1 : RLE_E_HIP;
}

// One buffer with its sizes by value (csrc/rle_dropin.cpp's zero-copy calls): the same
// instantiations as the batched launches above choose for these sizes.  1 launched, 0 the buffer
// does not qualify (the caller launches the one-wave kernels), < 0 a launch error.
namespace {
bool coop_one_on() {   // (A/B) RLE_MI355X_COOP_ONE=0: the batched entry points for single calls too
    static const bool on = [] {
        const char* e = getenv("RLE_MI355X_COOP_ONE");
        return e ? atoi(e) != 0 : true;
    }();
    return on;
}
}  // namespace
extern "C" int rle_encode_coop_one(const void* src, void* dst, uint64_t U, uint64_t* d_out_len, uint32_t* d_status,
                                   uint32_t flags, void* stream) {
    if (!coop_one_on()) return 0;
    if (U > rle::kEncStep * rle::kCoopMaxWaves * rle::kCoopEncRounds || U <= rle::kEncStep) return 0;
    const uint32_t tiles = (uint32_t)((U + rle::kEncStep - 1) / rle::kEncStep);
    if (g_coop_mode.load(std::memory_order_relaxed) == 0) return 0;
    const hipStream_t s = (hipStream_t)stream;
    const uint32_t wt = coop_store_policy(1u) | flags;
#define RLE_ENC_ONE(W, R)                                                                                          \
    do {                                                                                                           \
        if (!coop_admits<rle::enc_coop_kernel<W, R>>(64 * W, 1u)) return 0;                                       \
        hipLaunchKernelGGL((rle::enc_coop_one_kernel<W, R>), dim3(1), dim3(64 * W), 0, s, (const uint8_t*)src,     \
                           (uint8_t*)dst, U, d_out_len, d_status, wt);                                             \
    } while (0)
    if (tiles <= 2) RLE_ENC_ONE(2, 1);
    else if (tiles <= 3) RLE_ENC_ONE(3, 1);
    else if (tiles <= 4) RLE_ENC_ONE(4, 1);
    else if (tiles <= 6) RLE_ENC_ONE(6, 1);
    else if (tiles <= 8) RLE_ENC_ONE(8, 1);
    else if (tiles <= 12) RLE_ENC_ONE(12, 1);
    else if (tiles <= 16) RLE_ENC_ONE(16, 1);
    else if (tiles <= 32) RLE_ENC_ONE(16, 2);
    else RLE_ENC_ONE(16, 4);
#undef RLE_ENC_ONE
    return hipGetLastError() == hipSuccess ? 1 : RLE_E_HIP;
}
extern "C" int rle_decode_coop_one(const void* src, void* dst, uint64_t C, uint64_t U, uint64_t cap, uint32_t* d_status,
                                   uint32_t flags, void* stream) {
    if (!coop_one_on()) return 0;
    if (C > (uint64_t)rle::kTileStep * rle::kCoopMaxWaves * rle::kCoopDecRounds || C <= rle::kTileStep ||
        U > rle::kCoopDecUmax)
        return 0;
    const uint32_t tiles = (uint32_t)((C + rle::kTileStep - 1) / rle::kTileStep);
    if (g_coop_mode.load(std::memory_order_relaxed) == 0) return 0;
    const hipStream_t s = (hipStream_t)stream;
    const uint32_t wt = coop_store_policy(1u) | flags;
#define RLE_DEC_ONE_R(W, UM, R)                                                                                   \
    do {                                                                                                          \
        if (!coop_admits<rle::dec_coop_kernel<W, UM, R>>(64 * W, 1u)) return 0;                                   \
        hipLaunchKernelGGL((rle::dec_coop_one_kernel<W, UM, R>), dim3(1), dim3(64 * W), 0, s, (const uint8_t*)src, \
                           (uint8_t*)dst, C, U, cap, d_status, wt);                                               \
    } while (0)
#define RLE_DEC_ONE(W, UM) RLE_DEC_ONE_R(W, UM, 1)
    if (U > 32768u) {   // 32-64 KiB: rounds of 16 tiles
        RLE_DEC_ONE_R(16, 65536, 5);
    } else if (U > 16384u) {
        if (tiles <= 4) RLE_DEC_ONE(4, 32768);
        else if (tiles <= 8) RLE_DEC_ONE(8, 32768);
        else if (tiles <= 16) RLE_DEC_ONE(16, 32768);
        else if (tiles <= 48) RLE_DEC_ONE_R(16, 32768, 3);
        else RLE_DEC_ONE_R(16, 32768, 4);
    } else if (tiles > 16) {
        RLE_DEC_ONE_R(16, 16384, 2);
    } else if (U <= 4096u) {
        if (tiles <= 2) RLE_DEC_ONE(2, 4096);
        else if (tiles <= 3) RLE_DEC_ONE(3, 4096);
        else if (tiles <= 5) RLE_DEC_ONE(5, 4096);
        else RLE_DEC_ONE(8, 4096);
    } else {
        if (tiles <= 2) RLE_DEC_ONE(2, 16384);
        else if (tiles <= 3) RLE_DEC_ONE(3, 16384);
        else if (tiles <= 5) RLE_DEC_ONE(5, 16384);
        else if (tiles <= 8) RLE_DEC_ONE(8, 16384);
        else if (tiles <= 12) RLE_DEC_ONE(12, 16384);
        else RLE_DEC_ONE(16, 16384);
    }
#undef RLE_DEC_ONE
#undef RLE_DEC_ONE_R
    return hipGetLastError() == hipSuccess ? 1 : RLE_E_HIP;
}

#if RLE_VARIANTS
namespace {
std::atomic<int> g_stream_waves{0};   // 0: from RLE_MI355X_STREAM_WAVES at the first launch
}
// Tests: waves per workgroup of the one-pass kernels (4, 8 or 16).
extern "C" int rle_mi355x_set_stream_waves(int w) {
    if (w != 4 && w != 8 && w != 16) return RLE_E_INVAL;
    g_stream_waves.store(w, std::memory_order_relaxed);
    return RLE_OK;
}
// One workgroup per buffer over the whole buffer (enc_stream_body), any size: RLE_OK if launched.
// RLE_MI355X_STREAM_WAVES (8 or 16, default 16): waves per workgroup.
extern "C" int rle_encode_stream_launch(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len, void* d_out,
                                        const uint64_t* d_out_off, uint64_t* d_out_len, uint32_t* d_status, uint32_t n,
                                        uint32_t flags, void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return RLE_E_INVAL;
    const hipStream_t s = (hipStream_t)stream;
    const uint32_t wt = coop_store_policy(n) | flags;
    if (g_stream_waves.load(std::memory_order_relaxed) == 0) {
        const char* e = getenv("RLE_MI355X_STREAM_WAVES");
        g_stream_waves.store(e && atoi(e) == 8 ? 8 : 16, std::memory_order_relaxed);
    }
    if (g_stream_waves.load(std::memory_order_relaxed) == 4)
        hipLaunchKernelGGL(rle::enc_stream_kernel<4>, dim3(n), dim3(64 * 4), 0, s, (const uint8_t*)d_in, d_in_off,
                           d_in_len, (uint8_t*)d_out, d_out_off, d_out_len, d_status, n, wt);
    else if (g_stream_waves.load(std::memory_order_relaxed) == 8)
        hipLaunchKernelGGL(rle::enc_stream_kernel<8>, dim3(n), dim3(64 * 8), 0, s, (const uint8_t*)d_in, d_in_off,
                           d_in_len, (uint8_t*)d_out, d_out_off, d_out_len, d_status, n, wt);
    else
        hipLaunchKernelGGL(rle::enc_stream_kernel<16>, dim3(n), dim3(64 * 16), 0, s, (const uint8_t*)d_in, d_in_off,
                           d_in_len, (uint8_t*)d_out, d_out_off, d_out_len, d_status, n, wt);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}
#endif

// Tests: switch the cooperative mode in-process (0 never, 1 always, -1 residency-gated default).
extern "C" int rle_mi355x_set_coop_mode(int mode) {
    if (mode < -1 || mode > 1) return RLE_E_INVAL;
    g_coop_mode.store(mode, std::memory_order_relaxed);
    return RLE_OK;
}

#if RLE_VARIANTS
// The resident small-call service of one drop-in thread context (rle_service.h; launched by
// csrc/rle_dropin.cpp svc_ensure): one workgroup of kSvcWaves waves on the given stream, serving
// requests on the context's mapped buffer (d_src: input, d_dst: output) from sequence `done` on.
extern "C" int rle_service_launch(void* d_mail, const void* d_src, void* d_dst, uint32_t gen, uint32_t done,
                                  void* stream) {
    if (!d_mail || !d_src || !d_dst) return RLE_E_INVAL;
    const uint64_t tick_per_us = 100;   // wall_clock64: 100 MHz
    hipLaunchKernelGGL(rle::svc_kernel, dim3(1), dim3(rle::kWave * rle::kSvcWaves), 0, (hipStream_t)stream,
                       (rle::SvcMail*)d_mail, (const uint8_t*)d_src, (uint8_t*)d_dst, gen, done,
                       tick_per_us * rle::kSvcIdleUs, tick_per_us * rle::kSvcLifeUs);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}
#endif  // RLE_VARIANTS
