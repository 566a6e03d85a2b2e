// rle_round.h — large-batch decode in rounds: one workgroup of kW waves per buffer, wave w
// decoding tiles w, w + kW, w + 2 kW, ... of it (round r: tiles r kW .. r kW + kW - 1).
//
// Why (profiles/r6a_pattern_variants.md): with one wave per buffer (decode_kernel) the waves in
// flight on a CU read 1 KiB tiles from as many unrelated streams, and the memory pattern alone
// (no token work) moves 0.634 of 8 TB/s on a dec64k-shaped batch; when the waves of a workgroup
// take consecutive tiles of one buffer, the same bytes move at 0.678 (4 waves) to 0.690 (8 waves),
// as fast as a plain grid-strided copy.  The reference's decoder is sequential
// (src/rleCompression.c:50-60: the token phase and the output position carry from token to token),
// so a round crosses its tiles' state through LDS with two barriers:
//   A  every wave: its tile's token-phase map (dec_prepare)                     -> LDS; barrier
//   B  entry phase = the carried phase through the earlier waves' maps; the tile's decoded length
//      from that phase (literal analysis, the uniform test, or dec_lengths)      -> LDS; barrier
//   C  output offset = the carried offset plus the earlier waves' lengths; the tile's bytes are
//      stored at it.
// Every wave writes exactly its own tile's bytes [O, O + len): its buffer descriptor starts at the
// tile's output offset and ends at its length, so the 16-byte stores (unaligned where O is) never
// reach a neighbour's bytes, and the last 1-3 bytes that a clipped 16-byte store drops go out as
// one dword or byte store.  No partial chunk crosses from tile to tile.  The tile steps are the
// one-wave kernel's (rle_device.h: dec_prepare, dec_lit_an, dec_uniform_tile, dec_lengths,
// dec_scatter, dec_flush), so the output is the same bytes; streams the tiled path declines take
// the exact serial decoder, as there.
// Included by rle_kernels.hip (after the issue order's slot map, order_slot_local), whose launcher
// (decode_launch) instantiates it.
#pragma once
#include "rle_device.h"

namespace rle {

// One byte per lane (buffer_store_byte: low byte of v).
__device__ __forceinline__ void vstore1(u32x4 rs, u32 voff, u32 v, bool wt) {
    if (wt)
        asm volatile("buffer_store_byte %0, %1, %2, 0 offen " RLE_WT_BITS "\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs) : "memory");
    else
        asm volatile("buffer_store_byte %0, %1, %2, 0 offen\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs) : "memory");
}

enum : u32 { kTileNone = 0u, kTileUni = 1u, kTileLit = 2u, kTileGen = 3u, kTileSv = 4u };

// Phase C, single-value tiles: ttot copies of v from the tile's output start (rso: based there,
// clipped at ttot).  Returns the store instructions issued.
__device__ __forceinline__ u32 round_fill(u32 v, u32 ttot, u32 lane, u32x4 rso, bool wt) {
    const u32 vv = rep4(v);
    const u32 nch = (ttot + 15u) >> 4;   // (the last one clipped to its whole dwords)
    const u32 rounds = (nch + kWave - 1u) / kWave;
    for (u32 k = 0; k < rounds; ++k) {
        const u32 c = k * kWave + lane;
        vstore(rso, c < nch ? 16u * c : kOOB, u32x4{vv, vv, vv, vv}, wt);
    }
    if ((ttot & 3u) && ttot >= 4u) {
        vstore4(rso, lane == 0u ? ttot - 4u : kOOB, vv, wt);
        return rounds + 1u;
    }
    if (ttot & 3u) {   // (a tile of fewer than 4 bytes: one byte per lane)
        vstore1(rso, lane < ttot ? lane : kOOB, v, wt);
        return rounds + 1u;
    }
    return rounds;
}

// Phase C, literal tiles (dec_lit_an's analysis f): each lane's kept bytes as one 16-byte store at
// its offset (the compaction of dec_tile_fast), clipped at ttot, then the tile's last 4 bytes as one dword ending at
// ttot (dec_tile_fast's tail form).  ttot >= 16.
__device__ __forceinline__ u32 round_lit(const DecPrep& pr, const DecLit& f, u32 lane, const u32x4* clut, u32x4 rso,
                                         u32 ttot, bool wt) {
    const u32* w = pr.w;
    const u32 dm = lane < kOwnLanes ? f.del : 0u;
    const u32 t1 = (u32)__builtin_ctz(dm | 0x10000u);
    const u32 t2 = (u32)__builtin_ctz((dm & (dm - 1u)) | 0x10000u);
    u32 y[4] = {w[0], w[1], w[2], w[3]};
    if (__builtin_amdgcn_ballot_w64(t2 < 16u)) {
        const u32x4 s2 = clut[t2];
        const u32 y3 = __builtin_amdgcn_perm(y[3], y[3], s2.w);
        y[0] = __builtin_amdgcn_perm(y[1], y[0], s2.x);
        y[1] = __builtin_amdgcn_perm(y[2], y[1], s2.y);
        y[2] = __builtin_amdgcn_perm(y[3], y[2], s2.z);
        y[3] = y3;
    }
    const u32x4 sel = clut[t1];
    u32x4 o;
    o.x = __builtin_amdgcn_perm(y[1], y[0], sel.x);
    o.y = __builtin_amdgcn_perm(y[2], y[1], sel.y);
    o.z = __builtin_amdgcn_perm(y[3], y[2], sel.z);
    const u32 c3 = __builtin_amdgcn_perm(y[3], y[3], sel.w);
    const u32 n0 = from_next_lane(o.x, 0u);
    const u32 kept = f.kept;
    const u32 s3 = kept >= 16u ? 0x03020100u : kept == 15u ? 0x04020100u : 0x05040100u;
    o.w = lane < kOwnLanes ? __builtin_amdgcn_perm(n0, c3, s3) : c3;
    vstore(rso, kept ? f.oexcl : kOOB, o, wt);
    // (the clipped stores drop the dwords that reach past ttot: their offsets are the lanes', not
    // multiples of 4, so up to 3 bytes are missing whatever ttot % 4 is)
    // the last 4 bytes of each lane's output: from its own bytes, or with fewer than 4 the previous
    // (full) lane's last bytes and its own
    const u32 s = kept - 4u, qd = s >> 2;
    const u32 lo = qd == 0u ? o.x : qd == 1u ? o.y : qd == 2u ? o.z : o.w;
    const u32 hi = qd == 0u ? o.y : qd == 1u ? o.z : o.w;
    const u32 T4 = alignbyte(hi, lo, s & 3u);
    const u32 Tp = from_prev_lane(T4, 0u);
    const u32 T = kept >= 4u ? T4 : alignbyte(o.x, Tp, kept);
    const uint64_t has = __builtin_amdgcn_ballot_w64(kept != 0u);
    const u32 last = 63u - (u32)__builtin_clzll(has);
    vstore4(rso, lane == last ? ttot - 4u : kOOB, T, wt);
    return 2u;
}

// Phase C, general tiles (dec_lengths ln, its inclusive lane scan oincl, total ttot): the scatter
// into the wave's staging from relative position 0 and the flush at relative offsets, in passes of
// at most kChunks chunks (dec_tile_pr_body's loop); the final partial chunk byte by byte.  The
// staging is all zero on entry and on return (chunk 0, the guard, aside).
template <u32 kChunks>
__device__ __forceinline__ u32 round_gen(const DecPrep& pr, const DecLen& ln, u32 oincl, u32 ttot, u32 lane,
                                         uint8_t* stage, u32x4 rso, bool wt) {
    constexpr uint64_t kOwned = (1ull << kOwnLanes) - 1ull;
    constexpr bool kOnePass = kChunks >= 191u;
    constexpr u32 kPassCap = 16u * kChunks - 17u;
    static_assert(kChunks >= 16u, "a pass must hold at least one lane's output (144 B)");
    const u32* w = pr.w;
    Stamps sp{};
    u32 rounds = 0, done = 0, from = 0, flushed = 0, fillc = 0, head = 0;
    for (;;) {
        const u32 rel0 = done - flushed;
        u32 upto = kOwnLanes, pass = ttot - done;
        if (!kOnePass && rel0 + pass > kPassCap) {
            const uint64_t fit = __builtin_amdgcn_ballot_w64(oincl <= done + kPassCap - rel0) & kOwned;
            upto = (u32)__builtin_popcountll(fit);
            pass = readlane(oincl, upto - 1u) - done;
        }
        const u32 endk = lds_addr(stage) + 2u * (16u + rel0 + oincl - done - ln.nout);
        if (lane < upto && lane >= from) dec_scatter(ln, w, endk);
        wave_lds_sync();
        const u32 newrel = rel0 + pass;
        const u32 nfl = newrel >> 4;
        rounds += dec_flush(wt, nfl, lane, stage, rso, flushed, fillc, head, nullptr, sp);
        if (nfl) {   // the partial chunk to staging chunk 1
            if (lane < 8u) {
                auto* from4 = reinterpret_cast<__attribute__((address_space(3))) u32*>(sswz(lds_addr(stage) + 32u * (nfl + 1u) + 4u * lane));
                auto* to4 = reinterpret_cast<__attribute__((address_space(3))) u32*>(sswz(lds_addr(stage) + 32u + 4u * lane));
                *to4 = *from4;
                *from4 = 0u;
            }
            wave_lds_sync();
        }
        flushed += 16u * nfl;
        done += pass;
        from = upto;
        if (upto >= kOwnLanes) break;
    }
    const u32 rel = ttot - flushed;   // < 16
    if (rel) {
        u32x4 a, b;
        dec_read_chunk(reinterpret_cast<const u32x4*>(stage + 32u), a, b);
        u32 L[8];
        dec_fill_scan(a, b, L);
        const u32x4 f = dec_fill_out(L, fillc);
        const u32 q = lane & 15u;
        const u32 wv = q < 4u ? f.x : q < 8u ? f.y : q < 12u ? f.z : f.w;
        vstore1(rso, lane < rel ? flushed + lane : kOOB, wv >> (8u * (q & 3u)), wt);
        ++rounds;
    }
    wave_lds_sync();
    if (lane < 8u)   // staging chunk 1 back to zero
        *reinterpret_cast<__attribute__((address_space(3))) u32*>(sswz(lds_addr(stage) + 32u + 4u * lane)) = 0u;
    wave_lds_sync();
    return rounds;
}


#ifndef RLE_ROUND_WPE   // waves per SIMD the register allocation must allow (7: <= 72 VGPRs, the
#define RLE_ROUND_WPE 7     // 7 four-wave workgroups per CU the LDS allows)
#endif
template <u32 kW, u32 kChunks, bool kWt>
__global__ __launch_bounds__(kWave* kW) __attribute__((amdgpu_waves_per_eu(RLE_ROUND_WPE))) void dec_round_kernel(const uint8_t* __restrict__ in,
                                                               const uint64_t* __restrict__ in_off,
                                                               const uint64_t* __restrict__ in_len,
                                                               uint8_t* __restrict__ out,
                                                               const uint64_t* __restrict__ out_off,
                                                               const uint64_t* __restrict__ out_len,
                                                               const uint64_t* __restrict__ out_cap,
                                                               uint32_t* __restrict__ status, uint32_t n, uint32_t flags,
                                                               const uint32_t* __restrict__ order) {
    constexpr u32 kStageB = 32u * kChunks;
    constexpr uint64_t kOwned = (1ull << kOwnLanes) - 1ull;
    __shared__ __attribute__((aligned(16))) uint8_t slots_all[kW * 2u * kSlot];
    __shared__ __attribute__((aligned(128))) uint8_t stage_all[kW * kStageB];
    __shared__ __attribute__((aligned(16))) DecEntry tbl[256];
    __shared__ u32x4 clut[kCompactEntries];
    // per round and wave: the tile's phase map; its decoded length (bits 0..15), serial bit 16, and
    // the final unbounded token's byte 0x100 | v at bits 20..28 (the stream's last tile only)
    constexpr u32 kX = kW < 4u ? 4u : kW;
    __shared__ __attribute__((aligned(16))) u32 xmap[kX];
    __shared__ __attribute__((aligned(16))) u32 xtf[kX];
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    // with an issue order (dec_order_local_kernel), workgroup s takes the buffer at its slot
    u32 b = blockIdx.x;
    if (order) b = b < n ? uniform(order[order_slot_local(b, n)]) : n;
    if (b >= n) return;
    const uint64_t* capp = out_cap ? out_cap : out_len;
    const uint64_t C64 = in_len[b], U64 = out_len[b], cap = capp[b], ioff = in_off[b], ooff = out_off[b];
    __builtin_amdgcn_sched_barrier(0);
    for (u32 k = threadIdx.x; k < 256u; k += kWave * kW) tbl[k] = dec_entry_from(kDecTable.e[k]);
    for (u32 k = threadIdx.x; k < kCompactEntries; k += kWave * kW)
        clut[k] = u32x4{kCompactLut.s[4u * k], kCompactLut.s[4u * k + 1u], kCompactLut.s[4u * k + 2u], kCompactLut.s[4u * k + 3u]};
    const uint8_t* src = in + ioff;
    uint8_t* dst = out + ooff;
    u32 bad = ((((uintptr_t)src | (uintptr_t)dst) & 15u) || cap < U64) ? RLE_STATUS_MISALIGNED : 0u;
    if (C64 > kMaxBufferBytes || U64 > kMaxBufferBytes) bad |= RLE_STATUS_TOOLARGE;
    if (bad) {
        if (threadIdx.x == 0) put_status(status, b, bad, flags);
        return;
    }
    const u32 C = (u32)C64, U = (u32)U64;
    const u32x4 rsi = make_rsrc(src, (C + 15u) & ~15u);
    const u32 ntiles = ntiles_for(C);
    const u32 nrounds = (ntiles + kW - 1u) / kW;
    uint8_t* stage = stage_all + wid * kStageB;
    const uint8_t* slots = slots_all + wid * 2u * kSlot;
    const u32 l0 = uniform(lds_addr(slots)), lo = 16u * lane;
    asm volatile("s_nop 4" ::: "memory");   // descriptor words may be fresh
    if (wid < ntiles) dma_tile<true>(rsi, kTileStep * wid + lo, l0);
    if (wid + kW < ntiles) dma_tile<true>(rsi, kTileStep * (wid + kW) + lo, l0 + kSlot);
    for (u32 k = lane; k < kStageB / 16u; k += kWave) reinterpret_cast<u32x4*>(stage)[k] = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();   // tables and zeroed staging visible
    const DecK kc = dec_k();
    u32 d_c = 0u, O_c = 0u, tailb = 0u;
    bool sv = false;
    u32 p1 = 0u, p2 = 0u;   // store instructions of this wave's last round and the one before
    for (u32 r = 0; r < nrounds; ++r) {
        const u32 t = r * kW + wid;
        const bool act = t < ntiles;
        const u32 rt = ntiles - r * kW < kW ? ntiles - r * kW : kW;   // tiles of this round
        const u32 pos = kTileStep * t;
        // ---- A: this wave's tile and its phase map
        // (ops issued after this tile's load: stores of round r-2, the load of round r+1, stores of r-1)
        if (act) vm_wait(p2 + (t + kW < ntiles ? 1u : 0u) + p1);
        p2 = p1;
        p1 = 0u;
        const uint8_t* cs = slots + (r & 1u) * kSlot;
        // (no initialisers: a wave without a tile never reads them, and zero-initialised structs
        // cost a move per field wherever the paths merge)
        u32x4 cur{0u, 0u, 0u, 0u};
        DecPrep pr{};
        if (act) {
            cur = *reinterpret_cast<const u32x4*>(cs + 16u * lane);
            if (t + 2u * kW < ntiles) dma_tile<true>(rsi, kTileStep * (t + 2u * kW) + lo, l0 + (r & 1u) * kSlot);
            pr = dec_prepare(cur, pos, C, C, lane, tbl, kc);
            const u32 m = readlane(pr.incl, kOwnLanes - 1u);
            if (lane == 0u) xmap[wid] = m;
        }
        __syncthreads();
        // ---- B: entry phase, then the tile's path and decoded length
        // (the round's maps on the scalar unit: one broadcast LDS read per 4 waves)
        u32 mp[kX];
#pragma unroll
        for (u32 q = 0; q < kX; q += 4u) {
            const u32x4 m4 = *reinterpret_cast<const u32x4*>(xmap + q);
            mp[q] = uniform(m4.x);
            mp[q + 1u] = uniform(m4.y);
            mp[q + 2u] = uniform(m4.z);
            mp[q + 3u] = uniform(m4.w);
        }
        u32 d = d_c, d_next = d_c;
#pragma unroll
        for (u32 q = 0; q < kW; ++q) {
            if (q == wid) d = d_next;
            if (q < rt) d_next = bfe(mp[q], 8u * d_next, 8);
        }
        u32 kind = kTileNone, ttot = 0u, v = 0u, oincl = 0u, tflag = 0u;
        DecLit lit{};
        DecLen ln{};
        if (act) {
            // (the uniform test after a single-value tile of the same wave, as dec_tile's gate)
            if (sv && pos + kSlot + 2u <= C && dec_uniform_tile(cur, lane, kc.LM3, d, v)) {
                kind = kTileUni;
                ttot = kUniformOut;
            }
            if (kind == kTileNone && !pr.tail) {
                const u32 NE16 = (pr.xa >> 7) | (pr.xb << 1);
                if (!(__builtin_amdgcn_ballot_w64(__builtin_popcount(~NE16 & 0xFFFFu) > 2) & kOwned)) {
                    lit = dec_lit_an(pr, lane, d);
                    if (!__builtin_amdgcn_ballot_w64(lit.reject) && lit.ttot >= 16u) {
                        kind = kTileLit;
                        ttot = lit.ttot;
                    }
                }
            }
            if (kind == kTileNone) {
                ln = dec_lengths(pr, d);
                oincl = wave_scan_incl(ln.nout, 0u, OpAdd());
                ttot = readlane(oincl, kOwnLanes - 1u);
                if (__builtin_amdgcn_ballot_w64(ln.serial_lane) & kOwned) tflag |= 1u << 16;
                if (pr.tail) {
                    const uint64_t pfb = __builtin_amdgcn_ballot_w64(ln.PF != 0u) & kOwned;
                    if (pfb) {   // the final token's byte extends to U
                        const u32 jf = (u32)__builtin_ctz(ln.PF | 0x10000u) & 15u;
                        const u32* w = pr.w;
                        const u32 wf = jf < 4u ? w[0] : jf < 8u ? w[1] : jf < 12u ? w[2] : w[3];
                        tflag |= (0x100u | readlane(bfe(wf, 8u * (jf & 3u), 8), (u32)__builtin_ctzll(pfb))) << 20;
                    }
                }
                kind = kTileGen;
                // a tile whose tokens all carry one byte (zero-filled data past the uniform test)
                if (7u * ttot >= 20u * (C - pos < kTileStep ? C - pos : kTileStep)) {
                    const u32 vt = (readlane(pr.w[0], 0) >> (8u * d)) & 0xFFu;
                    const u32 vv = rep4(vt);
                    u32 bd = 0;
#pragma unroll
                    for (u32 k = 0; k < 4; ++k) {
                        const u32 x = pr.w[k] ^ vv;
                        bd |= bitop3<kOrAnd>(faddi<0x7F7F7F7Fu>(x & kc.K7F), x, kc.K80) & ln.S80[k];
                    }
                    if (!(__builtin_amdgcn_ballot_w64(bd != 0u) & kOwned)) {
                        kind = kTileSv;
                        v = vt;
                    }
                }
            }
            if (lane == 0u) xtf[wid] = (ttot > 0xFFFFu ? 0xFFFFu | (1u << 16) : ttot) | tflag;
        }
        __syncthreads();
        // ---- C: output offset, then the tile's bytes
        u32 tf[kX];
#pragma unroll
        for (u32 q = 0; q < kX; q += 4u) {
            const u32x4 t4 = *reinterpret_cast<const u32x4*>(xtf + q);
            tf[q] = uniform(t4.x);
            tf[q + 1u] = uniform(t4.y);
            tf[q + 2u] = uniform(t4.z);
            tf[q + 3u] = uniform(t4.w);
        }
        u32 O = O_c, sum = 0u, anyser = 0u, last = 0u;
#pragma unroll
        for (u32 q = 0; q < kW; ++q) {
            if (q == wid) O = O_c + sum;
            if (q < rt) {
                sum += tf[q] & 0xFFFFu;
                anyser |= tf[q];
                last = tf[q];
            }
        }
        const bool serial = ((anyser >> 16) & 1u) || sum > U - O_c;
        if (serial) {   // not encoder output: the exact serial decoder, by wave 0 (every wave agrees)
            vm_drain();   // (tile loads still in flight: nothing lands in LDS after the workgroup; and
            __syncthreads();   // every tile store is acknowledged before wave 0 rewrites the output)
            if (wid == 0u) {
                const u32 stat = dec_serial(src, C, U, cap, dst, lane, stage, kStageB);
                if (lane == 0) put_status(status, b, stat, flags);
            }
            return;
        }
        if (act) {
            const u32x4 rso = make_rsrc(dst + O, ttot);
            asm volatile("s_nop 4" ::: "memory");   // (fresh descriptor words)
            if (kind == kTileUni || kind == kTileSv) p1 = round_fill(v, ttot, lane, rso, kWt);
            else if (kind == kTileLit) p1 = round_lit(pr, lit, lane, clut, rso, ttot, kWt);
            else p1 = round_gen<kChunks>(pr, ln, oincl, ttot, lane, stage, rso, kWt);
            sv = kind == kTileUni || kind == kTileSv;
        }
        tailb = last >> 20;   // (the stream's last tile: its final token's byte)
        d_c = d_next;
        O_c += sum;
    }
    // [total, U): the final unbounded token's byte (zeros without one); only streams that decode to
    // fewer than U bytes (status SHORT) or end in such a token get here with total < U
    const u32 total = O_c;
    if (total < U && wid == 0u) {
        const u32 tb = tailb & 0xFFu;
        for (u32 q = total + lane; q < U; q += kWave) dst[q] = (uint8_t)tb;
    }
    if (flags & kLaunchFlag) {   // completion flag: every wave's stores acknowledged, then released (put_status)
        vm_drain();
        __syncthreads();
    }
    if (threadIdx.x == 0) put_status(status, b, total < U ? RLE_STATUS_SHORT : RLE_STATUS_OK, flags);
}

}  // namespace rle
