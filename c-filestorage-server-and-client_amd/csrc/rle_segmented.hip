// rle_segmented.hip — the codec for LARGE buffers: several waves per buffer.
//
// A one-wave-per-buffer launch walks a buffer's tiles one after another, so a single big buffer
// (the drop-in's one-call-per-file path, src/filesystemApi.c:766-775, or the large end of a
// mixed batch) runs at one wave's speed.  Here every buffer is cut into segments of 4..16 tiles
// (1008 input bytes each; the launcher aims at ~16 segments per CU) that separate waves process.
// The only state crossing a segment boundary is
// (the algebra, checked against the oracle on CPU: tests/seg_model.py, tests/test_seg_model.py):
//   encode  the run phase entering the segment.  A segment summary holds the offset L0 of its
//           first run boundary, its last boundary lb, whether a boundary-free segment's run
//           continues past it, and the compressed bytes of the tokens from L0 on; a per-buffer
//           scan turns them into each segment's entering run start rs (a running max of lb) and
//           output offset (the entering piece's tokens have a closed form in L0 and the phase).
//   decode  the token phase entering the segment (0..2).  A segment summary holds, for each of
//           the three possible entry phases, the exit phase, the decoded byte count and whether
//           the tiled path would decline; the per-buffer scan composes the exit maps (v_perm
//           selectors, like the in-wave scan) and sums the counts of the phases actually taken.
// Five launches per direction: plan (segments per buffer, exclusive scan), map (each segment's
// buffer), summary (waves over all segments), scan (one wave per buffer), write (waves over all
// segments, the tile steps of rle_device.h with absolute positions, an owned end and a first
// chunk shared with the previous segment written bytewise; encode writes a segment without a run
// boundary from its entering state alone).  Same output as rle_kernels.hip.
#include "rle_device.h"

namespace rle {

// The decode summary's phase-free count of literal tiles (dec_count_phasefree, round 6): off.  r6be /
// r6bf, rocprof medians of the summary kernel (1024 x 1 MiB random / runs50 / configs[2] mixed):
// tried on every tile 236.1 / 364.9 / 80.3 µs, with the back-off below 256.7 / 291.1 / 70.7, off
// 268.2-269.7 / 269.4-276.5 / 63.6-66.0.  The random gain does not pay for the run-heavy loss.
#ifndef RLE_SEG_PHASEFREE
#define RLE_SEG_PHASEFREE 0
#endif
#ifndef RLE_SEG_PF_WAIT
#define RLE_SEG_PF_WAIT 8
#endif

// Segment length: seg_tiles tiles of 1008 input bytes, a kernel argument chosen by the launcher
// (4..16 tiles: about 16 segments per CU over the batch).
#ifndef RLE_SEG_TILES_MAX   // 16 since r3s (was 64): more, shorter segments fill the chip better
#define RLE_SEG_TILES_MAX 16
#endif
constexpr u32 kSegTilesMin = 4, kSegTilesMax = RLE_SEG_TILES_MAX;
// decode write pass staging (chunks per wave, rle_device.h kDecChunks): the launcher takes the
// one-pass 192-chunk kernel when every segment is resident at once, else the 96-chunk one (7 instead
// of 4 workgroups per CU; r3s A/B: 1 MiB random -9 %, mixed batch -27 %, one 64 MiB file +7 % with 96)
constexpr u32 kSegDecChunksOne = RLE_DEC_CHUNKS, kSegDecChunksMany = 96;
constexpr u32 kSegWaves = 4;
constexpr u32 kSegBlock = kWave * kSegWaves;
constexpr u32 kNone = 0xFFFFFFFFu;
// per-buffer flags (workspace) written by the scans, read by the writers
constexpr u32 kFlagSkip = 1u;     // bad buffer: status already written
constexpr u32 kFlagSerial = 2u;   // decode: the exact serial path handles the whole buffer
// The write passes take the fast tile paths (round 3) and the segments last-summarised first
// (memory-side cache reuse; r3w, same process: configs[2] mixed batch encode -6 %, decode -2 %, 1 MiB
// kinds +-1 %); the summaries count uniform / literal tiles without the full analysis (round 3) and
// sum their lanes' counts once per segment, not per tile (round 5).

// Segments of an n-byte buffer: n = q S + r gives q + (r >= 3) segments (at least one); the last
// absorbs a remainder of 1-2 bytes, so a stream's final token never starts a segment of its own.
__device__ __forceinline__ u32 seg_count(u32 n, u32 sb) {
    const u32 k = (u32)(((uint64_t)n + sb - 3u) / sb);
    return k ? k : 1u;
}
__device__ __forceinline__ u32 len32(uint64_t n) { return n > kMaxBufferBytes ? 0u : (u32)n; }

// seg_first[i] = segments of buffers < i; seg_first[n] = total.  One workgroup.
__global__ __launch_bounds__(1024) void seg_plan_kernel(const uint64_t* __restrict__ len, u32 n, u32 sb,
                                                        u32* __restrict__ seg_first, u32* __restrict__ sflag,
                                                        u32 maxseg, u32* __restrict__ ticket,
                                                        u32* __restrict__ bclear) {
    __shared__ u32 part[1024];
    const u32 t = threadIdx.x;
    // (fused kernels) every segment's publication flag cleared, the ticket counter at 0, and (the
    // single-pass decode) every buffer's flags
    if (sflag)
        for (u32 i = t; i < maxseg; i += 1024u) sflag[i] = 0u;
    if (bclear)
        for (u32 i = t; i < n; i += 1024u) bclear[i] = 0u;
    if (ticket && t == 0u) *ticket = 0u;
    const u32 per = (n + 1023u) / 1024u;
    const u32 b0 = t * per < n ? t * per : n;
    const u32 b1 = b0 + per < n ? b0 + per : n;
    u32 s = 0;
    for (u32 i = b0; i < b1; ++i) s += seg_count(len32(len[i]), sb);
    part[t] = s;
    __syncthreads();
    for (u32 off = 1; off < 1024u; off <<= 1) {
        const u32 v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    u32 base = t ? part[t - 1] : 0u;
    for (u32 i = b0; i < b1; ++i) {
        seg_first[i] = base;
        base += seg_count(len32(len[i]), sb);
    }
    if (t == 1023u) seg_first[n] = part[1023];
}

// the buffer holding global segment g: seg_first[b] <= g < seg_first[b + 1] (every buffer has a
// segment, so seg_first is strictly increasing)
__device__ __forceinline__ u32 seg_buffer(const u32* seg_first, u32 n, u32 g) {
    u32 lo = 0, hi = n;
    while (hi - lo > 1u) {
        const u32 mid = (lo + hi) >> 1;
        if (uniform(seg_first[mid]) <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}
// seg_buf[g] = the buffer holding segment g, for every segment (one binary search per segment, all
// in parallel), so the persistent summary and write waves find a segment's buffer with one load
constexpr u32 kMapBlock = 256;
__global__ __launch_bounds__(kMapBlock) void seg_map_kernel(const u32* __restrict__ seg_first, u32 n, u32 maxseg,
                                                           u32* __restrict__ seg_buf) {
    const u32 g = blockIdx.x * kMapBlock + threadIdx.x;
    const u32 total = seg_first[n] < maxseg ? seg_first[n] : maxseg;
    if (g >= total) return;
    u32 lo = 0, hi = n;
    while (hi - lo > 1u) {
        const u32 mid = (lo + hi) >> 1;
        if (seg_first[mid] <= g) lo = mid;
        else hi = mid;
    }
    seg_buf[g] = lo;
}
// A launch of one buffer (the drop-in's single large calls) skips the plan and map launches: the
// launcher passes seg_first = seg_buf = nullptr, and every segment is buffer 0's, its segments
// [0, seg_count(in_len[0])) (round 5).
__device__ __forceinline__ u32 seg_total(const u32* seg_first, u32 n, const uint64_t* len, u32 sb) {
    return seg_first ? uniform(seg_first[n]) : seg_count(len32(len[0]), sb);
}
__device__ __forceinline__ u32 seg_of(const u32* seg_buf, u32 g) { return seg_buf ? uniform(seg_buf[g]) : 0u; }
__device__ __forceinline__ u32 seg_lo(const u32* seg_first, u32 b) { return seg_first ? uniform(seg_first[b]) : 0u; }
__device__ __forceinline__ u32 seg_hi(const u32* seg_first, u32 b, const uint64_t* len, u32 sb) {
    return seg_first ? uniform(seg_first[b + 1]) : seg_count(len32(len[0]), sb);
}
__device__ __forceinline__ void seg_range(u32 i, u32 nseg, u32 n, u32 sb, u32& p0, u32& p1) {
    p0 = i * sb;
    p1 = (i + 1u == nseg) ? n : p0 + sb;
}

__device__ __forceinline__ u32 wave_sum(u32 x) { return readlane(wave_scan_incl(x, 0u, OpAdd()), 63); }
// over the tile-owning lanes 0..62 (lane 63 holds the lookahead only)
__device__ __forceinline__ u32 owned_sum(u32 x) { return readlane(wave_scan_incl(x, 0u, OpAdd()), kOwnLanes - 1u); }
__device__ __forceinline__ bool owned_any(bool x) {
    return (__builtin_amdgcn_ballot_w64(x) & ((1ull << kOwnLanes) - 1ull)) != 0ull;
}

// A segment's tile walk: through the double-buffered LDS-DMA slots (walk_tiles), or (kRes) over a
// segment already resident in LDS (res_load): tile t at mem + 1008 t, nothing to load or wait for.
template <bool kRes, class Step>
__device__ __forceinline__ bool walk_seg(u32x4 rs, u32 start, u32 ntiles, u32 lane, const uint8_t* mem, Step step) {
    if (kRes) {
#pragma clang loop unroll(disable)
        for (u32 t = 0; t < ntiles; ++t)
            if (step(t, mem + t * kTileStep, Refill{rs, 0u, 0u, false, false}) == ~0u) {
                vm_drain();
                return true;
            }
        return false;
    }
    return walk_tiles(rs, start, ntiles, lane, mem, step);
}

// Resident segments (the single-pass kernels below): a segment of at most kResTiles tiles (segments
// are kResTiles - 1 tiles, a buffer's last one up to 2 bytes more) is loaded
// into the wave's LDS region once, [p0, p0 + 1008 nt + 16) in 1 KiB LDS-DMAs (range-checked: zeros
// past the buffer), and both its summary and its output walk read it there.
#ifndef RLE_RES_TILES
#define RLE_RES_TILES 8
#endif
constexpr u32 kResTiles = RLE_RES_TILES;
constexpr u32 kResBytes = (kResTiles * kTileStep + 16u + 1023u) & ~1023u;
[[maybe_unused]] constexpr u32 kResStride = kResBytes;
#ifndef RLE_RES_DEC_CHUNKS   // the resident decode's staging (chunks per wave; its region takes LDS too)
#define RLE_RES_DEC_CHUNKS 96
#endif
[[maybe_unused]] constexpr u32 kResDecChunks = RLE_RES_DEC_CHUNKS;
__device__ __forceinline__ void res_load(u32x4 rs, u32 p0, u32 nt, u32 lane, const uint8_t* region) {
    const u32 l0 = uniform(lds_addr(region));
    const u32 nd = uniform((nt * kTileStep + 16u + 1023u) >> 10);
    asm volatile("s_nop 4" ::: "memory");   // descriptor words may be fresh (walk_prime)
    for (u32 k = 0; k < nd; ++k) dma_tile<true>(rs, p0 + 1024u * k + 16u * lane, l0 + 1024u * k);
    vm_drain();
}

// ================================================================ ENCODE
// compressed bytes of the tokens starting in a segment's entering run piece (length L0) when the
// byte before the segment has run phase q; cont: the piece's run continues past the segment
__device__ __forceinline__ u32 enc_piece_count(u32 L0, u32 q, u32 cont) {
    const u32 k0 = q >= 8u ? 0u : 8u - q;
    if (L0 <= k0) return 0u;
    const u32 n = (L0 - 1u - k0) / 9u + 1u;
    const bool last_is_start = (L0 - 1u - k0) % 9u == 0u;
    return 3u * n - ((last_is_start && !cont) ? 2u : 0u);
}

// One segment's encode summary (L0, lb + 1 or 0, rest, cont; see the top of this file): a walk over
// its tiles, analysis only.  U > 0, src 16-byte aligned.
template <bool kRes = false>
__device__ __forceinline__ uint4 enc_seg_summarize(const uint8_t* src, u32 U, u32 p0, u32 p1, u32 lane,
                                                   const uint8_t* slots) {
    const u32x4 rsi = make_rsrc(src, (U + 15u) & ~15u);
    u32 prev_top = p0 ? (u32)src[p0 - 1u] << 24 : 0u;
    u32 rs = p0, fb = kNone, lb = kNone, rest = 0;
    u32 restl = 0u, lbl = 0u;   // the lane's token bytes and its last boundary + 1 (0: none), summed once per segment
    const EncK kc = enc_k();
    walk_seg<kRes>(rsi, p0, ntiles_for(p1 - p0), lane, slots, [&](u32 t, const uint8_t* cs, const Refill& nx) {
        const u32x4 cur = *reinterpret_cast<const u32x4*>(cs + 16u * lane);
        nx();
        const u32 pos = p0 + t * kTileStep;
        // (tried only when the run entering the tile is already 16 bytes long, a scalar test
        // that keeps the check off random and short-run tiles)
        if (pos != 0u && pos - rs >= 16u && pos + kTileStep < p1) {
            // a tile inside a run (every byte, and the first lookahead byte, equal to the byte
            // before the tile; never the buffer's first tile, whose position 0 is a boundary
            // whatever its byte): no boundary, so fb, lb and rs stay; the tokens count only past
            // the segment's first boundary, all 3-byte (the run goes on), one every 9 bytes
            // from the run start rs.  About 10 VALU against enc_analyze's ~75.
            const u32 v = uniform(readlane(cur.x, 0)) & 0xFFu;
            if ((prev_top >> 24) == v) {
                const u32 vrep = v * 0x01010101u;
                const bool diff = lane < kOwnLanes
                                      ? ((cur.x ^ vrep) | (cur.y ^ vrep) | (cur.z ^ vrep) | (cur.w ^ vrep)) != 0u
                                      : ((cur.x ^ vrep) & 0xFFu) != 0u;
                if (!__builtin_amdgcn_ballot_w64(diff)) {
                    if (fb != kNone) {
                        const u32 f = pos + (9u - (pos - rs) % 9u) % 9u;   // first token start
                        if (f < pos + kTileStep) rest += 3u * ((pos + kTileStep - 1u - f) / 9u + 1u);
                    }
                    return 0u;
                }
            }
        }
        const EncAn an = enc_analyze<false>(cur, uint2{0u, 0u}, pos, U, p1, lane, prev_top, rs, kc);
        // run boundaries inside the segment: the first one (L0) and the last one (lb)
        const u32 Bo = an.B & an.validm;
        // the first boundary on the scalar unit until found; the last one per lane (tiles come in
        // order, so a lane's latest is its last), the lanes' maximum taken once per segment (round 5:
        // the per-tile wave reductions it replaced measured within +-2 %)
        if (fb == kNone) {
            const uint64_t bl = __builtin_amdgcn_ballot_w64(Bo != 0u);
            if (bl) fb = readlane(an.p0 + (u32)__builtin_ctz(Bo | 0x10000u), (u32)__builtin_ctzll(bl));
        }
        lbl = Bo ? an.p0 + 32u - (u32)__builtin_clz(Bo) : lbl;
        // tokens at or after the first boundary do not depend on the entering run phase
        u32 fbm = 0u;
        if (fb != kNone) fbm = fb <= an.p0 ? 0xFFFFu : (fb >= an.p0 + 16u ? 0u : ~lowmask(fb - an.p0) & 0xFFFFu);
        restl += bcnt(an.T & fbm, 0u) + 2u * bcnt(an.P & fbm, 0u);
        prev_top = readlane(an.top, kOwnLanes - 1u);
        const u32 i63 = readlane(an.incl, kOwnLanes - 1u);
        rs = i63 > rs ? i63 : rs;
        return 0u;
    });
    rest += wave_sum(restl);
    const u32 m = readlane(wave_scan_incl(lbl, 0u, OpMax()), kWave - 1u);
    if (m) lb = m - 1u;
    const u32 L0 = fb == kNone ? p1 - p0 : fb - p0;
    const u32 cont = (fb == kNone && p1 < U && src[p1] == src[p1 - 1u]) ? 1u : 0u;
    return make_uint4(L0, lb == kNone ? 0u : lb + 1u, rest, cont);
}

__global__ __launch_bounds__(kSegBlock) void enc_seg_summary_kernel(const uint8_t* __restrict__ in,
                                                                    const uint64_t* __restrict__ in_off,
                                                                    const uint64_t* __restrict__ in_len, u32 n,
                                                                    const u32* __restrict__ seg_first, const u32* __restrict__ seg_buf, u32 maxseg, u32 sb,
                                                                    uint4* __restrict__ summ) {
    __shared__ __attribute__((aligned(16))) uint8_t slots_all[kSegWaves * 2 * kSlot];
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    const uint8_t* slots = slots_all + wid * 2 * kSlot;
    u32 total = seg_total(seg_first, n, in_len, sb);
    total = total < maxseg ? total : maxseg;
    for (u32 g = blockIdx.x * kSegWaves + wid; g < total; g += gridDim.x * kSegWaves) {
        const u32 b = seg_of(seg_buf, g);
        const u32 s0 = seg_lo(seg_first, b), nseg = seg_hi(seg_first, b, in_len, sb) - s0;
        const uint64_t U64 = in_len[b];
        const uint8_t* src = in + in_off[b];
        uint4 res = make_uint4(0u, 0u, 0u, 0u);
        if (U64 > 0 && U64 <= kMaxBufferBytes && !((uintptr_t)src & 15u)) {
            u32 p0, p1;
            seg_range(g - s0, nseg, (u32)U64, sb, p0, p1);
            res = enc_seg_summarize(src, (u32)U64, p0, p1, lane, slots);
        }
        if (lane == 0) summ[g] = res;
    }
}

// The carried state of an encode scan over a buffer's segments: max (lb + 1) so far, and the output
// offset.  One window of up to 64 consecutive segments (lane i: segment base + i, summary sm, first
// position p0), entered with c: each lane's entering run start and output offset; c advances past
// the window.  Shared by the per-buffer scan and the fused kernel's look-back.
struct EncCarry {
    u32 lb1, off;
};
__device__ __forceinline__ uint2 enc_seg_window(uint4 sm, bool valid, u32 p0, EncCarry& c) {
    const u32 incl = wave_scan_incl(valid ? sm.y : 0u, 0u, OpMax());
    const u32 ex = from_prev_lane(incl, 0u);
    const u32 rsp1 = ex > c.lb1 ? ex : c.lb1;
    const u32 rs = rsp1 ? rsp1 - 1u : 0u;
    const u32 piece = (valid && p0 > 0u) ? enc_piece_count(sm.x, mod9(p0 - 1u - rs), sm.w) : 0u;
    const u32 cnt = valid ? piece + sm.z : 0u;
    const u32 oincl = wave_scan_incl(cnt, 0u, OpAdd());
    const uint2 r = make_uint2(rs, c.off + oincl - cnt);
    const u32 i63 = readlane(incl, 63);
    c.lb1 = i63 > c.lb1 ? i63 : c.lb1;
    c.off += readlane(oincl, 63);
    return r;
}

// one wave per buffer: entering run start and output offset of every segment, C of the buffer
__global__ __launch_bounds__(kSegBlock) void enc_seg_scan_kernel(const uint8_t* __restrict__ in,
                                                                 const uint64_t* __restrict__ in_off,
                                                                 const uint64_t* __restrict__ in_len,
                                                                 uint8_t* __restrict__ out,
                                                                 const uint64_t* __restrict__ out_off,
                                                                 uint64_t* __restrict__ out_len,
                                                                 uint32_t* __restrict__ status, u32 n,
                                                                 const u32* __restrict__ seg_first, u32 maxseg, u32 sb,
                                                                 const uint4* __restrict__ summ, uint2* __restrict__ plan,
                                                                 u32* __restrict__ bflag) {
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 b = blockIdx.x * kSegWaves + uniform(threadIdx.x / kWave);
    if (b >= n) return;
    const uint64_t U64 = in_len[b];
    const uint8_t* src = in + in_off[b];
    uint8_t* dst = out + out_off[b];
    const u32 s0 = seg_lo(seg_first, b), s1 = seg_hi(seg_first, b, in_len, sb);
    u32 bad = (((uintptr_t)src | (uintptr_t)dst) & 15u) ? RLE_STATUS_MISALIGNED : 0u;
    if (U64 > kMaxBufferBytes || s1 > maxseg) bad |= RLE_STATUS_TOOLARGE;
    if (bad) {
        if (lane == 0) {
            out_len[b] = 0;
            if (status) status[b] = bad;
            bflag[b] = kFlagSkip;
        }
        return;
    }
    EncCarry c{0u, 0u};
    for (u32 base = s0; base < s1; base += kWave) {
        const u32 g = base + lane;
        const bool valid = g < s1;
        const uint4 sm = valid ? summ[g] : make_uint4(0u, 0u, 0u, 0u);
        const uint2 pl = enc_seg_window(sm, valid, (g - s0) * sb, c);
        if (valid) plan[g] = pl;
    }
    if (lane == 0) {
        out_len[b] = c.off;
        if (status) status[b] = RLE_STATUS_OK;
        bflag[b] = 0u;
    }
}

// One segment's output: the tile walk from its entering run start rs and output offset off.
template <bool kRes = false>
__device__ __forceinline__ void enc_seg_write(const uint8_t* src, uint8_t* dst, u32 U, u32 p0, u32 p1, u32 rs,
                                              u32 off, u32 lane, const uint8_t* slots, uint8_t* stage,
                                              const u32* elut) {
    const u32x4 rsi = make_rsrc(src, (U + 15u) & ~15u);
    const u32x4 rso = make_rsrc(dst, U + U / 2u);
    EncState st{off, off & ~15u, p0 ? (u32)src[p0 - 1u] << 24 : 0u, rs, off & 15u, false, {}};
    const EncK kc = enc_k();
    walk_seg<kRes>(rsi, p0, ntiles_for(p1 - p0), lane, slots, [&](u32 t, const uint8_t* cs, const Refill& nx) {
        // the fast tile paths (round 3; until then only the one-wave kernels took them): past the
        // segment's shared first chunk and before its last tile, as in a one-wave walk
        return enc_tile<false, true>(cs, nx, p0 + t * kTileStep, U, p1, lane, stage, dst, rso, st, kc, elut);
    });
    // the final partial chunk (< 16 bytes, staging chunk 1): byte stores, nothing past this
    // segment's output and nothing before it
    if (lane >= st.head && lane < st.out_pos - st.flushed) dst[st.flushed + lane] = stage[16u + lane];
    wave_lds_sync();
}

// A segment without a run boundary (every byte equals the byte before the segment, v: zero-filled
// data, long runs) encodes to "v v '9'" tokens every 9 bytes from the entering run start rs; only
// the last token's count depends on the input, through the (up to 8) run bytes after the segment.
// Its output is written from that alone, without reading the segment a second time (the summary
// pass has read it): aligned 16-byte chunks of the 3-periodic pattern, and the partial chunks at
// both ends, which the neighbouring segments share, bytewise.  (Round 3.)
#define RLE_SEG_UNIFORM_ATTR __attribute__((noinline))   // out of the write loop's hot code (r3x)
__device__ RLE_SEG_UNIFORM_ATTR void enc_seg_uniform(const uint8_t* src, uint8_t* dst, u32 U, u32 p0, u32 p1, u32 rs,
                                                u32 off, u32 lane) {
    const u32 v = src[p0];
    const bool eq = lane < 8u && p1 + lane < U && src[p1 + lane] == v;
    const u32 ext = (u32)__builtin_ctzll(__builtin_amdgcn_ballot_w64(!eq));   // run bytes past p1, <= 8
    const u32 f = p0 + (9u - (p0 - rs) % 9u) % 9u;   // the segment's first token start
    if (f >= p1) return;                             // none: the previous segment's token covers it
    const u32 ns = (p1 - 1u - f) / 9u + 1u;
    const u32 sl = f + 9u * (ns - 1u);
    const u32 cl = p1 + ext - sl < 9u ? p1 + ext - sl : 9u;   // the last token's count
    const u32 tot = 3u * (ns - 1u) + (cl >= 2u ? 3u : 1u);
    const u32 end = off + tot;
    const u32 ld = (cl >= 2u && cl < 9u) ? tot - 1u : ~0u;   // the output byte holding a count other than 9
    const u32 vv = rep4(v), d9 = 0x39393939u;
    auto byte_at = [&](u32 k) { return k % 3u != 2u ? v : (k == ld ? 0x30u + cl : 0x39u); };
    // aligned interior chunks [a0, a1)
    const u32 a0 = (off + 15u) & ~15u, a1 = end & ~15u;
    for (u32 c0 = a0; c0 < a1; c0 += 16u * kWave) {
        const u32 c = c0 + 16u * lane;
        const u32 k0 = c - off, ph = k0 % 3u;
        u32 o[4];
#pragma unroll
        for (u32 q = 0; q < 4u; ++q) {
            u32 mk[3];
#pragma unroll
            for (u32 p = 0; p < 3u; ++p) {
                u32 m = 0;
                for (u32 b = 0; b < 4u; ++b)
                    if ((p + 4u * q + b) % 3u == 2u) m |= 0xFFu << (8u * b);
                mk[p] = m;
            }
            const u32 dm = ph == 0u ? mk[0] : ph == 1u ? mk[1] : mk[2];
            o[q] = (vv & ~dm) | (d9 & dm);
        }
        const u32 kd = ld - k0;   // the odd count digit, when it falls in this chunk
        if (kd < 16u) {
            const u32 sh = 8u * (kd & 3u), q = kd >> 2;
            const u32 dv = (0x30u + cl) << sh, msk = 0xFFu << sh;
            o[0] = q == 0u ? (o[0] & ~msk) | dv : o[0];
            o[1] = q == 1u ? (o[1] & ~msk) | dv : o[1];
            o[2] = q == 2u ? (o[2] & ~msk) | dv : o[2];
            o[3] = q == 3u ? (o[3] & ~msk) | dv : o[3];
        }
        if (c < a1) *reinterpret_cast<u32x4*>(dst + c) = u32x4{o[0], o[1], o[2], o[3]};
    }
    // the partial chunks at both ends
    const u32 h1 = a0 < end ? a0 : end;
    if (lane < 16u && off + lane < h1) dst[off + lane] = (uint8_t)byte_at(lane);
    const u32 t0 = a1 > a0 ? a1 : a0;
    if (lane < 16u && t0 + lane < end) dst[t0 + lane] = (uint8_t)byte_at(t0 + lane - off);
}

__global__ __launch_bounds__(kSegBlock) void enc_seg_write_kernel(const uint8_t* __restrict__ in,
                                                                  const uint64_t* __restrict__ in_off,
                                                                  const uint64_t* __restrict__ in_len,
                                                                  uint8_t* __restrict__ out,
                                                                  const uint64_t* __restrict__ out_off, u32 n,
                                                                  const u32* __restrict__ seg_first, const u32* __restrict__ seg_buf, u32 maxseg, u32 sb,
                                                                  const uint2* __restrict__ plan,
                                                                  const u32* __restrict__ bflag,
                                                                  const uint4* __restrict__ summ) {
    __shared__ __attribute__((aligned(16))) uint8_t slots_all[kSegWaves * 2 * kSlot];
    __shared__ __attribute__((aligned(16))) uint8_t stage_all[kSegWaves * kEncStage];
    __shared__ __attribute__((aligned(16))) u32 elut[kInsWaveWords];   // enc_tile_fast's selectors
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    uint8_t* stage = stage_all + wid * kEncStage;
    const uint8_t* slots = slots_all + wid * 2 * kSlot;
    for (u32 k = threadIdx.x; k < kInsWaveWords; k += kSegBlock) elut[k] = kEncInsLut.s[k];
    __syncthreads();
    u32 total = seg_total(seg_first, n, in_len, sb);
    total = total < maxseg ? total : maxseg;
    for (u32 g0 = blockIdx.x * kSegWaves + wid; g0 < total; g0 += gridDim.x * kSegWaves) {
        const u32 g = total - 1u - g0;
        // (the segment's own plan and summary load with its buffer index, not after it)
        const uint2 pl = plan[g];
        const uint4 sm = summ[g];
        const u32 b = seg_of(seg_buf, g);
        if (uniform(bflag[b])) continue;
        const u32 s0 = seg_lo(seg_first, b), nseg = seg_hi(seg_first, b, in_len, sb) - s0;
        const u32 U = (u32)in_len[b];
        const uint8_t* src = in + in_off[b];
        uint8_t* dst = out + out_off[b];
        u32 p0, p1;
        seg_range(g - s0, nseg, U, sb, p0, p1);
        if (p0 > 0u) {
            if (uniform(sm.y) == 0u && uniform(sm.x) == p1 - p0) {   // no run boundary in the segment
                enc_seg_uniform(src, dst, U, p0, p1, uniform(pl.x), uniform(pl.y), lane);
                continue;
            }
        }
        enc_seg_write(src, dst, U, p0, p1, uniform(pl.x), uniform(pl.y), lane, slots, stage, elut);
    }
}

// ================================================================ measured-slower variants
// (RLE_VARIANTS builds only: the test library build/librle_mi355x_testhooks.so and `make variant`;
// never the product librle_mi355x.so.  VERDICT r3 item 8.)  The fused single-pass encode and the
// resident single-pass kernels are bit-exact and tested, but slower than the five-launch default
// ("Round 3: segmented path"), so the product does not carry them.
#if RLE_VARIANTS
// ---------------------------------------------------------------- fused single-pass encode
// One launch after the plan (SURVEY.md §5's single-pass form, with a decoupled look-back carry):
// waves take segments in ticket order (a global counter), summarise their segment, publish the
// summary (flag 1), derive their entering state from the published summaries and inclusive states
// of the segments before them in the same buffer, publish their own inclusive state (flag 2), and
// write their output at once: the segment's bytes are read a second time right after the first,
// while they are still in the caches, and no separate scan launch waits for the whole batch.
// Progress: a wave waits only on segments holding earlier tickets, whose waves are running and
// never wait on later ones, so the earliest unfinished segment always advances.  The wait is
// still bounded (kSpinMax polls); a wave that runs out publishes and marks its buffer
// RLE_STATUS_INTERNAL instead of hanging (never seen; tests check the status is clean).
constexpr u32 kSpinMax = 1u << 20;
constexpr u32 kFlagAgg = 1u, kFlagIncl = 2u;
// The hand-off follows MI355X_MICROARCH.md's write-through form (per-XCD L2s are not coherent, and
// an agent release fence would write back the XCD's whole dirty L2 after every segment): the
// publishing lane stores every payload word and the flag write-through (relaxed agent-scope atomic
// stores: `sc1`), with `s_waitcnt vmcnt(0)` between them; readers poll the flag and read the
// payload with `sc1` loads (relaxed agent-scope atomic loads), never plain or scalar-cache loads.
__device__ __forceinline__ u32 ld_relaxed(const u32* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(u32* p, u32 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 ld_relaxed4(const uint4* p) {
    const u32* w = reinterpret_cast<const u32*>(p);
    return make_uint4(ld_relaxed(w), ld_relaxed(w + 1), ld_relaxed(w + 2), ld_relaxed(w + 3));
}
// (one lane) payload, drain, flag
__device__ __forceinline__ void publish(uint4* slot, uint4 v, u32* flag, u32 f) {
    u32* w = reinterpret_cast<u32*>(slot);
    st_relaxed(w, v.x);
    st_relaxed(w + 1, v.y);
    st_relaxed(w + 2, v.z);
    st_relaxed(w + 3, v.w);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_relaxed(flag, f);
}
// The first segment this wave must combine forward: j + 1 for the nearest j in [s0, g) whose
// inclusive state is published, or s0 (the buffer's start state) when none is; on return every
// segment in [result, g) has published its summary.  Windows of 64 flags, nearest first.
__device__ __forceinline__ u32 seg_lookback(u32 g, u32 s0, const u32* sflag, u32 lane, bool& late) {
    u32 hi = g;
    for (;;) {
        const u32 lo = hi - s0 > kWave ? hi - kWave : s0;
        const bool valid = lane < hi - lo;
        const u32 j = valid ? hi - 1u - lane : hi - 1u;
        u32 f = valid ? ld_relaxed(sflag + j) : kFlagAgg;
        u32 polls = 0;
        // wait only for the segments between this one and the nearest published inclusive state
        // (or, when the window has none, for the whole window)
        for (;;) {
            const uint64_t m0 = __builtin_amdgcn_ballot_w64(f == 0u);
            const uint64_t m2 = __builtin_amdgcn_ballot_w64(valid && f == kFlagIncl);
            const uint64_t need = m2 ? (m2 & (0ull - m2)) - 1ull : ~0ull;
            if (!(m0 & need) || ++polls > kSpinMax) {
                if (m0 & need) late = true;
                if (m2) return hi - (u32)__builtin_ctzll(m2);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
            if (f == 0u) f = ld_relaxed(sflag + j);
        }
        if (lo == s0) return s0;
        hi = lo;
    }
}

__global__ __launch_bounds__(kSegBlock) void enc_seg_fused_kernel(const uint8_t* __restrict__ in,
                                                                  const uint64_t* __restrict__ in_off,
                                                                  const uint64_t* __restrict__ in_len,
                                                                  uint8_t* __restrict__ out,
                                                                  const uint64_t* __restrict__ out_off,
                                                                  uint64_t* __restrict__ out_len,
                                                                  uint32_t* __restrict__ status, u32 n,
                                                                  const u32* __restrict__ seg_first, u32 maxseg, u32 sb,
                                                                  uint4* __restrict__ summ, uint4* __restrict__ incl,
                                                                  u32* __restrict__ sflag, u32* __restrict__ ticket) {
    __shared__ __attribute__((aligned(16))) uint8_t slots_all[kSegWaves * 2 * kSlot];
    __shared__ __attribute__((aligned(16))) uint8_t stage_all[kSegWaves * kEncStage];
    __shared__ __attribute__((aligned(16))) u32 elut[kInsWaveWords];   // enc_tile_fast's selectors
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    uint8_t* stage = stage_all + wid * kEncStage;
    const uint8_t* slots = slots_all + wid * 2 * kSlot;
    for (u32 k = threadIdx.x; k < kInsWaveWords; k += kSegBlock) elut[k] = kEncInsLut.s[k];
    __syncthreads();
    u32 total = uniform(seg_first[n]);
    total = total < maxseg ? total : maxseg;
    for (;;) {
        u32 g = 0;
        if (lane == 0) g = atomicAdd(ticket, 1u);
        g = uniform(g);
        if (g >= total) break;
        const u32 b = seg_buffer(seg_first, n, g);
        const u32 s0 = uniform(seg_first[b]), s1 = uniform(seg_first[b + 1]), nseg = s1 - s0;
        const uint64_t U64 = in_len[b];
        const uint8_t* src = in + in_off[b];
        uint8_t* dst = out + out_off[b];
        u32 bad = (((uintptr_t)src | (uintptr_t)dst) & 15u) ? RLE_STATUS_MISALIGNED : 0u;
        if (U64 > kMaxBufferBytes || s1 > maxseg) bad |= RLE_STATUS_TOOLARGE;
        if (bad || U64 == 0u) {   // the buffer's segments all skip (an empty buffer is one segment)
            if (g == s0 && lane == 0) {
                out_len[b] = 0;
                if (status) status[b] = bad;
            }
            continue;
        }
        const u32 U = (u32)U64;
        u32 p0, p1;
        seg_range(g - s0, nseg, U, sb, p0, p1);
        const uint4 sm = enc_seg_summarize(src, U, p0, p1, lane, slots);
        if (lane == 0) publish(summ + g, sm, sflag + g, kFlagAgg);
        // the state entering this segment: the nearest published inclusive state (or the buffer's
        // start), then the summaries after it, 64 per window
        bool late = false;
        EncCarry c{0u, 0u};
        u32 lateb = 0u;
        if (g > s0) {
            const u32 from = seg_lookback(g, s0, sflag, lane, late);
            if (from > s0) {
                const uint4 in4 = ld_relaxed4(incl + (from - 1u));
                c = EncCarry{uniform(in4.x), uniform(in4.y)};
                lateb = uniform(in4.z);
            }
            for (u32 base = from; base < g; base += kWave) {
                const u32 j = base + lane;
                const bool valid = j < g;
                const uint4 smj = valid ? ld_relaxed4(summ + j) : make_uint4(0u, 0u, 0u, 0u);
                enc_seg_window(smj, valid, (j - s0) * sb, c);
            }
        }
        // this segment's own step (lane 0's window entry), published as its inclusive state
        const uint2 mine = enc_seg_window(sm, lane == 0u, p0, c);
        const u32 rs = uniform(mine.x), off = uniform(mine.y);
        lateb |= late ? RLE_STATUS_INTERNAL : 0u;
        if (lane == 0) {
            publish(incl + g, make_uint4(c.lb1, c.off, lateb, 0u), sflag + g, kFlagIncl);
            // the status words were cleared by the plan launch: a late segment ORs its bit in itself
            // (a later segment may rebuild its state from raw summaries and not carry it), and the
            // last segment ORs what it carries, so no bit is overwritten
            if (late && status) atomicOr(status + b, RLE_STATUS_INTERNAL);
            if (g + 1u == s1) {   // the buffer's last segment: C and the status
                out_len[b] = c.off;
                if (lateb && status) atomicOr(status + b, lateb);
            }
        }
        enc_seg_write(src, dst, U, p0, p1, rs, off, lane, slots, stage, elut);
    }
}


// ---------------------------------------------------------------- resident single-pass encode
// SURVEY.md §5's single pass, with the segment held in LDS: a wave takes a segment by ticket and
// loads its <= kResTiles tiles into its LDS region once, summarises them there, publishes the summary, derives its entering state with the
// decoupled look-back of the fused kernel above, publishes its inclusive state and walks the same
// LDS tiles again to write.  HBM sees the input once.  Progress: as in the fused kernel, a wave
// waits only on segments of earlier tickets, whose waves are running.
// One segment per ticket: a wave holding several consecutive segments publishes the later ones'
// summaries only after writing the earlier ones, so the waves behind it in the same buffer wait for
// its whole batch (measured: the look-backs run out of polls).  The next ticket is taken while the
// current segment is processed, which hides the atomic's latency and keeps progress (a wave's
// prefetched segment is always later than its current one).
// Since round 3 without the ticket counter: wave w of workgroup k takes segment 4 k + w of a grid
// of one wave per segment.  A workgroup is dispatched only after every lower-numbered
// workgroup of its XCD, so the lowest-numbered waiting segment's predecessors are all running or
// done, and the look-back cannot wait forever (and its polls are bounded regardless: a wave that
// runs out marks its buffer and exits).
__global__ __launch_bounds__(kSegBlock) void enc_seg_res_kernel(const uint8_t* __restrict__ in,
                                                                const uint64_t* __restrict__ in_off,
                                                                const uint64_t* __restrict__ in_len,
                                                                uint8_t* __restrict__ out,
                                                                const uint64_t* __restrict__ out_off,
                                                                uint64_t* __restrict__ out_len,
                                                                uint32_t* __restrict__ status, u32 n,
                                                                const u32* __restrict__ seg_first,
                                                                const u32* __restrict__ seg_buf, u32 maxseg, u32 sb,
                                                                uint4* __restrict__ summ, uint4* __restrict__ incl,
                                                                u32* __restrict__ sflag, u32* __restrict__ ticket) {
    __shared__ __attribute__((aligned(16))) uint8_t region_all[kSegWaves * kResStride];
    __shared__ __attribute__((aligned(16))) uint8_t stage_all[kSegWaves * kEncStage];
    __shared__ __attribute__((aligned(16))) u32 elut[kInsWaveWords];   // enc_tile_fast's selectors
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    uint8_t* stage = stage_all + wid * kEncStage;
    const uint8_t* region = region_all + wid * kResStride;
    for (u32 k = threadIdx.x; k < kInsWaveWords; k += kSegBlock) elut[k] = kEncInsLut.s[k];
    __syncthreads();
    u32 total = uniform(seg_first[n]);
    total = total < maxseg ? total : maxseg;
    (void)ticket;
    u32 gnext = blockIdx.x * kSegWaves + wid;   // one segment per wave
    for (;;) {
        const u32 g = uniform(gnext);
        if (g >= total) break;
        gnext = total;
        {
            const u32 b = uniform(seg_buf[g]);
            const u32 s0 = uniform(seg_first[b]), s1 = uniform(seg_first[b + 1]), nseg = s1 - s0;
            const uint64_t U64 = in_len[b];
            const uint8_t* src = in + in_off[b];
            uint8_t* dst = out + out_off[b];
            u32 bad = (((uintptr_t)src | (uintptr_t)dst) & 15u) ? RLE_STATUS_MISALIGNED : 0u;
            if (U64 > kMaxBufferBytes || s1 > maxseg) bad |= RLE_STATUS_TOOLARGE;
            if (bad || U64 == 0u) {   // the buffer's segments all skip (an empty buffer is one segment)
                if (g == s0 && lane == 0) {
                    out_len[b] = 0;
                    if (status) status[b] = bad;
                }
                continue;
            }
            const u32 U = (u32)U64;
            u32 p0, p1;
            seg_range(g - s0, nseg, U, sb, p0, p1);
            res_load(make_rsrc(src, (U + 15u) & ~15u), p0, ntiles_for(p1 - p0), lane, region);
            const uint4 sm = enc_seg_summarize<true>(src, U, p0, p1, lane, region);
            if (lane == 0) publish(summ + g, sm, sflag + g, kFlagAgg);
            bool late = false;
            EncCarry c{0u, 0u};
            u32 lateb = 0u;
            if (g > s0) {
                const u32 from = seg_lookback(g, s0, sflag, lane, late);
                if (from > s0) {
                    const uint4 in4 = ld_relaxed4(incl + (from - 1u));
                    c = EncCarry{uniform(in4.x), uniform(in4.y)};
                    lateb = uniform(in4.z);
                }
                for (u32 base = from; base < g; base += kWave) {
                    const u32 j = base + lane;
                    const bool valid = j < g;
                    const uint4 smj = valid ? ld_relaxed4(summ + j) : make_uint4(0u, 0u, 0u, 0u);
                    enc_seg_window(smj, valid, (j - s0) * sb, c);
                }
            }
            const uint2 mine = enc_seg_window(sm, lane == 0u, p0, c);
            lateb |= late ? RLE_STATUS_INTERNAL : 0u;
            if (lane == 0) {
                publish(incl + g, make_uint4(c.lb1, c.off, lateb, 0u), sflag + g, kFlagIncl);
                if (late && status) atomicOr(status + b, RLE_STATUS_INTERNAL);   // (as enc_seg_fused_kernel)
                if (g + 1u == s1) {   // the buffer's last segment: C and the status
                    out_len[b] = c.off;
                    if (lateb && status) atomicOr(status + b, lateb);
                }
            }
            enc_seg_write<true>(src, dst, U, p0, p1, uniform(mine.x), uniform(mine.y), lane, region, stage, elut);
        }
    }
}
#endif  // RLE_VARIANTS

// ================================================================ DECODE
// Decoded bytes of a non-tail tile entered at phase d when every pair token in it is "v v 2" (random
// and text-like data): then each token's output is its own bytes with the count digit deleted, so
// the count is the owned positions minus the pairs' digits minus the tile's first d positions (the
// literal path's count, dec_tile_fast, without its stores or its per-lane limits).  kNotFast when a
// pair has another count (the caller then runs dec_lengths).  About 40 VALU against ~100 for
// dec_lengths + its sum.
// kLane: the lane's own count (the caller sums the lanes once per segment).
template <bool kLane = false>
__device__ __forceinline__ u32 dec_count_literal(const DecPrep& pr, u32 d, u32 lane, const DecK& kc) {
    constexpr uint64_t kOwned = (1ull << kOwnLanes) - 1ull;
    const u32* w = pr.w;
    const u32 NE16 = (pr.xa >> 7) | (pr.xb << 1);
    // cheap reject first (runs): at most 2 equal neighbours per owned lane
    if (__builtin_amdgcn_ballot_w64(__builtin_popcount(~NE16 & 0xFFFFu) > 2) & kOwned) return kNotFast;
    const u32 dl = bfe(pr.excl, 8u * d, 8);
    const u32 mid = __builtin_amdgcn_perm(0u, pr.ta.y, 0x0C0C0C00u | dl);
    const u32 sa = __builtin_amdgcn_perm(0u, pr.ta.x, 0x0C0C0C00u | dl);
    const u32 sb = __builtin_amdgcn_perm(0u, pr.tb.x, 0x0C0C0C00u | mid);
    const u32 P16 = (sa | (sb << 8)) & ~NE16 & 0xFFFFu;   // pair starts
    const u32 dg[4] = {alignbyte(w[1], w[0], 2), alignbyte(w[2], w[1], 2), alignbyte(w[3], w[2], 2),
                       alignbyte(pr.la, w[3], 2)};
    u32 nz[4];
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 t = dg[k] ^ 0x32323232u;
        nz[k] = bitop3<kOrAnd>(faddi<0x7F7F7F7Fu>(t & kc.K7F), t, kc.K80);
    }
    const u32 za = __builtin_amdgcn_udot4(nz[1], kc.C2, __builtin_amdgcn_udot4(nz[0], kc.C1, 0u, false), false);
    const u32 zb = __builtin_amdgcn_udot4(nz[3], kc.C2, __builtin_amdgcn_udot4(nz[2], kc.C1, 0u, false), false);
    const u32 NZ16 = (za >> 7) | (zb << 1);   // digit position j + 2 holds something other than '2'
    const u32 prevP = from_prev_lane(P16, 0u);
    u32 del = ((P16 << 2) | (prevP >> 14)) & 0xFFFFu;
    if (lane == 0u) del |= lowmask(d);
    const u32 K = lane < kOwnLanes ? (~del & 0xFFFFu) : ((prevP >> 15) & 1u);
    if (__builtin_amdgcn_ballot_w64((P16 & NZ16) != 0u) & kOwned) return kNotFast;
    return kLane ? (u32)__builtin_popcount(K) : wave_sum((u32)__builtin_popcount(K));
}

// Decoded bytes of a non-tail tile of a literal stream, for every entry phase at once (round 6,
// the summary pass is VALU-bound, 137 VALU per random tile, profiles/
// r6bd_seg_sq_kinds.md).  Let EQ(j) be y[j] == y[j + 1].  When every EQ position j also has
// y[j + 1] != y[j + 2] and y[j + 2] == '2', then (whatever the entry phase d):
//   * no byte '2' is EQ (y[j + 1] would be '2' and differ from y[j + 2] == '2');
//   * from d on, every EQ position is a token start, i.e. a "v v 2" pair: the pair's second byte
//     is not EQ (y[j + 1] != y[j + 2]) nor is its '2', so nothing inside a pair is EQ, and a byte is
//     a one-byte token exactly where it is neither EQ nor inside a pair;
//   * positions 0 and 1 are required not EQ: below d they hold the end of a pair the previous tile
//     started, whose digit may be anything;
// so the tile decodes to (1008 - #EQ) - d + e bytes and leaves exit phase e = 2 / 1 / 0 for a pair
// at 1007 / 1006 / neither, the same for every d.  No phase table, no phase scan.  Returns the
// lane's count of non-EQ positions (0 on the lookahead lane) and e, or kNotFast when a position
// breaks the condition (the caller then takes dec_prepare and the general path).
constexpr u32 kEqBad = (~0xF0u & (~0xCCu | 0xAAu)) & 0xFFu;   // bitop3: ~a & (~b | c)
__device__ __forceinline__ u32 dec_count_phasefree(const u32x4 cur, u32 lane, const DecK& kc, u32& e) {
    constexpr uint64_t kOwned = (1ull << kOwnLanes) - 1ull;
    const u32 w[4] = {cur.x, cur.y, cur.z, cur.w};
    const u32 la = from_next_lane(w[0], 0u);
    const u32 nb[4] = {alignbyte(w[1], w[0], 1), alignbyte(w[2], w[1], 1), alignbyte(w[3], w[2], 1),
                       alignbyte(la, w[3], 1)};
    const u32 dg[4] = {alignbyte(w[1], w[0], 2), alignbyte(w[2], w[1], 2), alignbyte(w[3], w[2], 2),
                       alignbyte(la, w[3], 2)};
    const u32 K80 = kc.K80, K7F = kc.K7F;
    u32 ne[4];   // 0x80 per byte: y[j] != y[j + 1]
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 t = w[k] ^ nb[k];
        ne[k] = bitop3<kOrAnd>(faddi<0x7F7F7F7Fu>(t & K7F), t, K80);
    }
    const u32 nn = from_next_lane(ne[0], K80);   // the next lane's first positions
    u32 bad = 0u, cnt = 0u;
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 nen = alignbyte(k < 3u ? ne[k + 1u] : nn, ne[k], 1);   // y[j + 1] != y[j + 2]
        const u32 b = dg[k] ^ 0x32323232u;
        const u32 nd = bitop3<kOrAnd>(faddi<0x7F7F7F7Fu>(b & K7F), b, K80);   // y[j + 2] != '2'
        bad |= bitop3<kEqBad>(ne[k], nen, nd);   // EQ without NE(j + 1), or with a digit other than '2'
        cnt += (u32)__builtin_popcount(ne[k]);
    }
    if (__builtin_amdgcn_ballot_w64((bad & K80) != 0u) & kOwned) return kNotFast;
    if ((readlane(ne[0], 0) & 0x8080u) != 0x8080u) return kNotFast;   // EQ at position 0 or 1
    const u32 ne62 = readlane(ne[3], kOwnLanes - 1u);   // positions 1004..1007
    e = !(ne62 & 0x80000000u) ? 2u : (!(ne62 & 0x00800000u) ? 1u : 0u);
    return lane < kOwnLanes ? cnt : 0u;
}

// One segment's decode summary: for each entry phase 0..2, the decoded bytes (.x .y .z) and, in .w,
// the exit phases (2 bits each) and the phases whose tiled path declines (bits 8..10).  C > 0.
// Whether every token starting in this tile (entry phase d, starts S80 from dec_lengths) carries
// one byte v, the byte of the tile's first token.
__device__ __forceinline__ bool dec_tile_single(const DecPrep& pr, const DecLen& ln, u32 d, const DecK& kc, u32& v) {
    v = (readlane(pr.w[0], 0) >> (8u * d)) & 0xFFu;
    const u32 vv = rep4(v);
    u32 bad = 0;
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 t = pr.w[k] ^ vv;
        bad |= bitop3<kOrAnd>(faddi<0x7F7F7F7Fu>(t & kc.K7F), t, kc.K80) & ln.S80[k];
    }
    return !owned_any(bad != 0u);
}

// One segment's decode summary: for each entry phase 0..2, the decoded bytes (.x .y .z) and, in .w,
// the exit phases (2 bits each), the phases whose tiled path declines (bits 8..10) and the phases
// from which every token carries one byte (bits 11..13: the segment decodes to copies of that byte,
// the one at its first token; dec_seg_fill writes them without reading the segment).  C > 0.
template <bool kRes = false>
__device__ __forceinline__ uint4 dec_seg_summarize(const uint8_t* src, u32 C, u32 q0, u32 q1, u32 lane,
                                                   const uint8_t* slots, const DecEntry* tbl) {
    const u32x4 rsi = make_rsrc(src, (C + 15u) & ~15u);
    u32 d0 = 0u, d1 = 1u, d2 = 2u, c0 = 0u, c1 = 0u, c2 = 0u, badm = 0u;
    u32 uni = 7u, v0 = 0u, v1 = 0u, v2 = 0u;   // single-byte phases and their bytes
    u32 accm = 0u;       // the lane's decoded bytes over the tiles after the phases merged (summed once)
    bool badl = false;   // ... and whether the lane declined in one of them
    u32 a0 = 0u, a1 = 0u, a2 = 0u;   // phase-free tiles: e - d per entry phase (wave-uniform, wrapping)
    constexpr u32 kPfWait = RLE_SEG_PF_WAIT;
    u32 pf_wait = 0u;
    const DecK kc = dec_k();
    walk_seg<kRes>(rsi, q0, ntiles_for(q1 - q0), lane, slots, [&](u32 t, const uint8_t* cs, const Refill& nx) {
        const u32x4 cur = *reinterpret_cast<const u32x4*>(cs + 16u * lane);
        nx();
        const u32 pos = q0 + t * kTileStep;
        // (dec_prepare's non-tail tiles; after a tile the check declines, the next kPfWait tiles go
        // straight to the general path: run-heavy and zero-filled streams decline on every tile,
        // r6be: runs50 summary 276.5 -> 364.9 µs when every tile tried)
        if (pf_wait) {
            --pf_wait;
        } else if (RLE_SEG_PHASEFREE && pos + kSlot + 2u <= q1) {
            u32 e = 0u;
            const u32 tot = dec_count_phasefree(cur, lane, kc, e);
            if (tot == kNotFast) pf_wait = kPfWait;
            else {
                accm += tot;
                a0 += e - d0;
                a1 += e - d1;
                a2 += e - d2;
                d0 = d1 = d2 = e;
                uni = 0u;   // (as the literal path below)
                return 0u;
            }
        }
        const DecPrep pr = dec_prepare(cur, pos, C, q1, lane, tbl, kc);
        const u32 m63 = readlane(pr.incl, kOwnLanes - 1u);   // lane 63: lookahead only
        if (d0 == d1 && d1 == d2) {   // the three entry phases have merged: one evaluation
            u32 tot = !pr.tail ? dec_count_literal<true>(pr, d0, lane, kc) : kNotFast;
            if (tot == kNotFast) {
                const DecLen ln = dec_lengths(pr, d0);
                // the lane's count and decline, summed once per segment
                tot = lane < kOwnLanes ? ln.nout : 0u;
                badl |= lane < kOwnLanes && ln.serial_lane;
                if (uni) {
                    u32 v;
                    const bool one = dec_tile_single(pr, ln, d0, kc, v);
                    if (!one || v != v0) uni &= ~1u;
                    if (!one || v != v1) uni &= ~2u;
                    if (!one || v != v2) uni &= ~4u;
                }
            } else {
                uni = 0u;   // a literal tile (its own bytes, "v v 2" pairs): not counted as single-byte
            }
            accm += tot;
            d0 = d1 = d2 = bfe(m63, 8u * d0, 8);
        } else {
            const DecLen l0 = dec_lengths(pr, d0);
            c0 += owned_sum(l0.nout);
            badm |= owned_any(l0.serial_lane) ? 1u : 0u;
            const DecLen l1 = dec_lengths(pr, d1);
            c1 += owned_sum(l1.nout);
            badm |= owned_any(l1.serial_lane) ? 2u : 0u;
            const DecLen l2 = dec_lengths(pr, d2);
            c2 += owned_sum(l2.nout);
            badm |= owned_any(l2.serial_lane) ? 4u : 0u;
            if (uni) {
                u32 v;
                bool one = dec_tile_single(pr, l0, d0, kc, v);
                if (!one || (t && v != v0)) uni &= ~1u;
                v0 = t ? v0 : v;
                one = dec_tile_single(pr, l1, d1, kc, v);
                if (!one || (t && v != v1)) uni &= ~2u;
                v1 = t ? v1 : v;
                one = dec_tile_single(pr, l2, d2, kc, v);
                if (!one || (t && v != v2)) uni &= ~4u;
                v2 = t ? v2 : v;
            }
            d0 = bfe(m63, 8u * d0, 8);
            d1 = bfe(m63, 8u * d1, 8);
            d2 = bfe(m63, 8u * d2, 8);
        }
        return 0u;
    });
    const u32 cm = wave_sum(accm);
    c0 += cm + a0; c1 += cm + a1; c2 += cm + a2;
    badm |= __builtin_amdgcn_ballot_w64(badl) ? 7u : 0u;
    return make_uint4(c0, c1, c2, d0 | (d1 << 2) | (d2 << 4) | (badm << 8) | (uni << 11));
}
// the summary of an empty stream: counts 0, exit = entry
constexpr uint4 kDecEmpty = {0u, 0u, 0u, 0u | (1u << 2) | (2u << 4)};

__global__ __launch_bounds__(kSegBlock) void dec_seg_summary_kernel(const uint8_t* __restrict__ in,
                                                                    const uint64_t* __restrict__ in_off,
                                                                    const uint64_t* __restrict__ in_len, u32 n,
                                                                    const u32* __restrict__ seg_first, const u32* __restrict__ seg_buf, u32 maxseg, u32 sb,
                                                                    uint4* __restrict__ summ) {
    __shared__ __attribute__((aligned(16))) uint8_t slots_all[kSegWaves * 2 * kSlot];
    __shared__ DecEntry tbl[256];
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    for (u32 k = threadIdx.x; k < 256u; k += kSegBlock) tbl[k] = dec_entry_from(kDecTable.e[k]);
    __syncthreads();
    const uint8_t* slots = slots_all + wid * 2 * kSlot;
    u32 total = seg_total(seg_first, n, in_len, sb);
    total = total < maxseg ? total : maxseg;
    for (u32 g = blockIdx.x * kSegWaves + wid; g < total; g += gridDim.x * kSegWaves) {
        const u32 b = seg_of(seg_buf, g);
        const u32 s0 = seg_lo(seg_first, b), nseg = seg_hi(seg_first, b, in_len, sb) - s0;
        const uint64_t C64 = in_len[b];
        const uint8_t* src = in + in_off[b];
        uint4 res = kDecEmpty;
        if (C64 > 0 && C64 <= kMaxBufferBytes && !((uintptr_t)src & 15u)) {
            u32 q0, q1;
            seg_range(g - s0, nseg, (u32)C64, sb, q0, q1);
            res = dec_seg_summarize(src, (u32)C64, q0, q1, lane, slots, tbl);
        }
        if (lane == 0) summ[g] = res;
    }
}

// The carried state of a decode scan over a buffer's segments: the entry phase, the output offset
// and whether the buffer needs the exact serial path (a taken phase declines, or the stream decodes
// past U).  One window of up to 64 consecutive segments (lane i: segment base + i, summary sm); each
// lane gets its segment's entry phase and output offset; c advances past the window.  Shared by the
// per-buffer scan and the single-pass kernel's look-back.
struct DecCarry {
    u32 e, off;
    bool serial;
};
__device__ __forceinline__ uint2 dec_seg_window(uint4 sm, bool valid, u32 U, DecCarry& c) {
    const u32 sel = valid ? (bfe(sm.w, 0, 2) | (bfe(sm.w, 2, 2) << 8) | (bfe(sm.w, 4, 2) << 16) | (3u << 24)) : kMapId;
    const u32 incl = wave_scan_incl(sel, kMapId, OpMap());
    const u32 e = bfe(from_prev_lane(incl, kMapId), 8u * c.e, 8);
    const u32 cnt = valid ? (e == 0u ? sm.x : (e == 1u ? sm.y : sm.z)) : 0u;
    c.serial |= __builtin_amdgcn_ballot_w64(valid && ((sm.w >> (8u + e)) & 1u)) != 0;
    const u32 oincl = wave_scan_incl(cnt, 0u, OpAdd());
    const uint2 r = make_uint2(e, c.off + oincl - cnt);
    c.e = bfe(readlane(incl, 63), 8u * c.e, 8);
    const u32 add = readlane(oincl, 63);
    if (add > U - (c.off < U ? c.off : U)) c.serial = true;   // decodes past U
    c.off += add;
    return r;
}

// one wave per buffer: entry phase and output offset of every segment; serial when the taken
// path declines anywhere or decodes past U
__global__ __launch_bounds__(kSegBlock) void dec_seg_scan_kernel(const uint8_t* __restrict__ in,
                                                                 const uint64_t* __restrict__ in_off,
                                                                 const uint64_t* __restrict__ in_len,
                                                                 uint8_t* __restrict__ out,
                                                                 const uint64_t* __restrict__ out_off,
                                                                 const uint64_t* __restrict__ out_len,
                                                                 const uint64_t* __restrict__ out_cap,
                                                                 uint32_t* __restrict__ status, u32 n,
                                                                 const u32* __restrict__ seg_first, u32 maxseg, u32 sb,
                                                                 const uint4* __restrict__ summ, uint2* __restrict__ plan,
                                                                 u32* __restrict__ bflag) {
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 b = blockIdx.x * kSegWaves + uniform(threadIdx.x / kWave);
    if (b >= n) return;
    const uint64_t C64 = in_len[b], U64 = out_len[b];
    const uint64_t cap = out_cap ? out_cap[b] : U64;
    const uint8_t* src = in + in_off[b];
    uint8_t* dst = out + out_off[b];
    const u32 s0 = seg_lo(seg_first, b), s1 = seg_hi(seg_first, b, in_len, sb);
    u32 bad = ((((uintptr_t)src | (uintptr_t)dst) & 15u) || cap < U64) ? RLE_STATUS_MISALIGNED : 0u;
    if (C64 > kMaxBufferBytes || U64 > kMaxBufferBytes || s1 > maxseg) bad |= RLE_STATUS_TOOLARGE;
    if (bad) {
        if (lane == 0) {
            if (status) status[b] = bad;
            bflag[b] = kFlagSkip;
        }
        return;
    }
    const u32 U = (u32)U64;
    DecCarry c{0u, 0u, false};
    for (u32 base = s0; base < s1; base += kWave) {
        const u32 g = base + lane;
        const bool valid = g < s1;
        const uint4 sm = valid ? summ[g] : make_uint4(0u, 0u, 0u, 0u);
        const uint2 pl = dec_seg_window(sm, valid, U, c);
        if (valid) plan[g] = pl;
    }
    if (lane == 0) bflag[b] = c.serial ? kFlagSerial : 0u;
}

// A segment whose tokens all carry one byte v (summary bit 11 + e; never a stream's last segment,
// whose end dec_finish handles) decodes to cnt copies of v: written without reading the segment,
// aligned 16-byte chunks and, at both ends (shared with the neighbouring segments), single bytes.
__device__ RLE_SEG_UNIFORM_ATTR void dec_seg_fill(uint8_t* dst, u32 U, u32 off, u32 cnt, u32 v, u32 lane) {
    const u32 end = off + cnt;
    const u32 a0 = (off + 15u) & ~15u, a1 = end & ~15u;
    const u32 vv = rep4(v);
    for (u32 c0 = a0; c0 < a1; c0 += 16u * kWave) {
        const u32 c = c0 + 16u * lane;
        if (c < a1) *reinterpret_cast<u32x4*>(dst + c) = u32x4{vv, vv, vv, vv};
    }
    const u32 h1 = a0 < end ? a0 : end;
    if (lane < 16u && off + lane < h1) dst[off + lane] = (uint8_t)v;
    const u32 t0 = a1 > a0 ? a1 : a0;
    if (lane < 16u && t0 + lane < end) dst[t0 + lane] = (uint8_t)v;
}

// One segment's output: the tile walk from entry phase e and output offset off; the stream's last
// segment (last) also writes the bytes up to U and the status (st_b, when given).
template <bool kRes, u32 kChunks>
__device__ __forceinline__ void dec_seg_write(const uint8_t* src, uint8_t* dst, u32 C, u32 U, u32 q0, u32 q1, u32 e,
                                              u32 off, bool last, u32 lane, const uint8_t* slots, uint8_t* stage,
                                              const DecEntry* tbl, const u32x4* clut, uint32_t* st_b) {
    const u32x4 rsi = make_rsrc(src, (C + 15u) & ~15u);
    const u32x4 rso = make_rsrc(dst, U);
    DecState st{off, off & ~15u, e, 0u, 0u, off & 15u, 0u, false, {}};
    const DecK kc = dec_k();
    const bool serial = walk_seg<kRes>(rsi, q0, ntiles_for(q1 - q0), lane, slots, [&](u32 t, const uint8_t* cs, const Refill& nx) {
        // the fast tile paths (round 3): past the segment's shared first chunk, and the literal
        // path only on tiles a later tile of this segment follows (dec_tile)
        return dec_tile<true, kChunks, false>(cs, nx, q0 + t * kTileStep, C, q1, U, lane, tbl, stage, dst, rso, st, kc,
                                               clut);
    });
    dec_finish(st, last ? U : st.out_pos, lane, stage, rso, dst);
    if (last && lane == 0 && st_b) *st_b = serial ? (RLE_STATUS_SERIAL | RLE_STATUS_OVERFLOW) : dec_tiled_status(st, U);
}

template <u32 kSegDecChunks>
__global__ __launch_bounds__(kSegBlock) void dec_seg_write_kernel(const uint8_t* __restrict__ in,
                                                                  const uint64_t* __restrict__ in_off,
                                                                  const uint64_t* __restrict__ in_len,
                                                                  uint8_t* __restrict__ out,
                                                                  const uint64_t* __restrict__ out_off,
                                                                  const uint64_t* __restrict__ out_len,
                                                                  const uint64_t* __restrict__ out_cap,
                                                                  uint32_t* __restrict__ status, u32 n,
                                                                  const u32* __restrict__ seg_first, const u32* __restrict__ seg_buf, u32 maxseg, u32 sb,
                                                                  const uint2* __restrict__ plan,
                                                                  const u32* __restrict__ bflag,
                                                                  const uint4* __restrict__ summ) {
    __shared__ __attribute__((aligned(16))) uint8_t slots_all[kSegWaves * 2 * kSlot];
    constexpr u32 kStage = 32u * kSegDecChunks;
    __shared__ __attribute__((aligned(128))) uint8_t stage_all[kSegWaves * kStage];
    __shared__ DecEntry tbl[256];
    __shared__ u32x4 clut[kCompactEntries];   // dec_tile_fast's selectors
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    for (u32 k = threadIdx.x; k < 256u; k += kSegBlock) tbl[k] = dec_entry_from(kDecTable.e[k]);
    for (u32 k = threadIdx.x; k < kCompactEntries; k += kSegBlock)
        clut[k] = u32x4{kCompactLut.s[4u * k], kCompactLut.s[4u * k + 1u], kCompactLut.s[4u * k + 2u],
                        kCompactLut.s[4u * k + 3u]};
    uint8_t* stage = stage_all + wid * kStage;
    const uint8_t* slots = slots_all + wid * 2 * kSlot;
    for (u32 k = lane; k < kStage / 16u; k += kWave)
        reinterpret_cast<u32x4*>(stage)[k] = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    u32 total = seg_total(seg_first, n, in_len, sb);
    total = total < maxseg ? total : maxseg;
    for (u32 g0 = blockIdx.x * kSegWaves + wid; g0 < total; g0 += gridDim.x * kSegWaves) {
        const u32 g = total - 1u - g0;
        const uint2 pl = plan[g];
        const uint4 sm = summ[g];
        const u32 b = seg_of(seg_buf, g);
        const u32 flag = uniform(bflag[b]);
        if (flag & kFlagSkip) continue;
        const u32 s0 = seg_lo(seg_first, b), nseg = seg_hi(seg_first, b, in_len, sb) - s0;
        const u32 C = (u32)in_len[b], U = (u32)out_len[b];
        const uint8_t* src = in + in_off[b];
        uint8_t* dst = out + out_off[b];
        if (flag & kFlagSerial) {   // one wave decodes the whole buffer exactly
            if (g == s0) {
                const uint64_t cap = out_cap ? out_cap[b] : (uint64_t)U;
                const u32 stat = dec_serial(src, C, U, cap, dst, lane, stage, kStage);
                if (lane == 0 && status) status[b] = stat;
            }
            continue;
        }
        u32 q0, q1;
        seg_range(g - s0, nseg, C, sb, q0, q1);
        if (g + 1u != s0 + nseg) {   // one byte throughout: no second read
            const u32 e = uniform(pl.x);
            if ((uniform(sm.w) >> (11u + e)) & 1u) {
                const u32 cnt = uniform(e == 0u ? sm.x : (e == 1u ? sm.y : sm.z));
                dec_seg_fill(dst, U, uniform(pl.y), cnt, src[q0 + e], lane);
                continue;
            }
        }
        dec_seg_write<false, kSegDecChunks>(src, dst, C, U, q0, q1, uniform(pl.x), uniform(pl.y), g + 1u == s0 + nseg,
                                            lane, slots, stage, tbl, clut, status ? status + b : nullptr);
    }
}


#if RLE_VARIANTS
// ---------------------------------------------------------------- resident single-pass decode
// The decode form of enc_seg_res_kernel: a segment's summary is its three entry phases' counts and
// exits (dec_seg_summarize), its entering phase and offset come from the look-back (dec_seg_window
// over the published summaries), and its output walk reads the same LDS tiles.  A buffer that needs
// the exact serial path (a taken phase declines, the stream decodes past U, or a look-back ran out
// of polls) is only known once its last segment has combined: its segments skip their walks from
// the first one that knows, the buffer is flagged (bflag, cleared by the plan), and
// dec_seg_serial_kernel decodes it after this launch, over whatever the earlier segments wrote.
// kRes false (RLE_MI355X_SEG_RES=2, round 5): the same single pass without the LDS-resident segment
// (its 28 KB region per workgroup capped it at 3 workgroups per CU): the summary walks the segment
// through the two DMA slots, and the write walks it again, from the caches if it is still there.
template <bool kRes>
__global__ __launch_bounds__(kSegBlock) void dec_seg_res_kernel(const uint8_t* __restrict__ in,
                                                                const uint64_t* __restrict__ in_off,
                                                                const uint64_t* __restrict__ in_len,
                                                                uint8_t* __restrict__ out,
                                                                const uint64_t* __restrict__ out_off,
                                                                const uint64_t* __restrict__ out_len,
                                                                const uint64_t* __restrict__ out_cap,
                                                                uint32_t* __restrict__ status, u32 n,
                                                                const u32* __restrict__ seg_first,
                                                                const u32* __restrict__ seg_buf, u32 maxseg, u32 sb,
                                                                uint4* __restrict__ summ, uint4* __restrict__ incl,
                                                                u32* __restrict__ sflag, u32* __restrict__ ticket,
                                                                u32* __restrict__ bflag) {
    constexpr u32 kStage = 32u * kResDecChunks;
    constexpr u32 kRegion = kRes ? kResStride : 2u * kSlot;   // the resident segment, or two DMA slots
    __shared__ __attribute__((aligned(16))) uint8_t region_all[kSegWaves * kRegion];
    __shared__ __attribute__((aligned(128))) uint8_t stage_all[kSegWaves * kStage];
    __shared__ DecEntry tbl[256];
    __shared__ u32x4 clut[kCompactEntries];   // dec_tile_fast's selectors
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    for (u32 k = threadIdx.x; k < 256u; k += kSegBlock) tbl[k] = dec_entry_from(kDecTable.e[k]);
    for (u32 k = threadIdx.x; k < kCompactEntries; k += kSegBlock)
        clut[k] = u32x4{kCompactLut.s[4u * k], kCompactLut.s[4u * k + 1u], kCompactLut.s[4u * k + 2u],
                        kCompactLut.s[4u * k + 3u]};
    uint8_t* stage = stage_all + wid * kStage;
    const uint8_t* region = region_all + wid * kRegion;
    for (u32 k = lane; k < kStage / 16u; k += kWave) reinterpret_cast<u32x4*>(stage)[k] = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    u32 total = uniform(seg_first[n]);
    total = total < maxseg ? total : maxseg;
    (void)ticket;
    u32 gnext = blockIdx.x * kSegWaves + wid;   // one segment per wave
    for (;;) {
        const u32 g = uniform(gnext);
        if (g >= total) break;
        gnext = total;
        {
            const u32 b = uniform(seg_buf[g]);
            const u32 s0 = uniform(seg_first[b]), s1 = uniform(seg_first[b + 1]), nseg = s1 - s0;
            const uint64_t C64 = in_len[b], U64 = out_len[b];
            const uint64_t cap = out_cap ? out_cap[b] : U64;
            const uint8_t* src = in + in_off[b];
            uint8_t* dst = out + out_off[b];
            u32 bad = ((((uintptr_t)src | (uintptr_t)dst) & 15u) || cap < U64) ? RLE_STATUS_MISALIGNED : 0u;
            if (C64 > kMaxBufferBytes || U64 > kMaxBufferBytes || s1 > maxseg) bad |= RLE_STATUS_TOOLARGE;
            if (bad) {   // the buffer's segments all skip
                if (g == s0 && lane == 0 && status) status[b] = bad;
                continue;
            }
            const u32 C = (u32)C64, U = (u32)U64;
            u32 q0, q1;
            seg_range(g - s0, nseg, C, sb, q0, q1);
            uint4 sm = kDecEmpty;
            if (C) {
                if (kRes) res_load(make_rsrc(src, (C + 15u) & ~15u), q0, ntiles_for(q1 - q0), lane, region);
                sm = dec_seg_summarize<kRes>(src, C, q0, q1, lane, region, tbl);
            }
            if (lane == 0) publish(summ + g, sm, sflag + g, kFlagAgg);
            bool late = false;
            DecCarry c{0u, 0u, false};
            if (g > s0) {
                const u32 from = seg_lookback(g, s0, sflag, lane, late);
                if (from > s0) {
                    const uint4 in4 = ld_relaxed4(incl + (from - 1u));
                    c = DecCarry{uniform(in4.x), uniform(in4.y), uniform(in4.z) != 0u};
                }
                for (u32 base = from; base < g; base += kWave) {
                    const u32 j = base + lane;
                    const bool valid = j < g;
                    const uint4 smj = valid ? ld_relaxed4(summ + j) : make_uint4(0u, 0u, 0u, 0u);
                    dec_seg_window(smj, valid, U, c);
                }
            }
            const uint2 mine = dec_seg_window(sm, lane == 0u, U, c);
            c.serial = c.serial || late;
            const bool last = g + 1u == s1;
            if (lane == 0) {
                publish(incl + g, make_uint4(c.e, c.off, c.serial ? 1u : 0u, 0u), sflag + g, kFlagIncl);
                // the buffer's serial flag: from its last segment, or from any segment whose
                // look-back ran out (its state may not reach the last segment's combine)
                if ((last && c.serial) || late) atomicOr(bflag + b, kFlagSerial);
            }
            if (!c.serial)
                dec_seg_write<kRes, kResDecChunks>(src, dst, C, U, q0, q1, uniform(mine.x), uniform(mine.y), last, lane,
                                                   region, stage, tbl, clut, status ? status + b : nullptr);
        }
    }
}

// After dec_seg_res_kernel: the exact serial decode of the buffers it flagged, one wave each.
__global__ __launch_bounds__(kSegBlock) void dec_seg_serial_kernel(const uint8_t* __restrict__ in,
                                                                   const uint64_t* __restrict__ in_off,
                                                                   const uint64_t* __restrict__ in_len,
                                                                   uint8_t* __restrict__ out,
                                                                   const uint64_t* __restrict__ out_off,
                                                                   const uint64_t* __restrict__ out_len,
                                                                   const uint64_t* __restrict__ out_cap,
                                                                   uint32_t* __restrict__ status, u32 n,
                                                                   const u32* __restrict__ bflag) {
    __shared__ __attribute__((aligned(16))) uint8_t stage_all[kSegWaves * 1024];
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    const u32 b = blockIdx.x * kSegWaves + wid;
    if (b >= n || !(uniform(bflag[b]) & kFlagSerial)) return;
    const u32 U = (u32)out_len[b];
    const uint64_t cap = out_cap ? out_cap[b] : (uint64_t)U;
    const u32 stat = dec_serial(in + in_off[b], (u32)in_len[b], U, cap, out + out_off[b], lane, stage_all + wid * 1024, 1024);
    if (lane == 0 && status) status[b] = stat;
}

#endif  // RLE_VARIANTS

}  // namespace rle

// ================================================================ C-ABI launchers
#include <map>
#include <mutex>
#include <utility>

namespace {
// The workspace (seg_first, per-segment summaries and plans, per-buffer flags) belongs to the
// caller (rle_seg_workspace_bytes), like a cub temp-storage argument: the library keeps no
// device memory between calls and nothing tied to a stream or thread.  Host-side cache: CUs.
struct CuCache {
    std::mutex m;
    std::map<int, int> cus;
};
CuCache& cu_cache() {
    static CuCache* p = new CuCache();   // never destroyed: launches may run during exit
    return *p;
}
// 256 B-aligned carve-up of the workspace
struct Carve {
    uint32_t* seg_first;
    uint32_t* seg_buf;   // per-segment buffer index (seg_map_kernel)
    uint4* summ;
    uint2* plan;
    uint32_t* bflag;
    uint32_t* sflag;    // fused kernels: per-segment publication flag
    uint4* incl;        // fused kernels: per-segment inclusive state
    uint32_t* ticket;   // fused kernels: segment ticket counter
    size_t bytes;
};
inline size_t al(size_t x) { return (x + 255u) & ~(size_t)255u; }
Carve carve(char* base, uint32_t n, uint32_t maxseg) {
    Carve c;
    size_t o = 0;
    c.seg_first = reinterpret_cast<uint32_t*>(base + o); o += al(sizeof(uint32_t) * ((size_t)n + 1));
    c.seg_buf = reinterpret_cast<uint32_t*>(base + o);   o += al(sizeof(uint32_t) * (size_t)maxseg);
    c.summ = reinterpret_cast<uint4*>(base + o);         o += al(sizeof(uint4) * (size_t)maxseg);
    c.plan = reinterpret_cast<uint2*>(base + o);         o += al(sizeof(uint2) * (size_t)maxseg);
    c.bflag = reinterpret_cast<uint32_t*>(base + o);     o += al(sizeof(uint32_t) * (size_t)n);
    c.sflag = reinterpret_cast<uint32_t*>(base + o);     o += al(sizeof(uint32_t) * (size_t)maxseg);
    c.incl = reinterpret_cast<uint4*>(base + o);         o += al(sizeof(uint4) * (size_t)maxseg);
    c.ticket = reinterpret_cast<uint32_t*>(base + o);    o += al(sizeof(uint32_t));
    c.bytes = o;
    return c;
}
// upper bound on the segments of n buffers holding total bytes (each segment but a buffer's
// last covers sb bytes)
inline uint32_t max_segments(uint32_t n, uint64_t total, uint32_t sb) {
    const uint64_t m = total / (sb - 2u) + n;
    return m > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)m;
}
int device_cus(int* ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return RLE_E_HIP;
    CuCache& P = cu_cache();
    std::lock_guard<std::mutex> g(P.m);
    auto c = P.cus.find(dev);
    if (c == P.cus.end()) {
        int k = 0;
        if (hipDeviceGetAttribute(&k, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || k <= 0) k = 256;
        c = P.cus.emplace(dev, k).first;
    }
    *ncu = c->second;
    return RLE_OK;
}
// segment length in bytes: about 16 segments per CU over the batch, 4..16 tiles each
// (longer segments, caps of 32 / 64 tiles, measured slower on the mixed batch: r5w)
// The resident single-pass kernels (enc_seg_res_kernel / dec_seg_res_kernel): RLE_MI355X_SEG_RES=1|0
// overrides the build default.  Their segments are one tile shorter than an LDS region, so that a
// buffer's last segment (which absorbs a remainder of up to 2 bytes) still fits.  Segment lengths
// stay whole tiles: a segment's exit state is read after the last tile's last lane (an 8048-byte
// segment, measured, left the decode exit phase one lane late).
// 0 off, 1 the resident single pass, 2 the single pass without the resident segment (decode)
int seg_res_mode() {
    if (!RLE_VARIANTS) return 0;   // (product build: RLE_MI355X_SEG_RES is not read)
    static const int m = [] {
        const char* e = getenv("RLE_MI355X_SEG_RES");
        return e ? atoi(e) : 0;
    }();
    return m;
}
bool seg_res() { return seg_res_mode() == 1; }
inline uint32_t seg_bytes(uint64_t total, int ncu) {
    if (seg_res()) return (rle::kResTiles - 1u) * rle::kTileStep;
    const uint64_t tiles = (total + rle::kTileStep - 1) / rle::kTileStep;
    uint64_t per = tiles / ((uint64_t)ncu * 16u);
    per = per < rle::kSegTilesMin ? rle::kSegTilesMin : (per > rle::kSegTilesMax ? rle::kSegTilesMax : per);
    return (uint32_t)per * rle::kTileStep;
}
// persistent grids: enough workgroups to fill every CU (RLE_SEG_OCC per CU), never more than the
// segments
#ifndef RLE_SEG_OCC   // 24 since r3s (was 4): workgroups past residency queue behind the first ones
#define RLE_SEG_OCC 24
#endif
inline uint32_t seg_grid(uint32_t maxseg, int ncu) {
    const uint32_t need = (maxseg + rle::kSegWaves - 1) / rle::kSegWaves;
    const uint32_t fill = (uint32_t)ncu * RLE_SEG_OCC;
    const uint32_t g = need < fill ? need : fill;
    return g ? g : 1u;
}
inline uint32_t map_grid(uint32_t maxseg) { return (maxseg + rle::kMapBlock - 1) / rle::kMapBlock; }
inline uint32_t buf_grid(uint32_t n) { return (n + rle::kSegWaves - 1) / rle::kSegWaves; }
// the fused single-pass encode (RLE_MI355X_SEG_FUSED=1; measured slower than the four launches, §4)
[[maybe_unused]] bool seg_fused() {
    if (!RLE_VARIANTS) return false;   // (product build: RLE_MI355X_SEG_FUSED is not read)
    static const bool on = [] {
        const char* e = getenv("RLE_MI355X_SEG_FUSED");
        return e ? e[0] != '0' : false;
    }();
    return on;
}
}  // namespace

extern "C" size_t rle_seg_workspace_bytes(uint32_t n, uint64_t total_in_bytes) {
    int ncu = 0;
    if (device_cus(&ncu) != RLE_OK) ncu = 256;
    const uint32_t sb = seg_bytes(total_in_bytes, ncu);
    return carve(nullptr, n, max_segments(n, total_in_bytes, sb)).bytes;
}

extern "C" int rle_encode_batch_device_seg(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                           void* d_out, const uint64_t* d_out_off, uint64_t* d_out_len,
                                           uint32_t* d_status, uint32_t n, uint64_t total_in_bytes, void* d_workspace,
                                           size_t workspace_bytes, void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return RLE_E_INVAL;
    const hipStream_t s = (hipStream_t)stream;
    int ncu = 0;
    if (const int rc = device_cus(&ncu)) return rc;
    const uint32_t sb = seg_bytes(total_in_bytes, ncu);
    const uint32_t maxseg = max_segments(n, total_in_bytes, sb);
    const Carve w = carve(static_cast<char*>(d_workspace), n, maxseg);
    if (!d_workspace || workspace_bytes < w.bytes) return RLE_E_INVAL;
    const uint8_t* in = (const uint8_t*)d_in;
    uint8_t* out = (uint8_t*)d_out;
#if RLE_VARIANTS
    if (seg_res()) {   // (the plan clears the status words: the segments OR into them)
        hipLaunchKernelGGL(rle::seg_plan_kernel, dim3(1), dim3(1024), 0, s, d_in_len, n, sb, w.seg_first, w.sflag,
                           maxseg, w.ticket, d_status);
        hipLaunchKernelGGL(rle::seg_map_kernel, dim3(map_grid(maxseg)), dim3(rle::kMapBlock), 0, s, w.seg_first, n,
                           maxseg, w.seg_buf);
        hipLaunchKernelGGL(rle::enc_seg_res_kernel, dim3(buf_grid(maxseg)),
                           dim3(rle::kSegBlock), 0, s, in,
                           d_in_off, d_in_len, out, d_out_off, d_out_len, d_status, n, w.seg_first, w.seg_buf, maxseg,
                           sb, w.summ, w.incl, w.sflag, w.ticket);
        return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
    }
    if (seg_fused()) {   // (the plan clears the status words: the segments OR into them)
        hipLaunchKernelGGL(rle::seg_plan_kernel, dim3(1), dim3(1024), 0, s, d_in_len, n, sb, w.seg_first, w.sflag,
                           maxseg, w.ticket, d_status);
        hipLaunchKernelGGL(rle::enc_seg_fused_kernel, dim3(seg_grid(maxseg, ncu)), dim3(rle::kSegBlock), 0, s, in,
                           d_in_off, d_in_len, out, d_out_off, d_out_len, d_status, n, w.seg_first, maxseg, sb, w.summ,
                           w.incl, w.sflag, w.ticket);
        return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
    }
#endif
    const uint32_t grid = seg_grid(maxseg, ncu);
    // one buffer: no plan / map launches, the kernels take its segments from its length
    const bool one = n == 1u;
    uint32_t* const seg_first = one ? nullptr : w.seg_first;
    uint32_t* const seg_buf = one ? nullptr : w.seg_buf;
    if (!one) {
        hipLaunchKernelGGL(rle::seg_plan_kernel, dim3(1), dim3(1024), 0, s, d_in_len, n, sb, w.seg_first, nullptr, 0u,
                           nullptr, nullptr);
        hipLaunchKernelGGL(rle::seg_map_kernel, dim3(map_grid(maxseg)), dim3(rle::kMapBlock), 0, s, w.seg_first, n,
                           maxseg, w.seg_buf);
    }
    hipLaunchKernelGGL(rle::enc_seg_summary_kernel, dim3(grid), dim3(rle::kSegBlock), 0, s, in, d_in_off, d_in_len, n,
                       seg_first, seg_buf, maxseg, sb, w.summ);
    hipLaunchKernelGGL(rle::enc_seg_scan_kernel, dim3(buf_grid(n)), dim3(rle::kSegBlock), 0, s, in, d_in_off, d_in_len,
                       out, d_out_off, d_out_len, d_status, n, seg_first, maxseg, sb, w.summ, w.plan, w.bflag);
    hipLaunchKernelGGL(rle::enc_seg_write_kernel, dim3(grid), dim3(rle::kSegBlock), 0, s, in, d_in_off, d_in_len, out,
                       d_out_off, n, seg_first, seg_buf, maxseg, sb, w.plan, w.bflag, w.summ);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

extern "C" int rle_decode_batch_device_seg(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                           void* d_out, const uint64_t* d_out_off, const uint64_t* d_out_len,
                                           const uint64_t* d_out_cap, uint32_t* d_status, uint32_t n,
                                           uint64_t total_in_bytes, void* d_workspace, size_t workspace_bytes,
                                           void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return RLE_E_INVAL;
    const hipStream_t s = (hipStream_t)stream;
    int ncu = 0;
    if (const int rc = device_cus(&ncu)) return rc;
    const uint32_t sb = seg_bytes(total_in_bytes, ncu);
    const uint32_t maxseg = max_segments(n, total_in_bytes, sb);
    const Carve w = carve(static_cast<char*>(d_workspace), n, maxseg);
    if (!d_workspace || workspace_bytes < w.bytes) return RLE_E_INVAL;
    const uint8_t* in = (const uint8_t*)d_in;
    uint8_t* out = (uint8_t*)d_out;
#if RLE_VARIANTS
    if (seg_res_mode() == 1 || seg_res_mode() == 2) {
        hipLaunchKernelGGL(rle::seg_plan_kernel, dim3(1), dim3(1024), 0, s, d_in_len, n, sb, w.seg_first, w.sflag,
                           maxseg, w.ticket, w.bflag);
        hipLaunchKernelGGL(rle::seg_map_kernel, dim3(map_grid(maxseg)), dim3(rle::kMapBlock), 0, s, w.seg_first, n,
                           maxseg, w.seg_buf);
        hipLaunchKernelGGL(seg_res_mode() == 1 ? rle::dec_seg_res_kernel<true> : rle::dec_seg_res_kernel<false>,
                           dim3(buf_grid(maxseg)),
                           dim3(rle::kSegBlock), 0, s, in,
                           d_in_off, d_in_len, out, d_out_off, d_out_len, d_out_cap, d_status, n, w.seg_first,
                           w.seg_buf, maxseg, sb, w.summ, w.incl, w.sflag, w.ticket, w.bflag);
        hipLaunchKernelGGL(rle::dec_seg_serial_kernel, dim3(buf_grid(n)), dim3(rle::kSegBlock), 0, s, in, d_in_off,
                           d_in_len, out, d_out_off, d_out_len, d_out_cap, d_status, n, w.bflag);
        return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
    }
#endif
    const uint32_t grid = seg_grid(maxseg, ncu);
    const bool one = n == 1u;   // (as in the encode: no plan / map launches for one buffer)
    uint32_t* const seg_first = one ? nullptr : w.seg_first;
    uint32_t* const seg_buf = one ? nullptr : w.seg_buf;
    if (!one) {
        hipLaunchKernelGGL(rle::seg_plan_kernel, dim3(1), dim3(1024), 0, s, d_in_len, n, sb, w.seg_first, nullptr, 0u,
                           nullptr, nullptr);
        hipLaunchKernelGGL(rle::seg_map_kernel, dim3(map_grid(maxseg)), dim3(rle::kMapBlock), 0, s, w.seg_first, n,
                           maxseg, w.seg_buf);
    }
    hipLaunchKernelGGL(rle::dec_seg_summary_kernel, dim3(grid), dim3(rle::kSegBlock), 0, s, in, d_in_off, d_in_len, n,
                       seg_first, seg_buf, maxseg, sb, w.summ);
    hipLaunchKernelGGL(rle::dec_seg_scan_kernel, dim3(buf_grid(n)), dim3(rle::kSegBlock), 0, s, in, d_in_off, d_in_len,
                       out, d_out_off, d_out_len, d_out_cap, d_status, n, seg_first, maxseg, sb, w.summ, w.plan, w.bflag);
    const bool one_round = maxseg <= (uint32_t)ncu * 16u;   // the 192-chunk kernel's residency
    hipLaunchKernelGGL(one_round ? rle::dec_seg_write_kernel<rle::kSegDecChunksOne>
                                 : rle::dec_seg_write_kernel<rle::kSegDecChunksMany>,
                       dim3(grid), dim3(rle::kSegBlock), 0, s, in, d_in_off, d_in_len, out, d_out_off, d_out_len,
                       d_out_cap, d_status, n, seg_first, seg_buf, maxseg, sb, w.plan, w.bflag, w.summ);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}
