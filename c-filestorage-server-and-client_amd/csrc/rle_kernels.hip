// rle_kernels.hip — MI355X (gfx950, CDNA4) RLE codec: the batch kernels (one wave64 per buffer)
// and the C ABI of include/rle_mi355x.h for them.  Device building blocks: rle_device.h.
#include "rle_device.h"

#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>

namespace rle {

constexpr u32 kXcds = 8;
// Buffer of wave `wid` of workgroup `wg` when every XCD (workgroups are dealt to the 8 XCDs
// round-robin) takes a contiguous slice of the batch instead of every 8th buffer: a batch whose
// cost varies with a stride (e.g. i % 4) then still spreads evenly over the XCDs.
__device__ __forceinline__ u32 xcd_buffer(u32 wg, u32 ngrid, u32 waves, u32 wid) {
    const u32 per = ngrid / kXcds;   // launcher makes ngrid a multiple of 8
    return ((wg % kXcds) * per + wg / kXcds) * waves + wid;
}

#define RLE_NOWALK ((RLE_ABL & 128) != 0)   // fixed-cost probe builds only (wrong output): no tiles walked


// Diagnostic timeline builds (RLE_TIMELINE=1, never the product library): lane 0 of the wave of
// buffer b < kTlWaves records s_memrealtime (100 MHz) at kernel entry [0], walk start [1], the start
// of each of its first 8 tiles [2..9] and the end [10], plus HW_ID [11] and XCC_ID [12];
// rle_mi355x_timeline() reads them.
#ifndef RLE_TIMELINE
#define RLE_TIMELINE 0
#endif
#if RLE_TIMELINE
constexpr u32 kTlWaves = 16384, kTlEv = 16;
static __device__ unsigned long long g_tl[kTlWaves * kTlEv];
__device__ __forceinline__ void tl_mark(u32 b, u32 ev, u32 lane) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (lane == 0u && b < kTlWaves && ev < kTlEv) g_tl[b * kTlEv + ev] = t;
}
__device__ __forceinline__ unsigned long long tl_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void tl_put(u32 b, u32 ev, unsigned long long t, u32 lane) {
    if (lane == 0u && b < kTlWaves) g_tl[b * kTlEv + ev] = t;
}
__device__ __forceinline__ void tl_ids(u32 b, u32 lane) {
    const u32 hw = (u32)__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_ID
    const u32 xcc = (u32)__builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // XCC_ID
    if (lane == 0u && b < kTlWaves) {
        g_tl[b * kTlEv + 11] = hw;
        g_tl[b * kTlEv + 12] = xcc;
    }
}
#else
__device__ __forceinline__ unsigned long long tl_now() { return 0; }
__device__ __forceinline__ void tl_put(u32, u32, unsigned long long, u32) {}
__device__ __forceinline__ void tl_mark(u32, u32, u32) {}
__device__ __forceinline__ void tl_ids(u32, u32) {}
#endif

#ifndef RLE_ENC_WAVES
#define RLE_ENC_WAVES 4
#endif
constexpr u32 kEncWaves = RLE_ENC_WAVES;
#ifndef RLE_ENC_SMALL   // largest buffer encoded in 1024-byte tiles
#define RLE_ENC_SMALL 16384
#endif
constexpr u32 kEncSmall = RLE_ENC_SMALL;
constexpr u32 kEncBlock = kWave * kEncWaves;
// kWtMode: the output store policy fixed at compile time (1 write-through, 2 write-back; 0 the launch
// flag's bit 0 at run time), so that the tile steps carry no branch around each store (round 5).
// Two tile slots per wave (kDepth, the instantiation names of the profiles; deeper rings measured no
// faster).
template <u32 kDepth = 2u, u32 kWtMode = 0u>
__global__ __launch_bounds__(kEncBlock) void encode_kernel(const uint8_t* __restrict__ in,
                                                           const uint64_t* __restrict__ in_off,
                                                           const uint64_t* __restrict__ in_len,
                                                           uint8_t* __restrict__ out,
                                                           const uint64_t* __restrict__ out_off,
                                                           uint64_t* __restrict__ out_len,
                                                           uint32_t* __restrict__ status, uint32_t n, uint32_t wt) {
    const unsigned long long tl0 = tl_now();
    static_assert(kDepth == 2u, "two tile slots per wave");
    constexpr u32 kSlotsB = 2u * kEncSlot;
    __shared__ __attribute__((aligned(16))) uint8_t slots_all[kEncWaves * kSlotsB];
    __shared__ __attribute__((aligned(16))) uint8_t stage_all[kEncWaves * kEncStage];
    __shared__ __attribute__((aligned(16))) u32 elut_all[kEncWaves * kInsWaveWords];
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    uint8_t* stage = stage_all + wid * kEncStage;
    const uint8_t* slots = slots_all + wid * kSlotsB;
    const u32 b = xcd_buffer(blockIdx.x, gridDim.x, kEncWaves, wid);
    if (b >= n) return;
    tl_mark(b, 0, lane);
    tl_put(b, 13, tl0, lane);
    tl_ids(b, lane);
    const uint64_t U64 = in_len[b], ioff = in_off[b], ooff = out_off[b];
    __builtin_amdgcn_sched_barrier(0);   // the three loads in flight together (as in decode_kernel)
    const uint8_t* src = in + ioff;
    uint8_t* dst = out + ooff;
    u32 bad = (((uintptr_t)src | (uintptr_t)dst) & 15u) ? RLE_STATUS_MISALIGNED : 0u;
    if (U64 > kMaxBufferBytes) bad |= RLE_STATUS_TOOLARGE;
    if (bad) {
        if (lane == 0) {
            out_len[b] = 0;
            put_status(status, b, bad, wt);
        }
        return;
    }
    // this wave's copy of the insertion selectors (enc_tile_fast), by LDS-DMA ahead of the first
    // tile's: loads complete in issue order, so walk_tiles' wait for tile 0 covers it (no tile, no
    // load: nothing may land in LDS after the wave ends)
    const u32* elut = elut_all + wid * kInsWaveWords;
    if (U64 != 0u && !RLE_NOWALK && lane < kInsDmaLanes)
        dma_tile(make_rsrc(&kEncInsLut, 4u * kInsWaveWords), 16u * lane, uniform(lds_addr(elut)));
    const u32 U = (u32)U64;
    const u32x4 rsi = make_rsrc(src, (U + 15u) & ~15u);
    const u32x4 rso = make_rsrc(dst, U + U / 2u);
    EncState st{0u, 0u, 0u, 0u, 0u, kWtMode ? kWtMode == 1u : (wt & kLaunchWt) != 0u, {}};
    const EncK kc = enc_k();
#if RLE_STAMPS
    for (u32 k = 0; k < kStampSegs; ++k) st.sp.acc[k] = 0;
    st.sp.last = memtime();
#endif
    tl_mark(b, 1, lane);
    // 1024-byte tiles where they save a tile, up to kEncSmall (rle_device.h, enc_tile<true>)
    if (enc_ntiles_for(U) < ntiles_for(U) && U <= kEncSmall) {
        // two tiles per step (rle_device.h enc_pair)
        walk_pairs<kEncStep, true>(rsi, 0u, RLE_NOWALK ? 0u : enc_ntiles_for(U), lane, slots,
                   [&](u32 t, const uint8_t* sa, const uint8_t* sb, const Refill& na, const Refill& nb) {
                       tl_mark(b, 2u + t, lane);
                       tl_mark(b, 3u + t, lane);
                       return enc_pair<true>(sa, sb, na, nb, t * kEncStep, U, lane, stage, dst, rso, st, kc, elut);
                   },
                   [&](u32 t, const uint8_t* cs, const Refill& nx) {
                       tl_mark(b, 2u + t, lane);
                       return enc_tile<true, true>(cs, nx, t * kEncStep, U, U, lane, stage, dst, rso, st, kc, elut);
                   });
    } else {
        auto tile = [&](u32 t, const uint8_t* cs, const Refill& nx) {
            tl_mark(b, 2u + t, lane);
            return enc_tile<false, true>(cs, nx, t * kTileStep, U, U, lane, stage, dst, rso, st, kc, elut);
        };
        walk_tiles(rsi, 0u, RLE_NOWALK ? 0u : ntiles_for(U), lane, slots, tile);
    }
    RLE_STAMP(st.sp, 6);   // drain
    // the final partial chunk (< 16 bytes, staging chunk 1): byte stores, nothing past C
    if (lane < st.out_pos - st.flushed) dst[st.flushed + lane] = stage[16u + lane];
    if (lane == 0) {
        out_len[b] = st.out_pos;
        put_status(status, b, RLE_STATUS_OK, wt);
    }
    tl_mark(b, 10, lane);
    RLE_STAMP(st.sp, 7);   // finish
#if RLE_STAMPS
    if (lane == 0) {
        for (u32 k = 0; k < kStampSegs; ++k) atomicAdd(&g_stamps[k], (unsigned long long)st.sp.acc[k]);
        atomicAdd(&g_stamps[kStampSegs], 1ull);
    }
#endif
}

// ================================================================ DECODE (one wave per buffer)
#ifndef RLE_DEC_WAVES
#define RLE_DEC_WAVES 4
#endif
// Waves per workgroup: with one, the dispatcher starts the next buffer as soon as any wave ends,
// so short (highly compressed) and long buffers balance without a software queue.
constexpr u32 kDecWaves = RLE_DEC_WAVES;
constexpr u32 kDecBlock = kWave * kDecWaves;
// Issue order of a large decode batch (longest first): buffer indices sorted by descending tile
// count, a counting sort over kOrderBuckets clamped keys.  Heavy buffers then start in the first
// residency round, and the four waves of a workgroup, which hold its LDS until the last one ends,
// get buffers of similar cost.  Outputs do not depend on the order.
//
// One launch, no global counts (round 5): each workgroup sorts its own kLocalChunk buffers longest
// first (its LDS histogram, a descending scan of it, each buffer's place = its bucket's start + its
// rank in the bucket) into order[chunk * kLocalChunk ...], and the decode kernel interleaves the
// F = n / kLocalChunk full chunks (slot s takes place s / F of chunk s % F; the last partial chunk
// follows them): the i-th heaviest buffers of every chunk are issued together, which on batches
// whose chunks hold similar mixes (every bench and server batch) is the global longest-first order.
// Ties inside a bucket fall in LDS-atomic order, which scatters the concurrently issued buffers'
// offsets.  Measured and not kept: a global histogram + scatter in two launches
// (r5t: -1.8 % on dec64k without them), ties in index order or groups of consecutive places
// (+4-8 %: same-rank buffers of every chunk at a 16 MiB stride pile onto the same channels), ranks
// permuted per chunk, larger chunks (512-2048 buffers), each XCD walking its own slice, the
// metadata copied into issue order (all within +-1 % or slower).
constexpr u32 kOrderBuckets = 2048;
__device__ __forceinline__ u32 order_key(uint64_t C) {
    const uint64_t t = (C + kTileStep - 1u) / kTileStep;
    return t < kOrderBuckets - 1u ? (u32)t : kOrderBuckets - 1u;
}
// The lanes of a wave that share a key make one atomic: per distinct key, the first such lane adds
// the group's size, and each lane's place is the group's base plus its rank in the group (a
// uniform batch: one atomic per wave).  All 64 lanes call it; `on` marks the lanes with an item.
__device__ __forceinline__ u32 grouped_add(u32* hist, u32 key, bool on, u32 lane) {
    const uint64_t lt = (1ull << lane) - 1ull;
    u32 pos = 0u;
    uint64_t todo = __builtin_amdgcn_ballot_w64(on);
    while (todo) {
        const u32 lead = (u32)__builtin_ctzll(todo);
        const u32 kl = readlane(key, lead);
        const uint64_t grp = __builtin_amdgcn_ballot_w64(on && key == kl);
        u32 base = 0u;
        if (lane == lead) base = atomicAdd(&hist[kl], (u32)__builtin_popcountll(grp));
        base = readlane(base, lead);
        if ((grp >> lane) & 1ull) pos = base + (u32)__builtin_popcountll(grp & lt);
        todo &= ~grp;
    }
    return pos;
}
constexpr u32 kLocalPer = 1u, kLocalChunk = 256u * kLocalPer;   // buffers per thread / per workgroup
// The chunk's keys, its LDS histogram and each buffer's rank in its bucket.
__device__ __forceinline__ void order_local(const uint64_t* in_len, uint32_t n, u32* lh, u32 (&key)[kLocalPer],
                                            u32 (&rank)[kLocalPer]) {
    constexpr u32 kPer = kLocalPer;
    const u32 t = threadIdx.x, lane = t & (kWave - 1);
    // the lengths' loads first, so their latency overlaps the histogram's zeroing and barrier
    const u32 i0 = blockIdx.x * (256u * kPer) + t;
    uint64_t len[kPer];   // (every lane loads, index clamped: no branch, the wait lands at the first use)
#pragma unroll
    for (u32 j = 0; j < kPer; ++j) len[j] = in_len[i0 + 256u * j < n ? i0 + 256u * j : n - 1u];
    for (u32 k = t; k < kOrderBuckets; k += 256u) lh[k] = 0u;
    __syncthreads();
#pragma unroll
    for (u32 j = 0; j < kPer; ++j) key[j] = i0 + 256u * j < n ? order_key(len[j]) : 0u;
#pragma unroll
    for (u32 j = 0; j < kPer; ++j) rank[j] = grouped_add(lh, key[j], i0 + 256u * j < n, lane);
    __syncthreads();
}
__global__ __launch_bounds__(256) void dec_order_local_kernel(const uint64_t* __restrict__ in_len, uint32_t n,
                                                              uint32_t* __restrict__ order) {
    __shared__ u32 lh[kOrderBuckets];
    __shared__ u32 wsum[4];
    constexpr u32 kPerT = kOrderBuckets / 256u;
    const u32 t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
    u32 key[kLocalPer], rank[kLocalPer];
    order_local(in_len, n, lh, key, rank);   // (ends with a barrier: lh holds the chunk's counts)
    // thread t: the 8 buckets from B-1-8t down, in descending bucket order
    u32 c[kPerT], sum = 0u;
#pragma unroll
    for (u32 j = 0; j < kPerT; ++j) {
        c[j] = lh[kOrderBuckets - 1u - (kPerT * t + j)];
        sum += c[j];
    }
    const u32 incl = wave_scan_incl(sum, 0u, OpAdd());
    if (lane == kWave - 1) wsum[wv] = incl;
    __syncthreads();   // (every thread has read its counts: lh may be overwritten below)
    u32 base = incl - sum;
    for (u32 w = 0; w < wv; ++w) base += wsum[w];
#pragma unroll
    for (u32 j = 0; j < kPerT; ++j) {
        lh[kOrderBuckets - 1u - (kPerT * t + j)] = base;
        base += c[j];
    }
    __syncthreads();
    const u32 i0 = blockIdx.x * kLocalChunk + threadIdx.x;
#pragma unroll
    for (u32 j = 0; j < kLocalPer; ++j) {
        const u32 i = i0 + 256u * j;
        if (i >= n) continue;
        order[blockIdx.x * kLocalChunk + lh[key[j]] + rank[j]] = i;
    }
}
// The buffer a decode wave takes at issue slot s of an order made by dec_order_local_kernel.
__device__ __forceinline__ u32 order_slot_local(u32 s, u32 n) {
    const u32 F = n / kLocalChunk;   // full chunks, interleaved; the partial one after them
    if (s >= F * kLocalChunk) return s;
    return (s % F) * kLocalChunk + s / F;   // slot s takes place s / F of chunk s % F
}

// kChunks: staging chunks per wave (32 B each).  192 hold any tile's output in one pass; the
// launcher takes 96 (3 KiB per wave: 7 workgroups per CU instead of 4) for batches past one
// residency round, where the extra waves hide more latency than the two-pass staging of the
// output-heavy tiles costs.
// Two tile slots per wave (walk_tiles).  Measured and not kept: 3 / 4 slots in the
// large-batch kernel (r5c: 64 KiB runs50 / runs90 +4-6 %, dec64k +1.2 / +1.7 %), 8 slots for the
// drop-in's single calls (r5e: no faster from 4 KiB to 128 KiB: a lone wave's walk is bound by its
// tiles' dependent chains, not by loads in flight).  The uniform-tile test (dec_uniform_tile, gated:
// tried only after a single-value tile) runs in both kernels.  (kDepthT: kept 0, the instantiation
// names of the profiles.)
template <u32 kChunks, u32 kDepthT = 0u, u32 kWtMode = 0u>   // (kWtMode: as encode_kernel's)
__global__ __launch_bounds__(kDecBlock) void decode_kernel(const uint8_t* __restrict__ in,
                                                           const uint64_t* __restrict__ in_off,
                                                           const uint64_t* __restrict__ in_len,
                                                           uint8_t* __restrict__ out,
                                                           const uint64_t* __restrict__ out_off,
                                                           const uint64_t* __restrict__ out_len,
                                                           const uint64_t* __restrict__ out_cap,
                                                           uint32_t* __restrict__ status, uint32_t n, uint32_t wt,
                                                           const uint32_t* __restrict__ order) {
    const unsigned long long tl0 = tl_now();
    static_assert(kDepthT == 0u, "two tile slots per wave");
    constexpr u32 kDepth = 2u;
    __shared__ __attribute__((aligned(16))) uint8_t slots_all[kDecWaves * kDepth * kSlot];
    constexpr u32 kStageB = 32u * kChunks;
    __shared__ __attribute__((aligned(128))) uint8_t stage_all[kDecWaves * kStageB];
    __shared__ __attribute__((aligned(16))) DecEntry tbl[256];
    __shared__ u32x4 clut[kCompactEntries];
#ifdef RLE_LDS_PAD   // occupancy experiments only
    __shared__ uint8_t ldspad[RLE_LDS_PAD];
    if (threadIdx.x == 0) ((volatile uint8_t*)ldspad)[0] = 0;
#endif
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    // with an issue order, workgroups take its ranks in dispatch order (the heavy buffers first,
    // spread over every XCD); else each XCD takes a contiguous slice of the batch
    // (Measured and not kept, DESIGN.md §4: heavy / light workgroup blocks or waves alternating, the
    // order ignored, each XCD walking its own slice, the metadata copied into issue order.)
    u32 b;
    if (order) {
        u32 slot = blockIdx.x * kDecWaves + wid;
        if (slot < n) slot = uniform(order_slot_local(slot, n));
        b = slot < n ? uniform(order[slot]) : n;
    } else {
        b = xcd_buffer(blockIdx.x, gridDim.x, kDecWaves, wid);
    }
    // all five per-buffer words are loaded at once, unconditionally (index clamped; n >= 1)
    const u32 bi = b < n ? b : 0u;
    const uint64_t* capp = out_cap ? out_cap : out_len;
    const uint64_t C64 = in_len[bi], U64 = out_len[bi], cap = capp[bi], ioff = in_off[bi], ooff = out_off[bi];
    tl_mark(b, 0, lane);
    tl_put(b, 13, tl0, lane);
    tl_ids(b, lane);
    // all five loads in flight before the first use (else hipcc waits for in_off before issuing the
    // other four: two memory round trips ahead of the first tile's DMA instead of one)
    __builtin_amdgcn_sched_barrier(0);
    const uint8_t* src = in + ioff;
    uint8_t* dst = out + ooff;
    u32 bad = ((((uintptr_t)src | (uintptr_t)dst) & 15u) || cap < U64) ? RLE_STATUS_MISALIGNED : 0u;
    if (C64 > kMaxBufferBytes || U64 > kMaxBufferBytes) bad |= RLE_STATUS_TOOLARGE;
    const u32 C = (u32)C64, U = (u32)U64;
    const u32x4 rsi = make_rsrc(src, (C + 15u) & ~15u);
    const u32 ntiles = (b < n && !bad && !RLE_NOWALK) ? ntiles_for(C) : 0u;
    tl_mark(b, 14u + 0u * ntiles, lane);   // (diagnostic builds: the metadata has arrived)
    // Issue priority by walk length (log2 buckets of the tile count): where a SIMD holds waves of
    // unequal walks, the longest are the launch's critical path, and the short ones fill their
    // stalls: the one-round kernel (kChunks >= 191) only (every size measured within +-1 %, r5ah).
    if (kChunks >= 191u) {
        if (ntiles >= 32u) __builtin_amdgcn_s_setprio(3);
        else if (ntiles >= 8u) __builtin_amdgcn_s_setprio(2);
        else if (ntiles >= 3u) __builtin_amdgcn_s_setprio(1);
    }
    uint8_t* stage = stage_all + wid * kStageB;
    const uint8_t* slots = slots_all + wid * kDepth * kSlot;
    // The phase table and the compaction selectors, shared by the workgroup: wave 0 LDS-DMAs them
    // (2.3 KB) after every wave has issued its first tiles' loads, waits for its own table loads
    // (they complete in issue order, its tile loads after them may still be in flight), and one
    // barrier publishes them, normally before the first tile's data has landed.  (At kernel start
    // every wave's loads queue at once: one copy per workgroup instead of per wave keeps the
    // table traffic off the first tiles' path.)
    walk_prime(rsi, 0u, ntiles, lane, slots);
    tl_mark(b, 15, lane);   // (diagnostic builds: the first tiles' loads issued)
    if (wid == 0u) {
        const u32x4 rt = make_rsrc(&kDecTable, (u32)sizeof(DecTable));
        const u32 lt = uniform(lds_addr(tbl));
        asm volatile("s_nop 4" ::: "memory");   // descriptor words may be fresh
        dma_tile(rt, 16u * lane, lt);
        dma_tile(rt, 1024u + 16u * lane, lt + 1024u);
        if (lane < kCompactEntries)
            dma_tile(make_rsrc(&kCompactLut, (u32)sizeof(DecCompactLut)), 16u * lane, uniform(lds_addr(clut)));
    }
    for (u32 k = lane; k < kStageB / 16u; k += kWave)
        reinterpret_cast<u32x4*>(stage)[k] = u32x4{0u, 0u, 0u, 0u};
    if (wid == 0u) vm_drain();   // (its own tile loads were issued first: both are in)
    if (kDecWaves > 1) __syncthreads();
    else wave_lds_sync();

    if (b < n) {
        if (bad) {
            if (lane == 0) put_status(status, b, bad, wt);
            return;
        }
        const u32x4 rso = make_rsrc(dst, U);
        DecState st{0u, 0u, 0u, 0u, 0u, 0u, 0u, kWtMode ? kWtMode == 1u : (wt & kLaunchWt) != 0u, {}};
        const DecK kc = dec_k();
#if RLE_STAMPS
        for (u32 k = 0; k < kStampSegs; ++k) st.sp.acc[k] = 0;
        st.sp.last = memtime();
#endif
        tl_mark(b, 1, lane);
        auto tile = [&](u32 t, const uint8_t* cs, const Refill& nx) {
            tl_mark(b, 2u + t, lane);
            return dec_tile<true, kChunks, true>(cs, nx, t * kTileStep, C, C, U, lane, tbl, stage, dst, rso, st, kc, clut);
        };
        const bool serial = walk_tiles(rsi, 0u, ntiles, lane, slots, tile, true);
        RLE_STAMP(st.sp, 7);   // drain after the last tile
        u32 stat = RLE_STATUS_OK;
        if (serial) stat = dec_serial(src, C, U, cap, dst, lane, stage, kStageB);
        else {
            dec_finish(st, U, lane, stage, rso, dst);
            stat = dec_tiled_status(st, U);
        }
        RLE_STAMP(st.sp, 7);   // finish
#if RLE_STAMPS
        if (lane == 0) {
            for (u32 k = 0; k < kStampSegs; ++k) atomicAdd(&g_stamps[k], (unsigned long long)st.sp.acc[k]);
            atomicAdd(&g_stamps[kStampSegs], 1ull);
        }
#endif
        if (lane == 0) put_status(status, b, stat, wt);
        tl_mark(b, 10, lane);
    }
}

}  // namespace rle
#include "rle_round.h"   // the large-batch decode in rounds (dec_round_kernel)
namespace rle {

// ================================================================ synthetic generator
__device__ __forceinline__ uint64_t xs64(uint64_t& s) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    return s;
}

__global__ void gen_kernel(uint8_t* __restrict__ out, const uint64_t* __restrict__ off,
                           const uint64_t* __restrict__ len, const uint32_t* __restrict__ kind,
                           const uint64_t* __restrict__ index, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = kind ? kind[i] : 1u;
    uint64_t s = 0x9E3779B97F4A7C15ull + (index ? index[i] : (uint64_t)i);
    uint8_t* p = out + off[i];
    const uint64_t U = len[i];
    uint32_t acc = 0, prev = 0;
    const uint32_t P = k == 2 ? 50u : 90u;
    for (uint64_t q = 0; q < U; ++q) {
        uint32_t v;
        if (k == 0) v = 0;
        else if (k == 1) v = (uint32_t)xs64(s) & 0xFFu;
        else if (k == 2 || k == 3) {
            const uint64_t r = xs64(s);
            v = (q > 0 && (uint32_t)((r >> 32) % 100u) < P) ? prev : (uint32_t)r & 0xFFu;
        } else {
            if ((q & 1u) == 0) {
                v = (uint32_t)xs64(s) & 0xFFu;
                if (q > 0 && v == prev) v ^= 1u;
            } else {
                v = prev;
            }
        }
        prev = v;
        acc |= v << (8u * (uint32_t)(q & 3u));
        if ((q & 3u) == 3u) {
            *reinterpret_cast<uint32_t*>(p + (q & ~3ull)) = acc;
            acc = 0;
        }
    }
    for (uint64_t q = U & ~3ull; q < U; ++q) p[q] = (uint8_t)(acc >> (8u * (uint32_t)(q & 3u)));
}

// ================================================================ the decode's memory pattern (measurement only)
// bench.py's second north-star ceiling: the large-batch decode's memory traffic without its token
// work.  Each wave streams its buffer's C bytes in through decode_kernel's tile walk (1 KiB LDS-DMA
// tiles, two in flight, walk_tiles) and writes its U bytes out in 16-byte-per-lane stores, each tile
// taking its share of the output; workgroups, LDS (7 per CU) and the issue order as decode_kernel<96>.
// Not the codec: the output bytes are the tiles' bytes repeated.  Each tile's share ends on a
// 16-byte chunk, as the decode's stores do (128-byte shares measured 3 % faster, lanes shifted onto
// lines 0.6-1.1 %: r5ap / r5aq).
constexpr u32 kPatternPad = kDecWaves * 32u * 96u + (u32)sizeof(DecTable) + kCompactEntries * 16u;
__global__ __launch_bounds__(kDecBlock) void pattern_kernel(const uint8_t* __restrict__ in,
                                                            const uint64_t* __restrict__ in_off,
                                                            const uint64_t* __restrict__ in_len,
                                                            uint8_t* __restrict__ out,
                                                            const uint64_t* __restrict__ out_off,
                                                            const uint64_t* __restrict__ out_len, uint32_t n,
                                                            const uint32_t* __restrict__ order) {
    __shared__ __attribute__((aligned(16))) uint8_t slots_all[kDecWaves * 2u * kSlot];
    __shared__ uint8_t pad[kPatternPad];   // decode_kernel<96>'s staging, table and selectors: its occupancy
    const u32 lane = threadIdx.x & (kWave - 1);
    const u32 wid = uniform(threadIdx.x / kWave);
    if (threadIdx.x == 0) ((volatile uint8_t*)pad)[blockIdx.x % kPatternPad] = 0;
    u32 b;
    if (order) {
        const u32 slot = blockIdx.x * kDecWaves + wid;
        const u32 place = slot < n ? order_slot_local(slot, n) : n;
        b = place < n ? uniform(order[uniform(place)]) : n;
    } else {
        b = xcd_buffer(blockIdx.x, gridDim.x, kDecWaves, wid);
    }
    b = uniform(b);
    if (b >= n) return;
    auto u64 = [](uint64_t x) { return (uint64_t)uniform((u32)x) | ((uint64_t)uniform((u32)(x >> 32)) << 32); };
    const uint64_t C64 = u64(in_len[b]), U64 = u64(out_len[b]), ioff = u64(in_off[b]), ooff = u64(out_off[b]);
    if (C64 > kMaxBufferBytes || U64 > kMaxBufferBytes) return;
    const u32 C = (u32)C64, U = (u32)U64;
    const uint8_t* src = in + ioff;
    uint8_t* dst = out + ooff;
    if (((uintptr_t)src | (uintptr_t)dst) & 15u) return;
    const u32x4 rsi = make_rsrc(src, (C + 15u) & ~15u);
    const u32x4 rso = make_rsrc(dst, U);
    const uint8_t* slots = slots_all + wid * 2u * kSlot;
    const u32 ntiles = ntiles_for(C);
    u32 written = 0;
    walk_tiles(rsi, 0u, ntiles, lane, slots, [&](u32 t, const uint8_t* cs, const Refill& nx) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(cs + 16u * lane);
        nx();
        const u32 upto = t + 1u == ntiles ? U : (u32)(((uint64_t)(t + 1u) * U / ntiles) & ~(uint64_t)15u);
        u32 k = 0;
        const u32 nst = upto > written ? (upto - written + 16u * kWave - 1u) / (16u * kWave) : 0u;
        for (; k < nst; ++k) {
            const u32 a = written + 16u * (k * kWave + lane);
            vstore(rso, a >= written && a < upto ? a : kOOB, v, false);
        }
        written = upto;
        return k;
    });
}

// ================================================================ streaming copy (measurement only)
// bench.py's practical ceiling: HBM to HBM at 16 bytes per lane, four loads in
// flight per lane before their stores, grid-strided over a chip-filling grid.  Not part of the codec.
template <bool kNt>
__global__ __launch_bounds__(256) void copy_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 1024u;
    for (uint64_t base = (uint64_t)blockIdx.x * 1024u + threadIdx.x; base < n16; base += stride) {
        u32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t i = base + 256u * q;
            if (i < n16) v[q] = kNt ? __builtin_nontemporal_load(src + i) : src[i];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t i = base + 256u * q;
            if (i < n16) {
                if (kNt) __builtin_nontemporal_store(v[q], dst + i);
                else dst[i] = v[q];
            }
        }
    }
}

// ================================================================ DPP self-test
__global__ void selftest_kernel(uint32_t* err) {
    __shared__ uint32_t v[64];
    const uint32_t lane = threadIdx.x;
    const uint32_t x = (lane * 2654435761u) >> 7;
    v[lane] = x;
    __syncthreads();
    uint32_t e = 0;
    const uint32_t prev = from_prev_lane(x, 12345u), next = from_next_lane(x, 54321u);
    if (prev != (lane ? v[lane - 1] : 12345u)) e |= 1;
    if (next != (lane < 63 ? v[lane + 1] : 54321u)) e |= 2;
    const uint32_t sum = wave_scan_incl(x & 0xFFFu, 0u, OpAdd());
    uint32_t ref = 0;
    for (uint32_t l = 0; l <= lane; ++l) ref += v[l] & 0xFFFu;
    if (sum != ref) e |= 4;
    const uint32_t f = (x & 1u) ? 16u + (x >> 3) % 9u : (x >> 5) % 9u;
    const uint32_t sc = wave_scan_incl(f, 0u, OpPhase9());
    uint32_t rf = 0;
    for (uint32_t l = 0; l <= lane; ++l) {
        const uint32_t y = v[l];
        rf = OpPhase9()(rf, (y & 1u) ? 16u + (y >> 3) % 9u : (y >> 5) % 9u);
    }
    if (sc != rf) e |= 8;
    const uint32_t m = 0x03000000u | (x % 3u) | (((x >> 4) % 3u) << 8) | (((x >> 8) % 3u) << 16);
    const uint32_t sm = wave_scan_incl(m, kMapId, OpMap());
    uint32_t rm = kMapId;
    for (uint32_t l = 0; l <= lane; ++l) {
        const uint32_t y = v[l];
        const uint32_t my = 0x03000000u | (y % 3u) | (((y >> 4) % 3u) << 8) | (((y >> 8) % 3u) << 16);
        rm = OpMap()(rm, my);
    }
    if (sm != rm) e |= 16;
    const uint32_t mx = wave_scan_incl(x & 0xFFFFu, 0u, OpMax());
    uint32_t rx = 0;
    for (uint32_t l = 0; l <= lane; ++l) rx = (v[l] & 0xFFFFu) > rx ? (v[l] & 0xFFFFu) : rx;
    if (mx != rx) e |= 32;
    if (nz4(0x00FF0100u) != 0x6u || nz4(0x80000001u) != 0x9u || nz4(0u) != 0u || nz4(0xFFFFFFFFu) != 0xFu) e |= 64;
    if (mod9(1000000007u) != 1000000007u % 9u || mod9(0xFFFFFFFFu) != 0xFFFFFFFFu % 9u) e |= 128;
    if (e) atomicOr(err, e);
}

}  // namespace rle

// ================================================================ C-ABI launchers
namespace {
static_assert(RLE_LAUNCH_STATUS_FLAG == rle::kLaunchFlag, "launch flag bit (rle_device.h put_status)");
constexpr uint32_t kMaxGrid = 1u << 30;
// one buffer per wave, kWaves waves per workgroup, rounded up to whole rounds of the 8 XCDs
// (rle::xcd_buffer); the kernels have no grid-stride loop, so n is bounded (kMaxGrid)
inline uint32_t grid_for(uint32_t n, uint32_t waves) {
    const uint32_t g = (n + waves - 1) / waves;
    return (g + rle::kXcds - 1) / rle::kXcds * rle::kXcds;
}
// Output store policy of a launch (rle_device.h vstore): write through for batches of up to
// kWtBuffers buffers, whose output typically fits in the L2s and would otherwise all be written
// back at the kernel boundary (configs[1], 4096 x 4 KiB: decode 15.2 -> 13.1 us, encode 14.0 ->
// 12.6 us); plain stores above (16384 x 64 KiB: write-through 6-14 % slower).
// RLE_MI355X_STORE=wt / wb forces one policy (RLE_MI355X_STORE_ENC / _DEC: one kernel only).
constexpr uint32_t kWtBuffers = 4096;
int store_env(const char* name) {
    const char* e = getenv(name);
    return !e ? -1 : !strcmp(e, "wt") ? 1 : !strcmp(e, "wb") ? 0 : -1;
}
uint32_t store_policy(uint32_t n, bool enc) {
    static const int force = store_env("RLE_MI355X_STORE");
    static const int force_enc = store_env("RLE_MI355X_STORE_ENC"), force_dec = store_env("RLE_MI355X_STORE_DEC");
    const int f = enc ? (force_enc >= 0 ? force_enc : force) : (force_dec >= 0 ? force_dec : force);
    return f >= 0 ? (uint32_t)f : (n <= kWtBuffers ? 1u : 0u);
}

// Decode batches past one residency round of the chip (4 workgroups of 4 waves per CU) are
// issued longest first; RLE_MI355X_DEC_ORDER=0 turns that off.
constexpr uint32_t kDecRound = 4096;
#ifndef RLE_DEC_CHUNKS_LARGE   // staging chunks of the decode kernel for batches past kDecRound
#define RLE_DEC_CHUNKS_LARGE 96
#endif
constexpr uint32_t kDecChunksLarge = RLE_DEC_CHUNKS_LARGE;
// The large-batch decode in rounds (rle_round.h): waves per workgroup (4, 8 or 16; 0 off), for
// batches past one residency round whose largest stream is at least kRoundMinIn bytes (the sized
// entry points know it).  RLE_MI355X_DEC_ROUND overrides; tests switch it with rle_mi355x_set_dec_round.
constexpr uint64_t kRoundMinIn = 8u * rle::kTileStep;
std::atomic<int> g_dec_round{[] {
    const char* e = getenv("RLE_MI355X_DEC_ROUND");
    return e ? atoi(e) : 0;
}()};
bool dec_order_enabled() {
    static const bool on = !(getenv("RLE_MI355X_DEC_ORDER") && !strcmp(getenv("RLE_MI355X_DEC_ORDER"), "0"));
    return on;
}

// The issue order's device array.  A hipFreeAsync + hipMallocAsync pair per launch left a 5.8 us gap
// on the queue between back-to-back large decodes (profiles/r5an_order_gap.md); instead each
// (device, stream handle) keeps a grow-only array in one of kOrderStreams slots (launches being
// captured into a graph take the per-launch pair).  The lock is held until the order and decode
// kernels are both enqueued, so host threads sharing a stream cannot interleave their launches.
// A handle does not always name one queue: hipStreamPerThread is a different stream in
// every thread, and a destroyed stream's handle can come back for a new stream while the old one's
// decode still reads the array.  So every slot records an event after its last decode, and the
// next launch on the slot makes its stream wait for it before the order kernel rewrites the array:
// on one queue that wait is already satisfied by stream order; across queues it keeps the array's
// users in turn.  When all slots are taken, the least recently used one is handed over (its array
// freed behind its event on the new stream); rle_decode_release_stream frees a stream's slot.
struct OrderSlot {
    int dev = -1;
    hipStream_t s = nullptr;
    uint32_t* p = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;   // recorded after the slot's last decode launch
    bool recorded = false;
    uint64_t last = 0;           // LRU clock
};
struct OrderArray {
    uint32_t* p = nullptr;
    hipStream_t s = nullptr;
    bool pooled = false;        // a per-launch array: freed on the stream after the decode
    OrderSlot* slot = nullptr;  // a cached array: its event is recorded after the decode
    std::unique_lock<std::mutex> lk;
    ~OrderArray() {   // early returns (order_release clears p)
        if (pooled && p) (void)hipFreeAsync(p, s);
    }
};
constexpr uint32_t kOrderStreams = 16;
std::mutex g_order_mu;
OrderSlot g_order_slots[kOrderStreams];
uint64_t g_order_clock = 0;
// (g_order_mu held) the slot's array released behind its last decode, on stream `s`
void order_slot_drop(OrderSlot& e, hipStream_t s) {
    if (e.p) {
        if (e.recorded) (void)hipStreamWaitEvent(s, e.done, 0);
        (void)hipFreeAsync(e.p, s);
    }
    e.p = nullptr;
    e.cap = 0;
    e.recorded = false;
    e.s = nullptr;
    e.dev = -1;
}
void order_acquire(OrderArray& o, hipStream_t s, size_t bytes) {
    o.s = s;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusActive;
    int dev = -1;
    if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone &&
        hipGetDevice(&dev) == hipSuccess) {
        o.lk = std::unique_lock<std::mutex>(g_order_mu);
        OrderSlot* e = nullptr;
        for (uint32_t i = 0; i < kOrderStreams && !e; ++i)
            if (g_order_slots[i].p && g_order_slots[i].s == s && g_order_slots[i].dev == dev) e = &g_order_slots[i];
        if (!e) {   // a free slot of this device's, else the least recently used one
            for (uint32_t i = 0; i < kOrderStreams; ++i) {
                OrderSlot& c = g_order_slots[i];
                if (!e || (!c.p && e->p) || (!!c.p == !!e->p && c.last < e->last)) e = &c;
            }
            if (e->p && e->dev != dev) e = nullptr;   // (another device's array: not freed from here)
            if (e) {
                order_slot_drop(*e, s);
                e->dev = dev;
                e->s = s;
            }
        }
        if (e && !e->done && hipEventCreateWithFlags(&e->done, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            e->done = nullptr;
            e = nullptr;
        }
        if (e) {
            if (e->recorded && hipStreamWaitEvent(s, e->done, 0) != hipSuccess) {
                (void)hipGetLastError();
                e = nullptr;
            }
        }
        if (e && e->cap < bytes) {   // grow: the old array is freed behind the earlier decodes (the wait above)
            const size_t cap = bytes > (1u << 20) ? bytes : (1u << 20);
            uint32_t* q = nullptr;
            if (hipMallocAsync((void**)&q, cap, s) == hipSuccess) {
                if (e->p) (void)hipFreeAsync(e->p, s);
                e->p = q;
                e->cap = cap;
            } else {
                (void)hipGetLastError();
                e = nullptr;
            }
        }
        if (e) {
            o.p = e->p;
            o.slot = e;
            return;
        }
        o.lk.unlock();
    }
    (void)hipGetLastError();
    if (hipMallocAsync((void**)&o.p, bytes, s) != hipSuccess) {
        (void)hipGetLastError();
        o.p = nullptr;
        return;
    }
    o.pooled = true;
}
// After the decode's launch: frees a per-launch array on the stream, or records the cached slot's
// event (RLE_E_HIP when that fails).
bool order_release(OrderArray& o) {
    bool ok = !(o.pooled && o.p && hipFreeAsync(o.p, o.s) != hipSuccess);
    if (o.slot) {
        if (hipEventRecord(o.slot->done, o.s) == hipSuccess) {
            o.slot->recorded = true;
        } else {
            (void)hipGetLastError();
            order_slot_drop(*o.slot, o.s);   // (no event: the array goes behind this launch)
            ok = false;
        }
        o.slot->last = ++g_order_clock;
        o.slot = nullptr;
    }
    o.p = nullptr;
    if (o.lk.owns_lock()) o.lk.unlock();
    return ok;
}

}  // namespace

extern "C" size_t rle_max_compressed_size(size_t U) { return U + U / 2; }

namespace {
int encode_launch(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len, void* d_out,
                  const uint64_t* d_out_off, uint64_t* d_out_len, uint32_t* d_status, uint32_t n, uint32_t flags,
                  void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return RLE_E_INVAL;
    if (n > kMaxGrid) return RLE_E_INVAL;
    const uint32_t pol = store_policy(n, true);
    auto kern = pol ? rle::encode_kernel<2u, 1u> : rle::encode_kernel<2u, 2u>;
    hipLaunchKernelGGL(kern, dim3(grid_for(n, rle::kEncWaves)), dim3(rle::kEncBlock), 0, (hipStream_t)stream,
                       (const uint8_t*)d_in, d_in_off, d_in_len, (uint8_t*)d_out, d_out_off, d_out_len, d_status, n,
                       pol | flags);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}
}  // namespace

extern "C" int rle_encode_batch_device(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                       void* d_out, const uint64_t* d_out_off, uint64_t* d_out_len,
                                       uint32_t* d_status, uint32_t n, void* stream) {
    return encode_launch(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, d_status, n, 0u, stream);
}

namespace {
int decode_launch(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len, void* d_out,
                  const uint64_t* d_out_off, const uint64_t* d_out_len, const uint64_t* d_out_cap, uint32_t* d_status,
                  uint32_t n, uint32_t flags, void* stream, uint64_t max_in_len = 0) {
    if (n == 0) return RLE_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return RLE_E_INVAL;
    if (n > kMaxGrid) return RLE_E_INVAL;
    const hipStream_t s = (hipStream_t)stream;
    // more buffers than one residency round: issue them longest first (rle::dec_order_local_kernel,
    // one launch of chunk-local sorts into the [n] issue-order array)
    OrderArray oa;
    if (n > kDecRound && dec_order_enabled()) order_acquire(oa, s, sizeof(uint32_t) * (size_t)n);
    uint32_t* order = oa.p;
    if (order)
        hipLaunchKernelGGL(rle::dec_order_local_kernel, dim3((n + rle::kLocalChunk - 1u) / rle::kLocalChunk), dim3(256), 0,
                           s, d_in_len, n, order);
    const uint32_t pol = store_policy(n, false);
    const int rw = g_dec_round.load(std::memory_order_relaxed);
    if (n > kDecRound && rw != 0 && max_in_len >= kRoundMinIn) {   // rounds of rw tiles per buffer
        auto rk = rw == 4 ? (pol ? rle::dec_round_kernel<4, 96, true> : rle::dec_round_kernel<4, 96, false>)
                : rw == 2 ? (pol ? rle::dec_round_kernel<2, 96, true> : rle::dec_round_kernel<2, 96, false>)
                : rw == 16 ? (pol ? rle::dec_round_kernel<16, 64, true> : rle::dec_round_kernel<16, 64, false>)
                           : (pol ? rle::dec_round_kernel<8, 96, true> : rle::dec_round_kernel<8, 96, false>);
        const uint32_t threads = rle::kWave * (uint32_t)(rw == 2 || rw == 4 || rw == 16 ? rw : 8);
        hipLaunchKernelGGL(rk, dim3(n), dim3(threads), 0, s, (const uint8_t*)d_in, d_in_off, d_in_len, (uint8_t*)d_out,
                           d_out_off, d_out_len, d_out_cap, d_status, n, pol | flags, (const uint32_t*)order);
        if (!order_release(oa)) return RLE_E_HIP;
        return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
    }
    // past one residency round of the one-pass staging, the smaller staging (more waves per SIMD);
    // a few buffers (single drop-in calls): the deep tile ring
    const bool large = n > kDecRound && kDecChunksLarge != rle::kDecChunks;
    auto kern = large ? (pol ? rle::decode_kernel<kDecChunksLarge, 0u, 1u> : rle::decode_kernel<kDecChunksLarge, 0u, 2u>)
                      : (pol ? rle::decode_kernel<rle::kDecChunks, 0u, 1u> : rle::decode_kernel<rle::kDecChunks, 0u, 2u>);
    hipLaunchKernelGGL(kern, dim3(grid_for(n, rle::kDecWaves)), dim3(rle::kDecBlock), 0, s,
                       (const uint8_t*)d_in, d_in_off, d_in_len, (uint8_t*)d_out, d_out_off, d_out_len, d_out_cap,
                       d_status, n, pol | flags, (const uint32_t*)order);
    if (!order_release(oa)) return RLE_E_HIP;
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}
}  // namespace

extern "C" int rle_decode_batch_device(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                       void* d_out, const uint64_t* d_out_off, const uint64_t* d_out_len,
                                       const uint64_t* d_out_cap, uint32_t* d_status, uint32_t n, void* stream) {
    return decode_launch(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, d_out_cap, d_status, n, 0u, stream);
}

// Cooperative small-buffer kernels (rle_coop.hip): 1 if launched, 0 if the batch does not qualify.
extern "C" int rle_encode_coop_launch(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len, void* d_out,
                                      const uint64_t* d_out_off, uint64_t* d_out_len, uint32_t* d_status, uint32_t n,
                                      uint64_t max_len, uint32_t flags, void* stream);
extern "C" int rle_decode_coop_launch(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len, void* d_out,
                                      const uint64_t* d_out_off, const uint64_t* d_out_len, const uint64_t* d_out_cap,
                                      uint32_t* d_status, uint32_t n, uint64_t max_in_len, uint64_t max_out_len,
                                      uint32_t flags, void* stream);

extern "C" int rle_encode_batch_device_sized_flags(const void* d_in, const uint64_t* d_in_off,
                                                   const uint64_t* d_in_len, void* d_out, const uint64_t* d_out_off,
                                                   uint64_t* d_out_len, uint32_t* d_status, uint32_t n,
                                                   uint64_t max_in_len, uint32_t flags, void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return RLE_E_INVAL;
    if (n > kMaxGrid || (flags & ~(uint32_t)RLE_LAUNCH_STATUS_FLAG) || ((flags & RLE_LAUNCH_STATUS_FLAG) && !d_status))
        return RLE_E_INVAL;
    const int c = rle_encode_coop_launch(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, d_status, n, max_in_len,
                                         flags, stream);
    if (c != 0) return c > 0 ? RLE_OK : c;
    return encode_launch(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, d_status, n, flags, stream);
}

extern "C" int rle_encode_batch_device_sized(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                             void* d_out, const uint64_t* d_out_off, uint64_t* d_out_len,
                                             uint32_t* d_status, uint32_t n, uint64_t max_in_len, void* stream) {
    return rle_encode_batch_device_sized_flags(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, d_status, n,
                                               max_in_len, 0u, stream);
}

extern "C" int rle_decode_batch_device_sized_flags(const void* d_in, const uint64_t* d_in_off,
                                                   const uint64_t* d_in_len, void* d_out, const uint64_t* d_out_off,
                                                   const uint64_t* d_out_len, const uint64_t* d_out_cap,
                                                   uint32_t* d_status, uint32_t n, uint64_t max_in_len,
                                                   uint64_t max_out_len, uint32_t flags, void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return RLE_E_INVAL;
    if (n > kMaxGrid || (flags & ~(uint32_t)RLE_LAUNCH_STATUS_FLAG) || ((flags & RLE_LAUNCH_STATUS_FLAG) && !d_status))
        return RLE_E_INVAL;
    const int c = rle_decode_coop_launch(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, d_out_cap, d_status, n,
                                         max_in_len, max_out_len, flags, stream);
    if (c != 0) return c > 0 ? RLE_OK : c;
    return decode_launch(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, d_out_cap, d_status, n, flags, stream,
                         max_in_len);
}

// Tests / A-B: waves per workgroup of the large-batch decode in rounds (0 off, 4, 8, 16); -1 only
// reads.  Returns the previous setting, or RLE_E_INVAL.
// Frees the issue-order array cached for `stream` on the current device (behind the stream's earlier
// decodes); a caller about to destroy a stream, or done with a thread's per-thread stream, calls it.
extern "C" int rle_decode_release_stream(void* stream) {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return RLE_E_HIP;
    std::lock_guard<std::mutex> lk(g_order_mu);
    for (uint32_t i = 0; i < kOrderStreams; ++i) {
        OrderSlot& e = g_order_slots[i];
        if (e.p && e.s == (hipStream_t)stream && e.dev == dev) order_slot_drop(e, (hipStream_t)stream);
    }
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

extern "C" int rle_mi355x_set_dec_round(int waves) {
    if (waves == -1) return g_dec_round.load(std::memory_order_relaxed);
    if (waves != 0 && waves != 2 && waves != 4 && waves != 8 && waves != 16) return RLE_E_INVAL;
    return g_dec_round.exchange(waves, std::memory_order_relaxed);
}

extern "C" int rle_decode_batch_device_sized(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                             void* d_out, const uint64_t* d_out_off, const uint64_t* d_out_len,
                                             const uint64_t* d_out_cap, uint32_t* d_status, uint32_t n,
                                             uint64_t max_in_len, uint64_t max_out_len, void* stream) {
    return rle_decode_batch_device_sized_flags(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, d_out_cap,
                                               d_status, n, max_in_len, max_out_len, 0u, stream);
}

extern "C" int rle_gen_synthetic_device(void* d_out, const uint64_t* d_off, const uint64_t* d_len,
                                        const uint32_t* d_kind, const uint64_t* d_index, uint32_t n, void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_out || !d_off || !d_len) return RLE_E_INVAL;
    hipLaunchKernelGGL(rle::gen_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (uint8_t*)d_out,
                       d_off, d_len, d_kind, d_index, n);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

extern "C" int rle_decode_pattern_device(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                         void* d_out, const uint64_t* d_out_off, const uint64_t* d_out_len, uint32_t n,
                                         void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len || n > kMaxGrid) return RLE_E_INVAL;
    const hipStream_t s = (hipStream_t)stream;
    OrderArray oa;   // the decode's issue order (decode_launch)
    if (n > kDecRound && dec_order_enabled()) order_acquire(oa, s, sizeof(uint32_t) * (size_t)n);
    uint32_t* order = oa.p;
    if (order)
        hipLaunchKernelGGL(rle::dec_order_local_kernel, dim3((n + rle::kLocalChunk - 1u) / rle::kLocalChunk), dim3(256), 0,
                           s, d_in_len, n, order);
    hipLaunchKernelGGL(rle::pattern_kernel, dim3(grid_for(n, rle::kDecWaves)), dim3(rle::kDecBlock), 0, s,
                       (const uint8_t*)d_in, d_in_off, d_in_len, (uint8_t*)d_out, d_out_off, d_out_len, n,
                       (const uint32_t*)order);
    if (!order_release(oa)) return RLE_E_HIP;
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

namespace rle {
// Host path (csrc/rle_dropin.cpp, registered calls): the first *len bytes of src into dst, the
// caller's result block mapped for the call.  *len is read on the device (an encode's output length
// is known only there), the grid is sized for the worst case and idles past *len.  Whole 16-byte
// chunks below len & ~15, the last bytes one by one, so nothing past dst + *len is written.  (A
// completion word stored by the last workgroup, polled by the host, measured slower than the
// stream synchronize: every workgroup's system-scope release writes its L2 back; r6o, 1 MiB
// 112.6 against 84.5 µs.)
__global__ __launch_bounds__(256) void copy_len_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                       const uint64_t* __restrict__ len) {
    const uint64_t n = *len, n16 = n / 16u;
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n16; i += stride)
        reinterpret_cast<u32x4*>(dst)[i] = reinterpret_cast<const u32x4*>(src)[i];
    if (blockIdx.x == 0 && threadIdx.x < (uint32_t)(n & 15u)) dst[16u * n16 + threadIdx.x] = src[16u * n16 + threadIdx.x];
}
// Host path (registered calls, round 6): the caller's n input bytes, registered for the call, read
// over PCIe through their device address into device memory.  It replaces the DMA: the kernels after
// it start about 1 µs after it ends, against about 10 µs after a DMA (tools/probes/
// hostpath_kread_probe.hip, r6ax: 1 MiB 38.5 against 42.8 µs with a kernel after each).  Four 16-byte
// loads in flight per lane, the last n % 16 bytes one by one (nothing past src + n is read).
__global__ __launch_bounds__(256) void copy_in_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                      uint64_t n) {
    const uint64_t n16 = n / 16u, stride = (uint64_t)gridDim.x * 256u;
    uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    for (; i + 3u * stride < n16; i += 4u * stride) {
        const u32x4 a = src[i], b = src[i + stride], c = src[i + 2u * stride], d = src[i + 3u * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2u * stride] = c;
        dst[i + 3u * stride] = d;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x < (uint32_t)(n & 15u))
        reinterpret_cast<uint8_t*>(dst)[16u * n16 + threadIdx.x] =
            reinterpret_cast<const uint8_t*>(src)[16u * n16 + threadIdx.x];
}
}  // namespace rle

// (csrc/rle_dropin.cpp) dst and src 16-byte aligned (else RLE_E_INVAL: the caller takes the DMA)
int rle_copy_in_launch(void* dst, const void* src, uint64_t n, hipStream_t s) {
    if ((((uintptr_t)dst | (uintptr_t)src) & 15u) != 0) return RLE_E_INVAL;
    if (n == 0) return RLE_OK;
    // At most 64 workgroups (1 MiB of loads in flight): more outstanding reads over PCIe were slower
    // (r6az probe: 4 MiB 107.5 µs at 64, 122.7-123.7 at 256-1024; 1 MiB 37.7 against 38.4-39.3).
    // RLE_MI355X_KREAD_GRID overrides the cap (A/B).
    static const uint64_t cap = [] {
        const char* e = getenv("RLE_MI355X_KREAD_GRID");
        const long v = e ? atol(e) : 64;
        return (uint64_t)(v >= 1 && v <= 4096 ? v : 64);
    }();
    const uint64_t want = (n / 16u + 1023u) / 1024u;   // (four chunks per lane)
    const uint32_t grid = (uint32_t)(want < 1u ? 1u : (want < cap ? want : cap));
    hipLaunchKernelGGL(rle::copy_in_kernel, dim3(grid), dim3(256), 0, s, (rle::u32x4*)dst, (const rle::u32x4*)src, n);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

// (csrc/rle_dropin.cpp) dst and src 16-byte aligned, *d_len <= max_bytes
int rle_copy_len_launch(void* dst, const void* src, const uint64_t* d_len, uint64_t max_bytes, hipStream_t s) {
    if ((((uintptr_t)dst | (uintptr_t)src) & 15u) != 0) return RLE_E_INVAL;
    const uint64_t want = (max_bytes / 16u + 255u) / 256u;
    const uint32_t grid = (uint32_t)(want < 1u ? 1u : (want < 1024u ? want : 1024u));
    hipLaunchKernelGGL(rle::copy_len_kernel, dim3(grid), dim3(256), 0, s, (uint8_t*)dst, (const uint8_t*)src, d_len);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

extern "C" int rle_copy_device(void* d_dst, const void* d_src, uint64_t nbytes, void* stream) {
    if (nbytes == 0) return RLE_OK;
    if (!d_dst || !d_src || (nbytes & 15u) || (((uintptr_t)d_dst | (uintptr_t)d_src) & 15u)) return RLE_E_INVAL;
    const uint64_t n16 = nbytes / 16u;
    const uint64_t want = (n16 + 1023u) / 1024u;
    const uint32_t grid = (uint32_t)(want < 2048u ? want : 2048u);   // 8 workgroups per CU at most
    // non-temporal past the Infinity Cache's 256 MiB (dec64k's 1.82 GB: 311.6 against 331.8 us), plain
    // below it (configs[1]'s 28 MB: 4.7 against 5.5 us); RLE_MI355X_COPY_NT=0/1 forces either
    static const int force = getenv("RLE_MI355X_COPY_NT") ? atoi(getenv("RLE_MI355X_COPY_NT")) : -1;
    const bool nt = force >= 0 ? force != 0 : nbytes >= (256ull << 20);
    if (nt)
        hipLaunchKernelGGL(rle::copy_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (rle::u32x4*)d_dst,
                           (const rle::u32x4*)d_src, n16);
    else
        hipLaunchKernelGGL(rle::copy_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (rle::u32x4*)d_dst,
                           (const rle::u32x4*)d_src, n16);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

extern "C" int rle_mi355x_selftest(void) {
    uint32_t* d = nullptr;
    uint32_t h = 0;
    if (hipMalloc(&d, sizeof(uint32_t)) != hipSuccess) return RLE_E_HIP;
    if (hipMemset(d, 0, sizeof(uint32_t)) != hipSuccess) { (void)hipFree(d); return RLE_E_HIP; }
    hipLaunchKernelGGL(rle::selftest_kernel, dim3(1), dim3(64), 0, 0, d);
    const hipError_t e1 = hipMemcpy(&h, d, sizeof(uint32_t), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e1 != hipSuccess) return RLE_E_HIP;
    return (int)h;
}

extern "C" int rle_mi355x_timeline(unsigned long long* out, int reset) {
#if RLE_TIMELINE
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(rle::g_tl), sizeof(rle::g_tl)) != hipSuccess) return RLE_E_HIP;
    if (reset) {
        static unsigned long long z[rle::kTlWaves * rle::kTlEv];
        if (hipMemcpyToSymbol(HIP_SYMBOL(rle::g_tl), z, sizeof(z)) != hipSuccess) return RLE_E_HIP;
    }
    return RLE_OK;
#else
    (void)out;
    (void)reset;
    return RLE_E_INVAL;   // not a diagnostic build
#endif
}

extern "C" int rle_mi355x_stamps(unsigned long long* out, int reset) {
#if RLE_STAMPS
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(rle::g_stamps), sizeof(rle::g_stamps)) != hipSuccess)
        return RLE_E_HIP;
    if (reset) {
        unsigned long long z[rle::kStampSegs + 1] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(rle::g_stamps), z, sizeof(z)) != hipSuccess) return RLE_E_HIP;
    }
    return RLE_OK;
#else
    (void)out;
    (void)reset;
    return RLE_E_INVAL;   // not a diagnostic build
#endif
}

extern "C" int rle_mi355x_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" const char* rle_mi355x_version(void) { return "rle_mi355x 0.3 (gfx950, wave-per-buffer tiled codec)"; }
