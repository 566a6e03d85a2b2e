// rle_device.h — device-side building blocks of the MI355X (gfx950) RLE codec, shared by the
// one-wave-per-buffer batch kernels (rle_kernels.hip) and the multi-wave segmented kernels
// (rle_segmented.hip): cross-lane primitives, the hand-counted LDS-DMA tile pipeline, and the
// encode / decode tile steps (reference src/rleCompression.c:9-62; grammar in SURVEY.md App. A).
#pragma once
//
// Device-resident forms of the reference codec (samul-1/C-FileStorage-Server-and-Client
// src/rleCompression.c:9-62; grammar restated in SURVEY.md Appendix A):
//   encode: maximal runs cut into 9-byte chunks; a chunk of r bytes of v emits "v" (r == 1)
//           or "v v ('0'+r)" (r >= 2)                          — src/rleCompression.c:13-41
//   decode: token at j emits y[j]; when y[j] == y[j+1] the token is 3 bytes and adds
//           (signed char)y[j+2]-'0'-1 copies, capped at U      — src/rleCompression.c:50-60
//
// Execution model: a wave64 walks its buffer (or segment) in 1 KiB tiles, 16 bytes
// per lane.  Loads are range-checked LDS-DMA buffer_load_dwordx4 (two slots, two tiles in flight);
// their completion is counted by hand (s_waitcnt vmcnt(N), N = the memory ops issued since),
// because hipcc's own bookkeeping drains the queue at every loop header once a variable number of
// stores sits in the loop.  Run boundaries and token starts are 16-bit per-lane masks from SWAR
// byte compares; the sequential state (encode: run start position; decode: token phase 0..2 as a
// v_perm byte map) and output offsets cross lanes by DPP wave scans and cross tiles in scalar
// registers.  In the general path each lane scatters its output into a per-wave LDS staging area
// that is linear per tile, and complete 16-byte chunks leave as coalesced buffer_store_dwordx4.
// Tiles of common shapes skip the staging: literal tiles (runs <= 2: each
// lane's output is its bytes with <= 2 removed or inserted, one v_perm per dword, stored as
// unaligned 16-byte stores), encoder run tiles (a 3-periodic "v v 9" pattern) and decoder
// single-value tiles (rep4(v) chunks).  No MFMA: this is an HBM-bound byte scan.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rle_build.h"
#include "rle_mi355x.h"

namespace rle {

typedef uint32_t u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

constexpr u32 kWave = 64;
constexpr u32 kMaxBufferBytes = RLE_MAX_BUFFER_BYTES;   // per-buffer limit (32-bit in-buffer offsets)
constexpr u32 kOOB = 0x80000000u;               // store offset dropped by the range check
constexpr u32 kNotFast = 0xFFFFFFFEu;           // a fast tile path declined (the general path runs)

// ---------------------------------------------------------------- cross-lane primitives (DPP)
enum : int {
    kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118,
    kRowBcast15 = 0x142, kRowBcast31 = 0x143, kWaveShl1 = 0x130, kWaveShr1 = 0x138,
};

template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ u32 dpp(u32 old, u32 src) {
    return (u32)__builtin_amdgcn_update_dpp((int)old, (int)src, kCtrl, kRowMask, 0xf, false);
}
// value of lane-1 (lane 0 gets `fill`) / of lane+1 (lane 63 gets `fill`)
__device__ __forceinline__ u32 from_prev_lane(u32 v, u32 fill) { return dpp<kWaveShr1>(fill, v); }
__device__ __forceinline__ u32 from_next_lane(u32 v, u32 fill) { return dpp<kWaveShl1>(fill, v); }
__device__ __forceinline__ u32 readlane(u32 v, u32 l) { return (u32)__builtin_amdgcn_readlane((int)v, (int)l); }
__device__ __forceinline__ u32 uniform(u32 v) { return (u32)__builtin_amdgcn_readfirstlane((int)v); }

// Inclusive wave scan for an associative op(a_earlier, b_later) with identity `id`.
// Must be called with all 64 lanes active.
template <class Op>
__device__ __forceinline__ u32 wave_scan_incl(u32 x, u32 id, Op op) {
    x = op(dpp<kRowShr1>(id, x), x);
    x = op(dpp<kRowShr2>(id, x), x);
    x = op(dpp<kRowShr4>(id, x), x);
    x = op(dpp<kRowShr8>(id, x), x);
    x = op(dpp<kRowBcast15, 0xa>(id, x), x);
    x = op(dpp<kRowBcast31, 0xc>(id, x), x);
    return x;
}
struct OpAdd {
    __device__ __forceinline__ u32 operator()(u32 a, u32 b) const { return a + b; }
};
struct OpMax {
    __device__ __forceinline__ u32 operator()(u32 a, u32 b) const { return a > b ? a : b; }
};
// "latest present value": values are 0 (absent) or 0x100|byte
struct OpLatest {
    __device__ __forceinline__ u32 operator()(u32 a, u32 b) const { return b ? b : a; }
};
// token-phase maps {0,1,2} -> {0,1,2} as v_perm selectors: byte d = image of d; byte 3 = 3
constexpr u32 kMapId = 0x03020100u;
struct OpMap {
    __device__ __forceinline__ u32 operator()(u32 a, u32 b) const { return __builtin_amdgcn_perm(b, b, a); }
};
// encode phase transfer functions (self-test only): code >= 16 -> constant, else add mod 9
__device__ __forceinline__ u32 mod9s(u32 x) { return x >= 9u ? x - 9u : x; }
struct OpPhase9 {
    __device__ __forceinline__ u32 operator()(u32 a, u32 b) const {
        return b >= 16u ? b : (a >= 16u ? 16u + mod9s(a - 16u + b) : mod9s(a + b));
    }
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- byte SWAR helpers
// bit k (k = 0..3) set iff byte k of d is non-zero
__device__ __forceinline__ u32 nz4(u32 d) {
    u32 t = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
    t >>= 7;             // bytes' flags at bits 0, 8, 16, 24
    t |= t >> 7;         // ... at bits 0, 1 and 16, 17
    return (t | (t >> 14)) & 0xFu;
}
// byte 0 of x in all four bytes (v_perm: selector bytes 0..3 pick bytes of the second operand)
__device__ __forceinline__ u32 rep4(u32 x) { return __builtin_amdgcn_perm(0u, x, 0u); }
__device__ __forceinline__ u32 lowmask(u32 nbits) { return nbits >= 32u ? ~0u : ((1u << nbits) - 1u); }
__device__ __forceinline__ u32 alignbyte(u32 hi, u32 lo, u32 s) { return __builtin_amdgcn_alignbyte(hi, lo, s); }
__device__ __forceinline__ u32 bfe(u32 v, u32 off, u32 w) { return __builtin_amdgcn_ubfe(v, off, w); }
__device__ __forceinline__ u32 bcnt(u32 v, u32 acc) { return (u32)__builtin_popcount(v) + acc; }
// 4-bit mask -> bytes 0x01
__device__ __forceinline__ u32 nib_to_bytes(u32 n) { return (n * 0x00204081u) & 0x01010101u; }
// (a << s) + b in one full-rate op (left to itself the compiler folds a shift-add chain into a
// quarter-rate v_mul_lo_u32)
template <int kShift>
__device__ __forceinline__ u32 lshl_add(u32 a, u32 b) {
    u32 r;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(kShift), "v"(b));
    return r;
}
// 0xFF in every byte that is non-zero in m (bytes of m in 0..3: v_perm selectors 0x0C -> 0x00, 0x0D.. -> 0xFF)
__device__ __forceinline__ u32 bytes_ff(u32 m) { return __builtin_amdgcn_perm(0u, 0u, m | 0x0C0C0C0Cu); }
__device__ __forceinline__ u32 mod9(u32 x) {
    const u32 q = __umulhi(x, 0x38E38E39u) >> 1;
    return x - 9u * q;
}

// ---------------------------------------------------------------- memory pipeline (hand-counted)
// 128-bit buffer resource (raw buffer, stride 0): loads past num_records return 0, stores past
// it are dropped.  Built from wave-uniform values only.
__device__ __forceinline__ u32x4 make_rsrc(const void* base, u32 nbytes) {
    const uint64_t a = (uint64_t)base;
    u32x4 r;
    r.x = (u32)a;
    r.y = (u32)(a >> 32) & 0xFFFFu;
    r.z = nbytes;
    r.w = 0x00020000u;
    return r;
}
// LDS byte address of a __shared__ pointer
__device__ __forceinline__ u32 lds_addr(const void* p) {
    return (u32)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// Loads and stores in asm: hipcc neither counts nor waits for them; vm_wait() is the only wait
// for them.  Loads go straight to LDS (LDS-DMA: lane i's 16 bytes land at lds + 16 i), so no
// VGPR is in flight that the compiler could copy or reuse before the data lands.  (The non-
// temporal hint on the tile loads and on the large launches' stores measured slower everywhere,
// r3n: DESIGN.md §4.)
template <bool kStream = false>
__device__ __forceinline__ void dma_tile(u32x4 rs, u32 voff, u32 lds) {
    u32 keep;
    if (kStream)
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"   // earlier ds_reads of this slot have completed
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(voff), "s"(lds), "s"(rs)
            : "memory");
    else
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %2\n\t"
            "s_waitcnt lgkmcnt(0)\n\t"   // earlier ds_reads of this slot have completed
            "s_nop 0\n\t"
            "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(voff), "s"(lds), "s"(rs)
            : "memory");
}
// Output stores.  wt (wave-uniform): write through (sc1: the line leaves the XCD's L2 and is not
// kept dirty there).  A launch whose whole output fits in L2 otherwise ends with all of it dirty,
// and the kernel boundary writes it back at about 6 TB/s (MI355X_MICROARCH.md, kernel boundaries):
// 2.8 us for configs[1]'s 16.8 MB of decoded output.  Large launches store plainly, where writing
// through measured 6-14 % slower (the launchers choose; rle_kernels.hip).
#define RLE_WT_BITS "sc1"   // cache-policy bits of the write-through stores
#define RLE_WB_BITS ""
__device__ __forceinline__ void vstore(u32x4 rs, u32 voff, u32x4 v, bool wt) {
    if (wt)
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen " RLE_WT_BITS "\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs) : "memory");
    else
        asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" RLE_WB_BITS "\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs) : "memory");
}
// One 4-byte store (buffer_store_dword; offsets need not be aligned).
__device__ __forceinline__ void vstore4(u32x4 rs, u32 voff, u32 v, bool wt) {
    if (wt)
        asm volatile("buffer_store_dword %0, %1, %2, 0 offen " RLE_WT_BITS "\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs) : "memory");
    else
        asm volatile("buffer_store_dword %0, %1, %2, 0 offen" RLE_WB_BITS "\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rs) : "memory");
}

// wait until at most n vector-memory ops are outstanding
#define RLE_VMW(N)                                            \
    case N:                                                   \
        asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); \
        break;
// (n is wave-uniform; readfirstlane tells the compiler, which otherwise may lower the switch as an
// exec-masked VGPR compare tree)
__device__ __forceinline__ void vm_wait(u32 n) {
    n = uniform(n);
    switch (n < 15u ? n : 15u) {
        RLE_VMW(0) RLE_VMW(1) RLE_VMW(2) RLE_VMW(3) RLE_VMW(4) RLE_VMW(5) RLE_VMW(6) RLE_VMW(7) RLE_VMW(8)
        RLE_VMW(9) RLE_VMW(10) RLE_VMW(11) RLE_VMW(12) RLE_VMW(13) RLE_VMW(14) RLE_VMW(15)
        default: break;
    }
}
#undef RLE_VMW
// the same for the walks whose counts reach past 15 (enc_stream_body)
#define RLE_VMW2(N)                                           \
    case N:                                                   \
        asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); \
        break;
__device__ __forceinline__ void vm_wait_deep(u32 n) {
    n = uniform(n);
    switch (n < 39u ? n : 39u) {
        RLE_VMW2(0) RLE_VMW2(1) RLE_VMW2(2) RLE_VMW2(3) RLE_VMW2(4) RLE_VMW2(5) RLE_VMW2(6) RLE_VMW2(7)
        RLE_VMW2(8) RLE_VMW2(9) RLE_VMW2(10) RLE_VMW2(11) RLE_VMW2(12) RLE_VMW2(13) RLE_VMW2(14) RLE_VMW2(15)
        RLE_VMW2(16) RLE_VMW2(17) RLE_VMW2(18) RLE_VMW2(19) RLE_VMW2(20) RLE_VMW2(21) RLE_VMW2(22) RLE_VMW2(23)
        RLE_VMW2(24) RLE_VMW2(25) RLE_VMW2(26) RLE_VMW2(27) RLE_VMW2(28) RLE_VMW2(29) RLE_VMW2(30) RLE_VMW2(31)
        RLE_VMW2(32) RLE_VMW2(33) RLE_VMW2(34) RLE_VMW2(35) RLE_VMW2(36) RLE_VMW2(37) RLE_VMW2(38) RLE_VMW2(39)
        default: break;
    }
}
#undef RLE_VMW2
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Launch flags, the kernels' `wt` argument: bit 0 write-through output stores (vstore), bit 1 the
// status word is the caller's completion flag (include/rle_mi355x.h RLE_LAUNCH_STATUS_FLAG): every
// earlier store of the wave is released at system scope (L2 write-back + store acknowledgement)
// before the status store, so a host polling the status in mapped memory may then read the output.
// A store acknowledgement alone is not enough: without the L2 write-back the host read stale output
// words (tools/probes/sync_probe.hip, profiles/r4a_sync_probe.txt).
constexpr u32 kLaunchWt = 1u, kLaunchFlag = 2u;
__device__ __forceinline__ void put_status(uint32_t* status, u32 b, u32 v, u32 flags) {
    if (!status) return;
    if (flags & kLaunchFlag) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope
        __hip_atomic_store(status + b, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        status[b] = v;
    }
}

// Tiles overlap: tile t is input [1008 t, 1008 t + 1024); lanes 0..62 own its first 1008 bytes
// and lane 63 holds the next tile's first 16 bytes (the lookahead of lane 62).  Each tile is one
// LDS-DMA into one of two slots.  A step reads its slot once (one ds_read_b128 per lane) and then
// calls next() to refill that slot with tile t+2, so two tiles are in flight behind the one being
// processed.  step(t, slot, next) returns the store instructions it issued after next() (or ~0u to
// stop).  Vector-memory ops complete in issue order, so the wait for tile t+1 (issued inside step
// t-1, before that step's stores) leaves step t-1's stores, the refill and step t's stores in
// flight.  Loads past the buffer (t+2 >= ntiles) are range-checked to zero and cost no traffic.
//
// Encode of small buffers (enc_tile<true>): tiles do not overlap.  All 64 lanes own 16 bytes (tile t
// is [1024 t, 1024 t + 1024)), and the 16 bytes after the tile, which lane 63 looks ahead into,
// come with a second one-lane DMA into the slot's tail (kLook).  A 4 KiB buffer is then 4 tiles
// instead of 5; the extra work per tile (≈5 %) outweighs the saving from about 16 KiB up.
constexpr u32 kOwnLanes = 63;
constexpr u32 kTileStep = 16 * kOwnLanes;   // 1008: decode tiles
constexpr u32 kSlot = 16 * kWave;           // 1024
constexpr u32 kEncStep = 16 * kWave;        // 1024: encode tiles
constexpr u32 kEncSlot = kSlot + 16;        // ... and their 16-byte lookahead
struct Refill {
    u32x4 rs;
    u32 voff;    // lane byte offset of tile t+2
    u32 lds;     // slot LDS address
    bool on;     // tile t+2 exists (wave-uniform)
    bool look;   // kLook walks: lane 0 also loads the 16 bytes after the tile into the slot's tail
    __device__ __forceinline__ void operator()() const {
        if (on) {
            dma_tile<true>(rs, voff, lds);
            if (look) dma_tile<true>(rs, voff + kEncStep, lds + kSlot);
        }
    }
};
// Tiles start at `start` (bytes from the buffer descriptor's base): tile t is [start + 1008 t, ...).
// The first two tiles' loads; walk_tiles issues them itself unless the caller did (primed), e.g. to
// overlap their latency with its own setup.
// kStep: tile stride; kLook: encode tiles (kEncStep, slots of kEncSlot with the lookahead load).
template <u32 kStep = kTileStep, bool kLook = false>
__device__ __forceinline__ void walk_prime(u32x4 rs, u32 start, u32 ntiles, u32 lane, const uint8_t* slots) {
    constexpr u32 kStride = kLook ? kEncSlot : kSlot;
    const u32 lo = start + 16u * lane;
    const u32 l0 = uniform(lds_addr(slots)), l1 = l0 + kStride;
    asm volatile("s_nop 4" ::: "memory");   // descriptor words may be fresh
    if (ntiles) Refill{rs, lo, l0, true, kLook && lane == 0u}();
    if (ntiles > 1u) Refill{rs, kStep + lo, l1, true, kLook && lane == 0u}();
}
// Returns whether a step stopped the walk (~0u).
template <u32 kStep = kTileStep, bool kLook = false, class Step>
__device__ __forceinline__ bool walk_tiles(u32x4 rs, u32 start, u32 ntiles, u32 lane, const uint8_t* slots,
                                           Step step, bool primed = false) {
    constexpr u32 kStride = kLook ? kEncSlot : kSlot;
    constexpr u32 kLoads = kLook ? 2u : 1u;   // vector-memory ops per tile load
    const u32 lo = start + 16u * lane;
    const u32 l0 = uniform(lds_addr(slots)), l1 = l0 + kStride;
    const bool look = kLook && lane == 0u;
    // Only tiles that exist are loaded, so before step t the ops issued after tile t's load are
    // step t-2's stores, tile t+1's load (if t+1 < ntiles) and step t-1's stores.  Stores are never
    // waited for: nothing in the wave reads them back, and a wave may end with stores in flight.
    // Loads are all consumed by the last step, so only a walk that stops early (~0u) drains.
    if (!primed) walk_prime<kStep, kLook>(rs, start, ntiles, lane, slots);
    u32 p1 = 0, p2 = 0;   // stores of the last step and of the one before
    for (u32 t = 0; t < ntiles; t += 2) {
        vm_wait(p2 + (t + 1u < ntiles ? kLoads : 0u) + p1);
        p2 = p1;
        p1 = step(t, slots, Refill{rs, (t + 2u) * kStep + lo, l0, t + 2u < ntiles, look});
        if (p1 == ~0u) {
            vm_drain();
            return true;
        }
        if (t + 1u >= ntiles) break;
        vm_wait(p2 + (t + 2u < ntiles ? kLoads : 0u) + p1);
        p2 = p1;
        p1 = step(t + 1u, slots + kStride, Refill{rs, (t + 3u) * kStep + lo, l1, t + 3u < ntiles, look});
        if (p1 == ~0u) {
            vm_drain();
            return true;
        }
    }
    return false;
}
__device__ __forceinline__ u32 ntiles_for(u32 n) { return (n + kTileStep - 1u) / kTileStep; }
__device__ __forceinline__ u32 enc_ntiles_for(u32 n) { return (n + kEncStep - 1u) / kEncStep; }

// packed u16 max
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32 pkmax(u32 a, u32 b) {
    return __builtin_bit_cast(u32, __builtin_elementwise_max(__builtin_bit_cast(us2, a), __builtin_bit_cast(us2, b)));
}
// packed u16 max against b's high half in both halves: {max(a.lo, b.hi), max(a.hi, b.hi)} -- one
// v_pk_max_u16 with op_sel (the half selection folds into the source modifiers)
__device__ __forceinline__ u32 pkmax_bhi(u32 a, u32 b) {
    const us2 bv = __builtin_bit_cast(us2, b);
    return __builtin_bit_cast(u32, __builtin_elementwise_max(__builtin_bit_cast(us2, a), __builtin_shufflevector(bv, bv, 1, 1)));
}
// in-dword prefix max of a u16 pair: {a.lo, max(a.hi, a.lo)} -- one v_pk_max_u16 with op_sel_hi
__device__ __forceinline__ u32 pkmax_lo2hi(u32 a) {
    const us2 av = __builtin_bit_cast(us2, a);
    return __builtin_bit_cast(u32, __builtin_elementwise_max(av, __builtin_shufflevector(av, av, 0, 0)));
}

// ---------------------------------------------------------------- diagnostic builds
// Ablation builds (timing only, wrong output; never the product library), decode: 1 no phase scan,
// 2 no scatter, 4 no fill, 8 scatter without its LDS writes, 16 no count-digit validation (still
// exact on encoder output), 32 no uniform-tile test, 64 no flush stores; 128 (both kernels, in
// rle_kernels.hip) no tiles walked at all (the fixed per-buffer cost).
#ifndef RLE_ABL
#define RLE_ABL 0
#endif
// ---------------------------------------------------------------- diagnostic stamps
// RLE_STAMPS=1 builds (never the product library) sum s_memtime cycles per decode segment in
// each wave and add them into g_stamps; rle_mi355x_stamps() reads the sums.  Read shares only:
// each stamp drains the LDS queue (MI355X guide, "In-kernel stamps").
#ifndef RLE_STAMPS
#define RLE_STAMPS 0
#endif
#if RLE_STAMPS
constexpr u32 kStampSegs = 8;
static __device__ unsigned long long g_stamps[kStampSegs + 1];   // 8 segment sums, waves
struct Stamps {
    uint64_t acc[kStampSegs];
    uint64_t last;
};
__device__ __forceinline__ uint64_t memtime() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define RLE_STAMP(SP, I)                  \
    do {                                  \
        const uint64_t _t = memtime();    \
        (SP).acc[I] += _t - (SP).last;    \
        (SP).last = _t;                   \
    } while (0)
#else
struct Stamps {};
#define RLE_STAMP(SP, I) \
    do {                 \
    } while (0)
#endif

// ================================================================ fast-op helpers
// Instruction selection (measured, tools/probes/valu_rate_probe.hip, gfx950): v_add/v_sub/v_and/
// v_or/v_xor/v_lshrrev/v_not and v_bitop3 with VGPR or literal operands issue at ~1.9 cycles per
// wave-instruction with 4 waves per SIMD; everything else the codec uses (v_perm, v_alignbyte,
// v_bfe, v_lshlrev, v_mul*, v_dot4, SDWA, DPP, v_pk_*, v_and_or/v_lshl_or/v_add3, and ANY op with an
// SGPR operand) at ~3.  So the SWAR below keeps masks in 0x80-per-byte form (derived with right
// shifts), folds logic into v_bitop3 with constants held in VGPRs (vconst), and leaves the slow
// forms to the few places they replace several fast ops.
__device__ __forceinline__ u32 vconst(u32 c) {
    u32 r;
    asm("v_mov_b32 %0, %1" : "=v"(r) : "i"(c));
    return r;
}
template <u32 kImm>
__device__ __forceinline__ u32 bitop3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, kImm); }
// Plain VOP2 forms.  (Inline asm for them would make the hazard recognizer put an s_nop after each;
// the SDWA peephole that would fold them into slow-class byte/word-select adds is disabled for
// this code in the Makefile: -mllvm -amdgpu-sdwa-peephole=0.)
__device__ __forceinline__ u32 fadd(u32 a, u32 b) { return a + b; }
__device__ __forceinline__ u32 fsub(u32 a, u32 b) { return a - b; }
template <u32 kImm>
__device__ __forceinline__ u32 faddi(u32 a) { return a + kImm; }
template <u32 kImm>
__device__ __forceinline__ u32 fandi(u32 a) { return a & kImm; }
template <u32 kSh>
__device__ __forceinline__ u32 fshr(u32 a) { return a >> kSh; }
// bitop3 truth-table immediates (inputs a = 0xF0, b = 0xCC, c = 0xAA)
constexpr u32 kOrAnd = (0xF0 | 0xCC) & 0xAA;          // (a | b) & c
constexpr u32 kAndNot = 0xF0 & ~0xCC & 0xFF;          // a & ~b
constexpr u32 kSel = ((0xF0 & 0xAA) | (0xCC & ~0xAA)) & 0xFF;   // c ? a : b (bitwise)
constexpr u32 kBad = ((0xF0 | (~0xCC) | 0xAA)) & 0xFF;          // a | ~b | c
constexpr u32 kAndOr = ((0xF0 & 0xCC) | 0xAA) & 0xFF;           // (a & b) | c

// v - byte k of x (one SDWA subtract)
template <int kByte>
__device__ __forceinline__ u32 sub_byte(u32 v, u32 x) {
    u32 r;
    if constexpr (kByte == 0)
        asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(v), "v"(x));
    else if constexpr (kByte == 1)
        asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(v), "v"(x));
    else if constexpr (kByte == 2)
        asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(v), "v"(x));
    else
        asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(v), "v"(x));
    return r;
}

// ================================================================ ENCODE
// Staging (per wave): output position r of the tile (biased by 16: chunk 0 is a guard for the
// back-writes of non-starts) lives at byte r.
constexpr u32 kEncStage = 2048;   // >= 16 + 15 + 1512 + 2

struct EncState {
    u32 out_pos;    // compressed bytes produced so far
    u32 flushed;    // compressed bytes already stored (multiple of 16); staging chunk 1 = flushed
    u32 prev_top;   // input byte at tile_pos-1, in bits 24..31
    u32 rs;         // start position of the run holding input byte tile_pos-1
    u32 head;       // leading bytes of the first stored chunk that belong to the previous segment
    bool wt;        // write-through output stores (vstore)
    Stamps sp;      // diagnostic builds only
};

// Positions are absolute in the buffer.  Tokens start only below Uo (the end of the positions this
// wave owns: the buffer, or its segment); runs end at Ud (the buffer's end).
// Analysis of one encode tile (shared by enc_tile and the segment summary): per lane, the run
// boundary mask B (+ the next lane's 8 bits in B24), token starts T and 3-byte tokens P, and the
// wave max-scan of the last boundary position.  k64 (1024-byte tiles): all 64 lanes own their 16
// bytes, and `look` holds the first 8 bytes after the tile (the slot's tail, the same for every
// lane), from which lane 63 takes its next-lane bits.  Else lane 63 holds the next tile's first 16
// bytes (lookahead only) and `look` is unused.
struct EncAn {
    u32 w[4];
    u32 p0, validm, top, B, B24, incl, T, P;
};
// Register constants of the encode tile, made once per kernel (vconst: no rematerialisation).
struct EncK {
    u32 K80, C1, C2, V01;
};
__device__ __forceinline__ EncK enc_k() {
    return EncK{vconst(0x80808080u), vconst(0x08040201u), vconst(0x80402010u), vconst(0x01010101u)};
}
// enc_analyze_bounds: everything but the token masks, which depend on the run entering the tile
// (enc_tokens).
template <bool k64>
__device__ __forceinline__ EncAn enc_analyze_bounds(const u32x4 cur, const uint2 look, u32 pos, u32 Ud, u32 Uo,
                                                    u32 lane, u32 prev_top, const EncK& kc) {
    const bool owned = k64 || lane < kOwnLanes;
    EncAn a;
    a.w[0] = cur.x; a.w[1] = cur.y; a.w[2] = cur.z; a.w[3] = cur.w;
    const u32* w = a.w;
    const u32 p0 = pos + 16u * lane;
    a.p0 = p0;
    const u32 left = p0 < Ud ? Ud - p0 : 0u;
    const u32 nl = left < 16u ? left : 16u;
    const u32 lefto = p0 < Uo ? Uo - p0 : 0u;
    const u32 validm = owned ? lowmask(lefto < 16u ? lefto : 16u) : 0u;   // else lookahead only
    a.validm = validm;

    // run boundaries: bit j <=> x[p0+j] != x[p0+j-1] (or p0+j == 0); positions >= Ud end runs
    const u32 top = w[3] & 0xFF000000u;
    a.top = top;
    const u32 ptop = from_prev_lane(top, prev_top);
    const u32 pw[4] = {alignbyte(w[0], ptop, 3), alignbyte(w[1], w[0], 3), alignbyte(w[2], w[1], 3),
                       alignbyte(w[3], w[2], 3)};
    const u32 K80 = kc.K80;
    u32 g[4];   // 0x80 per byte that differs from the byte before it
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 t = w[k] ^ pw[k];
        g[k] = bitop3<kOrAnd>(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu), t, K80);
    }
    const u32 C1 = kc.C1, C2 = kc.C2;
    const u32 Ba = __builtin_amdgcn_udot4(g[1], C2, __builtin_amdgcn_udot4(g[0], C1, 0u, false), false);
    const u32 Bb = __builtin_amdgcn_udot4(g[3], C2, __builtin_amdgcn_udot4(g[2], C1, 0u, false), false);
    u32 B = (Ba >> 7) | (Bb + Bb);
    B |= (p0 == 0u) ? 1u : 0u;
    B |= ~lowmask(nl) & 0xFFFFu;
    a.B = B;
    // + the next lane's first 8 boundary bits (repeat lookahead); with k64, lane 63 compares the
    // tile's lookahead bytes against its last byte
    u32 Bn = 0xFFu;
    if (k64) {
        const u32 q0 = look.x ^ alignbyte(look.x, w[3], 3), q1 = look.y ^ alignbyte(look.y, look.x, 3);
        const u32 gq0 = bitop3<kOrAnd>(((q0 & 0x7F7F7F7Fu) + 0x7F7F7F7Fu), q0, K80);
        const u32 gq1 = bitop3<kOrAnd>(((q1 & 0x7F7F7F7Fu) + 0x7F7F7F7Fu), q1, K80);
        const u32 nl2 = left > 16u ? left - 16u : 0u;
        Bn = (__builtin_amdgcn_udot4(gq1, C2, __builtin_amdgcn_udot4(gq0, C1, 0u, false), false) >> 7) |
             (~lowmask(nl2 < 8u ? nl2 : 8u) & 0xFFu);
    }
    a.B24 = B | ((from_next_lane(B, Bn) & 0xFFu) << 16);

    // run start of byte p0-1: max-scan of the last boundary position per owning lane
    // (when every owned lane holds a boundary, each lane's own last one is already the running
    // max: the scan is skipped -- random and 50 %-runs data nearly always; without k64, lane 63's
    // value is then not the max, so consumers read the owned maximum from lane 62)
    const u32 lbp = (B && owned) ? p0 + 31u - (u32)__builtin_clz(B) : 0u;
    constexpr uint64_t kOwnedMask = k64 ? ~0ull : (1ull << kOwnLanes) - 1ull;
    const bool every = (__builtin_amdgcn_ballot_w64(B == 0u) & kOwnedMask) == 0ull;
    const u32 incl = every ? lbp : wave_scan_incl(lbp, 0u, OpMax());
    a.incl = incl;
    a.T = a.P = 0u;
    return a;
}
// Token masks of an analysed tile, given rs = the start of the run holding the byte before the
// tile: token starts T (run starts, 9 past a run start, and the continuation of the run entering
// the lane) and 3-byte tokens P.
__device__ __forceinline__ void enc_tokens(EncAn& a, u32 rs) {
    const u32 B = a.B;
    const u32 pm = from_prev_lane(a.incl, 0u);
    const u32 rsl = pm > rs ? pm : rs;
    const u32 qin = mod9(a.p0 - 1u - rsl);   // run phase of byte p0-1 (unused when p0 starts a run)
    const u32 f1 = (u32)__builtin_ctz(B | 0x10000u);
    u32 t8 = B | (B << 1);
    t8 |= t8 << 2;
    t8 |= t8 << 4;
    t8 |= B << 8;
    const u32 pre = (0x201u << (8u - qin)) & lowmask(f1);
    a.T = (B | ((B << 9) & ~t8) | pre) & a.validm;
    a.P = a.T & ~(a.B24 >> 1);   // 3-byte tokens: the run continues past the start
}
template <bool k64>
__device__ __forceinline__ EncAn enc_analyze(const u32x4 cur, const uint2 look, u32 pos, u32 Ud, u32 Uo, u32 lane,
                                             u32 prev_top, u32 rs, const EncK& kc) {
    EncAn a = enc_analyze_bounds<k64>(cur, look, pos, Ud, Uo, lane, prev_top, kc);
    enc_tokens(a, rs);
    return a;
}

// Pass 1 of enc_tile: every position writes its byte at its token's offset (starts) or at
// offset-2 of the next token (valid non-starts: its own token's second byte, a redundant identical
// write); positions past U write at the tile's output end, which is never stored.  e0 = staging
// address of the lane's first output byte; byte i of Q = output bytes of positions >= i of the
// dword (suffix sums by right shifts), so position i writes at endk - Q.byte_i (- 2).  kFull: all
// 16 positions of every owned lane are valid, so the non-starts are V01 - T01 (V01 = 0x01010101 on
// owned lanes, 0 on a lookahead lane) without an expansion of their own.
template <bool kFull>
__device__ __forceinline__ void enc_pass1(const u32* w, u32 T, u32 P, u32 NS, u32 e0, u32 V01) {
    u32 endk = e0;
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 T01 = nib_to_bytes(bfe(T, 4u * k, 4)), P01 = nib_to_bytes(bfe(P, 4u * k, 4));
        const u32 N01 = kFull ? V01 - T01 : nib_to_bytes(bfe(NS, 4u * k, 4));
        const u32 W = T01 + P01 + P01;
        u32 Q = W + (W >> 8);
        Q = Q + (Q >> 16);
        endk = endk + (Q & 0xFFu);
        const u32 R = Q + N01 + N01;
        auto put = [](u32 t, u32 v) { *reinterpret_cast<__attribute__((address_space(3))) uint8_t*>(t) = (uint8_t)v; };
        const u32 w8 = w[k] >> 8;
        put(sub_byte<0>(endk, R), w[k]);
        put(sub_byte<1>(endk, R), w8);
        put(sub_byte<2>(endk, R), w[k] >> 16);
        put(sub_byte<3>(endk, R), w8 >> 16);
    }
}

// ---------------------------------------------------------------- literal tiles (the fast path)
// A tile with no run longer than 2 (random and text-like data) encodes to its own bytes with a '2'
// inserted after each pair's second byte.  Each token belongs to the lane of its start, so a lane
// outputs its 16 bytes, less position 0 when that is the second byte of a pair started before the
// lane, plus the next lane's byte 0 when a pair starts at position 15, with <= 2 insertions (one
// LUT-selected v_perm per output dword): n = 15..19 bytes.  One 16-byte store writes its first 16
// output bytes (with 15, the 16th is the next lane's first: the bytes two lanes store twice are
// equal), a second one, for n > 16, its last 16.  Not for the last tile: the last owner's store
// may reach one byte past the tile's output, which the next tile rewrites (that byte is the next
// tile's first output: a lane outputs 15 bytes only when its position 15 starts a token that
// does not continue, so the next tile starts a token).  No staging, no pass 2.
// Insertion selectors: entry i (the output index of an inserted '2', 0 = none), dword q: the
// v_perm selector taking output bytes 4q..4q+3 from (S[q] : S[q-1] with bytes 0, 1 = '2').  Two
// insertions are two passes.  6 dwords per entry (5 used): 8-byte aligned reads.  Each wave
// LDS-DMAs its own copy (kInsDmaLanes x 16 bytes) ahead of its first tile.
constexpr u32 kInsEntries = 19u;
constexpr u32 kInsStride = 6u;
constexpr u32 kInsWords = kInsEntries * kInsStride;            // 114
constexpr u32 kInsDmaLanes = (4u * kInsWords + 15u) / 16u;      // 29
constexpr u32 kInsWaveWords = 4u * kInsDmaLanes;                // 116: one wave's copy
struct EncInsLut {
    u32 s[kInsWaveWords];
};
constexpr EncInsLut make_ins_lut() {
    EncInsLut t{};
    for (u32 i = 0; i < kInsEntries; ++i)
        for (u32 q = 0; q < 5u; ++q) {
            u32 sel = 0;
            for (u32 b = 0; b < 4u; ++b) {
                const u32 m = 4u * q + b;
                u32 v = 0;
                if (!(i && m == i)) v = m - ((i && i < m) ? 1u : 0u) - 4u * q + 4u;   // 3..7
                sel |= v << (8u * b);
            }
            t.s[i * kInsStride + q] = sel;
        }
    return t;
}
static __constant__ EncInsLut kEncInsLut = make_ins_lut();

// Returns the store instructions issued, or kNotFast (nothing done: the general path encodes the
// tile).  With st.head == 0.  kTail: the buffer's last tile (positions past U are neither tokens
// nor output).  Its output ends the stream at C = out_pos + ttot, so its stores go through a
// descriptor clipped at C (the range check drops dwords not wholly below it: nothing lands past
// C), and the last 4 output bytes are stored again as one dword ending at C, as in decode.
template <bool k64, bool kTail = false>
__device__ __forceinline__ u32 enc_tile_fast(const EncAn& a, const uint2 look, u32 pos, u32 lane, const u32* elut,
                                             uint8_t* stage, u32x4 rso, EncState& st) {
    constexpr u32 kLast = k64 ? 63u : kOwnLanes - 1u;
    const bool owned = k64 || lane < kOwnLanes;
    // continuations (bit j: byte j equals byte j-1) of the lane's 16 positions and the next lane's
    // first two; pairs: run starts whose run continues
    // (runs of 3+ first, in as few instructions as possible: run-heavy tiles leave here)
    const u32 C18 = ~a.B24 & 0x3FFFFu;
    if (__builtin_amdgcn_ballot_w64(((C18 & (C18 >> 1)) != 0u) && owned)) return kNotFast;
    const u32 vm = kTail ? a.validm : 0xFFFFu;   // positions below U (positions past U are boundaries)
    const u32 P = a.B & ~(a.B24 >> 1) & vm;
    if (__builtin_amdgcn_ballot_w64(__builtin_popcount(P) > 2 && owned)) return kNotFast;
    if ((readlane(C18, 0) & 1u) && st.rs + 1u != pos) return kNotFast;   // the run entering is longer
    const u32 del0 = C18 & 1u;
    const u32 nout = owned ? (u32)__builtin_popcount(vm) - del0 + ((P >> 15) & 1u) + (u32)__builtin_popcount(P) : 0u;
    const u32 oincl = wave_scan_incl(nout, 0u, OpAdd());
    const u32 ttot = readlane(oincl, 63);
    if (kTail) {
        if (ttot < 4u) return kNotFast;
        rso.z = uniform(st.out_pos + ttot);   // clip every store of this tile at C
        asm volatile("s_nop 4" ::: "memory");   // (the descriptor word is fresh)
    }

    u32 rounds = 0;
    const u32 rel0 = st.out_pos - st.flushed;
    if (rel0) {   // a general tile's partial chunk (its bytes past rel0 are rewritten below)
        const u32x4 v = *reinterpret_cast<const u32x4*>(stage + 16u);
        vstore(rso, lane == 0u ? st.flushed : kOOB, v, st.wt);
        rounds = 1;
    }
    // source bytes S' (the lane's 16 and the next lane's first, less position 0 when deleted)
    const u32* w = a.w;
    const u32 nw0 = from_next_lane(w[0], 0u);   // (all lanes: a DPP inside the select may run with lane 63 off)
    const u32 s4 = (k64 && lane == 63u) ? look.x : nw0;
    const u32 sh = 8u * del0;
    const u32 Sp[5] = {alignbyte(w[1], w[0], del0), alignbyte(w[2], w[1], del0), alignbyte(w[3], w[2], del0),
                       alignbyte(s4, w[3], del0), s4 >> sh};
    const u32 j1 = (u32)__builtin_ctz(P | 0x10000u), j2 = (u32)__builtin_ctz((P & (P - 1u)) | 0x10000u);
    const u32 k2 = 0x32323232u;
    typedef u32 u32x2 __attribute__((ext_vector_type(2)));
    // one insertion pass: out[q] = bytes of in[] with a '2' at output index i (0: none)
    auto insert = [&](const u32* in, u32 i, u32* out) {
        const u32* e = elut + i * kInsStride;
        const u32x2 e01 = *reinterpret_cast<const u32x2*>(e), e23 = *reinterpret_cast<const u32x2*>(e + 2),
                    e45 = *reinterpret_cast<const u32x2*>(e + 4);
        out[0] = __builtin_amdgcn_perm(in[0], k2, e01.x);
        out[1] = __builtin_amdgcn_perm(in[1], __builtin_amdgcn_perm(in[0], k2, 0x07060100u), e01.y);
        out[2] = __builtin_amdgcn_perm(in[2], __builtin_amdgcn_perm(in[1], k2, 0x07060100u), e23.x);
        out[3] = __builtin_amdgcn_perm(in[3], __builtin_amdgcn_perm(in[2], k2, 0x07060100u), e23.y);
        out[4] = __builtin_amdgcn_perm(in[4], __builtin_amdgcn_perm(in[3], k2, 0x07060100u), e45.x);
    };
    u32 out[5];
    insert(Sp, j1 < 16u ? j1 + 2u - del0 : 0u, out);
    if (__builtin_amdgcn_ballot_w64(j2 < 16u)) {   // second pairs (the '2' after the first counts)
        const u32 o1[5] = {out[0], out[1], out[2], out[3], out[4]};
        insert(o1, j2 < 16u ? j2 + 3u - del0 : 0u, out);
    }
    // the first 16 output bytes (with 15, the next lane's first byte last)
    const u32 n0 = from_next_lane(out[0], 0u);
    u32x4 va;
    va.x = out[0]; va.y = out[1]; va.z = out[2];
    va.w = __builtin_amdgcn_perm(n0, out[3], nout >= 16u ? 0x03020100u : 0x04020100u);
    const u32 o = st.out_pos + oincl - nout;
    vstore(rso, owned ? o : kOOB, va, st.wt);
    // the last 16, where there are more than 16
    if (__builtin_amdgcn_ballot_w64(nout > 16u)) {
        const u32 b = nout - 16u;
        u32x4 vb;
        vb.x = alignbyte(out[1], out[0], b); vb.y = alignbyte(out[2], out[1], b);
        vb.z = alignbyte(out[3], out[2], b); vb.w = alignbyte(out[4], out[3], b);
        vstore(rso, nout > 16u ? o + b : kOOB, vb, st.wt);
        ++rounds;
    }
    if (kTail) {
        // the last 4 bytes of each lane's output (n >= 15 on full lanes; with n < 4, the end of the
        // full lane before it first), stored by the last lane with output as a dword ending at C
        const u32 s4b = nout - 4u, qd = s4b >> 2;
        const u32 lo = qd == 0u ? out[0] : qd == 1u ? out[1] : qd == 2u ? out[2] : out[3];
        const u32 hi = qd == 0u ? out[1] : qd == 1u ? out[2] : qd == 2u ? out[3] : out[4];
        const u32 T4 = alignbyte(hi, lo, s4b & 3u);
        const u32 Tp = from_prev_lane(T4, 0u);
        const u32 T = nout >= 4u ? T4 : alignbyte(out[0], Tp, nout);
        const uint64_t has = __builtin_amdgcn_ballot_w64(nout != 0u);
        const u32 last = 63u - (u32)__builtin_clzll(has);
        vstore4(rso, lane == last ? st.out_pos + ttot - 4u : kOOB, T, st.wt);
        ++rounds;
    }
    st.out_pos += ttot;
    st.flushed = st.out_pos;
    st.prev_top = readlane(a.top, kLast);
    const u32 i63 = readlane(a.incl, kLast);
    st.rs = i63 > st.rs ? i63 : st.rs;
    return rounds + 1u;
}

// A tile that is one run (no run boundary past its first byte: zero data, long runs) encodes to
// the tokens "v v '9'" every 9 bytes from the run start, the last one's count from the bytes after
// the tile (up to 8 lookahead boundary bits), or a lone "v" when that count is 1.  Its output is
// then a 3-periodic pattern: lane c forms staged chunk c (the partial chunk's bytes first) and
// the flush stores it; the new partial chunk goes back to the staging.  Not for the last tile.
__device__ __forceinline__ u32 rep_byte(u32 v) { return __builtin_amdgcn_perm(0u, v, 0u); }
// The output of `span` bytes that are one run (from rs, run start; v its byte; ext: run bytes past
// the span, up to 8), after the partial chunk staged so far.  One store round: span <= 2048 gives
// at most 15 + 3 * 228 bytes, 44 chunks.
__device__ __forceinline__ void enc_run_emit(u32 pos, u32 span, u32 rs, u32 ext, u32 v, u32 lane, uint8_t* stage,
                                             u32x4 rso, EncState& st) {
    const u32 f = pos + (9u - (pos - rs) % 9u) % 9u;          // first token start in the span
    const u32 ns = (pos + span - f + 8u) / 9u;                // token starts in the span (>= 1)
    const u32 sl = f + 9u * (ns - 1u);
    const u32 cl = pos + span + ext - sl < 9u ? pos + span + ext - sl : 9u;     // last token's count
    const u32 tot = 3u * (ns - 1u) + (cl >= 2u ? 3u : 1u);
    const u32 rel0 = st.out_pos - st.flushed;
    const u32 rel = rel0 + tot, nfl = rel >> 4;
    // lane c: staged chunk c = output bytes k = 16 c + i - rel0 of this span (k < 0: the old partial)
    const u32 k0 = 16u * lane - rel0;                         // may wrap for lane 0
    const u32 ph = (16u * lane + 48u - rel0) % 3u;            // k0 mod 3
    const u32 vv = rep_byte(v), d9 = 0x39393939u;
    // byte i is the count digit where (ph + i) % 3 == 2
    u32 o[4];
#pragma unroll
    for (u32 q = 0; q < 4u; ++q) {
        // digit masks for phase 0, 1, 2 of dword q (i = 4q + b, digit when (ph + i) % 3 == 2)
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
    // the last token: count cl (digit at k = tot - 1 when cl >= 2)
    if (cl != 9u && cl >= 2u) {
        const u32 kd = tot - 1u - k0;                          // byte index in this lane's chunk
        if (kd < 16u) {
            const u32 sh = 8u * (kd & 3u);
            const u32 dv = (0x30u + cl) << sh, msk = 0xFFu << sh;
            const u32 q = kd >> 2;
            o[0] = q == 0u ? (o[0] & ~msk) | dv : o[0];
            o[1] = q == 1u ? (o[1] & ~msk) | dv : o[1];
            o[2] = q == 2u ? (o[2] & ~msk) | dv : o[2];
            o[3] = q == 3u ? (o[3] & ~msk) | dv : o[3];
        }
    }
    // chunk 0: the old partial chunk's rel0 bytes first
    const u32x4 old = *reinterpret_cast<const u32x4*>(stage + 16u);
    if (lane == 0u && rel0) {
        const u32 ov[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
        for (u32 q = 0; q < 4u; ++q) {
            const u32 nb = rel0 > 4u * q ? (rel0 - 4u * q < 4u ? rel0 - 4u * q : 4u) : 0u;
            const u32 m = lowmask(8u * nb);
            o[q] = (ov[q] & m) | (o[q] & ~m);
        }
    }
    const u32x4 ov4 = u32x4{o[0], o[1], o[2], o[3]};
    vstore(rso, lane < nfl ? st.flushed + 16u * lane : kOOB, ov4, st.wt);
    wave_lds_sync();   // every lane has read the old partial chunk
    if (lane == nfl) *reinterpret_cast<u32x4*>(stage + 16u) = ov4;   // the new partial chunk
    wave_lds_sync();
    st.flushed += 16u * nfl;
    st.out_pos += tot;
}
template <bool k64>
__device__ __forceinline__ u32 enc_tile_run(const EncAn& a, u32 pos, u32 lane, uint8_t* stage, u32x4 rso,
                                            EncState& st) {
    constexpr u32 kLast = k64 ? 63u : kOwnLanes - 1u;
    constexpr u32 kStep = k64 ? kEncStep : kTileStep;
    const bool owned = k64 || lane < kOwnLanes;
    if (__builtin_amdgcn_ballot_w64((a.B & (lane == 0u ? 0xFFFEu : 0xFFFFu)) != 0u && owned)) return kNotFast;
    const u32 rs = (readlane(a.B, 0) & 1u) ? pos : st.rs;     // the run's start
    const u32 ext = (u32)__builtin_ctz((readlane(a.B24, kLast) >> 16) | 0x100u);   // run bytes past the tile
    enc_run_emit(pos, kStep, rs, ext, readlane(a.w[0], 0) & 0xFFu, lane, stage, rso, st);
    st.prev_top = readlane(a.top, kLast);
    const u32 i63 = readlane(a.incl, kLast);
    st.rs = i63 > st.rs ? i63 : st.rs;
    return 1u;
}

// One tile from its boundary analysis (enc_analyze_bounds): the fast paths when they apply, else
// the general path.  Returns the store instructions issued.
template <bool k64, bool kFast = false>
__device__ __forceinline__ u32 enc_tile_an(EncAn an, const uint2 look, u32 pos, u32 Ud, u32 Uo, u32 lane,
                                           uint8_t* stage, uint8_t* dst, u32x4 rso, EncState& st, const EncK& kc,
                                           const u32* elut) {
    if (kFast && !st.head) {
        if (pos + (k64 ? kEncStep : kTileStep) < Uo) {
            u32 r = enc_tile_run<k64>(an, pos, lane, stage, rso, st);
            if (r != kNotFast) return r;
            r = enc_tile_fast<k64>(an, look, pos, lane, elut, stage, rso, st);
            if (r != kNotFast) return r;
        } else if (Uo == Ud) {   // the buffer's last tile (not a segment's)
            const u32 r = enc_tile_fast<k64, true>(an, look, pos, lane, elut, stage, rso, st);
            if (r != kNotFast) return r;
        }
    }
    enc_tokens(an, st.rs);
    constexpr u32 kLast = k64 ? 63u : kOwnLanes - 1u;   // the tile's last owning lane
    const u32* w = an.w;
    const u32 validm = an.validm, top = an.top, B24 = an.B24, incl = an.incl, T = an.T, P = an.P;

    const u32 nout = bcnt(P, bcnt(P, bcnt(T, 0u)));
    const u32 oincl = wave_scan_incl(nout, 0u, OpAdd());
    const u32 ttot = readlane(oincl, 63);
    const u32 rel0 = st.out_pos - st.flushed;   // 0..15: bytes of the partial chunk

    RLE_STAMP(st.sp, 1);   // boundaries, run phase, token masks, offsets
    // pass 1: every position writes its byte.  A start writes at its token's offset; a valid
    // non-start (inside a 3-byte token) writes the same byte at offset-2 of the NEXT token,
    // i.e. its own token's second byte (a redundant, identical write); positions past U write
    // at the tile's output end, which is never stored.  Per-position weights (T + 2P) and
    // back-offsets (2 for valid non-starts) are byte vectors.
    const u32 NS = validm & ~T;
#ifndef RLE_EABL   // encode ablation builds (timing only): 1 no pass 1, 2 no pass 2, 4 no flush stores
#define RLE_EABL 0
#endif
    // staging byte address after this lane's output; byte i of Q = output bytes of positions >= i
    // of the dword (suffix sums by right shifts), so position i writes at endk - Q.byte_i (- 2)
    if (!(RLE_EABL & 1)) {
        const u32 e0 = lds_addr(stage) + 16u + rel0 + oincl - nout;
        if (pos + (k64 ? kEncStep : kTileStep) <= Uo)
            enc_pass1<true>(w, T, P, NS, e0, (k64 || lane < kOwnLanes) ? kc.V01 : 0u);
        else enc_pass1<false>(w, T, P, NS, e0, 0u);
    }
    RLE_STAMP(st.sp, 2);   // pass 1
    // pass 2: the count digit of each 3-byte token, '0' + min(9, run left), at its start + 2.
    // (Pass 1 already wrote every token's second byte from the position holding it, except where
    // that position lies past the wave's owned range: those few are written after the loop.)
    const u32 obase = 16u + rel0 + oincl - nout;
    u32 prem = (RLE_EABL & 2) ? 0u : P;
    while (__builtin_amdgcn_ballot_w64(prem != 0u)) {
        if (prem) {
            const u32 j = (u32)__builtin_ctz(prem);
            prem &= prem - 1u;
            const u32 mj = lowmask(j);
            const u32 oj = bcnt(P & mj, bcnt(P & mj, bcnt(T & mj, obase)));
            stage[oj + 2u] = (uint8_t)('1' + (u32)__builtin_ctz((B24 >> (j + 1u)) | 0x100u));
        }
    }
    // second bytes whose position is not owned here (the lane's last valid position, when the
    // next one belongs to the next tile, segment or nothing)
    const u32 vnext = (validm >> 1) | ((from_next_lane(validm, 0u) & 1u) << 15);
    const u32 PX = (RLE_EABL & 2) ? 0u : (P & ~vnext);
    if (__builtin_amdgcn_ballot_w64(PX != 0u)) {
        if (PX) {
            const u32 j = (u32)__builtin_ctz(PX);
            const u32 mj = lowmask(j);
            const u32 oj = bcnt(P & mj, bcnt(P & mj, bcnt(T & mj, obase)));
            const u32 wj = j < 4u ? w[0] : j < 8u ? w[1] : j < 12u ? w[2] : w[3];
            stage[oj + 1u] = (uint8_t)(wj >> (8u * (j & 3u)));
        }
    }
    wave_lds_sync();
    RLE_STAMP(st.sp, 3);   // pass 2

    // store the completed 16-byte chunks (staging chunks 1..nfl), then move the partial one
    const u32 newrel = rel0 + ttot;
    const u32 nfl = newrel >> 4;
    const u32 rounds = (nfl + kWave - 1u) / kWave;
    for (u32 k = 0; k < rounds; ++k) {
        const u32 c = k * kWave + lane;
        // read unconditionally: an inactive lane's chunk (at most one past this wave's staging) is
        // garbage it never stores, and LDS reads do not fault
        const u32x4 v = *reinterpret_cast<const u32x4*>(stage + 16u * (c + 1u));
        const bool skip = st.head && c == 0u;   // shared with the previous segment: byte stores below
        vstore(rso, (c < nfl && !skip && !(RLE_EABL & 4)) ? st.flushed + 16u * c : kOOB, v, st.wt);
        if (skip && nfl) {
            const u32 wv[4] = {v.x, v.y, v.z, v.w};
            for (u32 j = st.head; j < 16u; ++j) dst[st.flushed + j] = (uint8_t)(wv[j >> 2] >> (8u * (j & 3u)));
        }
    }
    if (nfl) st.head = 0;
    RLE_STAMP(st.sp, 4);   // flush
    if (nfl && lane < 4u) {
        u32* s32 = reinterpret_cast<u32*>(stage);
        s32[4u + lane] = s32[4u * (nfl + 1u) + lane];
    }
    wave_lds_sync();
    st.flushed += 16u * nfl;
    st.out_pos += ttot;
    st.prev_top = readlane(top, kLast);
    const u32 i63 = readlane(incl, kLast);
    st.rs = i63 > st.rs ? i63 : st.rs;
    RLE_STAMP(st.sp, 5);   // partial-chunk move, state
    return rounds;
}
template <bool k64, bool kFast = false>
__device__ __forceinline__ u32 enc_tile(const uint8_t* cslot, const Refill& next, u32 pos, u32 Ud, u32 Uo,
                                        u32 lane, uint8_t* stage, uint8_t* dst, u32x4 rso, EncState& st,
                                        const EncK& kc, const u32* elut = nullptr) {
    RLE_STAMP(st.sp, 0);   // DMA wait + loop
    const u32x4 cur = *reinterpret_cast<const u32x4*>(cslot + 16u * lane);
    const uint2 look = k64 ? *reinterpret_cast<const uint2*>(cslot + kSlot) : uint2{0u, 0u};
    next();   // the slot is free once read
    const EncAn an = enc_analyze_bounds<k64>(cur, look, pos, Ud, Uo, lane, st.prev_top, kc);
    return enc_tile_an<k64, kFast>(an, look, pos, Ud, Uo, lane, stage, dst, rso, st, kc, elut);
}

__device__ __forceinline__ u32 max_u(u32 a, u32 b) { return a > b ? a : b; }
// ---------------------------------------------------------------- two tiles per step (1024-byte tiles)
// A lone wave spends ~0.9 us per tile (r3n timelines: one wave per SIMD), about 12 cycles per
// instruction: each tile is one dependent chain (LDS read, SWAR, DPP scans, readlanes, stores).
// The tiles of a buffer depend on each other only through a few scalars (the byte before the
// tile, the entering run start, the output offset), so a step takes two tiles: both analyses and
// both offset scans are independent, and the compiler interleaves them.  Pair forms:
//  * run pair: both tiles one run (a boundary at most at the first byte) -- one run emission over
//    2048 bytes (enc_run_emit);
//  * literal pair: both tiles literal (enc_tile_fast's conditions), the second possibly the
//    buffer's last tile (kTail1: its stores clipped at C, its last dword stored again).
// Anything else runs the two tiles one after the other from their analyses (enc_tile_an).
// literal output of one tile: the lane's bytes with the '2's inserted (enc_tile_fast's body)
struct EncLit {
    u32 out[5];
    u32 nout, j2;
};
__device__ __forceinline__ void enc_lit_insert(const u32* elut, const u32* in, u32 i, u32* out) {
    typedef u32 u32x2 __attribute__((ext_vector_type(2)));
    const u32 k2 = 0x32323232u;
    const u32* e = elut + i * kInsStride;
    const u32x2 e01 = *reinterpret_cast<const u32x2*>(e), e23 = *reinterpret_cast<const u32x2*>(e + 2),
                e45 = *reinterpret_cast<const u32x2*>(e + 4);
    out[0] = __builtin_amdgcn_perm(in[0], k2, e01.x);
    out[1] = __builtin_amdgcn_perm(in[1], __builtin_amdgcn_perm(in[0], k2, 0x07060100u), e01.y);
    out[2] = __builtin_amdgcn_perm(in[2], __builtin_amdgcn_perm(in[1], k2, 0x07060100u), e23.x);
    out[3] = __builtin_amdgcn_perm(in[3], __builtin_amdgcn_perm(in[2], k2, 0x07060100u), e23.y);
    out[4] = __builtin_amdgcn_perm(in[4], __builtin_amdgcn_perm(in[3], k2, 0x07060100u), e45.x);
}
// P (pair starts) and the lane's output count of a literal k64 tile; vm: valid positions
__device__ __forceinline__ u32 enc_lit_count(const EncAn& a, u32 vm, u32& P) {
    const u32 C18 = ~a.B24 & 0x3FFFFu;
    P = a.B & ~(a.B24 >> 1) & vm;
    return (u32)__builtin_popcount(vm) - (C18 & 1u) + ((P >> 15) & 1u) + (u32)__builtin_popcount(P);
}
__device__ __forceinline__ bool enc_lit_reject(const EncAn& a, u32 vm) {
    const u32 C18 = ~a.B24 & 0x3FFFFu;
    const u32 P = a.B & ~(a.B24 >> 1) & vm;
    return (C18 & (C18 >> 1)) != 0u || __builtin_popcount(P) > 2;
}
// Output offsets of a whole literal k64 tile (every position below U) without a DPP scan
// (RLE_ENC_MBCNT, round 5).  Lane l outputs n_l = 16 - del0_l + p15_l + pc_l (del0: its position 0
// continues a pair begun before the lane; p15: a pair starts at its position 15; pc <= 2: its pair
// starts).  With no run longer than 2, p15_l = del0_{l+1}, so the sum over the lanes before l
// telescopes: exclusive offset 16 l + del0_l - del0_0 + (pairs of the lanes before l, two ballots
// counted with v_mbcnt); the tile's total from the same ballots, p15_63 from lane 63's lookahead.
__device__ __forceinline__ u32 mbcnt64(uint64_t b) {
    return __builtin_amdgcn_mbcnt_hi((u32)(b >> 32), __builtin_amdgcn_mbcnt_lo((u32)b, 0u));
}
__device__ __forceinline__ void enc_lit_offsets(const EncAn& a, u32 P, u32 lane, u32& ox, u32& tot) {
    const u32 del0 = (~a.B24) & 1u;
    const u32 pc = (u32)__builtin_popcount(P);
    const uint64_t B1 = __builtin_amdgcn_ballot_w64(pc >= 1u), B2 = __builtin_amdgcn_ballot_w64(pc >= 2u);
    const uint64_t Bd = __builtin_amdgcn_ballot_w64(del0 != 0u);
    const uint64_t Bp = __builtin_amdgcn_ballot_w64(lane == 63u && ((P >> 15) & 1u) != 0u);
    const u32 d00 = (u32)Bd & 1u;
    ox = 16u * lane + del0 - d00 + mbcnt64(B1) + mbcnt64(B2);
    tot = 16u * kWave + (u32)(Bp >> 63) - d00 + (u32)__builtin_popcountll(B1) + (u32)__builtin_popcountll(B2);
}
// first insertion pass (the second, for lanes with two pairs, is the caller's: enc_lit_second)
__device__ __forceinline__ EncLit enc_lit_first(const EncAn& a, const uint2 look, u32 lane, u32 P, u32 nout,
                                                const u32* elut) {
    EncLit r;
    const u32* w = a.w;
    const u32 del0 = (~a.B24) & 1u;
    const u32 nw0 = from_next_lane(w[0], 0u);
    const u32 s4 = lane == 63u ? look.x : nw0;
    const u32 sh = 8u * del0;
    const u32 Sp[5] = {alignbyte(w[1], w[0], del0), alignbyte(w[2], w[1], del0), alignbyte(w[3], w[2], del0),
                       alignbyte(s4, w[3], del0), s4 >> sh};
    const u32 j1 = (u32)__builtin_ctz(P | 0x10000u), j2 = (u32)__builtin_ctz((P & (P - 1u)) | 0x10000u);
    enc_lit_insert(elut, Sp, j1 < 16u ? j1 + 2u - del0 : 0u, r.out);
    r.nout = nout;
    r.j2 = j2 < 16u ? j2 + 3u - del0 : 0u;
    return r;
}
__device__ __forceinline__ void enc_lit_second(EncLit& r, const u32* elut) {
    const u32 o1[5] = {r.out[0], r.out[1], r.out[2], r.out[3], r.out[4]};
    enc_lit_insert(elut, o1, r.j2, r.out);
}
// the stores of one literal tile whose output starts at base (va: first 16 bytes; vb: last 16);
// oexcl: the lane's exclusive output offset in the tile
__device__ __forceinline__ void enc_lit_store(const EncLit& r, u32 base, u32 oexcl, u32x4 rso, bool wt) {
    const u32 n0 = from_next_lane(r.out[0], 0u);
    u32x4 va;
    va.x = r.out[0]; va.y = r.out[1]; va.z = r.out[2];
    va.w = __builtin_amdgcn_perm(n0, r.out[3], r.nout >= 16u ? 0x03020100u : 0x04020100u);
    const u32 o = base + oexcl;
    vstore(rso, r.nout ? o : kOOB, va, wt);
}
__device__ __forceinline__ void enc_lit_store_b(const EncLit& r, u32 base, u32 oexcl, u32x4 rso, bool wt) {
    const u32 o = base + oexcl;
    const u32 b = r.nout - 16u;
    u32x4 vb;
    vb.x = alignbyte(r.out[1], r.out[0], b); vb.y = alignbyte(r.out[2], r.out[1], b);
    vb.z = alignbyte(r.out[3], r.out[2], b); vb.w = alignbyte(r.out[4], r.out[3], b);
    vstore(rso, r.nout > 16u ? o + b : kOOB, vb, wt);
}

// Two 1024-byte tiles (k64 walks: buffers up to 16 KiB) at pos and pos + 1024; slot A holds the
// first, slot B the second.  Returns the store instructions issued after the refills.
template <bool kFast>
__device__ __forceinline__ u32 enc_pair(const uint8_t* slotA, const uint8_t* slotB, const Refill& nxA,
                                        const Refill& nxB, u32 pos, u32 U, u32 lane, uint8_t* stage, uint8_t* dst,
                                        u32x4 rso, EncState& st, const EncK& kc, const u32* elut) {
    const u32x4 curA = *reinterpret_cast<const u32x4*>(slotA + 16u * lane);
    const uint2 lookA = *reinterpret_cast<const uint2*>(slotA + kSlot);
    const u32x4 curB = *reinterpret_cast<const u32x4*>(slotB + 16u * lane);
    const uint2 lookB = *reinterpret_cast<const uint2*>(slotB + kSlot);
    nxA();
    nxB();
    const u32 pos1 = pos + kEncStep;
    const EncAn a0 = enc_analyze_bounds<true>(curA, lookA, pos, U, U, lane, st.prev_top, kc);
    // the byte before tile 1: tile 0's last byte (lane 63's top), from the data
    const EncAn a1 = enc_analyze_bounds<true>(curB, lookB, pos1, U, U, lane, readlane(curA.w & 0xFF000000u, 63), kc);
    if (kFast && !st.head) {
        const bool last1 = pos1 + kEncStep >= U;   // tile 1 is the buffer's last tile
        // run pair: both tiles one run (tile 1's first byte continues tile 0's last)
        if (!last1) {
            const bool brk = (a0.B & (lane == 0u ? 0xFFFEu : 0xFFFFu)) != 0u || a1.B != 0u;
            if (!__builtin_amdgcn_ballot_w64(brk)) {
                const u32 rs = (readlane(a0.B, 0) & 1u) ? pos : st.rs;
                const u32 ext = (u32)__builtin_ctz((readlane(a1.B24, 63) >> 16) | 0x100u);
                enc_run_emit(pos, 2u * kEncStep, rs, ext, readlane(a0.w[0], 0) & 0xFFu, lane, stage, rso, st);
                st.prev_top = readlane(a1.top, 63);
                const u32 i63 = readlane(a1.incl, 63);
                st.rs = i63 > st.rs ? i63 : st.rs;
                return 1u;
            }
        }
        // literal pair
        const u32 vm1 = last1 ? a1.validm : 0xFFFFu;
        const bool rej = enc_lit_reject(a0, 0xFFFFu) || enc_lit_reject(a1, vm1);
        const u32 rs1 = max_u(readlane(a0.incl, 63), st.rs);   // the run holding tile 1's byte before
        if (!__builtin_amdgcn_ballot_w64(rej) && !((readlane(~a0.B24, 0) & 1u) && st.rs + 1u != pos) &&
            !((readlane(~a1.B24, 0) & 1u) && rs1 + 1u != pos1)) {
            u32 P0, P1;
            const u32 n0 = enc_lit_count(a0, 0xFFFFu, P0), n1 = enc_lit_count(a1, vm1, P1);
            u32 oi0, oi1, t0, t1;   // (exclusive offsets, totals)
            if (pos1 + kEncStep <= U) {   // both tiles whole
                enc_lit_offsets(a0, P0, lane, oi0, t0);
                enc_lit_offsets(a1, P1, lane, oi1, t1);
            } else {
                oi0 = wave_scan_incl(n0, 0u, OpAdd());
                oi1 = wave_scan_incl(n1, 0u, OpAdd());
                t0 = readlane(oi0, 63);
                t1 = readlane(oi1, 63);
                oi0 -= n0;
                oi1 -= n1;
            }
            if (!last1 || t1 >= 4u) {
                EncLit L0 = enc_lit_first(a0, lookA, lane, P0, n0, elut);
                EncLit L1 = enc_lit_first(a1, lookB, lane, P1, n1, elut);
                if (__builtin_amdgcn_ballot_w64(L0.j2 != 0u || L1.j2 != 0u)) {
                    enc_lit_second(L0, elut);
                    enc_lit_second(L1, elut);
                }
                u32 rounds = 2u;
                const u32 rel0 = st.out_pos - st.flushed;
                const u32 base0 = st.out_pos, base1 = st.out_pos + t0, C = base1 + t1;
                // a last pair clips every store at C (tile 0's reach past its output too)
                const u32x4 rsc = u32x4{rso.x, rso.y, uniform(last1 ? C : rso.z), rso.w};
                asm volatile("s_nop 4" ::: "memory");   // (the descriptor word is fresh)
                if (rel0) {   // a general tile's partial chunk (its bytes past rel0 are rewritten below)
                    const u32x4 v = *reinterpret_cast<const u32x4*>(stage + 16u);
                    vstore(rsc, lane == 0u ? st.flushed : kOOB, v, st.wt);
                    ++rounds;
                }
                enc_lit_store(L0, base0, oi0, rsc, st.wt);
                if (__builtin_amdgcn_ballot_w64(n0 > 16u)) {
                    enc_lit_store_b(L0, base0, oi0, rsc, st.wt);
                    ++rounds;
                }
                enc_lit_store(L1, base1, oi1, rsc, st.wt);
                if (__builtin_amdgcn_ballot_w64(n1 > 16u)) {
                    enc_lit_store_b(L1, base1, oi1, rsc, st.wt);
                    ++rounds;
                }
                if (last1) {
                    // tile 1's last 4 output bytes as one dword ending at C (enc_tile_fast<kTail>)
                    const u32 nout = n1;
                    const u32* out = L1.out;
                    const u32 s4b = nout - 4u, qd = s4b >> 2;
                    const u32 lo = qd == 0u ? out[0] : qd == 1u ? out[1] : qd == 2u ? out[2] : out[3];
                    const u32 hi = qd == 0u ? out[1] : qd == 1u ? out[2] : qd == 2u ? out[3] : out[4];
                    const u32 T4 = alignbyte(hi, lo, s4b & 3u);
                    const u32 Tp = from_prev_lane(T4, 0u);
                    const u32 T = nout >= 4u ? T4 : alignbyte(out[0], Tp, nout);
                    const uint64_t has = __builtin_amdgcn_ballot_w64(nout != 0u);
                    const u32 lastl = 63u - (u32)__builtin_clzll(has);
                    vstore4(rsc, lane == lastl ? C - 4u : kOOB, T, st.wt);
                    ++rounds;
                }
                st.out_pos = C;
                st.flushed = C;
                st.prev_top = readlane(a1.top, 63);
                const u32 i63 = readlane(a1.incl, 63);
                st.rs = i63 > rs1 ? i63 : rs1;
                return rounds;
            }
        }
    }
    // one after the other
    const u32 r0 = enc_tile_an<true, kFast>(a0, lookA, pos, U, U, lane, stage, dst, rso, st, kc, elut);
    const u32 r1 = enc_tile_an<true, kFast>(a1, lookB, pos1, U, U, lane, stage, dst, rso, st, kc, elut);
    return r0 + r1;
}
// A walk two tiles per step (slots A, B; the last tile of an odd count alone, in slot A).  As
// walk_tiles: the wait before a step leaves only the previous step's stores in flight; a step
// returning ~0u stops the walk (drained; returns true).
template <u32 kStep = kTileStep, bool kLook = false, class Pair, class Single>
__device__ __forceinline__ bool walk_pairs(u32x4 rs, u32 start, u32 ntiles, u32 lane, const uint8_t* slots, Pair pair,
                                           Single single, bool primed = false) {
    constexpr u32 kStride = kLook ? kEncSlot : kSlot;
    const u32 lo = start + 16u * lane;
    const u32 l0 = uniform(lds_addr(slots)), l1 = l0 + kStride;
    const bool look = kLook && lane == 0u;
    if (!primed) walk_prime<kStep, kLook>(rs, start, ntiles, lane, slots);
    u32 p1 = 0, t = 0;
    for (; t + 1u < ntiles; t += 2u) {
        vm_wait(p1);
        p1 = pair(t, slots, slots + kStride, Refill{rs, (t + 2u) * kStep + lo, l0, t + 2u < ntiles, look},
                  Refill{rs, (t + 3u) * kStep + lo, l1, t + 3u < ntiles, look});
        if (p1 == ~0u) {
            vm_drain();
            return true;
        }
    }
    if (t < ntiles) {
        vm_wait(p1);
        if (single(t, slots, Refill{rs, 0u, l0, false, look}) == ~0u) {
            vm_drain();
            return true;
        }
    }
    return false;
}

// ================================================================ DECODE
// Token-phase table, indexed by an 8-bit mask n of "byte j differs from byte j+1" (the complement
// of the 3-byte-token mask) and entry offset d (the first token start in the group, 0..2):
// .x byte d = token-start mask, .y byte d = offset of the first start past the group (.y byte 3
// = 3, so .y is a v_perm selector).
struct DecTable {
    uint2 e[256];
};
constexpr DecTable make_dec_table() {
    DecTable t{};
    for (u32 n = 0; n < 256; ++n) {
        const u32 e = ~n & 0xFFu;
        u32 masks = 0, exits = 3u << 24;
        for (u32 d = 0; d < 3; ++d) {
            u32 s = d, m = 0;
            while (s < 8) {
                m |= 1u << s;
                s += ((e >> s) & 1u) ? 3u : 1u;
            }
            masks |= m << (8u * d);
            exits |= (s - 8u) << (8u * d);
        }
        t.e[n].x = masks;
        t.e[n].y = exits;
    }
    return t;
}
static __constant__ DecTable kDecTable = make_dec_table();
typedef uint2 DecEntry;
__device__ __forceinline__ DecEntry dec_entry_from(uint2 e) { return e; }
__device__ __forceinline__ DecEntry lds_entry(u32 a) {
    typedef u32 u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = *reinterpret_cast<const __attribute__((address_space(3))) u32x2*>(a);
    return make_uint2(v.x, v.y);
}

// Staging (per wave): decoded position r (biased by 16: chunk 0 is a guard, never stored) holds a
// u16 key: 0x80 << 8 | byte where a token starts, else 0 or an unflagged byte.  Chunk c is the 32
// bytes at 32 c; the flush reads and re-zeroes a chunk with two 16-byte accesses and ORs each
// position's index into bits 8..11, so that a packed-u16 prefix max fills each run from its key.
// Every token start writes its key at its decoded position.  Every other owned position (the
// second byte and the count digit of a 3-byte token) writes its byte, unflagged, at the position
// before the running offset (its token's last decoded position, which holds no key: the tiled
// path declines count digit '1'), so no position needs a trash slot or a select.  A token decodes
// to at most 9 bytes, so every 16-byte chunk holds a key, and the byte entering a chunk is the
// last key of the chunk before it.
#ifndef RLE_DEC_CHUNKS   // staging chunks per wave; fewer: more waves per SIMD, tiles staged in passes
#define RLE_DEC_CHUNKS 192
#endif
constexpr u32 kDecChunks = RLE_DEC_CHUNKS;   // >= ceil((16 + 15 + 3024 + 1) / 16): a tile decodes to <= 3024 B
constexpr u32 kDecStage = 32u * kDecChunks;  // bytes per wave
constexpr bool kDecOnePass = kDecChunks >= 191u;   // a whole tile's output always fits
constexpr u32 kDecPassCap = 16u * kDecChunks - 17u;   // staged positions rel + pass may reach (rel < 16)
static_assert(kDecChunks >= 16u, "a pass must hold at least one lane's output (144 B) past rel < 16");
constexpr u32 kKeyFlag = 0x8000u;

struct DecState {
    u32 out_pos;   // decoded bytes produced so far
    u32 flushed;   // decoded bytes already stored (multiple of 16); staging chunk 1 = flushed
    u32 d;         // offset of the first token start in the current tile (0..2)
    u32 fillc;     // byte of the last stored position (run continuation carry)
    u32 tail;      // 0x100|byte when the stream ends in an unbounded-count token, else 0
    u32 head;      // leading bytes of the first stored chunk that belong to the previous segment
    u32 prev;      // stream byte before the current tile, in bits 24..31
    bool wt;       // write-through output stores (vstore)
    Stamps sp;     // diagnostic builds only
    u32 vrun = 0;       // 0x100 | v while the staged partial chunk is all v and staging
                        // chunk 1 holds exactly one key, kv at position 0 (after a single-value tile)
    bool sv = false;    // the last tile was single-value (dec_fill_run): the next tries the uniform test
};

// Staging address of a position's key.  Unswizzled, a random-data tile decodes 16 positions (32 B
// of keys) per lane, so the lanes of one scatter write sit 32 B apart and 8 of every 32-lane group
// share a bank; two XOR swizzles of the chunks over a 128-B row (dword-wise, 16-B-slot-wise) cut the
// conflicts but measured slower (runs50 +8 %, runs90 +5 %, r5p), so the staging is
// addressed linearly.  Every staging access still goes through sswz.
__device__ __forceinline__ u32 sswz(u32 t) { return t; }
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

// One 32-byte staging chunk (16 u16 keys) at s4.
__device__ __forceinline__ void dec_read_chunk(const u32x4* s4, u32x4& a, u32x4& b) {
    a = s4[0];
    b = s4[1];
}

// The flush's fill of one 32-byte staging chunk (16 u16 keys a, b): the position index p goes into
// bits 8..11 of each key (empty slots get the index alone, below every key and below the carry),
// and a packed-u16 prefix max inside the chunk carries each flagged key over the run it starts.
__device__ __forceinline__ void dec_fill_scan(u32x4 a, u32x4 b, u32 (&L)[8]) {
    L[0] = a.x | 0x01000000u; L[1] = a.y | 0x03000200u; L[2] = a.z | 0x05000400u; L[3] = a.w | 0x07000600u;
    L[4] = b.x | 0x09000800u; L[5] = b.y | 0x0B000A00u; L[6] = b.z | 0x0D000C00u; L[7] = b.w | 0x0F000E00u;
    // 15 op_sel max instructions (round 3; round 2's form took 23 with v_perm): prefix max inside
    // each dword (position 2m+1 takes 2m), then along the chunk: dword m takes the high half
    // (position 2m-1, the prefix so far) of dword m-1 in both halves
    if (!(RLE_ABL & 4)) {
#pragma unroll
        for (u32 m = 0; m < 8; ++m) L[m] = pkmax_lo2hi(L[m]);
#pragma unroll
        for (u32 m = 1; m < 8; ++m) L[m] = pkmax_bhi(L[m], L[m - 1]);
    }
}
// The chunk's 16 output bytes: each position's latest key at or before it, else the byte `carry`
// entering the chunk (a run entering a chunk covers at most its first 8 positions, dwords 0..3).
__device__ __forceinline__ u32x4 dec_fill_out_rep(const u32 (&L)[8], u32 crep);
__device__ __forceinline__ u32x4 dec_fill_out(const u32 (&L)[8], u32 carry) {
    return dec_fill_out_rep(L, carry | 0x10001000u | (carry << 16));
}
// The carry as 0x10vv in both u16 halves (below every key, above every empty slot).
__device__ __forceinline__ u32x4 dec_fill_out_rep(const u32 (&L)[8], u32 crep) {
    u32x4 o;
    o.x = __builtin_amdgcn_perm(pkmax(L[1], crep), pkmax(L[0], crep), 0x06040200u);
    o.y = __builtin_amdgcn_perm(pkmax(L[3], crep), pkmax(L[2], crep), 0x06040200u);
    o.z = __builtin_amdgcn_perm(L[5], L[4], 0x06040200u);
    o.w = __builtin_amdgcn_perm(L[7], L[6], 0x06040200u);
    return o;
}

// Store staged chunks 1..nfl (outputs [flushed, flushed + 16 nfl)) and re-zero them.
__device__ __forceinline__ u32 dec_flush(bool wt, u32 nfl, u32 lane, uint8_t* stage, u32x4 rso, u32 flushed, u32& fillc,
                                         u32& head, uint8_t* dst, Stamps& sp) {
    const u32 rounds = (nfl + kWave - 1u) / kWave;
    // the carry's fill halves (0x10 above the byte) in a VGPR, so the v_perm's selector can be the
    // one constant-bus operand (no per-round v_mov)
    const u32 k10 = rounds ? vconst(0x10101010u) : 0u;
    // the re-zeroing stores take a zero tuple held in VGPRs over the loop
    const u32x4 Z = rounds ? u32x4{vconst(0u), vconst(0u), vconst(0u), vconst(0u)} : u32x4{0u, 0u, 0u, 0u};
    for (u32 k = 0; k < rounds; ++k) {
        const u32 c = k * kWave + lane;
        const bool active = c < nfl;
        u32x4* s4 = reinterpret_cast<u32x4*>(stage + 32u * (c + 1u));
        // read unconditionally: an inactive lane's chunk is garbage it never stores.  With the
        // one-pass staging (192 chunks) it lies at most one chunk past this wave's staging; with
        // RLE_DEC_CHUNKS < 191 it can lie up to 64 * rounds - nfl chunks past it, in another wave's
        // staging or past the workgroup's LDS.  LDS reads do not fault (out-of-range reads return
        // 0), and from_prev_lane below hands the lane's value only to lanes that are inactive too
        // (a lane's carry comes from the lane before it, and the active lanes are 0..nfl-1), so no
        // stored byte depends on it.
        u32x4 a, b;
        dec_read_chunk(s4, a, b);
        RLE_STAMP(sp, 3);   // flush: staging reads
        u32 L[8];
        dec_fill_scan(a, b, L);
        // byte of the chunk's last key = its last output byte: bits 16..23 of L[7]; the carry moves
        // as the chunk's whole last dword, spread by one v_perm
        const u32 lastb = L[7];
        const u32 prev = from_prev_lane(L[7], fillc << 16);
        const u32x4 o = dec_fill_out_rep(L, __builtin_amdgcn_perm(prev, k10, 0x00060006u));
        RLE_STAMP(sp, 4);   // flush: fill + carry
        const bool skip = head && c == 0u;   // shared with the previous segment: byte stores below
        vstore(rso, (active && !skip && !(RLE_ABL & 64)) ? flushed + 16u * c : kOOB, o, wt);   // (RLE_ABL 64: diagnostic)
        if (skip && active) {
            const u32 wv[4] = {o.x, o.y, o.z, o.w};
            for (u32 j = head; j < 16u; ++j) dst[flushed + j] = (uint8_t)(wv[j >> 2] >> (8u * (j & 3u)));
        }
        head = 0;
        RLE_STAMP(sp, 5);   // flush: store issue
        if (active) {
            s4[0] = Z;
            s4[1] = Z;
        }
        const u32 lastlane = (nfl - 1u - k * kWave) < (kWave - 1u) ? (nfl - 1u - k * kWave) : (kWave - 1u);
        fillc = (readlane(lastb, lastlane) >> 16) & 0xFFu;
        wave_lds_sync();
        RLE_STAMP(sp, 6);   // flush: re-zero + sync
    }
    return rounds;
}

// Decode tile analysis (shared by dec_tile and the segment summary).  dec_prepare: the tile's
// bytes (zero past C), the per-byte "differs from the next byte" flags g (0x80 per byte: a token
// starting there is 1 byte long), their bit masks, and the wave scan of the lanes' token-phase
// maps.  Positions are absolute in the stream; tokens start only below Co (the end of the
// positions this wave owns: the stream, or its segment).  Lane 63 holds only the next tile's first
// 16 bytes (lookahead): its results are garbage and every consumer ignores it.
// Register constants of the decode tile, made once per kernel (vconst: no rematerialisation
// inside the tile loop).
struct DecK {
    u32 K80, K7F, C1, C2;
    u32 LM3;   // lane % 3 (dec_uniform_tile)
};
__device__ __forceinline__ DecK dec_k() {
    const u32 lane = threadIdx.x & (kWave - 1u);
    return DecK{vconst(0x80808080u), vconst(0x7F7F7F7Fu), vconst(0x08040201u), vconst(0x80402010u),
                lane - 3u * ((lane * 0xABu) >> 9)};
}
struct DecPrep {
    u32 w[4], g[4];
    u32 K80;
    u32 la;        // next lane's first 4 bytes (count digits of positions 14, 15)
    u32 left;      // stream bytes from the lane's first position
    u32 lefto;     // owned positions from the lane's first position
    u32 xa, xb;    // NE bits of positions 0..7 / 8..15, at bits 7..14
    u32 incl, excl;
    DecEntry ta, tb;
    bool tail;     // the tile reaches the owned end or the stream end (validity masks needed)
};
__device__ __forceinline__ DecPrep dec_prepare(const u32x4 cur, u32 pos, u32 C, u32 Co, u32 lane,
                                               const DecEntry* tbl, const DecK& kc) {
    DecPrep r;
    r.K80 = kc.K80;
    const u32 p0 = pos + 16u * lane;
    r.left = p0 < C ? C - p0 : 0u;
    r.lefto = p0 < Co ? Co - p0 : 0u;
    r.tail = pos + kSlot + 2u > Co;   // (Co <= C) positions >= Co or digits past C occur only here
    u32* w = r.w;
    w[0] = cur.x; w[1] = cur.y; w[2] = cur.z; w[3] = cur.w;
    if (pos + kSlot > C) {   // last tiles: bytes at index >= C read as the stream's zero padding
        const u32 nl = r.left < 16u ? r.left : 16u;
#pragma unroll
        for (u32 k = 0; k < 4; ++k) {
            const u32 nb = nl > 4u * k ? (nl - 4u * k < 4u ? nl - 4u * k : 4u) : 0u;
            w[k] &= lowmask(8u * nb);
        }
    }
    const u32 la = from_next_lane(w[0], 0u);
    r.la = la;
    const u32 K80 = kc.K80;
    const u32 nx[4] = {alignbyte(w[1], w[0], 1), alignbyte(w[2], w[1], 1), alignbyte(w[3], w[2], 1),
                       alignbyte(la, w[3], 1)};
    const u32 K7F = kc.K7F;   // in a VGPR: v_bitop3 with an SGPR operand is slow-class
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 t = w[k] ^ nx[k];
        const u32 u = faddi<0x7F7F7F7Fu>(t & K7F);
        r.g[k] = bitop3<kOrAnd>(u, t, K80);
    }
    const u32 C1 = kc.C1, C2 = kc.C2;
    r.xa = __builtin_amdgcn_udot4(r.g[1], C2, __builtin_amdgcn_udot4(r.g[0], C1, 0u, false), false);
    r.xb = __builtin_amdgcn_udot4(r.g[3], C2, __builtin_amdgcn_udot4(r.g[2], C1, 0u, false), false);
    const u32 tbase = lds_addr(tbl);
    r.ta = lds_entry(tbase + (r.xa >> 4));
    r.tb = lds_entry(tbase + (r.xb >> 4));
    const u32 map = __builtin_amdgcn_perm(r.tb.y, r.tb.y, r.ta.y);
    // The scan composes the lanes' maps.  Where every owned lane's map is constant (its three entry
    // phases reach one common token start inside the lane: nearly every lane of random, text-like
    // and run-heavy streams, since a byte that differs from the two before it always starts a
    // token), the composition up to lane l is lane l's own map, and the scan is skipped (the same
    // values on lanes 0..62; lane 63's incl, which no consumer reads, is then its own map).  Streams
    // whose lanes keep the phase open (a run of one digit-like byte) take the scan.  As the encode
    // tile's run-start scan (enc_analyze_bounds).
    constexpr uint64_t kOwnedLanes = (1ull << kOwnLanes) - 1ull;
    if (RLE_ABL & 1) r.incl = map;
    else if (!(__builtin_amdgcn_ballot_w64(map != __builtin_amdgcn_perm(map, map, 0x03000000u)) & kOwnedLanes))
        r.incl = map;
    else r.incl = wave_scan_incl(map, kMapId, OpMap());
    r.excl = from_prev_lane(r.incl, kMapId);
    return r;
}
// dec_lengths: for tile-entry phase d, the token-start bytes S01 (1 per start), the decoded length
// per position W (bytes), the lane's decoded byte count and whether the tiled path must decline
// (a count digit outside '1'..'9'); tail tiles also mask positions past the owned range and
// report PF (bits): pair starts whose count digit lies in the zero padding (the stream's final,
// unbounded token).
struct DecLen {
    u32 W[4], S01[4], S80[4], N02[4];   // N02: 2 at owned positions that are not token starts
    u32 nout, PF;
    bool serial_lane;
};
// 16-bit mask -> 0x80 per byte for the 4 positions of dword k ((nibble << 7) * 0x00204081 puts
// bit i at bit 8 i + 7)
__device__ __forceinline__ u32 expand80(u32 m16, u32 k, u32 K80) {
    return __umul24(bfe(m16, 4u * k, 4) << 7, 0x00204081u) & K80;
}
// kTail: the tile reaches the owned end or the stream end (p.tail); instantiated separately so the
// common tiles use the masks' constant values directly.
template <bool kTail>
__device__ __forceinline__ DecLen dec_lengths_t(const DecPrep& p, u32 d) {
    DecLen r;
    const u32* w = p.w;
    const u32 dl = bfe(p.excl, 8u * d, 8);                                    // lane entry phase
    const u32 mid = __builtin_amdgcn_perm(0u, p.ta.y, 0x0C0C0C00u | dl);      // phase entering position 8
    const u32 sa = __builtin_amdgcn_perm(0u, p.ta.x, 0x0C0C0C00u | dl);       // start bits 0..7
    const u32 sb = __builtin_amdgcn_perm(0u, p.tb.x, 0x0C0C0C00u | mid);      // start bits 8..15
    const u32 K80 = p.K80;
    const u32 sa7 = sa << 7, sb7 = sb << 7;
    u32 S80[4] = {__umul24(sa7 & 0x780u, 0x00204081u) & K80,
                  __umul24((sa7 >> 4) & 0x780u, 0x00204081u) & K80,
                  __umul24(sb7 & 0x780u, 0x00204081u) & K80,
                  __umul24((sb7 >> 4) & 0x780u, 0x00204081u) & K80};
    const u32 dg[4] = {alignbyte(w[1], w[0], 2), alignbyte(w[2], w[1], 2), alignbyte(w[3], w[2], 2),
                       alignbyte(p.la, w[3], 2)};
    u32 VD80[4] = {K80, K80, K80, K80};   // positions whose count digit lies inside the stream
    u32 O02[4] = {0x02020202u, 0x02020202u, 0x02020202u, 0x02020202u};   // 2 at owned positions
    r.PF = 0u;
    bool sf = false;
    if (kTail) {
        // owned: j < lefto; digit inside the stream: j + 2 < left; second byte inside: j + 1 < left
        const u32 lo16 = lowmask(p.lefto < 16u ? p.lefto : 16u);
        const u32 l18 = lowmask(p.left < 18u ? p.left : 18u);
        const u32 S16 = (sa | (sb << 8)) & lo16;
        const u32 NE16 = (p.xa >> 7) | (p.xb << 1);
        r.PF = S16 & ~NE16 & ~(l18 >> 2) & 0xFFFFu;   // pair starts whose digit is past C
        sf = (r.PF & (l18 >> 1)) != 0u;                // ... while the second byte is not: decline
#pragma unroll
        for (u32 k = 0; k < 4; ++k) {
            const u32 vo = expand80(lo16, k, K80);
            S80[k] &= vo;
            O02[k] = vo >> 6;
            VD80[k] = expand80(l18 >> 2, k, K80);
        }
    }
    u32 bad = 0u, sum = 0u;
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 P80 = bitop3<0xF0 & ~0xCC & 0xAA>(S80[k], p.g[k], VD80[k]);   // 3-byte start, digit in stream
        const u32 P7F = fsub(P80, fshr<7>(P80));
        const u32 xm = fandi<0x7F7F7F7Fu>(dg[k]);
        const u32 a = faddi<0x46464646u>(xm);   // bit 7: digit >= ':'
        const u32 b2 = faddi<0x4E4E4E4Eu>(xm);  // bit 7: digit >= '2'
        const u32 b = faddi<0x4F4F4F4Fu>(xm);   // low 7 bits: digit - '1'
        if (!(RLE_ABL & 16)) bad = bitop3<kAndOr>(bitop3<kBad>(a, b2, dg[k]), P80, bad);
        const u32 S01 = fshr<7>(S80[k]);
        r.S80[k] = S80[k];
        r.S01[k] = S01;
        // (only dword 3 needs it: interior positions of dwords 0..2 write at the next token's slot,
        // dec_scatter)
        r.N02[k] = k < 3u ? 0u : fsub(O02[k], fshr<6>(S80[k]));
        r.W[k] = fadd(S01, b & P7F);
        sum = fadd(sum, r.W[k]);
    }
    sum = fadd(sum, fshr<16>(sum));
    sum = fadd(sum, fshr<8>(sum));
    r.nout = fandi<0xFFu>(sum);
    r.serial_lane = (bad & K80) != 0u || sf;
    return r;
}
__device__ __forceinline__ DecLen dec_lengths(const DecPrep& p, u32 d) {
    return p.tail ? dec_lengths_t<true>(p, d) : dec_lengths_t<false>(p, d);
}

// The scatter of one lane's decoded positions into the staging (2 bytes per position): endk = the
// staging byte address of the lane's first decoded position.  u16 per position: the byte, with
// the start flag (0x80) as the high byte: 0x80vv at a token start, an unflagged 0x00vv (ignored by
// the fill) anywhere else.  Where an interior position (a 3-byte token's second byte or count digit)
// writes its unflagged key (round 4): positions 0..13 at the slot right after their
// own token's output, which is the next token's start slot: that token starts in the same lane (a
// token spans at most 3 positions), whose later write of the flagged key (program order) replaces
// it; positions 14 and 15, whose next token may start in the next lane (written by an earlier
// instruction there), keep round 3's rule: one slot back, their own token's last decoded position,
// which never holds a key (counts are >= 2 on this path).  Saves the N02 / R arithmetic of three of
// the four dwords.  (Measured and not kept: exec-masking the interior writes off, so that only
// token starts write, cut the bank conflicts by a third but cost 11-14 % more VALU and ran 10-12 %
// slower, r5ad; storing the odd positions from the high halves with ds_write_b16_d16_hi was
// neutral, r3j: DESIGN.md §4.)
__device__ __forceinline__ void dec_scatter(const DecLen& ln, const u32* w, u32 endk) {
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 xk_lo = __builtin_amdgcn_perm(ln.S80[k], w[k], 0x05010400u);
        const u32 xk_hi = __builtin_amdgcn_perm(ln.S80[k], w[k], 0x07030602u);
        u32 Q = fadd(ln.W[k], fshr<8>(ln.W[k]));
        Q = fadd(Q, fshr<16>(Q));                        // byte i: decoded bytes of positions >= i
        Q = Q << 1;                                      // 2 staging bytes per position
        endk = fadd(endk, fandi<0xFFu>(Q));              // staging address after the dword's output
        const u32 R = fadd(Q, ln.N02[k]);                // interior positions: one slot further back
        auto put = [](u32 t, u32 key) {
            if (RLE_ABL & 8) asm volatile("" ::"v"(t), "v"(key));   // ablation: no LDS write
            else *reinterpret_cast<__attribute__((address_space(3))) uint16_t*>(sswz(t)) = (uint16_t)key;
        };
        put(sub_byte<0>(endk, R), xk_lo);
        put(sub_byte<1>(endk, R), xk_lo >> 16);
        put(sub_byte<2>(endk, R), xk_hi);
        put(sub_byte<3>(endk, R), xk_hi >> 16);
    }
}

// ---------------------------------------------------------------- literal tiles (the fast path)
// A tile whose tokens are all 1-byte literals or 3-byte pairs "vv2" decodes to its own bytes with
// the count digits deleted: position j is kept unless it is a pair's digit, or lies before the
// tile's first token start (the previous tile's token, decoded there).  A pair started at the
// tile's last owned position keeps its second byte, lane 63's position 0 (the lookahead), so each
// tile's output is still exactly the tokens that start in it.  When every owned lane loses at most
// 2 positions, lane l's output is its 16 bytes with <= 2 removed (one LUT-selected v_perm per
// dword), stored with one 16-byte store at its output offset, which need not be aligned: the
// lane's 14..16 bytes are followed by the next lane's first bytes, so the bytes two lanes store
// twice are equal.  The last lane's store reaches <= 16 bytes past the tile's output; the next
// tile's (or the finish's) stores, issued later by the same wave, overwrite them.  No staging, no
// scatter, no fill: random and text-like data decode with about half the VALU work.
// Compaction selectors: entry t (a deleted position, 16 = none), dword q: the v_perm selector
// taking output bytes 4q..4q+3 from (y[q+1]:y[q]) once position t is removed.  A lane's two
// deletions are two passes, the higher position first.  17 entries of 16 bytes: every wave
// LDS-DMAs them (with the phase table) into the workgroup's copy ahead of its first tile.
constexpr u32 kCompactEntries = 17u;
struct DecCompactLut {
    u32 s[kCompactEntries * 4u];
};
constexpr DecCompactLut make_compact_lut() {
    DecCompactLut t{};
    for (u32 d = 0; d <= 16u; ++d)
        for (u32 q = 0; q < 4u; ++q) {
            u32 sel = 0;
            for (u32 b = 0; b < 4u; ++b) {
                const u32 m = 4u * q + b;
                sel |= (m + (m >= d ? 1u : 0u) - 4u * q) << (8u * b);   // 0..4
            }
            t.s[d * 4u + q] = sel;
        }
    return t;
}
static __constant__ DecCompactLut kCompactLut = make_compact_lut();

// Returns the store instructions issued, or kNotFast (nothing done: the general path decodes the
// tile).  A segment's first tile only when nothing is staged yet; a segment's last tile (kTail,
// Co < C on a tile edge) with its stores clipped at its output end (dec_tile_pr).
// kTail (pr.tail): positions past C are neither starts nor kept, a pair whose digit lies past C
// (the stream's final unbounded token) declines, and since the range check drops a store's dwords
// that are not wholly below U (tools/probes/range_clip_probe.hip), the tile's last 4 output bytes
// are stored again as one dword ending at its output end.
template <bool kTail>
__device__ __forceinline__ u32 dec_tile_fast(const DecPrep& pr, u32 lane, const u32x4* clut, uint8_t* stage,
                                             u32x4 rso, u32 U, DecState& st, const DecK& kc) {
    constexpr uint64_t kOwned = (1ull << kOwnLanes) - 1ull;
    const u32* w = pr.w;
    // positions below the owned end (the stream's end C, or a segment's end on a tile edge)
    const u32 lim = kTail ? lowmask(pr.lefto < 16u ? pr.lefto : 16u) : 0xFFFFu;
    const u32 NE16 = (pr.xa >> 7) | (pr.xb << 1);
    // cheap reject first (runs): at most 2 equal neighbours per owned lane
    if (__builtin_amdgcn_ballot_w64(__builtin_popcount(~NE16 & lim) > 2) & kOwned) return kNotFast;
    const u32 dl = bfe(pr.excl, 8u * st.d, 8);
    const u32 mid = __builtin_amdgcn_perm(0u, pr.ta.y, 0x0C0C0C00u | dl);
    const u32 sa = __builtin_amdgcn_perm(0u, pr.ta.x, 0x0C0C0C00u | dl);
    const u32 sb = __builtin_amdgcn_perm(0u, pr.tb.x, 0x0C0C0C00u | mid);
    const u32 P16 = (sa | (sb << 8)) & ~NE16 & lim;   // pair starts (bits 0..15)
    // deleted positions: digits of pairs started in this lane or (bits 14, 15) the lane before, and
    // in lane 0 the tile's first d positions; lane 63 keeps only a pair's second byte at position 0
    const u32 prevP = from_prev_lane(P16, 0u);
    const u32 dig = ((P16 << 2) | (prevP >> 14)) & lim;   // the digits
    const u32 del = lane == 0u ? dig | (lowmask(st.d) & lim) : dig;
    // every pair's count digit is '2': the digits are exactly the deleted positions other than lane
    // 0's first d (the previous tile's token, checked there) -- on lane 63 only those of lane 62's
    // pairs.  At most 2 per lane pass the limit below, so only those bytes are read (one v_perm pair
    // each), not a '2' test of every position (round 3).
    const u32 chk = lane < kOwnLanes ? dig : ((prevP >> 14) & 3u);
    const u32 c1 = (u32)__builtin_ctz(chk | 0x10000u), c2 = (u32)__builtin_ctz((chk & (chk - 1u)) | 0x10000u);
    auto byte_at = [&](u32 q) {   // byte q (0..15) of the lane's 16 bytes, in bits 0..7
        const u32 lo = __builtin_amdgcn_perm(w[1], w[0], q & 7u), hi = __builtin_amdgcn_perm(w[3], w[2], q & 7u);
        return (q & 8u) ? hi : lo;
    };
    const bool bad1 = c1 < 16u && (byte_at(c1) & 0xFFu) != 0x32u;
    const bool bad2 = c2 < 16u && (byte_at(c2) & 0xFFu) != 0x32u;
    // (lane 63's own pairs belong to the next tile: only its digit test counts, so the ballot below
    // takes every lane)
    bool reject = bad1 || bad2 || (lane < kOwnLanes && __builtin_popcount(del) > 2);
    if (kTail) reject = reject || (lane < kOwnLanes && (P16 & ~(lowmask(pr.left < 18u ? pr.left : 18u) >> 2)) != 0u);
    const u32 K = lane < kOwnLanes ? (~del & lim) : ((prevP >> 15) & 1u);
    const u32 kept = (u32)__builtin_popcount(K);
    // Output offsets.  A whole tile's owned lanes keep 16 - d bytes, d = their deletions (<= 2, else
    // the tile is rejected below), and lane 63 keeps 0 or 1: so the exclusive offset of lane l is
    // 16 l less the deletions of the lanes before it, two ballots counted with v_mbcnt, and the
    // tile's total comes from the same ballots on the scalar unit -- no DPP scan on the tile's
    // dependent chain (round 5).  Tail tiles (owned lanes cut short) take the scan.
    u32 oexcl, ttot;
    if (!kTail) {
        const u32 d = lane < kOwnLanes ? (u32)__builtin_popcount(del) : 0u;
        const uint64_t B1 = __builtin_amdgcn_ballot_w64(d >= 1u), B2 = __builtin_amdgcn_ballot_w64(d >= 2u);
        const uint64_t B3 = __builtin_amdgcn_ballot_w64(lane == kWave - 1u && kept != 0u);
        const u32 before = __builtin_amdgcn_mbcnt_hi((u32)(B1 >> 32), __builtin_amdgcn_mbcnt_lo((u32)B1, 0u)) +
                           __builtin_amdgcn_mbcnt_hi((u32)(B2 >> 32), __builtin_amdgcn_mbcnt_lo((u32)B2, 0u));
        oexcl = 16u * lane - before;
        ttot = 16u * kOwnLanes - (u32)__builtin_popcountll(B1) - (u32)__builtin_popcountll(B2) + (u32)(B3 >> 63);
    } else {
        const u32 oincl = wave_scan_incl(kept, 0u, OpAdd());
        ttot = readlane(oincl, kWave - 1u);
        oexcl = oincl - kept;
    }
    if (__builtin_amdgcn_ballot_w64(reject)) return kNotFast;
    if (kTail ? (ttot < 4u || st.out_pos + ttot > U) : st.out_pos + ttot + 16u > U) return kNotFast;
    if (kTail) {
        rso.z = uniform(st.out_pos + ttot);   // clip every store of this tile at its output end
        asm volatile("s_nop 4" ::: "memory");   // (the descriptor word is fresh)
    }

    u32 rounds = 0;
    const u32 rel0 = st.out_pos - st.flushed;
    if (rel0 && !st.head) {   // a general tile's partial chunk: store it (its bytes past rel0 are rewritten below)
        u32x4 a, b;
        dec_read_chunk(reinterpret_cast<const u32x4*>(stage + 32u), a, b);
        u32 L[8];
        dec_fill_scan(a, b, L);
        vstore(rso, lane == 0u ? st.flushed : kOOB, dec_fill_out(L, st.fillc), st.wt);
        wave_lds_sync();
        if (lane < 8u)
            *reinterpret_cast<__attribute__((address_space(3))) u32*>(sswz(lds_addr(stage) + 32u + 4u * lane)) = 0u;
        wave_lds_sync();
        rounds = 1;
    }
    const u32 dm = lane < kOwnLanes ? del : 0u;
    const u32 t1 = (u32)__builtin_ctz(dm | 0x10000u);
    const u32 t2 = (u32)__builtin_ctz((dm & (dm - 1u)) | 0x10000u);
    // remove t2 (if any lane has a second deletion), then t1
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
    // bytes kept..15 of the store: the next lane's first bytes (kept >= 14 on full owned lanes;
    // fewer only where the output ends)
    const u32 n0 = from_next_lane(o.x, 0u);
    const u32 s3 = kept >= 16u ? 0x03020100u : kept == 15u ? 0x04020100u : 0x05040100u;
    o.w = lane < kOwnLanes ? __builtin_amdgcn_perm(n0, c3, s3) : c3;
    vstore(rso, kept ? st.out_pos + oexcl : kOOB, o, st.wt);
    if (kTail) {
        // the last 4 bytes of each lane's output: from its own bytes, or with fewer than 4 the
        // previous (full) lane's last bytes and its own
        const u32 s = kept - 4u, qd = s >> 2;
        const u32 lo = qd == 0u ? o.x : qd == 1u ? o.y : qd == 2u ? o.z : o.w;
        const u32 hi = qd == 0u ? o.y : qd == 1u ? o.z : o.w;
        const u32 T4 = alignbyte(hi, lo, s & 3u);
        const u32 Tp = from_prev_lane(T4, 0u);
        const u32 T = kept >= 4u ? T4 : alignbyte(o.x, Tp, kept);
        const uint64_t has = __builtin_amdgcn_ballot_w64(kept != 0u);
        const u32 last = 63u - (u32)__builtin_clzll(has);
        vstore4(rso, lane == last ? st.out_pos + ttot - 4u : kOOB, T, st.wt);
        ++rounds;
    }
    st.out_pos += ttot;
    st.flushed = st.out_pos;
    st.head = 0;   // (a segment's first tile: everything from its output offset on is stored)
    st.d = bfe(readlane(pr.incl, kOwnLanes - 1u), 8u * st.d, 8);
    st.prev = readlane(w[3], kOwnLanes - 1u);
    return rounds + 1u;
}

// Single-value tile (dec_tile): ttot copies of v after the staged partial chunk.  The caller sets
// the tile's exit state (st.d, st.prev).  Measured and not kept (r5ar): stores
// shifted onto 128-byte lines, and holding back the chunks past the last line so that no line is
// written in two halves by two tiles: within 0.3 % on dec64k, +2 % on configs[1].
__device__ __forceinline__ u32 dec_fill_run(u32 v, u32 ttot, u32 lane, uint8_t* stage, u32x4 rso, DecState& st) {
    // the previous tile was single-value tile of the same byte that left staging chunk 1 as one key
    // kv at position 0 (st.vrun): the staged positions are all v, so chunk 0 is rep4(v) without
    // reading or filling the staging, and the staging stays as it is when this tile leaves a partial
    // chunk too
    const bool known = st.vrun == (0x100u | v);
    const u32 rel0 = st.out_pos - st.flushed, total = rel0 + ttot, nfl = total >> 4;
    const u32 vv = rep4(v);
    u32 c0[4] = {vv, vv, vv, vv};
    if (!known) {
        // chunk 0: the staged positions [0, rel0) filled like a flush, then v (every lane computes it)
        u32x4 a, b;
        dec_read_chunk(reinterpret_cast<const u32x4*>(stage + 32u), a, b);
        u32 L[8];
        dec_fill_scan(a, b, L);
        const u32x4 f = dec_fill_out(L, st.fillc);
        const u32 fv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
        for (u32 k = 0; k < 4; ++k) {
            const u32 nb = rel0 > 4u * k ? (rel0 - 4u * k < 4u ? rel0 - 4u * k : 4u) : 0u;
            const u32 m = lowmask(8u * nb);
            c0[k] = (fv[k] & m) | (vv & ~m);
        }
    }
    const u32 rounds = (nfl + kWave - 1u) / kWave;
    for (u32 k = 0; k < rounds; ++k) {
        const u32 c = k * kWave + lane;
        const u32x4 o = c == 0u ? u32x4{c0[0], c0[1], c0[2], c0[3]} : u32x4{vv, vv, vv, vv};
        vstore(rso, c < nfl ? st.flushed + 16u * c : kOOB, o, st.wt);
    }
    if (!(known && nfl != 0u && (total & 15u) != 0u)) {
        wave_lds_sync();   // every lane has read staging chunk 1
        // staging chunk 1 = the new partial chunk: the old keys plus a key at rel0 (nothing flushed),
        // else a key at position 0 (when anything is left) and zeros
        const u32 kv = kKeyFlag | v;
        if (lane == 0u) {
            if (nfl == 0u) {
                *reinterpret_cast<__attribute__((address_space(3))) uint16_t*>(sswz(lds_addr(stage) + 32u + 2u * rel0)) = (uint16_t)kv;
            } else {
                const u32 k0 = (total & 15u) ? kv : 0u;
                *reinterpret_cast<lds_u32x4*>(sswz(lds_addr(stage) + 32u)) = u32x4{k0, 0u, 0u, 0u};
                *reinterpret_cast<lds_u32x4*>(sswz(lds_addr(stage) + 48u)) = u32x4{0u, 0u, 0u, 0u};
            }
        }
        wave_lds_sync();
    }
    st.vrun = (nfl != 0u && (total & 15u) != 0u) ? (0x100u | v) : 0u;
    st.sv = true;
    st.fillc = v;
    st.flushed += 16u * nfl;
    st.out_pos += ttot;
    return rounds;
}
__device__ __forceinline__ u32 dec_tile_fill(u32 v, u32 ttot, u32 lane, uint8_t* stage, u32x4 rso, DecState& st,
                                             const DecPrep& pr) {
    const u32 rounds = dec_fill_run(v, ttot, lane, stage, rso, st);
    st.d = bfe(readlane(pr.incl, kOwnLanes - 1u), 8u * st.d, 8);
    st.prev = readlane(pr.w[3], kOwnLanes - 1u);
    return rounds;
}

// ---------------------------------------------------------------- uniform tiles (zero-filled data)
// A whole tile (not the stream's or segment's last) whose owned tokens are all "v v 9" from its
// entry offset d on -- long runs, zero-filled data -- decodes to 336 x 9 = 3024 copies of v and
// leaves the entry offset unchanged (1008 = 3 x 336).  Position p of the tile holds '9' where
// (p - d) mod 3 == 2, else v; with 16 l + 4 k = l + k (mod 3), dword k of lane l follows pattern
// (l + k - d) mod 3.  Tested before the tile analysis (dec_prepare, dec_lengths: about 135 VALU
// of the 266 a zero tile cost, profiles/r4a_sq_kinds.md): lane 0's first 8 bytes on the scalar
// unit, then every owned byte and the lookahead bytes its last token reads (lane 63's first d) on
// the vector unit, so other tiles pay a few scalar instructions.  Byte-identical to the general
// path: the same tokens, each 3 bytes long (its first two bytes are equal) with count 9.
constexpr u32 kUniformOut = 9u * (kTileStep / 3u);   // 3024
__device__ __forceinline__ u32 uniform_pat(u32 m, u32 vv) {
    return m == 0u ? ((vv & 0xFF00FFFFu) | 0x00390000u)
                   : m == 1u ? ((vv & 0xFFFF00FFu) | 0x00003900u) : ((vv & 0x00FFFF00u) | 0x39000039u);
}
// lm3 = lane % 3.  Returns whether the tile is uniform; v = its byte.
__device__ __forceinline__ bool dec_uniform_tile(const u32x4 cur, u32 lane, u32 lm3, u32 d, u32& v) {
    const u32 w0 = readlane(cur.x, 0), w1 = readlane(cur.y, 0);
    v = (w0 >> (8u * d)) & 0xFFu;
    const u32 vv = v * 0x01010101u;
    const u32 ms = d == 0u ? 0u : 3u - d;   // lane 0's dword-0 pattern
    const u32 dm = ~lowmask(8u * d);        // lane 0: positions before d belong to the previous tile
    if (((w0 ^ uniform_pat(ms, vv)) & dm) | (w1 ^ uniform_pat(ms == 2u ? 0u : ms + 1u, vv))) return false;
    const u32 t = lm3 + 3u - d;
    const u32 m0 = t >= 3u ? t - 3u : t;
    const u32 P0 = uniform_pat(0u, vv), P1 = uniform_pat(1u, vv), P2 = uniform_pat(2u, vv);
    const u32 pa = m0 == 0u ? P0 : m0 == 1u ? P1 : P2;
    const u32 pb = m0 == 0u ? P1 : m0 == 1u ? P2 : P0;
    const u32 pc = m0 == 0u ? P2 : m0 == 1u ? P0 : P1;
    // lane 63 (lookahead): only its first d bytes (the last token's second byte and digit)
    const u32 mx = lane == 0u ? dm : lane == kWave - 1u ? ~dm : ~0u;
    const u32 myzw = lane == kWave - 1u ? 0u : ~0u;
    const u32 diff = ((cur.x ^ pa) & mx) | (((cur.y ^ pb) | (cur.z ^ pc) | (cur.w ^ pa)) & myzw);
    return !__builtin_amdgcn_ballot_w64(diff != 0u);
}

// kChunks: the staging's chunks per wave (kDecChunks unless a kernel picks its own).
// One tile from its preparation (dec_prepare): returns the store instructions issued, or ~0u (the
// stream needs the exact serial path).
template <bool kFast = false, u32 kChunks = kDecChunks>
__device__ __forceinline__ u32 dec_tile_pr_body(const DecPrep& pr, u32 pos, u32 C, u32 Co, u32 U, u32 lane,
                                                uint8_t* stage, uint8_t* dst, u32x4 rso, DecState& st, const DecK& kc,
                                                const u32x4* clut);
template <bool kFast = false, u32 kChunks = kDecChunks>
__device__ __forceinline__ u32 dec_tile_pr(const DecPrep& pr, u32 pos, u32 C, u32 Co, u32 U, u32 lane,
                                           uint8_t* stage, uint8_t* dst, u32x4 rso, DecState& st, const DecK& kc,
                                           const u32x4* clut) {
    return dec_tile_pr_body<kFast, kChunks>(pr, pos, C, Co, U, lane, stage, dst, rso, st, kc, clut);
}
template <bool kFast, u32 kChunks>
__device__ __forceinline__ u32 dec_tile_pr_body(const DecPrep& pr, u32 pos, u32 C, u32 Co, u32 U, u32 lane,
                                                uint8_t* stage, uint8_t* dst, u32x4 rso, DecState& st, const DecK& kc,
                                                const u32x4* clut) {
    // Segments (Co < C; rle_segmented.hip) end on tile edges, so their last tile (a tail tile) is a
    // whole tile whose tail form clips its stores at its output end: the next segment's output is
    // another wave's.  A segment's first tile takes the literal path when nothing is staged yet (its
    // stores start at the segment's output offset, never before it).  (Round 2 kept the literal path
    // off a segment's first and last tile.)
    const u32 vrun = st.vrun;   // (the single-value path below keeps it; every other path changes the staging)
    st.vrun = 0u;
    st.sv = false;   // (dec_fill_run sets it again on the single-value path)
    const bool head_ok = !st.head || st.out_pos - st.flushed == st.head;
    // (Skipping the literal test for a few tiles after a failed one, round 4: runs50 -1 %, but
    // configs[1] decode +8 % and 64 KiB random +2 %; not kept.)
    if (kFast && head_ok) {
        const u32 r = pr.tail ? dec_tile_fast<true>(pr, lane, clut, stage, rso, U, st, kc)
                              : dec_tile_fast<false>(pr, lane, clut, stage, rso, U, st, kc);
        if (r != kNotFast) return r;
    }
    const DecLen ln = dec_lengths(pr, st.d);
    const u32* w = pr.w;
    const u32 oincl = wave_scan_incl(ln.nout, 0u, OpAdd());
    const u32 ttot = readlane(oincl, kOwnLanes - 1u);
    constexpr uint64_t kOwned = (1ull << kOwnLanes) - 1ull;
    if ((__builtin_amdgcn_ballot_w64(ln.serial_lane) & kOwned) || st.out_pos + ttot > U) {
        return ~0u;   // the stream needs the exact serial path
    }
    if (pr.tail) {
        const uint64_t pfb = __builtin_amdgcn_ballot_w64(ln.PF != 0u) & kOwned;
        if (pfb) {   // the final token's byte extends to U
            const u32 jf = (u32)__builtin_ctz(ln.PF | 0x10000u) & 15u;
            const u32 wf = jf < 4u ? w[0] : jf < 8u ? w[1] : jf < 12u ? w[2] : w[3];
            st.tail = 0x100u | readlane(bfe(wf, 8u * (jf & 3u), 8), (u32)__builtin_ctzll(pfb));
        }
    }

    // A tile whose tokens all carry one byte v and that expands >= 20/7 = 2.86x its bytes (zero-
    // filled data: "v v 9" tokens) decodes to ttot copies of v: the partial chunk staged so far, filled, then rep4(v)
    // chunks, stored without the scatter and the fill; the new partial chunk is one key.
    if (kFast && !st.head &&
        7u * ttot >= 20u * (C - pos < kTileStep ? C - pos : kTileStep)) {   // (C > pos: the tile exists)
        const u32 v = (readlane(w[0], 0) >> (8u * st.d)) & 0xFFu;   // the tile's first token byte
        const u32 vv = rep4(v);
        u32 bad = 0;
#pragma unroll
        for (u32 k = 0; k < 4; ++k) {
            const u32 t = w[k] ^ vv;
            bad |= bitop3<kOrAnd>(faddi<0x7F7F7F7Fu>(t & kc.K7F), t, kc.K80) & ln.S80[k];
        }
        if (!(__builtin_amdgcn_ballot_w64(bad != 0u) & kOwned)) {
            st.vrun = vrun;
            return dec_tile_fill(v, ttot, lane, stage, rso, st, pr);
        }
    }
    RLE_STAMP(st.sp, 1);   // phase maps, token starts, lengths, offsets
    // With the full staging (kDecChunks >= 191) a tile is one pass.  Smaller staging (more waves per
    // SIMD) stages and flushes a tile in passes over consecutive lanes, each as much as fits: a pass
    // boundary is a lane boundary, so it is a token boundary in the output, exactly like a tile
    // boundary (runs never cross it; interior positions of a token begun in the last pass write
    // one slot back, into a slot that holds no key).
    u32 rounds = 0, done = 0, from = 0;
    for (;;) {
        const u32 rel0 = st.out_pos + done - st.flushed;
        u32 upto = kOwnLanes, pass = ttot - done;
        constexpr bool kOnePass = kChunks >= 191u;
        constexpr u32 kPassCap = 16u * kChunks - 17u;
        static_assert(kChunks >= 16u, "a pass must hold at least one lane's output (144 B) past rel < 16");
        if (!kOnePass && rel0 + pass > kPassCap) {
            // lanes whose output ends within the staging; a prefix, since oincl is monotonic, and it
            // reaches past `from` (a lane decodes at most 144 bytes, rel0 < 16)
            const uint64_t fit = __builtin_amdgcn_ballot_w64(oincl <= done + kPassCap - rel0) & kOwned;
            upto = (u32)__builtin_popcountll(fit);
            pass = readlane(oincl, upto - 1u) - done;
        }
        // staging byte address after this lane's output (2 B per decoded position)
        u32 endk = lds_addr(stage) + 2u * (16u + rel0 + oincl - done - ln.nout);
        if (lane < upto && lane >= from && !(RLE_ABL & 2)) dec_scatter(ln, w, endk);
        wave_lds_sync();
        RLE_STAMP(st.sp, 2);   // scatter

        const u32 newrel = rel0 + pass;
        const u32 nfl = newrel >> 4;
        rounds += dec_flush(st.wt, nfl, lane, stage, rso, st.flushed, st.fillc, st.head, dst, st.sp);
        if (nfl) {   // move the partial chunk to staging chunk 1
            if (lane < 8u) {
                auto* from4 = reinterpret_cast<__attribute__((address_space(3))) u32*>(sswz(lds_addr(stage) + 32u * (nfl + 1u) + 4u * lane));
                auto* to4 = reinterpret_cast<__attribute__((address_space(3))) u32*>(sswz(lds_addr(stage) + 32u + 4u * lane));
                *to4 = *from4;
                *from4 = 0u;
            }
            wave_lds_sync();
        }
        st.flushed += 16u * nfl;
        done += pass;
        from = upto;
        if (upto >= kOwnLanes) break;
    }
    st.out_pos += ttot;
    st.d = bfe(readlane(pr.incl, kOwnLanes - 1u), 8u * st.d, 8);
    st.prev = readlane(w[3], kOwnLanes - 1u);
    RLE_STAMP(st.sp, 7);   // partial-chunk move, state
    return rounds;
}
// kUni: the uniform-tile test first (dec_uniform_tile): the one-wave kernel's walk (r4b same-process
// A/B: 64 KiB zero decode -1.9 %, 4 KiB zero -5 %, configs[1] -1 %), not the segmented write pass
// (r4d: mixed batch +5 %, 1 MiB runs50 +3.8 % with it).
template <bool kFast = false, u32 kChunks = kDecChunks, bool kUni = kFast>
__device__ __forceinline__ u32 dec_tile(const uint8_t* cslot, const Refill& next, u32 pos, u32 C, u32 Co, u32 U,
                                        u32 lane, const DecEntry* tbl, uint8_t* stage, uint8_t* dst, u32x4 rso,
                                        DecState& st, const DecK& kc, const u32x4* clut = nullptr) {
    RLE_STAMP(st.sp, 0);   // DMA wait + loop
    const u32x4 cur = *reinterpret_cast<const u32x4*>(cslot + 16u * lane);
    next();   // the slot is free once read
    // The uniform test only after a single-value tile (st.sv, round 5), so that it stays off the
    // dependent chain of every other kind of tile (it cost configs[1] decode 0.56-0.7 us and the
    // 64 KiB random / run-heavy kinds 2-3 %, profiles/r5b_ab.md, r5c_ab.md), while the long
    // zero-filled or single-byte stretches it is for take it from their second tile on.
    if (kUni && !(RLE_ABL & 32) && st.sv && !st.head &&
        pos + kSlot + 2u <= Co && st.out_pos + kUniformOut <= U) {
        u32 v;
        if (dec_uniform_tile(cur, lane, kc.LM3, st.d, v)) {
            const u32 r = dec_fill_run(v, kUniformOut, lane, stage, rso, st);
            st.prev = readlane(cur.w, kOwnLanes - 1u);   // (st.d unchanged)
            return r;
        }
    }
    const DecPrep pr = dec_prepare(cur, pos, C, Co, lane, tbl, kc);
    return dec_tile_pr<kFast, kChunks>(pr, pos, C, Co, U, lane, stage, dst, rso, st, kc, clut);
}

// ---------------------------------------------------------------- literal analysis, branch-free
// dec_tile_fast<false>'s test and offsets without its stores (the decode in rounds, rle_round.h,
// decides a tile's path before its output offset is known).  (Round 5 also walked two whole literal
// tiles per step with it in the one-round kernel: a lone wave -2 %, configs[1] decode +6 %; not
// kept)
struct DecLit {
    u32 del, kept, oexcl, ttot;
    bool reject;
};
__device__ __forceinline__ DecLit dec_lit_an(const DecPrep& pr, u32 lane, u32 d) {
    const u32* w = pr.w;
    const u32 NE16 = (pr.xa >> 7) | (pr.xb << 1);
    const u32 dl = bfe(pr.excl, 8u * d, 8);
    const u32 mid = __builtin_amdgcn_perm(0u, pr.ta.y, 0x0C0C0C00u | dl);
    const u32 sa = __builtin_amdgcn_perm(0u, pr.ta.x, 0x0C0C0C00u | dl);
    const u32 sb = __builtin_amdgcn_perm(0u, pr.tb.x, 0x0C0C0C00u | mid);
    const u32 P16 = (sa | (sb << 8)) & ~NE16 & 0xFFFFu;   // pair starts
    const u32 prevP = from_prev_lane(P16, 0u);
    const u32 dig = ((P16 << 2) | (prevP >> 14)) & 0xFFFFu;   // the pairs' count digits
    DecLit r;
    r.del = lane == 0u ? dig | lowmask(d) : dig;
    // every deleted digit is '2' (lane 63: those of lane 62's pairs), at most 2 per owned lane
    const u32 chk = lane < kOwnLanes ? dig : ((prevP >> 14) & 3u);
    const u32 c1 = (u32)__builtin_ctz(chk | 0x10000u), c2 = (u32)__builtin_ctz((chk & (chk - 1u)) | 0x10000u);
    auto byte_at = [&](u32 q) {
        const u32 lo = __builtin_amdgcn_perm(w[1], w[0], q & 7u), hi = __builtin_amdgcn_perm(w[3], w[2], q & 7u);
        return (q & 8u) ? hi : lo;
    };
    const bool bad1 = c1 < 16u && (byte_at(c1) & 0xFFu) != 0x32u;
    const bool bad2 = c2 < 16u && (byte_at(c2) & 0xFFu) != 0x32u;
    r.reject = bad1 || bad2 || (lane < kOwnLanes && __builtin_popcount(r.del) > 2);
    const u32 K = lane < kOwnLanes ? (~r.del & 0xFFFFu) : ((prevP >> 15) & 1u);
    r.kept = (u32)__builtin_popcount(K);
    const u32 nd = lane < kOwnLanes ? (u32)__builtin_popcount(r.del) : 0u;
    const uint64_t B1 = __builtin_amdgcn_ballot_w64(nd >= 1u), B2 = __builtin_amdgcn_ballot_w64(nd >= 2u);
    const uint64_t B3 = __builtin_amdgcn_ballot_w64(lane == kWave - 1u && r.kept != 0u);
    r.oexcl = 16u * lane - (__builtin_amdgcn_mbcnt_hi((u32)(B1 >> 32), __builtin_amdgcn_mbcnt_lo((u32)B1, 0u)) +
                            __builtin_amdgcn_mbcnt_hi((u32)(B2 >> 32), __builtin_amdgcn_mbcnt_lo((u32)B2, 0u)));
    r.ttot = 16u * kOwnLanes - (u32)__builtin_popcountll(B1) - (u32)__builtin_popcountll(B2) + (u32)(B3 >> 63);
    return r;
}
// After the last tile: outputs [flushed, end) = the partial chunk still staged (decoded positions
// < out_pos), then zeros or the final unbounded token's byte (end = U for a stream's last segment,
// end = out_pos for the others).  Bytes below flushed + head belong to the previous segment.
__device__ __forceinline__ void dec_finish(const DecState& st, u32 end, u32 lane, uint8_t* stage, u32x4 rso,
                                           uint8_t* dst) {
    const u32 rel = st.out_pos - st.flushed;   // < 16
    const u32 span = end - st.flushed;
    const u32 nq = (span + 15u) >> 4;
    if (nq == 0u) return;   // everything stored (a fast tail tile), nothing staged (rel <= span)
    const u32 tv = rep4(st.tail & 0xFFu);
    // chunk 0: the staged positions [0, rel) filled like a flush (every lane computes it from the
    // same two broadcast reads), the rest the tail byte
    u32x4 a, b;
    dec_read_chunk(reinterpret_cast<const u32x4*>(stage + 32u), a, b);
    u32 L[8];
    dec_fill_scan(a, b, L);
    const u32x4 f = dec_fill_out(L, st.fillc);
    const u32 fv[4] = {f.x, f.y, f.z, f.w};
    u32 c0[4];
#pragma unroll
    for (u32 k = 0; k < 4; ++k) {
        const u32 nb = rel > 4u * k ? (rel - 4u * k < 4u ? rel - 4u * k : 4u) : 0u;
        const u32 m = lowmask(8u * nb);
        c0[k] = (fv[k] & m) | (tv & ~m);
    }
    for (u32 q0 = 0; q0 < nq; q0 += kWave) {
        const u32 q = q0 + lane;
        if (q < nq) {
            u32 ob[4];
#pragma unroll
            for (u32 k = 0; k < 4; ++k) ob[k] = q == 0u ? c0[k] : tv;
            const u32 j0 = q == 0u ? st.head : 0u;
            if (16u * q + 16u <= span && j0 == 0u) {
                u32x4 o;
                o.x = ob[0]; o.y = ob[1]; o.z = ob[2]; o.w = ob[3];
                vstore(rso, st.flushed + 16u * q, o, st.wt);
            } else {
                for (u32 j = j0; j < 16u && 16u * q + j < span; ++j)
                    dst[st.flushed + 16u * q + j] = (uint8_t)(ob[j >> 2] >> (8u * (j & 3u)));
            }
        }
    }
    wave_lds_sync();
    if (lane < 8u)   // staging chunk 1 back to zero
        *reinterpret_cast<__attribute__((address_space(3))) u32*>(sswz(lds_addr(stage) + 32u + 4u * lane)) = 0u;
}

// Status of a stream the tiled path decoded (U = the buffer's decoded size): the info bit SHORT when
// its tokens decode to fewer than U bytes, which encoder output never does.  (An unbounded final
// token reaches the tiled path only as a single 0x00 byte followed by the zero padding, where the
// reference's fill to U writes the zeros its calloc'd block already holds: encoder output can end
// that way, so it is not flagged.)
__device__ __forceinline__ u32 dec_tiled_status(const DecState& st, u32 U) {
    return st.out_pos < U ? RLE_STATUS_SHORT : RLE_STATUS_OK;
}

// Exact serial decode (src/rleCompression.c:47-62 semantics, writes capped at cap) for the
// streams the tiled path declines: counts outside '1'..'9', unbounded counts before the last
// token, or streams that decode to more than U bytes.  One lane; the encoder never emits these.
__device__ u32 dec_serial(const uint8_t* src, u32 C, u32 U, uint64_t cap, uint8_t* dst, u32 lane,
                          uint8_t* stage, u32 stage_bytes = kDecStage) {
    for (u32 k = lane; k < stage_bytes / 16u; k += kWave)
        reinterpret_cast<u32x4*>(stage)[k] = u32x4{0u, 0u, 0u, 0u};
    for (uint64_t c = lane; c * 16u < cap; c += kWave) {
        if (c * 16u + 16u <= cap) *reinterpret_cast<u32x4*>(dst + c * 16u) = u32x4{0u, 0u, 0u, 0u};
        else
            for (uint64_t p = c * 16u; p < cap; ++p) dst[p] = 0;
    }
    vm_drain();
    wave_lds_sync();
    u32 st = RLE_STATUS_SERIAL;
    if (lane == 0) {
        uint64_t o = 0, j = 0;
        while (j < C) {
            if (o >= cap) { st |= RLE_STATUS_OVERFLOW; break; }
            const uint8_t v = src[j];
            dst[o++] = v;
            const uint8_t n1 = (j + 1 < C) ? src[j + 1] : (uint8_t)0;
            if (v == n1) {
                const uint8_t dgt = (j + 2 < C) ? src[j + 2] : (uint8_t)0;
                const int occ = (int)(int8_t)dgt - 48;
                const uint64_t ex = occ < 0 ? ~0ull : (occ >= 2 ? (uint64_t)(occ - 1) : 0ull);
                const uint64_t room = o < U ? U - o : 0;
                const uint64_t kk = ex < room ? ex : room;
                for (uint64_t i = 0; i < kk; ++i) dst[o + i] = v;
                o += kk;
                j += 3;
            } else {
                j += 1;
            }
        }
    }
    vm_drain();
    return readlane(st, 0);
}

}  // namespace rle
