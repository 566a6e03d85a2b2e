// rle_kernels.hip — MI355X (gfx950, CDNA4) RLE block codec kernels.
//
// Device-resident batch forms of the reference codec (samul-1/C-FileStorage-Server-and-Client
// src/rleCompression.c:9-62; grammar restated in SURVEY.md Appendix A):
//   encode: maximal runs cut into 9-byte chunks; a chunk of r bytes of v emits "v" (r == 1)
//           or "v v ('0'+r)" (r >= 2)                          — src/rleCompression.c:13-41
//   decode: token at j emits y[j]; when y[j] == y[j+1] the token is 3 bytes and adds
//           (signed char)y[j+2]-'0'-1 copies, capped at U      — src/rleCompression.c:50-60
//
// Execution model: one wave64 owns one buffer and walks it in 1 KiB tiles,
// 16 bytes per lane (one global_load_dwordx4 per lane, two tiles prefetched ahead).  Run
// boundaries / token starts are found with 16-bit per-lane masks built by SWAR byte compares;
// the sequential state (encode: run phase mod 9; decode: token phase 0..2) and the output
// offsets are carried across lanes with DPP wave scans (row_shr/row_bcast, no LDS round
// trip) and across tiles in scalar registers.  Output bytes are staged in a per-wave LDS
// ring (XOR-swizzled against bank conflicts) and leave as aligned, coalesced 16-byte stores.
// No MFMA: this is an HBM-bound byte scan.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rle_mi355x.h"

namespace rle {

constexpr uint32_t kWave = 64;
constexpr uint32_t kWavesPerBlock = 4;
constexpr uint32_t kBlock = kWave * kWavesPerBlock;
constexpr uint32_t kTile = 1024;      // input bytes per wave step (16 per lane)
constexpr uint32_t kEncRing = 2048;   // encode staging ring, bytes per wave (tile output <= 1.5 KiB + 15)
constexpr uint32_t kDecRing = 4096;   // decode staging ring, positions per wave (tile output <= 3078 + 15)
constexpr uint32_t kMaxBlocks = 8192;

// ---------------------------------------------------------------- cross-lane primitives (DPP)
enum : int {
    kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118,
    kRowBcast15 = 0x142, kRowBcast31 = 0x143, kWaveShl1 = 0x130, kWaveShr1 = 0x138,
};

template <int kCtrl, int kRowMask = 0xf>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, kCtrl, kRowMask, 0xf, false);
}
// value of lane-1 (lane 0 gets `fill`)
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v, uint32_t fill) { return dpp<kWaveShr1>(fill, v); }
// value of lane+1 (lane 63 gets `fill`)
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v, uint32_t fill) { return dpp<kWaveShl1>(fill, v); }

__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint32_t uniform(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// Inclusive wave scan for an associative op(a_earlier, b_later) with identity `id`.
// Must be called with all 64 lanes active.
template <class Op>
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x, uint32_t id, Op op) {
    x = op(dpp<kRowShr1>(id, x), x);
    x = op(dpp<kRowShr2>(id, x), x);
    x = op(dpp<kRowShr4>(id, x), x);
    x = op(dpp<kRowShr8>(id, x), x);
    x = op(dpp<kRowBcast15, 0xa>(id, x), x);
    x = op(dpp<kRowBcast31, 0xc>(id, x), x);
    return x;
}
struct OpAdd {
    __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};
// "latest present value": values are 0 (absent) or 0x100|byte
struct OpLatest {
    __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const { return b ? b : a; }
};
__device__ __forceinline__ uint32_t mod9(uint32_t x) { return x >= 9u ? x - 9u : x; }  // x <= 17
// Encode phase transfer functions: code >= 16 -> constant (code-16); code < 16 -> add code mod 9.
struct OpPhase9 {
    __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const {
        return b >= 16u ? b : (a >= 16u ? 16u + mod9(a - 16u + b) : mod9(a + b));
    }
};
__device__ __forceinline__ uint32_t apply9(uint32_t f, uint32_t q) { return f >= 16u ? f - 16u : mod9(q + f); }
// Decode token-phase maps {0,1,2} -> {0,1,2}, 2 bits per entry; identity = 0b100100.
constexpr uint32_t kMap3Id = 0u | (1u << 2) | (2u << 4);
struct OpMap3 {
    __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const {
        uint32_t r = 0;
#pragma unroll
        for (uint32_t d = 0; d < 3; ++d) {
            const uint32_t x = (a >> (2 * d)) & 3u;
            r |= ((b >> (2 * x)) & 3u) << (2 * d);
        }
        return r;
    }
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- byte SWAR helpers
// bit k (k=0..3) set iff byte k of d is non-zero
__device__ __forceinline__ uint32_t nz4(uint32_t d) {
    const uint32_t t = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
    return ((t >> 7) * 0x10204080u) >> 28;
}
__device__ __forceinline__ uint32_t lowmask(uint32_t nbits) { return nbits >= 32u ? ~0u : ((1u << nbits) - 1u); }
__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[4], uint32_t j) {  // j compile-time after unroll
    return (w[j >> 2] >> (8u * (j & 3u))) & 0xFFu;
}

// LDS ring swizzle: XOR dword-in-32B-group with the 128-B line index (bits 2..4 ^= bits 7..9).
__device__ __forceinline__ uint32_t swz(uint32_t a) { return a ^ (((a >> 7) & 7u) << 2); }

__device__ __forceinline__ void cswap(uint32_t& a, uint32_t& b, bool c) {
    const uint32_t ta = c ? b : a, tb = c ? a : b;
    a = ta; b = tb;
}
// out[k] = in[k ^ m] for 4 dwords
__device__ __forceinline__ uint4 perm4(uint4 v, uint32_t m) {
    cswap(v.x, v.y, m & 1u); cswap(v.z, v.w, m & 1u);
    cswap(v.x, v.z, m & 2u); cswap(v.y, v.w, m & 2u);
    return v;
}

__device__ __forceinline__ uint4 load_chunk(const uint8_t* base, uint64_t len, uint64_t off) {
    if (off < len) return *reinterpret_cast<const uint4*>(base + off);
    return make_uint4(0u, 0u, 0u, 0u);
}

// ================================================================ ENCODE
struct EncState {
    uint64_t out_pos;   // compressed bytes produced so far
    uint64_t flushed;   // compressed bytes already stored to HBM (multiple of 16)
    uint32_t prev_byte; // input byte at tile_pos-1
    uint32_t q;         // run phase ((i - runstart) mod 9) of input byte tile_pos-1
};

__device__ __forceinline__ void enc_tile(const uint4 cur, const uint4 nxt, uint64_t pos, uint64_t U,
                                         uint32_t lane, uint8_t* ring, uint8_t* dst, EncState& st) {
    const uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
    const uint64_t p0 = pos + 16u * lane;
    const uint32_t nl = p0 >= U ? 0u : (uint32_t)((U - p0) < 16u ? (U - p0) : 16u);
    const uint32_t validm = lowmask(nl);

    // run boundaries: bit j <=> x[p0+j] != x[p0+j-1] (or p0+j == 0); virtual boundaries past U
    const uint32_t last = w[3] >> 24;
    const uint32_t prevb = from_prev_lane(last, st.prev_byte);
    uint32_t B = nz4(w[0] ^ ((w[0] << 8) | prevb)) | (nz4(w[1] ^ ((w[1] << 8) | (w[0] >> 24))) << 4) |
                 (nz4(w[2] ^ ((w[2] << 8) | (w[1] >> 24))) << 8) | (nz4(w[3] ^ ((w[3] << 8) | (w[2] >> 24))) << 12);
    if (p0 == 0) B |= 1u;
    B |= ~validm & 0xFFFFu;

    // 8-byte lookahead (for the repeat count): next lane's boundaries; lane 63 reads the next tile
    const uint32_t nx0 = readlane(nxt.x, 0), nx1 = readlane(nxt.y, 0), last63 = readlane(last, 63);
    const uint64_t pn = pos + kTile;
    const uint32_t nvn = pn >= U ? 0u : (uint32_t)((U - pn) < 8u ? (U - pn) : 8u);
    const uint32_t B8 = (nz4(nx0 ^ ((nx0 << 8) | last63)) | (nz4(nx1 ^ ((nx1 << 8) | (nx0 >> 24))) << 4) |
                         (~lowmask(nvn))) & 0xFFu;
    const uint32_t B24 = B | ((from_next_lane(B, B8) & 0xFFu) << 16);

    // run phase carried across lanes: lane function q_in -> q_out
    const uint32_t fcode = B ? 16u + mod9(15u - (31u - (uint32_t)__builtin_clz(B))) : 7u;  // (q+16)%9 == (q+7)%9
    const uint32_t incl = wave_scan_incl(fcode, 0u, OpPhase9());
    const uint32_t excl = from_prev_lane(incl, 0u);
    const uint32_t qin = apply9(excl, st.q);

    // token starts: run starts, run start + 9, and the continuation of the run entering the lane
    const uint32_t f1 = B ? (uint32_t)__builtin_ctz(B) : 16u;
    uint32_t t8 = B | (B << 1);
    t8 |= t8 << 2;
    t8 |= t8 << 4;
    t8 |= B << 8;
    const uint32_t j0 = 8u - qin;
    const uint32_t pre = ((1u << j0) | (1u << (j0 + 9u))) & lowmask(f1);
    const uint32_t T = (B | ((B << 9) & ~t8) | pre) & validm;
    const uint32_t P = T & ~(B24 >> 1);  // 3-byte tokens (run continues past the start)

    const uint32_t nout = (uint32_t)__builtin_popcount(T) + 2u * (uint32_t)__builtin_popcount(P);
    const uint32_t oincl = wave_scan_incl(nout, 0u, OpAdd());
    const uint32_t ttot = readlane(oincl, 63);
    uint32_t o = (uint32_t)st.out_pos + (oincl - nout);   // ring index: low bits suffice

#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        if (T & (1u << j)) {
            const uint32_t x = byte_of(w, j);
            ring[swz(o & (kEncRing - 1))] = (uint8_t)x;
            if (P & (1u << j)) {
                const uint32_t rem = (uint32_t)__builtin_ctz((B24 >> (j + 1)) | 0x100u) + 1u;  // min(9, run left)
                ring[swz((o + 1) & (kEncRing - 1))] = (uint8_t)x;
                ring[swz((o + 2) & (kEncRing - 1))] = (uint8_t)('0' + rem);
                o += 3;
            } else {
                o += 1;
            }
        }
    }
    wave_lds_sync();

    // store every completed 16-byte chunk
    const uint64_t newpos = st.out_pos + ttot;
    const uint64_t c_hi = newpos >> 4;
    for (uint64_t c0 = st.flushed >> 4; c0 < c_hi; c0 += kWave) {
        const uint64_t c = c0 + lane;
        if (c < c_hi) {
            const uint32_t a = (uint32_t)(c * 16u) & (kEncRing - 1);
            const uint32_t s = (a >> 7) & 7u;
            uint4 v = *reinterpret_cast<const uint4*>(ring + (a ^ ((s & 4u) << 2)));
            v = perm4(v, s & 3u);
            *reinterpret_cast<uint4*>(dst + c * 16u) = v;
        }
    }
    wave_lds_sync();
    st.flushed = c_hi << 4;
    st.out_pos = newpos;
    st.prev_byte = last63;
    st.q = apply9(readlane(incl, 63), st.q);
}

__global__ __launch_bounds__(kBlock) void encode_kernel(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint64_t* __restrict__ in_len,
                                                        uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        uint64_t* __restrict__ out_len,
                                                        uint32_t* __restrict__ status, uint32_t n) {
    __shared__ __attribute__((aligned(16))) uint8_t ring_all[kWavesPerBlock * kEncRing];
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = uniform(threadIdx.x / kWave);
    uint8_t* ring = ring_all + wid * kEncRing;
    const uint32_t nw = gridDim.x * kWavesPerBlock;

    for (uint32_t b = blockIdx.x * kWavesPerBlock + wid; b < n; b += nw) {
        const uint64_t U = in_len[b];
        const uint8_t* src = in + in_off[b];
        uint8_t* dst = out + out_off[b];
        if (((uintptr_t)src | (uintptr_t)dst) & 15u) {
            if (lane == 0) {
                out_len[b] = 0;
                if (status) status[b] = RLE_STATUS_MISALIGNED;
            }
            continue;
        }
        EncState st{0, 0, 0, 0};
        const uint64_t ntiles = (U + kTile - 1) / kTile;
        uint4 cur = load_chunk(src, U, 16u * lane);
        uint4 nxt = load_chunk(src, U, kTile + 16u * lane);
        for (uint64_t t = 0; t < ntiles; ++t) {
            const uint64_t pos = t * kTile;
            const uint4 nn = load_chunk(src, U, pos + 2 * kTile + 16u * lane);
            enc_tile(cur, nxt, pos, U, lane, ring, dst, st);
            cur = nxt;
            nxt = nn;
        }
        // the final partial chunk (< 16 bytes): byte stores so no byte past C is touched
        const uint32_t rest = (uint32_t)(st.out_pos - st.flushed);
        if (lane < rest) {
            const uint32_t a = (uint32_t)(st.flushed + lane) & (kEncRing - 1);
            dst[st.flushed + lane] = ring[swz(a)];
        }
        if (lane == 0) {
            out_len[b] = st.out_pos;
            if (status) status[b] = RLE_STATUS_OK;
        }
        wave_lds_sync();
    }
}

// ================================================================ DECODE
// Token-phase table: for an 8-bit mask e of "byte j equals byte j+1" and entry offset d (the
// first token start in the group), entry[e] bits 10d..10d+7 = token starts, 10d+8..9 = exit offset.
__device__ __forceinline__ uint32_t dec_table_entry(uint32_t e) {
    uint32_t ent = 0;
    for (uint32_t d = 0; d < 3; ++d) {
        uint32_t s = d, m = 0;
        while (s < 8) {
            m |= 1u << s;
            s += ((e >> s) & 1u) ? 3u : 1u;
        }
        ent |= (m | ((s - 8u) << 8)) << (10u * d);
    }
    return ent;
}

struct DecState {
    uint64_t out_pos;   // decoded bytes produced so far
    uint64_t flushed;   // decoded bytes already stored (multiple of 16)
    uint32_t d;         // offset of the first token start in the current tile (0..2)
    uint32_t fillc;     // 0x100|byte of the last stored position (hole-fill carry)
    uint32_t tail;      // 0x100|byte when the stream ends in an unbounded-count token, else 0
    uint32_t serial;    // 1 -> stream needs the exact serial path
};

// Flush decoded chunks [c_lo, c_hi) from the hole-encoded u16 ring: positions hold 0x100|byte at
// token starts and 0 elsewhere; each run is filled forward from its start.  Positions >= `total`
// take `tailv` (0, or the unbounded final token's byte).  Chunks past U are never touched; the
// chunk holding U is written byte-wise.
__device__ __forceinline__ void dec_flush(uint64_t c_lo, uint64_t c_hi, uint64_t total, uint64_t U,
                                          uint32_t tailv, uint32_t lane, uint16_t* ring, uint8_t* dst,
                                          uint32_t& fillc) {
    for (uint64_t c0 = c_lo; c0 < c_hi; c0 += kWave) {
        const uint64_t c = c0 + lane;
        const bool active = c < c_hi;
        const bool in_ring = active && (c * 16u) < total;
        uint32_t L[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const uint32_t a = (uint32_t)(c * 32u) & (2u * kDecRing - 1u);  // byte address of the chunk
        const uint32_t s = (a >> 7) & 7u;
        if (in_ring) {
            const uint4 v0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(ring) + a);
            const uint4 v1 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(ring) + a + 16u);
            L[0] = v0.x; L[1] = v0.y; L[2] = v0.z; L[3] = v0.w;
            L[4] = v1.x; L[5] = v1.y; L[6] = v1.z; L[7] = v1.w;
            // undo the swizzle: logical dword k lives at physical k ^ s
            cswap(L[0], L[1], s & 1u); cswap(L[2], L[3], s & 1u); cswap(L[4], L[5], s & 1u); cswap(L[6], L[7], s & 1u);
            cswap(L[0], L[2], s & 2u); cswap(L[1], L[3], s & 2u); cswap(L[4], L[6], s & 2u); cswap(L[5], L[7], s & 2u);
            cswap(L[0], L[4], s & 4u); cswap(L[1], L[5], s & 4u); cswap(L[2], L[6], s & 4u); cswap(L[3], L[7], s & 4u);
        }
        uint32_t h[16];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
            h[2 * k] = L[k] & 0xFFFFu;
            h[2 * k + 1] = L[k] >> 16;
        }
        uint32_t lastp = 0;
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) lastp = h[j] ? h[j] : lastp;
        const uint32_t incl = wave_scan_incl(lastp, 0u, OpLatest());
        const uint32_t before = from_prev_lane(incl, 0u);
        uint32_t cur = before ? before : fillc;
        uint32_t ob[4] = {0, 0, 0, 0};
        const uint64_t pbase = c * 16u;
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) {
            cur = h[j] ? h[j] : cur;
            const uint32_t byte = (pbase + j) < total ? (cur & 0xFFu) : tailv;
            ob[j >> 2] |= byte << (8u * (j & 3u));
        }
        if (active) {
            if (pbase + 16u <= U) {
                *reinterpret_cast<uint4*>(dst + pbase) = make_uint4(ob[0], ob[1], ob[2], ob[3]);
            } else {
                for (uint32_t j = 0; j < 16u && pbase + j < U; ++j) dst[pbase + j] = (uint8_t)(ob[j >> 2] >> (8u * (j & 3u)));
            }
            if (in_ring) {
                *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(ring) + a) = make_uint4(0u, 0u, 0u, 0u);
                *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(ring) + a + 16u) = make_uint4(0u, 0u, 0u, 0u);
            }
        }
        const uint64_t lastlane = (c_hi - 1u - c0) < (kWave - 1u) ? (c_hi - 1u - c0) : (kWave - 1u);
        fillc = readlane(cur, (uint32_t)lastlane);
        wave_lds_sync();
    }
}

__device__ __forceinline__ void dec_tile(uint4 cur, const uint4 nxt, uint64_t pos, uint64_t C, uint64_t U,
                                         uint32_t lane, const uint32_t* tbl, uint16_t* ring, uint8_t* dst,
                                         DecState& st) {
    const uint64_t p0 = pos + 16u * lane;
    const uint32_t nl = p0 >= C ? 0u : (uint32_t)((C - p0) < 16u ? (C - p0) : 16u);
    const uint32_t validm = lowmask(nl);
    // bytes at index >= C read as the zero padding of the stored stream
    uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t nb = nl > 4u * k ? (nl - 4u * k < 4u ? nl - 4u * k : 4u) : 0u;
        w[k] &= lowmask(8u * nb);
    }
    // 2-byte lookahead: next lane's first bytes; lane 63 reads the next tile
    const uint64_t pn = pos + kTile;
    const uint32_t nvn = pn >= C ? 0u : (uint32_t)((C - pn) < 2u ? (C - pn) : 2u);
    const uint32_t nx = readlane(nxt.x, 0) & lowmask(8u * nvn);
    const uint32_t la = from_next_lane(w[0] & 0xFFFFu, nx) & 0xFFFFu;

    // E bit j <=> y[j] == y[j+1]  (a token starting at j is then 3 bytes long)
    const uint32_t NE = nz4(w[0] ^ ((w[0] >> 8) | (w[1] << 24))) | (nz4(w[1] ^ ((w[1] >> 8) | (w[2] << 24))) << 4) |
                        (nz4(w[2] ^ ((w[2] >> 8) | (w[3] << 24))) << 8) | (nz4(w[3] ^ ((w[3] >> 8) | (la << 24))) << 12);
    const uint32_t E = ~NE & 0xFFFFu;
    const uint32_t ta = tbl[E & 0xFFu], tb = tbl[E >> 8];
    uint32_t map = 0;
#pragma unroll
    for (uint32_t d = 0; d < 3; ++d) {
        const uint32_t mid = (ta >> (10u * d + 8u)) & 3u;
        map |= ((tb >> (10u * mid + 8u)) & 3u) << (2u * d);
    }
    const uint32_t incl = wave_scan_incl(map, kMap3Id, OpMap3());
    const uint32_t excl = from_prev_lane(incl, kMap3Id);
    const uint32_t dl = (excl >> (2u * st.d)) & 3u;
    const uint32_t mid = (ta >> (10u * dl + 8u)) & 3u;
    const uint32_t S = (((ta >> (10u * dl)) & 0xFFu) | (((tb >> (10u * mid)) & 0xFFu) << 8)) & validm;
    const uint32_t P = S & E;

    // token lengths: count = (signed char)digit - '0'; <=1 -> 1 byte; 2..9 -> count;
    // >9 -> serial path; <0 (unbounded, fills to U) -> allowed only as the final token
    uint32_t len[16];
    bool serial = false, inf = false;
    uint32_t infval = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        len[j] = 1u;
        if (P & (1u << j)) {
            const uint32_t db = (j + 2u) < 16u ? byte_of(w, j + 2u) : ((la >> (8u * (j + 2u - 16u))) & 0xFFu);
            const int v = (int)(int8_t)db - 48;
            if (v > 9) serial = true;
            else if (v >= 2) len[j] = (uint32_t)v;
            else if (v < 0) {
                inf = true;
                infval = 0x100u | byte_of(w, j);
                if (p0 + j + 3u < C) serial = true;   // not the final token
            }
        }
    }
    uint32_t nout = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) nout += (S & (1u << j)) ? len[j] : 0u;
    const uint32_t oincl = wave_scan_incl(nout, 0u, OpAdd());
    const uint32_t ttot = readlane(oincl, 63);
    const uint64_t newpos = st.out_pos + ttot;
    if (__any(serial) || newpos > U) {
        st.serial = 1;
        return;
    }
    const unsigned long long infb = __ballot(inf);
    if (infb) st.tail = readlane(infval, (uint32_t)__builtin_ctzll(infb));

    uint32_t o = (uint32_t)st.out_pos + (oincl - nout);
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        if (S & (1u << j)) {
            ring[swz(2u * (o & (kDecRing - 1))) >> 1] = (uint16_t)(0x100u | byte_of(w, j));
            o += len[j];
        }
    }
    wave_lds_sync();
    const uint64_t c_hi = newpos >> 4;
    dec_flush(st.flushed >> 4, c_hi, newpos, U, 0u, lane, ring, dst, st.fillc);
    st.flushed = c_hi << 4;
    st.out_pos = newpos;
    st.d = (readlane(incl, 63) >> (2u * st.d)) & 3u;
}

// Exact serial decode (src/rleCompression.c:47-62 semantics, writes capped at cap) for the
// streams the tiled path declines: counts > 9, unbounded counts before the last token, or
// streams that decode to more than U bytes.  One lane; such streams never come from the encoder.
__device__ uint32_t dec_serial(const uint8_t* src, uint64_t C, uint64_t U, uint64_t cap, uint8_t* dst,
                               uint32_t lane, uint16_t* ring) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (uint32_t k = lane; k < kDecRing * 2u / 16u; k += kWave)
        reinterpret_cast<uint4*>(ring)[k] = make_uint4(0u, 0u, 0u, 0u);
    for (uint64_t c = lane; c * 16u < cap; c += kWave) {
        if (c * 16u + 16u <= cap) *reinterpret_cast<uint4*>(dst + c * 16u) = make_uint4(0u, 0u, 0u, 0u);
        else
            for (uint64_t p = c * 16u; p < cap; ++p) dst[p] = 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_lds_sync();
    uint32_t st = RLE_STATUS_SERIAL;
    if (lane == 0) {
        uint64_t o = 0, j = 0;
        while (j < C) {
            if (o >= cap) { st |= RLE_STATUS_OVERFLOW; break; }
            const uint8_t v = src[j];
            dst[o++] = v;
            const uint8_t n1 = (j + 1 < C) ? src[j + 1] : (uint8_t)0;
            if (v == n1) {
                const uint8_t dg = (j + 2 < C) ? src[j + 2] : (uint8_t)0;
                const int occ = (int)(int8_t)dg - 48;
                const uint64_t extra = occ < 0 ? ~0ull : (occ >= 2 ? (uint64_t)(occ - 1) : 0ull);
                const uint64_t room = o < U ? U - o : 0;
                const uint64_t k = extra < room ? extra : room;
                for (uint64_t i = 0; i < k; ++i) dst[o + i] = v;
                o += k;
                j += 3;
            } else {
                j += 1;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return readlane(st, 0);
}

__global__ __launch_bounds__(kBlock) void decode_kernel(const uint8_t* __restrict__ in,
                                                        const uint64_t* __restrict__ in_off,
                                                        const uint64_t* __restrict__ in_len,
                                                        uint8_t* __restrict__ out,
                                                        const uint64_t* __restrict__ out_off,
                                                        const uint64_t* __restrict__ out_len,
                                                        const uint64_t* __restrict__ out_cap,
                                                        uint32_t* __restrict__ status, uint32_t n) {
    __shared__ __attribute__((aligned(16))) uint16_t ring_all[kWavesPerBlock * kDecRing];
    __shared__ uint32_t tbl[256];
    tbl[threadIdx.x] = dec_table_entry(threadIdx.x);
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wid = uniform(threadIdx.x / kWave);
    uint16_t* ring = ring_all + wid * kDecRing;
    for (uint32_t k = lane; k < kDecRing * 2u / 16u; k += kWave)
        reinterpret_cast<uint4*>(ring)[k] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    const uint32_t nw = gridDim.x * kWavesPerBlock;

    for (uint32_t b = blockIdx.x * kWavesPerBlock + wid; b < n; b += nw) {
        const uint64_t C = in_len[b];
        const uint64_t U = out_len[b];
        const uint64_t cap = out_cap ? out_cap[b] : U;
        const uint8_t* src = in + in_off[b];
        uint8_t* dst = out + out_off[b];
        if ((((uintptr_t)src | (uintptr_t)dst) & 15u) || cap < U) {
            if (lane == 0 && status) status[b] = RLE_STATUS_MISALIGNED;
            continue;
        }
        DecState st{0, 0, 0, 0, 0, 0};
        const uint64_t ntiles = (C + kTile - 1) / kTile;
        uint4 cur = load_chunk(src, C, 16u * lane);
        uint4 nxt = load_chunk(src, C, kTile + 16u * lane);
        for (uint64_t t = 0; t < ntiles; ++t) {
            const uint64_t pos = t * kTile;
            const uint4 nn = load_chunk(src, C, pos + 2 * kTile + 16u * lane);
            dec_tile(cur, nxt, pos, C, U, lane, tbl, ring, dst, st);
            if (st.serial) break;
            cur = nxt;
            nxt = nn;
        }
        uint32_t stat = RLE_STATUS_OK;
        if (st.serial) {
            stat = dec_serial(src, C, U, cap, dst, lane, ring);
        } else {
            // remaining positions: the partial chunk still in the ring, then [total, U)
            dec_flush(st.flushed >> 4, (U + 15u) >> 4, st.out_pos, U, st.tail & 0xFFu, lane, ring, dst, st.fillc);
        }
        if (lane == 0 && status) status[b] = stat;
        wave_lds_sync();
    }
}

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
    // phase-9 composition against a lane-serial fold
    const uint32_t f = (x & 1u) ? 16u + (x >> 3) % 9u : (x >> 5) % 9u;
    const uint32_t sc = wave_scan_incl(f, 0u, OpPhase9());
    uint32_t rf = 0;
    for (uint32_t l = 0; l <= lane; ++l) {
        const uint32_t y = v[l];
        rf = OpPhase9()(rf, (y & 1u) ? 16u + (y >> 3) % 9u : (y >> 5) % 9u);
    }
    if (sc != rf) e |= 8;
    const uint32_t m = ((x % 3u)) | (((x >> 4) % 3u) << 2) | (((x >> 8) % 3u) << 4);
    const uint32_t sm = wave_scan_incl(m, kMap3Id, OpMap3());
    uint32_t rm = kMap3Id;
    for (uint32_t l = 0; l <= lane; ++l) {
        const uint32_t y = v[l];
        rm = OpMap3()(rm, ((y % 3u)) | (((y >> 4) % 3u) << 2) | (((y >> 8) % 3u) << 4));
    }
    if (sm != rm) e |= 16;
    if (e) atomicOr(err, e);
}

}  // namespace rle

// ================================================================ C-ABI launchers
namespace {
inline uint32_t grid_for(uint32_t n) {
    uint32_t blocks = (n + rle::kWavesPerBlock - 1) / rle::kWavesPerBlock;
    if (blocks > rle::kMaxBlocks) blocks = rle::kMaxBlocks;
    return blocks ? blocks : 1u;
}
}  // namespace

extern "C" size_t rle_max_compressed_size(size_t U) { return U + U / 2; }

extern "C" int rle_encode_batch_device(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                       void* d_out, const uint64_t* d_out_off, uint64_t* d_out_len,
                                       uint32_t* d_status, uint32_t n, void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return RLE_E_INVAL;
    hipLaunchKernelGGL(rle::encode_kernel, dim3(grid_for(n)), dim3(rle::kBlock), 0, (hipStream_t)stream,
                       (const uint8_t*)d_in, d_in_off, d_in_len, (uint8_t*)d_out, d_out_off, d_out_len, d_status, n);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

extern "C" int rle_decode_batch_device(const void* d_in, const uint64_t* d_in_off, const uint64_t* d_in_len,
                                       void* d_out, const uint64_t* d_out_off, const uint64_t* d_out_len,
                                       const uint64_t* d_out_cap, uint32_t* d_status, uint32_t n, void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_in || !d_in_off || !d_in_len || !d_out || !d_out_off || !d_out_len) return RLE_E_INVAL;
    hipLaunchKernelGGL(rle::decode_kernel, dim3(grid_for(n)), dim3(rle::kBlock), 0, (hipStream_t)stream,
                       (const uint8_t*)d_in, d_in_off, d_in_len, (uint8_t*)d_out, d_out_off, d_out_len, d_out_cap,
                       d_status, n);
    return hipGetLastError() == hipSuccess ? RLE_OK : RLE_E_HIP;
}

extern "C" int rle_gen_synthetic_device(void* d_out, const uint64_t* d_off, const uint64_t* d_len,
                                        const uint32_t* d_kind, const uint64_t* d_index, uint32_t n, void* stream) {
    if (n == 0) return RLE_OK;
    if (!d_out || !d_off || !d_len) return RLE_E_INVAL;
    hipLaunchKernelGGL(rle::gen_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (uint8_t*)d_out,
                       d_off, d_len, d_kind, d_index, n);
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

extern "C" int rle_mi355x_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

extern "C" const char* rle_mi355x_version(void) { return "rle_mi355x 0.1 (gfx950, wave-per-buffer tiled codec)"; }
