/*
 * rle_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker; never shipped, never timed as
 * the product).  Clean-room restatement of the reference codec's *behaviour*
 * (src/rleCompression.c:9-62), written from SURVEY.md Appendix A, not from its code.
 */
#include "rle_oracle.h"

#include <pthread.h>
#include <string.h>

size_t oracle_rle_max_compressed(size_t U) { return U + U / 2; }

/* Encoder — closed form of src/rleCompression.c:9-45.
 * A maximal run [s,e) of byte v is cut into chunks that start at s, s+9, s+18, ...
 * (i.e. token starts are the positions with (i - runstart(i)) % 9 == 0); a chunk of
 * length r = min(9, e - start) emits "v" when r == 1 (:30-31) and "v v ('0'+r)" when
 * r >= 2 (:24-26 for full 9-chunks, :35-37 for the remainder). */
size_t oracle_rle_encode(const uint8_t* x, size_t U, uint8_t* out) {
    size_t o = 0, s = 0;
    while (s < U) {
        const uint8_t v = x[s];
        size_t e = s + 1;
        while (e < U && x[e] == v) e++;                 /* maximal run, :16-18 */
        for (size_t c = s; c < e; c += 9) {
            const size_t r = (e - c) < 9 ? (e - c) : 9;
            out[o++] = v;
            if (r >= 2) {
                out[o++] = v;
                out[o++] = (uint8_t)('0' + r);
            }
        }
        s = e;                                           /* :41 */
    }
    return o;                                            /* :43 */
}

/* Decoder — src/rleCompression.c:47-62 restated.
 *  token at j: emit y[j] unconditionally (:51); if y[j] == y[j+1] (:52) the token is 3 bytes
 *  and the count is occ = (signed char)y[j+2] - '0' evaluated as size_t (:53): negative
 *  values wrap to huge; extra copies = occ-1 (occ >= 2), capped so the output index stays
 *  below U (:54-56); bytes past C are the calloc padding (0). */
uint32_t oracle_rle_decode(const uint8_t* y, size_t C, size_t U, size_t cap, uint8_t* out,
                           size_t* written) {
    memset(out, 0, cap);                                 /* calloc(U+E) :48 */
    size_t o = 0, j = 0;
    uint32_t st = ORACLE_RLE_OK;
    while (j < C) {
        if (o >= cap) { st = ORACLE_RLE_OVERFLOW; break; }
        const uint8_t v = y[j];
        out[o++] = v;
        const uint8_t n1 = (j + 1 < C) ? y[j + 1] : 0;
        if (v == n1) {
            const uint8_t d = (j + 2 < C) ? y[j + 2] : 0;
            const long occ = (long)(int8_t)d - 48;
            size_t extra;
            if (occ < 0) extra = (size_t)-1;             /* size_t wrap: unbounded */
            else extra = occ >= 2 ? (size_t)(occ - 1) : 0;
            const size_t room = o < U ? U - o : 0;
            const size_t k = extra < room ? extra : room;
            memset(out + o, v, k);
            o += k;
            j += 3;
        } else {
            j += 1;
        }
    }
    if (written) *written = o;
    return st;
}

/* ---------------- batch helpers (pthreads) ---------------- */
typedef struct {
    int dec;
    const uint8_t* in; const uint64_t* in_off; const uint64_t* in_len;
    uint8_t* out; const uint64_t* out_off; uint64_t* out_len_w; const uint64_t* out_len_r;
    uint32_t* status; uint32_t n; int tid; int nt;
} job_t;

static void* worker(void* p) {
    job_t* j = (job_t*)p;
    for (uint32_t i = (uint32_t)j->tid; i < j->n; i += (uint32_t)j->nt) {
        if (!j->dec) {
            j->out_len_w[i] = oracle_rle_encode(j->in + j->in_off[i], j->in_len[i], j->out + j->out_off[i]);
        } else {
            const size_t U = j->out_len_r[i];
            const uint32_t st = oracle_rle_decode(j->in + j->in_off[i], j->in_len[i], U, U,
                                                  j->out + j->out_off[i], NULL);
            if (j->status) j->status[i] = st;
        }
    }
    return NULL;
}

static void run_batch(job_t proto, int nthreads) {
    if (nthreads <= 0) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job_t jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = proto; jobs[t].tid = t; jobs[t].nt = nthreads;
        if (nthreads == 1) { worker(&jobs[0]); return; }
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

void oracle_rle_encode_batch(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                             uint8_t* out, const uint64_t* out_off, uint64_t* out_len,
                             uint32_t n, int nthreads) {
    job_t j = {0, in, in_off, in_len, out, out_off, out_len, NULL, NULL, n, 0, 1};
    run_batch(j, nthreads);
}

void oracle_rle_decode_batch(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                             uint8_t* out, const uint64_t* out_off, const uint64_t* out_len,
                             uint32_t* status, uint32_t n, int nthreads) {
    job_t j = {1, in, in_off, in_len, out, out_off, NULL, out_len, status, n, 0, 1};
    run_batch(j, nthreads);
}

/* ---------------- synthetic generator ---------------- */
static inline uint64_t xs64(uint64_t* s) {
    uint64_t x = *s;
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    *s = x;
    return x;
}

void oracle_gen_buffer(uint32_t kind, uint64_t index, uint8_t* x, size_t U) {
    uint64_t s = 0x9E3779B97F4A7C15ULL + index;
    switch (kind) {
    case 0:
        memset(x, 0, U);
        break;
    case 1:
        for (size_t k = 0; k < U; k++) x[k] = (uint8_t)xs64(&s);
        break;
    case 2:
    case 3: {
        const uint32_t P = kind == 2 ? 50u : 90u;
        for (size_t k = 0; k < U; k++) {
            const uint64_t r = xs64(&s);
            if (k > 0 && (uint32_t)((r >> 32) % 100u) < P) x[k] = x[k - 1];
            else x[k] = (uint8_t)r;
        }
        break;
    }
    case 4:
    default:
        for (size_t k = 0; k < U; k += 2) {
            uint8_t v = (uint8_t)xs64(&s);
            if (k > 0 && v == x[k - 1]) v ^= 1u;
            x[k] = v;
            if (k + 1 < U) x[k + 1] = v;
        }
        break;
    }
}
