/*
 * ref_bench.c — TEST INFRASTRUCTURE ONLY: the CPU-baseline harness for bench.py.
 *
 * Linked (by oracle/Makefile) against the UNCHANGED reference codec compiled from
 * /root/reference/src/rleCompression.c, so the timed code is the reference's own
 * RLEcompress/RLEdecompress (src/rleCompression.c:9-62).  Inputs come from the
 * oracle's synthetic generator (same seeds as the GPU bench).  A bounded sample:
 * buffers are processed round-robin by T pthreads, repeating passes over the batch
 * until the time budget is spent (at least one full pass); the achieved rate is reported in U-GiB/s.
 *
 * usage: ref_bench --kinds 1,0 --size 4096 --count 4096 --threads 8 --seconds 10
 *        (--size 0 = mixed log-uniform 4 KiB..1 MiB sizes, see bench.py)
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rle_oracle.h"

char* RLEcompress(char* data, size_t origSize, size_t* compressedSize);
char* RLEdecompress(char* data, size_t compressedSize, size_t uncompressedSize, size_t extraAllocation);

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct {
    uint8_t** bufs; size_t* sizes; uint32_t n;
    int tid, nt; double deadline;
    uint64_t done_bytes, done_comp, done_bufs, c_first; int mismatch;
    double enc_s, dec_s;
} ctx_t;

static void* work(void* p) {
    ctx_t* c = (ctx_t*)p;
    for (uint64_t k = 0;; k++) {
        const uint32_t i = (uint32_t)((uint64_t)c->tid + k * (uint64_t)c->nt) % c->n;
        /* at least one full pass over this thread's share, then until the deadline */
        if ((uint64_t)c->tid + k * (uint64_t)c->nt >= c->n && now() > c->deadline) break;
        size_t C = 0;
        double t0 = now();
        char* z = RLEcompress((char*)c->bufs[i], c->sizes[i], &C);
        double t1 = now();
        char* d = RLEdecompress(z, C, c->sizes[i], 0);
        double t2 = now();
        if (memcmp(d, c->bufs[i], c->sizes[i]) != 0) c->mismatch = 1;
        free(z); free(d);
        c->enc_s += t1 - t0; c->dec_s += t2 - t1;
        if ((uint64_t)c->tid + k * (uint64_t)c->nt < c->n) c->c_first += C;  /* first pass: sum C of the batch */
        c->done_bytes += c->sizes[i]; c->done_comp += C; c->done_bufs++;
    }
    return NULL;
}

static uint64_t xs(uint64_t* s) { uint64_t x = *s; x ^= x << 13; x ^= x >> 7; x ^= x << 17; *s = x; return x; }

int main(int argc, char** argv) {
    const char* kinds = "1,0";
    size_t size = 4096; uint32_t count = 4096; int threads = 1; double seconds = 10.0;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--kinds")) kinds = argv[i + 1];
        else if (!strcmp(argv[i], "--size")) size = strtoull(argv[i + 1], NULL, 10);
        else if (!strcmp(argv[i], "--count")) count = (uint32_t)strtoul(argv[i + 1], NULL, 10);
        else if (!strcmp(argv[i], "--threads")) threads = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--seconds")) seconds = atof(argv[i + 1]);
    }
    uint32_t klist[16]; int nk = 0;
    for (const char* p = kinds; *p && nk < 16;) {
        klist[nk++] = (uint32_t)strtoul(p, (char**)&p, 10);
        if (*p == ',') p++;
    }
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    uint8_t** bufs = calloc(count, sizeof(*bufs));
    size_t* sizes = calloc(count, sizeof(*sizes));
    for (uint32_t i = 0; i < count; i++) {
        size_t U = size;
        if (size == 0) { /* mixed: same rule as bench.py mixed_sizes() */
            uint64_t s = 0x9E3779B97F4A7C15ULL + i + 0x5151ULL;
            uint64_t r = xs(&s);
            U = (size_t)1 << (12 + (r % 9));
            if ((r >> 8) & 1) U += (xs(&s) >> 16) % U;
        }
        sizes[i] = U;
        bufs[i] = malloc(U ? U : 1);
        oracle_gen_buffer(klist[i % (uint32_t)nk], i, bufs[i], U);
    }
    pthread_t th[256]; ctx_t cx[256];
    double t0 = now();
    for (int t = 0; t < threads; t++) {
        memset(&cx[t], 0, sizeof(cx[t]));
        cx[t].bufs = bufs; cx[t].sizes = sizes; cx[t].n = count; cx[t].tid = t; cx[t].nt = threads;
        cx[t].deadline = t0 + seconds;
        pthread_create(&th[t], NULL, work, &cx[t]);
    }
    uint64_t bytes = 0, comp = 0, nb = 0, cbatch = 0; int mism = 0; double es = 0, ds = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        bytes += cx[t].done_bytes; comp += cx[t].done_comp; nb += cx[t].done_bufs;
        mism |= cx[t].mismatch; cbatch += cx[t].c_first; es += cx[t].enc_s; ds += cx[t].dec_s;
    }
    double wall = now() - t0;
    const double gib = 1024.0 * 1024.0 * 1024.0;
    /* rt/enc/dec rates use the codec's busy time (summed over threads, / threads); wall_gibs
     * also includes the harness's verification memcmp */
    printf("{\"threads\": %d, \"buffers\": %llu, \"u_bytes\": %llu, \"c_bytes\": %llu, \"wall_s\": %.6f, "
           "\"wall_gibs\": %.6f, \"rt_gibs\": %.6f, \"enc_gibs\": %.6f, \"dec_gibs\": %.6f, \"c_batch\": %llu, \"roundtrip_ok\": %s}\n",
           threads, (unsigned long long)nb, (unsigned long long)bytes, (unsigned long long)comp, wall,
           (double)bytes / gib / wall, (es + ds) > 0 ? (double)bytes / gib / ((es + ds) / threads) : 0.0,
           es > 0 ? (double)bytes / gib / (es / threads) : 0.0,
           ds > 0 ? (double)bytes / gib / (ds / threads) : 0.0, (unsigned long long)cbatch, mism ? "false" : "true");
    for (uint32_t i = 0; i < count; i++) free(bufs[i]);
    free(bufs); free(sizes);
    return mism ? 1 : 0;
}
