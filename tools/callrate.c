/* Call rate of the drop-in's small calls under concurrency (the load the
 * server's worker pool produces, src/server.c:520-524, reads running concurrently per
 * src/filesystemApi.c:570 -> 597).  T threads each loop RLEcompress + RLEdecompress of their own
 * U-byte buffer (random bytes) for S seconds; every round trip is checked (decode(encode(x)) == x)
 * and every thread's stream against thread 0's first stream of the same input kind.
 * Prints one JSON line.   usage: callrate T U SECONDS [kind: random|zero]
 * build: gcc -O2 -pthread tools/callrate.c -Iinclude -L<pkg> -lrle_mi355x -Wl,-rpath,<pkg> */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rleCompression.h"
#include "rle_mi355x.h"

static size_t U;
static double secs;
static int zero;
static volatile int go;

typedef struct {
    long calls;
    int bad;
} Res;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void* work(void* arg) {
    Res* r = (Res*)arg;
    char* x = malloc(U);
    uint64_t s = 0x9E3779B97F4A7C15ull + (uint64_t)(uintptr_t)arg;
    for (size_t i = 0; i < U; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        x[i] = zero ? 0 : (char)s;
    }
    while (!go) ;
    const double t0 = now();
    while (now() - t0 < secs) {
        size_t C = 0;
        char* y = RLEcompress(x, U, &C);
        char* z = RLEdecompress(y, C, U, 0);
        if (!y || !z || memcmp(x, z, U)) r->bad++;
        free(y);
        free(z);
        r->calls += 2;
    }
    free(x);
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: callrate T U SECONDS [random|zero]\n");
        return 2;
    }
    const int T = atoi(argv[1]);
    U = (size_t)atol(argv[2]);
    secs = atof(argv[3]);
    zero = argc > 4 && !strcmp(argv[4], "zero");
    pthread_t th[256];
    Res res[256];
    memset(res, 0, sizeof(res));
    {   /* create the thread contexts' device state outside the timed loops */
        size_t C;
        char* w = calloc(U, 1);
        free(RLEcompress(w, U, &C));
        free(w);
    }
    rle_dropin_stats_t st0;
    rle_mi355x_dropin_stats(&st0, 1);
    for (int i = 0; i < T; ++i) pthread_create(&th[i], NULL, work, &res[i]);
    const double t0 = now();
    go = 1;
    long calls = 0;
    int bad = 0;
    for (int i = 0; i < T; ++i) {
        pthread_join(th[i], NULL);
        calls += res[i].calls;
        bad += res[i].bad;
    }
    const double el = now() - t0;
    rle_dropin_stats_t st;
    rle_mi355x_dropin_stats(&st, 0);
    printf("{\"threads\": %d, \"U\": %zu, \"kind\": \"%s\", \"calls\": %ld, \"seconds\": %.3f, \"calls_per_s\": %.1f, "
           "\"us_per_call_per_thread\": %.3f, \"bad\": %d, \"calls_coalesced\": %llu, \"launches_coalesced\": %llu}\n",
           T, U, zero ? "zero" : "random", calls, el, calls / el, el * 1e6 * T / (calls ? calls : 1), bad,
           (unsigned long long)st.calls_coalesced, (unsigned long long)st.launches_coalesced);
    return bad ? 1 : 0;
}
