/* CPU lifecycle driver of the drop-in library (tests/test_lifecycle.py).  Runs against a test build
 * of librle_mi355x (RLE_TEST_HOOKS) compiled with ASan or TSan, with RLE_MI355X_FAKE_DEVICES set: thread
 * contexts then hold no HIP object, so the start-up thread (rle_dropin.cpp preinit_*), its pool, the
 * pthread-key destructors (free_ctx), fork and the exit ordering (on_exit_handler) run without a GPU.
 * Scenarios (argv[1]), after the reference server's own lifecycle (src/server.c:520-524 worker pool,
 * :615-623 exit):
 *   exit     main returns at once, the start-up thread still building contexts
 *   workers  24 threads take contexts; half are joined, main exits while the rest are still in
 *            their key destructors
 *   fork     fork while the start-up thread runs; the child takes a context and exits
 *   dlopen   (not linked) the library is dlopen()ed after main started (argv[2]), threads take
 *            contexts, main exits
 * Exit status 0 on success. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

typedef int (*touch_fn)(void);
static touch_fn touch;

static void* worker(void* arg) {
    long k = (long)arg;
    if (touch() < 0) abort();
    usleep((useconds_t)(100 * (k % 7)));
    return NULL;
}

static int run_workers(int n, int join) {
    pthread_t th[64];
    for (long i = 0; i < n; ++i)
        if (pthread_create(&th[i], NULL, worker, (void*)i)) return 2;
    for (int i = 0; i < join; ++i) pthread_join(th[i], NULL);
    for (int i = join; i < n; ++i) pthread_detach(th[i]);
    return 0;
}

#ifndef LC_DLOPEN
int rle_test_touch_ctx(void);
int rle_mi355x_preinit_state(void);
#endif

int main(int argc, char** argv) {
    const char* sc = argc > 1 ? argv[1] : "exit";
#ifdef LC_DLOPEN
    if (argc < 3) return 2;
    usleep(1000);   /* well after start-up */
    void* h = dlopen(argv[2], RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 3; }
    touch = (touch_fn)dlsym(h, "rle_test_touch_ctx");
    int (*state)(void) = (int (*)(void))dlsym(h, "rle_mi355x_preinit_state");
    if (!touch || !state) return 4;
    if (state() != 1) { fprintf(stderr, "start-up not running after dlopen with RLE_MI355X_PREINIT\n"); return 5; }
    (void)sc;
    return run_workers(16, 8);
#else
    touch = rle_test_touch_ctx;
    if (rle_mi355x_preinit_state() != 1) { fprintf(stderr, "start-up not running in a linked program\n"); return 5; }
    if (!strcmp(sc, "exit")) return 0;
    if (!strcmp(sc, "workers")) return run_workers(24, 12);
    if (!strcmp(sc, "fork")) {
        pid_t p = fork();
        if (p < 0) return 6;
        if (p == 0) {
            if (touch() < 0) _exit(7);
            exit(0);   /* atexit handlers: the child has no start-up thread to join */
        }
        int st = 0;
        if (waitpid(p, &st, 0) != p) return 8;
        if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) { fprintf(stderr, "child status %d\n", st); return 9; }
        return run_workers(8, 8);
    }
    return 2;
#endif
}
