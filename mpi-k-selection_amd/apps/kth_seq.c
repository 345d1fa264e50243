/*
 * kth_seq.c -- drop-in for the reference's sequential driver
 * (kth-problem-seq.c:17-39) on libkth.so.
 *
 * Same input generator (kth-problem-seq.c:23-28: srand(time); for i = n..1:
 * VecAdd(i + rand() - rand()%i), evaluated left to right and wrapping like the
 * reference build), same IntVector container, same output format
 * ("Solution found solution=%d \ntime: %f\n", :37) -- but the select block
 * `VecQuickSort(pVec); solution = VecGet(pVec, k - 1);` (:32-33) becomes
 * VecKthSelectEx(pVec, k, &solution), i.e. the GPU selection through the
 * C-ABI, with an explicit status instead of VecGet's in-band sentinels.
 *
 * Usage: kth_seq [n=100000000] [k=250] [seed=time(NULL)] [--median] [--breakdown]
 *   --median    sets k = n/2 as in kth-problem-seq.c~:24.
 *   --breakdown starts the HIP runtime before the timed select (timed
 *               apart: runtime_init_s), and after the drop-in select times
 *               its parts on a fresh ctx (stderr, one JSON line): ctx
 *               creation, device allocation, the host-to-device copy of the
 *               keys, the first and a second select of the device-resident
 *               keys.
 * The reference times with clock() (CPU time, :30,35); this driver reports
 * the wall time of the select (the work happens on the GPU, so CPU time would
 * understate it) plus the same clock() figure on stderr.  That wall time is
 * end to end: the drop-in's first call creates the HIP runtime and its ctx,
 * stages the host keys to the device and selects.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "kth.h"
#include "vector.h"

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* The drop-in's one-shot cost, part by part, on a fresh ctx (the HIP runtime
 * is already up: the drop-in call created it). */
static int breakdown(const int *keys, long n, long k, int expect, double t_init)
{
    kth_ctx *ctx = NULL;
    int32_t *d = NULL, a1 = 0, a2 = 0;
    double t0 = now_s();
    if (kth_ctx_create(0, &ctx) != KTH_OK) return 1;
    double t1 = now_s();
    if (kth_ctx_reserve(ctx, n) != KTH_OK || hipMalloc((void **)&d, (size_t)n * 4) != hipSuccess) return 1;
    double t2 = now_s();
    if (hipMemcpy(d, keys, (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess) return 1;
    double t3 = now_s();
    if (kth_select_i32_ctx(ctx, d, n, k, &a1) != KTH_OK) return 1;
    double t4 = now_s();
    if (kth_select_i32_ctx(ctx, d, n, k, &a2) != KTH_OK) return 1;
    double t5 = now_s();
    fprintf(stderr,
            "{\"breakdown\": true, \"n\": %ld, \"k\": %ld, \"runtime_init_s\": %.6f, \"ctx_create_s\": %.6f, "
            "\"alloc_s\": %.6f, "
            "\"h2d_s\": %.6f, \"h2d_gbs\": %.2f, \"select_first_s\": %.6f, \"select_second_s\": %.6f, "
            "\"answers_agree\": %s}\n",
            n, k, t_init, t1 - t0, t2 - t1, t3 - t2, (double)n * 4 / (t3 - t2) / 1e9, t4 - t3, t5 - t4,
            (a1 == expect && a2 == expect) ? "true" : "false");
    hipFree(d);
    kth_ctx_destroy(ctx);
    return (a1 == expect && a2 == expect) ? 0 : 3;
}

int main(int argc, char **argv)
{
    long n = 100000000;
    long k = 250;
    unsigned seed = (unsigned)time(NULL);
    int median = 0, pos = 0, split = 0;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--median")) {
            median = 1;
            continue;
        }
        if (!strcmp(argv[i], "--breakdown")) {
            split = 1;
            continue;
        }
        long v = atol(argv[i]);
        if (pos == 0)
            n = v;
        else if (pos == 1)
            k = v;
        else if (pos == 2)
            seed = (unsigned)v;
        pos++;
    }
    if (median)
        k = n / 2;
    if (n < 1 || n > 0x7FFFFFFFL) {
        fprintf(stderr, "kth_seq: n must be in [1, 2^31-1] (IntVector sizes are int)\n");
        return 2;
    }

    IntVectorPtr pVec = VecNew((int)n);
    if (!pVec) {
        fprintf(stderr, "kth_seq: out of memory\n");
        return 1;
    }
    srand(seed);
    for (long i = n; i > 0; i--) {
        unsigned r1 = (unsigned)rand();
        unsigned r2 = (unsigned)rand();
        VecAdd(pVec, (int)((unsigned)i + r1 - r2 % (unsigned)i));
    }

    double t_init = 0.0;
    if (split) { /* the HIP runtime's start, timed apart from the select */
        const double i0 = now_s();
        (void)kth_device_count();
        t_init = now_s() - i0;
    }
    struct timespec w0, w1;
    clock_t start = clock();
    clock_gettime(CLOCK_MONOTONIC, &w0);
    int solution = 0;
    /* VecKthSelect keeps VecGet's in-band sentinels (a valid key could equal
     * one); the driver takes the explicit status so a failure is loud */
    const int rc = VecKthSelectEx(pVec, (int)k, &solution);
    clock_gettime(CLOCK_MONOTONIC, &w1);
    clock_t end = clock();
    if (rc != 0) {
        VecDelete(pVec);
        fprintf(stderr, "kth_seq: select failed: %s (no CPU fallback)\n", kth_strerror(rc));
        return 1;
    }

    double wall = (double)(w1.tv_sec - w0.tv_sec) + 1e-9 * (double)(w1.tv_nsec - w0.tv_nsec);
    printf("Solution found solution=%d \ntime: %f\n", solution, wall);
    fflush(stdout);
    fprintf(stderr, "cpu time (clock): %f\n", (end - start) / (double)CLOCKS_PER_SEC);
    const int brc = split ? breakdown(pVec->data, n, k, solution, t_init) : 0;
    VecDelete(pVec);
    return brc;
}
