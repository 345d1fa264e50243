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
 * Usage: kth_seq [n=100000000] [k=250] [seed=time(NULL)] [--median]
 *   --median sets k = n/2 as in kth-problem-seq.c~:24.
 * The reference times with clock() (CPU time, :30,35); this driver reports
 * the wall time of the select (the work happens on the GPU, so CPU time would
 * understate it) plus the same clock() figure on stderr.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "kth.h"
#include "vector.h"

int main(int argc, char **argv)
{
    long n = 100000000;
    long k = 250;
    unsigned seed = (unsigned)time(NULL);
    int median = 0, pos = 0;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--median")) {
            median = 1;
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

    struct timespec w0, w1;
    clock_t start = clock();
    clock_gettime(CLOCK_MONOTONIC, &w0);
    int solution = 0;
    /* VecKthSelect keeps VecGet's in-band sentinels (a valid key could equal
     * one); the driver takes the explicit status so a failure is loud */
    const int rc = VecKthSelectEx(pVec, (int)k, &solution);
    clock_gettime(CLOCK_MONOTONIC, &w1);
    clock_t end = clock();
    VecDelete(pVec);
    if (rc != 0) {
        fprintf(stderr, "kth_seq: select failed: %s (no CPU fallback)\n", kth_strerror(rc));
        return 1;
    }

    double wall = (double)(w1.tv_sec - w0.tv_sec) + 1e-9 * (double)(w1.tv_nsec - w0.tv_nsec);
    printf("Solution found solution=%d \ntime: %f\n", solution, wall);
    fprintf(stderr, "cpu time (clock): %f\n", (end - start) / (double)CLOCKS_PER_SEC);
    return 0;
}
