/*
 * kth_cgm.c -- drop-in for the reference's CGM driver (TODO-kth-problem-cgm.c:35-296)
 * on libkth.so: `mpirun -n P kth_cgm`, one MPI process per GPU.
 *
 * Kept from the reference:
 *   - rank 0 owns the input: MAX_NUMBERS keys from rand() % 99999999 + 1 after
 *     srand(time(NULL)) (:10-17, :64-66), or a raw int32 file (--input);
 *   - the block partition sizev[i] = n/P + (i < n%P) and MPI_Scatterv of the
 *     keys from rank 0 (:81-105);
 *   - MPI_Wtime from before the scatter to the answer (:76, :279) and rank 0's
 *     output lines: "kth element %d\n time: %f\n" (:289) when the answer is
 *     a window edge decided from the all-reduced counts (the reference's pivot
 *     found by its 3-way count, :194-201; on the gather path for tiny inputs:
 *     when every key equals the answer), else "kth element=%d \ntime: %f\n"
 *     (:280, the answer resolved from the candidates, as the reference's
 *     final gather + sort).  The reference's own choice is an artifact of its
 *     pivot sequence (it depends on P); the two rules agree on every input
 *     whose keys are all equal (:289) and differ elsewhere;
 *   - k is 1-based (VecGet(pVec, k - 1), :278).
 * Replaced: the local qsort (:115), the weighted-median rounds (:122-233) and
 * the final Gather/Gatherv + rank-0 sort (:235-278).  Each rank copies its shard
 * to its GPU and runs the kth_dist_* steps (include/kth.h); after each step the
 * ranks sum one 32 KiB slot of u64 counts:
 *   --comm rccl (default when every rank has its own GPU): ncclAllReduce /
 *       ncclAllGather over xGMI, device buffers, no host round trip;
 *   --comm mpi (default when ranks share a GPU, which RCCL refuses): the slot
 *       is staged through host memory and summed with MPI_Allreduce.
 * Every rank ends with the same answer; rank 0 prints it.
 *
 * Usage: mpirun -n P kth_cgm [n=100000000] [k=150] [seed=time(NULL)] [--median]
 *            [--input keys.bin] [--comm rccl|mpi] [--repeat R] [--check]
 *   --median   k = n/2 (TODO-kth-problem-cgm.c~:48)
 *   --repeat R also time R device-resident selects (stderr: per-select ms)
 *   --check    rank 0 verifies the answer with a sort (VecQuickSort of the twin)
 * Unlike the reference, P = 1 is allowed (the reference aborts below two
 * processes, :56-59, because its rank 0 is also the coordinator).
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "kth.h"
#include "vector.h"

#define DIE(...)                                      \
    do {                                              \
        fprintf(stderr, "kth_cgm: " __VA_ARGS__);     \
        fputc('\n', stderr);                          \
        MPI_Abort(MPI_COMM_WORLD, 1);                 \
    } while (0)
#define HIPCHK(x)                                                                 \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) DIE("%s: %s", #x, hipGetErrorString(e_));           \
    } while (0)
#define KTHCHK(x)                                                                 \
    do {                                                                          \
        int r_ = (x);                                                             \
        if (r_ < 0) DIE("%s: %s", #x, kth_strerror(r_));                          \
    } while (0)
#define NCCLCHK(x)                                                                \
    do {                                                                          \
        ncclResult_t r_ = (x);                                                    \
        if (r_ != ncclSuccess) DIE("%s: %s", #x, ncclGetErrorString(r_));         \
    } while (0)

typedef struct {
    int use_rccl;
    ncclComm_t comm;
    hipStream_t stream;
    uint64_t *h_slot; /* host staging (MPI mode) */
    uint32_t *h_sample, *h_sample_all;
} comm_t;

/* Sum slot i (KTH_STATS_WORDS u64) across ranks, in place on the device. */
static void allreduce_slot(comm_t *c, uint64_t *d_slots, int i)
{
    uint64_t *p = d_slots + (size_t)i * KTH_STATS_WORDS;
    if (c->use_rccl) {
        NCCLCHK(ncclAllReduce(p, p, KTH_STATS_WORDS, ncclUint64, ncclSum, c->comm, c->stream));
        return;
    }
    HIPCHK(hipMemcpyAsync(c->h_slot, p, KTH_STATS_WORDS * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    MPI_Allreduce(MPI_IN_PLACE, c->h_slot, KTH_STATS_WORDS, MPI_UINT64_T, MPI_SUM, MPI_COMM_WORLD);
    HIPCHK(hipMemcpyAsync(p, c->h_slot, KTH_STATS_WORDS * 8, hipMemcpyHostToDevice, c->stream));
}

static void allgather_sample(comm_t *c, const uint32_t *d_sample, uint32_t *d_all, int64_t s, int P)
{
    if (c->use_rccl) {
        NCCLCHK(ncclAllGather(d_sample, d_all, (size_t)s, ncclUint32, c->comm, c->stream));
        return;
    }
    HIPCHK(hipMemcpyAsync(c->h_sample, d_sample, (size_t)s * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    MPI_Allgather(c->h_sample, (int)s, MPI_UINT32_T, c->h_sample_all, (int)s, MPI_UINT32_T, MPI_COMM_WORLD);
    HIPCHK(hipMemcpyAsync(d_all, c->h_sample_all, (size_t)s * 4 * P, hipMemcpyHostToDevice, c->stream));
}

/* One sharded select of global rank k over every rank's d_keys[0..n_local).
 * *by_counts: the answer is a window edge, decided from the all-reduced counts
 * alone -- the analogue of the reference's pivot found by its 3-way count
 * (TODO-kth-problem-cgm.c:194-201, printed as :289); otherwise it was
 * resolved from the candidates' digits (the final gather + solve, :235-280). */
static int32_t dist_select(kth_ctx *ctx, comm_t *c, const int32_t *d_keys, int64_t n_local, int64_t n, int64_t k,
                           int P, uint64_t *d_slots, uint32_t *d_sample, uint32_t *d_sample_all, int64_t s,
                           int32_t *d_answer, int *by_counts)
{
    KTHCHK(kth_dist_begin(ctx, d_slots, n, k));
    KTHCHK(kth_dist_sample(ctx, d_keys, n_local, d_sample, s));
    allgather_sample(c, d_sample, d_sample_all, s, P);
    KTHCHK(kth_dist_window(ctx, d_sample_all, s * P));
    int slot = kth_dist_scan(ctx, d_keys, n_local);
    KTHCHK(slot);
    allreduce_slot(c, d_slots, slot);
    for (int l = 0;; ++l) { /* usually one level: two all-reduces in all */
        slot = kth_dist_level(ctx, d_keys, n_local, l);
        KTHCHK(slot);
        if (slot == KTH_DIST_DONE) break;
        allreduce_slot(c, d_slots, slot);
    }
    KTHCHK(kth_dist_result(ctx, d_answer));
    kth_stats st;
    KTHCHK(kth_ctx_last_stats(ctx, &st)); /* synchronises the stream */
    if (st.error != 0) DIE("sharded select: device error %d", st.error);
    const uint32_t key = (uint32_t)st.answer ^ 0x80000000u;
    if (by_counts) *by_counts = st.path == KTH_PATH_WINDOW && (key == st.lo_key || key == st.hi_key);
    int32_t ans = 0;
    HIPCHK(hipMemcpyAsync(&ans, d_answer, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return ans;
}

int main(int argc, char **argv)
{
    long long n = 100000000; /* MAX_NUMBERS, :45 */
    long long k = 150;       /* :48 */
    unsigned seed = (unsigned)time(NULL);
    int median = 0, pos = 0, repeat = 0, check = 0;
    const char *input = NULL, *comm_opt = NULL;

    MPI_Init(&argc, &argv);
    int P, rank;
    MPI_Comm_size(MPI_COMM_WORLD, &P);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);

    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--median")) median = 1;
        else if (!strcmp(argv[i], "--check")) check = 1;
        else if (!strcmp(argv[i], "--input") && i + 1 < argc) input = argv[++i];
        else if (!strcmp(argv[i], "--comm") && i + 1 < argc) comm_opt = argv[++i];
        else if (!strcmp(argv[i], "--repeat") && i + 1 < argc) repeat = atoi(argv[++i]);
        else {
            long long v = atoll(argv[i]);
            if (pos == 0) n = v;
            else if (pos == 1) k = v;
            else if (pos == 2) seed = (unsigned)v;
            pos++;
        }
    }
    if (median) k = n / 2;
    if (n < 1 || n > 0x7FFFFFFFLL) DIE("n must be in [1, 2^31-1] (the reference's int sizes)");
    if (k < 1 || k > n) DIE("k must be in [1, n]");

    /* one GPU per local rank; RCCL needs distinct devices */
    MPI_Comm node;
    MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node);
    int lrank, lsize;
    MPI_Comm_rank(node, &lrank);
    MPI_Comm_size(node, &lsize);
    int ndev = kth_device_count();
    if (ndev <= 0) DIE("no GPU visible (there is no CPU fallback)");
    int dev = lrank % ndev;
    HIPCHK(hipSetDevice(dev));
    int can_rccl = lsize <= ndev, all_rccl = 0;
    MPI_Allreduce(&can_rccl, &all_rccl, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
    comm_t c;
    memset(&c, 0, sizeof c);
    c.use_rccl = comm_opt ? !strcmp(comm_opt, "rccl") : all_rccl;
    if (c.use_rccl && !all_rccl) DIE("--comm rccl needs one GPU per rank (%d ranks per node, %d GPUs)", lsize, ndev);

    /* rank 0 owns the input (:51, :64-66); generated before the clock starts */
    IntVectorPtr pVec = NULL;
    if (rank == 0) {
        pVec = VecNew((int)n);
        if (!pVec) DIE("out of host memory for %lld keys", n);
        if (input) {
            FILE *f = fopen(input, "rb");
            if (!f) DIE("cannot open %s", input);
            size_t got = fread(pVec->data, sizeof(int), (size_t)n, f);
            fclose(f);
            if ((long long)got != n) DIE("%s holds %zu keys, need %lld", input, got, n);
            pVec->size = (int)n;
        } else {
            srand(seed);
            for (long long i = 0; i < n; ++i) VecAdd(pVec, rand() % 99999999 + 1);
        }
    }

    kth_ctx *ctx;
    KTHCHK(kth_ctx_create(dev, &ctx));
    HIPCHK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    KTHCHK(kth_ctx_set_stream(ctx, c.stream));
    if (c.use_rccl) {
        ncclUniqueId id;
        if (rank == 0) NCCLCHK(ncclGetUniqueId(&id));
        MPI_Bcast(&id, sizeof id, MPI_BYTE, 0, MPI_COMM_WORLD);
        NCCLCHK(ncclCommInitRank(&c.comm, P, id, rank));
    }

    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = MPI_Wtime(); /* :76 */

    /* block partition + scatter (:81-105) */
    int *sizev = (int *)malloc(sizeof(int) * P), *displs = (int *)malloc(sizeof(int) * P);
    for (int i = 0, d = 0; i < P; ++i) {
        sizev[i] = (int)(n / P) + (i < n % P);
        displs[i] = d;
        d += sizev[i];
    }
    const int64_t n_local = sizev[rank];
    int32_t *h_local = NULL;
    HIPCHK(hipHostMalloc((void **)&h_local, (size_t)(n_local > 0 ? n_local : 1) * 4, 0));
    MPI_Scatterv(rank == 0 ? pVec->data : NULL, sizev, displs, MPI_INT, h_local, (int)n_local, MPI_INT, 0,
                 MPI_COMM_WORLD);

    /* shard -> this rank's HBM */
    int32_t *d_keys = NULL, *d_answer = NULL;
    HIPCHK(hipMalloc((void **)&d_keys, (size_t)(n_local > 0 ? n_local : 1) * 4));
    HIPCHK(hipMalloc((void **)&d_answer, 4));
    HIPCHK(hipMemcpyAsync(d_keys, h_local, (size_t)n_local * 4, hipMemcpyHostToDevice, c.stream));

    int32_t answer;
    int by_counts = 0;
    /* Shards too small to sample (fewer than 64 keys on some rank): gather to
     * rank 0 and select there, as the reference's final step does (:235-278). */
    const int small = n / P < 64;
    uint64_t *d_slots = NULL;
    uint32_t *d_sample = NULL, *d_sample_all = NULL;
    int64_t s = 0;
    if (small) {
        int32_t *all = rank == 0 ? (int32_t *)malloc((size_t)n * 4) : NULL;
        MPI_Gatherv(h_local, (int)n_local, MPI_INT, all, sizev, displs, MPI_INT, 0, MPI_COMM_WORLD);
        if (rank == 0) {
            KTHCHK(kth_select_i32_ctx(ctx, all, n, k, &answer));
            /* one value: the select is decided by its counts (#< = 0, #== = n) */
            by_counts = 1;
            for (long long i = 0; i < n && by_counts; ++i) by_counts = all[i] == answer;
            free(all);
        }
        MPI_Bcast(&answer, 1, MPI_INT, 0, MPI_COMM_WORLD);
    } else {
        /* ~kth_dist_sample_size(n) sample keys in all, split over the ranks */
        s = kth_dist_sample_size(n) / P;
        s = s < 64 ? 64 : s & ~(int64_t)63;
        HIPCHK(hipMalloc((void **)&d_slots, 3 * (size_t)KTH_STATS_WORDS * 8));
        HIPCHK(hipMalloc((void **)&d_sample, (size_t)s * 4));
        HIPCHK(hipMalloc((void **)&d_sample_all, (size_t)s * 4 * P));
        if (!c.use_rccl) {
            c.h_slot = (uint64_t *)malloc(KTH_STATS_WORDS * 8);
            c.h_sample = (uint32_t *)malloc((size_t)s * 4);
            c.h_sample_all = (uint32_t *)malloc((size_t)s * 4 * P);
        }
        answer = dist_select(ctx, &c, d_keys, n_local, n, k, P, d_slots, d_sample, d_sample_all, s, d_answer,
                             &by_counts);
    }
    double t1 = MPI_Wtime();
    if (rank == 0) {
        if (by_counts) /* the answer is a pivot the 3-way count found (:194-201) */
            printf("kth element %d\n time: %f\n", answer, t1 - t0); /* :289 */
        else
            printf("kth element=%d \ntime: %f\n", answer, t1 - t0); /* :280 */
    }

    /* device-resident repeats: the select alone, keys already in HBM */
    if (repeat > 0 && !small) {
        MPI_Barrier(MPI_COMM_WORLD);
        double r0 = MPI_Wtime();
        for (int r = 0; r < repeat; ++r) {
            int32_t a = dist_select(ctx, &c, d_keys, n_local, n, k, P, d_slots, d_sample, d_sample_all, s, d_answer,
                                    NULL);
            if (a != answer) DIE("repeat %d: answer %d differs from %d", r, a, answer);
        }
        MPI_Barrier(MPI_COMM_WORLD);
        double r1 = MPI_Wtime();
        if (rank == 0)
            fprintf(stderr, "device-resident select: %.3f ms (%d repeats, %s, %d ranks) = %.2f Gkeys/s\n",
                    (r1 - r0) * 1e3 / repeat, repeat, c.use_rccl ? "rccl" : "mpi", P,
                    (double)n / ((r1 - r0) / repeat) / 1e9);
    }

    int rc = 0;
    if (check && rank == 0) {
        IntVectorPtr w = VecNew((int)n);
        memcpy(w->data, pVec->data, (size_t)n * 4);
        w->size = (int)n;
        VecQuickSort(w);
        int want = VecGet(w, (int)(k - 1));
        fprintf(stderr, "check: %s (sorted[k-1] = %d)\n", want == answer ? "ok" : "MISMATCH", want);
        rc = want == answer ? 0 : 3;
        VecDelete(w);
    }
    MPI_Bcast(&rc, 1, MPI_INT, 0, MPI_COMM_WORLD);

    if (c.use_rccl) ncclCommDestroy(c.comm);
    kth_ctx_destroy(ctx);
    hipFree(d_keys);
    hipFree(d_answer);
    if (d_slots) hipFree(d_slots);
    if (d_sample) hipFree(d_sample);
    if (d_sample_all) hipFree(d_sample_all);
    hipStreamDestroy(c.stream);
    hipHostFree(h_local);
    free(c.h_slot);
    free(c.h_sample);
    free(c.h_sample_all);
    free(sizev);
    free(displs);
    if (pVec) VecDelete(pVec);
    MPI_Comm_free(&node);
    MPI_Finalize();
    return rc;
}
