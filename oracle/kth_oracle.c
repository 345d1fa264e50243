/*
 * kth_oracle.c -- CPU restatement of the reference selection path.
 *
 * TEST INFRASTRUCTURE ONLY (see kth_oracle.h).  The product (libkth.so) never
 * links or calls this file.  Each function cites the reference file:line it
 * restates; all line numbers are into /root/reference at the surveyed commit.
 */
#include "kth_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ inputs */

uint64_t ko_hash(uint64_t seed, uint64_t i)
{
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static const int32_t ko_few[4] = {-5, 0, 7, 123456789};

void ko_gen(int32_t *out, int64_t n, int64_t offset, int64_t n_total, int dist,
            uint64_t seed, int32_t param)
{
    uint32_t step = 1;
    if (n_total > 0 && n_total <= (int64_t)0xFFFFFFFFLL) {
        uint64_t s = (1ULL << 32) / (uint64_t)n_total;
        step = s > 0xFFFFFFFFULL ? 0xFFFFFFFFu : (s ? (uint32_t)s : 1u);
    }
    for (int64_t j = 0; j < n; ++j) {
        uint64_t i = (uint64_t)(offset + j);
        uint64_t h = ko_hash(seed, i);
        uint32_t hi = (uint32_t)(h >> 32);
        int32_t v;
        switch (dist) {
        case KO_UNIFORM_FULL: v = (int32_t)hi; break;
        case KO_UNIFORM_HALF: v = ((int32_t)hi) >> 1; break;
        case KO_UNIFORM_REF: v = (int32_t)(hi % 99999999u) + 1; break;
        case KO_ALL_EQUAL: v = param; break;
        case KO_FEW_DISTINCT: v = ko_few[h >> 62]; break;
        case KO_SORTED_ASC: v = (int32_t)(0x80000000u + (uint32_t)i * step); break;
        case KO_SORTED_DESC: v = (int32_t)(0x7FFFFFFFu - (uint32_t)i * step); break;
        case KO_MOD_1000: v = (int32_t)(hi % 1000u); break;
        default: v = 0; break;
        }
        out[j] = v;
    }
}

/* ------------------------------------------------------------ true answer */

static int cmp_safe(const void *x, const void *y)
{
    int32_t a = *(const int32_t *)x, b = *(const int32_t *)y;
    return (a > b) - (a < b);
}

int ko_true_kth(const int32_t *a, int64_t n, int64_t k, int32_t *out)
{
    if (!a || n <= 0 || k < 1 || k > n || !out)
        return -1;
    int32_t *t = (int32_t *)malloc((size_t)n * sizeof(int32_t));
    if (!t)
        return -1;
    memcpy(t, a, (size_t)n * sizeof(int32_t));
    qsort(t, (size_t)n, sizeof(int32_t), cmp_safe);
    *out = t[k - 1];
    free(t);
    return 0;
}

void ko_rank_counts(const int32_t *a, int64_t n, int32_t v, int64_t *lt, int64_t *eq)
{
    int64_t l = 0, e = 0;
    for (int64_t i = 0; i < n; ++i) {
        l += a[i] < v;
        e += a[i] == v;
    }
    *lt = l;
    *eq = e;
}

int ko_rank_check(const int32_t *a, int64_t n, int64_t k, int32_t v)
{
    int64_t lt, eq;
    ko_rank_counts(a, n, v, &lt, &eq);
    return lt < k && k <= lt + eq;
}

/* ------------------------------------------------- restated reference seq */

/* vector.c:6-8 -- `*a - *b`.  The subtraction is done with wrap-around, which
 * is what gcc emits for the reference's signed overflow. */
static int cmp_ref(const void *x, const void *y)
{
    uint32_t a = (uint32_t) * (const int32_t *)x, b = (uint32_t) * (const int32_t *)y;
    return (int32_t)(a - b);
}

/* vector.c:209-218 (VecGet) with position = k - 1 as at kth-problem-seq.c:33 */
static int32_t vecget_ref(const int32_t *data, int64_t size, int64_t position)
{
    if (!data)
        return -1;
    if (position >= size || position < 0)
        return -2;
    return data[position];
}

int32_t ko_seq_ref_inplace(int32_t *a, int64_t n, int64_t k)
{
    /* kth-problem-seq.c:32  VecQuickSort(pVec) -> vector.c:239-241 qsort(compare) */
    qsort(a, (size_t)n, sizeof(int32_t), cmp_ref);
    /* kth-problem-seq.c:33  solution = VecGet(pVec, k - 1) */
    return vecget_ref(a, n, k - 1);
}

int32_t ko_seq_ref(const int32_t *a, int64_t n, int64_t k)
{
    int32_t *t = (int32_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    if (!t)
        return -1;
    if (n > 0)
        memcpy(t, a, (size_t)n * sizeof(int32_t));
    int32_t r = ko_seq_ref_inplace(t, n, k);
    free(t);
    return r;
}

/* ------------------------------------------------- restated reference CGM */

typedef struct {
    int32_t *data;
    int size;
} shard_t;

/* vector.c:108-121 (VecErase): O(1) delete that moves the last element in. */
static void vecerase_ref(shard_t *v, int position)
{
    if (position == v->size - 1)
        v->size--;
    else
        v->data[position] = v->data[--v->size];
}

int ko_cgm_ref(const int32_t *a, int n, int k, int P, int c, int32_t *out,
               int *rounds, int *found_in_round)
{
    if (!a || n < 0 || P < 2 || c <= 0 || !out) /* :56-59 aborts for P < 2 */
        return -1;
    int ret = -1;
    int nr = 0;
    shard_t *sh = (shard_t *)calloc((size_t)P, sizeof(shard_t));
    int *med = (int *)calloc((size_t)P, sizeof(int));
    int *ni = (int *)calloc((size_t)P, sizeof(int));
    if (!sh || !med || !ni)
        goto done;

    /* :81-100 block partition, sizev[i] = n/P + (i < n%P); :103 Scatterv */
    {
        int size = n / P, rem = n % P, displ = 0;
        for (int r = 0; r < P; ++r) {
            int sz = size + (r < rem);
            /* VecNew(sizev) then Scatterv.  A zero-size shard's buffer is never
             * written; the reference reads data[0] of a malloc(0) there (heap
             * garbage) -- the restatement pins that word to 0. */
            sh[r].data = (int32_t *)calloc((size_t)(sz > 0 ? sz : 1), sizeof(int32_t));
            if (!sh[r].data)
                goto done;
            if (sz > 0)
                memcpy(sh[r].data, a + displ, (size_t)sz * sizeof(int32_t));
            sh[r].size = sz;
            displ += sz;
        }
    }
    /* :115 VecQuickSort(local_pVec) -- reference comparator */
    for (int r = 0; r < P; ++r)
        qsort(sh[r].data, (size_t)sh[r].size, sizeof(int32_t), cmp_ref);

    int N = n;
    const int threshold = n / (c * P); /* :122 MAX_NUMBERS / (c * world_size) */
    while (N >= threshold) {
        /* 2.1 local medians, :125-131.  (a+b)/2 wraps like the reference's
         * signed overflow (defect 2).  For an empty shard the reference reads
         * data[-1], the high word of glibc's chunk-size header: 0. */
        for (int r = 0; r < P; ++r) {
            int sz = sh[r].size;
            if (sz % 2 == 0) {
                int32_t x = sh[r].data[sz / 2];
                int32_t y = (sz / 2 - 1 >= 0) ? sh[r].data[sz / 2 - 1] : 0;
                int32_t s = (int32_t)((uint32_t)x + (uint32_t)y);
                med[r] = s / 2;
            } else {
                med[r] = sh[r].data[sz / 2];
            }
            ni[r] = sz; /* 2.2 gathers, :135-136 */
        }
        /* 2.3 weighted median on rank 0, :139-165 */
        int M = med[0];
        for (int i = 0; i < P; ++i) {
            int mk = med[i], min_sum = 0, max_sum = 0;
            for (int j = 0; j < P; ++j) {
                if (med[j] < mk)
                    min_sum += ni[j];
                else if (med[j] > mk)
                    max_sum += ni[j];
            }
            if (min_sum <= N / 2 && max_sum <= N / 2) {
                M = med[i];
                break;
            }
        }
        /* 2.5-2.7 three-way counts + Allreduce SUM, :171-190 */
        int L = 0, E = 0, G = 0;
        for (int r = 0; r < P; ++r)
            for (int i = 0; i < sh[r].size; ++i) {
                int32_t x = sh[r].data[i];
                if (x < M)
                    L++;
                else if (x > M)
                    G++;
                else
                    E++;
            }
        nr++;
        /* 2.9, :194-225 */
        if (k > L && k <= L + E) {
            *out = M;
            if (found_in_round)
                *found_in_round = 1;
            ret = 0;
            goto done;
        }
        int before = 0, after = 0;
        for (int r = 0; r < P; ++r)
            before += sh[r].size;
        if (k <= L) {
            for (int r = 0; r < P; ++r)
                for (int i = 0; i < sh[r].size; i++)
                    if (sh[r].data[i] >= M) {
                        vecerase_ref(&sh[r], i);
                        i--;
                    }
            N = L;
        } else if (k > L + E) {
            for (int r = 0; r < P; ++r)
                for (int i = 0; i < sh[r].size; i++)
                    if (sh[r].data[i] <= M) {
                        vecerase_ref(&sh[r], i);
                        i--;
                    }
            N = G;
            k = k - L - E;
        }
        for (int r = 0; r < P; ++r)
            after += sh[r].size;
        /* Nothing discarded and N unchanged: every later round recomputes the
         * same medians and pivot -- the reference spins forever here. */
        if (after == before && N == before) {
            ret = 1;
            goto done;
        }
    }
    /* 3.-4. gather survivors in rank order, sort, VecGet(k-1), :235-278 */
    {
        int total = 0;
        for (int r = 0; r < P; ++r)
            total += sh[r].size;
        int32_t *all = (int32_t *)malloc((size_t)(total > 0 ? total : 1) * sizeof(int32_t));
        if (!all)
            goto done;
        int off = 0;
        for (int r = 0; r < P; ++r) {
            if (sh[r].size)
                memcpy(all + off, sh[r].data, (size_t)sh[r].size * sizeof(int32_t));
            off += sh[r].size;
        }
        qsort(all, (size_t)total, sizeof(int32_t), cmp_ref);
        *out = vecget_ref(all, total, (int64_t)k - 1);
        free(all);
        if (found_in_round)
            *found_in_round = 0;
        ret = 0;
    }
done:
    if (rounds)
        *rounds = nr;
    if (sh)
        for (int r = 0; r < P; ++r)
            free(sh[r].data);
    free(sh);
    free(med);
    free(ni);
    return ret;
}

/* ---------------------------------------- restated shipped input generators */

void ko_gen_shipped_seq(int32_t *out, int n, unsigned seed)
{
    /* kth-problem-seq.c:23-28.  gcc evaluates the left rand() first; the sum
     * wraps (the reference's signed overflow).  Pinned against a dump of the
     * shipped program's own VecAdd stream in tests/golden. */
    srand(seed);
    int j = 0;
    for (int i = n; i > 0; i--) {
        int r1 = rand();
        int r2 = rand();
        out[j++] = (int32_t)((uint32_t)i + (uint32_t)r1 - (uint32_t)(r2 % i));
    }
}

void ko_gen_shipped_cgm(int32_t *out, int n, unsigned seed)
{
    /* TODO-kth-problem-cgm.c:10-17 */
    srand(seed);
    for (int i = 0; i < n; i++)
        out[i] = rand() % 99999999 + 1;
}
