/*
 * kth_oracle.h -- CPU restatement of laertispappas/MPI-k-selection's selection path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker / CPU baseline, never as the
 * thing measured or shipped.
 *
 * Pinning: every function here is checked against golden vectors produced by
 * the reference itself, compiled from /root/reference by oracle/Makefile into
 * oracle/_ref/ (see tests/golden/make_golden.py and tests/test_oracle_golden.py).
 */
#ifndef KTH_ORACLE_H
#define KTH_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Synthetic input families shared bit-for-bit with the device generator
 * (kth_fill_synthetic in include/kth.h) and tests/golden/gen.py. */
enum ko_dist {
    KO_UNIFORM_FULL = 0,   /* int32(h >> 32): full int32 range                          */
    KO_UNIFORM_HALF = 1,   /* int32(h >> 32) >> 1: [-2^30, 2^30), reference well-defined */
    KO_UNIFORM_REF = 2,    /* (h>>32) % 99999999 + 1: TODO-kth-problem-cgm.c:16 range   */
    KO_ALL_EQUAL = 3,      /* every key = param                                         */
    KO_FEW_DISTINCT = 4,   /* 4 values {-5, 0, 7, 123456789} picked by h >> 62          */
    KO_SORTED_ASC = 5,     /* INT32_MIN + i*step, step = clamp(2^32 / n_total, 1, 2^32-1)          */
    KO_SORTED_DESC = 6,    /* INT32_MAX - i*step                                        */
    KO_MOD_1000 = 7,       /* (h>>32) % 1000: heavy duplicates, 1000 distinct values    */
};

/* splitmix64 of a counter: h(i) = mix(seed + (i + 1) * 0x9E3779B97F4A7C15). */
uint64_t ko_hash(uint64_t seed, uint64_t i);

/* Fill out[0..n) with keys for global indices offset .. offset+n of an input of
 * n_total keys. */
void ko_gen(int32_t *out, int64_t n, int64_t offset, int64_t n_total, int dist,
            uint64_t seed, int32_t param);

/* The true k-th smallest (k 1-based, signed int32 order) of a[0..n).  Copies and
 * sorts with an overflow-free comparator.  Returns 0, or -1 on bad k / OOM. */
int ko_true_kth(const int32_t *a, int64_t n, int64_t k, int32_t *out);

/* O(n) certificate: 1 iff #(a < v) < k <= #(a <= v). */
int ko_rank_check(const int32_t *a, int64_t n, int64_t k, int32_t v);

/* #(a < v) and #(a == v). */
void ko_rank_counts(const int32_t *a, int64_t n, int32_t v, int64_t *lt, int64_t *eq);

/* Restated sequential path, kth-problem-seq.c:32-33: qsort with the reference
 * comparator `*a - *b` (vector.c:6-8, overflows for keys > INT_MAX apart) on a
 * copy, then VecGet(k-1) with its in-band sentinels (vector.c:209-218). */
int32_t ko_seq_ref(const int32_t *a, int64_t n, int64_t k);

/* Same, but sorting in place (what the reference does; used for CPU timing). */
int32_t ko_seq_ref_inplace(int32_t *a, int64_t n, int64_t k);

/* Restated CGM weighted-median rounds, TODO-kth-problem-cgm.c:76-285, with P
 * simulated ranks in one thread.  Returns 0 (answer in *out, which may be a
 * VecGet sentinel exactly as the reference would print it), 1 if the rounds can
 * make no further progress (the reference livelocks: SURVEY.md 8(c) defect 2),
 * -1 on bad arguments / OOM.  *rounds = weighted-median rounds executed;
 * *found_in_round = 1 when the answer came from step 2.9 (printed as
 * "kth element %d" at :289) and 0 when from the final gather (:280). */
int ko_cgm_ref(const int32_t *a, int n, int k, int P, int c, int32_t *out,
               int *rounds, int *found_in_round);

/* Restated generators of the shipped programs (glibc rand()):
 *   kth-problem-seq.c:23-28   srand(seed); for i=n..1: i + rand() - rand()%i
 *   TODO-kth-problem-cgm.c:10-17  srand(seed); rand() % 99999999 + 1         */
void ko_gen_shipped_seq(int32_t *out, int n, unsigned seed);
void ko_gen_shipped_cgm(int32_t *out, int n, unsigned seed);

#ifdef __cplusplus
}
#endif
#endif
