/*
 * kth.h -- C-ABI of the MI355X k-th element selection engine (libkth.so).
 *
 * Drop-in boundary for laertispappas/MPI-k-selection's selection path.  The
 * reference has no plugin/FFI layer; its boundary is the C-level contract
 * (IntVector data, n = data->size, k) -> int value used at
 *   kth-problem-seq.c:32-33        VecQuickSort(pVec); solution = VecGet(pVec, k-1);
 *   TODO-kth-problem-cgm.c:76-278  CGM rounds + final gather/sort/VecGet on rank 0
 * Every entry point below replaces one of those call sites (cited per function).
 *
 * Conventions (all functions):
 *   - k is 1-based, 1 <= k <= n (as in the reference's VecGet(k-1) call sites).
 *   - Order is signed int32 order (float32: IEEE total order, see rows_f32).
 *   - The input is NOT modified (the reference sorts in place; both of its
 *     drivers discard the data afterwards, kth-problem-seq.c:36,
 *     TODO-kth-problem-cgm.c:283-284, so not mutating is strictly compatible).
 *   - Return value is 0 (KTH_OK) or a negative KTH_E* code; the answer goes to
 *     *out, never in-band (the in-band VecGet sentinels live in vector.h's
 *     VecKthSelect only).
 *   - Streams are passed as `void *` holding a hipStream_t (NULL = HIP's null
 *     stream).  A new ctx owns a private non-blocking stream until
 *     kth_ctx_set_stream replaces it.  No C++ or framework types cross this
 *     boundary.
 *   - A kth_ctx is not thread-safe: one ctx per host thread or device.
 *   - The product path has no CPU fallback: without a usable GPU every compute
 *     entry point returns KTH_ENODEV.
 */
#ifndef KTH_H
#define KTH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KTH_OK 0
#define KTH_EINVAL (-1)   /* bad n / k / pointer / shape                */
#define KTH_ENOMEM (-2)   /* device or pinned-host allocation failed    */
#define KTH_EHIP (-3)     /* HIP runtime or kernel launch error         */
#define KTH_ENODEV (-4)   /* no HIP device                              */
#define KTH_EINTERNAL (-5) /* device-side consistency check failed      */
#define KTH_ECOMM (-6)    /* RCCL missing or a collective failed        */

#define KTH_VERSION 1

/* Selection paths (kth_stats.path). */
#define KTH_PATH_LDS 1      /* n small: one workgroup, keys resident in LDS            */
#define KTH_PATH_RADIX 2    /* multi-pass radix select over the input                  */
#define KTH_PATH_WINDOW 3   /* sample window + one streaming pass + candidate radix    */
#define KTH_PATH_WINDOW_FALLBACK 4 /* window missed -> radix passes over the input     */

typedef struct kth_ctx kth_ctx;

typedef struct kth_stats {
    int32_t path;          /* KTH_PATH_*                                      */
    int32_t mode;          /* internal final mode (debug)                     */
    uint32_t lo_key, hi_key; /* sample window in order-preserving key space   */
    uint64_t n, k;
    uint64_t cnt_lt;       /* keys below the window                           */
    uint64_t cnt_eq_lo, cnt_eq_hi;
    uint64_t candidates;   /* keys strictly inside the window                 */
    uint64_t capacity;     /* candidate buffer capacity                       */
    int32_t answer;
    int32_t error;         /* device-side error word (0 = none)               */
} kth_stats;

const char *kth_strerror(int code);
int kth_version(void);
/* Hash of the sources this libkth.so was built from (16 hex digits; "unknown"
 * outside the in-tree Makefile).  bench.py uses a PMC measurement only when it
 * was taken on the same build. */
const char *kth_build_id(void);
int kth_device_count(void);

/* --- one-shot entry point -------------------------------------------------
 * Replaces kth-problem-seq.c:32-33 and TODO-kth-problem-cgm.c:76-278.
 * keys may be host or device memory (detected with hipPointerGetAttributes).
 * Synchronous; uses a lazily created per-thread ctx on device 0. */
int kth_select_i32(const int32_t *keys, int64_t n, int64_t k, int32_t *out);

/* --- context API (scratch reuse, streams) ---------------------------------- */
int kth_ctx_create(int device, kth_ctx **ctx);
int kth_ctx_destroy(kth_ctx *ctx);
int kth_ctx_set_stream(kth_ctx *ctx, void *hip_stream);
int kth_ctx_sync(kth_ctx *ctx);
/* Pre-size scratch for inputs of up to n keys (optional; grows on demand). */
int kth_ctx_reserve(kth_ctx *ctx, int64_t n);

/* Synchronous select through a ctx; keys host or device.  Same contract as
 * kth_select_i32. */
int kth_select_i32_ctx(kth_ctx *ctx, const int32_t *keys, int64_t n, int64_t k, int32_t *out);

/* Asynchronous select: d_keys and d_out are device memory; the work is
 * enqueued on the ctx stream and *d_out is written on the device.  No host
 * synchronisation and no allocation once the ctx is reserved for n
 * (graph-capturable). */
int kth_select_i32_async(kth_ctx *ctx, const int32_t *d_keys, int64_t n, int64_t k, int32_t *d_out);

/* Stats of the last select on this ctx (synchronises the ctx stream). */
int kth_ctx_last_stats(kth_ctx *ctx, kth_stats *st);

/* Diagnostics: 1 when the ctx runs the cooperative (grid-barrier) kernels,
 * 0 while it is on the per-level path -- for COOP_BACKOFF = 64 selections of
 * any entry point after a grid-barrier timeout (the synchronous entry points
 * redo the timed-out select; the asynchronous ones report it in the stats). */
int kth_ctx_coop(const kth_ctx *ctx);

/* --- test hooks (TEST ONLY: never set by the product path) ------------------
 * Fault injectors for the parity tests' error paths.  They are off in every
 * new ctx and are not read from the environment; only this call turns them on.
 *   KTH_HOOK_FAULT_TOPK_RANK  value != 0: kth_topk_i32 selects a neighbouring
 *                             rank, so its count pass must report the bracket
 *                             failure (outputs unwritten, stats .error set)
 *   KTH_HOOK_FAULT_BARRIER    1: every grid barrier of the cooperative kernels
 *                             reports a timeout; 2: only the next cooperative
 *                             launch does; 0: off
 *   KTH_HOOK_TOPK_SEG_CAP     entries per staged top-k segment (0 = sized from n;
 *                             small values force the segment-overflow fallback)
 * Returns KTH_EINVAL for an unknown hook or a bad value. */
#define KTH_HOOK_FAULT_TOPK_RANK 1
#define KTH_HOOK_FAULT_BARRIER 2
#define KTH_HOOK_TOPK_SEG_CAP 3
int kth_ctx_test_hook(kth_ctx *ctx, int hook, int64_t value);

/* --- timing (bench) ----------------------------------------------------------
 * When enabled, every select records HIP events on the ctx stream around the
 * streaming pass (the dominant kernel) and around the whole select. */
int kth_ctx_enable_timing(kth_ctx *ctx, int on);
/* Synchronises; returns sums over the selects since the last call and resets:
 * *n_selects, *main_ms (sum of dominant-kernel durations), *total_ms. */
int kth_ctx_take_timing(kth_ctx *ctx, int64_t *n_selects, double *main_ms, double *total_ms);

/* --- batched rows (BASELINE config 5; no reference counterpart) -------------
 * out[r] = k-th smallest of row r of a rows x cols row-major matrix.  cols <=
 * 4096: one wavefront per row, the row held in the wave's registers (64 keys a
 * lane at most); wider rows: one workgroup per row, the row resident in LDS.
 * 1 <= cols <= KTH_ROWS_MAX_COLS.
 * float32 order: IEEE total order with -0.0 < +0.0 and every NaN last
 * (a NaN answer is returned as the canonical quiet NaN 0x7FC00000). */
#define KTH_ROWS_MAX_COLS 16384
int kth_select_rows_i32(kth_ctx *ctx, const int32_t *d_keys, int64_t rows, int32_t cols, int32_t k,
                        int32_t *d_out);
int kth_select_rows_f32(kth_ctx *ctx, const float *d_keys, int64_t rows, int32_t cols, int32_t k,
                        float *d_out);

/* --- top-k per row (the MoE-routing shape) ---------------
 * The k smallest keys of each row (largest != 0: the k largest), with their
 * column indices, in column order; of the keys equal to the k-th, the first
 * ones by column.  d_vals: rows x k values, d_idx: rows x k int32 columns;
 * either may be NULL (not both).  1 <= k <= cols <= KTH_TOPK_MAX_COLS.  Same
 * orders as kth_select_rows_* (float: IEEE total order, NaN above +inf, so
 * NaNs come last for smallest and first for largest). */
#define KTH_TOPK_MAX_COLS 4096
int kth_topk_rows_i32(kth_ctx *ctx, const int32_t *d_keys, int64_t rows, int32_t cols, int32_t k, int largest,
                      int32_t *d_vals, int32_t *d_idx);
int kth_topk_rows_f32(kth_ctx *ctx, const float *d_keys, int64_t rows, int32_t cols, int32_t k, int largest,
                      float *d_vals, int32_t *d_idx);

/* --- top-k of one array ------------------------------------
 * The k smallest keys of d_keys[0..n) (largest != 0: the k largest) with their
 * int64 indices, in index order; of the keys equal to the k-th, the first ones
 * by index.  The reference implies this as sort(a)[0..k) after its select
 * block (kth-problem-seq.c:32-33, VecQuickSort then index); here it is the
 * select (kth_select_i32_async) plus a count pass, a chunk scan and an ordered
 * compaction that reads only the chunks holding output keys.  d_vals: k int32,
 * d_idx: k int64; either may be NULL (not both).  1 <= k <= n.  Asynchronous on
 * the ctx stream (device memory only); a device-side inconsistency leaves the
 * outputs unwritten and shows as kth_ctx_last_stats().error. */
int kth_topk_i32(kth_ctx *ctx, const int32_t *d_keys, int64_t n, int64_t k, int largest, int32_t *d_vals,
                 int64_t *d_idx);

/* --- synthetic inputs (bench / tests) --------------------------------------
 * Fills d_out[0..n) with the keys of global indices offset..offset+n of an
 * n_total-key input of family `dist` (oracle/kth_oracle.h enum ko_dist;
 * bit-identical to the CPU generator). */
int kth_fill_synthetic(kth_ctx *ctx, int32_t *d_out, int64_t n, int64_t offset, int64_t n_total,
                       int dist, uint64_t seed, int32_t param);

/* --- sharded selection, one process per GPU (TODO-kth-problem-cgm.c:76-278) --
 * The CGM rounds (local median :125-131, Gather :135-136, weighted median
 * :139-165, Bcast :168, 3-way count :171-185, Allreduce :190, discard
 * :194-225, final Gatherv + sort :242-278) become:
 *   every rank samples its shard -> the samples are all-gathered -> every rank
 *   derives the same window -> one streaming pass per shard (counts, local
 *   candidates and their first digit) -> per-rank histograms are all-reduced
 *   (uint64 SUM) after each step -> every rank picks the same digit from the
 *   same reduced histogram.
 * Collectives per selection: one all-gather and, when the window is at most
 * 2^24 key values wide (uniform 2^33 half-range keys: ~2^23.3), two
 * all-reduces; wider windows three; the exact fallback after a window miss or
 * a candidate overflow four; a selection decided by the window's counts alone
 * two (the second all-reduce carries an empty slot).
 * The host owns the collectives (RCCL through torch.distributed in
 * kselect/dist.py, or MPI/RCCL from C); these entry points only enqueue the
 * per-rank device work on the ctx stream.  The host waits once per selection:
 * kth_dist_level(1) waits for level 0's kernel (the device has the all-reduce
 * after it still queued) to learn how many levels follow.
 *
 * d_slots: caller-owned device memory of 3 * KTH_STATS_WORDS uint64 words,
 * bound by kth_dist_begin for one selection.  kth_dist_scan and
 * kth_dist_level return the index (0..2) of the slot the caller must
 * all-reduce (SUM) in place across ranks before the next call, or
 * KTH_DIST_DONE; every rank makes the same sequence of calls:
 *   kth_dist_begin   bind slots, set (n_total, k)
 *   kth_dist_sample  local sample of s_local keys of the shard -> d_sample
 *                    (order-preserving uint32 keys); caller all-gathers
 *   kth_dist_window  window from the gathered sample of s_total keys
 *   kth_dist_scan    streaming pass over the shard            -> slot
 *   kth_dist_level   level = 0, 1, 2, ... -> slot, until it returns
 *                    KTH_DIST_DONE (at most KTH_DIST_MAX_LEVELS slots)
 *   kth_dist_result  writes the k-th smallest of the union of all shards to
 *                    *d_out (device) */
#define KTH_STATS_WORDS (8 + 2 * 2048)
#define KTH_DIST_DONE 3
#define KTH_DIST_MAX_LEVELS 3
/* Deprecated (round-4 API): callers loop kth_dist_level until KTH_DIST_DONE;
 * kept so that code written against the old name still builds. */
#define KTH_DIST_LEVELS KTH_DIST_MAX_LEVELS
int kth_dist_begin(kth_ctx *ctx, uint64_t *d_slots, int64_t n_total, int64_t k);
int kth_dist_sample(kth_ctx *ctx, const int32_t *d_keys, int64_t n_local, uint32_t *d_sample,
                    int64_t s_local);
int kth_dist_window(kth_ctx *ctx, const uint32_t *d_sample, int64_t s_total);
int kth_dist_scan(kth_ctx *ctx, const int32_t *d_keys, int64_t n_local);
int kth_dist_level(kth_ctx *ctx, const int32_t *d_keys, int64_t n_local, int level);
int kth_dist_result(kth_ctx *ctx, int32_t *d_out);
/* Optional, right after level 0's slot is all-reduced and before
 * kth_dist_level(ctx, .., 1): enqueue the result as if level 0 were the last
 * (it is when the window is at most 2^24 values wide or decided by its counts),
 * so the device need not wait for the host's look at level 0's status.  If
 * more levels follow, it writes nothing and the protocol goes on; the closing
 * kth_dist_result with the same d_out is then the only launch that writes (and
 * costs nothing when the early one finished the select). */
int kth_dist_result_early(kth_ctx *ctx, int32_t *d_out);
/* The whole step sequence above in ONE call, for a caller that holds an RCCL
 * communicator (one process per GPU): kth_dist_begin .. kth_dist_result with
 * the all-gather of the samples and the slot all-reduces as ncclAllGather /
 * ncclAllReduce (uint64 SUM) on the ctx stream, the early result before
 * level 1 when `early` is nonzero.  nccl_all_reduce / nccl_all_gather are the
 * caller's ncclAllReduce / ncclAllGather entry points, so that the
 * communicator `nccl_comm` (an ncclComm_t of `world` ranks) and the calls come
 * from one RCCL copy.  d_sample: s_local uint32 words, d_gathered: world *
 * s_local; every rank passes the same (n_total, k, s_local).  The host waits
 * once, for level 0's status, as in the step sequence; the answer lands in
 * *d_out (device).  Replaces the per-step host round trips of a scripted
 * caller (kselect.dist uses it over RCCL). */
int kth_dist_select_rccl(kth_ctx *ctx, void *nccl_all_reduce, void *nccl_all_gather, void *nccl_comm, int world,
                         const int32_t *d_keys, int64_t n_local, int64_t n_total, int64_t k, uint64_t *d_slots,
                         uint32_t *d_sample, uint32_t *d_gathered, int64_t s_local, int32_t *d_out, int early);
/* Sample size for n keys (the single-GPU rule: min(2^20, n/64), a multiple
 * of 64).  Sharded callers take about kth_dist_sample_size(n_total) / P keys
 * per rank (a multiple of 64, at least 64), so that the all-gathered sample
 * has the single-GPU size. */
int64_t kth_dist_sample_size(int64_t n);
/* Sampler layout (diagnostics and tests): a sample of s keys from n is read as
 * ceil(s / C) chunks of C = kth_sample_chunk() consecutive keys, chunk c at
 * key c * (n / ceil(s / C)); the last chunk holds the remaining s mod C keys. */
int kth_sample_chunk(void);
/* Window half-width in sample standard deviations: the window ranks in a
 * sample of s keys for rank k of n are p*s -+ (z*sqrt(s*p*(1-p)) + 2), p = k/n
 * (KTH_WINDOW_Z overrides the built-in 5.0). */
double kth_window_z(void);
/* Candidate-buffer capacity (keys) of a streaming pass over n_local keys:
 * max(2^20, n_local / 32); more candidates than this on a rank set its
 * overflow count and the selection takes the exact fallback levels. */
int64_t kth_dist_cand_capacity(int64_t n_local);
/* Early-window slack of the sample phase, in 1/64ths: after each sample digit,
 * the window stops at the picked bins' edges when those hold at most
 * slack/64 times the sample keys the exact window would (96 = 1.5; the
 * KTH_HEAD_SLACK environment variable changes a new ctx's value, 0 = off). */
int kth_window_slack64(void);

/* --- sharded selection, one process driving several GPUs ---------------------
 * Replaces TODO-kth-problem-cgm.c:81-278 (block partition + Scatterv, the
 * weighted-median rounds, final Gatherv + rank-0 sort) for a caller holding one
 * shard per GPU in a single process: the kth_dist_* steps for every device,
 * with the collectives as grouped RCCL calls over communicators from
 * ncclCommInitAll (RCCL is dlopen'ed at first use: the librccl.so.1 already in
 * the process, else the system one; KTH_ECOMM if neither loads).
 * Local transport: ngpu > 1 copies of ONE device id (at most 64) put every
 * shard on that device with no RCCL: the same per-shard steps on one shared
 * stream, the samples gathered in place, each all-reduce a device-side sum of
 * the shards' slots (P shards of a 2^33-key input on one GPU).
 *   kth_sharded_create      devices[0..ngpu) distinct (RCCL), or all equal
 *                           (local); one ctx per shard, one stream and
 *                           communicator per device
 *   kth_sharded_select_i32  shard i = shards[i][0..shard_n[i]) in device
 *                           devices[i]'s memory; k-th smallest (1-based) of the
 *                           union -> *out (host).  Synchronous; the shards must
 *                           be complete when it is called (it does not order
 *                           against the caller's streams).  Shards of fewer
 *                           than 64 keys: the union is copied to device 0 and
 *                           selected there.  Any shard sizes are exact;
 *                           balanced shards (n/P + (i < n%P)) are the fast case.
 *   kth_select_i32_sharded  one-shot form; each shard's device is taken from
 *                           its pointer (device memory only), the handle is
 *                           cached per host thread for the same device list. */
typedef struct kth_sharded kth_sharded;
int kth_sharded_create(const int *devices, int ngpu, kth_sharded **out);
int kth_sharded_destroy(kth_sharded *h);
int kth_sharded_select_i32(kth_sharded *h, const int32_t *const *shards, const int64_t *shard_n, int64_t k,
                           int32_t *out);
int kth_select_i32_sharded(const int32_t *const *dev_shards, const int64_t *shard_n, int ngpu, int64_t k,
                           int32_t *out);
/* Per-shard sample sizes of kth_sharded_select_i32: about
 * kth_dist_sample_size(n_total) keys in all, split in proportion to the shard
 * sizes, each a multiple of 64, at least 64 and at most the shard rounded down
 * to 64.  Writes s_dev[0..P), returns their sum (KTH_EINVAL for bad input).
 * Host-only arithmetic (no device needed). */
int64_t kth_sharded_sample_split(const int64_t *shard_n, int P, int64_t *s_dev);
/* Diagnostics: host microseconds the last kth_sharded_select_i32 on h spent
 * enqueueing device work and collectives for every device (from its entry to
 * the last kth_dist_result enqueue; the wait for the answer excluded); -1 for
 * a NULL handle. */
double kth_sharded_enqueue_us(const kth_sharded *h);

#ifdef __cplusplus
}
#endif
#endif /* KTH_H */
