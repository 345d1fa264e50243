/*
 * kth_internal.h -- entry points shared by the two halves of libkth.so
 * (kth_api.hip: kernels + ctx; kth_sharded.cpp: the multi-shard driver).
 * Hidden: not part of the C ABI of include/kth.h.
 */
#ifndef KTH_INTERNAL_H
#define KTH_INTERNAL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Shards one kth_sharded handle may place on ONE device (the local transport). */
#define KTH_LOCAL_MAX_SHARDS 64

/* The local transport's all-reduce: slot `slot` (0..2) of every shard's
 * 3 * KTH_STATS_WORDS stats words summed (uint64) and written back to each of
 * them, enqueued on `stream` (a hipStream_t of the device holding every
 * slots[i]).  1 <= P <= KTH_LOCAL_MAX_SHARDS. */
__attribute__((visibility("hidden"))) int kth_internal_slots_sum(uint64_t *const *slots, int P, int slot,
                                                                 void *stream);

/* The local transport's window: after kth_dist_window(src), the window state
 * copied to every dst[i] (ctxs of the same device, each bound by
 * kth_dist_begin and sampled), enqueued on src's stream, as if each had run
 * kth_dist_window on the same gathered sample.  Returns 1 (nothing done; run
 * kth_dist_window on each) when src's window was not a cooperative one. */
struct kth_ctx;
__attribute__((visibility("hidden"))) int kth_internal_dist_window_share(struct kth_ctx *src,
                                                                         struct kth_ctx *const *dst, int P);

/* Every ctxs[i]'s last [answer, error] words (k_dresult's d_status) to
 * d_dst[2 i], d_dst[2 i + 1] (device-visible host memory), enqueued on
 * `stream`; ctxs of one device. */
__attribute__((visibility("hidden"))) int kth_internal_status_gather(struct kth_ctx *const *ctxs, int P,
                                                                     int32_t *d_dst, void *stream);

/* The ctx's stream (its own, or the one kth_ctx_set_stream gave it). */
__attribute__((visibility("hidden"))) void *kth_internal_ctx_stream(const struct kth_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* KTH_INTERNAL_H */
