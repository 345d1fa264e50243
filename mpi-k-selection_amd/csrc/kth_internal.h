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

#ifdef __cplusplus
}
#endif
#endif /* KTH_INTERNAL_H */
