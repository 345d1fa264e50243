// kth_device.hpp -- device-side building blocks of the MI355X (gfx950) k-th
// selection engine: key transforms, the per-selection state machine, and the
// block-wide digit pick shared by every kernel in kth_kernels.hip.
//
// Protocol (no in-kernel inter-workgroup hand-off anywhere):
//   kernel l reads the state St[l-1] and the (all-reduced, for N GPUs) stats
//   slot written by kernel l-1, EVERY workgroup redundantly advances the state
//   (picks the digit from the reduced histogram), then accumulates its own
//   histogram / counts into the next slot with device-scope atomics.
//   Workgroup 0 publishes St[l] and zeroes the slot kernel l+1 will accumulate
//   into.  Visibility comes from kernel boundaries only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kth {

typedef unsigned long long u64;

constexpr int WAVE = 64;
constexpr int DIGIT = 11;              // radix digit width (bits)
constexpr int NBINS = 1 << DIGIT;      // 2048 bins per digit
constexpr int NCOUNTS = 8;             // words of counts ahead of the histograms
constexpr int STATS_WORDS = NCOUNTS + 2 * NBINS;  // == KTH_STATS_WORDS

// stats slot layout
enum : int { C_LT = 0, C_EQLO = 1, C_EQHI = 2, C_IN = 3, C_OVF = 4 };

// selection modes
enum : uint32_t {
    MODE_SAMPLE = 0,  // resolving the window ranks r_lo/r_hi on the sample
    MODE_MAIN = 1,    // window known; streaming pass pending / done
    MODE_CAND = 2,    // resolving rank k among the window's candidates
    MODE_FULL = 3,    // resolving rank k by radix passes over the whole input
    MODE_DONE = 4,
};

// how a kernel obtains its state
enum : int {
    ADV_INIT_SAMPLE = 0,  // fresh selection, window phase (targets r_lo, r_hi)
    ADV_INIT_FULL = 1,    // fresh selection, plain radix passes over the input
    ADV_PICK = 2,         // consume the previous digit's reduced histogram
    ADV_DECIDE = 3,       // consume the streaming pass's reduced counts
    ADV_CARRY = 4,        // take the previous kernel's state as is (it resolved its own digits)
};

struct Target {
    u64 k;            // remaining 1-based rank among keys matching `prefix`
    uint32_t prefix;  // resolved high `done` bits of v = key - base, right-aligned
    uint32_t done;    // resolved bit count (of W)
    uint32_t active;  // target in use
    uint32_t pad;
};

struct alignas(16) SelState {
    u64 n, k;          // global input size and rank
    u64 s;             // sample size (window phase)
    u64 cnt[5];        // reduced streaming-pass counts (lt, eq_lo, eq_hi, inside, ovf)
    Target t[2];
    uint32_t mode, W, base, lo, hi, answer, error, path;
    uint32_t share;    // target 1 reads target 0's histogram this level
    uint32_t d0;       // width of a domain's first digit (0: DIGIT)
    uint32_t dw;       // width of its later digits (0: DIGIT; the sharded protocol's digits: DDIG)
    uint32_t pad;
    u64 below, eqv;    // done: keys below the answer, keys equal to it (0 = unknown); kth_topk_i32
};

__device__ __forceinline__ uint32_t key_of_i32(uint32_t bits) { return bits ^ 0x80000000u; }
__device__ __forceinline__ int32_t i32_of_key(uint32_t key) { return (int32_t)(key ^ 0x80000000u); }

// IEEE-754 total order with every NaN mapped above +inf.
__device__ __forceinline__ uint32_t key_of_f32(uint32_t b) {
    if ((b & 0x7FFFFFFFu) > 0x7F800000u) return 0xFFFFFFFFu;
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ uint32_t f32_of_key(uint32_t key) {
    if (key == 0xFFFFFFFFu) return 0x7FC00000u;
    return (key & 0x80000000u) ? (key & 0x7FFFFFFFu) : ~key;
}

__device__ __forceinline__ uint32_t digit_bits(uint32_t W, uint32_t done) {
    uint32_t r = W - done;
    return r < (uint32_t)DIGIT ? r : (uint32_t)DIGIT;
}
// the next digit of a selection state: the first one may be narrower (d0),
// the later ones are dw wide (DIGIT unless set)
__device__ __forceinline__ uint32_t digit_bits(const SelState &s, uint32_t done) {
    const uint32_t r = s.W - done, d = (done == 0 && s.d0) ? s.d0 : (s.dw ? s.dw : (uint32_t)DIGIT);
    return r < d ? r : d;
}

// does v (= key - base) match target's resolved prefix?
__device__ __forceinline__ bool prefix_match(uint32_t v, uint32_t W, uint32_t done, uint32_t prefix) {
    return done == 0 || (v >> (W - done)) == prefix;
}

// ---------------------------------------------------------------- block scan
// Exclusive prefix sum of one u64 per thread across a block of BLOCK threads.
// `wsum` is LDS scratch of BLOCK/64 words.  All threads must call.
template <int BLOCK>
__device__ __forceinline__ u64 block_exclusive_scan(u64 x, u64 *wsum, u64 *total) {
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    u64 inc = x;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        u64 y = __shfl_up(inc, o, WAVE);
        if (lane >= o) inc += y;
    }
    if (lane == WAVE - 1) wsum[wid] = inc;
    __syncthreads();
    u64 before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / WAVE; ++w) {
        u64 s = wsum[w];
        before += (w < wid) ? s : 0;
        all += s;
    }
    __syncthreads();
    if (total) *total = all;
    return before + inc - x;
}

// Find the bin holding the k-th (1-based) key of a histogram of nb bins
// (nb <= 2048).  hist(i) returns bin i's count.  Block-wide; returns true and
// (bin, keys below bin) in *out_bin / *out_below on every thread, or false if
// the histogram holds fewer than k keys.
template <int BLOCK, typename H>
__device__ bool block_pick(H hist, int nb, u64 k, uint32_t *out_bin, u64 *out_below, u64 *scratch) {
    // scratch: BLOCK/64 words for the scan + 3 words of result
    const int per = (nb + BLOCK - 1) / BLOCK;
    const int b0 = threadIdx.x * per;
    u64 sum = 0;
    for (int j = 0; j < per; ++j) {
        int b = b0 + j;
        if (b < nb) sum += hist(b);
    }
    u64 total;
    u64 pre = block_exclusive_scan<BLOCK>(sum, scratch, &total);
    u64 *res = scratch + BLOCK / WAVE;
    if (threadIdx.x == 0) res[0] = 0;
    __syncthreads();
    if (k >= 1 && k > pre && k <= pre + sum) {
        u64 cum = pre;
        for (int j = 0; j < per; ++j) {
            int b = b0 + j;
            u64 h = hist(b);
            if (cum + h >= k) {
                res[0] = 1;
                res[1] = (u64)b;
                res[2] = cum;
                break;
            }
            cum += h;
        }
    }
    __syncthreads();
    bool ok = res[0] != 0;
    *out_bin = (uint32_t)res[1];
    *out_below = res[2];
    __syncthreads();
    return ok;
}


// block_pick over values the caller already holds: thread t owns bins
// [t*PER, t*PER + PER) of an (NB = BLOCK*PER)-bin histogram.  Lets a kernel
// issue its histogram loads together with its other loads.
template <int BLOCK, int PER>
__device__ bool block_pick_vals(const u64 (&h)[PER], u64 k, uint32_t *out_bin, u64 *out_below, u64 *scratch) {
    u64 sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) sum += h[j];
    u64 total;
    const u64 pre = block_exclusive_scan<BLOCK>(sum, scratch, &total);
    u64 *res = scratch + BLOCK / WAVE;
    if (threadIdx.x == 0) res[0] = 0;
    __syncthreads();
    if (k >= 1 && k > pre && k <= pre + sum) {
        u64 cum = pre;
        bool found = false;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            if (!found && cum + h[j] >= k) {
                res[0] = 1;
                res[1] = (u64)(threadIdx.x * PER + j);
                res[2] = cum;
                found = true;
            }
            cum += h[j];
        }
    }
    __syncthreads();
    const bool ok = res[0] != 0;
    *out_bin = (uint32_t)res[1];
    *out_below = res[2];
    __syncthreads();
    return ok;
}


// ------------------------------------------------------ two-target block pick
// DPP row shifts / broadcasts: a u64 moves as two dwords and is added with a
// carry, so the scans need no LDS round trip and no per-lane addresses.
template <int CTRL, int ROWS>
__device__ __forceinline__ u64 dpp64(u64 x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, ROWS, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, ROWS, 0xF, false);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 wave_incl_scan64(u64 x) {
    x += dpp64<0x111, 0xF>(x);  // row_shr:1
    x += dpp64<0x112, 0xF>(x);  // row_shr:2
    x += dpp64<0x114, 0xF>(x);  // row_shr:4
    x += dpp64<0x118, 0xF>(x);  // row_shr:8
    x += dpp64<0x142, 0xA>(x);  // row_bcast:15
    x += dpp64<0x143, 0xC>(x);  // row_bcast:31
    return x;
}

template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
    x += dpp32<0x111, 0xF>(x);  // row_shr:1
    x += dpp32<0x112, 0xF>(x);  // row_shr:2
    x += dpp32<0x114, 0xF>(x);  // row_shr:4
    x += dpp32<0x118, 0xF>(x);  // row_shr:8
    x += dpp32<0x142, 0xA>(x);  // row_bcast:15
    x += dpp32<0x143, 0xC>(x);  // row_bcast:31
    return x;
}

// block_pick_vals for two targets at once (target t's histogram in h[t],
// thread i owning bins [i*PER, i*PER + PER)): one wave scan per target, both
// chains interleaved, and two barriers in all.  want[t] = false skips target
// t (its outputs are then unspecified).  ok[t] false if the histogram holds
// fewer than k[t] keys; cnt[t] = keys in the picked bin.  `scratch` holds
// 2 * (BLOCK/64) + 8 words.
template <int BLOCK, int PER>
__device__ void block_pick2(const u64 (&h0)[PER], const u64 (&h1)[PER], const bool want[2], const u64 k[2],
                            uint32_t bin[2], u64 below[2], bool ok[2], u64 *scratch, u64 cnt[2]) {
    constexpr int NW = BLOCK / WAVE;
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    u64 sum0 = 0, sum1 = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        sum0 += h0[j];
        sum1 += h1[j];
    }
    const u64 inc0 = wave_incl_scan64(sum0), inc1 = wave_incl_scan64(sum1);
    u64 *wsum = scratch, *res = scratch + 2 * NW;
    if (lane == WAVE - 1) {
        wsum[wid] = inc0;
        wsum[NW + wid] = inc1;
    }
    if (threadIdx.x < 8) res[threadIdx.x] = 0;
    __syncthreads();
    u64 pre0 = inc0 - sum0, pre1 = inc1 - sum1;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        if (w < wid) {
            pre0 += wsum[w];
            pre1 += wsum[NW + w];
        }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const u64 kt = k[t], pre = t ? pre1 : pre0, sum = t ? sum1 : sum0;
        if (want[t] && kt >= 1 && kt > pre && kt <= pre + sum) {  // exactly one thread
            u64 cum = pre;
            bool found = false;
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                const u64 hj = t ? h1[j] : h0[j];
                if (!found && cum + hj >= kt) {
                    res[4 * t + 0] = 1;
                    res[4 * t + 1] = (u64)(threadIdx.x * PER + j);
                    res[4 * t + 2] = cum;
                    res[4 * t + 3] = hj;
                    found = true;
                }
                cum += hj;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        ok[t] = res[4 * t] != 0;
        bin[t] = (uint32_t)res[4 * t + 1];
        below[t] = res[4 * t + 2];
        cnt[t] = res[4 * t + 3];
    }
}

}  // namespace kth
