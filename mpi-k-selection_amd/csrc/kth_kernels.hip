// kth_kernels.hip -- MI355X (gfx950, CDNA4) kernels of the exact k-th selection
// engine.  Pure HBM-streaming integer work: no MFMA anywhere.
//
// Paths (host side in kth_api.hip chooses):
//   LDS     n <= 16384: one 1024-thread workgroup, keys resident in LDS, three
//           11-bit radix levels in LDS (k_small).
//   RADIX   n <= 4M: radix levels over the input (k_level x3 + k_result).
//   WINDOW  larger n: k_gather samples 2^20 keys in 64-key chunks and builds the
//           first histogram -> two k_level passes resolve the sample ranks
//           r_lo / r_hi (window [lo, hi]) -> k_main streams the input ONCE:
//           counts #<lo, #==lo, #==hi and compacts keys strictly inside the
//           window (LDS-staged, one global reservation per workgroup) ->
//           k_level decides: answer is lo or hi, or among the candidates
//           (radix levels over the compacted buffer), or the window missed
//           (radix levels over the input) -> k_result.
// Replaces the CGM rounds of TODO-kth-problem-cgm.c:122-233 (local median,
// weighted median, 3-way count, discard) and the final solve :235-278; and the
// qsort + VecGet of kth-problem-seq.c:32-33.
#include "kth_device.hpp"

namespace kth {

constexpr int BLK = 256;
constexpr int MAIN_UNROLL = 4;
constexpr int LBUF = 4096;            // per-workgroup candidate staging (16 KiB LDS)
constexpr u64 LEVEL_MIN_PER_WG = 1ull << 14;
constexpr int SAMPLE_CHUNK = 64;      // keys per sampled chunk = one wave's 256-B load
constexpr int SMALL_BLOCK = 1024;
constexpr int ROWS_BLOCK = 256;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16-byte streaming load that does not allocate in the caches.
__device__ __forceinline__ uint4 load_nt(const uint4 *p) {
    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
}

struct StepArgs {
    const SelState *st_in;
    SelState *st_out;
    const u64 *stats_in;   // reduced stats consumed by the advance
    u64 *stats_acc;        // stats accumulated by this kernel
    u64 *stats_zero;       // slot the NEXT kernel accumulates into (zeroed by WG 0)
    const uint32_t *sample;
    u64 sample_count;
    const uint32_t *cand;
    u64 *cand_count;       // local candidate count (not reduced)
    u64 cap;
    const int32_t *keys;
    u64 n_local;
    int adv;
    u64 init_n, init_k, init_s, r_lo, r_hi;
};

// ------------------------------------------------------------- the advance
__device__ __forceinline__ void resolve(SelState &s) {
    if (s.mode == MODE_SAMPLE) {
        const bool r0 = !s.t[0].active || s.t[0].done == s.W;
        const bool r1 = !s.t[1].active || s.t[1].done == s.W;
        if (r0 && r1) {
            s.lo = s.t[0].active ? s.base + s.t[0].prefix : 0u;
            s.hi = s.t[1].active ? s.base + s.t[1].prefix : 0xFFFFFFFFu;
            s.mode = MODE_MAIN;
        }
    } else if (s.mode == MODE_CAND || s.mode == MODE_FULL) {
        if (s.t[0].done == s.W) {
            s.answer = s.base + s.t[0].prefix;
            s.mode = MODE_DONE;
        }
    }
}

// Streaming-pass counts -> next mode.  Exact: the answer is lo iff
// #<lo < k <= #<lo + #==lo, and so on up the window.
__device__ __forceinline__ void decide(SelState &s, const u64 *c) {
    const u64 L = c[C_LT], E1 = c[C_EQLO], M = c[C_IN], ovf = c[C_OVF];
    const u64 E2 = (s.lo == s.hi) ? 0 : c[C_EQHI];
    for (int i = 0; i < 5; ++i) s.cnt[i] = c[i];
    const u64 k = s.k;
    s.t[1].active = 0;
    s.t[0] = Target{k, 0, 0, 1, 0};
    s.path = 3;  // KTH_PATH_WINDOW
    if (k > L && k <= L + E1) {
        s.answer = s.lo;
        s.mode = MODE_DONE;
    } else if (k > L + E1 && k <= L + E1 + M && ovf == 0) {
        s.base = s.lo + 1u;
        const uint32_t range = s.hi - s.lo - 2u;  // candidates lie in [base, base + range]
        s.W = range ? 32u - (uint32_t)__clz(range) : 0u;
        s.t[0].k = k - L - E1;
        s.mode = MODE_CAND;
        if (s.W == 0) {
            s.answer = s.base;
            s.mode = MODE_DONE;
        }
    } else if (k > L + E1 + M && k <= L + E1 + M + E2) {
        s.answer = s.hi;
        s.mode = MODE_DONE;
    } else {
        s.mode = MODE_FULL;
        s.W = 32;
        s.base = 0;
        s.path = 4;  // KTH_PATH_WINDOW_FALLBACK
    }
}

template <int BLOCK>
__device__ void advance(SelState &ss, const StepArgs &a, u64 *scratch) {
    if (threadIdx.x == 0) {
        if (a.adv == ADV_INIT_SAMPLE || a.adv == ADV_INIT_FULL) {
            SelState s;
            memset(&s, 0, sizeof s);
            s.n = a.init_n;
            s.k = a.init_k;
            s.s = a.init_s;
            s.W = 32;
            s.base = 0;
            s.lo = 0;
            s.hi = 0xFFFFFFFFu;
            if (a.adv == ADV_INIT_SAMPLE) {
                s.mode = MODE_SAMPLE;
                s.path = 3;
                s.t[0] = Target{a.r_lo, 0, 0, (a.r_lo >= 1 && a.r_lo <= a.init_s) ? 1u : 0u, 0};
                s.t[1] = Target{a.r_hi, 0, 0, (a.r_hi >= 1 && a.r_hi <= a.init_s) ? 1u : 0u, 0};
                resolve(s);
            } else {
                s.mode = MODE_FULL;
                s.path = 2;
                s.t[0] = Target{a.init_k, 0, 0, 1, 0};
            }
            ss = s;
        } else {
            ss = *a.st_in;
        }
    }
    __syncthreads();
    if (a.adv == ADV_DECIDE) {
        if (threadIdx.x == 0 && ss.mode == MODE_MAIN) decide(ss, a.stats_in);
        __syncthreads();
    } else if (a.adv == ADV_PICK) {
        for (int t = 0; t < 2; ++t) {
            const uint32_t mode = ss.mode;
            const bool need = (mode == MODE_SAMPLE || mode == MODE_CAND || mode == MODE_FULL) &&
                              ss.t[t].active && ss.t[t].done < ss.W;
            if (!need) continue;  // block-uniform: read from LDS after a barrier
            const uint32_t d = digit_bits(ss.W, ss.t[t].done);
            const int src = (t == 1 && ss.share) ? 0 : t;
            const u64 *h = a.stats_in + NCOUNTS + src * NBINS;
            uint32_t bin;
            u64 below;
            const bool ok = block_pick<BLOCK>([&](int i) { return h[i]; }, 1 << d, ss.t[t].k, &bin, &below, scratch);
            if (threadIdx.x == 0) {
                if (!ok) {
                    ss.error = 1 + t;
                    ss.mode = MODE_DONE;
                } else {
                    ss.t[t].k -= below;
                    ss.t[t].prefix = (ss.t[t].prefix << d) | bin;
                    ss.t[t].done += d;
                }
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) resolve(ss);
        __syncthreads();
    }
}

// ----------------------------------------------------------------- streaming
// Visit n 32-bit words at p (4-byte aligned) as keys, f(key, valid).  Calls
// are wave-convergent (every lane calls f the same number of times; `valid`
// masks the lanes past the end), so f may use ballots.  Block-contiguous tiles
// of BLOCK * UNROLL 16-byte vectors, grid-strided.  XOR flips the sign bit
// (int32 -> order-preserving uint32).
template <int BLOCK, int UNROLL, bool XOR, typename F>
__device__ __forceinline__ void stream_keys(const uint32_t *__restrict__ p, u64 n, uint32_t wg, uint32_t nwg,
                                            F &&f) {
    const uint32_t X = XOR ? 0x80000000u : 0u;
    const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
    u64 head = ((16u - (uint32_t)(addr & 15u)) & 15u) >> 2;
    if (head > n) head = n;
    const uint4 *__restrict__ v = reinterpret_cast<const uint4 *>(p + head);
    const u64 nv = (n - head) >> 2;
    const u64 tail0 = head + (nv << 2);
    const u64 tile = (u64)BLOCK * UNROLL;
    for (u64 t0 = (u64)wg * tile; t0 < nv; t0 += (u64)nwg * tile) {
        uint4 x[UNROLL];
        if (t0 + tile <= nv) {
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) x[u] = load_nt(&v[t0 + u * BLOCK + threadIdx.x]);
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                f(x[u].x ^ X, true);
                f(x[u].y ^ X, true);
                f(x[u].z ^ X, true);
                f(x[u].w ^ X, true);
            }
        } else {
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const u64 i = t0 + u * BLOCK + threadIdx.x;
                const bool ok = i < nv;
                x[u] = ok ? v[i] : make_uint4(0, 0, 0, 0);
                f(x[u].x ^ X, ok);
                f(x[u].y ^ X, ok);
                f(x[u].z ^ X, ok);
                f(x[u].w ^ X, ok);
            }
        }
    }
    if (wg == 0) {  // ragged head and tail: < 4 keys each
        const u64 j = threadIdx.x;
        const bool okh = j < head, okt = j < n - tail0;
        const uint32_t xh = okh ? p[j] : 0u, xt = okt ? p[tail0 + j] : 0u;
        f(xh ^ X, okh);
        f(xt ^ X, okt);
    }
}

// -------------------------------------------------------------- histograms
struct HistPlan {
    bool h[2];
    uint32_t W, base, shift[2], mask[2], done[2], prefix[2];
};

__device__ __forceinline__ HistPlan make_plan(const SelState &ss, bool *share) {
    HistPlan p;
    const uint32_t mode = ss.mode;
    const bool live = mode == MODE_SAMPLE || mode == MODE_CAND || mode == MODE_FULL;
    p.W = ss.W;
    p.base = ss.base;
    for (int t = 0; t < 2; ++t) {
        p.h[t] = live && ss.t[t].active && ss.t[t].done < ss.W;
        const uint32_t d = p.h[t] ? digit_bits(ss.W, ss.t[t].done) : 0u;
        p.done[t] = ss.t[t].done;
        p.prefix[t] = ss.t[t].prefix;
        p.shift[t] = p.h[t] ? ss.W - ss.t[t].done - d : 0u;
        p.mask[t] = (1u << d) - 1u;
    }
    *share = p.h[0] && p.h[1] && p.done[0] == p.done[1] && p.prefix[0] == p.prefix[1];
    if (*share) p.h[1] = false;
    return p;
}

template <int BLOCK>
__device__ __forceinline__ void hist_add(uint32_t (*lh)[NBINS], const HistPlan &p, uint32_t key, bool ok) {
    const uint32_t v = key - p.base;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        if (p.h[t] && ok && prefix_match(v, p.W, p.done[t], p.prefix[t]))
            atomicAdd(&lh[t][(v >> p.shift[t]) & p.mask[t]], 1u);
    }
}

template <int BLOCK>
__device__ __forceinline__ void hist_flush(uint32_t (*lh)[NBINS], const HistPlan &p, u64 *acc) {
    __syncthreads();
    for (int t = 0; t < 2; ++t) {
        if (!p.h[t]) continue;
        for (uint32_t b = threadIdx.x; b <= p.mask[t]; b += BLOCK) {
            const uint32_t c = lh[t][b];
            if (c) atomicAdd(&acc[NCOUNTS + t * NBINS + b], (u64)c);
        }
    }
}

template <int BLOCK>
__device__ __forceinline__ void publish(const SelState &ss, uint32_t share, const StepArgs &a) {
    if (blockIdx.x != 0) return;
    if (threadIdx.x == 0) {
        SelState o = ss;
        o.share = share;
        *a.st_out = o;
    }
    if (a.stats_zero)
        for (int i = threadIdx.x; i < STATS_WORDS; i += BLOCK) a.stats_zero[i] = 0;
}

// =================================================================== kernels

// One radix level: advance, then histogram the next digit of every
// unresolved target over the current domain (sample / candidates / input).
__global__ __launch_bounds__(BLK) void k_level(StepArgs a) {
    __shared__ SelState ss;
    __shared__ u64 scratch[BLK / WAVE + 4];
    __shared__ uint32_t lh[2][NBINS];
    advance<BLK>(ss, a, scratch);
    bool share;
    const HistPlan plan = make_plan(ss, &share);
    const uint32_t mode = ss.mode;
    u64 count = 0;
    if (plan.h[0] || plan.h[1]) {
        if (mode == MODE_SAMPLE) count = a.sample_count;
        else if (mode == MODE_CAND) count = min(*a.cand_count, a.cap);
        else if (mode == MODE_FULL) count = a.n_local;
    }
    publish<BLK>(ss, share, a);
    const u64 want = (count + LEVEL_MIN_PER_WG - 1) / LEVEL_MIN_PER_WG;
    const uint32_t active = (uint32_t)min((u64)gridDim.x, want);
    if (blockIdx.x >= active) return;
    for (int i = threadIdx.x; i < 2 * NBINS; i += BLK) (&lh[0][0])[i] = 0;
    __syncthreads();
    auto f = [&](uint32_t key, bool ok) { hist_add<BLK>(lh, plan, key, ok); };
    if (mode == MODE_FULL)
        stream_keys<BLK, 4, true>(reinterpret_cast<const uint32_t *>(a.keys), count, blockIdx.x, active, f);
    else
        stream_keys<BLK, 4, false>(mode == MODE_SAMPLE ? a.sample : a.cand, count, blockIdx.x, active, f);
    hist_flush<BLK>(lh, plan, a.stats_acc);
}

// Sample gather: s keys in chunks of 64 contiguous keys spread evenly over the
// shard (stride = chunk distance in keys).  With FUSE the first digit's
// histogram of the sample is built too (single-GPU: the sample is complete).
template <bool FUSE>
__global__ __launch_bounds__(BLK) void k_gather(StepArgs a, const int32_t *__restrict__ keys, u64 stride,
                                                uint32_t *__restrict__ sample, u64 s) {
    __shared__ SelState ss;
    __shared__ u64 scratch[BLK / WAVE + 4];
    __shared__ uint32_t lh[2][NBINS];
    HistPlan plan;
    bool share = false;
    if (FUSE) {
        advance<BLK>(ss, a, scratch);
        plan = make_plan(ss, &share);
        publish<BLK>(ss, share, a);
        for (int i = threadIdx.x; i < 2 * NBINS; i += BLK) (&lh[0][0])[i] = 0;
        __syncthreads();
    }
    const int lane = threadIdx.x & (WAVE - 1);
    const u64 nchunks = s / SAMPLE_CHUNK;
    const u64 gw = ((u64)blockIdx.x * BLK + threadIdx.x) / WAVE, nw = (u64)gridDim.x * (BLK / WAVE);
    for (u64 c = gw; c < nchunks; c += nw) {
        const uint32_t key = key_of_i32((uint32_t)keys[c * stride + lane]);
        sample[c * SAMPLE_CHUNK + lane] = key;
        if (FUSE) hist_add<BLK>(lh, plan, key, true);
    }
    if (FUSE) hist_flush<BLK>(lh, plan, a.stats_acc);
}

// The streaming pass.  Window [lo, hi] comes from the advance (last sample
// digit).  Per key: #<lo, #==lo, #==hi in registers; keys strictly inside the
// window are compacted through an LDS buffer (one LDS atomic per wave-key
// group that has any, one global reservation per workgroup).
__global__ __launch_bounds__(BLK) void k_main(StepArgs a, uint32_t *__restrict__ cand_out) {
    __shared__ SelState ss;
    __shared__ u64 scratch[BLK / WAVE + 4];
    __shared__ uint32_t lbuf[LBUF];
    __shared__ uint32_t lcount;
    __shared__ u64 red[3][BLK / WAVE];
    __shared__ u64 gbase;
    advance<BLK>(ss, a, scratch);
    publish<BLK>(ss, 0, a);
    if (ss.mode != MODE_MAIN) return;  // block-uniform (error or resolved)
    const uint32_t lo = ss.lo, hi = ss.hi;
    const u64 cap = a.cap;
    u64 *const cand_count = a.cand_count;
    u64 *const acc = a.stats_acc;
    if (threadIdx.x == 0) lcount = 0;
    __syncthreads();
    const int lane = threadIdx.x & (WAVE - 1);
    uint32_t clt = 0, ceqlo = 0, ceqhi = 0;
    stream_keys<BLK, MAIN_UNROLL, true>(
        reinterpret_cast<const uint32_t *>(a.keys), a.n_local, blockIdx.x, gridDim.x, [&](uint32_t u, bool ok) {
            clt += (ok & (u < lo)) ? 1u : 0u;
            ceqlo += (ok & (u == lo)) ? 1u : 0u;
            ceqhi += (ok & (u == hi)) ? 1u : 0u;
            const bool in = ok & (u > lo) & (u < hi);
            const u64 m = __ballot(in);
            if (m) {
                const uint32_t cnt = (uint32_t)__popcll(m);
                const uint32_t rank =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                const int leader = __ffsll((long long)m) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(&lcount, cnt);
                base = __shfl(base, leader, WAVE);
                const uint32_t pos = base + rank;
                if (in && pos < LBUF) lbuf[pos] = u;
                if (base + cnt > LBUF) {  // staging full: this group goes straight to HBM
                    const bool spill = in && pos >= LBUF;
                    const u64 ms = __ballot(spill);
                    const uint32_t cs = (uint32_t)__popcll(ms);
                    const uint32_t rs =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(ms >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ms, 0u));
                    const int l2 = __ffsll((long long)ms) - 1;
                    u64 g = 0;
                    if (lane == l2) {
                        g = atomicAdd(cand_count, (u64)cs);
                        if (g <= cap && g + cs > cap) atomicAdd(&acc[C_OVF], 1ull);
                    }
                    g = __shfl(g, l2, WAVE);
                    if (spill && g + rs < cap) cand_out[g + rs] = u;
                }
            }
        });
    // counts: wave reduce -> LDS -> one atomic per workgroup
    u64 r0 = clt, r1 = ceqlo, r2 = ceqhi;
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) {
        r0 += __shfl_xor(r0, o, WAVE);
        r1 += __shfl_xor(r1, o, WAVE);
        r2 += __shfl_xor(r2, o, WAVE);
    }
    const int wid = threadIdx.x / WAVE;
    if (lane == 0) {
        red[0][wid] = r0;
        red[1][wid] = r1;
        red[2][wid] = r2;
    }
    __syncthreads();
    const uint32_t total = lcount;
    const uint32_t nl = total < (uint32_t)LBUF ? total : (uint32_t)LBUF;
    if (threadIdx.x == 0) {
        u64 s0 = 0, s1 = 0, s2 = 0;
        for (int w = 0; w < BLK / WAVE; ++w) {
            s0 += red[0][w];
            s1 += red[1][w];
            s2 += red[2][w];
        }
        if (s0) atomicAdd(&acc[C_LT], s0);
        if (s1) atomicAdd(&acc[C_EQLO], s1);
        if (s2) atomicAdd(&acc[C_EQHI], s2);
        if (total) atomicAdd(&acc[C_IN], (u64)total);
        u64 g = 0;
        if (nl) {
            g = atomicAdd(cand_count, (u64)nl);
            if (g <= cap && g + nl > cap) atomicAdd(&acc[C_OVF], 1ull);
        }
        gbase = g;
    }
    __syncthreads();
    const u64 g = gbase;
    for (uint32_t i = threadIdx.x; i < nl; i += BLK)
        if (g + i < cap) cand_out[g + i] = lbuf[i];
}

// Final digit: one workgroup.  Writes the answer and the error word, then
// zeroes the ctx-internal slots (and local candidate count) for the next call.
__global__ __launch_bounds__(BLK) void k_result(StepArgs a, int32_t *d_out, int32_t *d_status, u64 *izero,
                                                u64 izero_words) {
    __shared__ SelState ss;
    __shared__ u64 scratch[BLK / WAVE + 4];
    advance<BLK>(ss, a, scratch);
    if (threadIdx.x == 0) {
        SelState o = ss;
        if (o.mode != MODE_DONE && !o.error) o.error = 16 + o.mode;
        *a.st_out = o;
        if (d_out) *d_out = i32_of_key(o.answer);
        if (d_status) {
            d_status[0] = i32_of_key(o.answer);
            d_status[1] = (int32_t)o.error;
        }
    }
    __syncthreads();
    for (u64 i = threadIdx.x; i < izero_words; i += BLK) izero[i] = 0;
}

// n <= 16384: whole selection in one workgroup, keys in LDS.
__global__ __launch_bounds__(SMALL_BLOCK) void k_small(const int32_t *__restrict__ keys, u64 n, u64 k,
                                                       int32_t *d_out, int32_t *d_status, SelState *st_out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t skeys[];
    __shared__ uint32_t hist[NBINS];
    __shared__ u64 scratch[SMALL_BLOCK / WAVE + 4];
    for (u64 i = threadIdx.x; i < n; i += SMALL_BLOCK) skeys[i] = key_of_i32((uint32_t)keys[i]);
    uint32_t prefix = 0, done = 0;
    u64 kk = k;
    bool ok = true;
    while (done < 32) {
        const uint32_t d = digit_bits(32, done), shift = 32 - done - d, mask = (1u << d) - 1u;
        for (int i = threadIdx.x; i < NBINS; i += SMALL_BLOCK) hist[i] = 0;
        __syncthreads();
        for (u64 i = threadIdx.x; i < n; i += SMALL_BLOCK) {
            const uint32_t v = skeys[i];
            if (prefix_match(v, 32, done, prefix)) atomicAdd(&hist[(v >> shift) & mask], 1u);
        }
        __syncthreads();
        uint32_t bin;
        u64 below;
        ok = block_pick<SMALL_BLOCK>([&](int i) { return (u64)hist[i]; }, 1 << d, kk, &bin, &below, scratch);
        if (!ok) break;
        kk -= below;
        prefix = (prefix << d) | bin;
        done += d;
    }
    if (threadIdx.x == 0) {
        if (d_out) d_out[0] = i32_of_key(prefix);
        if (d_status) {
            d_status[0] = i32_of_key(prefix);
            d_status[1] = ok ? 0 : 1;
        }
        if (st_out) {
            SelState o;
            memset(&o, 0, sizeof o);
            o.n = n;
            o.k = k;
            o.mode = MODE_DONE;
            o.W = 32;
            o.answer = prefix;
            o.error = ok ? 0 : 1;
            o.path = 1;  // KTH_PATH_LDS
            o.hi = 0xFFFFFFFFu;
            *st_out = o;
        }
    }
}

// Batched rows: one workgroup per row, row resident in LDS; F32 selects the
// float total-order key transform.  Grid-strided over rows.
template <bool F32>
__global__ __launch_bounds__(ROWS_BLOCK) void k_rows(const uint32_t *__restrict__ m, u64 rows, uint32_t cols, u64 k,
                                                     uint32_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t rk[];
    __shared__ uint32_t hist[NBINS];
    __shared__ u64 scratch[ROWS_BLOCK / WAVE + 4];
    for (u64 r = blockIdx.x; r < rows; r += gridDim.x) {
        const uint32_t *row = m + r * (u64)cols;
        const bool vec = ((reinterpret_cast<uintptr_t>(row) & 15u) == 0) && (cols % 4 == 0);
        if (vec) {
            const uint4 *rv = reinterpret_cast<const uint4 *>(row);
            for (uint32_t i = threadIdx.x; i < cols / 4; i += ROWS_BLOCK) {
                uint4 x = load_nt(&rv[i]);
                uint4 y;
                y.x = F32 ? key_of_f32(x.x) : key_of_i32(x.x);
                y.y = F32 ? key_of_f32(x.y) : key_of_i32(x.y);
                y.z = F32 ? key_of_f32(x.z) : key_of_i32(x.z);
                y.w = F32 ? key_of_f32(x.w) : key_of_i32(x.w);
                reinterpret_cast<uint4 *>(rk)[i] = y;
            }
        } else {
            for (uint32_t i = threadIdx.x; i < cols; i += ROWS_BLOCK)
                rk[i] = F32 ? key_of_f32(row[i]) : key_of_i32(row[i]);
        }
        uint32_t prefix = 0, done = 0;
        u64 kk = k;
        while (done < 32) {
            const uint32_t d = digit_bits(32, done), shift = 32 - done - d, mask = (1u << d) - 1u;
            for (int i = threadIdx.x; i < NBINS; i += ROWS_BLOCK) hist[i] = 0;
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < cols; i += ROWS_BLOCK) {
                const uint32_t v = rk[i];
                if (prefix_match(v, 32, done, prefix)) atomicAdd(&hist[(v >> shift) & mask], 1u);
            }
            __syncthreads();
            uint32_t bin;
            u64 below;
            if (!block_pick<ROWS_BLOCK>([&](int i) { return (u64)hist[i]; }, 1 << d, kk, &bin, &below, scratch))
                break;
            kk -= below;
            prefix = (prefix << d) | bin;
            done += d;
        }
        if (threadIdx.x == 0) out[r] = F32 ? f32_of_key(prefix) : (uint32_t)i32_of_key(prefix);
        __syncthreads();
    }
}

// Counter-based synthetic keys; bit-identical to ko_gen (oracle/kth_oracle.c)
// and tests/golden/gen.py.
__device__ __forceinline__ u64 splitmix(u64 seed, u64 i) {
    u64 z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(BLK) void k_fill(int32_t *__restrict__ out, u64 n, u64 offset, uint32_t step, int dist,
                                              u64 seed, int32_t param) {
    const int32_t few[4] = {-5, 0, 7, 123456789};
    for (u64 j = (u64)blockIdx.x * BLK + threadIdx.x; j < n; j += (u64)gridDim.x * BLK) {
        const u64 i = offset + j;
        const u64 h = splitmix(seed, i);
        const uint32_t hi = (uint32_t)(h >> 32);
        int32_t v;
        switch (dist) {
        case 0: v = (int32_t)hi; break;
        case 1: v = ((int32_t)hi) >> 1; break;
        case 2: v = (int32_t)(hi % 99999999u) + 1; break;
        case 3: v = param; break;
        case 4: v = few[h >> 62]; break;
        case 5: v = (int32_t)(0x80000000u + (uint32_t)i * step); break;
        case 6: v = (int32_t)(0x7FFFFFFFu - (uint32_t)i * step); break;
        case 7: v = (int32_t)(hi % 1000u); break;
        default: v = 0; break;
        }
        out[j] = v;
    }
}

}  // namespace kth
