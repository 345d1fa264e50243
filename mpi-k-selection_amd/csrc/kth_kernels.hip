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
#include <type_traits>

#include "kth_device.hpp"
#include "kth_gridbar.hpp"

namespace kth {

#define KTH_STR2(x) #x
#define KTH_STR(x) KTH_STR2(x)
constexpr int BLK = 256;
#ifndef KTH_MAIN_UNROLL
#define KTH_MAIN_UNROLL 8
#endif
constexpr int MAIN_UNROLL = KTH_MAIN_UNROLL;  // 16-B loads in flight per thread in k_main (multiple of 8)
constexpr int MAIN_SUB = MAIN_UNROLL < 8 ? MAIN_UNROLL : 8;  // loads per scanned key group
#ifndef KTH_WREG
#define KTH_WREG 2048
#endif
constexpr int WREG = KTH_WREG;        // per-wave candidate staging region (words of LDS)
#ifndef KTH_WREG5
#define KTH_WREG5 2496
#endif
// k_main<5/6>'s per-wave region (the ordered staging of the top-k): as large as
// 4 workgroups a CU allow (40432 of 40960 B of LDS each).  Every flush of a
// region costs the streaming wave the wait for its stores, so fewer, larger
// flushes: 1984 entries instead of 1600, k_main<5> at k = 2^26 968-975 ->
// 947 us, whole calls -1.5 % (2^24 -1 %; profiles/r6_topk_seg_store_ab.txt)
constexpr int WREG5 = KTH_WREG5;
constexpr int LEVEL_UNROLL = 8;       // 16-B loads in flight per thread in k_level
constexpr int DENSE_BLK = 1024;       // workgroup size of the dense-histogram levels
#ifndef KTH_SAMPLE_CK
#define KTH_SAMPLE_CK 16
#endif
constexpr int SAMPLE_CK = KTH_SAMPLE_CK;            // sampled keys per lane per chunk (1, 4, 16, 64)
constexpr int SAMPLE_CHUNK = WAVE * SAMPLE_CK;      // keys per sampled chunk = one wave's load
constexpr int GATHER_BATCH = SAMPLE_CK < 16 ? 16 / SAMPLE_CK : 1;  // sampled chunks in flight per wave
constexpr int SMALL_BLOCK = 1024;
constexpr int ROWS_BLOCK = 256;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// 16-byte streaming load that does not allocate in the caches.
__device__ __forceinline__ uint4 load_nt(const uint4 *p) {
    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ uint32_t load_nt(const uint32_t *p) { return __builtin_nontemporal_load(p); }

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
    u64 min_per_wg;        // keys per active workgroup (sets how many WGs flush a histogram)
    u64 *stamps;           // KTH_STAMPS diagnostics: [gridDim.x][8] wall-clock stamps, else null
    u64 zero_words;        // k_gather<false> (sharded sample): clear stats_zero[0 .. zero_words)
    uint32_t *host_status; // k_dlevel, level 0 of the sharded protocol: DistStatus in host-visible memory
    uint32_t tag;          // ... with this tag (the host's call counter)
    u64 dense_per_wg;      // k_dlevel: keys per active workgroup for a domain's first digit
    uint32_t *pre_hist;    // k_main<0> (single-GPU window path): the candidates' first digit (PreHist), or null
};

// k_finish's first candidate digit: FIN_D0 bits ([513, 1024] bins used: ~6-12 K
// keys a bin from 6.3 M candidates at 2^30 -- the tail's one workgroup then
// resolves half the keys it did at 9 bits), wider only when W > 32 would need it
#ifndef KTH_FIN_D0
#define KTH_FIN_D0 10
#endif
constexpr uint32_t FIN_D0 = KTH_FIN_D0;
__host__ __device__ __forceinline__ uint32_t fin_first_digit(uint32_t W) {
    return W > FIN_D0 + 2u * DIGIT ? W - 2u * DIGIT : FIN_D0;  // (then two DIGIT-bit digits)
}

// The candidates' first digit, histogrammed by k_main<0> at the end of each
// workgroup from its waves' staging regions (every candidate of a workgroup
// is still there unless a wave had to flush its region mid-pass, which the
// workgroup then reports in `incomplete` instead), into PRE_COPIES copies
// (workgroup b adds to copy b % PRE_COPIES: 256 same-address adders a bin, not
// 1024, and they finish over the pass's ~80 us of workgroup end times).  k_finish picks the digit from it without a histogram pass, a flush
// or a grid barrier.  Two sets, alternate selects (k_finish clears the other).
#ifndef KTH_PRE_COPIES
#define KTH_PRE_COPIES 4
#endif
constexpr int PRE_COPIES = KTH_PRE_COPIES, PRE_BINS = 1024;  // a first digit of at most 10 bits (W <= 32)
static_assert(FIN_D0 <= 10, "PreHist holds a first digit of at most 10 bits");
constexpr int PRE_WORDS = PRE_COPIES * PRE_BINS + 64;  // u32: the copies, then `incomplete` (own 256-B line)
constexpr int PRE_INCOMPLETE = PRE_COPIES * PRE_BINS;
// the candidate domain of k_finish's decide(): v = key - (lo + 1) in [0, 2^W)
__device__ __forceinline__ uint32_t cand_width(uint32_t lo, uint32_t hi) {
    const uint32_t range = hi - lo - 2u;
    return range ? 32u - (uint32_t)__clz(range) : 0u;
}

// Diagnostic phase stamps (KTH_STAMPS=1 only; null pointer in the product):
// thread 0 of each workgroup records the 100 MHz wall clock at point i.
// Compiled in only with -DKTH_STAMPS_BUILD (tools' diagnostic variant): the
// runtime null check alone made every kernel wait for that kernel argument
// before issuing its first loads.
#ifdef KTH_STAMPS_BUILD
#define KTH_STAMP(a, i)                                                                          \
    do {                                                                                         \
        if ((a).stamps && threadIdx.x == 0)                                                      \
            (a).stamps[(u64)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();           \
    } while (0)
#else
#define KTH_STAMP(a, i) \
    do {                \
    } while (0)
#endif

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

// Early window (cooperative head only): once both window targets have picked
// a digit, the window may stop at the current digit resolution -- lo = lower
// edge of r_lo's bin, hi = upper edge of r_hi's bin -- when the sample keys
// inside those edges are within `slack64`/64 of the r_hi - r_lo + 1 the exact
// window holds.  Any [lo, hi] keeps decide() exact; this only trades a wider
// window (more candidates) for fewer sample levels.  A heavy-duplicate bin
// fails the test and keeps refining, down to exact sample keys.
struct EarlyWindow {
    u64 r_lo, r_hi;   // the sample ranks of the targets (0 / s+1: no bound)
    uint32_t slack64; // 0: off
    u64 abs_min;      // a span of up to this many sample keys is taken whatever the slack (0: none)
};

__device__ __forceinline__ void early_window(SelState &s, const EarlyWindow &e, u64 cnt1) {
    if (e.slack64 == 0 || s.mode != MODE_SAMPLE) return;
    const bool a0 = s.t[0].active, a1 = s.t[1].active;
    if ((a0 && s.t[0].done == 0) || (a1 && s.t[1].done == 0)) return;
    const u64 below0 = a0 ? e.r_lo - s.t[0].k : 0;           // sample keys under r_lo's bin
    const u64 upto1 = a1 ? e.r_hi - s.t[1].k + cnt1 : s.s;    // sample keys up to r_hi's bin's top
    const u64 want = (a1 ? e.r_hi : s.s) - (a0 ? e.r_lo : 1) + 1;
    if (upto1 < below0 || ((upto1 - below0) * 64 > want * (u64)e.slack64 && upto1 - below0 > e.abs_min)) return;
    const uint32_t w0 = s.W - s.t[0].done, w1 = s.W - s.t[1].done;
    s.lo = a0 ? s.base + (w0 >= 32 ? 0u : s.t[0].prefix << w0) : 0u;
    s.hi = a1 ? s.base + (w1 >= 32 ? 0xFFFFFFFFu : (s.t[1].prefix << w1) | ((1u << w1) - 1u)) : 0xFFFFFFFFu;
    s.mode = MODE_MAIN;
}

// Pick every live target's next digit from a histogram the caller holds in
// registers (thread i owns bins [i*PER, i*PER + PER) of target t in h[t];
// `share`: target 1 reads target 0's histogram).  Thread 0 updates ss; ends
// with a barrier.  cnt0 (LDS, optional): keys in target 0's picked bin.
template <int BLOCK, int PER>
__device__ __forceinline__ void pick_state(SelState &ss, const u64 (&h0)[PER], const u64 (&h1)[PER], bool share,
                                           u64 *scratch, const EarlyWindow *ew = nullptr, u64 *cnt0 = nullptr) {
    const uint32_t mode = ss.mode;
    const bool live = mode == MODE_SAMPLE || mode == MODE_CAND || mode == MODE_FULL;
    bool want[2];
    u64 kt[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        want[t] = live && ss.t[t].active && ss.t[t].done < ss.W;
        kt[t] = ss.t[t].k;
    }
    uint32_t bin[2];
    u64 below[2], cnt[2] = {0, 0};
    bool ok[2];
    if (want[0] || want[1]) block_pick2<BLOCK, PER>(h0, share ? h0 : h1, want, kt, bin, below, ok, scratch, cnt);
    if (threadIdx.x == 0) {
        for (int t = 0; t < 2; ++t) {
            if (!want[t] || ss.mode == MODE_DONE) continue;
            const uint32_t d = digit_bits(ss, ss.t[t].done);
            if (!ok[t] || bin[t] >= (1u << d)) {
                ss.error = 1 + t;
                ss.mode = MODE_DONE;
            } else {
                ss.t[t].k -= below[t];
                ss.t[t].prefix = (ss.t[t].prefix << d) | bin[t];
                ss.t[t].done += d;
            }
        }
        resolve(ss);
        if (ew && want[0] == ss.t[0].active && want[1] == ss.t[1].active) early_window(ss, *ew, cnt[1]);
        if (cnt0) *cnt0 = want[0] ? cnt[0] : ~0ull;
    }
    __syncthreads();
}

template <int BLOCK>
__device__ void advance(SelState &ss, const StepArgs &a, u64 *scratch) {
    // Histogram words are loaded by every thread up front, in parallel with the
    // state: a digit has at most NBINS bins and bins past 2^d are zero in a
    // zeroed slot, so picking over all NBINS is exact for any digit width.
    constexpr int PER = NBINS / BLOCK;
    constexpr int SV = sizeof(SelState) / 16;
    static_assert(sizeof(SelState) % 16 == 0 && SV <= BLOCK, "state moves as 16-byte words");
    // The previous kernel's state, loaded by the first SV threads as 16-byte
    // words before anything else, so its latency overlaps the histogram's
    // (thread 0 loading it after the histogram serialised two HBM round trips).
    const bool carry = a.adv != ADV_INIT_SAMPLE && a.adv != ADV_INIT_FULL;
    uint4 sv = make_uint4(0u, 0u, 0u, 0u);
    if (carry && threadIdx.x < SV) sv = reinterpret_cast<const uint4 *>(a.st_in)[threadIdx.x];
    // the streaming pass's counts travel with the state (one round trip)
    constexpr int CT = (SV + WAVE - 1) / WAVE * WAVE;  // first thread of the counts (next wave)
    static_assert(CT + NCOUNTS <= BLOCK, "counts load beside the state");
    u64 cv = 0;
    if (a.adv == ADV_DECIDE && threadIdx.x >= CT && threadIdx.x < CT + NCOUNTS) cv = a.stats_in[threadIdx.x - CT];
    u64 h0[PER], h1[PER];
    if (a.adv == ADV_PICK) {
        const u64 *b0 = a.stats_in + NCOUNTS + threadIdx.x * PER;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            h0[j] = b0[j];
            h1[j] = b0[NBINS + j];
        }
    }
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
        }
    }
    if (carry && threadIdx.x < SV) reinterpret_cast<uint4 *>(&ss)[threadIdx.x] = sv;
    if (a.adv == ADV_DECIDE && threadIdx.x >= CT && threadIdx.x < CT + NCOUNTS) scratch[threadIdx.x - CT] = cv;
    __syncthreads();
    if (a.adv == ADV_DECIDE) {
        if (threadIdx.x == 0 && ss.mode == MODE_MAIN) decide(ss, scratch);
        __syncthreads();
    } else if (a.adv == ADV_PICK) {
        // both targets' digits in one pass (two barriers); target 1 reads
        // target 0's histogram when they share a prefix
        pick_state<BLOCK, PER>(ss, h0, h1, ss.share, scratch);
    }
}

// ----------------------------------------------------------------- streaming
// Visit n 32-bit words at p (4-byte aligned) as keys, one TILE per thread at a
// time: f(keys[4 * UNROLL], valid_mask), key j of a thread's tile being
// component j % 4 of its (j / 4)-th 16-byte vector.  Calls are wave-convergent
// (every lane calls f the same number of times; invalid keys are masked off),
// so f may use ballots and shuffles.  Block-contiguous tiles of BLOCK * UNROLL
// 16-byte vectors (each wave-instruction reads 1 KiB contiguous), grid-strided;
// all UNROLL loads of a tile are issued before any is used.  XOR flips the sign
// bit (int32 -> order-preserving uint32).
template <int BLOCK, int UNROLL, bool XOR, typename F>
__device__ __forceinline__ void stream_tiles(const uint32_t *__restrict__ p, u64 n, uint32_t wg, uint32_t nwg,
                                             F &&f) {
    constexpr uint32_t X = XOR ? 0x80000000u : 0u;
    constexpr int K = 4 * UNROLL;
    static_assert(K <= 32, "valid mask is 32 bits");
    const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
    u64 head = ((16u - (uint32_t)(addr & 15u)) & 15u) >> 2;
    if (head > n) head = n;
    const uint4 *__restrict__ v = reinterpret_cast<const uint4 *>(p + head);
    const u64 nv = (n - head) >> 2;
    const u64 tail0 = head + (nv << 2);
    const u64 tile = (u64)BLOCK * UNROLL;
    uint32_t k[K];
    for (u64 t0 = (u64)wg * tile; t0 < nv; t0 += (u64)nwg * tile) {
        uint4 x[UNROLL];
        uint32_t valid = 0xFFFFFFFFu;
        if (t0 + tile <= nv) {
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) x[u] = load_nt(&v[t0 + u * BLOCK + threadIdx.x]);
        } else {
            valid = 0;
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const u64 i = t0 + u * BLOCK + threadIdx.x;
                const bool ok = i < nv;
                x[u] = ok ? v[i] : make_uint4(0, 0, 0, 0);
                valid |= ok ? (0xFu << (4 * u)) : 0u;
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            k[4 * u + 0] = x[u].x ^ X;
            k[4 * u + 1] = x[u].y ^ X;
            k[4 * u + 2] = x[u].z ^ X;
            k[4 * u + 3] = x[u].w ^ X;
        }
        if (valid == 0xFFFFFFFFu)
            f(k, valid, std::true_type{});
        else
            f(k, valid, std::false_type{});
    }
    if (wg == 0) {  // ragged head and tail: < 4 keys each, one tile
        const u64 j = threadIdx.x;
        const bool okh = j < head, okt = j < n - tail0;
#pragma unroll
        for (int i = 0; i < K; ++i) k[i] = 0;
        k[0] = (okh ? p[j] : 0u) ^ X;
        k[1] = (okt ? p[tail0 + j] : 0u) ^ X;
        f(k, (okh ? 1u : 0u) | (okt ? 2u : 0u), std::false_type{});
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
        const uint32_t d = p.h[t] ? digit_bits(ss, ss.t[t].done) : 0u;
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
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_level(StepArgs a) {
    __shared__ SelState ss;
    __shared__ u64 scratch[2 * (BLOCK / WAVE) + 8];
    __shared__ __attribute__((aligned(16))) uint32_t lh[2][NBINS];
    KTH_STAMP(a, 0);
    // zero the histogram while the advance's loads are in flight (its barrier orders it)
    for (int i = threadIdx.x; i < 2 * NBINS / 4; i += BLOCK) reinterpret_cast<uint4 *>(&lh[0][0])[i] = make_uint4(0, 0, 0, 0);
    advance<BLOCK>(ss, a, scratch);
    KTH_STAMP(a, 1);
    bool share;
    const HistPlan plan = make_plan(ss, &share);
    const uint32_t mode = ss.mode;
    u64 count = 0;
    if (plan.h[0] || plan.h[1]) {
        if (mode == MODE_SAMPLE) count = a.sample_count;
        else if (mode == MODE_CAND) count = min(*a.cand_count, a.cap);
        else if (mode == MODE_FULL) count = a.n_local;
    }
    publish<BLOCK>(ss, share, a);
    // Few workgroups per histogram keeps the number of same-address global
    // atomics per bin (the flush's serialisation) low; min_per_wg is the host's
    // choice per level (dense levels: large).
    const u64 want = (count + a.min_per_wg - 1) / a.min_per_wg;
    const uint32_t active = (uint32_t)min((u64)gridDim.x, want);
    if (blockIdx.x >= active) return;
    KTH_STAMP(a, 2);
    auto f = [&](const uint32_t *k, uint32_t valid, auto full) {
#pragma unroll
        for (int j = 0; j < 4 * LEVEL_UNROLL; ++j)
            hist_add<BLOCK>(lh, plan, k[j], decltype(full)::value || ((valid >> j) & 1u));
    };
    if (mode == MODE_FULL)
        stream_tiles<BLOCK, LEVEL_UNROLL, true>(reinterpret_cast<const uint32_t *>(a.keys), count, blockIdx.x, active,
                                                f);
    else
        stream_tiles<BLOCK, LEVEL_UNROLL, false>(mode == MODE_SAMPLE ? a.sample : a.cand, count, blockIdx.x, active,
                                                 f);
    KTH_STAMP(a, 3);
    hist_flush<BLOCK>(lh, plan, a.stats_acc);
    KTH_STAMP(a, 5);
}

// Sample gather: s keys in chunks of SAMPLE_CHUNK contiguous keys spread
// evenly over the shard (stride = chunk distance in keys), by waves gw of nw
// (WAVES per workgroup).  With FUSE the keys also go into the LDS histograms
// of `plan` (single GPU: the sample is complete).  COHERENT: write-through
// (sc1) stores, for readers in other workgroups of the same kernel (k_head).
template <int BLOCK, bool FUSE, bool COHERENT = false>
__device__ __forceinline__ void gather_chunks(const int32_t *__restrict__ keys, u64 n_keys, u64 stride,
                                              uint32_t *__restrict__ sample, u64 s, uint32_t (*lh)[NBINS],
                                              const HistPlan &plan) {
    const int lane = threadIdx.x & (WAVE - 1);
    // chunks of SAMPLE_CHUNK keys at `stride`; the last one holds s % SAMPLE_CHUNK
    // keys when that is nonzero (scalar loads, guarded by s and n_keys)
    const u64 nfull = s / SAMPLE_CHUNK, nchunks = (s + SAMPLE_CHUNK - 1) / SAMPLE_CHUNK;
    const u64 gw = ((u64)blockIdx.x * BLOCK + threadIdx.x) / WAVE, nw = (u64)gridDim.x * (BLOCK / WAVE);
    // every wave owns GATHER_BATCH consecutive chunk slots per round; all loads
    // of a round are in flight together.  Chunks of >= 256 keys are read as
    // 16-byte loads, q-th load of the wave = 1 KiB contiguous (lane-major).
    const bool vec = SAMPLE_CK >= 4 && (reinterpret_cast<uintptr_t>(keys) & 15u) == 0 && stride % 4 == 0;
    constexpr int NV = SAMPLE_CK >= 4 ? SAMPLE_CK / 4 : 1;  // 16-byte loads per lane per chunk
    auto off_of = [&](int q) -> u64 {  // key q of this lane within its chunk
        return SAMPLE_CK >= 4 ? 4 * ((u64)(q / 4) * WAVE + lane) + (q & 3) : (u64)lane;
    };
    for (u64 c0 = gw * GATHER_BATCH; c0 < nchunks; c0 += nw * GATHER_BATCH) {
        uint32_t kk[GATHER_BATCH][SAMPLE_CK];
#pragma unroll
        for (int j = 0; j < GATHER_BATCH; ++j) {
            const u64 c = c0 + j;
            if (SAMPLE_CK >= 4 && vec && c < nfull) {
                const uint4 *src = reinterpret_cast<const uint4 *>(keys + c * stride);
#pragma unroll
                for (int q = 0; q < NV; ++q) {
                    const uint4 x = src[q * WAVE + lane];
                    kk[j][4 * q + 0] = key_of_i32(x.x);
                    kk[j][4 * q + 1] = key_of_i32(x.y);
                    kk[j][4 * q + 2] = key_of_i32(x.z);
                    kk[j][4 * q + 3] = key_of_i32(x.w);
                }
            } else {
#pragma unroll
                for (int q = 0; q < SAMPLE_CK; ++q) {
                    const u64 off = off_of(q);
                    const bool ok = c < nchunks && c * SAMPLE_CHUNK + off < s && c * stride + off < n_keys;
                    kk[j][q] = ok ? key_of_i32((uint32_t)keys[c * stride + off]) : 0u;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < GATHER_BATCH; ++j) {
            const u64 c = c0 + j;
            if (c < nchunks) {
#pragma unroll
                for (int q = 0; q < SAMPLE_CK; ++q) {
                    const u64 off = off_of(q);
                    if (c * SAMPLE_CHUNK + off < s) {
                        if (COHERENT)
                            __hip_atomic_store(&sample[c * SAMPLE_CHUNK + off], kk[j][q], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        else
                            sample[c * SAMPLE_CHUNK + off] = kk[j][q];
                        if (FUSE) hist_add<BLOCK>(lh, plan, kk[j][q], true);
                    }
                }
            }
        }
    }
}

template <bool FUSE>
__global__ __launch_bounds__(DENSE_BLK) void k_gather(StepArgs a, const int32_t *__restrict__ keys, u64 n_keys,
                                                u64 stride, uint32_t *__restrict__ sample, u64 s) {
    __shared__ SelState ss;
    __shared__ u64 scratch[2 * (DENSE_BLK / WAVE) + 8];
    __shared__ __attribute__((aligned(16))) uint32_t lh[2][NBINS];
    HistPlan plan{};
    bool share = false;
    KTH_STAMP(a, 0);
    if (FUSE) {
        advance<DENSE_BLK>(ss, a, scratch);
        plan = make_plan(ss, &share);
        publish<DENSE_BLK>(ss, share, a);
        for (int i = threadIdx.x; i < 2 * NBINS; i += DENSE_BLK) (&lh[0][0])[i] = 0;
        __syncthreads();
    }
    if (!FUSE) {  // the sharded protocol's slots, cleared here instead of by a memset launch
        for (u64 i = (u64)blockIdx.x * DENSE_BLK + threadIdx.x; i < a.zero_words; i += (u64)gridDim.x * DENSE_BLK)
            a.stats_zero[i] = 0;
    }
    // (sharded sample, full aligned chunks: a chunk is copied as 16-byte words
    // in the layout gather_chunks writes -- the per-key path took ~8 us)
    const bool vec = !FUSE && s % SAMPLE_CHUNK == 0 && (reinterpret_cast<uintptr_t>(keys) & 15u) == 0 &&
                     stride % 4 == 0 && SAMPLE_CK == 16;
    if (vec) {
        const int lane = threadIdx.x & (WAVE - 1);
        const u64 nch = s / SAMPLE_CHUNK;
        for (u64 c = ((u64)blockIdx.x * DENSE_BLK + threadIdx.x) / WAVE; c < nch; c += (u64)gridDim.x * (DENSE_BLK / WAVE)) {
            const uint4 *src = reinterpret_cast<const uint4 *>(keys + c * stride);
            uint4 *dst = reinterpret_cast<uint4 *>(sample + c * SAMPLE_CHUNK);
            uint4 q[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) q[r] = src[r * WAVE + lane];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                dst[r * WAVE + lane] = make_uint4(q[r].x ^ 0x80000000u, q[r].y ^ 0x80000000u, q[r].z ^ 0x80000000u,
                                                  q[r].w ^ 0x80000000u);
        }
    } else {
        gather_chunks<DENSE_BLK, FUSE>(keys, n_keys, stride, sample, s, lh, plan);
    }
    KTH_STAMP(a, 3);
    if (FUSE) hist_flush<DENSE_BLK>(lh, plan, a.stats_acc);
    KTH_STAMP(a, 5);
}

// Load a level's reduced histograms (thread i: bins [i*PER, i*PER + PER)) with
// device-coherent loads, and pick.
template <int BLOCK>
__device__ __forceinline__ void pick_slot(SelState &ss, const u64 *slot, bool share, u64 *scratch,
                                          const EarlyWindow *ew, u64 *cnt0 = nullptr) {
    constexpr int PER = NBINS / BLOCK;
    u64 h0[PER], h1[PER];
    const u64 *b0 = slot + NCOUNTS + threadIdx.x * PER;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        h0[j] = __hip_atomic_load(b0 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        h1[j] = share ? 0ull : __hip_atomic_load(b0 + NBINS + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    pick_state<BLOCK, PER>(ss, h0, h1, share, scratch, ew, cnt0);
}

// k_head's gather of the full 1024-key sample chunks: the first digit of a
// fresh selection has one histogram (both window targets share the empty
// prefix) and no prefix test, so a key costs a shift and one LDS atomic; the
// chunk is written through as 16-byte stores (per-key 4-byte atomic stores and
// bounds tests made the gather ~8 us of VALU issue in 64 CUs).  Chunk c of the
// sample = keys[c * stride, + SAMPLE_CHUNK); lane l holds 16-byte words l, l+64,
// l+128, l+192 of it.  Returns false (nothing done) unless every chunk is full
// and 16-byte aligned; the caller then uses gather_chunks.
// STORE = false: the chunk's keys only go into the histogram (the sample is
// not kept: a later sample level re-reads the chunks from the input).
// wg / nwg: this workgroup among the nwg that share the chunks.
#ifndef KTH_HEAD_UNI
#define KTH_HEAD_UNI 1
#endif
constexpr bool HEAD_UNI = KTH_HEAD_UNI != 0;  // the head's one-bin chunks as one atomic (below)
template <int BLOCK, bool STORE = true>
__device__ __forceinline__ bool gather_head_fast(const int32_t *__restrict__ keys, u64 stride, uint32_t *sample,
                                                 u64 s, uint32_t (*lh)[NBINS], const HistPlan &plan,
                                                 uint32_t wg, uint32_t nwg) {
    static_assert(SAMPLE_CK == 16, "four 16-byte words per lane and chunk");
    // (selects, not plan.x[t]: a runtime index made the plan a private array
    // that the compiler moved into 44 KiB of LDS)
    const bool one = plan.h[0] != plan.h[1];  // exactly one histogram
    const bool t1 = !plan.h[0];
    if (s % SAMPLE_CHUNK != 0 || (reinterpret_cast<uintptr_t>(keys) & 15u) != 0 || stride % 4 != 0 || !one ||
        (t1 ? plan.done[1] : plan.done[0]) != 0 || plan.base != 0u)
        return false;
    const uint32_t sh = t1 ? plan.shift[1] : plan.shift[0], mask = t1 ? plan.mask[1] : plan.mask[0];
    uint32_t *h = t1 ? lh[1] : lh[0];
    const __amdgpu_buffer_rsrc_t out =
        __builtin_amdgcn_make_buffer_rsrc(sample, (short)0, (int)(s * 4), 0x00020000);
    const int lane = threadIdx.x & (WAVE - 1);
    const u64 nchunks = s / SAMPLE_CHUNK;
    const u64 gw = ((u64)wg * BLOCK + threadIdx.x) / WAVE, nw = (u64)nwg * (BLOCK / WAVE);
    for (u64 c = gw; c < nchunks; c += nw) {
        const uint4 *src = reinterpret_cast<const uint4 *>(keys + c * stride);
        uint4 q[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) q[r] = src[r * WAVE + lane];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            q[r].x ^= 0x80000000u;
            q[r].y ^= 0x80000000u;
            q[r].z ^= 0x80000000u;
            q[r].w ^= 0x80000000u;
            if (STORE) {
                u32x4 v = {q[r].x, q[r].y, q[r].z, q[r].w};
                __builtin_amdgcn_raw_buffer_store_b128(v, out, (int)((c * SAMPLE_CHUNK + 4 * (r * WAVE + lane)) * 4),
                                                       0, 16 /* sc1: written through */);
            }
        }
        // a chunk whose 1024 keys share one bin (sorted or few-valued input:
        // consecutive keys, one digit) is one atomic, not 1024 serialised on
        // one LDS address (sorted / all-equal 2^30: gather + first digit
        // 16 us against 4.5 for uniform keys)
        const uint32_t f = __builtin_amdgcn_readfirstlane((q[0].x >> sh) & mask);
        bool same = true;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            same = same && ((q[r].x >> sh) & mask) == f && ((q[r].y >> sh) & mask) == f &&
                   ((q[r].z >> sh) & mask) == f && ((q[r].w >> sh) & mask) == f;
        if (HEAD_UNI && __ballot(!same) == 0) {  // wave-uniform
            if (lane == 0) atomicAdd(&h[f], (uint32_t)SAMPLE_CHUNK);
            continue;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            atomicAdd(&h[(q[r].x >> sh) & mask], 1u);
            atomicAdd(&h[(q[r].y >> sh) & mask], 1u);
            atomicAdd(&h[(q[r].z >> sh) & mask], 1u);
            atomicAdd(&h[(q[r].w >> sh) & mask], 1u);
        }
    }
    return true;
}

// A later sample digit over the full 1024-key chunks of the input themselves
// (the fast gather keeps no sample): workgroup wg of nwg, plan's histograms.
template <int BLOCK>
__device__ __forceinline__ void head_hist_chunks(const int32_t *__restrict__ keys, u64 stride, u64 s,
                                                 uint32_t (*lh)[NBINS], const HistPlan &plan, uint32_t wg,
                                                 uint32_t nwg) {
    const int lane = threadIdx.x & (WAVE - 1);
    const u64 nchunks = s / SAMPLE_CHUNK;
    const u64 gw = ((u64)wg * BLOCK + threadIdx.x) / WAVE, nw = (u64)nwg * (BLOCK / WAVE);
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    // a key's bin for target t, or NONE (no histogram / prefix mismatch)
    auto code = [&](uint32_t key, int t) {
        const uint32_t v = key - plan.base;
        return plan.h[t] && prefix_match(v, plan.W, plan.done[t], plan.prefix[t])
                   ? (v >> plan.shift[t]) & plan.mask[t]
                   : NONE;
    };
    for (u64 c = gw; c < nchunks; c += nw) {  // wave-convergent
        const uint4 *src = reinterpret_cast<const uint4 *>(keys + c * stride);
        uint4 q[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) q[r] = src[r * WAVE + lane];
        // the whole chunk in one bin per target (sorted / few-valued input):
        // one atomic per target (as in gather_head_fast)
        const uint32_t f0 = __builtin_amdgcn_readfirstlane(code(q[0].x ^ 0x80000000u, 0)),
                       f1 = __builtin_amdgcn_readfirstlane(code(q[0].x ^ 0x80000000u, 1));
        bool same = true;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t k4[4] = {q[r].x ^ 0x80000000u, q[r].y ^ 0x80000000u, q[r].z ^ 0x80000000u,
                                    q[r].w ^ 0x80000000u};
#pragma unroll
            for (int j = 0; j < 4; ++j) same = same && code(k4[j], 0) == f0 && code(k4[j], 1) == f1;
        }
        if (HEAD_UNI && __ballot(!same) == 0) {  // wave-uniform
            if (lane == 0) {
                if (f0 != NONE) atomicAdd(&lh[0][f0], (uint32_t)SAMPLE_CHUNK);
                if (f1 != NONE) atomicAdd(&lh[1][f1], (uint32_t)SAMPLE_CHUNK);
            }
            continue;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            hist_add<BLOCK>(lh, plan, q[r].x ^ 0x80000000u, true);
            hist_add<BLOCK>(lh, plan, q[r].y ^ 0x80000000u, true);
            hist_add<BLOCK>(lh, plan, q[r].z ^ 0x80000000u, true);
            hist_add<BLOCK>(lh, plan, q[r].w ^ 0x80000000u, true);
        }
    }
}

// The streaming pass.  Window [lo, hi] comes from the advance (last sample
// digit).  Per key: #<lo, #==lo, #==hi in per-lane registers.  Keys strictly
// inside the window are staged in the wave's private LDS region one key slot
// at a time: for slot j the ballot B of the lanes whose j-th key is inside
// gives each such lane its position (wfill + mbcnt(B)) and advances the
// wave-uniform fill by popc(B) -- scalar bookkeeping only, no wave scan, no
// per-lane position chain, no LDS atomics, no barriers (uniform keys: B is
// empty for ~2/3 of the slots and the branch is skipped).  A wave flushes its
// region to the candidate buffer itself, with one global reservation, when the
// next slot might not fit -- so staging never overflows however many keys a
// workgroup streams.  Candidate order in the buffer is irrelevant (the levels
// after the pass histogram it as a multiset).

// Reserve `cnt` slots of the candidate buffer for one wave (lane WAVE-1 does the
// atomic); flags the per-rank overflow word exactly once, on the crossing.
__device__ __forceinline__ u64 reserve_cands(u64 *cand_count, u64 *acc, u64 cap, uint32_t cnt) {
    const int lane = threadIdx.x & (WAVE - 1);
    u64 g = 0;
    if (lane == WAVE - 1) {
        g = atomicAdd(cand_count, (u64)cnt);
        if (g <= cap && g + cnt > cap) atomicAdd(&acc[C_OVF], 1ull);
    }
    return __shfl(g, WAVE - 1, WAVE);
}

// Candidate stores are write-through (agent-scope relaxed atomic store: sc1),
// so the candidates reach memory while the pass streams instead of sitting as
// dirty L2 lines that the kernel boundary writes back (measured: the pass
// 691 -> 683 us and the select 772 -> 764 us at 2^30).
__device__ __forceinline__ void put_cand(uint32_t *p, uint32_t x) {
    __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ROWS (k_main<3/4>, top-k): every candidate also carries the 1024-key row it
// came from (wave-uniform per key slot), staged in the region's upper half and
// written to rows_out beside it; ~0u = a row outside k_main's full tiles.
template <bool ROWS = false>
struct Stager {
    static constexpr uint32_t CAP = ROWS ? WREG / 2 : WREG;  // keys the region holds
    uint32_t *reg;       // this wave's LDS region (WREG words)
    uint32_t wfill;      // wave-uniform fill of the region
    u64 winside;         // wave-uniform count of candidates seen
    u64 *cand_count, *acc, cap;
    uint32_t *cand_out;
    uint32_t *rows_out;  // ROWS only
    uint32_t flushed;    // wave-uniform: the region was flushed mid-pass (its keys left LDS)

    // the region's first `cnt` keys (and rows) to candidates [g, g + cnt)
    __device__ __forceinline__ void put(u64 g, uint32_t cnt) const {
        const int lane = threadIdx.x & (WAVE - 1);
        for (uint32_t i = lane; i < cnt; i += WAVE)
            if (g + i < cap) {
                put_cand(&cand_out[g + i], reg[i]);
                if (ROWS) put_cand(&rows_out[g + i], reg[CAP + i]);
            }
    }

    __device__ __forceinline__ void flush() {
        __builtin_amdgcn_wave_barrier();
        const u64 g = reserve_cands(cand_count, acc, cap, wfill);
        put(g, wfill);
        __builtin_amdgcn_wave_barrier();
        wfill = 0;
        flushed = 1u;
    }

    // One key slot of the wave, as the streaming pass sees it: `near` = this
    // lane's key lies in the closed window [lo, hi].  Only a slot where some
    // lane's key does (uniform keys: ~1/3 of the slots at 2^30) tells the
    // edges from the inside: the keys equal to lo / hi are counted, the
    // others are staged.  (Counting both edges on every key cost two compares
    // and two adds per key; with them here the pass issues ~3 VALU ops a key
    // fewer.)
    __device__ __forceinline__ void slot_near(int32_t x, bool near, int32_t slo, int32_t shi, uint32_t &ceqlo,
                                              uint32_t &ceqhi, uint32_t row = ~0u) {
        if (__builtin_amdgcn_ballot_w64(near) == 0) return;  // wave-uniform
        ceqlo += (near & (x == slo)) ? 1u : 0u;
        ceqhi += (near & (x == shi)) ? 1u : 0u;
        slot((uint32_t)x ^ 0x80000000u, near & (x != slo) & (x != shi), row);
    }

    // One key slot of the wave: `in` = this lane's key is a candidate.
    __device__ __forceinline__ void slot(uint32_t key, bool in, uint32_t row = ~0u) {
        const unsigned long long B = __builtin_amdgcn_ballot_w64(in);
#ifdef KTH_DIAG_NOSTAGE
        if (B == 0x123456789ull) {  // diagnostic build only: measures the staging cost
#else
        if (B) {  // wave-uniform
#endif
            const uint32_t nb = (uint32_t)__popcll(B);
            if (wfill + nb > CAP) flush();
            const uint32_t below =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(B >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)B, 0u));
            if (in) {
                reg[wfill + below] = key;
                if (ROWS) reg[CAP + wfill + below] = row;
            }
            wfill += nb;
            winside += nb;
        }
    }
};

// TF 5 / 6 (top-k, k smallest / largest, n/65536 < k <= n/16): every key on
// the kept side of the window's far edge (x <= hi / x >= lo: the keys certainly
// in the output, the candidates and both edges) is staged IN INDEX ORDER with
// its position in its wave-row (one byte) into the wave's own segment of the
// top-k staging buffer -- segment g = the wave's global id, filled
// sequentially: no atomics, no reservation.  The select's candidates (lo < x <
// hi) are filtered out of the region into the candidate buffer when it is
// flushed (the region holds raw int32 keys).  Per wave-row (the 256 keys of a
// k_main row one wave loads), the staged count goes to the row words; the
// top-k then never reads the input for those rows (k_tk5_count /
// k_tk5_write).  A segment that overflows sets seg.ovf: the top-k then counts
// and writes from the input (exact, slower).
struct TkSeg {
    int32_t *vals;     // nwaves * cap raw keys
    uint8_t *pos;      // their positions in their wave-rows
    uint32_t cap;      // entries per segment
    uint32_t *ovf;     // set to 1 when any segment overflows
    uint32_t *wstart;  // nwaves * nwin: entries a wave staged before each window of TK5_WIN_TILES tiles
    uint32_t nwin;     // windows per wave
    uint32_t nt;       // 1: segment stores with the non-temporal hint (dense staging, k >= n / 32)
};
constexpr int TK5_WIN_TILES = 8;  // a window of the staged top-k kernels: 8 tiles = 64 wave-rows a wave

struct OrdStager {
    static constexpr uint32_t CAP = ((uint32_t)WREG5 * 4 / 5) & ~63u;  // keys; CAP position bytes follow
    uint32_t *reg;
    uint32_t wfill;      // wave-uniform
    uint32_t seg_fill;   // wave-uniform: entries already in the segment
    u64 winside;         // wave-uniform: candidates seen
    u64 seg_base;        // this wave's segment (entries)
    int32_t slo, shi;
    u64 *cand_count, *acc, cap;
    uint32_t *cand_out;
    TkSeg seg;

    // The region's entries to the wave's segment, as 16-byte key stores and
    // 4-byte position stores (the segment is 16-byte aligned and a mid-pass
    // flush writes a multiple of 4 entries: the 0-3 left over move to the
    // region's front; `last` writes them too), and the flushed entries'
    // candidates (lo < x < hi) to the candidate buffer.  Latency, not work,
    // is what a flush costs the streaming wave (it issues no loads meanwhile):
    // every LDS read of a step is issued before any is used -- lane l takes
    // the 4-entry groups l, l + 64, .. (FQ of them) -- and the candidates,
    // an unordered multiset, are counted per lane, placed by one wave scan and
    // one reservation, and written by each lane from its own groups (a
    // ballot + mbcnt loop over the region waited one LDS round trip per 64
    // entries, twice: ~2 us a flush, ~90 flushes a wave at k = n / 16).
    static constexpr int FQ = (int)((CAP + 4 * WAVE - 1) / (4 * WAVE));  // 4-entry groups per lane
    static constexpr int FH = (FQ + 1) / 2;                              // groups per half (registers)
    __device__ __forceinline__ void flush(bool last = false) {
        const int lane = threadIdx.x & (WAVE - 1);
        __builtin_amdgcn_wave_barrier();
        uint8_t *pb = reinterpret_cast<uint8_t *>(reg + CAP);
        const uint32_t n4 = wfill & ~3u, nw = last ? wfill : n4;  // entries written now
        const u64 base = seg_base + seg_fill;                     // a multiple of 4
        const uint32_t room = seg_fill < seg.cap ? seg.cap - seg_fill : 0u;  // entries the segment still holds
        const uint4 *r4 = reinterpret_cast<const uint4 *>(reg);
        const uint32_t *p4 = reinterpret_cast<const uint32_t *>(pb);
        auto is_cand = [&](uint32_t x, uint32_t e) { return e < nw && (int32_t)x > slo && (int32_t)x < shi; };
        // pass 1: segment stores + this lane's candidate count, half the groups at a time
        uint32_t nc = 0;
#pragma unroll 1
        for (int h = 0; h < 2; ++h) {
            uint4 kv[FH];
            uint32_t pv[FH];
#pragma unroll
            for (int j = 0; j < FH; ++j) {
                const uint32_t g = (uint32_t)((h * FH + j) * WAVE + lane);
                kv[j] = 4 * g < nw ? r4[g] : make_uint4(0u, 0u, 0u, 0u);
                pv[j] = 4 * g < nw ? p4[g] : 0u;
            }
#pragma unroll
            for (int j = 0; j < FH; ++j) {
                const uint32_t g = (uint32_t)((h * FH + j) * WAVE + lane), e = 4 * g;
#ifndef KTH_DIAG_TK5_NOSEGSTORE  // diagnostic builds only (wrong top-k results): cost of the segment stores
                if (e + 4 <= n4 && e + 4 <= room) {
                    if (seg.nt) {  // wave-uniform
                        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                        const v4u kvv = {kv[j].x, kv[j].y, kv[j].z, kv[j].w};
                        __builtin_nontemporal_store(kvv, reinterpret_cast<v4u *>(seg.vals + base + e));
                        __builtin_nontemporal_store(pv[j], reinterpret_cast<uint32_t *>(seg.pos + base + e));
                    } else {
                        *reinterpret_cast<uint4 *>(seg.vals + base + e) = kv[j];
                        *reinterpret_cast<uint32_t *>(seg.pos + base + e) = pv[j];
                    }
                } else if (last && e < nw) {  // the last 1-3 entries (unaligned tail)
                    const uint32_t kq[4] = {kv[j].x, kv[j].y, kv[j].z, kv[j].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (e + q < nw && e + q < room) {
                            seg.vals[base + e + q] = (int32_t)kq[q];
                            seg.pos[base + e + q] = (uint8_t)(pv[j] >> (8 * q));
                        }
                }
#endif
                nc += (is_cand(kv[j].x, e) ? 1u : 0u) + (is_cand(kv[j].y, e + 1) ? 1u : 0u) +
                      (is_cand(kv[j].z, e + 2) ? 1u : 0u) + (is_cand(kv[j].w, e + 3) ? 1u : 0u);
            }
        }
        if (seg_fill + nw > seg.cap && lane == 0) *seg.ovf = 1u;
#ifndef KTH_DIAG_TK5_NOCANDS  // diagnostic builds only (wrong results): cost of the candidate filter
        // pass 2: one reservation for the wave, each lane its candidates from its offset
        const uint32_t incl = wave_incl_scan32(nc);
        const uint32_t nin = (uint32_t)__builtin_amdgcn_readlane((int)incl, WAVE - 1);
        if (nin) {  // wave-uniform
            const u64 g0 = reserve_cands(cand_count, acc, cap, nin);
            u64 o = g0 + incl - nc;
#pragma unroll 1
            for (int h = 0; h < 2; ++h) {
                uint4 kv[FH];
#pragma unroll
                for (int j = 0; j < FH; ++j) {
                    const uint32_t g = (uint32_t)((h * FH + j) * WAVE + lane);
                    kv[j] = 4 * g < nw ? r4[g] : make_uint4(0u, 0u, 0u, 0u);
                }
#pragma unroll
                for (int j = 0; j < FH; ++j) {
                    const uint32_t e = 4u * (uint32_t)((h * FH + j) * WAVE + lane);
                    const uint32_t kq[4] = {kv[j].x, kv[j].y, kv[j].z, kv[j].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (is_cand(kq[q], e + q)) {
                            if (o < cap) put_cand(&cand_out[o], kq[q] ^ 0x80000000u);
                            ++o;
                        }
                }
            }
            winside += nin;
        }
#endif
        // the 0-3 entries not written move to the front (read before any write: one wave, in order)
        const uint32_t left = wfill - nw;
        uint32_t kx = 0;
        uint8_t px = 0;
        if ((uint32_t)lane < left) {
            kx = reg[nw + lane];
            px = pb[nw + lane];
        }
        __builtin_amdgcn_wave_barrier();
        if ((uint32_t)lane < left) {
            reg[lane] = kx;
            pb[lane] = px;
        }
        seg_fill += nw;
        wfill = left;
        __builtin_amdgcn_wave_barrier();
    }

    // One wave-row slot: this lane's keys q.x .. q.w at positions lane, 64 +
    // lane, 128 + lane, 192 + lane of the wave-row (k_main<5/6> loads a
    // wave-row as 4 dwords a lane, so that the order of the 4 ballots is the
    // index order); stages the keys on the kept side of the far edge (x <= hi
    // for TF 5, x >= lo for TF 6) in index order.  Returns the wave's count
    // (wave-uniform).  Key j's slot is the fill plus the popcounts of ballots
    // 0 .. j-1 plus its mbcnt in ballot j: no per-lane scan, whatever the
    // density.  (Round 5 loaded 4 consecutive keys a lane, position 4 lane + j:
    // a lane staging two of its keys -- most wave-rows at k = n / 16 -- then
    // needed a wave scan of the per-lane counts, k_main<5> 994 us at k = 2^26.)
    // The keys equal to lo / hi are on the kept side too, so they are counted
    // here, behind the same wave-uniform test (ceqlo / ceqhi: this lane's).
    template <int TF>
    __device__ __forceinline__ uint32_t row(const uint4 &q, uint32_t lane, uint32_t &ceqlo, uint32_t &ceqhi) {
        auto f1 = [&](uint32_t x) { return TF == 5 ? (int32_t)x <= shi : (int32_t)x >= slo; };
        const bool c0 = f1(q.x), c1 = f1(q.y), c2 = f1(q.z), c3 = f1(q.w);
        const unsigned long long b0 = __builtin_amdgcn_ballot_w64(c0), b1 = __builtin_amdgcn_ballot_w64(c1),
                                 b2 = __builtin_amdgcn_ballot_w64(c2), b3 = __builtin_amdgcn_ballot_w64(c3);
        if ((b0 | b1 | b2 | b3) == 0) return 0u;  // wave-uniform
        {
            const int32_t x0 = (int32_t)q.x, x1 = (int32_t)q.y, x2 = (int32_t)q.z, x3 = (int32_t)q.w;
            ceqlo += ((c0 & (x0 == slo)) ? 1u : 0u) + ((c1 & (x1 == slo)) ? 1u : 0u) +
                     ((c2 & (x2 == slo)) ? 1u : 0u) + ((c3 & (x3 == slo)) ? 1u : 0u);
            ceqhi += ((c0 & (x0 == shi)) ? 1u : 0u) + ((c1 & (x1 == shi)) ? 1u : 0u) +
                     ((c2 & (x2 == shi)) ? 1u : 0u) + ((c3 & (x3 == shi)) ? 1u : 0u);
        }
        const uint32_t n0 = (uint32_t)__popcll(b0), n1 = (uint32_t)__popcll(b1), n2 = (uint32_t)__popcll(b2);
        const uint32_t total = n0 + n1 + n2 + (uint32_t)__popcll(b3);
#ifdef KTH_DIAG_TK5_NOSTAGE  // diagnostic builds only (wrong top-k results): cost of the staging
        return total;
#endif
        if (wfill + total > CAP) flush();
        uint8_t *pb = reinterpret_cast<uint8_t *>(reg + CAP);
        auto at = [](unsigned long long b, uint32_t base) {
            return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, base));
        };
        const uint32_t a0 = at(b0, wfill), a1 = at(b1, wfill + n0), a2 = at(b2, wfill + n0 + n1),
                       a3 = at(b3, wfill + n0 + n1 + n2);
        if (c0) { reg[a0] = q.x; pb[a0] = (uint8_t)lane; }
        if (c1) { reg[a1] = q.y; pb[a1] = (uint8_t)(WAVE + lane); }
        if (c2) { reg[a2] = q.z; pb[a2] = (uint8_t)(2 * WAVE + lane); }
        if (c3) { reg[a3] = q.w; pb[a3] = (uint8_t)(3 * WAVE + lane); }
        wfill += total;
        return total;
    }
};
static_assert(OrdStager::CAP + OrdStager::CAP / 4 <= (uint32_t)WREG5 && OrdStager::CAP >= 4 * WAVE && WREG <= WREG5,
              "OrdStager region: keys + position bytes in one wave's region, >= one wave-row");

// Count and stage K keys of this lane (key j valid iff bit j of `valid`).  The
// keys are the raw int32 words: signed compares against the signed window
// bounds order them exactly like the order-preserving keys (no per-key xor);
// only a staged candidate is converted.
// DPP-shifted copy of x (0 where the shift has no source lane), for wave scans
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ uint32_t dpp_add(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, false);
}

// k_main<3/4>'s per-row tallies of one tile (this lane): RW 4: #>hi of row u
// in r[u] (one add-with-carry a key); RW 3: the lane's running #<lo (clt)
// after row u, differenced per row afterwards (no extra work per key).  Counted
// where the compares are made (a second set of compares elsewhere kept compare
// masks live in SGPRs and made the loop spill them).
struct RowAcc {
    uint32_t r[8];
};

// ROWS: key j lies in row row0 + j / 4 (row0 = ~0u: not tracked).  RW 3 / 4:
// tally rows into ra (FULL tiles of 32 keys per lane only).
template <int K, bool FULL, bool ROWS, int RW = 0>
__device__ __forceinline__ void scan_keys(const uint32_t (&xw)[K], uint32_t valid, int32_t slo, int32_t shi,
                                          uint32_t &clt, uint32_t &ceqlo, uint32_t &ceqhi, Stager<ROWS> &st,
                                          uint32_t row0 = ~0u, RowAcc *ra = nullptr) {
    static_assert(RW == 0 || (FULL && K == 32), "row tallies cover a full tile's 8 rows");
    const uint32_t span = (uint32_t)shi - (uint32_t)slo;  // [lo, hi] as an unsigned distance from lo (key order)
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const int32_t x = (int32_t)xw[j];
        const bool ok = FULL || ((valid >> j) & 1u);
        clt += (ok & (x < slo)) ? 1u : 0u;
        if constexpr (RW == 3) {  // #<lo is clt's own count: a snapshot after each row's 4 keys
            if ((j & 3) == 3) ra->r[j / 4] = clt;
        } else if constexpr (RW == 4) {
            ra->r[j / 4] += x > shi ? 1u : 0u;
        }
        // (x - lo as u32 is the distance in key order: flipping the sign bit is adding 2^31)
        st.slot_near(x, ok & (xw[j] - (uint32_t)slo <= span), slo, shi, ceqlo, ceqhi,
                     row0 == ~0u ? ~0u : row0 + (uint32_t)(j / 4));
    }
}

// TF (top-k variant, kth_topk.hpp): 0 = plain select; 1 / 2 = also record, per
// full tile, wave and row (the tile's u-th run of 4 * BLK keys), one bit "some
// key <= hi" (1, k smallest) or "some key >= lo" (2, k largest): bit u of
// ((uint8_t *)(tflags + 4))[fl_index(tile, wave)]; and the window as tflags[0..2] =
// {lo, hi, 1} (signed).  A row with no bit set in any wave holds no output key
// of the top-k when its k-th lies inside the window.
// 3 / 4 (k smallest / largest, k > n / 1024): per full tile, row u and wave,
// one word #beyond (#<lo for 3, #>hi for 4; <= 256 keys a wave-row), or'ed
// with TK_RECOUNT when the wave-tile holds a key equal to lo or hi, at
// tflags[rw_index(row, wave)], row = tile * U + u; and every candidate's row
// in cand_rows.  With the candidates these give every unmarked row's #better /
// #equal for any k-th inside the window, so the top-k re-reads only marked
// rows to count (k_topk_count<.., META>).
constexpr uint32_t TK_RECOUNT = 1u << 31;
// Where k_main<TF >= 3> keeps wave w's word of row r: in wave-major segments
// (one per k_main wave, `seg` words: 8 per tile the workgroup streams,
// rounded up to 64), tile i of the workgroup at word 8 i.  A wave collects the
// words of 128 tiles in RW_REGS = 16 registers of its 64 lanes and stores
// them as 16 256-byte lines every 128th tile (at 2^30: once, after the loop).  Stores count in vmcnt in issue order, so a
// store in the loop makes the next tile's first load wait for the store's
// acknowledgement, which under the streaming reads takes microseconds: a
// store per tile cost the pass ~80 us at 2^30, one per 8 tiles ~60 us, one
// per 64 tiles ~30 us.
// Words start after a 64-word header (lo, hi, valid, segment overflow);
// tflags is 256-byte aligned.
constexpr u64 TF_W0 = 64;
constexpr int RW_REGS = 16;  // registers of row words a k_main<TF >= 3> wave holds (8 tiles each)
struct RowWords {
    u64 G;    // k_main's grid (workgroups)
    u64 seg;  // words per wave segment
};
__host__ __device__ __forceinline__ u64 rw_seg_words(u64 nfull, u64 G) {
    return ((nfull + G - 1) / G * MAIN_UNROLL + 63) / 64 * 64;
}
// k_main<1/2>'s flag bytes (one per wave and tile, bit u = row u), the same
// way: wave-major segments of `seg` bytes (tiles per workgroup, rounded up to
// 256), byte i = the workgroup's tile i, after tflags' 16-byte header; a wave
// collects 256 tiles' bytes in one register of its 64 lanes.
__host__ __device__ __forceinline__ u64 fl_seg_bytes(u64 nfull, u64 G) { return ((nfull + G - 1) / G + 255) / 256 * 256; }
__host__ __device__ __forceinline__ u64 fl_index(const RowWords &L, u64 t, uint32_t w) {
    return ((t % L.G) * (BLK / WAVE) + w) * L.seg + t / L.G;
}
__host__ __device__ __forceinline__ u64 rw_index(const RowWords &L, u64 r, uint32_t w) {
    const u64 t = r / MAIN_UNROLL;
    return TF_W0 + ((t % L.G) * (BLK / WAVE) + w) * L.seg + (t / L.G) * MAIN_UNROLL + r % MAIN_UNROLL;
}
static_assert(MAIN_UNROLL <= 8, "k_main<TF> keeps one row bit per 16-B load slot in a byte");
static_assert(BLK / WAVE == 4, "k_main<TF> stores one flag byte per wave, four per tile (tk_row_flagged's mask)");
template <int TF>
__global__ __launch_bounds__(BLK) void k_main(StepArgs a, uint32_t *__restrict__ cand_out,
                                              uint32_t *__restrict__ tflags, uint32_t *__restrict__ cand_rows,
                                              TkSeg seg) {
    constexpr int U = MAIN_UNROLL, S = MAIN_SUB, K = 4 * S;
#ifdef KTH_DIAG_NOROWS  // diagnostic builds only (wrong top-k results): cost of the row tags
    constexpr bool ROWS = false;
#else
    constexpr bool ROWS = TF == 3 || TF == 4;
#endif
    constexpr bool ORD = TF >= 5;  // index-ordered staging of the kept side (OrdStager)
    static_assert(U % S == 0, "MAIN_UNROLL is a multiple of MAIN_SUB");
    __shared__ SelState ss;
    __shared__ u64 scratch[2 * (BLK / WAVE) + 8];
    __shared__ __attribute__((aligned(16))) uint32_t region[BLK / WAVE][TF >= 5 ? WREG5 : WREG];
    __shared__ u64 red[6][BLK / WAVE];
    __shared__ uint32_t rowx[BLK / WAVE][4];  // k_main<3/4>: a wave's row sums in transit
    KTH_STAMP(a, 0);
    const uint32_t *p = reinterpret_cast<const uint32_t *>(a.keys);
    const u64 n = a.n_local;
    u64 head = ((16u - (uint32_t)(reinterpret_cast<uintptr_t>(p) & 15u)) & 15u) >> 2;
    if (head > n) head = n;
    const uint4 *__restrict__ v = reinterpret_cast<const uint4 *>(p + head);
    const u64 nv = (n - head) >> 2, tail0 = head + (nv << 2);
    const u64 tile = (u64)BLK * U, nfull = nv / tile;
    // Full tiles are dealt grid-strided.  (Workgroups on every other XCD finish
    // ~5 % later; handing the last 25 % of the tiles out dynamically per XCD
    // evened the finish times but not the pass time: it is HBM-bound, and the
    // early finishers' bandwidth goes to the rest.  DESIGN.md.)
    auto load_tile = [&](uint4 (&x)[U], u64 t) {
        const uint4 *src = v + t * tile + threadIdx.x;
        // One load, wait for it, then the other U-1, in every variant.  Measured
        // at 2^30 (k_main<0>, A/B in one process): the compiler's own order --
        // two loads, wait for the first, then six -- 0.637 ms; one first
        // 0.633 ms (select 1540 -> 1551 Gkeys/s); two then both 0.643; three
        // or four then one 0.640-0.641; all eight first (a sched_barrier) 0.685;
        // the next tile's first 1 / 2 / 4 loads issued before this tile is used
        // 0.703 / 0.695 / 0.689.  The top-k variants' own schedule sent all
        // eight first: k_main<5> ~750 us.  Fewer requests in flight per wave
        // at a tile's start stream faster here, not more.  Plain loads instead
        // of nontemporal ones: select 0.676 -> 0.762 ms, top-k k = 2^24 / 2^27
        // 1.003 / 2.015 -> 1.082 / 2.126 ms (one box, round 5).
#ifndef KTH_MAIN_FIRST  // design exploration: loads before the wait, and the wait's vmcnt
#define KTH_MAIN_FIRST 1
#define KTH_MAIN_WAITN 0
#endif
#pragma unroll
        for (int u = 0; u < KTH_MAIN_FIRST; ++u) x[u] = load_nt(src + u * BLK);
        asm volatile("s_waitcnt vmcnt(" KTH_STR(KTH_MAIN_WAITN) ")" ::: "memory");
#pragma unroll
        for (int u = KTH_MAIN_FIRST; u < U; ++u) x[u] = load_nt(src + u * BLK);
    };
    // (Issuing the first tile's loads before the advance made the pass slower,
    // 656 vs 642 us: the advance's histogram loads then wait behind them.)
    advance<BLK>(ss, a, scratch);
    publish<BLK>(ss, 0, a);
    KTH_STAMP(a, 1);
    if (ss.mode != MODE_MAIN) return;  // block-uniform (error or resolved)
    const int32_t slo = i32_of_key(ss.lo), shi = i32_of_key(ss.hi);
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    if constexpr (TF != 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            tflags[0] = (uint32_t)slo;
            tflags[1] = (uint32_t)shi;
            tflags[2] = 1u;
        }
    }
    Stager<ROWS> st{region[wid], 0u, 0ull, a.cand_count, a.stats_acc, a.cap, cand_out, cand_rows, 0u};
    OrdStager os{region[wid], 0u, 0u, 0ull, ((u64)blockIdx.x * (BLK / WAVE) + wid) * seg.cap, slo, shi,
                 a.cand_count, a.stats_acc, a.cap, cand_out, seg};
    uint32_t clt = 0, ceqlo = 0, ceqhi = 0;  // per lane
    // TF 5 / 6: the counts of one wave-row slot's 4 keys (as scan_keys) and
    // their ordered staging (full tiles only)
    auto ord_keys = [&](const uint4 &q) -> uint32_t {
#ifdef KTH_DIAG_TK5_NOROW  // diagnostic builds only (wrong results): the pass without the staging compares
        clt += q.x < (uint32_t)slo;
        return 0u;
#endif
        clt += ((int32_t)q.x < slo ? 1u : 0u) + ((int32_t)q.y < slo ? 1u : 0u) + ((int32_t)q.z < slo ? 1u : 0u) +
               ((int32_t)q.w < slo ? 1u : 0u);
        return os.template row<TF>(q, (uint32_t)lane, ceqlo, ceqhi);  // (the edges are counted there)
    };
    // TF 5 / 6 load a tile's wave-rows as dwords: row u of wave w is the 256
    // keys u * 4 BLK + 256 w + [0, 256) (the same keys as the 16-byte loads'
    // row u of the wave), lane l taking keys 64 j + l (j = 0..3) into x[u].
    // Then the 4 ballots of a slot are in the wave-row's index order.  One
    // load, a wait, then the rest, as load_tile.
    auto load_tile_ord = [&](uint4 (&x)[U], u64 t) {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(v + t * tile) + wid * (4 * WAVE) + lane;
        x[0].x = load_nt(src);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        x[0].y = load_nt(src + WAVE);
        x[0].z = load_nt(src + 2 * WAVE);
        x[0].w = load_nt(src + 3 * WAVE);
#pragma unroll
        for (int u = 1; u < U; ++u) {
            const uint32_t *r = src + u * (4 * BLK);
            x[u] = make_uint4(load_nt(r), load_nt(r + WAVE), load_nt(r + 2 * WAVE), load_nt(r + 3 * WAVE));
        }
    };

    // a tile is consumed in groups of 4 * MAIN_SUB keys
    constexpr int RW = (TF == 3 || TF == 4) ? TF : 0;
    auto scan_tile = [&](const uint4 (&x)[U], u64 t, RowAcc &ra) {
        static_assert(RW == 0 || U == S, "row tallies: one key group per tile");
#pragma unroll
        for (int h = 0; h < U / S; ++h) {
            uint32_t kk[K];
#pragma unroll
            for (int u = 0; u < S; ++u) {
                kk[4 * u + 0] = x[h * S + u].x;
                kk[4 * u + 1] = x[h * S + u].y;
                kk[4 * u + 2] = x[h * S + u].z;
                kk[4 * u + 3] = x[h * S + u].w;
            }
            scan_keys<K, true, ROWS, RW>(kk, 0xFFFFFFFFu, slo, shi, clt, ceqlo, ceqhi, st,
                                         ROWS ? (uint32_t)(t * U + h * S) : ~0u, &ra);
        }
    };
    // (e0: this lane's ceqlo + ceqhi before the tile; a change = a key on an edge)
    // TF >= 3: lanes 0..U-1 leave the tile's row words in tile_word; lane
    // 8 (i % 8) + u of grp collects row u of the workgroup's tile i, and the
    // 64 lanes store every 8th tile (rw_index)
    uint32_t tiles_done = 0;  // TF >= 1: this workgroup's tiles so far
    uint32_t tile_word = 0, grp[RW_REGS], wsr = 0, facc = 0;
    uint32_t *const fseg = TF == 1 || TF == 2
                               ? tflags + 4 + ((u64)blockIdx.x * (BLK / WAVE) + wid) * (fl_seg_bytes(nfull, gridDim.x) / 4)
                               : nullptr;
#pragma unroll
    for (int q = 0; q < RW_REGS; ++q) grp[q] = 0u;
    const u64 seg_words = rw_seg_words(nfull, gridDim.x);
    uint32_t *const wseg = tflags + TF_W0 + ((u64)blockIdx.x * (BLK / WAVE) + wid) * seg_words;
    auto flag_tile = [&](const uint4 (&x)[U], u64 t, RowAcc &ra, uint32_t e0, uint32_t c0) {
        if constexpr (TF == 1 || TF == 2) {
            // bit u of the wave's byte: some key of row u (the tile's u-th run of
            // 4 * BLK keys) in this wave's part is <= hi (TF 1) / >= lo (TF 2)
            uint32_t rows = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int32_t a0 = (int32_t)x[u].x, a1 = (int32_t)x[u].y, a2 = (int32_t)x[u].z, a3 = (int32_t)x[u].w;
                const bool nr = TF == 1 ? min(min(a0, a1), min(a2, a3)) <= shi : max(max(a0, a1), max(a2, a3)) >= slo;
                rows |= (__builtin_amdgcn_ballot_w64(nr) != 0 ? 1u : 0u) << u;
            }
            // byte tiles_done % 4 of lane (tiles_done / 4) % 64 (stored every 256 tiles)
            facc = (uint32_t)lane == (tiles_done / 4) % WAVE ? facc | rows << (8 * (tiles_done % 4)) : facc;
        }
#ifdef KTH_DIAG_NOROWW  // diagnostic builds only (wrong top-k results): cost of the row words
        if constexpr (TF >= 5) {
#else
        if constexpr (TF >= 3) {
#endif
            static_assert(U == 8, "k_main<3/4> packs four rows' counts into each of two words");
            // #beyond per row: a lane holds <= 4 keys of a row, so rows 0-3 / 4-7
            // fit 8-bit fields of b0 / b1 over a 32-lane half (<= 128); two DPP
            // half-wave scans.  The halves' sums go through the wave's LDS words
            // to lanes 0..7 (readlanes into SGPRs made the loop spill SGPRs).  A
            // wave-tile with a key on a window edge (uniform keys: never) is
            // marked TK_RECOUNT instead: the count pass reads those rows (per-row
            // edge tallies here made the loop spill SGPRs too).
            if constexpr (TF == 3) {  // running #<lo snapshots -> per-row counts
#pragma unroll
                for (int u = U - 1; u > 0; --u) ra.r[u] -= ra.r[u - 1];
                ra.r[0] -= c0;
            }
            // rows 0-3 / 4-7 into the 8-bit fields of b0 / b1 (a lane's row count <= 4)
            uint32_t b0 = ra.r[0] | ra.r[1] << 8 | ra.r[2] << 16 | ra.r[3] << 24;
            uint32_t b1 = ra.r[4] | ra.r[5] << 8 | ra.r[6] << 16 | ra.r[7] << 24;
            auto half_scan = [](uint32_t c) {
                c += dpp_add<0x111>(c);       // row_shr:1
                c += dpp_add<0x112>(c);       // row_shr:2
                c += dpp_add<0x114>(c);       // row_shr:4
                c += dpp_add<0x118>(c);       // row_shr:8
                c += dpp_add<0x142, 0xA>(c);  // row_bcast:15 -> lanes 31, 63: the halves' sums
                return c;
            };
#ifndef KTH_DIAG_NOSCAN  // diagnostic builds only (wrong top-k results)
            b0 = half_scan(b0);
            b1 = half_scan(b1);
#endif
            uint32_t *rx = rowx[wid];
            if ((lane & 31) == 31) {
                rx[lane >> 5] = b0;
                rx[2 + (lane >> 5)] = b1;
            }
            const uint32_t mark = __builtin_amdgcn_ballot_w64(ceqlo + ceqhi != e0) != 0 ? TK_RECOUNT : 0u;
            __builtin_amdgcn_wave_barrier();  // a wave's LDS accesses are in order
            if (lane < U) {
                const uint32_t q = lane < 4 ? 0u : 2u, sh = 8 * (lane & 3);
                const uint32_t word = ((rx[q] >> sh) & 0xFFu) + ((rx[q + 1] >> sh) & 0xFFu);
                tile_word = word | mark;
            }
            __builtin_amdgcn_wave_barrier();
        }
    };
    static_assert(TK5_WIN_TILES * U == WAVE, "a group of row words is one window of the staged kernels");
    for (u64 t = blockIdx.x; t < nfull; t += gridDim.x) {
        uint4 x[U];
        RowAcc ra{{0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}};
        const uint32_t e0 = ceqlo + ceqhi, c0 = clt;
        if constexpr (ORD)
            load_tile_ord(x, t);
        else
            load_tile(x, t);
        if constexpr (ORD) {
            // row u: this lane's keys l, 64 + l, 128 + l, 192 + l of the wave's
            // 256 (its wave-row); lane u keeps row u's staged count for the row words
            uint32_t rw = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t tot = ord_keys(x[u]);
                rw = lane == u ? tot : rw;
            }
            tile_word = rw;
        } else {
            scan_tile(x, t, ra);
            flag_tile(x, t, ra, e0, c0);
        }
        if constexpr (TF == 1 || TF == 2) {
            ++tiles_done;
            if (tiles_done % (4 * WAVE) == 0) {  // wave-uniform: 256 tiles' bytes
                fseg[(tiles_done - 4 * WAVE) / 4 + lane] = facc;
                facc = 0;
            }
        }
        if constexpr (TF >= 3) {
            // lane 8 (i % 8) + u of grp[(i / 8) % RW_REGS] <- row u of tile i
            const uint32_t v = (uint32_t)__shfl((int)tile_word, lane & (U - 1), WAVE);
            const bool mine = (uint32_t)(lane / U) == tiles_done % TK5_WIN_TILES;
            const uint32_t gi = (tiles_done / TK5_WIN_TILES) % RW_REGS;
#pragma unroll
            for (int q = 0; q < RW_REGS; ++q) grp[q] = mine && gi == (uint32_t)q ? v : grp[q];
            ++tiles_done;
#ifndef KTH_DIAG_NOPEND  // diagnostic builds only (wrong top-k results): cost of the row-word stores
            if (tiles_done % (RW_REGS * TK5_WIN_TILES) == 0) {  // wave-uniform: 128 tiles' words
#pragma unroll
                for (int q = 0; q < RW_REGS; ++q)
                    wseg[(tiles_done - RW_REGS * TK5_WIN_TILES) * U + q * WAVE + lane] = grp[q];
            }
#endif
            // TF 5 / 6: the entries staged before each window (lane w % 64 of
            // wsr), so the staged top-k kernels take the windows independently
            if constexpr (ORD)
                if (tiles_done % TK5_WIN_TILES == 0) {  // wave-uniform
                    const uint32_t wi = tiles_done / TK5_WIN_TILES;
                    wsr = (uint32_t)lane == wi % WAVE ? os.seg_fill + os.wfill : wsr;
                    if (wi % WAVE == WAVE - 1 && wi - (WAVE - 1) + lane < seg.nwin)
                        seg.wstart[((u64)blockIdx.x * (BLK / WAVE) + wid) * seg.nwin + wi - (WAVE - 1) + lane] = wsr;
                }
        }
    }
    if constexpr (TF == 1 || TF == 2) {  // the last partial word group
        const uint32_t left = tiles_done % (4 * WAVE);
        if (left != 0 && (uint32_t)lane < (left + 3) / 4) fseg[(tiles_done - left) / 4 + lane] = facc;
    }
    if constexpr (TF >= 3) {  // the last partial groups
        const uint32_t g0 = tiles_done - tiles_done % (RW_REGS * TK5_WIN_TILES);  // first tile not stored
#pragma unroll
        for (int q = 0; q < RW_REGS; ++q) {
            const uint32_t t0 = g0 + (uint32_t)q * TK5_WIN_TILES;
            if (t0 < tiles_done && (uint32_t)lane < (tiles_done - t0 < TK5_WIN_TILES ? tiles_done - t0 : TK5_WIN_TILES) * U)
                wseg[t0 * U + lane] = grp[q];
        }
        if constexpr (ORD) {
            const uint32_t wl = tiles_done / TK5_WIN_TILES, w0 = wl - wl % WAVE;  // windows w0 .. wl not stored
            if (wl % WAVE != WAVE - 1 && (uint32_t)lane <= wl % WAVE && w0 + lane < seg.nwin)
                seg.wstart[((u64)blockIdx.x * (BLK / WAVE) + wid) * seg.nwin + w0 + lane] = wsr;
        }
    }
    // TF 5 / 6: the wave's last entries (and its candidates, reserved by the
    // wave); its LDS region is then free for the ragged keys below, which are
    // outside k_main's full tiles (the top-k reads those rows from the input):
    // they only count and go to the candidates, like the plain pass's keys
    if constexpr (ORD) os.flush(true);
    // ragged end: the last partial tile, as masked groups of one workgroup
    const u64 rem0 = nfull * tile;
    if (blockIdx.x == (uint32_t)(nfull % gridDim.x))
        for (int h = 0; h < U / S; ++h) {
            uint32_t kk[K];
            uint32_t ok = 0;
#pragma unroll
            for (int u = 0; u < S; ++u) {
                const u64 i = rem0 + (h * S + u) * BLK + threadIdx.x;
                const bool in = i < nv;
                const uint4 x = in ? v[i] : make_uint4(0, 0, 0, 0);
                kk[4 * u + 0] = x.x;
                kk[4 * u + 1] = x.y;
                kk[4 * u + 2] = x.z;
                kk[4 * u + 3] = x.w;
                ok |= in ? (0xFu << (4 * u)) : 0u;
            }
            scan_keys<K, false>(kk, ok, slo, shi, clt, ceqlo, ceqhi, st);
        }
    if (blockIdx.x == 0) {  // the < 4-key unaligned head and tail
        const bool okh = threadIdx.x < head, okt = threadIdx.x < n - tail0;
        const uint32_t kk[2] = {okh ? p[threadIdx.x] : 0u, okt ? p[tail0 + threadIdx.x] : 0u};
        scan_keys<2, false>(kk, (okh ? 1u : 0u) | (okt ? 2u : 0u), slo, shi, clt, ceqlo, ceqhi, st);
    }
    // counts: wave reduce -> LDS -> one atomic per workgroup and counter; the
    // waves' final region fills are combined the same way, so the candidate
    // buffer sees one reservation per workgroup at the end of the pass
    u64 r0 = clt, r1 = ceqlo, r2 = ceqhi;
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) {
        r0 += __shfl_xor(r0, o, WAVE);
        r1 += __shfl_xor(r1, o, WAVE);
        r2 += __shfl_xor(r2, o, WAVE);
    }
    if (lane == 0) {
        red[0][wid] = r0;
        red[1][wid] = r1;
        red[2][wid] = r2;
        red[3][wid] = (ORD ? os.winside : 0ull) + st.winside;
        red[4][wid] = st.wfill;
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        u64 sum = 0;
        for (int w = 0; w < BLK / WAVE; ++w) sum += red[threadIdx.x][w];
        if (threadIdx.x == 4) {
            u64 g = 0;
            if (sum) {
                g = atomicAdd(a.cand_count, sum);
                if (g <= a.cap && g + sum > a.cap) atomicAdd(&a.stats_acc[C_OVF], 1ull);
            }
            red[5][0] = g;
        } else {
            const int slot[4] = {C_LT, C_EQLO, C_EQHI, C_IN};
            if (sum) atomicAdd(&a.stats_acc[slot[threadIdx.x]], sum);
        }
    }
    __syncthreads();
    if (st.wfill) {  // this wave's final region, at its share of the reservation
        u64 g = red[5][0];
        for (int w = 0; w < wid; ++w) g += red[4][w];
        st.put(g, st.wfill);
    }
    if constexpr (TF == 0) {
        if (a.pre_hist) {  // kernel-uniform: the candidates' first digit for k_finish (PreHist)
            __shared__ uint32_t phist[PRE_BINS];
            __shared__ uint32_t pflushed;
            const uint32_t W = cand_width(ss.lo, ss.hi);
            const uint32_t d = min(W, fin_first_digit(W)), sh = W - d, base = ss.lo + 1u;
            if (threadIdx.x == 0) pflushed = 0u;
            for (int b = threadIdx.x; b < PRE_BINS; b += BLK) phist[b] = 0u;
            __syncthreads();
            if (lane == 0 && st.flushed) atomicOr(&pflushed, 1u);
            __syncthreads();
            if (pflushed) {  // block-uniform: some of its candidates left LDS
                if (threadIdx.x == 0) atomicAdd(&a.pre_hist[PRE_INCOMPLETE], 1u);
            } else if (W > 0u) {
#pragma unroll
                for (int q = 0; q < BLK / WAVE; ++q) {
                    const uint32_t nq = (uint32_t)red[4][q];
                    for (uint32_t i = threadIdx.x; i < nq; i += BLK) {
                        // a wave-instruction's candidates in one bin (sorted input:
                        // a workgroup's candidates are a run of values) add once
                        const uint32_t b = (region[q][i] - base) >> sh, f = __builtin_amdgcn_readfirstlane(b);
                        const u64 act = __ballot(true);
                        if (HEAD_UNI && __ballot(b != f) == 0) {
                            if ((uint32_t)lane == (uint32_t)__builtin_ctzll(act)) atomicAdd(&phist[f], (uint32_t)__popcll(act));
                        } else {
                            atomicAdd(&phist[b], 1u);
                        }
                    }
                }
                __syncthreads();
                uint32_t *dst = a.pre_hist + (blockIdx.x % PRE_COPIES) * PRE_BINS;
                for (uint32_t b = threadIdx.x; b < (1u << d); b += BLK) {
                    const uint32_t c = phist[b];
                    if (c) atomicAdd(&dst[b], c);
                }
            }
        }
    }
    KTH_STAMP(a, 5);
}

// Final digit: one workgroup.  Writes the answer and the error word, then
// zeroes the ctx-internal slots (and local candidate count) for the next call.
__global__ __launch_bounds__(BLK) void k_result(StepArgs a, int32_t *d_out, int32_t *d_status, u64 *izero,
                                                u64 izero_words) {
    __shared__ SelState ss;
    __shared__ u64 scratch[2 * (BLK / WAVE) + 8];
    KTH_STAMP(a, 0);
    advance<BLK>(ss, a, scratch);
    if (threadIdx.x == 0) {
        SelState o = ss;
        if (o.mode != MODE_DONE && !o.error) o.error = 16 + o.mode;
        *a.st_out = o;
        if (d_out && !o.error) *d_out = i32_of_key(o.answer);  // only a verified answer reaches d_out
        if (d_status) {
            d_status[0] = i32_of_key(o.answer);
            d_status[1] = (int32_t)o.error;
        }
    }
    __syncthreads();
    for (u64 i = threadIdx.x; i < izero_words; i += BLK) izero[i] = 0;
    KTH_STAMP(a, 5);
}

// ------------------------------------------------ sharded protocol (kth_dist_*)
// One all-gather (the samples) and, in the common case, two all-reduces per
// selection (TODO-kth-problem-cgm.c:122-233 runs 2 gathers, a broadcast and an
// all-reduce per round, ~12 rounds):
//   kth_dist_scan   k_main<0> (counts) + k_dscan_hist: this rank's candidates'
//                   FIRST digit into the same slot             -> all-reduce 1
//   level 0         k_dlevel: decide from the reduced counts, pick the first
//                   candidate digit from the same slot, histogram the next
//                                                                -> all-reduce 2
//   result          k_dresult: pick the last digit
// The candidate domain's digits are taken relative to lo + 1 and are DDIG = 12
// bits wide (one target: a slot's two 2048-word histograms hold one 4096-bin
// digit), the narrow one first, so a window of width <= 2^24 needs exactly
// these two.  Wider windows and the exact fallback over the whole shard (a
// window miss or a candidate overflow: 8 + 12 + 12 bits) take more levels;
// level 0 tells the host how many (DistStatus), so every rank makes the same
// calls.
constexpr int DDIG = 12;
constexpr int DNB = 1 << DDIG;
static_assert(DNB == 2 * NBINS, "a stats slot's histogram words hold one DDIG-bit digit");
constexpr uint32_t DIST_FULL_D0 = 32 - 2 * DDIG;  // the fallback's first digit (8 bits)

// The candidate domain of a window [lo, hi]: keys lo < x < hi, as x - base in
// [0, 2^W) with base = lo + 1; d0 = first digit width (the later ones DDIG).
struct CandDom {
    uint32_t base, W, d0;
};
__device__ __forceinline__ CandDom cand_domain(uint32_t lo, uint32_t hi) {
    CandDom d{lo + 1u, 0u, 0u};
    if (hi - lo < 2u) return d;  // no key strictly inside
    const uint32_t range = hi - lo - 2u;
    d.W = range ? 32u - (uint32_t)__clz(range) : 0u;
    const uint32_t nd = (d.W + DDIG - 1) / DDIG;
    d.d0 = d.W - (uint32_t)DDIG * (nd ? nd - 1u : 0u);
    return d;
}

// decide() for the sharded protocol: the same rule, the DDIG-bit digits
__device__ __forceinline__ void decide_dist(SelState &s, const u64 *c) {
    const u64 L = c[C_LT], E1 = c[C_EQLO], M = c[C_IN], ovf = c[C_OVF];
    const u64 E2 = (s.lo == s.hi) ? 0 : c[C_EQHI];
    for (int i = 0; i < 5; ++i) s.cnt[i] = c[i];
    const u64 k = s.k;
    s.t[1].active = 0;
    s.t[0] = Target{k, 0, 0, 1, 0};
    s.path = 3;  // KTH_PATH_WINDOW
    s.dw = DDIG;
    if (k > L && k <= L + E1) {
        s.answer = s.lo;
        s.mode = MODE_DONE;
    } else if (k > L + E1 && k <= L + E1 + M && ovf == 0) {
        const CandDom d = cand_domain(s.lo, s.hi);
        s.base = d.base;
        s.W = d.W;
        s.d0 = d.d0;
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
        s.d0 = DIST_FULL_D0;
        s.path = 4;  // KTH_PATH_WINDOW_FALLBACK
    }
}

__device__ __forceinline__ bool dist_live(const SelState &s) {
    return (s.mode == MODE_CAND || s.mode == MODE_FULL) && s.t[0].done < s.W;
}

// The pick of one DDIG-bit digit: thread i holds bins [i*PER, i*PER + PER).
template <int BLOCK>
__device__ __forceinline__ void pick_wide(SelState &ss, const u64 (&h)[DNB / BLOCK], u64 *scratch) {
    if (!dist_live(ss)) return;  // block-uniform (ss in LDS after a barrier)
    uint32_t bin;
    u64 below;
    const bool ok = block_pick_vals<BLOCK, DNB / BLOCK>(h, ss.t[0].k, &bin, &below, scratch);
    if (threadIdx.x == 0) {
        const uint32_t d = digit_bits(ss, ss.t[0].done);
        if (!ok || bin >= (1u << d)) {
            ss.error = 1;
            ss.mode = MODE_DONE;
        } else {
            ss.t[0].k -= below;
            ss.t[0].prefix = (ss.t[0].prefix << d) | bin;
            ss.t[0].done += d;
            resolve(ss);
        }
    }
    __syncthreads();
}

// The state of the previous step (a.st_in) into LDS; ADV_DECIDE (level 0):
// the decide from a.stats_in's reduced counts.  Everything a workgroup needs
// to know whether it has work (the domain and its size) comes from this
// alone, so idle workgroups leave before loading a histogram.
template <int BLOCK>
__device__ __forceinline__ void dist_state(SelState &ss, const StepArgs &a, u64 *cnts) {
    constexpr int SV = sizeof(SelState) / 16;
    static_assert(SV <= BLOCK && NCOUNTS <= BLOCK, "state and counts load in one step");
    uint4 sv = make_uint4(0u, 0u, 0u, 0u);
    if (threadIdx.x < SV) sv = reinterpret_cast<const uint4 *>(a.st_in)[threadIdx.x];
    if (a.adv == ADV_DECIDE && threadIdx.x < NCOUNTS) cnts[threadIdx.x] = a.stats_in[threadIdx.x];
    if (threadIdx.x < SV) reinterpret_cast<uint4 *>(&ss)[threadIdx.x] = sv;
    __syncthreads();
    if (a.adv == ADV_DECIDE) {
        if (threadIdx.x == 0 && ss.mode == MODE_MAIN) decide_dist(ss, cnts);
        __syncthreads();
    }
}

// The digit pick of a step: level 0 picks the candidates' first digit (the
// scan's slot holds it; the fallback has none yet), later steps the digit
// the previous level histogrammed.
template <int BLOCK>
__device__ __forceinline__ void dist_pick(SelState &ss, const StepArgs &a, u64 *scratch) {
    if (a.adv == ADV_DECIDE ? ss.mode != MODE_CAND : !dist_live(ss)) return;  // block-uniform
    constexpr int PER = DNB / BLOCK;
    const u64 *b = a.stats_in + NCOUNTS + threadIdx.x * PER;
    u64 h[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) h[j] = b[j];
    pick_wide<BLOCK>(ss, h, scratch);
}

// Histogram digit `d` (bits [W - done - d, W - done) of key - base) of the keys
// of `dom` whose resolved prefix matches, into LDS, and flush it to acc's
// histogram words.  XOR: the domain is the raw int32 shard.
template <int BLOCK, bool XOR>
__device__ __forceinline__ void dist_hist(uint32_t *lh, const uint32_t *dom, u64 count, uint32_t active,
                                          uint32_t base, uint32_t W, uint32_t done, uint32_t prefix, uint32_t d,
                                          u64 *acc) {
    const uint32_t sh = W - done - d, mask = (1u << d) - 1u, msh = W - done;
    auto f = [&](const uint32_t *k, uint32_t valid, auto full) {
#pragma unroll
        for (int j = 0; j < 4 * LEVEL_UNROLL; ++j) {
            const uint32_t v = k[j] - base;
            // (a 64-bit shift: msh is 32 before the first digit)
            if ((decltype(full)::value || ((valid >> j) & 1u)) && ((u64)v >> msh) == (u64)prefix)
                atomicAdd(&lh[(v >> sh) & mask], 1u);
        }
    };
    if (blockIdx.x < active) stream_tiles<BLOCK, LEVEL_UNROLL, XOR>(dom, count, blockIdx.x, active, f);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b <= mask; b += BLOCK) {
        const uint32_t c = lh[b];
        if (c) atomicAdd(&acc[NCOUNTS + b], (u64)c);
    }
}

// What level 0 tells the host (written to host-visible memory by workgroup 0):
// how many kth_dist_level calls return a slot to all-reduce (level 0's
// included), so that every rank stops at the same call; the mode and W after
// level 0's pick; the host's tag of the call.
struct DistStatus {
    uint32_t levels, mode, W, tag;
};
constexpr int DIST_STATUS_WORDS = sizeof(DistStatus) / 4;

// kth_dist_scan's second kernel: this rank's candidates' first digit (the
// domain of cand_domain(lo, hi)) into the count slot a.stats_acc.  The window
// is in a.st_in (k_main's state).  Nothing to do when the window holds no key
// strictly inside or one value (W = 0: decide needs no digit).
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_dscan_hist(StepArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lh[DNB];
    const SelState *st = a.st_in;
    const uint32_t mode = st->mode, lo = st->lo, hi = st->hi;
    const u64 count = min(*a.cand_count, a.cap);
    if (mode != MODE_MAIN) return;
    const CandDom dm = cand_domain(lo, hi);
    if (dm.W == 0 || count == 0) return;
    const uint32_t active = (uint32_t)min((u64)gridDim.x, (count + a.min_per_wg - 1) / a.min_per_wg);
    if (blockIdx.x >= active) return;
    for (int i = threadIdx.x; i < DNB / 4; i += BLOCK) reinterpret_cast<uint4 *>(lh)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    dist_hist<BLOCK, false>(lh, a.cand, count, active, dm.base, dm.W, 0u, 0u, dm.d0, a.stats_acc);
}

// One level of the sharded protocol: the state (and at level 0 the decide),
// the pick, then the next digit's histogram over the candidates (MODE_CAND)
// or the shard (MODE_FULL): keys per workgroup a.min_per_wg for a digit under
// a resolved prefix (sparse), a.dense_per_wg for a domain's first digit (every
// key lands: the fallback's level 0).  Workgroup 0 publishes the state,
// clears the slot the next level accumulates into and (level 0) writes the
// DistStatus.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_dlevel(StepArgs a) {
    __shared__ SelState ss;
    __shared__ u64 scratch[2 * (BLOCK / WAVE) + 8];
    __shared__ u64 cnts[NCOUNTS];
    __shared__ __attribute__((aligned(16))) uint32_t lh[DNB];
    const u64 cand_n = min(*a.cand_count, a.cap);
    dist_state<BLOCK>(ss, a, cnts);
    {  // workgroups without keys to histogram leave before the pick's loads
        const uint32_t m = ss.mode;
        // the digit after the pick is a domain's first only for the fallback's
        // level 0 (no pick there); a live state otherwise picks one first
        const bool first = a.adv == ADV_DECIDE && m == MODE_FULL;
        const u64 count = m == MODE_CAND ? cand_n : m == MODE_FULL ? a.n_local : 0;
        const u64 per = first ? a.dense_per_wg : a.min_per_wg;
        if (blockIdx.x != 0 && (u64)blockIdx.x * per >= count) return;  // block-uniform
    }
    for (int i = threadIdx.x; i < DNB / 4; i += BLOCK) reinterpret_cast<uint4 *>(lh)[i] = make_uint4(0, 0, 0, 0);
    dist_pick<BLOCK>(ss, a, scratch);
    __syncthreads();
    const bool live = dist_live(ss);
    const uint32_t mode = ss.mode, W = ss.W, done = ss.t[0].done, prefix = ss.t[0].prefix, base = ss.base;
    const uint32_t d = live ? digit_bits(ss, done) : 0u;
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            *a.st_out = ss;
            if (a.host_status) {
                // this level's slot, then one per DDIG bits left after its digit
                const uint32_t left = live ? W - done - d : 0u;
                const uint32_t v[DIST_STATUS_WORDS] = {1u + (left + DDIG - 1) / DDIG, mode, W, a.tag};
#pragma unroll
                for (int i = 0; i < DIST_STATUS_WORDS; ++i)
                    __hip_atomic_store(&a.host_status[i], v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        if (a.stats_zero)
            for (int i = threadIdx.x; i < STATS_WORDS; i += BLOCK) a.stats_zero[i] = 0;
    }
    if (!live) return;  // block-uniform
    const u64 count = mode == MODE_CAND ? cand_n : a.n_local;
    const u64 per = done == 0 ? a.dense_per_wg : a.min_per_wg;
    const uint32_t active = (uint32_t)min((u64)gridDim.x, (count + per - 1) / per);
    if (blockIdx.x >= active) return;
    if (mode == MODE_FULL)
        dist_hist<BLOCK, true>(lh, reinterpret_cast<const uint32_t *>(a.keys), count, active, base, W, done, prefix,
                               d, a.stats_acc);
    else
        dist_hist<BLOCK, false>(lh, a.cand, count, active, base, W, done, prefix, d, a.stats_acc);
}

// The sharded protocol's last step: workgroup 0 picks the last digit and
// writes the answer (only a verified one reaches d_out); every workgroup
// zeroes its share of the ctx-internal slots (16-byte stores).
template <int BLOCK>
// early (kth_dist_result_early: enqueued before the host knows how many levels
// the protocol takes): every workgroup picks, and while the picked state is
// still live (more digits to come, no error) nothing is written or cleared --
// the protocol then goes on and its final k_dresult does the work.
__global__ __launch_bounds__(BLOCK) void k_dresult(StepArgs a, int32_t *d_out, int32_t *d_status, u64 *izero,
                                                   u64 izero_words, uint32_t early) {
    __shared__ SelState ss;
    __shared__ u64 scratch[2 * (BLOCK / WAVE) + 8];
    __shared__ u64 cnts[NCOUNTS];
    if (blockIdx.x == 0 || early) {  // grid-uniform
        dist_state<BLOCK>(ss, a, cnts);
        dist_pick<BLOCK>(ss, a, scratch);
        // early: leave only while the protocol goes on (a live state, no
        // error); a finished state -- an answer or an error -- is written
        // here, since kth_dist_result does not relaunch after one level
        if (early && dist_live(ss) && !ss.error) return;  // block-uniform (the same pick in every block)
    }
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            SelState o = ss;
            if (o.mode != MODE_DONE && !o.error) o.error = 16 + o.mode;
            *a.st_out = o;
            if (d_out && !o.error) *d_out = i32_of_key(o.answer);
            if (d_status) {
                d_status[0] = i32_of_key(o.answer);
                d_status[1] = (int32_t)o.error;
            }
        }
    }
    // (izero is 16-byte aligned; an odd word count leaves one u64)
    uint4 *z = reinterpret_cast<uint4 *>(izero);
    const u64 nz = izero_words / 2;
    for (u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x; i < nz; i += (u64)gridDim.x * BLOCK) z[i] = make_uint4(0, 0, 0, 0);
    if ((izero_words & 1) && blockIdx.x == 0 && threadIdx.x == 0) izero[izero_words - 1] = 0;
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
        if (d_out && ok) d_out[0] = i32_of_key(prefix);
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

// The local transport of a one-device sharded handle (kth_sharded.cpp): the
// all-reduce of one stats slot across the shards' slot buffers -- each word
// summed over the P shards and written back to every one of them.
constexpr int SLOTS_SUM_MAX = 64;  // == KTH_LOCAL_MAX_SHARDS
struct SlotPtrs {
    u64 *p[SLOTS_SUM_MAX];
};
__global__ __launch_bounds__(BLK) void k_slots_sum(SlotPtrs s, int P, u64 words) {
    for (u64 i = (u64)blockIdx.x * BLK + threadIdx.x; i < words; i += (u64)gridDim.x * BLK) {
        u64 sum = 0;
        for (int r = 0; r < P; ++r) sum += s.p[r][i];
        for (int r = 0; r < P; ++r) s.p[r][i] = sum;
    }
}

// The sharded handle's final read-back: every shard's [answer, error] words
// (the ctx's d_status, written by k_dresult) into one host-visible array, so
// one synchronisation reads them all.
struct StatusPtrs {
    const int32_t *p[SLOTS_SUM_MAX];
};
__global__ __launch_bounds__(WAVE) void k_status_gather(StatusPtrs src, int P, int32_t *dst) {
    for (int i = threadIdx.x; i < 2 * P; i += WAVE)
        __hip_atomic_store(&dst[i], src.p[i / 2][i % 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The local transport's window: every shard derives the same window from the
// same gathered sample, so on one device it is computed once (k_head on
// shard 0's ctx) and its state copied to the other shards' ctxs.
struct StatePtrs {
    SelState *p[SLOTS_SUM_MAX];
};
__global__ __launch_bounds__(BLK) void k_state_bcast(const SelState *src, StatePtrs dst, int P) {
    constexpr int SV = sizeof(SelState) / 16;
    for (int i = threadIdx.x; i < SV * P; i += BLK)
        reinterpret_cast<uint4 *>(dst.p[i / SV])[i % SV] = reinterpret_cast<const uint4 *>(src)[i % SV];
}

}  // namespace kth

#include "kth_coop.hpp"
#include "kth_rows.hpp"
