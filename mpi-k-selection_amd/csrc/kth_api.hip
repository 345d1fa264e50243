// kth_api.hip -- extern "C" boundary of libkth.so (include/kth.h).
//
// Host-side orchestration of the kernels in kth_kernels.hip: context and
// scratch management, path choice, the per-path launch sequences, timing
// events, and the per-rank steps of the sharded protocol.  No host
// synchronisation inside a select except in the synchronous wrappers, no
// allocation once a ctx is reserved, no CPU fallback: without a device every
// compute entry point returns KTH_ENODEV.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kth.h"
#include "kth_internal.h"
#include "kth_kernels.hip"
#include "kth_topk.hpp"

using kth::SelState;
using kth::StepArgs;
using kth::u64;

namespace {

constexpr int64_t SMALL_N = 16384;           // LDS path
constexpr int64_t RADIX_MAX_N = 1ll << 22;   // radix path up to here, window path above
constexpr int64_t SAMPLE_MAX = 1ll << 20;    // sample keys (single GPU / total over ranks)
constexpr double WINDOW_Z = 5.0;             // window half-width in sample standard deviations (two-sided miss 5.7e-7)
// KTH_WINDOW_Z overrides it (design exploration); read once
double window_z() {
    static const double z = [] {
        const char *e = getenv("KTH_WINDOW_Z");
        const double v = e ? atof(e) : 0.0;
        return v > 0.0 ? v : WINDOW_Z;
    }();
    return z;
}
constexpr int LEVEL_GRID_MAX = 1024;
constexpr int POST_DENSE_GRID = 256;  // the candidates need ~100 dense WGs; the rare fallback streams the input with 256
constexpr int HEAD_GRID_MAX = 64;  // k_head workgroups at most: 2^20 sample keys / (16 chunks of 1024 a workgroup)
int gather_grid(u64 nchunks) {
    const u64 per_wg = (u64)(kth::DENSE_BLK / kth::WAVE) * kth::GATHER_BATCH;  // chunks per workgroup round
    return (int)std::max<u64>(1, (nchunks + per_wg - 1) / per_wg);
}
constexpr size_t ISLOT_WORDS = 3 * (size_t)kth::STATS_WORDS + 2;  // 3 slots + cand_count + pad
// after the islots, in the same allocation: k_head's and k_finish's level
// slots (zero between selects), then the grid-barrier words (never cleared by
// a select: the barrier resets itself)
constexpr size_t HSLOT_OFF = ISLOT_WORDS;
constexpr size_t HSLOT_WORDS = (size_t)kth::HEAD_LEVELS * kth::STATS_WORDS;
constexpr size_t FSLOT_OFF = HSLOT_OFF + HSLOT_WORDS;  // two sets, alternate k_finish launches
constexpr size_t FSLOT_WORDS = (size_t)kth::FIN_LEVELS * kth::STATS_WORDS;
constexpr size_t PRE_OFF = FSLOT_OFF + 2 * FSLOT_WORDS;  // two PreHist sets (u32 words), alternate selects
constexpr size_t PRE_SET_WORDS = (size_t)kth::PRE_WORDS / 2;  // (in u64 words)
static_assert(kth::PRE_WORDS % 4 == 0, "PreHist sets stay 16-byte aligned");
constexpr size_t ZERO_WORDS = PRE_OFF + 2 * PRE_SET_WORDS;
constexpr size_t BAR_OFF = ZERO_WORDS;
constexpr size_t TAIL_OFF = BAR_OFF + kth::BAR_WORDS / 2;  // k_finish's tail keys (FIN_LDS_KEYS u32)
constexpr size_t SLOT_ALLOC_WORDS = TAIL_OFF + kth::FIN_LDS_KEYS / 2;
static_assert(kth::BAR_TAIL % 2 == 0, "the tail word is a u64");
constexpr u64 FIN_SPARSE_PER_WG = (u64)kth::DENSE_BLK * kth::FIN_UNROLL * 4;  // one k_finish tile
constexpr double HEAD_SLACK = 1.5;  // k_head early window (EarlyWindow); KTH_HEAD_SLACK overrides, 0 = off
static_assert(KTH_STATS_WORDS == kth::STATS_WORDS, "include/kth.h slot size");
constexpr int MAX_EVENTS = 4 * 2048;
constexpr u64 TK_STAGE_MAX_FRAC = 16;  // staged top-k (k_main<5/6>) for k <= n / 16
constexpr int TK5_SPLIT = 4;            // workgroups per k_main workgroup in k_tk5_count / k_tk5_write (window-parallel)
constexpr int COOP_BACKOFF = 64;        // synchronous selects on the per-level path after a grid-barrier timeout
constexpr uint64_t DSCAN_PER_WG = 1ull << 16;  // candidates per workgroup of the sharded scan's first-digit histogram

#define HIP_TRY(x)                                                                                    \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) {                                                                       \
            if (getenv("KTH_DEBUG")) fprintf(stderr, "kth: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return KTH_EHIP;                                                                          \
        }                                                                                             \
    } while (0)

#define KTH_TRY(x)              \
    do {                        \
        int r_ = (x);           \
        if (r_ != KTH_OK) return r_; \
    } while (0)

}  // namespace

struct kth_ctx {
    int device = 0;
    int main_grid[7] = {0, 0, 0, 0, 0, 0, 0};  // streaming-pass workgroups per k_main<TF> variant (KTH_MAIN_WG_PER_CU overrides)
    bool fault_topk_rank = false;  // KTH_HOOK_FAULT_TOPK_RANK (tests): top-k selects a wrong rank on purpose
    bool fault_barrier = false;    // KTH_HOOK_FAULT_BARRIER (tests): the grid barriers report a timeout
    bool fault_once = false;       // (value 2) only the next cooperative launch does
    bool topk_stage = true;        // staged top-k (k_main<5/6>); KTH_TOPK_STAGE=0 turns it off
    u64 topk_seg_cap = 0;          // KTH_HOOK_TOPK_SEG_CAP (tests): entries per staging segment (0 = sized from n)
    u64 sparse_per_wg = 0;  // keys per workgroup of the sparse levels (KTH_SPARSE_PER_WG; 0 = default)
    int post_dense_grid = POST_DENSE_GRID;    // decide level after the pass (KTH_POST_DENSE_GRID)
    int post_sparse_grid = LEVEL_GRID_MAX;    // candidate levels (KTH_POST_SPARSE_GRID)
    bool coop = true;          // window / radix paths as k_head + k_main + k_finish (KTH_COOP=0: per-level launches)
    bool coop_wanted = true;   // coop as configured (env, LDS, residency); coop may be off for a while after a timeout
    int coop_backoff = 0;      // synchronous selects left on the per-level path after a grid-barrier timeout
    bool coop_resident = true; // the cooperative grids fit the device at once (occupancy check at ctx creation)
    int fin_grid = 256;        // k_finish workgroups (one per CU; KTH_FIN_GRID)
    uint32_t head_slack64 = (uint32_t)(HEAD_SLACK * 64);
    uint32_t head_abs_div = 1024;  // plain select: early-window floor s / head_abs_div sample keys (KTH_HEAD_ABS; 0 = off)
    int fin_set = 0;           // k_finish slot set of the next launch (the other one is cleared by it)
    bool pre_hist = true;      // k_main<0> histograms the candidates' first digit for k_finish (KTH_PRE_HIST=0: off)
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int num_cu = 256;
    SelState *st = nullptr;   // 2 states (ping-pong)
    u64 *islots = nullptr;    // ISLOT_WORDS
    uint32_t *sample = nullptr;
    u64 sample_cap = 0;
    uint32_t *cand = nullptr;
    u64 cand_cap = 0;
    uint32_t *cand_rows = nullptr;  // k_main<3/4>: each candidate's 1024-key row (top-k)
    u64 cand_rows_cap = 0;
    // k_main<5/6> (top-k): per-wave segments of staged keys + positions, per wave-row counts
    int32_t *tk_segv = nullptr;
    u64 tk_segv_cap = 0;
    uint8_t *tk_segp = nullptr;
    u64 tk_segp_cap = 0;
    uint32_t *tk_wcnt = nullptr;
    u64 tk_wcnt_cap = 0;
    uint32_t *tk_wstart = nullptr;  // staged top-k: entries before each window, per wave
    u64 tk_wstart_cap = 0;
    kth::TkSeg tk_seg{};  // the segments of the next launch_main<5/6>
    int32_t *staging = nullptr;
    u64 staging_cap = 0;
    u64 *topk = nullptr;  // top-k chunk counts, bases, [need, error]
    u64 topk_cap = 0;
    int32_t *d_status = nullptr;  // [answer, error]
    int32_t *h_status = nullptr;  // pinned
    SelState *h_state = nullptr;  // pinned
    int last_state = -1;
    // timing: event pairs around the streaming pass and around whole selects
    bool timing = false;
    std::vector<hipEvent_t> ev_main, ev_total;
    int main_used = 0, total_used = 0;
    bool dirty = false;  // a launch sequence was cut short: re-zero the slots
    bool dist_zero = false;  // sharded: the bound slots still need clearing
    bool dist_open = false;  // sharded: begun, kth_dist_result not yet enqueued
    bool dist_coop_window = false;  // sharded: the window came from k_head (state carried, no pick left)
    bool counts_left = false;  // a cooperative window select left islot(1) / cand_count for the next k_head to clear
    // KTH_STAMPS=1 diagnostics: per-launch [WG][8] wall-clock stamps, dumped after each select
    u64 *stamps = nullptr;
    int stamp_next = 0;
    // sharded protocol
    u64 *uslots = nullptr;
    int64_t dist_n = 0, dist_k = 0, dist_cap = 0;
    int dist_level_next = 0;   // the next kth_dist_level call's level (-1: none expected)
    u64 dscan_per_wg = DSCAN_PER_WG;  // k_dscan_hist keys per workgroup (KTH_DSCAN_PER_WG)
    int dist_levels = -1;      // level calls that return a slot (from level 0's DistStatus; -1: unknown yet)
    int dist_result_slot = -1; // the slot the last level accumulated into (kth_dist_result reads it)
    int32_t *dist_early_out = nullptr;  // kth_dist_result_early's answer buffer this select (null: none)
    uint32_t *h_dist = nullptr;  // DistStatus, host-visible (pinned, mapped), written by level 0's k_dlevel
    uint32_t *d_dist = nullptr;  // ... its device address
    hipEvent_t ev_dist = nullptr;  // recorded after level 0
    uint32_t dist_tag = 0;     // level 0 calls so far (the DistStatus tag)
};

namespace {

u64 *islot(kth_ctx *c, int i) { return c->islots + (size_t)i * kth::STATS_WORDS; }
u64 *cand_count(kth_ctx *c) { return c->islots + 3 * (size_t)kth::STATS_WORDS; }

int set_device(kth_ctx *c) {
    HIP_TRY(hipSetDevice(c->device));
    return KTH_OK;
}

int grow(void **p, u64 *cap, u64 want_bytes) {
    if (*cap >= want_bytes) return KTH_OK;
    (void)hipDeviceSynchronize();  // in-flight work may still use the old buffer
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc(p, want_bytes) != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        return KTH_ENOMEM;
    }
    *cap = want_bytes;
    return KTH_OK;
}

u64 cand_capacity(int64_t n) { return std::max<u64>(1ull << 20, (u64)n / 32); }

int64_t sample_size(int64_t n) {
    int64_t s = (n / 64) & ~int64_t(63);
    return std::min<int64_t>(SAMPLE_MAX, std::max<int64_t>(s, 64));
}

int reserve_cand(kth_ctx *c, int64_t n) {
    u64 bytes = cand_capacity(n) * 4;
    return grow(reinterpret_cast<void **>(&c->cand), &c->cand_cap, bytes);
}

// Window ranks in a sample of s keys for rank k of n: +-Z sample sigmas.
void window_ranks(int64_t n, int64_t k, int64_t s, u64 *r_lo, u64 *r_hi) {
    const double p = (double)k / (double)n;
    const double r = p * (double)s;
    const double sig = std::sqrt(std::max(1.0, (double)s * p * (1.0 - p)));
    const double z = window_z();
    const double lo = std::floor(r - z * sig - 2.0), hi = std::ceil(r + z * sig + 2.0);
    *r_lo = lo < 1.0 ? 0 : (u64)lo;                       // 0 = no lower bound
    *r_hi = hi > (double)s ? (u64)s + 1 : (u64)std::max(1.0, hi);  // s+1 = no upper bound
}

constexpr int STAMP_LAUNCHES = 16, STAMP_WGS = 4096;
u64 *next_stamps(kth_ctx *c) {
    if (!c->stamps || c->stamp_next >= STAMP_LAUNCHES) return nullptr;
    return c->stamps + (size_t)(c->stamp_next++) * STAMP_WGS * 8;
}

// Per launch of the last select: WGs, and mean / max of each stamp relative to
// the launch's first entry, then the gap to the next launch (microseconds).
void dump_stamps(kth_ctx *c) {
    if (!c->stamps) return;
    std::vector<u64> h((size_t)STAMP_LAUNCHES * STAMP_WGS * 8);
    (void)hipStreamSynchronize(c->stream);
    (void)hipMemcpy(h.data(), c->stamps, h.size() * 8, hipMemcpyDeviceToHost);
    u64 prev_end = 0;
    for (int l = 0; l < c->stamp_next; ++l) {
        const u64 *b = h.data() + (size_t)l * STAMP_WGS * 8;
        u64 t0 = ~0ull, tend = 0;
        int nwg = 0;
        for (int w = 0; w < STAMP_WGS; ++w)
            if (b[w * 8]) {
                nwg++;
                t0 = std::min(t0, b[w * 8]);
                for (int i = 0; i < 8; ++i) tend = std::max(tend, b[w * 8 + i]);
            }
        if (!nwg) continue;
        fprintf(stderr, "kth-stamps launch %d wgs %4d gap %7.2f |", l, nwg, prev_end ? (t0 - prev_end) / 100.0 : 0.0);
        for (int i = 0; i < 8; ++i) {
            double sum = 0, mx = 0;
            int cnt = 0;
            for (int w = 0; w < STAMP_WGS; ++w)
                if (b[w * 8] && b[w * 8 + i]) {
                    const double d = (b[w * 8 + i] - t0) / 100.0;
                    sum += d;
                    mx = std::max(mx, d);
                    cnt++;
                }
            if (cnt) fprintf(stderr, " p%d %6.2f/%6.2f", i, sum / cnt, mx);
        }
        fprintf(stderr, "\n");
        if (nwg >= 512) {  // end times (p5): percentiles over workgroups, and per blockIdx % 8
            std::vector<double> e;
            std::vector<double> ex[8];
            for (int w = 0; w < STAMP_WGS; ++w)
                if (b[w * 8] && b[w * 8 + 5]) {
                    const double d = (b[w * 8 + 5] - t0) / 100.0;
                    e.push_back(d);
                    ex[w % 8].push_back(d);
                }
            std::sort(e.begin(), e.end());
            if (!e.empty()) {
                auto pc = [&](double q) { return e[std::min(e.size() - 1, (size_t)(q * (double)e.size()))]; };
                fprintf(stderr, "kth-stamps   p5 pct: 1%% %.1f 10%% %.1f 25%% %.1f 50%% %.1f 75%% %.1f 90%% %.1f 99%% %.1f max %.1f\n",
                        pc(0.01), pc(0.10), pc(0.25), pc(0.50), pc(0.75), pc(0.90), pc(0.99), e.back());
                fprintf(stderr, "kth-stamps   p5 mean by wg%%8:");
                for (int x = 0; x < 8; ++x) {
                    double sm = 0;
                    for (double d : ex[x]) sm += d;
                    fprintf(stderr, " %.1f", ex[x].empty() ? 0.0 : sm / ex[x].size());
                }
                fprintf(stderr, "\n");
            }
        }
        if (nwg >= 512) {  // streaming pass: finish times (p3) by blockIdx % 8 (XCD under round-robin dispatch)
            for (int x = 0; x < 8; ++x) {
                double sum = 0, mn = 1e30, mx = 0;
                int cnt = 0;
                for (int w = x; w < STAMP_WGS; w += 8)
                    if (b[w * 8] && b[w * 8 + 3]) {
                        const double d = (b[w * 8 + 3] - t0) / 100.0;
                        sum += d;
                        mn = std::min(mn, d);
                        mx = std::max(mx, d);
                        cnt++;
                    }
                if (cnt) fprintf(stderr, "kth-stamps   wg%%8=%d p3 min %7.2f mean %7.2f max %7.2f\n", x, mn, sum / cnt, mx);
            }
        }
        prev_end = tend;
    }
    (void)hipMemsetAsync(c->stamps, 0, h.size() * 8, c->stream);
    c->stamp_next = 0;
}

StepArgs step(kth_ctx *c, int adv, int st_in, int st_out, const u64 *in, u64 *acc, u64 *zero) {
    StepArgs a;
    memset(&a, 0, sizeof a);
    a.stamps = next_stamps(c);
    a.st_in = st_in >= 0 ? c->st + st_in : nullptr;
    a.st_out = c->st + st_out;
    a.stats_in = in;
    a.stats_acc = acc;
    a.stats_zero = zero;
    a.adv = adv;
    a.cand = c->cand;
    a.cand_count = cand_count(c);
    a.cap = c->cand_cap / 4;
    return a;
}

// Record one event of a (start, end) pair; pairs are never split because the
// pool sizes are even and start/end are always recorded together.
void ev_mark(kth_ctx *c, std::vector<hipEvent_t> &pool, int &used) {
    if (!c->timing || used >= (int)pool.size()) return;
    (void)hipEventRecord(pool[used++], c->stream);
}
void ev_main(kth_ctx *c) { ev_mark(c, c->ev_main, c->main_used); }

int launch_check() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        if (getenv("KTH_DEBUG")) fprintf(stderr, "kth: launch failed: %s\n", hipGetErrorString(e));
        return KTH_EHIP;
    }
    return KTH_OK;
}

// Histogram levels.  Dense levels (every key of the domain lands in the
// histogram: the first digit of a domain) run few 1024-thread workgroups of
// DENSE_PER_WG keys, so at most ~domain/DENSE_PER_WG workgroups add to each
// global bin; sparse levels (only keys matching the prefix) run many small ones.
constexpr u64 DENSE_PER_WG = 1ull << 16;
constexpr u64 SPARSE_PER_WG = (u64)kth::BLK * kth::LEVEL_UNROLL * 4;

int level_grid(u64 count, u64 per_wg) {
    u64 g = (count + per_wg - 1) / per_wg;
    return (int)std::max<u64>(1, std::min<u64>(LEVEL_GRID_MAX, g));
}

u64 sparse_wg(const kth_ctx *c) { return c->sparse_per_wg ? c->sparse_per_wg : SPARSE_PER_WG; }

void launch_level(kth_ctx *c, StepArgs a, bool dense, int grid) {
    if (dense) {
        a.min_per_wg = DENSE_PER_WG;
        kth::k_level<kth::DENSE_BLK><<<grid, kth::DENSE_BLK, 0, c->stream>>>(a);
    } else {
        a.min_per_wg = sparse_wg(c);
        kth::k_level<kth::BLK><<<grid, kth::BLK, 0, c->stream>>>(a);
    }
}

// ---------------------------------------------------------------- paths
int run_small(kth_ctx *c, const int32_t *keys, int64_t n, int64_t k, int32_t *d_out, int32_t *d_status) {
    c->last_state = 1;
    ev_main(c);
    kth::k_small<<<1, kth::SMALL_BLOCK, (size_t)n * 4, c->stream>>>(keys, (u64)n, (u64)k, d_out, d_status,
                                                                    c->st + 1);
    ev_main(c);
    return launch_check();
}

kth::CoopArgs coop_args(kth_ctx *c, u64 slot_off, int32_t *d_out, int32_t *d_status) {
    kth::CoopArgs x;
    memset(&x, 0, sizeof x);
    x.slots = c->islots + slot_off;
    x.bar = reinterpret_cast<uint32_t *>(c->islots + BAR_OFF);
    x.tail = reinterpret_cast<uint32_t *>(c->islots + TAIL_OFF);
    x.d_out = d_out;
    x.d_status = d_status;
    x.dense_per_wg = DENSE_PER_WG;
    x.sparse_per_wg = FIN_SPARSE_PER_WG;
    x.slack64 = c->head_slack64;
    x.fault = c->fault_barrier ? 1u : 0u;
    if (c->fault_once) c->fault_barrier = false;
    return x;
}

// k_finish: the finish phase in one launch, on slot set fin_set; it clears the
// other set and the sample phase's slots for the next select
constexpr size_t FIN_DYN_LDS = (size_t)kth::FIN_LDS_KEYS * 4;
uint32_t *pre_set(kth_ctx *c, int set) {
    return reinterpret_cast<uint32_t *>(c->islots + PRE_OFF + (size_t)set * PRE_SET_WORDS);
}

// with_pre: this select's k_main<0> histogrammed the candidates' first digit
// into PreHist set fin_set
void launch_finish(kth_ctx *c, StepArgs a, int32_t *d_out, int32_t *d_status, bool with_pre = false) {
    const size_t mine = FSLOT_OFF + (size_t)c->fin_set * FSLOT_WORDS;
    a.stats_zero = c->islots + FSLOT_OFF + (size_t)(1 - c->fin_set) * FSLOT_WORDS;
    a.zero_words = FSLOT_WORDS;
    kth::CoopArgs x = coop_args(c, mine, d_out, d_status);
    x.zero2 = c->islots + HSLOT_OFF;
    x.zero2_words = HSLOT_WORDS;
    x.pre = with_pre ? pre_set(c, c->fin_set) : nullptr;
    x.pre_zero = pre_set(c, 1 - c->fin_set);
    kth::k_finish<<<c->fin_grid, kth::DENSE_BLK, FIN_DYN_LDS, c->stream>>>(a, x);
    c->fin_set ^= 1;
}

int run_radix(kth_ctx *c, const int32_t *keys, int64_t n, int64_t k, int32_t *d_out, int32_t *d_status) {
    if (c->coop) {  // three radix levels over the input in one launch
        StepArgs a = step(c, kth::ADV_INIT_FULL, -1, 1, nullptr, nullptr, nullptr);
        a.keys = keys;
        a.n_local = (u64)n;
        a.init_n = (u64)n;
        a.init_k = (u64)k;
        ev_main(c);
        launch_finish(c, a, d_out, d_status);
        ev_main(c);
        c->last_state = 1;
        return launch_check();
    }
    StepArgs a = step(c, kth::ADV_INIT_FULL, -1, 0, nullptr, islot(c, 1), islot(c, 2));
    a.keys = keys;
    a.n_local = (u64)n;
    a.init_n = (u64)n;
    a.init_k = (u64)k;
    ev_main(c);  // the first radix pass is the dominant kernel here
    launch_level(c, a, true, level_grid((u64)n, DENSE_PER_WG));
    ev_main(c);
    a = step(c, kth::ADV_PICK, 0, 1, islot(c, 1), islot(c, 2), islot(c, 0));
    a.keys = keys;
    a.n_local = (u64)n;
    launch_level(c, a, false, level_grid((u64)n, sparse_wg(c)));
    a = step(c, kth::ADV_PICK, 1, 0, islot(c, 2), islot(c, 0), islot(c, 1));
    a.keys = keys;
    a.n_local = (u64)n;
    launch_level(c, a, false, level_grid((u64)n, sparse_wg(c)));
    a = step(c, kth::ADV_PICK, 0, 1, islot(c, 0), nullptr, nullptr);
    kth::k_result<<<1, kth::BLK, 0, c->stream>>>(a, d_out, d_status, c->islots, ISLOT_WORDS);
    c->last_state = 1;
    return launch_check();
}

// The streaming pass, plain (tflag 0) or with the top-k records of k_main<tflag>.
void launch_main(kth_ctx *c, const StepArgs &a, int tflag, uint32_t *tflags) {
    const int g = c->main_grid[tflag];
    const kth::TkSeg none{};
    switch (tflag) {
    case 1: kth::k_main<1><<<g, kth::BLK, 0, c->stream>>>(a, c->cand, tflags, nullptr, none); break;
    case 2: kth::k_main<2><<<g, kth::BLK, 0, c->stream>>>(a, c->cand, tflags, nullptr, none); break;
    case 3: kth::k_main<3><<<g, kth::BLK, 0, c->stream>>>(a, c->cand, tflags, c->cand_rows, none); break;
    case 4: kth::k_main<4><<<g, kth::BLK, 0, c->stream>>>(a, c->cand, tflags, c->cand_rows, none); break;
    case 5: kth::k_main<5><<<g, kth::BLK, 0, c->stream>>>(a, c->cand, tflags, nullptr, c->tk_seg); break;
    case 6: kth::k_main<6><<<g, kth::BLK, 0, c->stream>>>(a, c->cand, tflags, nullptr, c->tk_seg); break;
    default: kth::k_main<0><<<g, kth::BLK, 0, c->stream>>>(a, c->cand, nullptr, nullptr, none); break;
    }
}

// The main pass + candidate levels + result, shared by the single-GPU window
// path.  Expects the window state in st[0] and the last sample digit's
// histogram in islot(0).
int run_window(kth_ctx *c, const int32_t *keys, int64_t n, int64_t k, int32_t *d_out, int32_t *d_status,
               int tflag = 0, uint32_t *tflags = nullptr) {
    const int64_t s = sample_size(n);
    const u64 nchunks = ((u64)s + kth::SAMPLE_CHUNK - 1) / kth::SAMPLE_CHUNK;
    const u64 stride = (u64)n / nchunks;
    u64 r_lo, r_hi;
    window_ranks(n, k, s, &r_lo, &r_hi);
    KTH_TRY(grow(reinterpret_cast<void **>(&c->sample), &c->sample_cap, (u64)s * 4));
    KTH_TRY(reserve_cand(c, n));

    if (c->coop) {
        // sample phase in one launch -> window state in st[0]
        // (it also clears the streaming pass's count slot islot(1) and the candidate count)
        StepArgs a = step(c, kth::ADV_INIT_SAMPLE, -1, 0, nullptr, nullptr, islot(c, 1));
        a.zero_words = 2 * (u64)kth::STATS_WORDS + 1;
        a.init_n = (u64)n;
        a.init_k = (u64)k;
        a.init_s = (u64)s;
        a.r_lo = r_lo;
        a.r_hi = r_hi;
        // the plain select takes a first-level window of up to s / head_abs_div
        // sample keys (~n / 1024 candidates) whatever the slack: at k near 1 or
        // n it spares the second sample level (the top-k variants keep the
        // narrow window: their count pass loads the rows below its far edge).
        // Sorted input at k = 1 / n: 0.672-0.675 -> 0.654-0.658 ms; uniform
        // keys unchanged (their edge bin holds ~1024 sample keys: s / 256 took
        // them, ~1 M candidates, and cost ~10 us more than the level saves)
        kth::CoopArgs hx = coop_args(c, HSLOT_OFF, nullptr, nullptr);
        if (tflag == 0 && c->head_abs_div) hx.abs_min = (u64)s / c->head_abs_div;
        kth::k_head<<<gather_grid(nchunks), kth::DENSE_BLK, 0, c->stream>>>(a, hx, keys, (u64)n, stride, c->sample,
                                                                          (u64)s);
        // the streaming pass: counts into islot(1) (zero between selects);
        // the plain pass also histograms the candidates' first digit for k_finish
        a = step(c, kth::ADV_CARRY, 0, 1, nullptr, islot(c, 1), nullptr);
        a.keys = keys;
        a.n_local = (u64)n;
        const bool pre = tflag == 0 && c->pre_hist;
        if (pre) a.pre_hist = pre_set(c, c->fin_set);
        ev_main(c);
        launch_main(c, a, tflag, tflags);
        ev_main(c);
        // decide + candidate (or fallback) levels + answer in one launch
        a = step(c, kth::ADV_DECIDE, 1, 0, islot(c, 1), nullptr, nullptr);
        a.keys = keys;
        a.n_local = (u64)n;
        launch_finish(c, a, d_out, d_status, pre);
        c->last_state = 0;
        c->counts_left = true;  // (k_head clears them; a sharded select on this ctx must too)
        return launch_check();
    }
    // sample + first digit of the sample
    StepArgs a = step(c, kth::ADV_INIT_SAMPLE, -1, 0, nullptr, islot(c, 1), islot(c, 2));
    a.init_n = (u64)n;
    a.init_k = (u64)k;
    a.init_s = (u64)s;
    a.r_lo = r_lo;
    a.r_hi = r_hi;
    kth::k_gather<true><<<gather_grid(nchunks), kth::DENSE_BLK, 0, c->stream>>>(a, keys, (u64)n, stride, c->sample,
                                                                              (u64)s);
    // digits 2, 3 of the sample ranks (sparse: only keys in the picked bins)
    const int gs = level_grid((u64)s, sparse_wg(c));
    a = step(c, kth::ADV_PICK, 0, 1, islot(c, 1), islot(c, 2), islot(c, 0));
    a.sample = c->sample;
    a.sample_count = (u64)s;
    launch_level(c, a, false, gs);
    a = step(c, kth::ADV_PICK, 1, 0, islot(c, 2), islot(c, 0), islot(c, 1));
    a.sample = c->sample;
    a.sample_count = (u64)s;
    launch_level(c, a, false, gs);
    // the streaming pass
    a = step(c, kth::ADV_PICK, 0, 1, islot(c, 0), islot(c, 1), islot(c, 2));
    a.keys = keys;
    a.n_local = (u64)n;
    ev_main(c);
    launch_main(c, a, tflag, tflags);
    ev_main(c);
    // decide + candidate (or fallback) levels.  The grids cover the fallback
    // (whole input); in the common case only the WGs the candidates need run.
    a = step(c, kth::ADV_DECIDE, 1, 0, islot(c, 1), islot(c, 2), islot(c, 0));
    a.keys = keys;
    a.n_local = (u64)n;
    launch_level(c, a, true, c->post_dense_grid);
    a = step(c, kth::ADV_PICK, 0, 1, islot(c, 2), islot(c, 0), islot(c, 1));
    a.keys = keys;
    a.n_local = (u64)n;
    launch_level(c, a, false, c->post_sparse_grid);
    a = step(c, kth::ADV_PICK, 1, 0, islot(c, 0), islot(c, 1), islot(c, 2));
    a.keys = keys;
    a.n_local = (u64)n;
    launch_level(c, a, false, c->post_sparse_grid);
    a = step(c, kth::ADV_PICK, 0, 1, islot(c, 1), nullptr, nullptr);
    kth::k_result<<<1, kth::BLK, 0, c->stream>>>(a, d_out, d_status, c->islots, ISLOT_WORDS);
    c->last_state = 1;
    return launch_check();
}

// After a grid-barrier timeout the cooperative kernels stay off for
// COOP_BACKOFF selections of any entry point (synchronous, asynchronous,
// top-k, sharded); each one counts down here, then they are tried again.
void coop_tick(kth_ctx *c) {
    if (c->coop_backoff > 0 && --c->coop_backoff == 0) c->coop = c->coop_wanted;
}

int select_async(kth_ctx *c, const int32_t *d_keys, int64_t n, int64_t k, int32_t *d_out, int32_t *d_status,
                 int tflag = 0, uint32_t *tflags = nullptr) {
    if (!c || !d_keys || (!d_out && !d_status) || n < 1 || k < 1 || k > n) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    coop_tick(c);
    if (c->dirty) {
        HIP_TRY(hipMemsetAsync(c->islots, 0, SLOT_ALLOC_WORDS * sizeof(u64), c->stream));
        c->dirty = false;
    }
    int rc;
    ev_mark(c, c->ev_total, c->total_used);
    if (n <= SMALL_N)
        rc = run_small(c, d_keys, n, k, d_out, d_status);
    else if (n <= RADIX_MAX_N)
        rc = run_radix(c, d_keys, n, k, d_out, d_status);
    else
        rc = run_window(c, d_keys, n, k, d_out, d_status, tflag, tflags);
    ev_mark(c, c->ev_total, c->total_used);
    if (rc != KTH_OK) c->dirty = true;
    if (c->stamps) dump_stamps(c);
    return rc;
}

bool is_device_ptr(const void *p) {
    hipPointerAttribute_t at;
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

thread_local kth_ctx *tl_ctx = nullptr;

// Rows: the wave-per-row register kernel (kth_rows.hpp) for cols <= 4096,
// KPL keys per lane; the LDS workgroup-per-row kernel above that.
#ifndef KTH_ROWS_R0
#define KTH_ROWS_R0 4  // first-pass histogram copies per wave in k_rows_reg
#endif
template <bool F32, int KPL, bool TOPK>
void launch_rows_reg(kth_ctx *c, bool vec, int g, const uint32_t *d_keys, u64 R, uint32_t C, uint32_t K,
                     uint32_t *d_out, uint32_t flip, uint32_t *vals, int32_t *idx) {
    if (vec && C == (uint32_t)(KPL * kth::WAVE))
        kth::k_rows_reg<F32, KPL, true, KTH_ROWS_R0, TOPK, true>
            <<<g, kth::RW_BLOCK, 0, c->stream>>>(d_keys, R, C, K, d_out, flip, vals, idx);
    else if (vec)
        kth::k_rows_reg<F32, KPL, true, KTH_ROWS_R0, TOPK, false>
            <<<g, kth::RW_BLOCK, 0, c->stream>>>(d_keys, R, C, K, d_out, flip, vals, idx);
    else
        kth::k_rows_reg<F32, KPL, false, KTH_ROWS_R0, TOPK, false>
            <<<g, kth::RW_BLOCK, 0, c->stream>>>(d_keys, R, C, K, d_out, flip, vals, idx);
}

// k-th per row (TOPK = false, into d_out) or top-k per row (into vals / idx;
// cols <= KTH_TOPK_MAX_COLS, checked by the caller).
template <bool F32, bool TOPK>
int launch_rows(kth_ctx *c, const uint32_t *d_keys, int64_t rows, int32_t cols, int32_t k, uint32_t *d_out,
                uint32_t flip = 0, uint32_t *vals = nullptr, int32_t *idx = nullptr) {
    const bool vec = (reinterpret_cast<uintptr_t>(d_keys) & 15u) == 0 && cols % 4 == 0;
    const int rows_per_wg = kth::RW_BLOCK / kth::WAVE;
    const int64_t g64 = (rows + rows_per_wg - 1) / rows_per_wg;  // one row per wave
    if (g64 > 0x7FFFFFFF) return KTH_EINVAL;
    const int g = (int)g64;
    const u64 R = (u64)rows;
    const uint32_t C = (uint32_t)cols, K = (uint32_t)k;
    if (cols <= 1024)
        launch_rows_reg<F32, 16, TOPK>(c, vec, g, d_keys, R, C, K, d_out, flip, vals, idx);
    else if (cols <= 2048)
        launch_rows_reg<F32, 32, TOPK>(c, vec, g, d_keys, R, C, K, d_out, flip, vals, idx);
    else if (cols <= 4096)
        launch_rows_reg<F32, 64, TOPK>(c, vec, g, d_keys, R, C, K, d_out, flip, vals, idx);
    else if (!TOPK)
        kth::k_rows<F32><<<(int)std::min<int64_t>(rows, 1 << 20), kth::ROWS_BLOCK, (size_t)cols * 4, c->stream>>>(
            d_keys, R, C, (u64)k, d_out);
    return launch_check();
}

}  // namespace

// ====================================================================== API
extern "C" {

const char *kth_strerror(int code) {
    switch (code) {
    case KTH_OK: return "ok";
    case KTH_EINVAL: return "invalid argument";
    case KTH_ENOMEM: return "out of memory";
    case KTH_EHIP: return "HIP runtime error";
    case KTH_ENODEV: return "no HIP device";
    case KTH_EINTERNAL: return "device-side consistency check failed";
    case KTH_ECOMM: return "RCCL unavailable or a collective failed";
    default: return "unknown error";
    }
}

int kth_version(void) { return KTH_VERSION; }

#ifndef KTH_BUILD_ID
#define KTH_BUILD_ID "unknown"
#endif
const char *kth_build_id(void) { return KTH_BUILD_ID; }

int kth_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int kth_ctx_create(int device, kth_ctx **out) {
    if (!out) return KTH_EINVAL;
    *out = nullptr;
    int ndev = kth_device_count();
    if (ndev <= 0) return KTH_ENODEV;
    if (device < 0 || device >= ndev) return KTH_EINVAL;
    kth_ctx *c = new kth_ctx();
    c->device = device;
    if (getenv("KTH_STAMPS")) {
        const size_t bytes = (size_t)STAMP_LAUNCHES * STAMP_WGS * 8 * 8;
        if (hipMalloc(reinterpret_cast<void **>(&c->stamps), bytes) != hipSuccess || hipMemset(c->stamps, 0, bytes) != hipSuccess) {
            (void)hipGetLastError();
            c->stamps = nullptr;
        }
    }
    int rc = KTH_OK;
    do {
        if (hipSetDevice(device) != hipSuccess) { rc = KTH_EHIP; break; }
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            c->num_cu = prop.multiProcessorCount;
        {
            // One resident wave of workgroups: every WG streams an equal share
            // and no tail of late WGs.  Residency from each k_main variant's own
            // VGPR and LDS use (4 waves per 256-thread WG = one per SIMD; a SIMD
            // holds 512 / alloc(VGPR) waves, MI355X_MICROARCH.md register files);
            // the top-k variants keep more keys live and may allocate more VGPRs.
            // hipOccupancyMaxActiveBlocksPerMultiprocessor under-reports here.
            const void *fns[7] = {reinterpret_cast<const void *>(kth::k_main<0>),
                                  reinterpret_cast<const void *>(kth::k_main<1>),
                                  reinterpret_cast<const void *>(kth::k_main<2>),
                                  reinterpret_cast<const void *>(kth::k_main<3>),
                                  reinterpret_cast<const void *>(kth::k_main<4>),
                                  reinterpret_cast<const void *>(kth::k_main<5>),
                                  reinterpret_cast<const void *>(kth::k_main<6>)};
            const char *e = getenv("KTH_MAIN_WG_PER_CU");
            for (int v = 0; v < 7; ++v) {
                int per = 4;
                hipFuncAttributes fa;
                if (hipFuncGetAttributes(&fa, fns[v]) == hipSuccess && fa.numRegs > 0) {
                    const int alloc = (fa.numRegs + 7) / 8 * 8;
                    const int by_vgpr = std::min(8, 512 / alloc);
                    const int lds = (int)fa.sharedSizeBytes;
                    const int by_lds = lds > 0 ? (160 * 1024) / lds : 8;
                    per = std::max(1, std::min(by_vgpr, by_lds));
                }
                (void)hipGetLastError();
                if (e && atoi(e) > 0) per = atoi(e);
                c->main_grid[v] = c->num_cu * per;
            }
            if (const char *g = getenv("KTH_SPARSE_PER_WG")) c->sparse_per_wg = (u64)std::max(0, atoi(g));
            if (const char *g = getenv("KTH_DSCAN_PER_WG")) c->dscan_per_wg = (u64)std::max(1024, atoi(g));
            if (const char *g = getenv("KTH_POST_DENSE_GRID")) c->post_dense_grid = std::max(1, atoi(g));
            if (const char *g = getenv("KTH_POST_SPARSE_GRID")) c->post_sparse_grid = std::max(1, atoi(g));
            if (const char *g = getenv("KTH_COOP")) c->coop = atoi(g) != 0;
            if (const char *g = getenv("KTH_PRE_HIST")) c->pre_hist = atoi(g) != 0;
            c->fin_grid = c->num_cu;
            if (const char *g = getenv("KTH_FIN_GRID")) c->fin_grid = std::max(1, std::min(atoi(g), c->num_cu));
            if (const char *g = getenv("KTH_HEAD_SLACK")) c->head_slack64 = (uint32_t)std::max(0.0, atof(g) * 64.0);
            if (const char *g = getenv("KTH_HEAD_ABS")) c->head_abs_div = (uint32_t)std::max(0, atoi(g));
            if (const char *g = getenv("KTH_TOPK_STAGE")) c->topk_stage = atoi(g) != 0;
            // (the fault injectors are not read from the environment: only
            // kth_ctx_test_hook, which tests call explicitly, turns them on)
        }
        if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { rc = KTH_EHIP; break; }
        c->own_stream = true;
        if (hipMalloc(reinterpret_cast<void **>(&c->st), 2 * sizeof(SelState)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&c->islots), SLOT_ALLOC_WORDS * sizeof(u64)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void **>(&c->d_status), 4 * sizeof(int32_t)) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void **>(&c->h_status), 4 * sizeof(int32_t), 0) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void **>(&c->h_state), sizeof(SelState), 0) != hipSuccess) {
            rc = KTH_ENOMEM;
            break;
        }
        if (hipMemset(c->st, 0, 2 * sizeof(SelState)) != hipSuccess ||
            hipMemset(c->islots, 0, SLOT_ALLOC_WORDS * sizeof(u64)) != hipSuccess) {
            rc = KTH_EHIP;
            break;
        }
        // dynamic LDS beyond the 64 KiB default for the LDS / rows kernels
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kth::k_small),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, SMALL_N * 4);
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kth::k_rows<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, KTH_ROWS_MAX_COLS * 4);
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kth::k_rows<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, KTH_ROWS_MAX_COLS * 4);
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(kth::k_finish),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)FIN_DYN_LDS) != hipSuccess)
            c->coop = false;  // no LDS-resident finish: per-level launches
        (void)hipGetLastError();
        // The grid barriers of k_head / k_finish need every workgroup resident
        // at once.  Their grids are sized for that (k_finish: one 1024-thread
        // workgroup per CU with ~145 KiB of LDS; k_head: at most 64
        // workgroups); check it against the occupancy query once, and refuse
        // the cooperative path when the device cannot hold the grid (a plain
        // launch checks nothing).  Residency can still be taken away at run
        // time by other streams or processes: the spins are bounded, a timeout
        // is reported (state error ERR_BARRIER, d_out untouched) and
        // kth_select_i32_ctx (hence kth_select_i32 and VecKthSelect) redoes the
        // select on the per-level path and stays on it for the next
        // COOP_BACKOFF synchronous selects.  The asynchronous entry points
        // (kth_select_i32_async, kth_topk_i32, kth_dist_*) report the error in
        // the state (kth_ctx_last_stats) and leave the retry to the caller.
        {
            int fin_per_cu = 0, head_per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&fin_per_cu, reinterpret_cast<const void *>(kth::k_finish),
                                                             kth::DENSE_BLK, FIN_DYN_LDS) != hipSuccess ||
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&head_per_cu, reinterpret_cast<const void *>(kth::k_head),
                                                             kth::DENSE_BLK, 0) != hipSuccess)
                fin_per_cu = head_per_cu = -1;  // query unavailable: trust the static sizing
            (void)hipGetLastError();
            if (fin_per_cu >= 0 &&
                ((int64_t)fin_per_cu * c->num_cu < c->fin_grid || (int64_t)head_per_cu * c->num_cu < HEAD_GRID_MAX)) {
                c->coop = false;
                c->coop_resident = false;
            }
        }
    } while (0);
    c->coop_wanted = c->coop;
    if (rc != KTH_OK) {
        kth_ctx_destroy(c);
        return rc;
    }
    *out = c;
    return KTH_OK;
}

int kth_ctx_test_hook(kth_ctx *c, int hook, int64_t value) {
    if (!c || value < 0) return KTH_EINVAL;
    switch (hook) {
    case KTH_HOOK_FAULT_TOPK_RANK: c->fault_topk_rank = value != 0; return KTH_OK;
    case KTH_HOOK_FAULT_BARRIER:
        if (value > 2) return KTH_EINVAL;
        c->fault_barrier = value != 0;
        c->fault_once = value == 2;
        return KTH_OK;
    case KTH_HOOK_TOPK_SEG_CAP:
        if (value > (int64_t)1 << 40) return KTH_EINVAL;
        c->topk_seg_cap = (u64)value;
        return KTH_OK;
    default: return KTH_EINVAL;
    }
}

int kth_ctx_destroy(kth_ctx *c) {
    if (!c) return KTH_EINVAL;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (hipEvent_t e : c->ev_main) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_total) (void)hipEventDestroy(e);
    if (c->st) (void)hipFree(c->st);
    if (c->islots) (void)hipFree(c->islots);
    if (c->sample) (void)hipFree(c->sample);
    if (c->cand) (void)hipFree(c->cand);
    if (c->cand_rows) (void)hipFree(c->cand_rows);
    if (c->tk_segv) (void)hipFree(c->tk_segv);
    if (c->tk_segp) (void)hipFree(c->tk_segp);
    if (c->tk_wcnt) (void)hipFree(c->tk_wcnt);
    if (c->tk_wstart) (void)hipFree(c->tk_wstart);
    if (c->staging) (void)hipFree(c->staging);
    if (c->topk) (void)hipFree(c->topk);
    if (c->d_status) (void)hipFree(c->d_status);
    if (c->stamps) (void)hipFree(c->stamps);
    if (c->h_status) (void)hipHostFree(c->h_status);
    if (c->h_state) (void)hipHostFree(c->h_state);
    if (c->h_dist) (void)hipHostFree(c->h_dist);
    if (c->ev_dist) (void)hipEventDestroy(c->ev_dist);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    if (tl_ctx == c) tl_ctx = nullptr;
    delete c;
    return KTH_OK;
}

int kth_ctx_set_stream(kth_ctx *c, void *s) {
    if (!c) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    if (c->own_stream && c->stream) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamDestroy(c->stream);
        c->own_stream = false;
    }
    // NULL is HIP's null stream (what torch calls the default stream): it
    // orders against every blocking stream of the device, as a caller that
    // passes its "current stream" expects.
    c->stream = reinterpret_cast<hipStream_t>(s);
    return KTH_OK;
}

int kth_ctx_sync(kth_ctx *c) {
    if (!c) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return KTH_OK;
}

int kth_ctx_reserve(kth_ctx *c, int64_t n) {
    if (!c || n < 0) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    if (n > RADIX_MAX_N) {
        KTH_TRY(grow(reinterpret_cast<void **>(&c->sample), &c->sample_cap, (u64)sample_size(n) * 4));
        KTH_TRY(reserve_cand(c, n));
    }
    return KTH_OK;
}

int kth_select_i32_async(kth_ctx *c, const int32_t *d_keys, int64_t n, int64_t k, int32_t *d_out) {
    if (!d_out) return KTH_EINVAL;
    return select_async(c, d_keys, n, k, d_out, nullptr);
}

int kth_select_i32_ctx(kth_ctx *c, const int32_t *keys, int64_t n, int64_t k, int32_t *out) {
    if (!c || !keys || !out || n < 1 || k < 1 || k > n) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    const int32_t *dk = keys;
    if (!is_device_ptr(keys)) {
        KTH_TRY(grow(reinterpret_cast<void **>(&c->staging), &c->staging_cap, (u64)n * 4));
        HIP_TRY(hipMemcpyAsync(c->staging, keys, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
        dk = c->staging;
    }
    KTH_TRY(select_async(c, dk, n, k, nullptr, c->d_status));
    HIP_TRY(hipMemcpyAsync(c->h_status, c->d_status, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->h_status[1] == (int32_t)kth::ERR_BARRIER && c->coop) {
        // a cooperative grid was not co-resident (another stream or process
        // held CUs): redo the select on the per-level path, which needs no
        // residency; the slots are re-zeroed first (dirty)
        // (sticky for COOP_BACKOFF synchronous selects: while the CUs stay
        // contended, every cooperative launch would spin out its barriers)
        c->dirty = true;
        c->coop = false;
        c->coop_backoff = COOP_BACKOFF + 1;  // (the retry below counts one)
        KTH_TRY(select_async(c, dk, n, k, nullptr, c->d_status));
        HIP_TRY(hipMemcpyAsync(c->h_status, c->d_status, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    if (c->h_status[1] != 0) {
        c->dirty = true;
        return KTH_EINTERNAL;
    }
    *out = c->h_status[0];
    return KTH_OK;
}

int kth_select_i32(const int32_t *keys, int64_t n, int64_t k, int32_t *out) {
    if (!keys || !out || n < 1 || k < 1 || k > n) return KTH_EINVAL;
    if (!tl_ctx) {
        int dev = 0;
        if (kth_device_count() <= 0) return KTH_ENODEV;
        if (hipGetDevice(&dev) != hipSuccess) {
            (void)hipGetLastError();
            dev = 0;
        }
        KTH_TRY(kth_ctx_create(dev, &tl_ctx));
    }
    return kth_select_i32_ctx(tl_ctx, keys, n, k, out);
}

int kth_ctx_coop(const kth_ctx *c) {
    if (!c) return KTH_EINVAL;
    return c->coop ? 1 : 0;
}

int kth_ctx_last_stats(kth_ctx *c, kth_stats *out) {
    if (!c || !out) return KTH_EINVAL;
    if (c->last_state < 0) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    HIP_TRY(hipMemcpyAsync(c->h_state, c->st + c->last_state, sizeof(SelState), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const SelState &s = *c->h_state;
    memset(out, 0, sizeof *out);
    out->path = (int32_t)s.path;
    out->mode = (int32_t)s.mode;
    out->lo_key = s.lo;
    out->hi_key = s.hi;
    out->n = s.n;
    out->k = s.k;
    out->cnt_lt = s.cnt[kth::C_LT];
    out->cnt_eq_lo = s.cnt[kth::C_EQLO];
    out->cnt_eq_hi = s.cnt[kth::C_EQHI];
    out->candidates = s.cnt[kth::C_IN];
    out->capacity = c->cand_cap / 4;
    out->answer = (int32_t)(s.answer ^ 0x80000000u);
    out->error = (int32_t)s.error;
    return KTH_OK;
}

int kth_ctx_enable_timing(kth_ctx *c, int on) {
    if (!c) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    if (on && c->ev_main.empty()) {
        c->ev_main.resize(MAX_EVENTS);
        c->ev_total.resize(MAX_EVENTS);
        for (auto &e : c->ev_main) HIP_TRY(hipEventCreate(&e));
        for (auto &e : c->ev_total) HIP_TRY(hipEventCreate(&e));
    }
    c->timing = on != 0;
    c->main_used = c->total_used = 0;
    return KTH_OK;
}

int kth_ctx_take_timing(kth_ctx *c, int64_t *n_sel, double *main_ms, double *total_ms) {
    if (!c || !n_sel || !main_ms || !total_ms) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    HIP_TRY(hipStreamSynchronize(c->stream));
    double m = 0, t = 0;
    int64_t nm = 0;
    for (int i = 0; i + 1 < c->main_used; i += 2) {
        float a = 0;
        HIP_TRY(hipEventElapsedTime(&a, c->ev_main[i], c->ev_main[i + 1]));
        m += a;
        nm++;
    }
    for (int i = 0; i + 1 < c->total_used; i += 2) {
        float b = 0;
        HIP_TRY(hipEventElapsedTime(&b, c->ev_total[i], c->ev_total[i + 1]));
        t += b;
    }
    c->main_used = c->total_used = 0;
    *n_sel = nm;
    *main_ms = m;
    *total_ms = t;
    return KTH_OK;
}

int kth_select_rows_i32(kth_ctx *c, const int32_t *d_keys, int64_t rows, int32_t cols, int32_t k, int32_t *d_out) {
    if (!c || !d_keys || !d_out || rows < 0 || cols < 1 || cols > KTH_ROWS_MAX_COLS || k < 1 || k > cols)
        return KTH_EINVAL;
    if (rows == 0) return KTH_OK;
    KTH_TRY(set_device(c));
    return launch_rows<false, false>(c, reinterpret_cast<const uint32_t *>(d_keys), rows, cols, k,
                              reinterpret_cast<uint32_t *>(d_out));
}

int kth_select_rows_f32(kth_ctx *c, const float *d_keys, int64_t rows, int32_t cols, int32_t k, float *d_out) {
    if (!c || !d_keys || !d_out || rows < 0 || cols < 1 || cols > KTH_ROWS_MAX_COLS || k < 1 || k > cols)
        return KTH_EINVAL;
    if (rows == 0) return KTH_OK;
    KTH_TRY(set_device(c));
    return launch_rows<true, false>(c, reinterpret_cast<const uint32_t *>(d_keys), rows, cols, k,
                             reinterpret_cast<uint32_t *>(d_out));
}

int kth_topk_rows_i32(kth_ctx *c, const int32_t *d_keys, int64_t rows, int32_t cols, int32_t k, int largest,
                      int32_t *d_vals, int32_t *d_idx) {
    if (!c || !d_keys || (!d_vals && !d_idx) || rows < 0 || cols < 1 || cols > KTH_TOPK_MAX_COLS || k < 1 ||
        k > cols)
        return KTH_EINVAL;
    if (rows == 0) return KTH_OK;
    KTH_TRY(set_device(c));
    return launch_rows<false, true>(c, reinterpret_cast<const uint32_t *>(d_keys), rows, cols, k, nullptr,
                                    largest ? 0xFFFFFFFFu : 0u, reinterpret_cast<uint32_t *>(d_vals), d_idx);
}

int kth_topk_rows_f32(kth_ctx *c, const float *d_keys, int64_t rows, int32_t cols, int32_t k, int largest,
                      float *d_vals, int32_t *d_idx) {
    if (!c || !d_keys || (!d_vals && !d_idx) || rows < 0 || cols < 1 || cols > KTH_TOPK_MAX_COLS || k < 1 ||
        k > cols)
        return KTH_EINVAL;
    if (rows == 0) return KTH_OK;
    KTH_TRY(set_device(c));
    return launch_rows<true, true>(c, reinterpret_cast<const uint32_t *>(d_keys), rows, cols, k, nullptr,
                                   largest ? 0xFFFFFFFFu : 0u, reinterpret_cast<uint32_t *>(d_vals), d_idx);
}

int kth_topk_i32(kth_ctx *c, const int32_t *d_keys, int64_t n, int64_t k, int largest, int32_t *d_vals,
                 int64_t *d_idx) {
    if (!c || !d_keys || (!d_vals && !d_idx) || n < 1 || k < 1 || k > n) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    const u64 ntiles = ((u64)n + kth::TK_TILE - 1) / kth::TK_TILE;
    const u64 nblk = (ntiles + kth::TK_TILES_PER_BLOCK - 1) / kth::TK_TILES_PER_BLOCK;
    // k_main's tile geometry (its flags cover the full tiles after the unaligned head)
    u64 head = ((16u - (uint32_t)(reinterpret_cast<uintptr_t>(d_keys) & 15u)) & 15u) >> 2;
    if (head > (u64)n) head = (u64)n;
    const u64 nfull = (((u64)n - head) >> 2) / ((u64)kth::BLK * kth::MAIN_UNROLL);
    // k_main's top-k records (only on the window path, n > RADIX_MAX_N):
    //   16-byte aligned keys: per wave-row counts + candidate rows, and the
    //   count pass loads no tile k_main covered (tf 3 / 4) -- unless k is so
    //   small that the rows holding output are a few per cent (k * 64 Ki <=
    //   n: one flag bit per row, the count pass loads only flagged tiles,
    //   tf 1 / 2; measured ~equal there, and it needs no alignment)
    //   and for n / 64 Ki < k <= n / 16 (16-byte aligned), every key on the
    //   kept side of the window's far edge staged in index order (tf 5 / 6):
    //   neither the count nor the write pass reads the input (KTH_TOPK_STAGE=0: tf 3 / 4)
    const bool aligned = (reinterpret_cast<uintptr_t>(d_keys) & 15u) == 0;
    const bool window = n > RADIX_MAX_N;
    const bool few = (u64)k * kth::TK_TILE * 64 <= (u64)n;
    const bool staged = aligned && window && !few && (u64)k * TK_STAGE_MAX_FRAC <= (u64)n && c->topk_stage;
    const int tf = staged                                  ? (largest ? 6 : 5)
                   : (aligned && window && !few)           ? (largest ? 4 : 3)
                   : (u64)k * kth::TK_TILE <= (u64)n ? (largest ? 2 : 1)
                                                             : 0;
    const u64 ncov = tf >= 3 ? nfull * kth::MAIN_UNROLL : 0;  // tiles = k_main rows (head == 0)
    // tflags: the header and TF 1 / 2's flag bytes after 4 words, TF >= 3's
    // row words after TF_W0 in per-wave segments (kth::rw_index); 256-byte
    // aligned, so that a wave's group of 64 words fills one line
    const u64 Gm = (u64)c->main_grid[tf];
    const kth::RowWords rwl{Gm, tf >= 3 ? kth::rw_seg_words(nfull, Gm) : kth::fl_seg_bytes(nfull, Gm)};
    const u64 fwords = tf >= 3 ? kth::TF_W0 + rwl.G * (kth::BLK / kth::WAVE) * rwl.seg
                               : 4 + rwl.G * (kth::BLK / kth::WAVE) * rwl.seg / 4;
    const u64 fw64 = (fwords + 1) / 2, before = (ntiles + 1) / 2 + ntiles + 4 * nblk + 2;
    const u64 words = before + fw64 + 32;
    KTH_TRY(grow(reinterpret_cast<void **>(&c->topk), &c->topk_cap, words * sizeof(u64)));
    const u64 foff = (before + 31) & ~31ull;  // + fw64 <= words
    uint32_t *tflags = reinterpret_cast<uint32_t *>(c->topk + foff);
    HIP_TRY(hipMemsetAsync(tflags, 0, 16, c->stream));  // window header: not valid until k_main<TF> runs
    if (tf == 3 || tf == 4) {
        KTH_TRY(reserve_cand(c, n));
        KTH_TRY(grow(reinterpret_cast<void **>(&c->cand_rows), &c->cand_rows_cap, c->cand_cap));
    }
    u64 seg_cap = 0;
    uint32_t nwin = 0;
    if (tf >= 5) {  // the staging segments: one per k_main wave, n / 16 entries in all
        const u64 nwaves = (u64)c->main_grid[tf] * (kth::BLK / kth::WAVE);
        // entries: the k kept keys, the candidates (~0.6 % of n at 2^30) and the
        // waves' imbalance; a segment that overflows sends the top-k to the
        // input-reading path (exact)
        const u64 seg_total = std::max<u64>({1ull << 20, (u64)n / 16, (u64)k + (u64)k / 8 + (u64)n / 64});
        seg_cap = c->topk_seg_cap ? c->topk_seg_cap : (seg_total + nwaves - 1) / nwaves;
        seg_cap = (seg_cap + 3) & ~3ull;  // segments start 16-byte aligned (k_main<5/6> stores 4 entries a lane)
        KTH_TRY(reserve_cand(c, n));
        KTH_TRY(grow(reinterpret_cast<void **>(&c->tk_segv), &c->tk_segv_cap, seg_cap * nwaves * 4));
        KTH_TRY(grow(reinterpret_cast<void **>(&c->tk_segp), &c->tk_segp_cap, seg_cap * nwaves));
        KTH_TRY(grow(reinterpret_cast<void **>(&c->tk_wcnt), &c->tk_wcnt_cap, ncov * (kth::BLK / kth::WAVE) * 4 + 16));
        // per wave and window (TK5_WIN_TILES of its tiles): the entries staged before it
        const u64 G = (u64)c->main_grid[tf];
        nwin = (uint32_t)(((nfull + G - 1) / G + kth::TK5_WIN_TILES - 1) / kth::TK5_WIN_TILES);
        KTH_TRY(grow(reinterpret_cast<void **>(&c->tk_wstart), &c->tk_wstart_cap, nwaves * std::max(nwin, 1u) * 4));
        // dense staging (k >= n / 32) stores the segments non-temporally: k_main<5> at k = 2^26 964-976
        // against 980-984 us, whole calls -0.5 to -2 %; at k = 2^24 k_main<5> gains ~6 us but
        // k_tk5_count, which then reads the entries from HBM, loses ~8; at 2^20 +0.8 %
        // (profiles/r6_topk_seg_store_ab.txt)
        const uint32_t nt = (u64)k * 32 >= (u64)n ? 1u : 0u;
        c->tk_seg = kth::TkSeg{c->tk_segv, c->tk_segp, (uint32_t)seg_cap, tflags + 3, c->tk_wstart, nwin, nt};
    }
    // the k-th smallest (largest: the (n-k+1)-th smallest) -> d_status[0], on the device
    int64_t rank = largest ? n - k + 1 : k;
    if (c->fault_topk_rank && n > 1) rank = rank < n ? rank + 1 : rank - 1;
    KTH_TRY(select_async(c, d_keys, n, rank, nullptr, c->d_status, tf, tflags));
    const uint32_t *keys = reinterpret_cast<const uint32_t *>(d_keys);
    const uint32_t flip = largest ? 0xFFFFFFFFu : 0u;
    u64 *toff = c->topk, *bsum = toff + ntiles, *bbase = bsum + 2 * nblk, *meta = bbase + 2 * nblk;
    uint32_t *tcnt = reinterpret_cast<uint32_t *>(meta + 2);
    const SelState *sel_st = c->st + c->last_state;
    // count and write passes: one wave per 64 tiles
    const int waves = kth::TK_BLOCK / kth::WAVE;
    const int g = (int)std::min<u64>((ntiles + waves * kth::WAVE - 1) / (waves * kth::WAVE), (u64)c->num_cu * 16);
    if (tf >= 5) {  // the staged entries (rows < ncov), then the ragged rows from the input
        auto tk5c = (u64)k * 64 >= (u64)n ? kth::k_tk5_count<true> : kth::k_tk5_count<false>;  // dense windows: chunked
        tk5c<<<c->main_grid[tf] * TK5_SPLIT, kth::TK_BLOCK, 0, c->stream>>>(
            c->tk_segv, seg_cap, c->tk_wstart, nwin, (u64)c->main_grid[tf], tflags, nfull, c->d_status, flip,
            c->tk_wcnt, tcnt);
        kth::k_topk_count<true, 2><<<g, kth::TK_BLOCK, 0, c->stream>>>(keys, (u64)n, ntiles, c->d_status, flip, tcnt,
                                                                       tflags, head, nfull, sel_st, ncov);
    } else if (tf >= 3) {  // candidates' share first (atomics into zeroed counts), then the rows' words
        HIP_TRY(hipMemsetAsync(tcnt, 0, ntiles * 4, c->stream));
        kth::k_topk_cands<<<c->num_cu * 8, kth::TK_BLOCK, 0, c->stream>>>(
            c->cand, c->cand_rows, cand_count(c), c->cand_cap / 4, c->d_status, flip, tcnt, tflags, sel_st);
        kth::k_topk_count<true, 1><<<g, kth::TK_BLOCK, 0, c->stream>>>(keys, (u64)n, ntiles, c->d_status, flip,
                                                                          tcnt, tflags, head, nfull, sel_st, ncov, rwl);
    } else if (aligned) {
        kth::k_topk_count<true, 0><<<g, kth::TK_BLOCK, 0, c->stream>>>(keys, (u64)n, ntiles, c->d_status, flip,
                                                                           tcnt, tflags, head, nfull, sel_st, 0, rwl);
    } else {
        kth::k_topk_count<false, 0><<<g, kth::TK_BLOCK, 0, c->stream>>>(keys, (u64)n, ntiles, c->d_status, flip,
                                                                            tcnt, tflags, head, nfull, sel_st, 0, rwl);
    }
    // tile offsets, block bases and need in one launch (a bracket failure --
    // counts that do not hold the k-th -- lands in the select's state, where
    // kth_ctx_last_stats reports it as .error)
    kth::k_topk_bases<<<(int)nblk, kth::TK_BLOCK, 0, c->stream>>>(
        tcnt, ntiles, toff, bsum, (u64)k, bbase, meta, c->st + c->last_state,
        reinterpret_cast<uint32_t *>(c->islots + BAR_OFF) + kth::BAR_TOPK_ARRIVE);
    if (tf >= 5) {
        auto tk5w = (u64)k * 32 <= (u64)n ? kth::k_tk5_write<kth::TK5_STAGE_SMALL> : kth::k_tk5_write<kth::TK5_STAGE_LARGE>;
        tk5w<<<c->main_grid[tf] * TK5_SPLIT, kth::TK_BLOCK, 0, c->stream>>>(
            c->tk_segv, c->tk_segp, seg_cap, c->tk_wstart, nwin, (u64)c->main_grid[tf], tflags, nfull, c->d_status,
            flip, c->tk_wcnt, tcnt, toff, bbase, meta, d_vals, d_idx);
        kth::k_topk_write<true, true><<<g, kth::TK_BLOCK, 0, c->stream>>>(keys, (u64)n, ntiles, c->d_status, flip,
                                                                          tcnt, toff, bbase, meta, d_vals, d_idx,
                                                                          tflags, ncov);
    } else if (aligned)
        kth::k_topk_write<true><<<g, kth::TK_BLOCK, 0, c->stream>>>(keys, (u64)n, ntiles, c->d_status, flip, tcnt,
                                                                    toff, bbase, meta, d_vals, d_idx);
    else
        kth::k_topk_write<false><<<g, kth::TK_BLOCK, 0, c->stream>>>(keys, (u64)n, ntiles, c->d_status, flip, tcnt,
                                                                     toff, bbase, meta, d_vals, d_idx);
    return launch_check();
}

int kth_fill_synthetic(kth_ctx *c, int32_t *d_out, int64_t n, int64_t offset, int64_t n_total, int dist, uint64_t seed,
                       int32_t param) {
    if (!c || (!d_out && n > 0) || n < 0 || offset < 0 || dist < 0 || dist > 7) return KTH_EINVAL;
    if (n == 0) return KTH_OK;
    KTH_TRY(set_device(c));
    uint32_t step = 1;
    if (n_total > 0 && n_total <= (int64_t)0xFFFFFFFFll) {
        u64 s = (1ull << 32) / (u64)n_total;
        step = s > 0xFFFFFFFFull ? 0xFFFFFFFFu : (s ? (uint32_t)s : 1u);
    }
    const int g = (int)std::min<int64_t>((n + kth::BLK - 1) / kth::BLK, (int64_t)c->num_cu * 16);
    kth::k_fill<<<g, kth::BLK, 0, c->stream>>>(d_out, (u64)n, (u64)offset, step, dist, seed, param);
    return launch_check();
}

// ------------------------------------------------------- sharded protocol
int64_t kth_dist_sample_size(int64_t n) { return sample_size(n); }

int kth_sample_chunk(void) { return kth::SAMPLE_CHUNK; }

double kth_window_z(void) { return window_z(); }

int64_t kth_dist_cand_capacity(int64_t n_local) { return (int64_t)cand_capacity(std::max<int64_t>(n_local, 1)); }

int kth_window_slack64(void) { return (int)(HEAD_SLACK * 64); }

int kth_dist_begin(kth_ctx *c, uint64_t *d_slots, int64_t n_total, int64_t k) {
    if (!c || !d_slots || n_total < 1 || k < 1 || k > n_total) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    if (!c->h_dist) {  // level 0's DistStatus: host-visible memory the kernel writes, an event after it
        if (hipHostMalloc(reinterpret_cast<void **>(&c->h_dist), kth::DIST_STATUS_WORDS * sizeof(uint32_t),
                          hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
            (void)hipGetLastError();
            c->h_dist = nullptr;
            return KTH_ENOMEM;
        }
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&c->d_dist), c->h_dist, 0));
        HIP_TRY(hipEventCreateWithFlags(&c->ev_dist, hipEventDisableTiming));
    }
    coop_tick(c);
    c->uslots = reinterpret_cast<u64 *>(d_slots);
    c->dist_n = n_total;
    c->dist_k = k;
    c->dist_level_next = -1;  // kth_dist_scan first
    c->dist_levels = -1;
    c->dist_result_slot = -1;
    c->dist_early_out = nullptr;
    c->dist_zero = true;  // kth_dist_sample clears the slots inside its kernel
    // the ctx's own slots are left zeroed by every completed k_result; a
    // sequence cut short (dirty, or a dist selection never finished) re-zeroes,
    // and so does a cooperative single-GPU window select, which leaves its
    // count slot and candidate count for its next k_head to clear (the
    // streaming pass would append after a stale count, and the candidate
    // levels would histogram the previous select's keys)
    if (c->dirty || c->dist_open || c->counts_left)
        HIP_TRY(hipMemsetAsync(c->islots, 0, SLOT_ALLOC_WORDS * sizeof(u64), c->stream));
    c->dirty = false;
    c->counts_left = false;
    c->dist_open = true;
    return KTH_OK;
}

int kth_dist_sample(kth_ctx *c, const int32_t *d_keys, int64_t n_local, uint32_t *d_sample, int64_t s_local) {
    if (!c || !d_keys || !d_sample || s_local < 64 || s_local % 64 || n_local < s_local) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    const u64 nchunks = ((u64)s_local + kth::SAMPLE_CHUNK - 1) / kth::SAMPLE_CHUNK;
    const u64 stride = (u64)n_local / nchunks;
    StepArgs a;
    memset(&a, 0, sizeof a);
    if (c->dist_zero && c->uslots) {
        a.stats_zero = c->uslots;
        a.zero_words = 3 * (u64)KTH_STATS_WORDS;
    }
    kth::k_gather<false><<<gather_grid(nchunks), kth::DENSE_BLK, 0, c->stream>>>(a, d_keys, (u64)n_local, stride, d_sample,
                                                                                (u64)s_local);
    KTH_TRY(launch_check());
    if (a.zero_words) c->dist_zero = false;
    return KTH_OK;
}

int kth_dist_window(kth_ctx *c, const uint32_t *d_sample, int64_t s_total) {
    if (!c || !d_sample || s_total < 1 || !c->uslots) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    if (c->dist_zero) {  // no kth_dist_sample since kth_dist_begin (samples from elsewhere)
        HIP_TRY(hipMemsetAsync(c->uslots, 0, 3 * (size_t)KTH_STATS_WORDS * 8, c->stream));
        c->dist_zero = false;
    }
    u64 r_lo, r_hi;
    window_ranks(c->dist_n, c->dist_k, s_total, &r_lo, &r_hi);
    if (c->coop && s_total % 64 == 0 && s_total < (1ll << 29)) {
        // one cooperative launch over the gathered sample (k_head without its
        // gather): the digits behind grid barriers, the early window; the state
        // is left resolved in st[0] for kth_dist_scan (ADV_CARRY).  Its slots
        // are cleared by kth_dist_result's k_result.
        StepArgs a = step(c, kth::ADV_INIT_SAMPLE, -1, 0, nullptr, nullptr, nullptr);
        a.init_n = (u64)c->dist_n;
        a.init_k = (u64)c->dist_k;
        a.init_s = (u64)s_total;
        a.r_lo = r_lo;
        a.r_hi = r_hi;
        kth::CoopArgs x = coop_args(c, HSLOT_OFF, nullptr, nullptr);
        x.sample_ready = 1;
        const int grid = (int)std::min<int64_t>(64, std::max<int64_t>(1, s_total / (16 * 1024)));
        kth::k_head<<<grid, kth::DENSE_BLK, 0, c->stream>>>(a, x, nullptr, 0, 0, const_cast<uint32_t *>(d_sample),
                                                           (u64)s_total);
        c->dist_coop_window = true;
        return launch_check();
    }
    c->dist_coop_window = false;
    StepArgs a = step(c, kth::ADV_INIT_SAMPLE, -1, 0, nullptr, islot(c, 1), islot(c, 2));
    a.init_n = (u64)c->dist_n;
    a.init_k = (u64)c->dist_k;
    a.init_s = (u64)s_total;
    a.r_lo = r_lo;
    a.r_hi = r_hi;
    a.sample = d_sample;
    a.sample_count = (u64)s_total;
    launch_level(c, a, true, level_grid((u64)s_total, DENSE_PER_WG));
    const int gs = level_grid((u64)s_total, sparse_wg(c));
    a = step(c, kth::ADV_PICK, 0, 1, islot(c, 1), islot(c, 2), islot(c, 0));
    a.sample = d_sample;
    a.sample_count = (u64)s_total;
    launch_level(c, a, false, gs);
    a = step(c, kth::ADV_PICK, 1, 0, islot(c, 2), islot(c, 0), islot(c, 1));
    a.sample = d_sample;
    a.sample_count = (u64)s_total;
    launch_level(c, a, false, gs);
    return launch_check();
}

int kth_dist_scan(kth_ctx *c, const int32_t *d_keys, int64_t n_local) {
    if (!c || !d_keys || n_local < 0 || !c->uslots) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    KTH_TRY(reserve_cand(c, std::max<int64_t>(n_local, 1)));
    u64 *U0 = c->uslots;
    StepArgs a = c->dist_coop_window ? step(c, kth::ADV_CARRY, 0, 1, nullptr, U0, nullptr)
                                     : step(c, kth::ADV_PICK, 0, 1, islot(c, 0), U0, nullptr);
    a.keys = d_keys;
    a.n_local = (u64)n_local;
    ev_main(c);
    kth::k_main<0><<<c->main_grid[0], kth::BLK, 0, c->stream>>>(a, c->cand, nullptr, nullptr, kth::TkSeg{});
    ev_main(c);
    KTH_TRY(launch_check());
    // this rank's candidates' first digit into the same slot (one all-reduce
    // carries the counts and the digit)
    a = step(c, kth::ADV_CARRY, 1, 1, nullptr, U0, nullptr);
    a.min_per_wg = c->dscan_per_wg;
    kth::k_dscan_hist<kth::DENSE_BLK><<<level_grid(cand_capacity(std::max<int64_t>(n_local, 1)), c->dscan_per_wg),
                                        kth::DENSE_BLK, 0, c->stream>>>(a);
    KTH_TRY(launch_check());
    c->dist_level_next = 0;
    c->dist_levels = -1;
    return 0;
}

// Level l reads state l+1 (mod 2) and slot l (mod 3), writes state l (mod 2),
// accumulates into slot l+1 and clears slot l+2; level 0 also tells the host
// (DistStatus) how many level calls return a slot, so that level 1 can answer
// KTH_DIST_DONE without a collective.  Level 0 is enqueued without waiting
// for anything; level 1 waits for level 0 (the host reads the DistStatus) --
// while the all-reduce after level 0 is still queued on the device.
int kth_dist_level(kth_ctx *c, const int32_t *d_keys, int64_t n_local, int level) {
    if (!c || !d_keys || n_local < 0 || !c->uslots || level < 0 || level != c->dist_level_next) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    if (level >= 1 && c->dist_levels < 0) {
        HIP_TRY(hipEventSynchronize(c->ev_dist));
        const uint32_t *h = c->h_dist;
        const uint32_t levels = __atomic_load_n(&h[0], __ATOMIC_ACQUIRE), tag = __atomic_load_n(&h[3], __ATOMIC_ACQUIRE);
        if (tag != c->dist_tag || levels < 1 || levels > KTH_DIST_MAX_LEVELS) {
            c->dirty = true;
            return KTH_EINTERNAL;
        }
        c->dist_levels = (int)levels;
    }
    if (level >= 1 && level >= c->dist_levels) {
        c->dist_result_slot = level % 3;  // accumulated by level - 1
        c->dist_level_next = -1;
        return KTH_DIST_DONE;
    }
    u64 *U[3] = {c->uslots, c->uslots + KTH_STATS_WORDS, c->uslots + 2 * KTH_STATS_WORDS};
    const int in = level % 3, acc = (level + 1) % 3, zero = (level + 2) % 3;
    StepArgs a = step(c, level == 0 ? kth::ADV_DECIDE : kth::ADV_PICK, (level + 1) % 2, level % 2, U[in], U[acc],
                      U[zero]);
    a.keys = d_keys;
    a.n_local = (u64)n_local;
    a.min_per_wg = sparse_wg(c);     // a digit under a resolved prefix: only that bin's keys
    a.dense_per_wg = DENSE_PER_WG;   // the fallback's first digit over the whole shard
    if (level == 0) {
        a.host_status = c->d_dist;
        a.tag = ++c->dist_tag;
    }
    // (the active workgroups follow the domain's size: candidates or the shard)
    kth::k_dlevel<kth::BLK><<<LEVEL_GRID_MAX, kth::BLK, 0, c->stream>>>(a);
    KTH_TRY(launch_check());
    if (level == 0) HIP_TRY(hipEventRecord(c->ev_dist, c->stream));
    c->dist_level_next = level + 1;
    return acc;
}

int kth_internal_slots_sum(uint64_t *const *slots, int P, int slot, void *stream) {
    static_assert(kth::SLOTS_SUM_MAX == KTH_LOCAL_MAX_SHARDS, "one limit");
    if (!slots || P < 1 || P > KTH_LOCAL_MAX_SHARDS || slot < 0 || slot > 2) return KTH_EINVAL;
    kth::SlotPtrs s{};
    for (int i = 0; i < P; ++i) {
        if (!slots[i]) return KTH_EINVAL;
        s.p[i] = reinterpret_cast<u64 *>(slots[i]) + (size_t)slot * KTH_STATS_WORDS;
    }
    constexpr int g = (KTH_STATS_WORDS + kth::BLK - 1) / kth::BLK;
    kth::k_slots_sum<<<g, kth::BLK, 0, reinterpret_cast<hipStream_t>(stream)>>>(s, P, (u64)KTH_STATS_WORDS);
    return launch_check();
}

void *kth_internal_ctx_stream(const kth_ctx *c) { return c ? reinterpret_cast<void *>(c->stream) : nullptr; }

int kth_internal_status_gather(kth_ctx *const *ctxs, int P, int32_t *d_dst, void *stream) {
    if (!ctxs || !d_dst || P < 1 || P > KTH_LOCAL_MAX_SHARDS) return KTH_EINVAL;
    kth::StatusPtrs p{};
    for (int i = 0; i < P; ++i) {
        if (!ctxs[i] || ctxs[i]->device != ctxs[0]->device) return KTH_EINVAL;
        p.p[i] = ctxs[i]->d_status;
    }
    KTH_TRY(set_device(ctxs[0]));
    kth::k_status_gather<<<1, kth::WAVE, 0, reinterpret_cast<hipStream_t>(stream)>>>(p, P, d_dst);
    return launch_check();
}

int kth_internal_dist_window_share(kth_ctx *src, kth_ctx *const *dst, int P) {
    if (!src || !dst || P < 0 || P > KTH_LOCAL_MAX_SHARDS) return KTH_EINVAL;
    if (!src->dist_coop_window) return 1;  // per-level window: its last pick is the scan's, nothing to copy
    kth::StatePtrs d{};
    for (int i = 0; i < P; ++i) {
        if (!dst[i] || dst[i]->device != src->device || !dst[i]->uslots) return KTH_EINVAL;
        d.p[i] = dst[i]->st;  // (the window's state is st[0], kth_dist_scan carries it)
    }
    if (P == 0) return KTH_OK;
    KTH_TRY(set_device(src));
    kth::k_state_bcast<<<1, kth::BLK, 0, src->stream>>>(src->st, d, P);
    KTH_TRY(launch_check());
    for (int i = 0; i < P; ++i) {
        dst[i]->dist_coop_window = true;
        dst[i]->dist_zero = false;
    }
    return KTH_OK;
}

// k_dresult after L levels: state (L + 1) % 2 and slot L % 3 in, the other state out
static int launch_dresult(kth_ctx *c, int L, int32_t *d_out, uint32_t early) {
    const int st_in = (L + 1) % 2;
    StepArgs a = step(c, kth::ADV_PICK, st_in, 1 - st_in, c->uslots + (size_t)(L % 3) * KTH_STATS_WORDS,
                      nullptr, nullptr);
    // (the islots and, right after them, k_head's slots of a cooperative window)
    static_assert(ISLOT_WORDS % 2 == 0, "k_dresult zeroes 16-byte words from the islots on");
    kth::k_dresult<kth::BLK><<<16, kth::BLK, 0, c->stream>>>(a, d_out, c->d_status, c->islots,
                                                            ISLOT_WORDS + HSLOT_WORDS, early);
    c->last_state = 1 - st_in;
    return launch_check();
}

int kth_dist_result_early(kth_ctx *c, int32_t *d_out) {
    // right after level 0's slot was all-reduced, before kth_dist_level(1):
    // the result as if level 0 were the last (it is whenever the window is at
    // most 2^24 values wide or decided by its counts)
    if (!c || !d_out || !c->uslots || c->dist_level_next != 1 || c->dist_levels >= 0) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    KTH_TRY(launch_dresult(c, 1, d_out, 1u));
    c->dist_early_out = d_out;
    return KTH_OK;
}

int kth_dist_result(kth_ctx *c, int32_t *d_out) {
    if (!c || !d_out || !c->uslots || c->dist_result_slot < 0) return KTH_EINVAL;
    KTH_TRY(set_device(c));
    const int L = c->dist_levels;  // levels enqueued: the last wrote state (L - 1) % 2
    if (!(L == 1 && c->dist_early_out == d_out))  // else the early result did it
        KTH_TRY(launch_dresult(c, L, d_out, 0u));
    c->dist_early_out = nullptr;
    c->dist_level_next = -1;
    c->dist_result_slot = -1;
    c->dist_open = false;
    return KTH_OK;
}

}  // extern "C"
