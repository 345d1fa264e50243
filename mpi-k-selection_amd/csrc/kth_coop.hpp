// kth_coop.hpp -- the single-GPU window path's sample phase and finish phase,
// each as ONE launch whose workgroups meet at grid barriers between radix
// levels (gfx950).  Included by kth_kernels.hip.
//
// The per-level launches of the sharded protocol (k_gather, k_level, k_result
// in kth_kernels.hip) pay a launch, a kernel-boundary cache flush and a
// histogram re-read per level: ~10 us each at 2^30, ~70 us of the 0.72 ms
// select (profiles/r2_start_kernel_trace_summary.txt).  On one GPU there is
// no all-reduce between levels, so a level's histogram only has to reach the
// other workgroups of the same kernel:
//   k_head    gather the sample + its first digit -> barrier -> pick ->
//             (while the window is not narrow enough) one sample level ->
//             barrier -> pick; publishes the window for k_main (ADV_CARRY)
//   k_finish  decide from k_main's counts -> per level: histogram the
//             candidates (or, after a window miss, the input) -> barrier ->
//             pick; writes the answer and leaves every slot zeroed
// Both grids are small enough to be co-resident (one workgroup per CU at
// most); the barrier is hierarchical (8 group counters, then one top counter:
// same-address atomics serialise) and sense-reversing (the last arrivers reset
// the counters, so nothing has to be zeroed between calls).  Every spin is
// bounded: a barrier that never completes raises an error, it never hangs.
#pragma once

namespace kth {

struct CoopArgs {
    u64 *slots;        // HEAD_LEVELS / FIN_LEVELS histogram slots of STATS_WORDS, zero on entry
    uint32_t *bar;     // BAR_WORDS of barrier state
    int32_t *d_out, *d_status;
    u64 dense_per_wg, sparse_per_wg;  // keys per active workgroup: first digit of a domain / later digits
    uint32_t slack64;  // k_head early window (EarlyWindow); 0 = exact sample ranks
    u64 abs_min;       // ... and its absolute floor in sample keys (EarlyWindow::abs_min)
    u64 *zero2;        // k_finish: a second region to clear (the sample phase's slots)
    u64 zero2_words;
    uint32_t *tail;    // k_finish: FIN_LDS_KEYS keys of the last bin (finish_tail)
    uint32_t sample_ready;  // k_head: the sample (order keys) is already in `sample` (sharded window)
    uint32_t fault;    // test hook (KTH_HOOK_FAULT_BARRIER): the grid barriers and the tail wait report a timeout
    const uint32_t *pre;  // k_finish: k_main<0>'s first candidate digit (PreHist), or null
    uint32_t *pre_zero;   // k_finish: the other PreHist set, cleared for the next select
};

// The dense first digit of k_finish (nb <= NBINS / copies bins) is flushed
// into `copies` histogram copies (workgroup w adds to copy w % copies: fewer
// same-address atomics); the pick loads the NBINS words once and sums them.
template <int BLOCK>
__device__ __forceinline__ void pick_slot_copies(SelState &ss, const u64 *slot, uint32_t nb, uint32_t copies,
                                                 u64 *tmp /* NBINS u64 of LDS */, u64 *scratch, u64 *cnt0) {
    constexpr int PER = NBINS / BLOCK;
#pragma unroll
    for (int j = 0; j < PER; ++j)
        tmp[threadIdx.x * PER + j] =
            __hip_atomic_load(slot + NCOUNTS + threadIdx.x * PER + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    u64 h0[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t b = threadIdx.x * PER + j;
        u64 sum = 0;
        if (b < nb)
            for (uint32_t c = 0; c < copies; ++c) sum += tmp[c * nb + b];
        h0[j] = sum;
    }
    __syncthreads();
    pick_state<BLOCK, PER>(ss, h0, h0, true, scratch, nullptr, cnt0);
}

// The first candidate digit from k_main<0>'s PreHist (nb <= PRE_BINS bins in
// PRE_COPIES copies; written by the previous kernel: plain loads), summed per
// bin, and picked (target 0).
template <int BLOCK>
__device__ __forceinline__ void pick_pre(SelState &ss, const uint32_t *pre, uint32_t nb, u64 *scratch, u64 *cnt0) {
    constexpr int PER = NBINS / BLOCK;
    u64 h0[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const uint32_t b = threadIdx.x * PER + j;
        uint32_t sum = 0;
        if (b < nb)
#pragma unroll
            for (int c = 0; c < PRE_COPIES; ++c) sum += pre[c * PRE_BINS + b];
        h0[j] = sum;
    }
    pick_state<BLOCK, PER>(ss, h0, h0, true, scratch, nullptr, cnt0);
}

// hist_flush into copy (blockIdx % copies) of a bins-wide histogram (target 0 only)
template <int BLOCK>
__device__ __forceinline__ void hist_flush_copies(uint32_t (*lh)[NBINS], uint32_t nb, uint32_t copies, u64 *acc) {
    __syncthreads();
    u64 *dst = acc + NCOUNTS + (blockIdx.x % copies) * nb;
    for (uint32_t b = threadIdx.x; b < nb; b += BLOCK) {
        const uint32_t c = lh[0][b];
        if (c) atomicAdd(&dst[b], (u64)c);
    }
}

__device__ __forceinline__ uint32_t active_wgs(u64 count, u64 per_wg) {
    const u64 want = (count + per_wg - 1) / per_wg;
    return (uint32_t)(want < (u64)gridDim.x ? want : (u64)gridDim.x);
}

// Sample phase (x.sample_ready: the sharded window over an all-gathered
// sample -- no gather, the first digit read from `sample`): init
// (ADV_INIT_SAMPLE: a.init_*, a.r_lo / r_hi) -> gather +
// first digit -> up to two more sample digits, each behind a grid barrier.
// Workgroup 0 publishes the state in a.st_out: MODE_MAIN with the window, or
// MODE_DONE with an error.  Replaces k_gather<true> + two k_level launches.
__global__ __launch_bounds__(DENSE_BLK) void k_head(StepArgs a, CoopArgs x, const int32_t *__restrict__ keys,
                                                    u64 n_keys, u64 stride, uint32_t *__restrict__ sample, u64 s) {
    __shared__ SelState ss;
    __shared__ u64 scratch[2 * (DENSE_BLK / WAVE) + 8];
    __shared__ __attribute__((aligned(16))) uint32_t lh[2][NBINS];
    __shared__ uint32_t s_base[BAR_NG];
    KTH_STAMP(a, 0);
    GridBar gb = grid_bar_init(x.bar, s_base);
    for (int i = threadIdx.x; i < 2 * NBINS / 4; i += DENSE_BLK) reinterpret_cast<uint4 *>(&lh[0][0])[i] = make_uint4(0, 0, 0, 0);
    // the streaming pass's count slot and the candidate count: k_finish of the
    // previous select read them last and nothing here reads them, so every
    // workgroup clears its share first, under the gather (workgroup 0 alone
    // clearing them at the end: the same select time, 4 interleaved rounds)
    for (u64 i = (u64)blockIdx.x * DENSE_BLK + threadIdx.x; i < a.zero_words; i += (u64)gridDim.x * DENSE_BLK)
        a.stats_zero[i] = 0;
    advance<DENSE_BLK>(ss, a, scratch);
    bool share;
    HistPlan plan = make_plan(ss, &share);
    // a digit of the sample (written through by every workgroup's gather, or
    // already there) in 16-byte sc1 loads, HEAD_UNROLL per thread in flight;
    // s is a multiple of 64
    auto hist_sample = [&]() {
        const CoherentBuf sb(sample, (uint32_t)(s * 4));
        const uint32_t nv = (uint32_t)(s / 4), per = DENSE_BLK * HEAD_UNROLL;
        for (uint32_t v0 = blockIdx.x * per; v0 < nv; v0 += gridDim.x * per) {
            uint4 q[HEAD_UNROLL];
#pragma unroll
            for (int u = 0; u < HEAD_UNROLL; ++u) {
                const uint32_t v = v0 + u * DENSE_BLK + threadIdx.x;
                q[u] = sb.load16(v < nv ? v * 16u : 0u);
            }
#pragma unroll
            for (int u = 0; u < HEAD_UNROLL; ++u) {
                const bool in = v0 + u * DENSE_BLK + threadIdx.x < nv;
                hist_add<DENSE_BLK>(lh, plan, q[u].x, in);
                hist_add<DENSE_BLK>(lh, plan, q[u].y, in);
                hist_add<DENSE_BLK>(lh, plan, q[u].z, in);
                hist_add<DENSE_BLK>(lh, plan, q[u].w, in);
            }
        }
    };
    bool from_chunks = false;  // block-uniform (kernel arguments and the fresh state)
#ifdef KTH_HEAD_STORE_SAMPLE  // design exploration: the round-4 head (sample written through)
    constexpr bool kHeadStore = true;
#else
    constexpr bool kHeadStore = false;
#endif
    if (x.sample_ready)
        hist_sample();
    else if (gather_head_fast<DENSE_BLK, kHeadStore>(keys, stride, sample, s, lh, plan, blockIdx.x, gridDim.x))
        from_chunks = !kHeadStore;
    else
        gather_chunks<DENSE_BLK, true, true>(keys, n_keys, stride, sample, s, lh, plan);
#ifdef KTH_HEAD_DIAG  // diagnostic build: gather / flush / drain times (slots 4-6 are free on an early window)
    KTH_STAMP(a, 4);
#endif
    hist_flush<DENSE_BLK>(lh, plan, x.slots);
    KTH_STAMP(a, 1);
#ifdef KTH_HEAD_DIAG
    wait_mem();
    KTH_STAMP(a, 6);
#endif
    const EarlyWindow ew{a.r_lo, a.r_hi, x.slack64, x.abs_min};
    bool ok = true;
    for (int L = 0;; ++L) {
        grid_sync(gb, s_base, ok);
        if (x.fault) ok = false;  // test hook: as if this barrier had timed out
        if (L == 0) KTH_STAMP(a, 2);
        if (L == 1) KTH_STAMP(a, 5);
        pick_slot<DENSE_BLK>(ss, x.slots + (size_t)L * STATS_WORDS, share, scratch, &ew);
        if (L == 0) KTH_STAMP(a, 3);
        if (L == 1) KTH_STAMP(a, 6);
        if (ss.mode != MODE_SAMPLE || L + 1 >= HEAD_LEVELS) break;  // block-uniform
        plan = make_plan(ss, &share);
        for (int i = threadIdx.x; i < 2 * NBINS / 4; i += DENSE_BLK)
            reinterpret_cast<uint4 *>(&lh[0][0])[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        if (from_chunks)  // (the fast gather keeps no sample: writing 4 MiB through and waiting
                          // for it before the barrier cost more than re-reading the chunks)
            head_hist_chunks<DENSE_BLK>(keys, stride, s, lh, plan, blockIdx.x, gridDim.x);
        else
            hist_sample();
        hist_flush<DENSE_BLK>(lh, plan, x.slots + (size_t)(L + 1) * STATS_WORDS);
        if (L == 0) KTH_STAMP(a, 4);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        SelState o = ss;
        // a timed-out barrier of any workgroup (consumed here, so that a
        // sharded window -- k_head without a k_finish -- leaves no flag behind)
        const uint32_t berr = __hip_atomic_exchange(x.bar + BAR_ERR, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((!ok || berr) && !o.error) {
            o.error = ERR_BARRIER;
            o.mode = MODE_DONE;
        } else if (o.mode == MODE_SAMPLE && !o.error) {
            o.error = 16 + o.mode;
            o.mode = MODE_DONE;
        }
        o.share = 0;
        *a.st_out = o;
    }
    grid_bar_finish(gb, s_base);
    KTH_STAMP(a, 7);
}

// Finish phase: a.adv = ADV_DECIDE (state a.st_in + counts a.stats_in from the
// streaming pass; the candidates in a.cand) or ADV_INIT_FULL (radix path:
// a.init_n / init_k over a.keys).  Up to FIN_LEVELS digits, each behind a grid
// barrier, then the answer.  Replaces the decide level, the candidate levels
// and k_result.
//   * The domain is read from HBM once: when it fits (count <= grid *
//     FIN_LDS_KEYS), every workgroup keeps its contiguous slice in LDS and the
//     later digits scan LDS (each candidate level re-read the 21 MB of
//     candidates: ~6 us a level at 2^30).
//   * The first digit is 10 bits wide (FIN_D0; wider only when W > 32 would
//     need it): every key of the domain lands in it, so every workgroup
//     flushes nearly all of its bins -- 1024 global atomics a workgroup into 2
//     copies, not 2048 onto one.  When k_main<0> has histogrammed it already
//     (x.pre, PreHist: complete unless a workgroup flushed its staging
//     mid-pass), it is picked from there: no histogram, flush or barrier.  The later digits only see the keys of one bin, and
//     once that bin fits one workgroup's LDS, finish_tail ends the launch.
//   * Slots come in two sets used by alternate launches (x.slots: this
//     launch's, a.stats_zero: the other set, cleared here for the next one),
//     and the sample phase's slots (x.zero2) are cleared here too: no barrier
//     after the last level.
constexpr int FIN_LDS_KEYS = 32768;  // LDS-resident keys per workgroup (128 KiB of dynamic LDS)
constexpr int FIN_UNROLL = 4;        // 16-B loads in flight per thread (1024-thread workgroups: <= 128 VGPRs)

__device__ __forceinline__ void finish_keys(uint32_t (*lh)[NBINS], const HistPlan &plan, const uint4 &x, bool xr,
                                            uint32_t valid4) {
    const uint32_t X = xr ? 0x80000000u : 0u;
    hist_add<DENSE_BLK>(lh, plan, x.x ^ X, valid4 & 1u);
    hist_add<DENSE_BLK>(lh, plan, x.y ^ X, valid4 & 2u);
    hist_add<DENSE_BLK>(lh, plan, x.z ^ X, valid4 & 4u);
    hist_add<DENSE_BLK>(lh, plan, x.w ^ X, valid4 & 8u);
}

// The tail of k_finish: once a level's picked bin holds <= FIN_LDS_KEYS keys,
// the remaining digits need no more grid barriers.  Every workgroup appends
// its slice's keys of that bin to x.tail: one atomic on the tail word adds
// its key count to the low half (its offset) and its arrival to the high half;
// each writes its keys and then counts itself written (a non-returning add).
// The workgroup that reserved last waits until the others are written, loads
// every key of the tail into its LDS and resolves the remaining digits alone,
// with block barriers only.  (A grid level costs ~10
// us: flush round trip + barrier + pick; the tail ~3 round trips.)  One CU
// scans ~0.6 keys a clock (a 64-lane VALU op takes 4 clocks), so every pass
// over keys here is lean: one scan of the slice (staged in LDS), 16-byte LDS
// reads and one target in the finisher's levels.  Returns true on the
// workgroup that finished.  Keys go to x.tail as order keys (xr: the domain
// is the raw int32 input).
constexpr uint32_t TAIL_STAGE = 2 * NBINS;  // keys a workgroup stages in LDS (the histogram's space)
// One atomic reserves and arrives (see finish_tail): select 0.6769 -> 0.6749
// ms against a reservation and then an arrival (4 interleaved rounds, one
// box).  (Loading k_finish's slice by LDS-DMA instead of registers when
// PreHist gives the first digit measured equal, 0.6729 vs 0.6723 ms: the
// slice lands ~3.5 us after the decide either way; reading and picking
// PreHist takes ~4 us more, profiles/r5_select_stamps.txt.)

__device__ bool finish_tail(const StepArgs &a, SelState &ss, const CoopArgs &x, uint4 *res, u64 nk, bool xr,
                            uint32_t (*lh)[NBINS], u64 *scratch) {
    __shared__ uint32_t s_n, s_last, s_total, s_ln;
    __shared__ uint32_t s_list[WAVE];
    __shared__ u64 s_off, s_c;
    const uint32_t X = xr ? 0x80000000u : 0u;
    const uint32_t W = ss.W, base = ss.base, done = ss.t[0].done, prefix = ss.t[0].prefix;
    const uint32_t psh = W - done;  // done >= 1: a level was picked
    const uint32_t nv = (uint32_t)((nk + 3) / 4);
    u64 *ctl = reinterpret_cast<u64 *>(x.bar + BAR_TAIL);
    uint32_t *stage = &lh[0][0];
    const int lane = threadIdx.x & (WAVE - 1);
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    // one scan: the bin's keys appended to the LDS stage (ballot + mbcnt, one
    // LDS atomic a wave and key slot that has any); a slice with more than
    // TAIL_STAGE of them (skewed data) is written by a second scan instead
    auto keep = [&](uint32_t key, bool valid) {
        const bool m = valid && ((key - base) >> psh) == prefix;
        const u64 b = __ballot(m);
        if (b == 0) return;  // wave-uniform
        uint32_t at = 0;
        if (lane == 0) at = atomicAdd(&s_n, (uint32_t)__popcll(b));
        at = __shfl(at, 0, WAVE);
        const uint32_t i = at + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        if (m && i < TAIL_STAGE) stage[i] = key;
    };
    for (uint32_t v0 = 0; v0 < nv; v0 += DENSE_BLK) {  // wave-convergent
        const uint32_t v = v0 + threadIdx.x;
        uint4 q = make_uint4(0, 0, 0, 0);
        uint32_t valid4 = 0;
        if (v < nv) {
            q = res[v];
            const u64 e = 4ull * v;
            valid4 = nk - e >= 4 ? 0xFu : (1u << (uint32_t)(nk - e)) - 1u;
        }
        keep(q.x ^ X, valid4 & 1u);
        keep(q.y ^ X, valid4 & 2u);
        keep(q.z ^ X, valid4 & 4u);
        keep(q.w ^ X, valid4 & 8u);
    }
    __syncthreads();
    const uint32_t n_mine = s_n;
    if (threadIdx.x == 0) {  // the reservation is the arrival: one round trip
        const u64 old = __hip_atomic_fetch_add(ctl, (1ull << 32) | n_mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_off = (uint32_t)old;
        s_last = (uint32_t)(old >> 32) == gridDim.x - 1u;
        s_total = (uint32_t)old + n_mine;
    }
    __syncthreads();
    const uint32_t off = (uint32_t)s_off;
    if (n_mine <= TAIL_STAGE) {
        for (uint32_t i = threadIdx.x; i < n_mine; i += DENSE_BLK)
            if (off + i < (uint32_t)FIN_LDS_KEYS)
                __hip_atomic_store(x.tail + off + i, stage[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {  // block-uniform: every key of the bin again, in a second scan
        __shared__ uint32_t s_pos;
        if (threadIdx.x == 0) s_pos = 0;
        __syncthreads();
        for (uint32_t v = threadIdx.x; v < nv; v += DENSE_BLK) {
            const uint4 q = res[v];
            const u64 e = 4ull * v;
            const uint32_t valid4 = nk - e >= 4 ? 0xFu : (1u << (uint32_t)(nk - e)) - 1u;
            const uint32_t k4[4] = {q.x ^ X, q.y ^ X, q.z ^ X, q.w ^ X};
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (((valid4 >> j) & 1u) && ((k4[j] - base) >> psh) == prefix) {
                    const uint32_t i = atomicAdd(&s_pos, 1u);
                    if (off + i < (uint32_t)FIN_LDS_KEYS)
                        __hip_atomic_store(x.tail + off + i, k4[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
        }
    }
    wait_mem();
    __syncthreads();
    // the others' keys are in once each has counted itself written (a
    // non-returning add after its stores are performed); the last to
    // reserve waits for that, bounded, and resets both words
    uint32_t *written = x.bar + BAR_TAIL_WRITTEN;
    if (!s_last) {
        if (threadIdx.x == 0) __hip_atomic_fetch_add(written, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        KTH_STAMP(a, 5);
        return false;
    }
    if (threadIdx.x == 0) {
        uint32_t spins = 0;
        while (__hip_atomic_load(written, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gridDim.x - 1u) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins >= BAR_SPIN_LIMIT) {
                ss.error = ERR_BARRIER;
                ss.mode = MODE_DONE;
                break;
            }
        }
        __hip_atomic_store(written, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next select
        __hip_atomic_store(ctl, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (x.fault) {  // test hook: as if this wait had timed out (the PreHist path has no grid barrier)
            ss.error = ERR_BARRIER;
            ss.mode = MODE_DONE;
        }
    }
    __syncthreads();
    KTH_STAMP(a, 5);
    if (ss.error) return true;  // block-uniform (the state carries the timeout)
    const uint32_t total = s_total;
    if (total > (uint32_t)FIN_LDS_KEYS) {  // cannot happen: the bin's reduced count was checked
        if (threadIdx.x == 0) {
            ss.error = 32;
            ss.mode = MODE_DONE;
        }
        __syncthreads();
        return true;
    }
    // 16-byte device-coherent loads, FIN_UNROLL in flight per thread (a
    // per-key loop waited one round trip per key); the last vector is padded
    // with a key of another bin of the entry digit, which matches no later
    // prefix either
    const uint32_t nq = (total + 3) / 4;
    const uint32_t pad = base + ((prefix ^ 1u) << psh);  // a key of another bin of the entry digit
    {
        constexpr int TU = FIN_LDS_KEYS / 4 / DENSE_BLK;
        static_assert(TU % FIN_UNROLL == 0, "tail loads in FIN_UNROLL batches");
        const CoherentBuf tb(x.tail, FIN_LDS_KEYS * 4);
        for (int u0 = 0; u0 < TU; u0 += FIN_UNROLL) {
            if ((uint32_t)(u0 * DENSE_BLK) >= nq) break;  // block-uniform
            uint4 q[FIN_UNROLL];
#pragma unroll
            for (int u = 0; u < FIN_UNROLL; ++u) {
                const uint32_t v = (u0 + u) * DENSE_BLK + threadIdx.x;
                q[u] = v < nq ? tb.load16(v * 16u) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < FIN_UNROLL; ++u) {
                const uint32_t v = (u0 + u) * DENSE_BLK + threadIdx.x;
                if (v == total / 4 && (total & 3u)) {
                    if ((total & 3u) <= 1) q[u].y = pad;
                    if ((total & 3u) <= 2) q[u].z = pad;
                    q[u].w = pad;
                }
                res[(u0 + u) * DENSE_BLK + threadIdx.x] = q[u];
            }
        }
        __syncthreads();
    }
    KTH_STAMP(a, 6);
    // the remaining digits in LDS, one target (pick_state ends with a barrier)
    constexpr int PER = NBINS / DENSE_BLK;
    for (int it = 0; ss.mode == MODE_CAND || ss.mode == MODE_FULL; ++it) {  // block-uniform
        (void)it;
        const uint32_t dn = ss.t[0].done, pf = ss.t[0].prefix, d = digit_bits(ss, dn);
        const uint32_t msh = W - dn, sh = W - dn - d, mask = (1u << d) - 1u;
        for (int i = threadIdx.x; i < NBINS / 4; i += DENSE_BLK) reinterpret_cast<uint4 *>(&lh[0][0])[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        auto add = [&](uint32_t key) {
            const uint32_t v = key - base;
            if ((v >> msh) == pf) atomicAdd(&lh[0][(v >> sh) & mask], 1u);  // msh < 32: dn >= 1
        };
        for (uint32_t v = threadIdx.x; v < nq; v += DENSE_BLK) {
            const uint4 q = res[v];
            add(q.x);
            add(q.y);
            add(q.z);
            add(q.w);
        }
        __syncthreads();
        u64 h0[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) h0[j] = lh[0][threadIdx.x * PER + j];
        pick_state<DENSE_BLK, PER>(ss, h0, h0, true, scratch, nullptr, &s_c);
#ifdef KTH_STAMPS_BUILD
        if (it < 2) KTH_STAMP(a, 1 + it);  // diagnostic only: the finisher overwrites its own early stamps
#endif
        // <= 64 keys left in the picked bin (uniform keys: ~8): list them and
        // rank them in one wave instead of another histogram level
        if ((ss.mode == MODE_CAND || ss.mode == MODE_FULL) && s_c <= (u64)WAVE) {  // block-uniform
            const uint32_t dl = ss.t[0].done, pl = ss.t[0].prefix, msl = W - dl;  // 1 <= dl < W
            if (threadIdx.x == 0) s_ln = 0;
            __syncthreads();
            auto put = [&](uint32_t key) {  // wave-convergent
                const bool m = ((key - base) >> msl) == pl;
                const u64 b = __ballot(m);
                if (b == 0) return;
                uint32_t at = 0;
                if (lane == 0) at = atomicAdd(&s_ln, (uint32_t)__popcll(b));
                at = __shfl(at, 0, WAVE);
                const uint32_t i = at + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
                if (m && i < (uint32_t)WAVE) s_list[i] = key;
            };
            for (uint32_t v0 = 0; v0 < nq; v0 += DENSE_BLK) {
                const uint32_t v = v0 + threadIdx.x;
                const uint4 q = v < nq ? res[v] : make_uint4(pad, pad, pad, pad);
                put(q.x);
                put(q.y);
                put(q.z);
                put(q.w);
            }
            __syncthreads();
            if (threadIdx.x < WAVE) {
                const uint32_t ln = s_ln < (uint32_t)WAVE ? s_ln : (uint32_t)WAVE;
                const uint32_t mine = (uint32_t)lane < ln ? s_list[lane] : 0u;
                uint32_t lt = 0, le = 0;
                for (uint32_t j = 0; j < ln; ++j) {
                    const uint32_t o = s_list[j];
                    lt += o < mine ? 1u : 0u;
                    le += o <= mine ? 1u : 0u;
                }
                const u64 kk = ss.t[0].k;
                const bool hit = (uint32_t)lane < ln && (u64)lt < kk && kk <= (u64)le;
                if (hit) ss.answer = mine;  // equal keys write the same value
                if (__ballot(hit) == 0 && lane == 0) ss.error = 33;
            }
            __syncthreads();
            if (threadIdx.x == 0) ss.mode = MODE_DONE;
            __syncthreads();
            break;
        }
    }
    KTH_STAMP(a, 3);
    return true;
}

__global__ __launch_bounds__(DENSE_BLK) void k_finish(StepArgs a, CoopArgs x) {
    __shared__ SelState ss;
    __shared__ u64 scratch[2 * (DENSE_BLK / WAVE) + 8];
    __shared__ __attribute__((aligned(16))) uint32_t lh[2][NBINS];
    extern __shared__ uint4 res[];  // FIN_LDS_KEYS / 4 entries (dynamic)
    __shared__ uint32_t s_base[BAR_NG];
    __shared__ u64 s_cnt0;
    KTH_STAMP(a, 0);
    GridBar gb = grid_bar_init(x.bar, s_base);
    for (int i = threadIdx.x; i < 2 * NBINS / 4; i += DENSE_BLK) reinterpret_cast<uint4 *>(&lh[0][0])[i] = make_uint4(0, 0, 0, 0);
    const uint32_t pre_incomplete = x.pre ? x.pre[PRE_INCOMPLETE] : 1u;  // (loaded beside the state)
    advance<DENSE_BLK>(ss, a, scratch);
    if (threadIdx.x == 0 && (ss.mode == MODE_CAND || ss.mode == MODE_FULL) && ss.t[0].done == 0)
        ss.d0 = fin_first_digit(ss.W);
    __syncthreads();
    // the candidates' first digit from k_main (grid-uniform: every workgroup reads the same words)
    const bool use_pre = pre_incomplete == 0u && ss.mode == MODE_CAND && ss.t[0].done == 0;
    KTH_STAMP(a, 1);
    // the domain (block-uniform): candidates or the input, and this workgroup's slice
    const uint32_t mode0 = ss.mode;
    const bool live = mode0 == MODE_CAND || mode0 == MODE_FULL;
    const uint32_t *dom = mode0 == MODE_FULL ? reinterpret_cast<const uint32_t *>(a.keys) : a.cand;
    const u64 count = mode0 == MODE_CAND ? min(*a.cand_count, a.cap) : a.n_local;
    const bool xr = mode0 == MODE_FULL;  // input keys: int32 -> order-preserving
    const bool aligned = (reinterpret_cast<uintptr_t>(dom) & 15u) == 0;
    const bool resident = live && count <= (u64)gridDim.x * FIN_LDS_KEYS;
    u64 b0 = 0, nk = 0;  // slice [b0, b0 + nk) of the domain
    if (resident) {
        const u64 per = ((count + gridDim.x - 1) / gridDim.x + 3) & ~(u64)3;
        b0 = min((u64)blockIdx.x * per, count);
        nk = min(per, count - b0);
    }
    bool ok = true, tail = false;
    for (int L = 0; L < FIN_LEVELS; ++L) {
        const uint32_t mode = ss.mode;
        if (mode != MODE_CAND && mode != MODE_FULL) break;  // block-uniform
        bool share;
        const HistPlan plan = make_plan(ss, &share);
        if (L > 0) {
            for (int i = threadIdx.x; i < 2 * NBINS / 4; i += DENSE_BLK)
                reinterpret_cast<uint4 *>(&lh[0][0])[i] = make_uint4(0, 0, 0, 0);
            __syncthreads();
        }
        const bool pre0 = L == 0 && use_pre;  // the digit is picked from PreHist below
        if (resident) {
            const uint32_t nv = (uint32_t)((nk + 3) / 4);
            if (L == 0) {  // HBM -> registers -> histogram + LDS (pre0: LDS only)
                // the domain's first digit: one target, no prefix yet, so a full
                // vector's keys cost a subtract, a shift and an LDS atomic each
                // (hist_add's generic two-target path was ~2x the VALU issue)
                const bool one = plan.h[0] && !plan.h[1] && plan.done[0] == 0;
                const uint32_t X = xr ? 0x80000000u : 0u, bs = plan.base, sh = plan.shift[0], mk = plan.mask[0];
                auto add4 = [&](const uint4 &q) {
                    atomicAdd(&lh[0][(((q.x ^ X) - bs) >> sh) & mk], 1u);
                    atomicAdd(&lh[0][(((q.y ^ X) - bs) >> sh) & mk], 1u);
                    atomicAdd(&lh[0][(((q.z ^ X) - bs) >> sh) & mk], 1u);
                    atomicAdd(&lh[0][(((q.w ^ X) - bs) >> sh) & mk], 1u);
                };
                if (aligned) {
                    const uint4 *src = reinterpret_cast<const uint4 *>(dom + b0);
                    for (uint32_t v0 = 0; v0 < nv; v0 += FIN_UNROLL * DENSE_BLK) {
                        uint4 q[FIN_UNROLL];
#pragma unroll
                        for (int u = 0; u < FIN_UNROLL; ++u) {
                            const uint32_t v = v0 + u * DENSE_BLK + threadIdx.x;
                            q[u] = v < nv ? load_nt(src + v) : make_uint4(0, 0, 0, 0);
                        }
#pragma unroll
                        for (int u = 0; u < FIN_UNROLL; ++u) {
                            const uint32_t v = v0 + u * DENSE_BLK + threadIdx.x;
                            if (v < nv) {
                                const u64 e = 4ull * v;
                                res[v] = q[u];
                                if (pre0)
                                    ;  // (the digit comes from PreHist)
                                else if (one && nk - e >= 4)
                                    add4(q[u]);
                                else
                                    finish_keys(lh, plan, q[u], xr, nk - e >= 4 ? 0xFu : (1u << (uint32_t)(nk - e)) - 1u);
                            }
                        }
                    }
                } else {
                    for (uint32_t v = threadIdx.x; v < nv; v += DENSE_BLK) {
                        uint4 q = make_uint4(0, 0, 0, 0);
                        const u64 e = b0 + 4ull * v, left = b0 + nk - e;
                        q.x = dom[e];
                        if (left > 1) q.y = dom[e + 1];
                        if (left > 2) q.z = dom[e + 2];
                        if (left > 3) q.w = dom[e + 3];
                        res[v] = q;
                        if (!pre0) finish_keys(lh, plan, q, xr, left >= 4 ? 0xFu : (1u << (uint32_t)left) - 1u);
                    }
                }
            } else {  // the slice from LDS
                for (uint32_t v = threadIdx.x; v < nv; v += DENSE_BLK) {
                    const u64 e = 4ull * v;
                    finish_keys(lh, plan, res[v], xr, nk - e >= 4 ? 0xFu : (1u << (uint32_t)(nk - e)) - 1u);
                }
            }
        } else if (!pre0) {
            // streamed from HBM every level (a domain larger than the grid's LDS)
            const uint32_t active = active_wgs(count, L == 0 ? x.dense_per_wg : x.sparse_per_wg);
            auto f = [&](const uint32_t *k, uint32_t valid, auto full) {
#pragma unroll
                for (int j = 0; j < 4 * FIN_UNROLL; ++j)
                    hist_add<DENSE_BLK>(lh, plan, k[j], decltype(full)::value || ((valid >> j) & 1u));
            };
            if (blockIdx.x < active) {
                if (xr)
                    stream_tiles<DENSE_BLK, FIN_UNROLL, true>(dom, count, blockIdx.x, active, f);
                else
                    stream_tiles<DENSE_BLK, FIN_UNROLL, false>(dom, count, blockIdx.x, active, f);
            }
        }
#ifdef KTH_STAMPS_BUILD  // diagnostic: the slice landed (p2 is free on the PreHist path)
        if (pre0) {
            wait_mem();
            KTH_STAMP(a, 2);
        }
#endif
        u64 *slot = x.slots + (size_t)L * STATS_WORDS;
        // first digit: every key lands, so every workgroup flushes nearly every
        // bin -- into NBINS / bins copies; later digits see one bin's keys
        const uint32_t nb = plan.mask[0] + 1u, copies = L == 0 ? NBINS / nb : 1u;
        if (pre0) {
            pick_pre<DENSE_BLK>(ss, x.pre, nb, scratch, &s_cnt0);
        } else {
            if (copies > 1)
                hist_flush_copies<DENSE_BLK>(lh, nb, copies, slot);
            else
                hist_flush<DENSE_BLK>(lh, plan, slot);
            if (L == 0) KTH_STAMP(a, 2);
            grid_sync(gb, s_base, ok);
            if (x.fault) ok = false;  // test hook: as if this barrier had timed out
            if (L == 0) KTH_STAMP(a, 3);
            if (copies > 1)
                pick_slot_copies<DENSE_BLK>(ss, slot, nb, copies, reinterpret_cast<u64 *>(&lh[0][0]), scratch, &s_cnt0);
            else
                pick_slot<DENSE_BLK>(ss, slot, share, scratch, nullptr, &s_cnt0);
        }
        KTH_STAMP(a, 4 + L);
        // a small bin left: the last workgroup to arrive finishes alone (block-uniform)
        if (resident && (ss.mode == MODE_CAND || ss.mode == MODE_FULL) && s_cnt0 <= (u64)FIN_LDS_KEYS) {
            tail = true;
            break;
        }
    }
    grid_bar_finish(gb, s_base);
    bool writer = blockIdx.x == 0;
    if (tail) {
        writer = finish_tail(a, ss, x, res, nk, xr, lh, scratch);
    }
    if (writer && threadIdx.x == 0) {
        SelState o = ss;
        const uint32_t berr = __hip_atomic_exchange(x.bar + BAR_ERR, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((!ok || berr) && !o.error) o.error = ERR_BARRIER;
        if (o.mode != MODE_DONE && !o.error) o.error = 16 + o.mode;
        *a.st_out = o;
        // only a verified answer reaches d_out: after a barrier timeout (a grid
        // that was not co-resident) or a failed check d_out keeps its value and
        // the error is in the state (kth_ctx_last_stats) and d_status[1]
        if (x.d_out && !o.error) *x.d_out = i32_of_key(o.answer);
        if (x.d_status) {
            x.d_status[0] = i32_of_key(o.answer);
            x.d_status[1] = (int32_t)o.error;
        }
    }
    // the other slot set and the sample phase's slots, for the next select
    for (u64 i = (u64)blockIdx.x * DENSE_BLK + threadIdx.x; i < a.zero_words; i += (u64)gridDim.x * DENSE_BLK)
        a.stats_zero[i] = 0;
    for (u64 i = (u64)blockIdx.x * DENSE_BLK + threadIdx.x; i < x.zero2_words; i += (u64)gridDim.x * DENSE_BLK)
        x.zero2[i] = 0;
    if (x.pre_zero)
        for (u64 i = (u64)blockIdx.x * DENSE_BLK + threadIdx.x; i < (u64)PRE_WORDS; i += (u64)gridDim.x * DENSE_BLK)
            x.pre_zero[i] = 0u;
    KTH_STAMP(a, 7);
}

}  // namespace kth
