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

constexpr int HEAD_LEVELS = 3;       // sample digits: 11 + 11 + 10 bits
constexpr int FIN_LEVELS = 3;        // candidate / input digits
constexpr int HEAD_UNROLL = 4;       // 16-B loads per thread per sample tile (16 Ki keys per 1024-thread tile)
constexpr int BAR_GROUP_STRIDE = 64; // words between group counters (separate 256-B lines)
constexpr int BAR_BASE = 8 * BAR_GROUP_STRIDE, BAR_ERR = BAR_BASE + BAR_GROUP_STRIDE;
constexpr int BAR_WORDS = BAR_ERR + BAR_GROUP_STRIDE;  // u32 words of barrier state per ctx
constexpr uint32_t BAR_SPIN_LIMIT = 1u << 21;         // polls before a barrier gives up (seconds)
constexpr uint32_t ERR_BARRIER = 64;

struct CoopArgs {
    u64 *slots;        // HEAD_LEVELS / FIN_LEVELS histogram slots of STATS_WORDS, zero on entry
    uint32_t *bar;     // BAR_WORDS of barrier state
    int32_t *d_out, *d_status;
    u64 dense_per_wg, sparse_per_wg;  // keys per active workgroup: first digit of a domain / later digits
    uint32_t slack64;  // k_head early window (EarlyWindow); 0 = exact sample ranks
    u64 *zero2;        // k_finish: a second region to clear (the sample phase's slots)
    u64 zero2_words;
};

// This wave's outstanding global accesses (atomics, write-through stores) are
// performed: every wave of a workgroup waits before its barrier arrival.
__device__ __forceinline__ void wait_mem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Grid-wide barrier of the calling kernel (all threads call).  Data crosses
// workgroups inside these kernels only through device-coherent accesses --
// histogram atomics, write-through (sc1) stores, sc1 loads -- so the barrier
// needs no L2 write-back / invalidate (an agent-scope release / acquire fence
// per workgroup made every barrier ~10 us: 32 workgroups per XCD each
// flushing and invalidating the shared L2).  Each wave waits for its own
// accesses to be performed before the workgroup arrives.
//
// Arrival is one non-returning atomic add on the workgroup's group counter
// (blockIdx % 8: same-address atomics serialise, ~36 ns each); lanes 0..7 of
// wave 0 then poll all group counters at once until each has reached its
// target.  Counters only grow (u32, compared modulo 2^32): the value a group
// counter had when the kernel started is kept in bar[BAR_BASE + g], written
// by workgroup 0 of the previous barrier kernel at its end (GridBar::finish),
// so no reset, no last-arriver hand-off and nothing zeroed between calls --
// two memory round trips on the critical path.  Every spin is bounded: a
// barrier that does not complete raises bar[BAR_ERR] and returns ok = false.
struct GridBar {
    uint32_t *bar;
    uint32_t n;  // barriers passed in this kernel
};

__device__ __forceinline__ uint32_t group_size(uint32_t g) { return (gridDim.x - g + 7u) / 8u; }

// Kernel start: every thread calls; s_base is LDS of 8 words.
__device__ __forceinline__ GridBar grid_bar_init(uint32_t *bar, uint32_t *s_base) {
    if (threadIdx.x < 8) s_base[threadIdx.x] = bar[BAR_BASE + threadIdx.x];
    return GridBar{bar, 0u};
}

__device__ __forceinline__ void grid_sync(GridBar &gb, const uint32_t *s_base, bool &ok) {
    __shared__ uint32_t s_ok;
    wait_mem();
    __syncthreads();
    gb.n++;
    if (threadIdx.x < WAVE) {
        const uint32_t lane = threadIdx.x, groups = gridDim.x < 8u ? gridDim.x : 8u;
        if (lane == 0)
            __hip_atomic_fetch_add(gb.bar + (blockIdx.x & 7u) * BAR_GROUP_STRIDE, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t target = lane < groups ? s_base[lane] + gb.n * group_size(lane) : 0u;
        bool done = lane >= groups;
        uint32_t spins = 0, good = 1;
        while (true) {
            if (!done) {
                const uint32_t v = __hip_atomic_load(gb.bar + lane * BAR_GROUP_STRIDE, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                done = (int32_t)(v - target) >= 0;
            }
            if (__ballot(!done) == 0) break;  // wave-uniform
            __builtin_amdgcn_s_sleep(1);
            if (++spins >= BAR_SPIN_LIMIT) {
                good = 0;
                if (lane == 0) __hip_atomic_fetch_or(gb.bar + BAR_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        if (lane == 0) s_ok = good;
    }
    __syncthreads();
    ok = ok && s_ok != 0;
}

// Kernel end, workgroup 0 (after its last barrier): the counters' values for
// the next barrier kernel.  Every workgroup passes the same number of barriers.
__device__ __forceinline__ void grid_bar_finish(const GridBar &gb, const uint32_t *s_base) {
    if (blockIdx.x == 0 && threadIdx.x < 8) gb.bar[BAR_BASE + threadIdx.x] = s_base[threadIdx.x] + gb.n * group_size(threadIdx.x);
}

// Load a level's reduced histograms (thread i: bins [i*PER, i*PER + PER)) with
// device-coherent loads, and pick.
template <int BLOCK>
__device__ __forceinline__ void pick_slot(SelState &ss, const u64 *slot, bool share, u64 *scratch,
                                          const EarlyWindow *ew) {
    constexpr int PER = NBINS / BLOCK;
    u64 h0[PER], h1[PER];
    const u64 *b0 = slot + NCOUNTS + threadIdx.x * PER;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        h0[j] = __hip_atomic_load(b0 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        h1[j] = share ? 0ull : __hip_atomic_load(b0 + NBINS + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    pick_state<BLOCK, PER>(ss, h0, h1, share, scratch, ew);
}

// The dense first digit of k_finish (nb <= NBINS / copies bins) is flushed
// into `copies` histogram copies (workgroup w adds to copy w % copies: fewer
// same-address atomics); the pick loads the NBINS words once and sums them.
template <int BLOCK>
__device__ __forceinline__ void pick_slot_copies(SelState &ss, const u64 *slot, uint32_t nb, uint32_t copies,
                                                 u64 *tmp /* NBINS u64 of LDS */, u64 *scratch) {
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
    pick_state<BLOCK, PER>(ss, h0, h0, true, scratch, nullptr);
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

// Device-coherent (sc1) 16-byte loads of a buffer other workgroups of this
// kernel wrote with write-through stores (k_head's sample).
struct CoherentBuf {
    __amdgpu_buffer_rsrc_t r;
    __device__ CoherentBuf(const void *p, uint32_t bytes)
        : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000)) {}
    __device__ __forceinline__ uint4 load16(uint32_t byte_off) const {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 16 /* sc1 */);
        return make_uint4(v[0], v[1], v[2], v[3]);
    }
};

__device__ __forceinline__ uint32_t active_wgs(u64 count, u64 per_wg) {
    const u64 want = (count + per_wg - 1) / per_wg;
    return (uint32_t)(want < (u64)gridDim.x ? want : (u64)gridDim.x);
}

// Sample phase: init (ADV_INIT_SAMPLE: a.init_*, a.r_lo / r_hi) -> gather +
// first digit -> up to two more sample digits, each behind a grid barrier.
// Workgroup 0 publishes the state in a.st_out: MODE_MAIN with the window, or
// MODE_DONE with an error.  Replaces k_gather<true> + two k_level launches.
__global__ __launch_bounds__(DENSE_BLK) void k_head(StepArgs a, CoopArgs x, const int32_t *__restrict__ keys,
                                                    u64 n_keys, u64 stride, uint32_t *__restrict__ sample, u64 s) {
    __shared__ SelState ss;
    __shared__ u64 scratch[2 * (DENSE_BLK / WAVE) + 8];
    __shared__ __attribute__((aligned(16))) uint32_t lh[2][NBINS];
    __shared__ uint32_t s_base[8];
    KTH_STAMP(a, 0);
    GridBar gb = grid_bar_init(x.bar, s_base);
    for (int i = threadIdx.x; i < 2 * NBINS / 4; i += DENSE_BLK) reinterpret_cast<uint4 *>(&lh[0][0])[i] = make_uint4(0, 0, 0, 0);
    advance<DENSE_BLK>(ss, a, scratch);
    bool share;
    HistPlan plan = make_plan(ss, &share);
    gather_chunks<DENSE_BLK, true, true>(keys, n_keys, stride, sample, s, lh, plan);
    hist_flush<DENSE_BLK>(lh, plan, x.slots);
    KTH_STAMP(a, 1);
    const EarlyWindow ew{a.r_lo, a.r_hi, x.slack64};
    bool ok = true;
    for (int L = 0;; ++L) {
        grid_sync(gb, s_base, ok);
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
        // the sample (written through by every workgroup's gather) in 16-byte
        // sc1 loads, HEAD_UNROLL per thread in flight; s is a multiple of 64
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
        hist_flush<DENSE_BLK>(lh, plan, x.slots + (size_t)(L + 1) * STATS_WORDS);
        if (L == 0) KTH_STAMP(a, 4);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        SelState o = ss;
        if (!ok && !o.error) {
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
    // the streaming pass's count slot and the candidate count (k_finish read them last)
    if (blockIdx.x == 0)
        for (u64 i = threadIdx.x; i < a.zero_words; i += DENSE_BLK) a.stats_zero[i] = 0;
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
//   * The first digit is 8 bits wide (FIN_D0; wider only when W > 30 needs
//     it): every key of the domain lands in it, so every workgroup flushes
//     nearly all of its bins -- 256 global atomics a workgroup, not 2048.  The
//     later digits only see the keys of one bin.
//   * Slots come in two sets used by alternate launches (x.slots: this
//     launch's, a.stats_zero: the other set, cleared here for the next one),
//     and the sample phase's slots (x.zero2) are cleared here too: no barrier
//     after the last level.
constexpr int FIN_LDS_KEYS = 32768;  // LDS-resident keys per workgroup (128 KiB of dynamic LDS)
constexpr int FIN_UNROLL = 4;        // 16-B loads in flight per thread (1024-thread workgroups: <= 128 VGPRs)
constexpr uint32_t FIN_D0 = 8;

__device__ __forceinline__ void finish_keys(uint32_t (*lh)[NBINS], const HistPlan &plan, const uint4 &x, bool xr,
                                            uint32_t valid4) {
    const uint32_t X = xr ? 0x80000000u : 0u;
    hist_add<DENSE_BLK>(lh, plan, x.x ^ X, valid4 & 1u);
    hist_add<DENSE_BLK>(lh, plan, x.y ^ X, valid4 & 2u);
    hist_add<DENSE_BLK>(lh, plan, x.z ^ X, valid4 & 4u);
    hist_add<DENSE_BLK>(lh, plan, x.w ^ X, valid4 & 8u);
}

__global__ __launch_bounds__(DENSE_BLK) void k_finish(StepArgs a, CoopArgs x) {
    __shared__ SelState ss;
    __shared__ u64 scratch[2 * (DENSE_BLK / WAVE) + 8];
    __shared__ __attribute__((aligned(16))) uint32_t lh[2][NBINS];
    extern __shared__ uint4 res[];  // FIN_LDS_KEYS / 4 entries (dynamic)
    __shared__ uint32_t s_base[8];
    KTH_STAMP(a, 0);
    GridBar gb = grid_bar_init(x.bar, s_base);
    for (int i = threadIdx.x; i < 2 * NBINS / 4; i += DENSE_BLK) reinterpret_cast<uint4 *>(&lh[0][0])[i] = make_uint4(0, 0, 0, 0);
    advance<DENSE_BLK>(ss, a, scratch);
    if (threadIdx.x == 0 && (ss.mode == MODE_CAND || ss.mode == MODE_FULL) && ss.t[0].done == 0)
        ss.d0 = ss.W > 30u ? ss.W - 22u : FIN_D0;
    __syncthreads();
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
    bool ok = true;
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
        if (resident) {
            const uint32_t nv = (uint32_t)((nk + 3) / 4);
            if (L == 0) {  // HBM -> registers -> histogram + LDS
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
                                const uint32_t valid4 = nk - e >= 4 ? 0xFu : (1u << (uint32_t)(nk - e)) - 1u;
                                res[v] = q[u];
                                finish_keys(lh, plan, q[u], xr, valid4);
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
                        finish_keys(lh, plan, q, xr, left >= 4 ? 0xFu : (1u << (uint32_t)left) - 1u);
                    }
                }
            } else {  // the slice from LDS
                for (uint32_t v = threadIdx.x; v < nv; v += DENSE_BLK) {
                    const u64 e = 4ull * v;
                    finish_keys(lh, plan, res[v], xr, nk - e >= 4 ? 0xFu : (1u << (uint32_t)(nk - e)) - 1u);
                }
            }
        } else {
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
        u64 *slot = x.slots + (size_t)L * STATS_WORDS;
        // first digit: every key lands, so every workgroup flushes nearly every
        // bin -- into NBINS / bins copies; later digits see one bin's keys
        const uint32_t nb = plan.mask[0] + 1u, copies = L == 0 ? NBINS / nb : 1u;
        if (copies > 1)
            hist_flush_copies<DENSE_BLK>(lh, nb, copies, slot);
        else
            hist_flush<DENSE_BLK>(lh, plan, slot);
        if (L == 0) KTH_STAMP(a, 2);
        grid_sync(gb, s_base, ok);
        if (L == 0) KTH_STAMP(a, 3);
        if (copies > 1)
            pick_slot_copies<DENSE_BLK>(ss, slot, nb, copies, reinterpret_cast<u64 *>(&lh[0][0]), scratch);
        else
            pick_slot<DENSE_BLK>(ss, slot, share, scratch, nullptr);
        KTH_STAMP(a, 4 + L);
    }
    grid_bar_finish(gb, s_base);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        SelState o = ss;
        const uint32_t berr = __hip_atomic_exchange(x.bar + BAR_ERR, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((!ok || berr) && !o.error) o.error = ERR_BARRIER;
        if (o.mode != MODE_DONE && !o.error) o.error = 16 + o.mode;
        *a.st_out = o;
        if (x.d_out) *x.d_out = i32_of_key(o.answer);
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
    KTH_STAMP(a, 7);
}

}  // namespace kth
