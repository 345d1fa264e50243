// kth_gridbar.hpp -- grid-wide barriers of the cooperative kernels (k_head,
// k_finish) and the device-coherent buffer reads they use.
// Included by kth_kernels.hip before the kernels.
#pragma once
#include "kth_device.hpp"

namespace kth {

constexpr int HEAD_LEVELS = 3;       // sample digits: 11 + 11 + 10 bits
constexpr int FIN_LEVELS = 3;        // candidate / input digits
constexpr int HEAD_UNROLL = 4;       // 16-B loads per thread per sample tile (16 Ki keys per 1024-thread tile)
constexpr int BAR_GROUP_STRIDE = 64; // words between group counters (separate 256-B lines)
constexpr int BAR_NG = 64;           // group counters (workgroup w arrives on w % BAR_NG; wave 0's 64 lanes poll them)
constexpr int BAR_BASE = BAR_NG * BAR_GROUP_STRIDE;   // the groups' base values (BAR_NG words)
constexpr int BAR_ERR = BAR_BASE + BAR_GROUP_STRIDE;
constexpr int BAR_TAIL = BAR_ERR + BAR_GROUP_STRIDE;  // u64 at this u32 index: k_finish tail (arrivals << 32 | keys)
constexpr int BAR_TAIL_WRITTEN = BAR_TAIL + 32;       // k_finish tail: workgroups whose keys are written
constexpr int BAR_TOPK_ARRIVE = BAR_TAIL + 48;        // k_topk_bases: arrivals (zeroed by the last one)
constexpr int BAR_WORDS = BAR_TAIL + BAR_GROUP_STRIDE;  // u32 words of barrier state per ctx
static_assert(BAR_TAIL_WRITTEN >= BAR_TAIL + 2 && BAR_TOPK_ARRIVE > BAR_TAIL_WRITTEN && BAR_TOPK_ARRIVE < BAR_WORDS,
              "the tail word (u64), its written count and the top-k arrival counter are distinct words");
static_assert(BAR_NG <= WAVE && BAR_NG <= BAR_GROUP_STRIDE, "one wave polls every group; the bases fit one stride");
constexpr uint32_t BAR_SPIN_LIMIT = 1u << 21;         // polls before a barrier gives up (seconds)
constexpr uint32_t ERR_BARRIER = 64;

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
// (blockIdx % BAR_NG: same-address atomics serialise, ~36 ns each, so a
// 1024-workgroup grid arrives 16 to a counter); lanes 0..BAR_NG-1 of wave 0
// then poll all group counters at once until each has reached its target.  Counters only grow (u32, compared modulo 2^32): the value a group
// counter had when the kernel started is kept in bar[BAR_BASE + g], written
// by workgroup 0 of the previous barrier kernel at its end (GridBar::finish),
// so no reset, no last-arriver hand-off and nothing zeroed between calls --
// two memory round trips on the critical path.  Every spin is bounded: a
// barrier that does not complete raises bar[BAR_ERR] and returns ok = false.
struct GridBar {
    uint32_t *bar;
    uint32_t n;  // barriers passed in this kernel
};

__device__ __forceinline__ uint32_t group_size(uint32_t g) { return (gridDim.x - g + BAR_NG - 1u) / BAR_NG; }

// Kernel start: every thread calls; s_base is LDS of BAR_NG words.
__device__ __forceinline__ GridBar grid_bar_init(uint32_t *bar, uint32_t *s_base) {
    if (threadIdx.x < BAR_NG) s_base[threadIdx.x] = bar[BAR_BASE + threadIdx.x];
    return GridBar{bar, 0u};
}

__device__ __forceinline__ void grid_sync(GridBar &gb, const uint32_t *s_base, bool &ok) {
    __shared__ uint32_t s_ok;
    wait_mem();
    __syncthreads();
    gb.n++;
    if (threadIdx.x < WAVE) {
        const uint32_t lane = threadIdx.x, groups = gridDim.x < (uint32_t)BAR_NG ? gridDim.x : (uint32_t)BAR_NG;
        if (lane == 0)
            __hip_atomic_fetch_add(gb.bar + (blockIdx.x % BAR_NG) * BAR_GROUP_STRIDE, 1u, __ATOMIC_RELAXED,
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
    if (blockIdx.x == 0 && threadIdx.x < BAR_NG)
        gb.bar[BAR_BASE + threadIdx.x] = s_base[threadIdx.x] + gb.n * group_size(threadIdx.x);
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

}  // namespace kth
