// wmix_probe.hip -- the HBM ceiling for top-k's write mix (not part of the
// product; a design probe).  kth_topk_i32 at k = n/2 reads 4 B per key and
// writes 12 B per kept key (int32 value + int64 index): 4n B in, 6n B out.
//   copy<U>        float4 copy, n words in and out (the plain copy ceiling)
//   mix_vec<U>     per 16-B load: 8 B of values + 16 B of indices out, 16-B /
//                  8-B stores, perfectly coalesced (the mix's ceiling)
//   mix_lane<U>    the same bytes as per-lane 4-B value and 8-B index stores
//                  (what k_topk_write's copy-out issues)
// Usage: wmix_probe [log2n=30]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

template <int U>
__global__ __launch_bounds__(256) void copy(const u32x4 *__restrict__ in, u32x4 *__restrict__ out,
                                            unsigned long long nv) {
    const unsigned long long tile = 256ull * U;
    for (unsigned long long t0 = (unsigned long long)blockIdx.x * tile; t0 < nv; t0 += (unsigned long long)gridDim.x * tile) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(&in[t0 + u * 256 + threadIdx.x]);
#pragma unroll
        for (int u = 0; u < U; ++u) out[t0 + u * 256 + threadIdx.x] = x[u];
    }
}

// half the keys "kept": keys 2j, 2j+1 of a 4-key load -> one u32x2 of values
// and one u32x4 (two int64) of indices
template <int U>
__global__ __launch_bounds__(256) void mix_vec(const u32x4 *__restrict__ in, u32x2 *__restrict__ vals,
                                               u32x4 *__restrict__ idx, unsigned long long nv) {
    const unsigned long long tile = 256ull * U;
    for (unsigned long long t0 = (unsigned long long)blockIdx.x * tile; t0 < nv; t0 += (unsigned long long)gridDim.x * tile) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(&in[t0 + u * 256 + threadIdx.x]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned long long i = t0 + u * 256 + threadIdx.x;
            vals[i] = u32x2{x[u].x, x[u].z};
            idx[i] = u32x4{(unsigned)(4 * i), (unsigned)(i >> 30), (unsigned)(4 * i + 2), (unsigned)(i >> 30)};
        }
    }
}

// the same bytes, as per-lane 4-B / 8-B stores of a contiguous output run per wave
template <int U>
__global__ __launch_bounds__(256) void mix_lane(const u32x4 *__restrict__ in, unsigned *__restrict__ vals,
                                                unsigned long long *__restrict__ idx, unsigned long long nv) {
    const unsigned long long tile = 256ull * U;
    const int lane = threadIdx.x & 63, w = threadIdx.x / 64;
    for (unsigned long long t0 = (unsigned long long)blockIdx.x * tile; t0 < nv; t0 += (unsigned long long)gridDim.x * tile) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = __builtin_nontemporal_load(&in[t0 + u * 256 + threadIdx.x]);
        // the wave's U * 64 loads keep 2 keys each: a run of U * 128 outputs
        const unsigned long long o0 = (t0 + (unsigned long long)w * 64) * 2;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned long long o = o0 + (unsigned long long)u * 512;
            vals[o + lane] = x[u].x;
            vals[o + 64 + lane] = x[u].z;
            idx[o + lane] = o + lane;
            idx[o + 64 + lane] = o + 64 + lane;
        }
    }
}

int main(int argc, char **argv) {
    const int log2n = argc > 1 ? atoi(argv[1]) : 30;
    const unsigned long long n = 1ull << log2n, nv = n / 4;
    u32x4 *in, *out;
    unsigned *vals;
    unsigned long long *idx;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&vals, n * 2));
    CK(hipMalloc(&idx, n * 4));
    CK(hipMemset(in, 0x3c, n * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char *name, double bytes, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(a));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        printf("%-14s %8.1f us  %6.3f TB/s (%.2f GB moved)\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12, bytes / 1e9);
    };
    const dim3 blk(256);
    for (int g : {1024, 2048, 4096}) {
        printf("grid %d\n", g);
        run("copy<4>", 8.0 * n, [&] { hipLaunchKernelGGL((copy<4>), dim3(g), blk, 0, 0, in, out, nv); });
        run("copy<8>", 8.0 * n, [&] { hipLaunchKernelGGL((copy<8>), dim3(g), blk, 0, 0, in, out, nv); });
        run("mix_vec<4>", 10.0 * n, [&] {
            hipLaunchKernelGGL((mix_vec<4>), dim3(g), blk, 0, 0, in, reinterpret_cast<u32x2 *>(vals),
                               reinterpret_cast<u32x4 *>(idx), nv);
        });
        run("mix_vec<8>", 10.0 * n, [&] {
            hipLaunchKernelGGL((mix_vec<8>), dim3(g), blk, 0, 0, in, reinterpret_cast<u32x2 *>(vals),
                               reinterpret_cast<u32x4 *>(idx), nv);
        });
        run("mix_lane<4>", 10.0 * n, [&] { hipLaunchKernelGGL((mix_lane<4>), dim3(g), blk, 0, 0, in, vals, idx, nv); });
        run("mix_lane<8>", 10.0 * n, [&] { hipLaunchKernelGGL((mix_lane<8>), dim3(g), blk, 0, 0, in, vals, idx, nv); });
    }
    return 0;
}
