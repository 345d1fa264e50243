// stream_probe.hip -- measures the HBM read ceiling for the streaming pass's
// access pattern on this GPU (not part of the product; a design probe).
//   read_sum<U,NT>   : 16-B loads, U loads in flight per thread, NT = nontemporal
//   read_cmp<U,NT>   : the k_main per-key work without compaction (3 counters)
//   read_ballot<U>   : + the per-key ballot the candidate compaction needs
// Usage: stream_probe [log2n=30] [bump]
//   bump: after a 2 s idle pause, 40 back-to-back read_sum<8,nt> passes, each
//   timed by events (is the select's slowdown a few passes after an idle
//   start the device's, or ours?)
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_sum(const u32x4 *__restrict__ v, unsigned long long nv, unsigned *out) {
    unsigned acc = 0;
    const unsigned long long tile = 256ull * U;
    for (unsigned long long t0 = (unsigned long long)blockIdx.x * tile; t0 < nv; t0 += (unsigned long long)gridDim.x * tile) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<NT>(&v[t0 + u * 256 + threadIdx.x]);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_cmp(const u32x4 *__restrict__ v, unsigned long long nv, unsigned lo,
                                                unsigned hi, unsigned long long *out) {
    unsigned a = 0, b = 0, c = 0;
    const unsigned long long tile = 256ull * U;
    for (unsigned long long t0 = (unsigned long long)blockIdx.x * tile; t0 < nv; t0 += (unsigned long long)gridDim.x * tile) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<NT>(&v[t0 + u * 256 + threadIdx.x]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                unsigned k = x[u][j] ^ 0x80000000u;
                a += k < lo;
                b += k == lo;
                c += k == hi;
            }
        }
    }
    if (a + b + c == 0x12345678u) out[0] = a;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_ballot(const u32x4 *__restrict__ v, unsigned long long nv, unsigned lo,
                                                   unsigned hi, unsigned long long *out) {
    __shared__ unsigned lbuf[4096];
    __shared__ unsigned lcount;
    if (threadIdx.x == 0) lcount = 0;
    __syncthreads();
    unsigned a = 0, b = 0, c = 0;
    const int lane = threadIdx.x & 63;
    const unsigned long long tile = 256ull * U;
    for (unsigned long long t0 = (unsigned long long)blockIdx.x * tile; t0 < nv; t0 += (unsigned long long)gridDim.x * tile) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<NT>(&v[t0 + u * 256 + threadIdx.x]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                unsigned k = x[u][j] ^ 0x80000000u;
                a += k < lo;
                b += k == lo;
                c += k == hi;
                bool in = (k > lo) & (k < hi);
                unsigned long long m = __ballot(in);
                if (m) {
                    unsigned cnt = __popcll(m);
                    unsigned r = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                    int ld0 = __ffsll((long long)m) - 1;
                    unsigned base = 0;
                    if (lane == ld0) base = atomicAdd(&lcount, cnt);
                    base = __shfl(base, ld0, 64);
                    if (in && base + r < 4096) lbuf[base + r] = k;
                }
            }
        }
    }
    __syncthreads();
    if (a + b + c == 0x12345678u || lbuf[lcount & 4095] == 0x12345678u) out[0] = a;
}

__global__ void fill_random(unsigned *p, unsigned long long n) {
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        unsigned long long z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = (unsigned)((z ^ (z >> 31)) >> 32);
    }
}

template <typename K, typename... A>
float timeit(K kern, int grid, int reps, A... args) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, args...);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, args...);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char **argv) {
    int log2n = argc > 1 ? atoi(argv[1]) : 30;
    unsigned long long n = 1ull << log2n, nv = n / 4;
    u32x4 *v;
    unsigned *o;
    unsigned long long *o2;
    CK(hipMalloc(&v, n * 4));
    CK(hipMalloc(&o, 64));
    CK(hipMalloc(&o2, 64));
    CK(hipMemset(v, 0x3c, n * 4));
    // lo/hi chosen so ~0.6% of keys fall inside (keys are 0x3c3c3c3c -> use the byte pattern + a window)
    unsigned lo = 0xbc3c3c3cu - 1, hi = 0xbc3c3c3cu + 1;  // all keys "inside": worst case for ballots
    unsigned lo0 = 0x10u, hi0 = 0x20u;                      // no keys inside
    const double gb = n * 4.0 / 1e9;
    if (argc > 2 && !strcmp(argv[2], "bump")) {
        // random keys (a constant fill toggles no bits: less power than real data)
        hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, reinterpret_cast<unsigned *>(v), n);
        CK(hipDeviceSynchronize());
        const unsigned wlo = 0x7F000000u, whi = 0x7F000000u + (1u << 24);  // ~0.4 % of random keys inside
        for (int kind = 0; kind < 3; ++kind) {
            sleep(2);
            hipEvent_t ev[41];
            for (auto &evt : ev) CK(hipEventCreate(&evt));
            CK(hipEventRecord(ev[0]));
            for (int i = 0; i < 40; ++i) {
                if (kind == 0) hipLaunchKernelGGL((read_sum<8, true>), dim3(1024), dim3(256), 0, 0, v, nv, o);
                else if (kind == 1) hipLaunchKernelGGL((read_cmp<4, true>), dim3(1024), dim3(256), 0, 0, v, nv, wlo, whi, o2);
                else hipLaunchKernelGGL((read_ballot<4, true>), dim3(1024), dim3(256), 0, 0, v, nv, wlo, whi, o2);
                CK(hipEventRecord(ev[i + 1]));
            }
            CK(hipEventSynchronize(ev[40]));
            printf("bump %s ms:", kind == 0 ? "read_sum" : kind == 1 ? "read_cmp" : "read_ballot");
            for (int i = 0; i < 40; ++i) {
                float ms;
                CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
                printf(" %.3f", ms);
            }
            printf("\n");
        }
        return 0;
    }
    int grids[] = {1024, 2048, 4096, 8192};
    for (int g : grids) {
        printf("grid %5d  sum U1 %6.0f  U2 %6.0f  U4 %6.0f  U8 %6.0f | nt U2 %6.0f  U4 %6.0f  U8 %6.0f GB/s\n", g,
               gb / timeit(read_sum<1, false>, g, 10, v, nv, o) * 1e3,
               gb / timeit(read_sum<2, false>, g, 10, v, nv, o) * 1e3,
               gb / timeit(read_sum<4, false>, g, 10, v, nv, o) * 1e3,
               gb / timeit(read_sum<8, false>, g, 10, v, nv, o) * 1e3,
               gb / timeit(read_sum<2, true>, g, 10, v, nv, o) * 1e3,
               gb / timeit(read_sum<4, true>, g, 10, v, nv, o) * 1e3,
               gb / timeit(read_sum<8, true>, g, 10, v, nv, o) * 1e3);
    }
    for (int g : grids) {
        printf("grid %5d  cmp U2 %6.0f U4 %6.0f nt U2 %6.0f U4 %6.0f | ballot(none in) U2 %6.0f U4 %6.0f | ballot(all in) U4 %6.0f GB/s\n",
               g, gb / timeit(read_cmp<2, false>, g, 10, v, nv, lo0, hi0, o2) * 1e3,
               gb / timeit(read_cmp<4, false>, g, 10, v, nv, lo0, hi0, o2) * 1e3,
               gb / timeit(read_cmp<2, true>, g, 10, v, nv, lo0, hi0, o2) * 1e3,
               gb / timeit(read_cmp<4, true>, g, 10, v, nv, lo0, hi0, o2) * 1e3,
               gb / timeit(read_ballot<2, true>, g, 10, v, nv, lo0, hi0, o2) * 1e3,
               gb / timeit(read_ballot<4, true>, g, 10, v, nv, lo0, hi0, o2) * 1e3,
               gb / timeit(read_ballot<4, true>, g, 10, v, nv, lo, hi, o2) * 1e3);
    }
    return 0;
}
