// latency_probe.hip -- design probe (not product code): what a short dependent
// kernel costs on MI355X, to price the small kernels around the streaming pass.
// Each case launches REPS back-to-back kernels on one stream and reports the
// event-timed time per kernel (launch + boundary + body).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 1023 && blockIdx.x == 1u << 30) p[0] = 1;
}

// every WG reads a 32 KiB histogram (16 u64 per thread), block-reduces, writes
__global__ __launch_bounds__(256) void k_histread(const u64 *h, u64 *out) {
    __shared__ u64 s[256];
    u64 a = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) a += h[threadIdx.x * 16 + j];
    s[threadIdx.x] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 t = 0;
        for (int i = 0; i < 256; ++i) t += s[i];
        out[blockIdx.x] = t;
    }
}

// one dependent chain: load state -> load data -> atomic
__global__ __launch_bounds__(256) void k_chain(const u64 *st, const uint4 *data, u64 *acc) {
    const u64 off = st[0] & 1023;
    const uint4 x = data[(blockIdx.x * 256 + threadIdx.x + off) & ((1 << 20) - 1)];
    if (x.x == 12345u) atomicAdd(&acc[threadIdx.x], 1ull);
}

// 1 WG zeroing 98 KiB
__global__ __launch_bounds__(256) void k_zero(u64 *p, u64 n) {
    for (u64 i = threadIdx.x; i < n; i += 256) p[i] = 0;
}

// 2048-bin LDS histogram flushed with u64 global atomics (all bins nonzero)
__global__ __launch_bounds__(256) void k_flush(u64 *acc) {
    __shared__ unsigned h[2048];
    for (int i = threadIdx.x; i < 2048; i += 256) h[i] = i + 1;
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += 256) atomicAdd(&acc[i], (u64)h[i]);
}

int main(int argc, char **argv) {
    const int REPS = argc > 1 ? atoi(argv[1]) : 200;
    hipStream_t s;
    hipStreamCreate(&s);
    u64 *h, *out, *acc;
    uint4 *data;
    hipMalloc(&h, 1 << 20);
    hipMalloc(&out, 1 << 20);
    hipMalloc(&acc, 1 << 20);
    hipMalloc(&data, (1 << 20) * 16);
    hipMemset(h, 0, 1 << 20);
    hipMemset(acc, 0, 1 << 20);
    hipMemset(data, 0, (1 << 20) * 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char *name, auto launch) {
        for (int i = 0; i < 20; ++i) launch();
        hipStreamSynchronize(s);
        hipEventRecord(a, s);
        for (int i = 0; i < REPS; ++i) launch();
        hipEventRecord(b, s);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        printf("%-36s %8.2f us/kernel\n", name, ms * 1e3 / REPS);
    };
    run("empty 1x64", [&] { k_empty<<<1, 64, 0, s>>>(nullptr); });
    run("empty 128x256", [&] { k_empty<<<128, 256, 0, s>>>(nullptr); });
    run("empty 1024x1024", [&] { k_empty<<<1024, 1024, 0, s>>>(nullptr); });
    run("histread 128x256", [&] { k_histread<<<128, 256, 0, s>>>(h, out); });
    run("histread 1024x256", [&] { k_histread<<<1024, 256, 0, s>>>(h, out); });
    run("chain 128x256", [&] { k_chain<<<128, 256, 0, s>>>(h, data, acc); });
    run("chain 1024x256", [&] { k_chain<<<1024, 256, 0, s>>>(h, data, acc); });
    run("zero98K 1x256", [&] { k_zero<<<1, 256, 0, s>>>(out, 12314); });
    run("flush2048 64x256", [&] { k_flush<<<64, 256, 0, s>>>(acc); });
    run("flush2048 768x256", [&] { k_flush<<<768, 256, 0, s>>>(acc); });
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
