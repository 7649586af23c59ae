// Diagnostic: rate of non-returning 32-bit global atomic adds on random words of a
// 65 536-word (k = 8) table, issued by every lane of 1 024-thread workgroups over all
// CUs — the question being whether the vector memory path could take a share of the
// k = 8 kernel's window adds off its LDS array (round 6).  Modes:
//   0  agent scope, one table for the whole grid
//   1  agent scope, one table per XCD (workgroup id mod 8, the dispatcher's round robin)
//   2  workgroup scope, one table per XCD
//   3  LDS adds (ds_add_u32) on a 65 536-word-equivalent 16-bit-packed table, for scale
//   4  as 3, but every 16th add goes to the XCD's global table (agent scope) instead
//   5  as 3, but every 32nd add goes to the XCD's global table (agent scope) instead
// Prints adds per second for each mode.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

template <int MODE>
__global__ __launch_bounds__(1024) void gadd(uint32_t *tab, int iters, uint32_t seed, uint32_t *sink) {
    __shared__ uint32_t lds[32768];
    uint32_t x = seed ^ ((blockIdx.x * 1024u + threadIdx.x) * 0x9E3779B9u);
    uint32_t *t = tab + (MODE == 0 ? 0u : (blockIdx.x & 7u) * 65536u);
    if (MODE >= 3) {
        for (int i = threadIdx.x; i < 32768; i += 1024) lds[i] = 0;
        __syncthreads();
    }
#pragma unroll 32
    for (int i = 0; i < iters; ++i) {
        x = x * 1664525u + 1013904223u;
        const uint32_t b = x >> 16;
        if (MODE == 0 || MODE == 1)
            __hip_atomic_fetch_add(t + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (MODE == 2)
            __hip_atomic_fetch_add(t + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else if ((MODE == 4 && (i & 15) == 15) || (MODE == 5 && (i & 31) == 31))
            __hip_atomic_fetch_add(t + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            __hip_atomic_fetch_add(lds + (b & 32767u), (b & 32768u) ? 65536u : 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (MODE >= 3) {
        __syncthreads();
        uint32_t s = 0;
        for (int i = threadIdx.x; i < 32768; i += 1024) s += lds[i];
        if (s == 0x12345678u) sink[blockIdx.x] = s;
    }
}

template <int MODE>
static void run(uint32_t *tab, uint32_t *sink, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    gadd<MODE><<<blocks, 1024>>>(tab, 8, 1u, sink);
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(a);
        gadd<MODE><<<blocks, 1024>>>(tab, iters, 7u + r, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    const double n = (double)blocks * 1024.0 * iters;
    printf("{\"mode\": %d, \"blocks\": %d, \"iters\": %d, \"ms\": %.4f, \"adds_per_s\": %.4g}\n", MODE, blocks, iters,
           best, n / (best * 1e-3));
    hipEventDestroy(a);
    hipEventDestroy(b);
}

int main(int argc, char **argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 256;
    const int iters = argc > 2 ? atoi(argv[2]) : 512;
    uint32_t *tab, *sink;
    if (hipMalloc(&tab, 8u * 65536u * 4u) != hipSuccess || hipMalloc(&sink, 65536u * 4u) != hipSuccess) return 1;
    hipMemset(tab, 0, 8u * 65536u * 4u);
    run<0>(tab, sink, blocks, iters);
    run<1>(tab, sink, blocks, iters);
    run<2>(tab, sink, blocks, iters);
    run<3>(tab, sink, blocks, iters);
    run<4>(tab, sink, blocks, iters);
    run<5>(tab, sink, blocks, iters);
    run<3>(tab, sink, blocks, iters);
    hipDeviceSynchronize();
    return 0;
}
