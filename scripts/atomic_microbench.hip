// Diagnostic: throughput of returning device-scope (agent) atomic adds on a few
// hot global addresses, as a per-record output cursor would see them (one lane
// per workgroup adds, workgroups spread over every CU).  Prints ns per atomic.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void hot_atomics(unsigned long long *ctr, int naddr, int iters, unsigned long long *sink) {
    unsigned long long acc = 0;
    if (threadIdx.x == 0) {
        for (int i = 0; i < iters; ++i) {
            const int a = (blockIdx.x + i) % naddr;
            acc += __hip_atomic_fetch_add(&ctr[a * 16], 7ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_s_sleep(1);
        }
        sink[blockIdx.x] = acc;
    }
}

int main(int argc, char **argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 512;
    unsigned long long *ctr, *sink;
    hipMalloc(&ctr, 64 * 16 * 8);
    hipMalloc(&sink, 65536 * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int naddr : {1, 8, 25, 64}) {
        for (int iters : {200, 2000}) {
            hipMemset(ctr, 0, 64 * 16 * 8);
            hot_atomics<<<blocks, 64>>>(ctr, naddr, 10, sink);
            hipEventRecord(a);
            hot_atomics<<<blocks, 64>>>(ctr, naddr, iters, sink);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double n = (double)blocks * iters;
            printf("{\"blocks\": %d, \"addresses\": %d, \"iters\": %d, \"ms\": %.4f, \"ns_per_atomic\": %.3f, "
                   "\"atomics_per_us\": %.1f}\n", blocks, naddr, iters, ms, ms * 1e6 / n, n / (ms * 1e3));
        }
    }
    return 0;
}
