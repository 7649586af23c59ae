// spin_kernel.hip — DIAGNOSTIC (scripts/interfere.py): a stand-in for the RCCL
// all-reduce kernel that bench.py overlaps with the next step's counting.  `nwg`
// workgroups of 256 threads, each holding `lds` bytes of LDS (so that it cannot
// share a CU with a 128 KB count workgroup), busy-wait for `ticks` of the 100 MHz
// wall clock and exit.  Never loaded by the library or the tests.
#include <hip/hip_runtime.h>

#include <cstdint>

__global__ __launch_bounds__(256) void spin_kernel(uint64_t ticks, uint32_t *sink) {
    extern __shared__ uint32_t lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const uint64_t t0 = wall_clock64();
    uint32_t acc = 0;
    while (wall_clock64() - t0 < ticks) acc += lds[(threadIdx.x + acc) & 255];
    if (acc == 0xFFFFFFFFu) sink[0] = acc;  // keeps the loop; never true in practice
}

extern "C" int spin_launch(int nwg, uint64_t ticks, int lds_bytes, uint32_t *sink, hipStream_t st) {
    hipLaunchKernelGGL(spin_kernel, dim3(nwg), dim3(256), lds_bytes, st, ticks, sink);
    return (int)hipGetLastError();
}
