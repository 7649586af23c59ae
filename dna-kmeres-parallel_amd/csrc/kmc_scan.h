// kmc_scan.h — exclusive prefix sum of a uint32 array into uint64 offsets, on
// the device, in three launches (per-tile totals, one-block scan of the totals,
// per-tile apply).  Shared by the radix partition (bucket offsets) and the
// canonical table compaction (output positions).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kmc {
namespace {

constexpr int kScanBlock = 1024, kScanPer = 4, kScanTile = kScanBlock * kScanPer;

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *sh, uint64_t &total) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (wid == 0) {
        uint64_t t = lane < kScanBlock / 64 ? sh[lane] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(t, o);
            if (lane >= o) t += y;
        }
        if (lane < kScanBlock / 64) sh[lane] = t;
    }
    __syncthreads();
    total = sh[kScanBlock / 64 - 1];
    const uint64_t before = wid ? sh[wid - 1] : 0;
    __syncthreads();
    return before + x - v;
}

// gate (optional): the launch does nothing unless *gate != 0 (a conditional rerun)
__device__ __forceinline__ bool scan_gated_off(const uint32_t *gate) {
    return gate != nullptr && __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
}

__global__ __launch_bounds__(kScanBlock) void scan_reduce_kernel(const uint32_t *in, int64_t m, uint64_t *bsum,
                                                                 const uint32_t *gate) {
    __shared__ uint64_t sh[kScanBlock / 64];
    if (scan_gated_off(gate)) return;
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    uint64_t v = 0;
    for (int q = 0; q < kScanPer; ++q) {
        const int64_t i = base + (int64_t)q * kScanBlock + threadIdx.x;
        if (i < m) v += in[i];
    }
    uint64_t total;
    block_excl_scan(v, sh, total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanBlock) void scan_blocks_kernel(uint64_t *bsum, int64_t nb, const uint32_t *gate) {
    __shared__ uint64_t sh[kScanBlock / 64];
    if (scan_gated_off(gate)) return;
    uint64_t carry = 0;
    for (int64_t base = 0; base < nb; base += kScanBlock) {
        const int64_t i = base + threadIdx.x;
        const uint64_t v = i < nb ? bsum[i] : 0;
        uint64_t total;
        const uint64_t ex = block_excl_scan(v, sh, total);
        if (i < nb) bsum[i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(const uint32_t *in, int64_t m, const uint64_t *bsum,
                                                                uint64_t *out, const uint32_t *gate) {
    __shared__ uint64_t sh[kScanBlock / 64];
    if (scan_gated_off(gate)) return;
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPer;
    uint64_t v[kScanPer], tsum = 0;
    for (int q = 0; q < kScanPer; ++q) {
        v[q] = (base + q < m) ? in[base + q] : 0;
        tsum += v[q];
    }
    uint64_t total;
    uint64_t run = bsum[blockIdx.x] + block_excl_scan(tsum, sh, total);
    for (int q = 0; q < kScanPer; ++q) {
        if (base + q < m) out[base + q] = run;
        run += v[q];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kScanBlock - 1) out[m] = run;  // grand total
}

// out[0..m] = exclusive scan of in[0..m) (out[m] = total); bsum: scan_tiles(m) uint64;
// gate: see scan_gated_off
inline int64_t scan_tiles(int64_t m) { return (m + kScanTile - 1) / kScanTile; }

inline void excl_scan_u32(const uint32_t *in, int64_t m, uint64_t *bsum, uint64_t *out, hipStream_t st,
                          const uint32_t *gate = nullptr) {
    const int64_t nt = scan_tiles(m) > 0 ? scan_tiles(m) : 1;
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nt), dim3(kScanBlock), 0, st, in, m, bsum, gate);
    hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(kScanBlock), 0, st, bsum, nt, gate);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nt), dim3(kScanBlock), 0, st, in, m, bsum, out, gate);
}

}  // namespace
}  // namespace kmc
