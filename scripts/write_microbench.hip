// Diagnostic: HBM write rate of the R3 ring scatter's write pattern (64-byte list
// segments, 1024 open lists per workgroup, one workgroup per CU) against plain
// coalesced streaming writes, with and without the concurrent input read R3 does
// (10 GB read per 20 GB written).  Prints one JSON line per pattern.
//   hipcc --offload-arch=gfx950 -O3 scripts/write_microbench.hip -o scripts/bin/write_microbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kBlock = 1024;

// one 64 << SEGLOG2 / 64-byte segment per thread per iteration, thread t of
// workgroup w appending to its own list region (t * G + w) like R3's lists
template <int SEGQ, bool READ>
__global__ __launch_bounds__(kBlock) void seg_writes(uint4 *out, const uint4 *in, long long per_stream_q,
                                                     long long iters, long long in_q_per_wg, uint4 *sink) {
    const int t = threadIdx.x, w = blockIdx.x;
    // list regions of ragged length in R3: a per-stream jitter of 0..255 64-byte
    // units keeps the streams off a common channel phase
    const uint32_t sid = (uint32_t)t * gridDim.x + w;
    const uint32_t jit = ((sid * 2654435761u) >> 24) * 4u;
    uint4 *dst = out + (long long)sid * (per_stream_q + 1024) + jit;
    const uint4 *src = in + (long long)w * in_q_per_wg;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (long long i = 0; i < iters; ++i) {
        if (READ) {  // SEGQ / 2 coalesced 16-byte loads per thread: half the bytes written
#pragma unroll
            for (int q = 0; q < SEGQ / 2; ++q) {
                const uint4 v = src[(i * (SEGQ / 2) + q) * kBlock + t];
                acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
            }
        }
#pragma unroll
        for (int q = 0; q < SEGQ; ++q) dst[i * SEGQ + q] = make_uint4((uint32_t)i, t, w, q);
    }
    if (acc.x == 0x12345678u) sink[w] = acc;
}

// as seg_writes<4>, but the four lanes of a group write the four quads of one
// segment (16 contiguous 64-byte pieces per store instruction instead of 64
// scattered 16-byte ones): group g serves streams 4g..4g+3 in turn
template <bool READ>
__global__ __launch_bounds__(kBlock) void seg_writes_coal(uint4 *out, const uint4 *in, long long per_stream_q,
                                                          long long iters, long long in_q_per_wg, uint4 *sink) {
    const int t = threadIdx.x, w = blockIdx.x, q = t & 3, g = t >> 2;
    uint4 *dst[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t sid = (uint32_t)(4 * g + k) * gridDim.x + w;
        const uint32_t jit = ((sid * 2654435761u) >> 24) * 4u;
        dst[k] = out + (long long)sid * (per_stream_q + 1024) + jit;
    }
    const uint4 *src = in + (long long)w * in_q_per_wg;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (long long i = 0; i < iters; ++i) {
        if (READ) {
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint4 v = src[(i * 2 + r) * kBlock + t];
                acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k][i * 4 + q] = make_uint4((uint32_t)i, t, w, k);
    }
    if (acc.x == 0x12345678u) sink[w] = acc;
}

// coalesced: iteration i of workgroup w writes kBlock consecutive uint4 (SEGQ times)
template <int SEGQ, bool READ>
__global__ __launch_bounds__(kBlock) void seq_writes(uint4 *out, const uint4 *in, long long q_per_wg, long long iters,
                                                     long long in_q_per_wg, uint4 *sink) {
    const int t = threadIdx.x, w = blockIdx.x;
    uint4 *dst = out + (long long)w * q_per_wg;
    const uint4 *src = in + (long long)w * in_q_per_wg;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (long long i = 0; i < iters; ++i) {
        if (READ) {
#pragma unroll
            for (int q = 0; q < SEGQ / 2; ++q) {
                const uint4 v = src[(i * (SEGQ / 2) + q) * kBlock + t];
                acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
            }
        }
#pragma unroll
        for (int q = 0; q < SEGQ; ++q) dst[(i * SEGQ + q) * kBlock + t] = make_uint4((uint32_t)i, t, w, q);
    }
    if (acc.x == 0x12345678u) sink[w] = acc;
}

template <class F>
static void timeit(const char *name, F launch, double wbytes, double rbytes) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    printf("{\"pattern\": \"%s\", \"ms\": %.3f, \"write_GB\": %.2f, \"read_GB\": %.2f, \"GBps\": %.0f}\n", name, best,
           wbytes / 1e9, rbytes / 1e9, (wbytes + rbytes) / best / 1e6);
    fflush(stdout);
}

int main(int argc, char **argv) {
    int G = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) == hipSuccess) G = prop.multiProcessorCount;
    const double wtarget = argc > 1 ? atof(argv[1]) * 1e9 : 20e9;  // bytes written
    // per-stream quads for 20 GB over G * 1024 streams, a multiple of 16 (256 B)
    const long long per_stream_q = ((long long)(wtarget / 16 / (G * (double)kBlock)) / 16) * 16;
    const long long wq = per_stream_q * G * kBlock;
    const double wbytes = (double)wq * 16;
    const long long in_q_per_wg = per_stream_q * kBlock / 2;
    const double rbytes = (double)in_q_per_wg * G * 16;
    uint4 *out, *in, *sink;
    if (hipMalloc(&out, (wq + 1024LL * G * kBlock) * 16) != hipSuccess || hipMalloc(&in, in_q_per_wg * G * 16 + 4096) != hipSuccess ||
        hipMalloc(&sink, G * 16) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    hipMemset(in, 1, in_q_per_wg * G * 16);
    printf("{\"cus\": %d, \"streams\": %d, \"per_stream_bytes\": %lld}\n", G, G * kBlock, per_stream_q * 16);
    timeit("seq_write+read", [&] { seq_writes<4, true><<<G, kBlock>>>(out, in, per_stream_q * kBlock, per_stream_q / 4, in_q_per_wg, sink); }, wbytes, rbytes);
    timeit("seg64_lane_write+read", [&] { seg_writes<4, true><<<G, kBlock>>>(out, in, per_stream_q, per_stream_q / 4, in_q_per_wg, sink); }, wbytes, rbytes);
    timeit("seg64_quad_write+read", [&] { seg_writes_coal<true><<<G, kBlock>>>(out, in, per_stream_q, per_stream_q / 4, in_q_per_wg, sink); }, wbytes, rbytes);
    timeit("seg128_lane_write+read", [&] { seg_writes<8, true><<<G, kBlock>>>(out, in, per_stream_q, per_stream_q / 8, in_q_per_wg, sink); }, wbytes, rbytes);
    hipFree(out);
    hipFree(in);
    hipFree(sink);
    return 0;
}
