// Diagnostic (round 4): HBM rate of K3b's write pattern -- each workgroup (one per
// CU) appends to 256 open list regions in whole segments while it streams an equal
// number of bytes in -- for 64-byte segments (K3b today: a lane quad stores one,
// 16 bytes per lane) against 128-byte segments (a whole L2 line: the quad stores
// it with two instructions, or a lane octet with one), and plain streaming writes.
//   hipcc --offload-arch=gfx950 -O3 scripts/seg_microbench.hip -o scripts/bin/seg_microbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kBlock = 1024;
constexpr int kStreams = 256;  // open regions per workgroup (K3b: lists per coarse bucket)

// GL lanes per segment of SEGQ 16-byte pieces; group g of the workgroup owns
// streams g, g + ngroups, ... (kStreams / ngroups of them, in turn)
template <int SEGQ, int GL>
__global__ __launch_bounds__(kBlock) void segw(uint4 *out, const uint4 *in, long long per_stream_q, long long iters,
                                               long long in_q_per_wg, uint4 *sink) {
    constexpr int NG = kBlock / GL, PER = kStreams / NG;  // streams per group
    const int t = threadIdx.x, w = blockIdx.x, q = t % GL, g = t / GL;
    const uint4 *src = in + (long long)w * in_q_per_wg;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (long long i = 0; i < iters; ++i) {
        // read as many bytes as the round writes (K3b: 8 bytes in per 8 out)
        constexpr int RQ = SEGQ * PER * NG / kBlock;  // uint4 per thread per iteration
#pragma unroll
        for (int r = 0; r < RQ; ++r) {
            const uint4 v = src[(i * RQ + r) * kBlock + t];
            acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const uint32_t sid = (uint32_t)(g + k * NG) * gridDim.x + w;
            const uint32_t jit = ((sid * 2654435761u) >> 24) * 8u;  // 128-byte aligned, ragged
            uint4 *dst = out + (long long)sid * (per_stream_q + 2048) + jit;
#pragma unroll
            for (int c = 0; c < SEGQ / GL; ++c) dst[i * SEGQ + c * GL + q] = make_uint4((uint32_t)i, t, w, c);
        }
    }
    if (acc.x == 0x12345678u) sink[w] = acc;
}

__global__ __launch_bounds__(kBlock) void seqw(uint4 *out, const uint4 *in, long long q_per_wg, long long iters,
                                               long long in_q_per_wg, uint4 *sink) {
    const int t = threadIdx.x, w = blockIdx.x;
    uint4 *dst = out + (long long)w * q_per_wg;
    const uint4 *src = in + (long long)w * in_q_per_wg;
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (long long i = 0; i < iters; ++i) {
        const uint4 v = src[i * kBlock + t];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
        dst[i * kBlock + t] = make_uint4((uint32_t)i, t, w, 0);
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
    const double wtarget = argc > 1 ? atof(argv[1]) * 1e9 : 16e9;
    // per-stream quads, a multiple of 8 (128 B), over G * kStreams streams
    const long long per_stream_q = ((long long)(wtarget / 16 / (G * (double)kStreams)) / 64) * 64;
    const long long wq = per_stream_q * G * kStreams;
    const double wbytes = (double)wq * 16;
    const long long in_q_per_wg = per_stream_q * kStreams;  // read = written
    const double rbytes = (double)in_q_per_wg * G * 16;
    uint4 *out, *in, *sink;
    if (hipMalloc(&out, (per_stream_q + 2048) * 16 * (long long)G * kStreams + 4096) != hipSuccess ||
        hipMalloc(&in, in_q_per_wg * G * 16 + 4096) != hipSuccess || hipMalloc(&sink, G * 16) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    hipMemset(in, 1, in_q_per_wg * G * 16);
    printf("{\"cus\": %d, \"streams\": %d, \"per_stream_bytes\": %lld}\n", G, G * kStreams, per_stream_q * 16);
    for (int rep = 0; rep < 2; ++rep) {
        timeit("seq_write+read", [&] { seqw<<<G, kBlock>>>(out, in, in_q_per_wg, in_q_per_wg / kBlock, in_q_per_wg, sink); }, wbytes, rbytes);
        timeit("seg64_quad", [&] { segw<4, 4><<<G, kBlock>>>(out, in, per_stream_q, per_stream_q / 4, in_q_per_wg, sink); }, wbytes, rbytes);
        timeit("seg128_quad_x2", [&] { segw<8, 4><<<G, kBlock>>>(out, in, per_stream_q, per_stream_q / 8, in_q_per_wg, sink); }, wbytes, rbytes);
        timeit("seg128_octet", [&] { segw<8, 8><<<G, kBlock>>>(out, in, per_stream_q, per_stream_q / 8, in_q_per_wg, sink); }, wbytes, rbytes);
        timeit("seg256_quad_x4", [&] { segw<16, 4><<<G, kBlock>>>(out, in, per_stream_q, per_stream_q / 16, in_q_per_wg, sink); }, wbytes, rbytes);
    }
    hipFree(out);
    hipFree(in);
    hipFree(sink);
    return 0;
}
