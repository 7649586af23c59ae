// reread_microbench.hip — DIAGNOSTIC: can a workgroup read a chunk of its range
// twice (a count pass, then a scatter pass over the same bytes) for the price of
// one HBM read, the second read served by L2 / the 256 MB MALL?  Each of G = 256
// persistent 1024-thread workgroups streams its contiguous 1/G of a 10 GB buffer
// in chunks of C bytes; mode 1 reads every chunk once, mode 2 reads each chunk,
// then reads it again (dependent on a workgroup barrier, as a scatter pass after a
// count pass would).  16-byte loads, 4 in flight per lane.  Prints ms per pass.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/lib/reread scripts/reread_microbench.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int NT>
__device__ __forceinline__ uint32_t read_span(const char *p, int64_t n) {
    uint32_t acc = 0;
    const int64_t step = 1024 * 16;
    for (int64_t o = threadIdx.x * 16; o < n; o += 4 * step) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t q = o + u * step;
            if (q < n) {
                if (NT) v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p + q));
                else v[u] = *reinterpret_cast<const u32x4 *>(p + q);
            } else {
                v[u] = u32x4{0, 0, 0, 0};
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
    return acc;
}

template <int MODE, int NT1, int NT2>
__global__ __launch_bounds__(1024) void reread_kernel(const char *buf, int64_t per_wg, int64_t chunk, uint32_t *sink) {
    const char *base = buf + (int64_t)blockIdx.x * per_wg;
    uint32_t acc = 0;
    for (int64_t c = 0; c < per_wg; c += chunk) {
        const int64_t n = per_wg - c < chunk ? per_wg - c : chunk;
        acc += read_span<NT1>(base + c, n);
        if (MODE == 2) {
            __syncthreads();
            acc += read_span<NT2>(base + c, n);
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int MODE, int NT1, int NT2>
float run(const char *buf, int64_t per_wg, int64_t chunk, uint32_t *sink, int G) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((reread_kernel<MODE, NT1, NT2>), dim3(G), dim3(1024), 0, 0, buf, per_wg, chunk, sink);
    std::vector<float> ts;
    for (int i = 0; i < 7; ++i) {
        hipEventRecord(a, 0);
        hipLaunchKernelGGL((reread_kernel<MODE, NT1, NT2>), dim3(G), dim3(1024), 0, 0, buf, per_wg, chunk, sink);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[3];
}

int main() {
    const int G = 256;
    const int64_t total = 10000000000ll;
    const int64_t per_wg = (total / G) & ~(int64_t)4095;
    char *buf = nullptr;
    uint32_t *sink = nullptr;
    if (hipMalloc(&buf, per_wg * G) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, per_wg * G);
    hipDeviceSynchronize();
    const double gb = (double)per_wg * G / 1e9;
    const float once = run<1, 0, 0>(buf, per_wg, per_wg, sink, G);
    const float once_nt = run<1, 1, 0>(buf, per_wg, per_wg, sink, G);
    printf("{\"mode\": \"once\", \"ms\": %.4f, \"GBps\": %.1f}\n", once, gb / once * 1e3);
    printf("{\"mode\": \"once_nt\", \"ms\": %.4f, \"GBps\": %.1f}\n", once_nt, gb / once_nt * 1e3);
    for (int64_t chunk : {64ll << 10, 128ll << 10, 256ll << 10, 512ll << 10, 1ll << 20, 2ll << 20, 4ll << 20}) {
        const float t = run<2, 0, 0>(buf, per_wg, chunk, sink, G);
        const float t2 = run<2, 0, 1>(buf, per_wg, chunk, sink, G);
        printf("{\"mode\": \"twice\", \"chunk_kib\": %lld, \"ms\": %.4f, \"ms_second_nt\": %.4f, \"vs_once\": %.3f}\n",
               (long long)(chunk >> 10), t, t2, t / once);
        fflush(stdout);
    }
    hipFree(buf);
    hipFree(sink);
    return 0;
}
