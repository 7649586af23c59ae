// lds_microbench.hip — DIAGNOSTIC ONLY (never part of libkmc.so).
//
// Measures LDS atomic/store throughput per CU on gfx950 for the access shapes the
// dense histogram kernels use, with no global-memory traffic in the loop:
//   mode 0  ds_add_u32, random word of a 128 KiB table (k = 8 packed-16 layout)
//   mode 1  ds_add_u32, conflict-free (lane i of a 32-lane group -> bank i)
//   mode 2  ds_add_u64, random qword of a 128 KiB table (pair layout)
//   mode 3  ds_add_u64, conflict-free (32 lanes -> 64 distinct banks)
//   mode 4  ds_write_b32, random word (no read-modify-write)
//   mode 5  ds_add_u32, random word of a 64 KiB table, 32 replicas interleaved by lane (k <= 4 layout; conflict-free)
//   mode 6  ds_add_u32, random but bank forced to (lane % 32) via addr = (r & ~31) | lane%32 (conflict-free, random rows)
//   mode 7  ds_add_rtn_u32, random word (returning form)
//   mode 8  ds_add_u32, random word of a 64 KiB table (16 384 words: k = 7, R = 1)
//   mode 9  ds_add_u32, two lanes of each 32-lane group on a shared bank (2-way conflict, fixed)
//   mode 10 ds_add_u32, random word of 16 384, 2 replicas interleaved by lane parity (32 768 words)
//   mode 11 ds_add_u32, random word of 8 192, 4 replicas interleaved by lane % 4
//   mode 12 ds_add_u32, random word of 32 768, replica-free, but only lanes 0-31 active
//   mode 13 ds_add_u64, random qword of 8 192, 2 replicas interleaved by lane parity
//   mode 14 ds_cmpst_rtn_b64, random qword of 16 384 (the compare never matches: no store)
//   mode 15 ds_cmpst_rtn_b64, conflict-free (lane -> its own qword)
//   mode 16 ds_cmpst_rtn_b64, random, only lanes 0-15 active
//   mode 17 ds_cmpst_rtn_b32, random word of 32 768
//   mode 18 ds_read_b64, random qword of 16 384
//   mode 19 ds_cmpst_rtn_b64, random, one wait per op (dependent chain: latency)
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_microbench scripts/lds_microbench.hip
// Run:   ./lds_microbench      (one JSON line per mode)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

constexpr int BLOCK = 1024;
constexpr int OPS = 16;  // atomics per lane per iteration (like one tile)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(BLOCK) void lds_kernel(int iters, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint32_t h[32768];
    for (int i = threadIdx.x; i < 32768; i += BLOCK) h[i] = 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    uint32_t a[OPS];
#pragma unroll
    for (int j = 0; j < OPS; ++j) a[j] = mix(blockIdx.x * 0x9E3779B9u + threadIdx.x * 977u + j * 0x85EBCA6Bu);
    uint32_t acc = 0u;
    uint64_t *h64 = reinterpret_cast<uint64_t *>(h);
    for (int it = 0; it < iters; ++it) {
        const uint32_t salt = mix(it * 0x27d4eb2fu + blockIdx.x);  // uniform per iteration
#pragma unroll
        for (int j = 0; j < OPS; ++j) {
            const uint32_t r = a[j] ^ salt;
            if constexpr (MODE == 0) {
                __hip_atomic_fetch_add(&h[r & 0x7FFFu], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 1) {
                __hip_atomic_fetch_add(&h[((r & 0x3FFu) << 5) | (lane & 31)], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 2) {
                __hip_atomic_fetch_add(&h64[r & 0x3FFFu], 0x0000000100000001ull, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 3) {
                __hip_atomic_fetch_add(&h64[((r & 0x1FFu) << 5) | (lane & 31)], 0x0000000100000001ull,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 4) {
                __hip_atomic_store(&h[r & 0x7FFFu], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 5) {
                __hip_atomic_fetch_add(&h[((r & 0x1FFu) << 5) | (lane & 31)], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 6) {
                __hip_atomic_fetch_add(&h[(r & 0x7FE0u) | (lane & 31)], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 7) {
                acc += __hip_atomic_fetch_add(&h[r & 0x7FFFu], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 8) {
                __hip_atomic_fetch_add(&h[r & 0x3FFFu], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 10) {
                __hip_atomic_fetch_add(&h[((r & 0x3FFFu) << 1) | (lane & 1)], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 11) {
                __hip_atomic_fetch_add(&h[((r & 0x1FFFu) << 2) | (lane & 3)], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 12) {
                if (lane < 32)
                    __hip_atomic_fetch_add(&h[r & 0x7FFFu], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 13) {
                __hip_atomic_fetch_add(&h64[((r & 0x1FFFu) << 1) | (lane & 1)], 0x0000000100000001ull,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 14) {
                uint64_t c = 1ull;  // the table holds even values only
                __hip_atomic_compare_exchange_strong(&h64[r & 0x3FFFu], &c, 3ull, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
                acc += (uint32_t)c;
            } else if constexpr (MODE == 15) {
                uint64_t c = 1ull;
                __hip_atomic_compare_exchange_strong(&h64[((r & 0xFFu) << 6) | lane], &c, 3ull, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                acc += (uint32_t)c;
            } else if constexpr (MODE == 16) {
                if (lane < 16) {
                    uint64_t c = 1ull;
                    __hip_atomic_compare_exchange_strong(&h64[r & 0x3FFFu], &c, 3ull, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    acc += (uint32_t)c;
                }
            } else if constexpr (MODE == 17) {
                uint32_t c = 1u;
                __hip_atomic_compare_exchange_strong(&h[r & 0x7FFFu], &c, 3u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
                acc += c;
            } else if constexpr (MODE == 18) {
                acc += (uint32_t)__hip_atomic_load(&h64[r & 0x3FFFu], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if constexpr (MODE == 19) {
                uint64_t c = 1ull;
                __hip_atomic_compare_exchange_strong(&h64[(r ^ acc) & 0x3FFFu], &c, 3ull, __ATOMIC_RELAXED,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                acc += (uint32_t)c;
            } else if constexpr (MODE == 9) {
                __hip_atomic_fetch_add(&h[((r & 0x3FFu) << 5) | ((lane & 31) >> 1)], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    __syncthreads();
    uint32_t s = acc;
    for (int i = threadIdx.x; i < 32768; i += BLOCK) s += h[i];
    if (s == 0x12345678u) out[blockIdx.x] = s;  // keep the table live
}

template <int MODE>
int run(int cus, int iters, uint32_t *out, const char *name) {
    hipEvent_t b, e;
    CHECK(hipEventCreate(&b));
    CHECK(hipEventCreate(&e));
    hipLaunchKernelGGL(lds_kernel<MODE>, dim3(cus), dim3(BLOCK), 0, 0, iters, out);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHECK(hipEventRecord(b, 0));
        hipLaunchKernelGGL(lds_kernel<MODE>, dim3(cus), dim3(BLOCK), 0, 0, iters, out);
        CHECK(hipEventRecord(e, 0));
        CHECK(hipEventSynchronize(e));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, b, e));
        if (ms < best) best = ms;
    }
    const double insts_per_cu = (double)iters * OPS * (BLOCK / 64);
    const double ns = best * 1e6;
    printf("{\"mode\": %d, \"name\": \"%s\", \"ms\": %.4f, \"wave_insts_per_cu\": %.0f, \"ns_per_wave_inst\": %.4f, "
           "\"cyc_per_wave_inst_at_2.4GHz\": %.3f}\n",
           MODE, name, best, insts_per_cu, ns / insts_per_cu, ns / insts_per_cu * 2.4);
    fflush(stdout);
    CHECK(hipEventDestroy(b));
    CHECK(hipEventDestroy(e));
    return 0;
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *out = nullptr;
    CHECK(hipMalloc(&out, cus * sizeof(uint32_t)));
    const int iters = 2000;
    int r = 0;
    r |= run<0>(cus, iters, out, "add_u32 random 32K words");
    r |= run<1>(cus, iters, out, "add_u32 conflict-free");
    r |= run<2>(cus, iters, out, "add_u64 random 16K qwords");
    r |= run<3>(cus, iters, out, "add_u64 conflict-free");
    r |= run<4>(cus, iters, out, "write_b32 random");
    r |= run<5>(cus, iters, out, "add_u32 R=32 interleaved");
    r |= run<6>(cus, iters, out, "add_u32 random rows, bank=lane");
    r |= run<7>(cus, iters, out, "add_rtn_u32 random");
    r |= run<8>(cus, iters, out, "add_u32 random 16K words");
    r |= run<9>(cus, iters, out, "add_u32 2-way conflict");
    r |= run<10>(cus, iters, out, "add_u32 random, 2 replicas by lane parity");
    r |= run<11>(cus, iters, out, "add_u32 random, 4 replicas by lane%4");
    r |= run<12>(cus, iters, out, "add_u32 random, lanes 0-31 only");
    r |= run<13>(cus, iters, out, "add_u64 random, 2 replicas by lane parity");
    r |= run<14>(cus, iters, out, "cmpst_rtn_b64 random (no store)");
    r |= run<15>(cus, iters, out, "cmpst_rtn_b64 conflict-free");
    r |= run<16>(cus, iters, out, "cmpst_rtn_b64 random, 16 lanes");
    r |= run<17>(cus, iters, out, "cmpst_rtn_b32 random");
    r |= run<18>(cus, iters, out, "read_b64 random");
    r |= run<19>(cus, iters, out, "cmpst_rtn_b64 random, dependent chain");
    CHECK(hipFree(out));
    return r;
}
