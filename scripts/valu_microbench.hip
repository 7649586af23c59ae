// Diagnostic: issue cost of the integer VALU instructions the canonical walks (K1 /
// K3a) spend their time on -- 32-bit multiplies, the 64-bit multiply-add, 64-bit
// shifts, byte permutes, bit-field extracts, compares -- against v_add_u32.  Eight
// independent chains per lane, 8 waves per SIMD on every CU; prints cycles per
// wave-instruction per SIMD at the clock given (default 2.4 GHz; the ratio to the
// v_add_u32 row is what matters).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHAINS8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(256) void valu_loop(unsigned *out, int iters, unsigned seed) {
    unsigned a[8];
    unsigned long long w[8];
#define INIT(i) a[i] = seed * (threadIdx.x + 17u * i + 1u); w[i] = ((unsigned long long)a[i] << 32) | (a[i] ^ 0x9E37u);
    CHAINS8(INIT)
    const unsigned c = seed | 1u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int rep = 0; rep < 4; ++rep) {
            if constexpr (OP == 0) {
#define X(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 1) {
#define X(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 2) {
#define X(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 3) {
#define X(i) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(w[i]) : "v"(a[i]), "v"(c) : "s0", "s1");
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 4) {
#define X(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(c));
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 5) {
#define X(i) asm volatile("v_lshlrev_b64 %0, 2, %0" : "+v"(w[i]));
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 6) {
#define X(i) asm volatile("v_alignbit_b32 %0, %0, %1, 6" : "+v"(a[i]) : "v"(c));
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 7) {
#define X(i) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(c));
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 8) {
#define X(i) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(a[i]));
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 9) {
#define X(i) asm volatile("v_cmp_lt_u64_e64 s[2:3], %0, %1\n\tv_cndmask_b32_e64 %2, %2, %3, s[2:3]" \
                          : "+v"(w[i]), "+v"(w[(i + 1) & 7]), "+v"(a[i]) : "v"(c) : "s2", "s3");
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 10) {
#define X(i) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(w[i]));
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 11) {
#define X(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
                CHAINS8(X)
#undef X
            } else if constexpr (OP == 12) {
#define X(i) asm volatile("v_mul_lo_u32 %0, %0, %1\n\tv_add_u32 %2, %2, %1\n\tv_add_u32 %3, %3, %1" \
                          : "+v"(a[i]), "+v"(a[(i + 3) & 7]), "+v"(a[(i + 5) & 7]) : "v"(c));
                CHAINS8(X)
#undef X
            }
        }
    }
    unsigned s = 0;
#define SUM(i) s += a[i] + (unsigned)w[i] + (unsigned)(w[i] >> 32);
    CHAINS8(SUM)
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

static const char *kNames[] = {"v_add_u32",      "v_mul_lo_u32",  "v_mul_hi_u32",  "v_mad_u64_u32", "v_mul_u32_u24",
                               "v_lshlrev_b64",  "v_alignbit_b32", "v_perm_b32",   "v_bfe_u32",
                               "v_cmp_lt_u64+v_cndmask (2 instr)", "v_lshrrev_b64", "v_xor_b32",
                               "v_mul_lo_u32+2 v_add_u32 (3 instr)"};

template <int OP>
static void run(int cus, double ghz, unsigned *out) {
    const int blocks = cus * 8;  // 8 waves of 64 per SIMD (256-thread blocks, 4 waves each, 2 per SIMD x 4 ... )
    const int iters = 4096;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    valu_loop<OP><<<blocks, 256>>>(out, 64, 12345u);
    hipEventRecord(e0);
    valu_loop<OP><<<blocks, 256>>>(out, iters, 12345u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const int per_iter = (OP == 9 ? 2 : OP == 12 ? 3 : 1) * 8 * 4;
    const double wave_instr = (double)blocks * 4 * iters * per_iter;  // 4 waves per block
    const double per_simd = wave_instr / (cus * 4.0);
    printf("{\"op\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_instr_per_simd\": %.3f}\n", kNames[OP], ms,
           ms * 1e-3 * ghz * 1e9 / per_simd);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main(int argc, char **argv) {
    const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
    hipDeviceProp_t pr;
    hipGetDeviceProperties(&pr, 0);
    unsigned *out;
    hipMalloc(&out, (size_t)pr.multiProcessorCount * 8 * 256 * 4);
    const int cus = pr.multiProcessorCount;
    run<0>(cus, ghz, out); run<1>(cus, ghz, out); run<2>(cus, ghz, out); run<3>(cus, ghz, out);
    run<4>(cus, ghz, out); run<5>(cus, ghz, out); run<6>(cus, ghz, out); run<7>(cus, ghz, out);
    run<8>(cus, ghz, out); run<9>(cus, ghz, out); run<10>(cus, ghz, out); run<11>(cus, ghz, out);
    run<12>(cus, ghz, out);
    hipFree(out);
    return 0;
}
