// kmc_synth.hip — synthetic benchmark input written straight into HBM.
//
// Layout of SURVEY.md §8(d): records of record_len uniform iid ACGT bases, each
// followed by a '\0' terminator (the reference buffer convention, main.cu:537-543);
// base g = "ACGT"[(splitmix64_n(g/32) >> 2*(g%32)) & 3].  tests/ regenerate the same
// bytes on the host (numpy) to check the kernel byte for byte.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kmc.h"
#include "kmc_internal.h"

namespace kmc {
namespace {

// data[b] = global byte start + b of the record stream (record r at r*rec_bytes),
// b < total.
__global__ __launch_bounds__(256) void synth_kernel(char *data, uint64_t total, uint64_t start, uint64_t rec_bytes,
                                                    uint64_t record_len, uint64_t seed, uint64_t first_base) {
    const uint64_t nchunks = (total + 15) / 16;
    for (uint64_t ch = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; ch < nchunks;
         ch += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b0 = ch * 16;
        uint64_t r = (start + b0) / rec_bytes;
        uint64_t off = (start + b0) - r * rec_bytes;
        uint64_t cached_n = ~0ull, word = 0;
        uint32_t v[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            uint32_t byte = 0;
            if (b0 + i < total) {
                if (off < record_len) {
                    const uint64_t g = first_base + r * record_len + off;
                    const uint64_t n = g >> 5;
                    if (n != cached_n) {
                        word = splitmix64_at(seed, n);
                        cached_n = n;
                    }
                    const uint32_t c = (uint32_t)(word >> (2 * (g & 31))) & 3u;
                    byte = (0x54474341u >> (8 * c)) & 0xFFu;  // "ACGT"[c]
                }
            }
            v[i >> 2] |= byte << (8 * (i & 3));
            if (++off == rec_bytes) {
                off = 0;
                ++r;
            }
        }
        if (b0 + 16 <= total) {
            *reinterpret_cast<uint4 *>(data + b0) = make_uint4(v[0], v[1], v[2], v[3]);
        } else {
            for (int i = 0; b0 + i < total; ++i) data[b0 + i] = (char)((v[i >> 2] >> (8 * (i & 3))) & 0xFFu);
        }
    }
}

int launch_synth(char *data, uint64_t total, uint64_t start, uint64_t record_len, uint64_t seed,
                 uint64_t first_base, hipStream_t stream) {
    const uint64_t nchunks = (total + 15) / 16;
    uint64_t blocks = (nchunks + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, data, total, start,
                       record_len + 1, record_len, seed, first_base);
    return (int)hipGetLastError();
}

}  // namespace
}  // namespace kmc

extern "C" int kmc_synth_fill(char *data, uint64_t num_records, uint64_t record_len, uint64_t seed,
                              uint64_t first_base, hipStream_t stream) {
    if (num_records == 0) return KMC_OK;
    if (!data) return KMC_ERR_INVALID_ARG;
    if (reinterpret_cast<uintptr_t>(data) & 15u) return KMC_ERR_ALIGNMENT;
    return kmc::launch_synth(data, num_records * (record_len + 1), 0, record_len, seed, first_base, stream);
}

extern "C" int kmc_synth_fill_range(char *data, uint64_t lo, uint64_t hi, uint64_t record_len, uint64_t seed,
                                    hipStream_t stream) {
    if (hi < lo) return KMC_ERR_INVALID_ARG;
    if (hi == lo) return KMC_OK;
    if (!data) return KMC_ERR_INVALID_ARG;
    if (reinterpret_cast<uintptr_t>(data) & 15u) return KMC_ERR_ALIGNMENT;
    return kmc::launch_synth(data, hi - lo, lo, record_len, seed, 0, stream);
}

extern "C" void kmc_synth_indices(int64_t *indices, uint64_t num_records, uint64_t record_len) {
    for (uint64_t r = 0; r <= num_records; ++r) indices[r] = (int64_t)(r * (record_len + 1));
}
