// kmc_dist.hip — pairwise k-mer distance over the count matrix.
//
// The reference's step 2 launches minKmeres2 (kernels.h:85-109) once per record
// from a host loop with a device sync after each launch (main.cu:326-335); its CPU
// twin is the pair loop of sequentialKmerCount2 (main.cu:604-619).  Both compute,
// for every pair i < j,
//
//     d(i, j) = 1 - S_ij / (min(len_i, len_j) - k + 1),
//     S_ij    = sum over codes of min(count_i[code], count_j[code]),
//     len_s   = indices[s+1] - indices[s] - 1,
//
// stored at getIdxTriangularMatrixRowMajor(i+1, j-i, n) (kernels.h:46-48) of a
// packed upper triangle.  Here all pairs are one launch: the pair matrix is tiled
// (64 x 64 records, or 16 x 16 when num_seqs <= 16), the bin axis is streamed
// through LDS in chunks of 32 codes and, when there are too few tiles to fill the
// chip, split across workgroups whose exact integer partial sums meet in a uint64
// scratch (atomics; integer addition is order-free).  S_ij is exact (uint64), as
// in the CPU path (`long sum`, main.cu:612): the float result is the CPU path's
// bit for bit, and the GPU kernel's (float accumulation, kernels.h:103) whenever
// its running sum stays below 2^24.
//
// minKmeres2_hip is the drop-in for one reference launch, accumulating in float in
// code order exactly like kernels.h:103 so its output matches that kernel bit for
// bit at any record length.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <vector>

#include "kmc.h"

namespace kmc {
namespace {

constexpr int kChunk = 32;  // codes per LDS chunk

struct DParams {
    const int32_t *sum;
    int64_t ld;
    const int64_t *indices;
    int64_t n;
    int k;
    int64_t nbins;
    int64_t split_len;  // codes per split (multiple of kChunk)
    int tiles;          // tiles per side
    float *out;
    unsigned long long *acc;  // [npairs] when split, else null
};

// packed upper triangle, row-major: getIdxTriangularMatrixRowMajor(i+1, j-i, n)
// (kernels.h:46-48) = n*i - i*(i-1)/2 + (j - i) - (i + 1)
__device__ __forceinline__ int64_t tri_index(int64_t i, int64_t j, int64_t n) {
    return n * i - (i * (i - 1)) / 2 + (j - i) - (i + 1);
}

// The CPU formula, main.cu:614: 1 - (float)sum / (minLength - k + 1), the long
// denominator converted to float by the usual arithmetic conversions.
__device__ __forceinline__ float distance_of(uint64_t s, int64_t li, int64_t lj, int k) {
    const int64_t m = li < lj ? li : lj;
    return 1.0f - (float)s / (float)(m - k + 1);
}

__device__ __forceinline__ int64_t rec_len(const int64_t *idx, int64_t s) { return idx[s + 1] - idx[s] - 1; }

// TT records per tile side; each thread owns TM x TN pairs and every Z-th code
// of a chunk (TT/TM * TT/TN * Z = 256 threads).
template <int TT, int TM, int TN>
__global__ __launch_bounds__(256) void pair_min_kernel(DParams p) {
    constexpr int NX = TT / TN, NY = TT / TM, Z = 256 / (NX * NY);
    static_assert(NX * NY * Z == 256, "thread layout");
    const int tj = blockIdx.x, ti = blockIdx.y;
    if (ti > tj) return;
    const bool diag = ti == tj;
    __shared__ __attribute__((aligned(16))) uint32_t A[kChunk][TT];
    __shared__ __attribute__((aligned(16))) uint32_t B[kChunk][TT];
    __shared__ unsigned long long red[Z > 1 ? 256 : 1];

    const int tid = threadIdx.x;
    const int tx = tid % NX, ty = (tid / NX) % NY, tz = tid / (NX * NY);
    const int64_t c0 = (int64_t)blockIdx.z * p.split_len;
    const int64_t c1 = (c0 + p.split_len) < p.nbins ? (c0 + p.split_len) : p.nbins;
    const int64_t ri0 = (int64_t)ti * TT, rj0 = (int64_t)tj * TT;

    uint64_t tot[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) tot[a][b] = 0;

    for (int64_t c = c0; c < c1; c += kChunk) {
        // stage counts[code c..c+31][records of the two tiles]; rows are contiguous in records
        for (int e = tid; e < kChunk * TT; e += 256) {
            const int r = e / TT, col = e % TT;
            const int64_t code = c + r;
            const bool okc = code < c1;
            const int64_t ra = ri0 + col, rb = rj0 + col;
            A[r][col] = (okc && ra < p.n) ? (uint32_t)p.sum[ra + p.ld * code] : 0u;
            if (!diag) B[r][col] = (okc && rb < p.n) ? (uint32_t)p.sum[rb + p.ld * code] : 0u;
        }
        __syncthreads();
        const uint32_t(*Bs)[TT] = diag ? A : B;
        uint32_t part[TM][TN];
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) part[a][b] = 0;
#pragma unroll 8
        for (int r = tz; r < kChunk; r += Z) {
            uint32_t va[TM], vb[TN];
#pragma unroll
            for (int a = 0; a < TM; ++a) va[a] = A[r][ty * TM + a];
#pragma unroll
            for (int b = 0; b < TN; ++b) vb[b] = Bs[r][tx * TN + b];
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b) part[a][b] += va[a] < vb[b] ? va[a] : vb[b];
        }
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) tot[a][b] += part[a][b];
        __syncthreads();
    }

    // combine the Z code lanes of each pair, then publish
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            uint64_t s = tot[a][b];
            if constexpr (Z > 1) {
                red[tid] = s;
                __syncthreads();
                if (tz == 0)
                    for (int z = 1; z < Z; ++z) s += red[tid + z * NX * NY];
                __syncthreads();
                if (tz != 0) continue;
            }
            const int64_t i = ri0 + ty * TM + a, j = rj0 + tx * TN + b;
            if (i >= j || j >= p.n) continue;
            const int64_t q = tri_index(i, j, p.n);
            if (p.acc)
                atomicAdd(&p.acc[q], (unsigned long long)s);
            else
                p.out[q] = distance_of(s, rec_len(p.indices, i), rec_len(p.indices, j), p.k);
        }
    }
}

// split path: acc[pair] -> out[pair]
__global__ __launch_bounds__(256) void pair_finish_kernel(DParams p) {
    const int64_t npairs = p.n * (p.n - 1) / 2;
    for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < npairs; q += (int64_t)gridDim.x * 256) {
        // invert q = tri_index(i, j): row i starts at n*i - i*(i+1)/2 (found by search from a float guess)
        const double nn = (double)p.n;
        int64_t i = (int64_t)((2 * nn - 1 - sqrt((2 * nn - 1) * (2 * nn - 1) - 8.0 * (double)q)) / 2);
        if (i < 0) i = 0;
        while (i > 0 && p.n * i - i * (i + 1) / 2 > q) --i;
        while (p.n * (i + 1) - (i + 1) * (i + 2) / 2 <= q) ++i;
        const int64_t j = q - (p.n * i - i * (i + 1) / 2) + i + 1;
        p.out[q] = distance_of(p.acc[q], rec_len(p.indices, i), rec_len(p.indices, j), p.k);
    }
}

// Drop-in for one minKmeres2 launch (kernels.h:85-109): row current_seq against
// every later record, K = KMC_DROPIN_K codes, float accumulation in code order.
__global__ __launch_bounds__(256) void min_kmeres2_kernel(const int *sums, float *mins, int n, int cur,
                                                          const int *indexes) {
    constexpr int P = 1 << (2 * KMC_DROPIN_K);
    __shared__ int row[P];
    for (int t = threadIdx.x; t < P; t += 256) row[t] = sums[t * n + cur];
    __syncthreads();
    const int j = cur + 1 + (int)(blockIdx.x * 256 + threadIdx.x);
    if (j >= n) return;
    float s = 0.0f;
    for (int t = 0; t < P; ++t) {
        const int b = sums[j + n * t];
        s += (float)(row[t] < b ? row[t] : b);
    }
    int le = indexes[cur + 1] - indexes[cur] - 1, lc = indexes[j + 1] - indexes[j] - 1;
    if (le < lc) lc = le;
    s = 1.0f - s / (float)(lc - KMC_DROPIN_K + 1);
    mins[tri_index(cur, j, n)] = s;
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
struct Plan {
    bool small;
    int tiles;
    int64_t split_len, splits;
    size_t ws;
};

inline Plan plan_for(int64_t n, int k, int cus) {
    Plan P;
    P.small = n <= 16;
    const int TT = P.small ? 16 : 64;
    P.tiles = (int)((n + TT - 1) / TT);
    const int64_t nbins = (int64_t)1 << (2 * k);
    const int64_t tile_pairs = (int64_t)P.tiles * (P.tiles + 1) / 2;
    const int64_t want = 4LL * cus;  // workgroups to fill the chip
    int64_t splits = tile_pairs >= want ? 1 : (want + tile_pairs - 1) / tile_pairs;
    const int64_t max_splits = (nbins + 4 * kChunk - 1) / (4 * kChunk);  // >= 4 chunks per split
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    int64_t len = (nbins + splits - 1) / splits;
    len = (len + kChunk - 1) / kChunk * kChunk;
    P.split_len = len;
    P.splits = (nbins + len - 1) / len;
    P.ws = P.splits > 1 ? (size_t)(n * (n - 1) / 2) * 8 : 0;
    return P;
}

std::mutex d_mu;
std::vector<int> d_cus;
std::vector<std::pair<void *, size_t>> d_ws;

int cus_of(int device, int &cus) {
    std::lock_guard<std::mutex> lk(d_mu);
    if ((int)d_cus.size() <= device) d_cus.resize(device + 1, 0);
    if (d_cus[device] == 0) {
        hipError_t e = hipDeviceGetAttribute(&d_cus[device], hipDeviceAttributeMultiprocessorCount, device);
        if (e != hipSuccess) return (int)e;
    }
    cus = d_cus[device];
    return 0;
}

}  // namespace
}  // namespace kmc

using namespace kmc;

extern "C" size_t kmc_pair_distances_workspace_size(uint64_t num_seqs, int k, int device) {
    if (k < 1 || k > KMC_DENSE_MAX_K || num_seqs < 2) return 0;
    int cus = 0;
    if (cus_of(device, cus)) return 0;
    return plan_for((int64_t)num_seqs, k, cus).ws;
}

extern "C" int kmc_pair_distances(const int32_t *sum, uint64_t sum_ld, const int64_t *indices, uint64_t num_seqs,
                                  int k, float *out, void *workspace, size_t workspace_bytes, hipStream_t stream) {
    if (k < 1 || k > KMC_DENSE_MAX_K) return KMC_ERR_UNSUPPORTED_K;
    if (num_seqs < 2) return KMC_OK;
    if (!sum || !indices || !out) return KMC_ERR_INVALID_ARG;
    if (sum_ld != 0 && sum_ld < num_seqs) return KMC_ERR_INVALID_ARG;
    if (num_seqs > (1ull << 31)) return KMC_ERR_INVALID_ARG;
    int device = 0;
    hipError_t he = hipGetDevice(&device);
    if (he != hipSuccess) return (int)he;
    int cus = 0;
    int e = cus_of(device, cus);
    if (e) return e;
    const int64_t n = (int64_t)num_seqs;
    const Plan P = plan_for(n, k, cus);
    if (P.tiles > 65535) return KMC_ERR_INVALID_ARG;
    void *ws = workspace;
    if (P.ws) {
        if (ws == nullptr) {
            std::lock_guard<std::mutex> lk(d_mu);
            if ((int)d_ws.size() <= device) d_ws.resize(device + 1, {nullptr, 0});
            auto &c = d_ws[device];
            if (c.second < P.ws) {
                if (c.first && hipFree(c.first) != hipSuccess) return KMC_ERR_NOMEM;
                c = {nullptr, 0};
                if (hipMalloc(&c.first, P.ws) != hipSuccess) return KMC_ERR_NOMEM;
                c.second = P.ws;
            }
            ws = c.first;
        } else if (workspace_bytes < P.ws) {
            return KMC_ERR_WORKSPACE;
        }
    }
    DParams p;
    p.sum = sum;
    p.ld = sum_ld ? (int64_t)sum_ld : n;
    p.indices = indices;
    p.n = n;
    p.k = k;
    p.nbins = (int64_t)1 << (2 * k);
    p.split_len = P.split_len;
    p.tiles = P.tiles;
    p.out = out;
    p.acc = P.ws ? static_cast<unsigned long long *>(ws) : nullptr;
    if (p.acc) {
        he = hipMemsetAsync(p.acc, 0, P.ws, stream);
        if (he != hipSuccess) return (int)he;
    }
    const dim3 grid((unsigned)P.tiles, (unsigned)P.tiles, (unsigned)P.splits);
    if (P.small)
        hipLaunchKernelGGL((pair_min_kernel<16, 1, 4>), grid, dim3(256), 0, stream, p);
    else
        hipLaunchKernelGGL((pair_min_kernel<64, 4, 4>), grid, dim3(256), 0, stream, p);
    if (p.acc) {
        const int64_t npairs = n * (n - 1) / 2;
        int64_t blocks = (npairs + 255) / 256;
        if (blocks > 8192) blocks = 8192;
        hipLaunchKernelGGL(pair_finish_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, p);
    }
    return (int)hipGetLastError();
}

extern "C" int minKmeres2_hip(int *sums, float *mins, int num_seqs, int current_seq, int *indexes,
                              hipStream_t stream) {
    if (num_seqs < 0 || current_seq < 0) return KMC_ERR_INVALID_ARG;
    if (current_seq >= num_seqs - 1) return KMC_OK;  // no later record: the reference writes nothing
    if (!sums || !mins || !indexes) return KMC_ERR_INVALID_ARG;
    const int rest = num_seqs - 1 - current_seq;
    hipLaunchKernelGGL(min_kmeres2_kernel, dim3((unsigned)((rest + 255) / 256)), dim3(256), 0, stream, sums, mins,
                       num_seqs, current_seq, indexes);
    return (int)hipGetLastError();
}
