// kmc_hash.hip — canonical k-mer counting for k <= 31 (BASELINE config C4,
// SURVEY.md §8(b) kmc_count_canonical_hash).  No reference counterpart: the
// reference stops at dense 4^k tables (permutationsCountAll, main.cu:636-646), which
// are infeasible beyond k ~ 13.  Same window and record rules as the dense path;
// the key of a valid window is its 2-bit MSB-first encoding (A0 C1 G2 T3, first
// base most significant, i.e. lexicographic), canonicalised to
// min(key(window), key(reverse complement)) unless KMC_CANON_FORWARD is given.
//
// Layout in HBM: one open-addressing table segment per record, sized from the
// record's window count (load <= 0.7), SoA slots keys[u64] / counts[u32], empty key
// = ~0 (no k-mer reaches it: 62 bits at most).  A slot's count word holds the
// occurrences minus one: insert = a 64-bit CAS on the home slot, which claims an
// empty slot (the first occurrence: nothing else to do) or returns the key that
// holds it (the same key: one 32-bit add), linear probing inside the record's
// segment.  Compaction is a stream compaction of the slot array in slot order:
// live slots per 4096-slot tile, an exclusive scan over tiles (kmc_scan.h), each
// record's output offset = the live slots before its segment, then every tile
// writes its (key, count) pairs at its offset.  Records are contiguous segments,
// so each record's pairs come out contiguous, as the ABI requires.
//
// Bound: random device-scope atomics (one per k-mer when keys are distinct,
// memory-side), not HBM streaming; SURVEY.md §8(d) prices a k-mer at 1 B in +
// 16 B of table.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <vector>

#include "kmc.h"
#include "kmc_scan.h"
#include "kmc_stream.h"

namespace kmc {
namespace {

constexpr uint64_t kEmpty = ~0ull;

struct HParams {
    const char *data;     // global offsets (data[p] is byte p)
    const int64_t *idx;   // device, n + 1
    int64_t n;
    int64_t lo, hi;       // window starts in [lo, hi) (= [idx[0], idx[n]))
    int k;
    uint32_t flags;
    const uint64_t *tbase;  // device, n + 1: table segment of record r
    unsigned long long *keys;
    uint32_t *counts;            // occurrences - 1 of the slot's key
    uint64_t nslots;
    uint32_t *tile_cnt;          // [ntiles] live slots per compaction tile
    uint64_t *tile_off;          // [ntiles + 1] exclusive scan of tile_cnt
    uint64_t *rec_off;           // [n + 1] output offsets
    uint64_t *out_keys;
    uint32_t *out_counts;
};

__device__ __forceinline__ uint64_t fmix64(uint64_t h) {  // MurmurHash3 finaliser
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    h *= 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 33;
    return h;
}

// LE 2-bit code (first base in the low bits, the dense path's order) -> MSB-first
__device__ __forceinline__ uint64_t reverse_groups(uint64_t c, int k) {
    uint64_t x = __builtin_bitreverse64(c);
    x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
    return x >> (64 - 2 * k);
}

__device__ __forceinline__ int64_t upper_record(const int64_t *idx, int64_t n, int64_t p) {
    // largest r in [0, n) with idx[r] <= p (callers guarantee idx[0] <= p < idx[n])
    int64_t a = 0, b = n;  // idx[a] <= p < idx[b]
    while (b - a > 1) {
        const int64_t m = (a + b) >> 1;
        if (idx[m] <= p) a = m; else b = m;
    }
    return a;
}

__device__ __forceinline__ uint4 load16(const char *data, int64_t q, int64_t hi_byte) {
    // 16 bytes at q (16-aligned); bytes at or past hi_byte read as 0
    if (q + 16 <= hi_byte) return *reinterpret_cast<const uint4 *>(data + q);
    uint32_t v[4] = {0u, 0u, 0u, 0u};
    for (int i = 0; i < 16; ++i)
        if (q + i < hi_byte) v[i >> 2] |= (uint32_t)(uint8_t)data[q + i] << (8 * (i & 3));
    return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void chunk_codes(uint4 r, bool soft, uint32_t &code, uint32_t &bad) {
    if (soft) {  // lowercase acgt -> ACGT (clearing bit 5 maps no other byte onto a base letter)
        r.x &= 0xDFDFDFDFu; r.y &= 0xDFDFDFDFu; r.z &= 0xDFDFDFDFu; r.w &= 0xDFDFDFDFu;
    }
    uint32_t any;
    decode16(r, code, any);
    bad = any ? bad_mask16(r) : 0u;
}

// One thread per 16-byte chunk (grid-stride): the chunk's 16 window starts, with
// the next 32 bytes as halo (k <= 31 reaches 30 bytes past the chunk).
__global__ __launch_bounds__(256) void hash_insert_kernel(HParams p) {
    const int k = p.k;
    const bool soft = p.flags & KMC_CANON_SOFTMASK;
    const bool fwd_only = p.flags & KMC_CANON_FORWARD;
    const uint64_t kmask = k == 32 ? ~0ull : ((1ull << (2 * k)) - 1);
    const uint64_t wmask = (1ull << k) - 1;
    const int64_t c_lo = p.lo >> 4, c_hi = (p.hi + 15) >> 4;
    const int64_t hi_byte = p.idx[p.n];
    for (int64_t c = c_lo + (int64_t)blockIdx.x * 256 + threadIdx.x; c < c_hi; c += (int64_t)gridDim.x * 256) {
        const int64_t q = c << 4;
        uint32_t cd[3], bd[3];
#pragma unroll
        for (int h = 0; h < 3; ++h) chunk_codes(load16(p.data, q + 16 * h, hi_byte), soft, cd[h], bd[h]);
        const uint64_t lo64 = (uint64_t)cd[0] | ((uint64_t)cd[1] << 32);
        const uint64_t badm = (uint64_t)bd[0] | ((uint64_t)bd[1] << 16) | ((uint64_t)bd[2] << 32);
        const int64_t first = q > p.lo ? q : p.lo;
        int64_t r = upper_record(p.idx, p.n, first);
        int64_t rend = p.idx[r + 1];
        for (int j = (int)(first - q); j < 16; ++j) {
            const int64_t pos = q + j;
            if (pos >= p.hi) break;
            while (pos >= rend) {  // next record (short records: several per chunk)
                ++r;
                rend = p.idx[r + 1];
            }
            if (pos > rend - 1 - k) continue;           // window runs into the terminator
            if ((badm >> j) & wmask) continue;          // invalid base in the window
            const uint64_t le = (j == 0 ? lo64 : ((lo64 >> (2 * j)) | ((uint64_t)cd[2] << (64 - 2 * j)))) & kmask;
            const uint64_t fw = reverse_groups(le, k);
            const uint64_t key = fwd_only ? fw : (fw < (le ^ kmask) ? fw : (le ^ kmask));
            const uint64_t base = p.tbase[r], cap = p.tbase[r + 1] - base;
            uint64_t s = __umul64hi(fmix64(key), cap);
            for (;;) {
                const unsigned long long cur = atomicCAS(&p.keys[base + s], kEmpty, (unsigned long long)key);
                if (cur == kEmpty) break;  // claimed: first occurrence (count word stays 0)
                if (cur == key) {
                    __hip_atomic_fetch_add(&p.counts[base + s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                s = (s + 1 == cap) ? 0 : s + 1;
            }
        }
    }
}

// Stream compaction of the slot array.  A tile is kCompTile consecutive slots,
// kScanBlock threads x 4 slots each (two uint4 key loads, one uint4 count load).
constexpr int kCompPer = 4;
constexpr int64_t kCompTile = (int64_t)kScanBlock * kCompPer;

__device__ __forceinline__ uint32_t live4(const HParams &p, uint64_t s0, unsigned long long k[4]) {
    uint32_t m = 0;
    if (s0 + 4 <= p.nslots) {
        const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(p.keys + s0);
        const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(p.keys + s0 + 2);
        k[0] = a.x; k[1] = a.y; k[2] = b.x; k[3] = b.y;
    } else {
        for (int q = 0; q < 4; ++q) k[q] = s0 + q < p.nslots ? p.keys[s0 + q] : kEmpty;
    }
    for (int q = 0; q < 4; ++q) m |= (uint32_t)(k[q] != kEmpty) << q;
    return m;
}

// live slots per tile
__global__ __launch_bounds__(kScanBlock) void hash_tilecount_kernel(HParams p) {
    __shared__ uint64_t sh[kScanBlock / 64];
    const uint64_t s0 = (uint64_t)blockIdx.x * kCompTile + (uint64_t)threadIdx.x * kCompPer;
    unsigned long long k[4];
    const uint32_t m = live4(p, s0, k);
    uint64_t total;
    block_excl_scan((uint64_t)__popc(m), sh, total);
    if (threadIdx.x == 0) p.tile_cnt[blockIdx.x] = (uint32_t)total;
}

// rec_off[r] = live slots before record r's segment (one wave per record; r = n: the total)
__global__ __launch_bounds__(256) void hash_recoff_kernel(HParams p, int64_t ntiles) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r > p.n) return;
    if (r == p.n) {
        if (lane == 0) p.rec_off[r] = p.tile_off[ntiles];
        return;
    }
    const uint64_t pos = p.tbase[r];
    const uint64_t t = pos / (uint64_t)kCompTile, t0 = t * (uint64_t)kCompTile;
    uint32_t c = 0;
    for (uint64_t s = t0 + lane; s < pos; s += 64) c += p.keys[s] != kEmpty;
    c = wave_sum(c);
    if (lane == 0) p.rec_off[r] = p.tile_off[t] + c;
}

// (key, count) of every live slot, in slot order, at its tile's offset
__global__ __launch_bounds__(kScanBlock) void hash_emit_kernel(HParams p) {
    __shared__ uint64_t sh[kScanBlock / 64];
    const uint64_t s0 = (uint64_t)blockIdx.x * kCompTile + (uint64_t)threadIdx.x * kCompPer;
    unsigned long long k[4];
    const uint32_t m = live4(p, s0, k);
    uint64_t total;
    uint64_t o = p.tile_off[blockIdx.x] + block_excl_scan((uint64_t)__popc(m), sh, total);
    if (m) {
        uint32_t c[4];
        if (s0 + 4 <= p.nslots) {
            const uint4 v = *reinterpret_cast<const uint4 *>(p.counts + s0);
            c[0] = v.x; c[1] = v.y; c[2] = v.z; c[3] = v.w;
        } else {
            for (int q = 0; q < 4; ++q) c[q] = s0 + q < p.nslots ? p.counts[s0 + q] : 0u;
        }
        for (int q = 0; q < 4; ++q) {
            if ((m >> q) & 1u) {
                p.out_keys[o] = k[q];
                p.out_counts[o] = c[q] + 1u;
                ++o;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
struct HCache {
    void *ptr = nullptr;
    size_t bytes = 0;
};
std::mutex h_mu;
std::vector<HCache> h_ws;

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// slots of record r: windows / 0.7, at least 16
inline uint64_t seg_cap(int64_t len_with_term, int k) {
    const int64_t w = len_with_term - k > 0 ? len_with_term - k : 0;
    uint64_t c = (uint64_t)w + (uint64_t)w * 3 / 7 + 1;
    return c < 16 ? 16 : c;
}

}  // namespace
}  // namespace kmc

using namespace kmc;

extern "C" int kmc_count_canonical_hash(const char *data, const int64_t *indices, uint64_t num_seqs, int k,
                                        unsigned flags, uint64_t *keys, uint32_t *counts, uint64_t capacity,
                                        uint64_t *rec_offsets, uint64_t *num_distinct, hipStream_t stream) {
    if (k < 1 || k > KMC_CANON_MAX_K) return KMC_ERR_UNSUPPORTED_K;
    if (!num_distinct) return KMC_ERR_INVALID_ARG;
    *num_distinct = 0;
    if (num_seqs == 0) return KMC_OK;
    if (!data || !indices || !rec_offsets) return KMC_ERR_INVALID_ARG;
    if (reinterpret_cast<uintptr_t>(data) & 15u) return KMC_ERR_ALIGNMENT;
    const int64_t n = (int64_t)num_seqs;
    std::vector<int64_t> hidx(n + 1);
    hipError_t he = hipMemcpyAsync(hidx.data(), indices, (n + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, stream);
    if (he == hipSuccess) he = hipStreamSynchronize(stream);
    if (he != hipSuccess) return (int)he;
    std::vector<uint64_t> tb(n + 1);
    tb[0] = 0;
    for (int64_t r = 0; r < n; ++r) {
        if (hidx[r + 1] < hidx[r]) return KMC_ERR_INVALID_ARG;
        tb[r + 1] = tb[r] + seg_cap(hidx[r + 1] - hidx[r], k);
    }
    const uint64_t nslots = tb[n];
    const int64_t ntiles = (int64_t)((nslots + kCompTile - 1) / kCompTile);
    // workspace: tbase, keys, counts, tile counts, tile offsets, scan block sums
    size_t o = 0;
    const size_t o_tb = o; o += al256((n + 1) * 8);
    const size_t o_keys = o; o += al256(nslots * 8);
    const size_t o_cnt = o; o += al256(nslots * 4);
    const size_t o_tc = o; o += al256((size_t)ntiles * 4);
    const size_t o_to = o; o += al256((size_t)(ntiles + 1) * 8);
    const size_t o_bs = o; o += al256((size_t)(scan_tiles(ntiles) + 1) * 8);
    const size_t total = o;
    int device = 0;
    he = hipGetDevice(&device);
    if (he != hipSuccess) return (int)he;
    char *ws;
    {
        std::lock_guard<std::mutex> lk(h_mu);
        if ((int)h_ws.size() <= device) h_ws.resize(device + 1);
        HCache &c = h_ws[device];
        if (c.bytes < total) {
            if (c.ptr && hipFree(c.ptr) != hipSuccess) return KMC_ERR_NOMEM;
            c.ptr = nullptr;
            c.bytes = 0;
            if (hipMalloc(&c.ptr, total) != hipSuccess) return KMC_ERR_NOMEM;
            c.bytes = total;
        }
        ws = static_cast<char *>(c.ptr);
    }
    HParams p{};
    p.data = data;
    p.idx = indices;
    p.n = n;
    p.lo = hidx[0];
    p.hi = hidx[n];
    p.k = k;
    p.flags = flags;
    p.tbase = reinterpret_cast<uint64_t *>(ws + o_tb);
    p.keys = reinterpret_cast<unsigned long long *>(ws + o_keys);
    p.counts = reinterpret_cast<uint32_t *>(ws + o_cnt);
    p.nslots = nslots;
    p.tile_cnt = reinterpret_cast<uint32_t *>(ws + o_tc);
    p.tile_off = reinterpret_cast<uint64_t *>(ws + o_to);
    uint64_t *bsum = reinterpret_cast<uint64_t *>(ws + o_bs);
    p.rec_off = rec_offsets;
    p.out_keys = keys;
    p.out_counts = counts;
    if ((he = hipMemcpyAsync((void *)p.tbase, tb.data(), (n + 1) * 8, hipMemcpyHostToDevice, stream)) ||
        (he = hipMemsetAsync(p.keys, 0xFF, nslots * 8, stream)) || (he = hipMemsetAsync(p.counts, 0, nslots * 4, stream)))
        return (int)he;
    const int64_t chunks = ((p.hi + 15) >> 4) - (p.lo >> 4);
    if (chunks > 0) {
        const int64_t blocks = std::min<int64_t>((chunks + 255) / 256, 1 << 16);
        hipLaunchKernelGGL(hash_insert_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, p);
    }
    hipLaunchKernelGGL(hash_tilecount_kernel, dim3((unsigned)ntiles), dim3(kScanBlock), 0, stream, p);
    excl_scan_u32(p.tile_cnt, ntiles, bsum, p.tile_off, stream);
    hipLaunchKernelGGL(hash_recoff_kernel, dim3((unsigned)((n + 1 + 3) / 4)), dim3(256), 0, stream, p, ntiles);
    uint64_t distinct = 0;
    if ((he = hipGetLastError()) ||
        (he = hipMemcpyAsync(&distinct, p.rec_off + n, 8, hipMemcpyDeviceToHost, stream)) ||
        (he = hipStreamSynchronize(stream)))
        return (int)he;
    *num_distinct = distinct;
    if (distinct > capacity) return KMC_ERR_CAPACITY;
    if (distinct && (!keys || !counts)) return KMC_ERR_INVALID_ARG;
    hipLaunchKernelGGL(hash_emit_kernel, dim3((unsigned)ntiles), dim3(kScanBlock), 0, stream, p);
    if ((he = hipGetLastError()) || (he = hipStreamSynchronize(stream))) return (int)he;
    return KMC_OK;
}
