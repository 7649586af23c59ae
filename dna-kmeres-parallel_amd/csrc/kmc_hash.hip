// kmc_hash.hip — canonical k-mer counting for k <= 31 (BASELINE config C4,
// SURVEY.md §8(b) kmc_count_canonical_hash).  No reference counterpart: the
// reference stops at dense 4^k tables (permutationsCountAll, main.cu:636-646), which
// are infeasible beyond k ~ 13.  Same window and record rules as the dense path;
// the key of a valid window is its 2-bit MSB-first encoding (A0 C1 G2 T3, first
// base most significant, i.e. lexicographic), canonicalised to
// min(key(window), key(reverse complement)) unless KMC_CANON_FORWARD is given.
//
// Hash-partitioned counting, so that no table lives in HBM and no k-mer costs a
// device-scope atomic:
//   K1 count    workgroups walk contiguous chunk ranges record piece by record
//               piece; each window's list is (record r, top bits of fmix64(key)),
//               nb_r = 2^lg_r lists per record (about 4 K windows each); per-piece
//               LDS counters -> cnt[(r, list, workgroup)]
//   K2 scan     exclusive prefix sum: every list contiguous, workgroup segments
//               inside it (kmc_scan.h)
//   K3 scatter  the same walk writes each window's key at its list position
//               (LDS 64-bit cursors per list)
//   K4 count    one workgroup per list: an LDS open-addressing table (64-bit CAS
//               claim, 32-bit add) counts the list, in as many passes over it as
//               keep a pass's distinct keys under the table's capacity (selected
//               by further hash bits); each pass's (key, count) pairs are compacted
//               to the list's output segment; distinct keys per list
//   K5 place    exclusive scan of the distinct counts; each list's pairs are copied
//               to their final place; records are contiguous runs of lists
// Bytes per window: the input twice (K1, K3), an 8-byte key written and read, at
// most 12 bytes of pairs written, read and written again.
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

constexpr uint64_t kEmpty = ~0ull;           // no k-mer key reaches it (62 bits at most)
// K3 walks a piece once per group of lists, 2^KMC_CANON_SCATTER_LG groups at
// most (write locality, see K3)
#ifndef KMC_CANON_SCATTER_LG
#define KMC_CANON_SCATTER_LG 2
#endif
constexpr int kWalkBlock = 1024;             // K1 / K3 threads per workgroup
constexpr int kMaxLg = 14;                   // at most 16 384 lists per record (more lists: more open write segments in K3)
constexpr int64_t kListTarget = 4096;        // windows per list aimed at
constexpr int kCountBlock = 1024;            // K4 threads per workgroup
constexpr int kTableSlots = 12288;           // K4 LDS table: 12 288 x (8 + 4) B = 144 KB
constexpr int kPassDistinct = 8192;          // keys per K4 pass aimed at (table load <= 2/3)

struct HParams {
    const char *data;        // global offsets (data[p] is byte p)
    const int64_t *idx;      // device, n + 1
    int64_t n;
    int64_t lo, hi;          // window starts in [lo, hi) (= [idx[0], idx[n]))
    int k;
    uint32_t flags;
    int G;                   // K1 / K3 workgroups
    int64_t c_lo, cpw;       // chunk range start, chunks per workgroup
    const uint8_t *lg;       // [n] log2 lists of each record
    const int64_t *cbase;    // [n] cnt index of (r, list 0, its first workgroup)
    const int32_t *w0;       // [n] first workgroup holding windows of r
    const int32_t *nwg;      // [n] workgroups holding windows of r
    const int64_t *lbase;    // [n + 1] global id of list 0 of record r (lbase[n] = lists)
    uint32_t *cnt;           // [M] windows per (record, list, workgroup)
    uint64_t *off;           // [M + 1] exclusive scan of cnt
    uint64_t *ent;           // [windows] keys, list by list
    uint64_t *list_start;    // [lists + 1]
    uint64_t *pk;            // [windows] K4 pairs: keys
    uint32_t *pc;            // [windows] K4 pairs: counts
    uint32_t *ndist;         // [lists] distinct keys per list
    uint64_t *dist_off;      // [lists + 1] exclusive scan of ndist
    int64_t lists;
    uint64_t *rec_off;       // [n + 1] output offsets
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

// Calls f(key) for every valid window of record piece [ps, pe) (window starts) of
// a record whose terminator is at rend - 1; the workgroup's threads take the
// piece's 16-byte chunks in turn.  Every thread runs the same number of rounds.
template <class F>
__device__ __forceinline__ void walk_piece(const HParams &p, int64_t ps, int64_t pe, int64_t rend, F &&f) {
    const int k = p.k;
    const bool soft = p.flags & KMC_CANON_SOFTMASK;
    const bool fwd_only = p.flags & KMC_CANON_FORWARD;
    const uint64_t kmask = (1ull << (2 * k)) - 1;
    const uint64_t wmask = (1ull << k) - 1;
    const int64_t hi_byte = p.idx[p.n];
    const int64_t c0 = ps >> 4, c1 = ((pe - 1) >> 4) + 1;
    for (int64_t c = c0 + threadIdx.x; c < c1; c += kWalkBlock) {
        const int64_t q = c << 4;
        uint32_t cd[3], bd[3];
#pragma unroll
        for (int h = 0; h < 3; ++h) chunk_codes(load16(p.data, q + 16 * h, hi_byte), soft, cd[h], bd[h]);
        const uint64_t lo64 = (uint64_t)cd[0] | ((uint64_t)cd[1] << 32);
        const uint64_t badm = (uint64_t)bd[0] | ((uint64_t)bd[1] << 16) | ((uint64_t)bd[2] << 32);
#pragma unroll 4
        for (int j = 0; j < 16; ++j) {
            const int64_t pos = q + j;
            if (pos < ps || pos >= pe || pos > rend - 1 - k) continue;
            if ((badm >> j) & wmask) continue;  // invalid base in the window
            const uint64_t le = (j == 0 ? lo64 : ((lo64 >> (2 * j)) | ((uint64_t)cd[2] << (64 - 2 * j)))) & kmask;
            const uint64_t fw = reverse_groups(le, k);
            f(fwd_only ? fw : (fw < (le ^ kmask) ? fw : (le ^ kmask)));
        }
    }
}

// The workgroup's chunk range and its record pieces: f(r, ps, pe, rend).
template <class F>
__device__ __forceinline__ void for_each_piece(const HParams &p, int64_t *s_first, F &&f) {
    const int w = blockIdx.x;
    const int64_t cb = p.c_lo + (int64_t)w * p.cpw;
    const int64_t wlo = std::max<int64_t>(cb << 4, p.lo), whi = std::min<int64_t>((cb + p.cpw) << 4, p.hi);
    if (wlo >= whi) return;
    if (threadIdx.x == 0) {  // last record r with idx[r] <= wlo
        int64_t a = 0, b = p.n - 1;
        while (a < b) {
            const int64_t m = (a + b + 1) >> 1;
            if (p.idx[m] <= wlo) a = m; else b = m - 1;
        }
        *s_first = a;
    }
    __syncthreads();
    for (int64_t r = *s_first; r < p.n; ++r) {
        const int64_t a = p.idx[r], e = p.idx[r + 1];
        if (a >= whi) break;
        const int64_t nw = e - a - p.k > 0 ? e - a - p.k : 0;
        const int64_t ps = std::max(a, wlo), pe = std::min(a + nw, whi);
        if (ps >= pe) continue;
        f(r, ps, pe, e);
    }
}

__device__ __forceinline__ uint32_t list_of(uint64_t key, int lg) {
    return lg ? (uint32_t)(fmix64(key) >> (64 - lg)) : 0u;
}

// K1: windows per (record, list, workgroup)
__global__ __launch_bounds__(kWalkBlock) void canon_count_kernel(HParams p) {
    __shared__ uint32_t c[1 << kMaxLg];
    __shared__ int64_t s_first;
    const int w = blockIdx.x;
    for_each_piece(p, &s_first, [&](int64_t r, int64_t ps, int64_t pe, int64_t rend) {
        const int lg = p.lg[r];
        const int nb = 1 << lg;
        for (int b = threadIdx.x; b < nb; b += kWalkBlock) c[b] = 0u;
        __syncthreads();
        walk_piece(p, ps, pe, rend, [&](uint64_t key) {
            __hip_atomic_fetch_add(&c[list_of(key, lg)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        });
        __syncthreads();
        const int64_t base = p.cbase[r] + (w - p.w0[r]);
        for (int b = threadIdx.x; b < nb; b += kWalkBlock) p.cnt[base + (int64_t)b * p.nwg[r]] = c[b];
        __syncthreads();
    });
}

// K3: every window's key at its list position
__global__ __launch_bounds__(kWalkBlock) void canon_scatter_kernel(HParams p) {
    __shared__ uint32_t cur[1 << kMaxLg];  // relative to the record's first entry (< 2^32 per record)
    __shared__ int64_t s_first;
    const int w = blockIdx.x;
    for_each_piece(p, &s_first, [&](int64_t r, int64_t ps, int64_t pe, int64_t rend) {
        const int lg = p.lg[r];
        const int nb = 1 << lg;
        const int64_t base = p.cbase[r] + (w - p.w0[r]);
        const uint64_t rbase = p.off[p.cbase[r]];
        for (int b = threadIdx.x; b < nb; b += kWalkBlock)
            cur[b] = (uint32_t)(p.off[base + (int64_t)b * p.nwg[r]] - rbase);
        __syncthreads();
        uint64_t *ent = p.ent + rbase;
        // the piece is walked once per group of lists: a workgroup keeps one
        // partially written 128-B line open per list it writes, and with all of a
        // record's lists open on every workgroup those lines overflow the
        // Infinity Cache, turning each 8-B key store into a read-modify-write in HBM
        const int glg = lg < KMC_CANON_SCATTER_LG ? lg : KMC_CANON_SCATTER_LG;  // log2 groups
        const int gshift = lg - glg;
        const uint32_t ng = 1u << glg;
        for (uint32_t g = 0; g < ng; ++g) {
            walk_piece(p, ps, pe, rend, [&](uint64_t key) {
                const uint32_t l = list_of(key, lg);
                if ((l >> gshift) != g) return;
                const uint32_t i = __hip_atomic_fetch_add(&cur[l], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                ent[i] = key;
            });
        }
        __syncthreads();
    });
}

// list boundaries: list (r, b) = off[cbase_r + b*nwg_r] .. off[cbase_r + (b+1)*nwg_r];
// one thread per list (lbase is sorted: the record is a binary search)
__global__ void canon_list_start_kernel(HParams p) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l > p.lists) return;
    if (l == p.lists) {
        p.list_start[l] = p.off[p.cbase[p.n]];  // = off[M], every entry
        return;
    }
    int64_t a = 0, b = p.n - 1;  // last record r with lbase[r] <= l
    while (a < b) {
        const int64_t m = (a + b + 1) >> 1;
        if (p.lbase[m] <= l) a = m; else b = m - 1;
    }
    p.list_start[l] = p.off[p.cbase[a] + (l - p.lbase[a]) * p.nwg[a]];
}

// K4: one workgroup per list.  Pass q of P counts the keys whose hash bits
// [32, 32 + log2 P) equal q; a pass whose keys overflow the table is split again.
__global__ __launch_bounds__(kCountBlock) void canon_table_kernel(HParams p) {
    __shared__ unsigned long long tk[kTableSlots];
    __shared__ uint32_t tc[kTableSlots];
    __shared__ uint32_t s_misc[4 + kCountBlock / 64];
    const int64_t l = blockIdx.x;
    const uint64_t beg = p.list_start[l], end = p.list_start[l + 1];
    const uint64_t n = end - beg;
    uint32_t P = 1;
    while ((uint64_t)P * kPassDistinct < n) P <<= 1;
    uint64_t out = beg;  // next free pair of this list's segment
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (uint32_t q = 0; q < P;) {
        for (int i = tid; i < kTableSlots; i += kCountBlock) {
            tk[i] = kEmpty;
            tc[i] = 0u;
        }
        if (tid == 0) s_misc[0] = 0u;  // overflow flag
        __syncthreads();
        const uint32_t lgP = 31 - __builtin_clz(P);
        // the list in batches of kBatch keys per thread: all loads of a batch are in
        // flight together (one HBM latency per batch, not per key)
        constexpr int kBatch = 8;
        for (uint64_t i0 = beg; i0 < end; i0 += (uint64_t)kBatch * kCountBlock) {
            unsigned long long kb[kBatch];
#pragma unroll
            for (int j = 0; j < kBatch; ++j) {
                const uint64_t i = i0 + (uint64_t)j * kCountBlock + tid;
                kb[j] = i < end ? p.ent[i] : kEmpty;
            }
#pragma unroll
            for (int j = 0; j < kBatch; ++j) {
                const unsigned long long key = kb[j];
                if (key == kEmpty) continue;
                const uint64_t h = fmix64(key);
                if (lgP && (uint32_t)((h >> 32) & (P - 1)) != q) continue;
                uint32_t s = (uint32_t)(((h & 0xFFFFFFFFull) * kTableSlots) >> 32);
                uint32_t probes = 0;
                for (;;) {
                    const unsigned long long cur = atomicCAS(&tk[s], kEmpty, key);
                    if (cur == kEmpty) break;  // claimed: first occurrence (tc holds occurrences - 1)
                    if (cur == key) {
                        __hip_atomic_fetch_add(&tc[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        break;
                    }
                    if (++probes == kTableSlots) {  // table full: this pass splits in two
                        s_misc[0] = 1u;
                        break;
                    }
                    s = s + 1 == (uint32_t)kTableSlots ? 0u : s + 1;
                }
            }
        }
        __syncthreads();
        if (s_misc[0]) {
            // restart with twice the passes (pass q -> passes 2q, 2q+1); the pairs of
            // the passes already written stay, since the pass split refines them
            __syncthreads();
            P <<= 1;
            q <<= 1;
            continue;
        }
        // compact the live slots to the list's segment, slot order
        constexpr int PER = kTableSlots / kCountBlock;
        uint32_t live = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) live += tk[tid * PER + j] != kEmpty;
        uint32_t x = live;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_misc[4 + wid] = x;
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (int i2 = 0; i2 < kCountBlock / 64; ++i2) {
            if (i2 < wid) before += s_misc[4 + i2];
            total += s_misc[4 + i2];
        }
        uint64_t o2 = out + before + x - live;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const unsigned long long key = tk[tid * PER + j];
            if (key != kEmpty) {
                p.pk[o2] = key;
                p.pc[o2] = tc[tid * PER + j] + 1u;
                ++o2;
            }
        }
        out += total;
        __syncthreads();
        ++q;
    }
    if (tid == 0) p.ndist[l] = (uint32_t)(out - beg);
}

// K5: pairs to their final place; record offsets
__global__ __launch_bounds__(256) void canon_place_kernel(HParams p) {
    const int64_t l = blockIdx.x;
    const uint64_t src = p.list_start[l], dst = p.dist_off[l], m = p.ndist[l];
    for (uint64_t i = threadIdx.x; i < m; i += 256) {
        p.out_keys[dst + i] = p.pk[src + i];
        p.out_counts[dst + i] = p.pc[src + i];
    }
}

__global__ void canon_recoff_kernel(HParams p) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r <= p.n) p.rec_off[r] = p.dist_off[p.lbase[r]];
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
    for (int64_t r = 0; r < n; ++r)
        if (hidx[r + 1] < hidx[r]) return KMC_ERR_INVALID_ARG;
    int device = 0, cus = 0;
    if ((he = hipGetDevice(&device)) || (he = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device)))
        return (int)he;
    // geometry of K1 / K3: G workgroups over the window chunks
    HParams p{};
    p.data = data;
    p.idx = indices;
    p.n = n;
    p.lo = hidx[0];
    p.hi = hidx[n];
    p.k = k;
    p.flags = flags;
    p.c_lo = p.lo >> 4;
    const int64_t chunks = p.hi > p.lo ? ((p.hi + 15) >> 4) - p.c_lo : 0;
    p.G = (int)std::max<int64_t>(1, std::min<int64_t>(cus, chunks));
    p.cpw = std::max<int64_t>(1, (chunks + p.G - 1) / p.G);
    // per record: lists, workgroups holding its windows, cnt layout, list ids
    std::vector<uint8_t> lg(n);
    std::vector<int32_t> w0(n), nwg(n);
    std::vector<int64_t> cbase(n + 1), lbase(n + 1);
    int64_t M = 0, L = 0, windows = 0;
    for (int64_t r = 0; r < n; ++r) {
        const int64_t a = hidx[r], nw = std::max<int64_t>(0, hidx[r + 1] - a - k);
        windows += nw;
        int g = 0;
        while (g < kMaxLg && ((int64_t)kListTarget << g) < nw) ++g;
        lg[r] = (uint8_t)g;
        if (nw > 0) {
            const int64_t cf = a >> 4, cl = (a + nw - 1) >> 4;
            w0[r] = (int32_t)((cf - p.c_lo) / p.cpw);
            nwg[r] = (int32_t)((cl - p.c_lo) / p.cpw) - w0[r] + 1;
        } else {
            w0[r] = 0;
            nwg[r] = 0;
        }
        cbase[r] = M;
        lbase[r] = L;
        M += ((int64_t)1 << g) * nwg[r];
        L += (int64_t)1 << g;
    }
    cbase[n] = M;
    lbase[n] = L;
    p.lists = L;
    const int64_t cap_w = std::max<int64_t>(windows, 1);
    // workspace
    size_t o = 0;
    const size_t o_lg = o; o += al256(n);
    const size_t o_cb = o; o += al256((n + 1) * 8);
    const size_t o_w0 = o; o += al256(n * 4);
    const size_t o_nw = o; o += al256(n * 4);
    const size_t o_lb = o; o += al256((n + 1) * 8);
    const size_t o_cnt = o; o += al256((size_t)std::max<int64_t>(M, 1) * 4);
    const size_t o_off = o; o += al256((size_t)(M + 1) * 8);
    const size_t o_bs = o; o += al256((size_t)(scan_tiles(std::max<int64_t>(M, L)) + 1) * 8);
    const size_t o_ent = o; o += al256((size_t)cap_w * 8);
    const size_t o_ls = o; o += al256((size_t)(L + 1) * 8);
    const size_t o_pk = o; o += al256((size_t)cap_w * 8);
    const size_t o_pc = o; o += al256((size_t)cap_w * 4);
    const size_t o_nd = o; o += al256((size_t)L * 4);
    const size_t o_do = o; o += al256((size_t)(L + 1) * 8);
    const size_t total = o;
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
    p.lg = reinterpret_cast<uint8_t *>(ws + o_lg);
    p.cbase = reinterpret_cast<int64_t *>(ws + o_cb);
    p.w0 = reinterpret_cast<int32_t *>(ws + o_w0);
    p.nwg = reinterpret_cast<int32_t *>(ws + o_nw);
    p.lbase = reinterpret_cast<int64_t *>(ws + o_lb);
    p.cnt = reinterpret_cast<uint32_t *>(ws + o_cnt);
    p.off = reinterpret_cast<uint64_t *>(ws + o_off);
    uint64_t *bsum = reinterpret_cast<uint64_t *>(ws + o_bs);
    p.ent = reinterpret_cast<uint64_t *>(ws + o_ent);
    p.list_start = reinterpret_cast<uint64_t *>(ws + o_ls);
    p.pk = reinterpret_cast<uint64_t *>(ws + o_pk);
    p.pc = reinterpret_cast<uint32_t *>(ws + o_pc);
    p.ndist = reinterpret_cast<uint32_t *>(ws + o_nd);
    p.dist_off = reinterpret_cast<uint64_t *>(ws + o_do);
    p.rec_off = rec_offsets;
    p.out_keys = keys;
    p.out_counts = counts;
    if ((he = hipMemcpyAsync((void *)p.lg, lg.data(), n, hipMemcpyHostToDevice, stream)) ||
        (he = hipMemcpyAsync((void *)p.cbase, cbase.data(), (n + 1) * 8, hipMemcpyHostToDevice, stream)) ||
        (he = hipMemcpyAsync((void *)p.w0, w0.data(), n * 4, hipMemcpyHostToDevice, stream)) ||
        (he = hipMemcpyAsync((void *)p.nwg, nwg.data(), n * 4, hipMemcpyHostToDevice, stream)) ||
        (he = hipMemcpyAsync((void *)p.lbase, lbase.data(), (n + 1) * 8, hipMemcpyHostToDevice, stream)))
        return (int)he;
    if (M > 0) {
        if ((he = hipMemsetAsync(p.cnt, 0, (size_t)M * 4, stream))) return (int)he;
        hipLaunchKernelGGL(canon_count_kernel, dim3(p.G), dim3(kWalkBlock), 0, stream, p);
    }
    excl_scan_u32(p.cnt, M, bsum, p.off, stream);
    hipLaunchKernelGGL(canon_scatter_kernel, dim3(p.G), dim3(kWalkBlock), 0, stream, p);
    hipLaunchKernelGGL(canon_list_start_kernel, dim3((unsigned)((L + 1 + 255) / 256)), dim3(256), 0, stream, p);
    hipLaunchKernelGGL(canon_table_kernel, dim3((unsigned)L), dim3(kCountBlock), 0, stream, p);
    excl_scan_u32(p.ndist, L, bsum, p.dist_off, stream);
    hipLaunchKernelGGL(canon_recoff_kernel, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, stream, p);
    uint64_t distinct = 0;
    if ((he = hipGetLastError()) ||
        (he = hipMemcpyAsync(&distinct, p.dist_off + L, 8, hipMemcpyDeviceToHost, stream)) ||
        (he = hipStreamSynchronize(stream)))
        return (int)he;
    *num_distinct = distinct;
    if (distinct > capacity) return KMC_ERR_CAPACITY;
    if (distinct && (!keys || !counts)) return KMC_ERR_INVALID_ARG;
    hipLaunchKernelGGL(canon_place_kernel, dim3((unsigned)L), dim3(256), 0, stream, p);
    if ((he = hipGetLastError()) || (he = hipStreamSynchronize(stream))) return (int)he;
    return KMC_OK;
}
