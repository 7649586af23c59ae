// kmc_radix.hip — dense k-mer histograms for 9 <= k <= KMC_DENSE_MAX_K (BASELINE
// config C3: k = 13, 67 M bins per record), whose 4^k bins cannot be privatised
// in LDS.  Same counting contract and output layout as kmc_dense.hip (the
// generalisation of permutationsCountAll, main.cu:636-646, in the GPU layout of
// kernels.h:142), computed by a two-level radix partition:
//
//   R1 count    every workgroup streams its tiles (kmc_stream.h) and counts, per
//               record piece, the windows of each bucket b = code >> 15 in LDS
//               -> cnt[(s*NBK + b)*G + w]
//   R2 scan     exclusive prefix sum -> 64-bit offsets: list (s, b) is contiguous,
//               workgroup segments inside it in w order
//   R3 scatter  the same traversal writes each window's low 15 code bits
//               (uint16) at its list position (LDS 64-bit cursors per bucket)
//   R4 hist     one workgroup per list: 32 768-bin LDS histogram of its entries ->
//               stage[s][b*32768 + c] (record-major, coalesced)
//   R5 place    transpose stage into sum[s + ld*code] (k-mer-major, coalesced)
//
// Bytes per k-mer: 1 (R1) + 1 (R3) input, 2 written + 2 read entries, plus the
// output twice; the LDS histograms see the same bank-conflict-bound atomic rate
// as the k <= 8 kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <vector>

#include "kmc.h"
#include "kmc_internal.h"
#include "kmc_scan.h"
#include "kmc_stream.h"

// Diagnostic builds only (scripts/kbench.py timing): 1 = no list stores, 2 = also
// non-returning bucket counts, 3 = staging without the flush.  Results are wrong.
#ifndef KMC_RSCAT_ABL
#define KMC_RSCAT_ABL 0
#endif
// tile prefetch depth of the scatter pass (register pressure: the round's windows
// stay in registers across the barrier)
#ifndef KMC_RSCAT_PF
#define KMC_RSCAT_PF 2
#endif
// tiles per wave in one R3 round (the round is counting-sorted in LDS: 64 KB of
// staging per tile and wave group)
#ifndef KMC_RSCAT_RT
#define KMC_RSCAT_RT 2
#endif
// write-out loop unroll (entries in flight per lane; register pressure)
#ifndef KMC_RSCAT_WU
#define KMC_RSCAT_WU 16
#endif

namespace kmc {
namespace {

// Low code bits resolved by the per-list LDS histogram (2^low bins, at most
// 128 KB); the rest select the bucket.  At least 64 buckets per record, so the
// bucket counters of R1/R3 see few same-address LDS atomics.
#ifndef KMC_RADIX_LOW_MAX
#define KMC_RADIX_LOW_MAX 16
#endif
// (16 low bits — two 16-bit R4 bins per LDS word — from k = 12 on: half the
// buckets, so R3's runs per bucket and round are twice as long; at k = 11 the
// 64 buckets per record would leave R4 too few workgroups)
__host__ __device__ constexpr int low_bits(int k) {
    return 2 * k - 6 < (k >= 12 ? KMC_RADIX_LOW_MAX : 15) ? 2 * k - 6 : (k >= 12 ? KMC_RADIX_LOW_MAX : 15);
}

struct RParams {
    const char *data;
    const void *indices;
    int64_t n;
    int64_t wl, wh, rl, rh;
    int derive;
    int G;           // workgroups of R1/R3
    int nbk;         // buckets per record
    int b_lo, b_hi;  // R3: buckets scattered by this launch
    uint32_t *cnt;   // [n][nbk][G]
    uint64_t *off;   // [n*nbk*G + 1] exclusive prefix of cnt
    uint16_t *ent;   // entries
    uint32_t *stage; // [n][4^k]
    int32_t *sum;
    int64_t ld;
    int32_t *invalid;
};

template <int K>
struct RCountOp {
    static constexpr int LOW = low_bits(K);
    uint32_t *c;  // LDS bucket counters
    __device__ void before_tile() {}
    template <bool MASKED>
    __device__ __forceinline__ void tile(uint32_t lo, uint32_t hi, uint32_t W) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t code = window_code_rt<K>(lo, hi, j);
            if (!MASKED || ((W >> j) & 1u))
                __hip_atomic_fetch_add(&c[code >> LOW], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __device__ void after_iter(int64_t, int64_t, bool) {}
};

// R3 op.  Scattering every window straight to its list costs one L2 write
// request per 2-byte entry (64 per wave store); instead each round of RT tiles
// per wave is counting-sorted by bucket in LDS and written out so that
// consecutive lanes store consecutive entries of one list.  A window's rank in
// its bucket is taken (returning LDS add) as the tile is decoded; the lane keeps
// only the tile's bases (lo, hi, valid mask) and the ranks, and recomputes the
// codes once the round's scan has placed the buckets.
//   srt  [NW*1024*RT] the round sorted by bucket
//   off  [NBK + 1]    bucket counts -> exclusive offsets within srt
//   gcur [NBK]        global position of each list's next entry (this workgroup)
//   gdel [NBK]        this round: global position of srt index 0 of each bucket's run
// Only buckets [b_lo, b_lo + b_n) are scattered (bucket-group launches).
template <int K, int NW, int RT>
struct RStageOp {
    static constexpr int LOW = low_bits(K);
    static constexpr int NBK = 1 << (2 * K - LOW);
    static constexpr int BATCH = NW * 1024 * RT;
    static_assert(BATCH <= 65536, "ranks are 16-bit");
    static constexpr uint32_t kNone = 0xFFFFFFFFu;
    uint32_t *srt, *off, *nw;
    unsigned long long *gcur;
    long long *gdel;
    uint16_t *ent;
    uint32_t b_lo, b_n;
    int wave, lane, tid;
    int slot;              // tiles of this round held (workgroup-uniform)
    uint32_t lo[RT], hi[RT], wm[RT];  // per held tile: bases and windows taken (0: none)
    uint32_t rank[RT][8];  // their ranks in their buckets, two 16-bit ranks per word (< BATCH)

    __device__ void before_tile() {}

    __device__ __forceinline__ bool take(uint32_t c, uint32_t W, int j) const {
        return ((W >> j) & 1u) && ((c >> LOW) - b_lo) < b_n;
    }

    template <int S>
    __device__ __forceinline__ void rank_tile(uint32_t l, uint32_t h, uint32_t W) {
        lo[S] = l;
        hi[S] = h;
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t c = window_code_rt<K>(l, h, j);
            const bool v = take(c, W, j);
            uint32_t r = 0;
            if (v) r = __hip_atomic_fetch_add(&off[(c >> LOW) - b_lo], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            m |= (uint32_t)v << j;
            if (j & 1) rank[S][j >> 1] |= r << 16;
            else rank[S][j >> 1] = r;
        }
        wm[S] = m;
    }

    template <bool MASKED>
    __device__ __forceinline__ void tile(uint32_t l, uint32_t h, uint32_t W) {
        if constexpr (RT == 1) {
            rank_tile<0>(l, h, W);
        } else {
            static_assert(RT == 2, "one or two tiles per round");
            if (slot == 0) rank_tile<0>(l, h, W);
            else rank_tile<1>(l, h, W);
        }
    }

    __device__ void after_iter(int64_t i, int64_t per, bool) {
        if (++slot < RT && i + 1 < per) return;  // round not full (i, per, slot: workgroup-uniform)
        slot = 0;
        lds_barrier();  // every rank taken
#if KMC_RSCAT_ABL == 3
#pragma unroll
        for (int S = 0; S < RT; ++S) wm[S] = 0u;
        lds_barrier();
        return;  // diagnostic: ranking only
#endif
        // exclusive scan of the bucket counts (off[b_n] = round total)
        block_scan_inplace(off, (int)b_n);
        // counting-sort the round into srt; per bucket, the global position of srt
        // index 0 (gdel = cursor - offset) and the advanced cursor
#pragma unroll
        for (int S = 0; S < RT; ++S) {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t c = window_code_rt<K>(lo[S], hi[S], j);
                if ((wm[S] >> j) & 1u)
                    srt[off[(c >> LOW) - b_lo] + ((rank[S][j >> 1] >> (16 * (j & 1))) & 0xFFFFu)] = c;
            }
            wm[S] = 0u;
        }
        for (uint32_t b = tid; b < b_n; b += NW * 64) {
            const uint32_t o0 = off[b], o1 = off[b + 1];
            const unsigned long long g = gcur[b];
            gdel[b] = (long long)g - (long long)o0;
            gcur[b] = g + (o1 - o0);
        }
        const uint32_t total = off[b_n];
        lds_barrier();
        // coalesced write-out: srt[i] is entry i + gdel[b] of bucket b's list; the
        // counts are cleared for the next round (nothing reads them until then)
        for (uint32_t b = tid; b <= b_n; b += NW * 64) off[b] = 0u;
#pragma unroll KMC_RSCAT_WU
        for (int q = 0; q < 16 * RT; ++q) {
            const uint32_t i = tid + q * NW * 64;
            if (i >= total) break;
            const uint32_t c = srt[i];
            const long long pos = gdel[(c >> LOW) - b_lo] + (long long)i;
#if KMC_RSCAT_ABL >= 1
            if (c == 0xFFFFFFFEu)  // diagnostic: never true, keeps the loads
#endif
            ent[pos] = (uint16_t)(c & ((1u << LOW) - 1));
        }
        lds_barrier();  // srt and the counts are free for the next round
    }

    // in-place exclusive scan of a[0..m) with a[m] = total; all NW*64 threads
    __device__ __forceinline__ void block_scan_inplace(uint32_t *a, int m) {
        constexpr int T = NW * 64;
        const int per = (m + T - 1) / T;  // consecutive elements per thread
        const int beg = tid * per;
        uint32_t loc = 0;
        for (int q = 0; q < per; ++q)
            if (beg + q < m) loc += a[beg + q];
        // wave inclusive scan of loc
        uint32_t x = loc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) nw[NW + wave] = x;  // wave totals after the per-wave counts
        lds_barrier();
        uint32_t wbase = 0;
        for (int w2 = 0; w2 < wave; ++w2) wbase += nw[NW + w2];
        uint32_t run = wbase + x - loc;
        lds_barrier();  // everyone has read its inputs before they are overwritten
        for (int q = 0; q < per; ++q) {
            if (beg + q < m) {
                const uint32_t v = a[beg + q];
                a[beg + q] = run;
                run += v;
            }
        }
        if (tid == T - 1) a[m] = run;
        lds_barrier();
    }
};

// R1 and R3: the piece walk of the dense kernel; SCATTER selects the op.  The
// scatter variant needs the whole 160 KB LDS (one workgroup per CU).
template <int K, class Idx, bool SCATTER, int BLOCK>
__global__ __launch_bounds__(BLOCK) void radix_pass_kernel(RParams p) {
    constexpr int NWAVES = BLOCK / 64;
    constexpr int NBK = 1 << (2 * K - low_bits(K));
    __shared__ __attribute__((aligned(16))) unsigned long long lds64[NBK];
    __shared__ int64_t s_first;
    uint32_t *lds32 = reinterpret_cast<uint32_t *>(lds64);
    constexpr int SB = SCATTER ? NWAVES * 1024 * KMC_RSCAT_RT : 1;
    __shared__ __attribute__((aligned(16))) uint32_t s_srt[SB];
    __shared__ uint32_t s_off[SCATTER ? NBK + 1 : 1];
    __shared__ long long s_gdel[SCATTER ? NBK : 1];
    __shared__ uint32_t s_nw[2 * NWAVES];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = blockIdx.x;
    const Geom g = make_geom<Idx>(p);
    const int64_t tb = g.T0 + (int64_t)w * g.tpw;
    const int64_t te = (tb + g.tpw) < g.T1 ? (tb + g.tpw) : g.T1;
    if (tb >= te) return;
    const int64_t R0 = (tb << kTileShift) > g.wl ? (tb << kTileShift) : g.wl;
    const int64_t R1 = (te << kTileShift) < g.wh ? (te << kTileShift) : g.wh;
    if (tid == 0) s_first = first_record_at<Idx>(p, R0);
    __syncthreads();
    for (int64_t s = s_first; s < p.n; ++s) {
        if (rec_off<Idx>(p, s) >= R1) break;
        int64_t ca, ce;
        record_windows<K, Idx>(p, g, s, ca, ce);
        const int64_t ps = ca > R0 ? ca : R0;
        const int64_t pe = ce < R1 ? ce : R1;
        if (ps >= pe) continue;
        const int64_t lbase = (s * NBK) * p.G + w;  // cnt/off index of (s, b=0, w); stride G per bucket
        for (int b = tid; b < NBK; b += BLOCK) {
            if (SCATTER) {
                if (b >= p.b_lo && b < p.b_hi) lds64[b - p.b_lo] = p.off[lbase + (int64_t)b * p.G];
            } else {
                lds32[b] = 0u;
            }
        }
        if (SCATTER)
            for (int b = tid; b <= NBK; b += BLOCK) s_off[b] = 0u;
        __syncthreads();
        const int64_t tp0 = ps >> kTileShift;
        const int64_t tp1 = ((pe - 1) >> kTileShift) + 1;
        const int64_t per = (tp1 - tp0 + NWAVES - 1) / NWAVES;
        const int64_t a0 = tp0 + (int64_t)wave * per;
        const int64_t a1 = (a0 + per) < tp1 ? (a0 + per) : tp1;
        if constexpr (SCATTER) {
            using Op = RStageOp<K, NWAVES, KMC_RSCAT_RT>;
            Op op{s_srt, s_off, s_nw, lds64, s_gdel, p.ent, (uint32_t)p.b_lo, (uint32_t)(p.b_hi - p.b_lo),
                  wave, lane, tid, 0, {}, {}, {}, {}};
#pragma unroll
            for (int S = 0; S < KMC_RSCAT_RT; ++S) op.wm[S] = 0u;
            stream_tiles<K, Op, KMC_RSCAT_PF>(p.data, a0, a1, per, ps, pe, g.rl, g.rh, lane, op);
        } else {
            RCountOp<K> op{lds32};
            stream_tiles<K>(p.data, a0, a1, per, ps, pe, g.rl, g.rh, lane, op);
        }
        __syncthreads();
        if constexpr (!SCATTER) {
            for (int b = tid; b < NBK; b += BLOCK) p.cnt[lbase + (int64_t)b * p.G] = lds32[b];
        }
        __syncthreads();
    }
}


// R4: one workgroup per list (s, b).
template <int LOW>
__device__ __forceinline__ void hist_add(uint32_t *h, uint32_t e) {
    if constexpr (LOW <= 15) {
        __hip_atomic_fetch_add(&h[e], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {  // two 16-bit bins per word
        __hip_atomic_fetch_add(&h[e >> 1], (e & 1u) ? 0x10000u : 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// The entries [beg, end) of one list into h (hist_add<LOW>); entries whose top
// bit differs from `half` are skipped when HALF (the 32-bit recount of LOW = 16).
template <int LOW, bool HALF>
__device__ __forceinline__ void hist_list(const uint16_t *ent, uint64_t beg, uint64_t end, uint32_t *h, uint32_t half) {
    const auto add = [&](uint32_t e) {
        if constexpr (HALF) {
            if ((e >> 15) == half) __hip_atomic_fetch_add(&h[e & 0x7FFFu], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            hist_add<LOW>(h, e);
        }
    };
    // head up to 8-entry alignment, 16-B vector body, tail
    uint64_t a = beg;
    const uint64_t abody = (beg + 7) & ~(uint64_t)7;
    if (a + threadIdx.x < (abody < end ? abody : end)) add(ent[a + threadIdx.x]);
    a = abody;
    if (a < end) {
        const uint64_t nvec = (end - a) / 8;
        const uint4 *v = reinterpret_cast<const uint4 *>(ent + a);
        for (uint64_t i = threadIdx.x; i < nvec; i += 1024) {
            const uint4 x = v[i];
            const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                add(w[q] & 0xFFFFu);
                add(w[q] >> 16);
            }
        }
        const uint64_t t = a + nvec * 8;
        if (t + threadIdx.x < end) add(ent[t + threadIdx.x]);
    }
}

// R4: one workgroup per list (s, b): 2^LOW-bin LDS histogram -> stage.  LOW = 16
// packs two 16-bit bins per word (128 KB); a bin that reaches 65 536 within the
// list wraps, which lowers the sum of the bins below the list length (a carry
// into the neighbour costs 65 535, one out of the word 65 536), and the list is
// then recounted exactly in two 32 768-bin halves.
template <int LOW>
__global__ __launch_bounds__(1024) void radix_hist_kernel(RParams p, int64_t nbins) {
    constexpr int kBucketBins = 1 << LOW;
    constexpr int kWords = LOW <= 15 ? kBucketBins : kBucketBins / 2;
    __shared__ __attribute__((aligned(16))) uint32_t h[kWords];
    __shared__ unsigned long long s_sum;
    const int64_t nlists = p.n * p.nbk;
    for (int64_t list = blockIdx.x; list < nlists; list += gridDim.x) {  // list = s*nbk + b
        const int64_t s = list / p.nbk, b = list % p.nbk;
        for (int i = threadIdx.x; i < kWords; i += 1024) h[i] = 0u;
        if (threadIdx.x == 0) s_sum = 0ull;
        __syncthreads();
        const uint64_t beg = p.off[list * p.G], end = p.off[(list + 1) * p.G];
        hist_list<LOW, false>(p.ent, beg, end, h, 0u);
        __syncthreads();
        uint32_t *dst = p.stage + s * nbins + b * kBucketBins;
        if constexpr (LOW <= 15) {
            for (int i = threadIdx.x; i < kBucketBins; i += 1024) dst[i] = h[i];
        } else {
            uint32_t part = 0u;
            for (int i = threadIdx.x; i < kWords; i += 1024) part += (h[i] & 0xFFFFu) + (h[i] >> 16);
            atomicAdd(&s_sum, (unsigned long long)part);
            __syncthreads();
            if (s_sum == end - beg) {
                for (int i = threadIdx.x; i < kWords; i += 1024) {
                    const uint32_t w = h[i];
                    reinterpret_cast<uint2 *>(dst)[i] = make_uint2(w & 0xFFFFu, w >> 16);
                }
            } else {  // a bin wrapped: exact recount, half of the bins at a time
                for (uint32_t half = 0; half < 2; ++half) {
                    __syncthreads();
                    for (int i = threadIdx.x; i < kWords; i += 1024) h[i] = 0u;
                    __syncthreads();
                    hist_list<LOW, true>(p.ent, beg, end, h, half);
                    __syncthreads();
                    for (int i = threadIdx.x; i < kWords; i += 1024) dst[half * kWords + i] = h[i];
                }
            }
        }
        __syncthreads();  // h and s_sum are reused by the next list
    }
}

// R5: stage [n][nbins] -> sum[s + ld*code]; one workgroup per 256 codes.
__global__ __launch_bounds__(256) void radix_place_kernel(RParams p, int64_t nbins) {
    const int64_t c0 = (int64_t)blockIdx.x * 256;
    const int64_t total = 256 * p.n;  // outputs of this block: codes c0..c0+255, all records
    for (int64_t i = threadIdx.x; i < total; i += 256) {
        const int64_t c = c0 + i / p.n, s = i % p.n;  // consecutive threads -> consecutive records
        if (c < nbins) p.sum[s + p.ld * c] = (int32_t)p.stage[s * nbins + c];
    }
}

// invalid[s] = windows in range - sum of the record's bucket counts; records
// blockIdx.x, blockIdx.x + gridDim.x, ...
template <int K, class Idx>
__global__ __launch_bounds__(256) void radix_invalid_kernel(RParams p) {
    const int64_t m = (int64_t)p.nbk * p.G;
    __shared__ uint64_t red[256];
    for (int64_t s = blockIdx.x; s < p.n; s += gridDim.x) {
        uint64_t acc = 0;
        for (int64_t i = threadIdx.x; i < m; i += 256) acc += p.cnt[s * m + i];
        red[threadIdx.x] = acc;
        __syncthreads();
        for (int st = 128; st > 0; st >>= 1) {
            if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            const Geom g = make_geom<Idx>(p);
            int64_t ca, ce;
            record_windows<K, Idx>(p, g, s, ca, ce);
            const int64_t nw = ce > ca ? ce - ca : 0;
            p.invalid[s] = (int32_t)(nw - (int64_t)red[0]);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
constexpr int kPassBlock = 1024;
// target footprint of the list lines one R3 launch keeps open (G x buckets x 128 B)
#ifndef KMC_OPEN_LIST_MB
#define KMC_OPEN_LIST_MB 64
#endif
constexpr size_t kOpenListBytes = (size_t)KMC_OPEN_LIST_MB << 20;

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct RLayout {
    size_t cnt, off, bsum, ent, stage, total;
    int64_t m, nscan;
};

inline RLayout r_layout(int k, int64_t n, int G, int64_t ent_cap) {
    RLayout L;
    const int64_t nbk = (int64_t)1 << (2 * k - low_bits(k));
    L.m = n * nbk * G;
    L.nscan = (L.m + kScanTile - 1) / kScanTile;
    size_t o = 0;
    L.cnt = o;
    o += al256((size_t)L.m * 4);
    L.off = o;
    o += al256((size_t)(L.m + 1) * 8);
    L.bsum = o;
    o += al256((size_t)(L.nscan + 1) * 8);
    L.ent = o;
    o += al256((size_t)ent_cap * 2 + 16);
    L.stage = o;
    o += al256((size_t)n * ((size_t)1 << (2 * k)) * 4);
    L.total = o;
    return L;
}

std::mutex r_mu;
std::vector<int> r_cus;  // CUs per device

int r_grid(int device, int &G) {
    std::lock_guard<std::mutex> lk(r_mu);
    if ((int)r_cus.size() <= device) r_cus.resize(device + 1, 0);
    if (r_cus[device] == 0) {
        int v = 0;
        hipError_t e = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device);
        if (e != hipSuccess) return (int)e;
        r_cus[device] = v;
    }
    G = r_cus[device];  // one 16-wave workgroup per CU: fewer open lists than more, smaller groups
    return 0;
}

struct RCache {
    void *ptr = nullptr;
    size_t bytes = 0;
};
std::vector<RCache> r_ws;

template <int K>
int run_radix(const kmc_dense_args *a, hipStream_t st, bool size_only, size_t *size_out) {
    int device = 0;
    hipError_t he = hipGetDevice(&device);
    if (he != hipSuccess) return (int)he;
    int G = 0;
    int e = r_grid(device, G);
    if (e) return e;
    const int64_t wl = (int64_t)a->win_lo, wh = (int64_t)a->win_hi;
    const int64_t tiles = wh > wl ? ((wh + kTile - 1) >> kTileShift) - (wl >> kTileShift) : 0;
    if (tiles < G) G = tiles > 0 ? (int)tiles : 1;
    const int64_t n = (int64_t)a->num_seqs;
    const int64_t ent_cap = wh > wl ? wh - wl : 0;  // >= valid windows in range
    const RLayout L = r_layout(K, n, G, ent_cap);
    if (size_only) {
        *size_out = L.total;
        return 0;
    }
    void *ws = a->workspace;
    if (ws == nullptr) {
        std::lock_guard<std::mutex> lk(r_mu);
        if ((int)r_ws.size() <= device) r_ws.resize(device + 1);
        RCache &c = r_ws[device];
        if (c.bytes < L.total) {
            if (c.ptr) {
                he = hipFree(c.ptr);
                if (he != hipSuccess) return (int)he;
            }
            c.ptr = nullptr;
            c.bytes = 0;
            if (hipMalloc(&c.ptr, L.total) != hipSuccess) return KMC_ERR_NOMEM;
            c.bytes = L.total;
        }
        ws = c.ptr;
    } else if (a->workspace_bytes < L.total) {
        return KMC_ERR_WORKSPACE;
    }
    char *base = static_cast<char *>(ws);
    RParams p;
    p.data = a->data;
    p.indices = a->indices;
    p.n = n;
    p.wl = wl;
    p.wh = wh;
    p.rl = (int64_t)a->read_lo;
    p.rh = (int64_t)a->read_hi;
    p.derive = 0;
    p.G = G;
    p.nbk = 1 << (2 * K - low_bits(K));
    p.b_lo = 0;
    p.b_hi = p.nbk;
    p.cnt = reinterpret_cast<uint32_t *>(base + L.cnt);
    p.off = reinterpret_cast<uint64_t *>(base + L.off);
    p.ent = reinterpret_cast<uint16_t *>(base + L.ent);
    p.stage = reinterpret_cast<uint32_t *>(base + L.stage);
    p.sum = a->sum;
    p.ld = a->sum_ld ? (int64_t)a->sum_ld : n;
    p.invalid = a->invalid;
    uint64_t *bsum = reinterpret_cast<uint64_t *>(base + L.bsum);
    const int64_t nbins = (int64_t)1 << (2 * K);

    if (t_trace_before) {
        he = hipEventRecord(t_trace_before, st);
        if (he != hipSuccess) return (int)he;
    }
    he = hipMemsetAsync(p.cnt, 0, (size_t)L.m * 4, st);
    if (he != hipSuccess) return (int)he;
    hipLaunchKernelGGL((radix_pass_kernel<K, int64_t, false, kPassBlock>), dim3(G), dim3(kPassBlock), 0, st, p);
    excl_scan_u32(p.cnt, L.m, bsum, p.off, st);
    // R3 in bucket groups whose open lines (G x buckets x 128 B) fit kOpenListBytes
    int groups = 1;
    while ((size_t)G * (size_t)(p.nbk / groups) * 128 > kOpenListBytes && groups < p.nbk) groups *= 2;
    for (int gi = 0; gi < groups; ++gi) {
        p.b_lo = gi * (p.nbk / groups);
        p.b_hi = p.b_lo + p.nbk / groups;
        hipLaunchKernelGGL((radix_pass_kernel<K, int64_t, true, kPassBlock>), dim3(G), dim3(kPassBlock), 0, st, p);
    }
    hipLaunchKernelGGL((radix_hist_kernel<low_bits(K)>), dim3((unsigned)std::min<int64_t>(n * p.nbk, kMaxGridX)),
                       dim3(1024), 0, st, p, nbins);
    hipLaunchKernelGGL(radix_place_kernel, dim3((unsigned)((nbins + 255) / 256)), dim3(256), 0, st, p, nbins);
    if (t_trace_after) {
        he = hipEventRecord(t_trace_after, st);
        if (he != hipSuccess) return (int)he;
    }
    if (a->invalid)
        hipLaunchKernelGGL((radix_invalid_kernel<K, int64_t>), dim3((unsigned)std::min<int64_t>(n, kMaxGridX)),
                           dim3(256), 0, st, p);
    he = hipGetLastError();
    return (int)he;
}

}  // namespace

// Entry used by kmc_dense.hip for 9 <= k <= KMC_DENSE_MAX_K.
int radix_dense(const kmc_dense_args *a, hipStream_t st, bool size_only, size_t *size_out) {
    switch (a->k) {
        case 9: return run_radix<9>(a, st, size_only, size_out);
        case 10: return run_radix<10>(a, st, size_only, size_out);
        case 11: return run_radix<11>(a, st, size_only, size_out);
        case 12: return run_radix<12>(a, st, size_only, size_out);
        case 13: return run_radix<13>(a, st, size_only, size_out);
        default: return KMC_ERR_UNSUPPORTED_K;
    }
}

}  // namespace kmc
