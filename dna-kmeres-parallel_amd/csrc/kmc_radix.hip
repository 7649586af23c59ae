// kmc_radix.hip — dense k-mer histograms for 9 <= k <= KMC_DENSE_MAX_K (BASELINE
// config C3: k = 13, 67 M bins per record), whose 4^k bins cannot be privatised
// in LDS.  Same counting contract and output layout as kmc_dense.hip (the
// generalisation of permutationsCountAll, main.cu:636-646, in the GPU layout of
// kernels.h:142), computed by a two-level radix partition:
//
//   R1 count    every workgroup streams its tiles (kmc_stream.h) and counts, per
//               record piece, the windows of each bucket b = code >> LOW in LDS
//               -> cnt[(s*NBK + b)*G + w]
//   R2 scan     exclusive prefix sum -> 64-bit offsets: list (s, b) is contiguous,
//               workgroup segments inside it in w order
//   R3 scatter  the same traversal appends each window's low LOW code bits
//               (uint16) to its bucket's LDS ring and writes complete 64-byte
//               list segments (radix_ring_kernel)
//   R4 hist     one workgroup per list: 2^LOW-bin LDS histogram of its entries ->
//               stage[s][b*2^LOW + c] (record-major, coalesced)
//   R5 place    transpose stage into sum[s + ld*code] (k-mer-major, coalesced)
//
// Sampled mode (large inputs: >= 4096 windows per (record, bucket, workgroup) on
// average, e.g. C3): R1's full read of the input is replaced by a 1-in-16 tile sample
// (S1, the same kernel with sample_tiles) whose weighted counts size one region
// per (s, b, w) with a margin (radix_cap_kernel); R2 scans the capacities, R3
// writes into the regions and records each one's fill in cnt, R4 walks a list as
// its G regions.  A region that overflows (or capacities beyond the entry array)
// raises a flag, and the exact R1 + R2 + R3, launched behind it and gated on it,
// rerun on the device -- no host sync, exact either way.
//
// LOW = min(2k - 6, 15), 16 from k = 12 on (low_bits).  Bytes per k-mer: 1 (R1;
// 1/8 sampled) + 1 (R3) input, 2 written + 2 read entries, plus the output twice;
// the LDS histograms see the same bank-conflict-bound atomic rate as the k <= 8
// kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <mutex>
#include <vector>

#include "kmc.h"
#include "kmc_internal.h"
#include "kmc_scan.h"
#include "kmc_stream.h"

namespace kmc {
namespace {

// Tile prefetch depth and nt loads of the count (R1) and scatter (R3) walks, each
// from a same-box A/B: R1 PF 3 + nt 2.04-2.06 -> 1.95-2.01 ms; R3 PF 2-4 equal, and
// nt loads made it slower.
constexpr int kRScatPF = 2, kRCountPF = 3, kRCountNT = 1;
// R4: 16-byte entry loads in flight per lane (2 / 4 / 8 measured equal, same box)
constexpr int kR4U = 4;

// Low code bits resolved by the per-list LDS histogram (2^low bins, at most
// 128 KB); the rest select the bucket.  At least 64 buckets per record, so the
// bucket counters of R1/R3 see few same-address LDS atomics.  16 low bits -- two
// 16-bit R4 bins per LDS word -- from k = 12 on: half the buckets, so R3's runs
// per bucket and round are twice as long; at k = 11 the 64 buckets per record
// would leave R4 too few workgroups.
__host__ __device__ constexpr int low_bits(int k) {
    return 2 * k - 6 < (k >= 12 ? 16 : 15) ? 2 * k - 6 : (k >= 12 ? 16 : 15);
}

struct RParams {
    const char *data;        // 16-byte aligned
    const void *indices;
    int64_t ibias;           // added to every indices[] value (kmc_stream.h rec_off)
    int64_t n;
    int64_t wl, wh, rl, rh;
    int derive;
    int G;           // workgroups of R1/R3
    int nbk;         // buckets per record
    uint32_t *cnt;   // [n][nbk][G] entries of list (s, b) from workgroup w
    uint64_t *off;   // [n*nbk*G + 1] start of each (s, b, w) region of ent
    uint16_t *ent;   // entries
    uint32_t *stage; // [n][4^k]
    int32_t *sum;
    int64_t ld;
    int32_t *invalid;
    // sampled mode (radix_count_kernel<SAMPLE>): regions sized from a 1-in-16 tile sample
    uint32_t *capv;      // [n][nbk][G] region capacities (multiples of 32); null: exact offsets
    uint32_t *flag;      // overflow lists full (or capacities beyond ent_cap): exact rerun
    const uint32_t *gate;  // non-null: the kernel runs only if *gate != 0 (the exact rerun)
    uint64_t ent_cap;    // entries ent holds
    unsigned long long *ovf;  // [G][ovf_cap] entries past their region, as stage indices
    uint32_t *ovf_cnt;   // [G]
    uint32_t ovf_cap;
    float cap_scale;     // test hook: capacities scaled (< 1 forces overflows)
    uint32_t *status;    // the call's status word (kmc_dense_args::status, set by kmc_count_dense_ex)
};

// A launch of the exact rerun returns at once unless the sampled pass overflowed.
__device__ __forceinline__ bool gated_off(const RParams &p) {
    return p.gate != nullptr && __hip_atomic_load(p.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
}

// R1 op: bucket counters with kCountRep replicas interleaved (counter b of lane l
// at word b*kCountRep + l % kCountRep), so the 32 lanes of an LDS lane group
// always hit 32 different banks (1 024 buckets x 32 replicas = 128 KB at k = 13).
constexpr int kCountRep = 32;
template <int K>
struct RCountOp {
    static constexpr int LOW = low_bits(K);
    uint32_t *c;  // LDS bucket counters (this lane's replica)
    uint32_t wgt;  // added per window (the sampled walk: its tile stride)
    __device__ void before_tile() {}
    template <bool MASKED>
    __device__ __forceinline__ void tile(uint32_t lo, uint32_t hi, uint32_t W) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t code = window_code_rt<K>(lo, hi, j);
            if (!MASKED || ((W >> j) & 1u))
                __hip_atomic_fetch_add(&c[(code >> LOW) * kCountRep], wgt, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __device__ void after_iter(int64_t, int64_t, bool) {}
};

// The sampled walk of a wave run [a0, a1): one tile in kSampleStride (a pseudo-random
// phase per run; every tile of runs up to kSampleAll tiles), each window counted
// with weight = the stride, kSampleFlight tiles in flight.  A sampled tile has no next tile:
// the windows of lane 63 that need its halo are skipped (1.2 % of them at k = 13),
// which the capacities' margin covers.
constexpr int kSampleStride = 16, kSampleAll = 16, kSampleFlight = 8;
constexpr int kSampleLog = __builtin_ctz(kSampleStride);
static_assert((kSampleStride & (kSampleStride - 1)) == 0, "the phase takes log2(stride) hash bits");
template <int K, class Op>
__device__ __forceinline__ void sample_tiles(const char *__restrict__ data, int64_t a0, int64_t a1, int64_t ps,
                                             int64_t pe, int64_t rl, int64_t rh, int lane, uint32_t seed, Op &op) {
    const int64_t len = a1 - a0;
    if (len <= 0) return;
    const int stride = len <= kSampleAll ? 1 : kSampleStride;
    op.wgt = (uint32_t)stride;
    const int64_t phase = stride == 1 ? 0 : (int64_t)((seed * 0x9E3779B1u) >> (32 - kSampleLog));
    for (int64_t t = a0 + phase; t < a1; t += kSampleFlight * stride) {
        uint4 r[kSampleFlight];
#pragma unroll
        for (int u = 0; u < kSampleFlight; ++u) {
            const int64_t tt = t + (int64_t)u * stride;
            r[u] = tt < a1 ? load_lane(data, tt, lane, rl, rh) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < kSampleFlight; ++u) {
            const int64_t tt = t + (int64_t)u * stride;
            if (tt >= a1) break;  // wave-uniform
            uint32_t code, bad;
            decode16(r[u], code, bad);
            const uint32_t hc = from_next_lane(code);
            const uint32_t b_own = bad_mask16(r[u]);
            uint32_t b_next = from_next_lane(b_own);
            if (lane == 63) b_next = 0xFFFFu;  // no halo: its windows across the tile end are skipped
            const int64_t pos = (tt << kTileShift) + (int64_t)lane * 16;
            const int64_t dlo = ps - pos, dhi = pe - pos;
            const uint32_t mhi = dhi >= 16 ? 0xFFFFu : (dhi <= 0 ? 0u : ((1u << (uint32_t)dhi) - 1u));
            const uint32_t mlo = dlo <= 0 ? 0xFFFFu : (dlo >= 16 ? 0u : ((0xFFFFu << (uint32_t)dlo) & 0xFFFFu));
            const uint32_t W = ~smear<K>(b_own | (b_next << 16)) & mhi & mlo & 0xFFFFu;
            op.template tile<true>(code, hc, W);
        }
    }
}

// R1: the piece walk of the dense kernel, counting per record piece the windows
// of each bucket in LDS -> cnt[(s*NBK + b)*G + w].  SAMPLE: the sampled walk
// (sample_tiles), whose weighted counts estimate the same numbers.
template <int K, class Idx, bool SAMPLE = false>
__global__ __launch_bounds__(1024) void radix_count_kernel(RParams p) {
    constexpr int BLOCK = 1024;
    constexpr int NWAVES = BLOCK / 64;
    constexpr int NBK = 1 << (2 * K - low_bits(K));
    __shared__ uint32_t s_cnt[NBK * kCountRep];
    __shared__ int64_t s_first;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = blockIdx.x;
    if (gated_off(p)) return;
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
        const int64_t lbase = (s * NBK) * p.G + w;  // cnt index of (s, b=0, w); stride G per bucket
        for (int i = tid; i < NBK * kCountRep; i += BLOCK) s_cnt[i] = 0u;
        __syncthreads();
        const int64_t tp0 = ps >> kTileShift;
        const int64_t tp1 = ((pe - 1) >> kTileShift) + 1;
        const int64_t per = (tp1 - tp0 + NWAVES - 1) / NWAVES;
        const int64_t a0 = tp0 + (int64_t)wave * per;
        const int64_t a1 = (a0 + per) < tp1 ? (a0 + per) : tp1;
        RCountOp<K> op{s_cnt + (lane & (kCountRep - 1)), 1u};
        if constexpr (SAMPLE) {
            sample_tiles<K>(p.data, a0, a1, ps, pe, g.rl, g.rh, lane, (uint32_t)(w * 16 + wave) ^ (uint32_t)s, op);
        } else {
            stream_tiles<K, RCountOp<K>, kRCountPF, kRCountNT>(p.data, a0, a1, per, ps, pe, g.rl, g.rh, lane, op);
        }
        __syncthreads();
        for (int b = tid; b < NBK; b += BLOCK) {
            const uint4 *r4 = reinterpret_cast<const uint4 *>(s_cnt + b * kCountRep);
            uint32_t t = 0u;
#pragma unroll
            for (int q = 0; q < kCountRep / 4; ++q) {
                const uint4 v = r4[(q + b) & (kCountRep / 4 - 1)];  // rotated: spread the banks
                t += v.x + v.y + v.z + v.w;
            }
            p.cnt[lbase + (int64_t)b * p.G] = t;
        }
        __syncthreads();
    }
}

// Sampled mode: the region capacity of every (s, b, w) from the weighted sample
// count c (an estimate of the region's entries): 1.05 c + 6 sigma + 64, sigma =
// sqrt(16 c) the Poisson error of a 1-in-16 sample, rounded up to 32 entries (whole
// 64-byte segments: regions stay segment-aligned) and at most the piece's windows;
// 0 where workgroup w holds no piece of record s (whatever cnt held there).  Clears
// cnt: R3 writes the fills, an exact rerun's R1 the counts.
template <int K, class Idx>
__global__ __launch_bounds__(256) void radix_cap_kernel(RParams p) {
    const int64_t m = p.n * p.nbk * p.G;
    const Geom g = make_geom<Idx>(p);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (int64_t)gridDim.x * 256) {
        const int64_t w = i % p.G, s = i / ((int64_t)p.nbk * p.G);
        const int64_t tb = g.T0 + w * g.tpw;
        const int64_t te = (tb + g.tpw) < g.T1 ? (tb + g.tpw) : g.T1;
        int64_t ca, ce;
        record_windows<K, Idx>(p, g, s, ca, ce);
        const int64_t R0 = (tb << kTileShift) > g.wl ? (tb << kTileShift) : g.wl;
        const int64_t R1 = (te << kTileShift) < g.wh ? (te << kTileShift) : g.wh;
        const int64_t ps = ca > R0 ? ca : R0, pe = ce < R1 ? ce : R1;
        uint32_t cap = 0u;
        if (tb < te && ps < pe) {
            const float c = (float)p.cnt[i];
            const float x = (1.05f * c + 6.0f * sqrtf((float)kSampleStride * c) + 64.0f) * p.cap_scale;
            const int64_t pmax = (pe - ps + 31) & ~(int64_t)31;
            cap = x >= (float)pmax ? (uint32_t)pmax : (((uint32_t)x + 31u) & ~31u);
        }
        p.capv[i] = cap;
        p.cnt[i] = 0u;
    }
}

// R3: every window's low code bits go to its list (s, bucket) through a ring of
// RING uint16 entries per bucket in LDS; whenever a 64-byte-aligned segment of the
// list (32 entries) is complete in a ring it is written out whole.  Each round is
// one tile per wave (16 K windows):
//   A  per valid window one returning LDS add of 2 on its bucket's word W[b], which
//      holds (halfword index of the bucket's ring | its swizzle) << 16 | 2 * (fill
//      of the ring: the carried partial segment + windows ranked so far).  The
//      returned value o gives the entry's LDS byte address in two VALU ops,
//      (o >> 15) ^ (o & (2 RING - 1)), and whether it fits in one 16-bit compare
//      (low half < 2 RING).  The ds_write_b16 is unconditional (windows that are
//      invalid or do not fit write a per-lane dummy word); entries that do not fit
//      go straight to their list position in a cold path (uncoalesced 2-byte
//      stores; skewed input only);
//   B  after a barrier, the TPB threads of bucket b (all keeping the bucket's state
//      in registers: F = list index of its next entry, V = first index still to be
//      written from the ring) write its complete segments (4 ds_read_b128 + 4
//      global 16-byte stores each), thread 0 of the group moves the partial last
//      segment to the ring's start (at most 4 b128 copies) and sets up the other W
//      buffer (W alternates per round, so the reset needs no third barrier).
// Between flushes list position g of bucket b lives in ring slot (g - H) ^ swz(b),
// H = the start of the round's first (partial) segment: the ring never wraps, and
// the per-bucket XOR swizzle (a multiple of 8 slots) spreads the phase-B 16-byte
// reads of neighbouring buckets over the banks; the TPB threads of one bucket read
// their segments' chunks in rotated order for the same reason.  Positions below V
// (before this workgroup's segment of the list, or already stored directly) are
// never written from the ring.  At the end of a piece the partial segment left in
// a ring is written entry by entry.
// Per window: 1 returning LDS atomic + 1 ds_write_b16 + 4 VALU ops (the staged
// counting sort this replaces needed 4 LDS accesses, a block scan and 5 barriers
// per round), and every global write is a whole 64-byte segment except at list
// ends.
template <int K>
struct RingGeom {
    static constexpr int LOW = low_bits(K);
    static constexpr int NBK = 1 << (2 * K - LOW);
    static constexpr int BLOCK = 1024;
    static constexpr int TPB = BLOCK / NBK;     // threads per bucket in phase B
    static constexpr int RING = 65536 / NBK;    // entries per bucket ring (128 KB in all)
    static_assert(NBK <= BLOCK && RING >= 64 && (RING & (RING - 1)) == 0, "ring geometry");
    // the fill (in bytes) of one round stays below 2^16: it cannot carry into the ring field
    static_assert(2 * (BLOCK * 16 + 32) < 65536, "one tile per wave per round");
};

// slot swizzle of bucket b (XOR mask, a multiple of 8 slots below 64)
__device__ __forceinline__ uint32_t ring_swz(uint32_t b) { return ((b >> 1) & 7u) * 8u; }

// W word of bucket b for a round whose first entry goes to ring slot f0 (< 32)
template <int K>
__device__ __forceinline__ uint32_t ring_word(uint32_t b, uint32_t f0) {
    return ((b * (uint32_t)RingGeom<K>::RING | ring_swz(b)) << 16) | (f0 << 1);
}

// circular ring (RING = 64, k = 13): list index g in slot (g mod 64) ^ swz, so the
// partial last segment stays in place (no tail move in the flush; the other
// geometries rebase the ring every round, the partial segment copied to its
// start).  Round 4, same box (profiles/r04b_r3_variants.txt): R3 8.78-8.83 ->
// 8.34-8.40 ms, C3 14.59-14.65 -> 14.14-14.18 ms.  (Reading a segment's chunks
// only when the quad stores one, instead of unconditionally, made R3 24 ms: the
// flush is latency-bound, and the predicated reads serialised it.)
// The round's entries start at list index
// f (relative to the piece's 32-aligned base); its first segment h = f & ~31 lives
// in ring half (h & 32), which is folded into the swizzle: with x = (f & 31) + rank
// < 64, (h + x) mod 64 = x ^ (h & 32)
template <int K>
__device__ __forceinline__ uint32_t ring_word_circ(uint32_t b, uint32_t f) {
    return ((b * (uint32_t)RingGeom<K>::RING | (ring_swz(b) ^ (f & 32u))) << 16) | ((f & 31u) << 1);
}
template <int K>
constexpr bool ring_circ() { return RingGeom<K>::RING == 64; }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

// SAMPLED: regions with capacities and overflow lists (radix_count_kernel<SAMPLE>);
// otherwise exact offsets, and none of that code.
template <int K, bool SAMPLED>
struct RRingOp {
    using RG = RingGeom<K>;
    uint16_t *ring;        // LDS, NBK * RING entries
    uint32_t *W;           // LDS, [2][NBK]
    unsigned long long *gH;  // LDS, [NBK]: list index of every bucket's ring slot 0 this round
    unsigned long long *lim;  // LDS, [NBK]: end of the bucket's region (sampled mode; else ~0)
    uint16_t *dummy;       // LDS, 2 halfwords per lane
    uint16_t *ent;
    int tid, lane;
    uint32_t par;          // W buffer of this round
    // phase-B state of bucket tid / TPB (replicated over its TPB threads), list
    // indices relative to P0 = this piece's first list index rounded down to 32:
    // f = next entry, v = first entry still to be written from the ring
    unsigned long long P0;
    uint32_t f, v;
    uint32_t f0;           // f at the piece start (the piece's entries: f - f0)
    uint32_t cap;          // end of the region (relative to P0; ~0: exact offsets)
    // sampled mode: this workgroup's overflow list and its LDS counter; stage index
    // of the piece's record
    unsigned long long *ovf;
    uint32_t *ovf_n;
    uint32_t ovf_cap;
    unsigned long long sbase;

    __device__ void before_tile() {}

    // an entry e of bucket b past its region -> the overflow list (added into stage
    // by radix_overflow_kernel after R4; a full list raises the exact rerun).  (Out
    // of line, this and ovf_seg made R3 5 % slower: calls, a stack, spills.)
    __device__ __forceinline__ void ovf_put(uint32_t b, uint32_t e) const {
        const uint32_t i = atomicAdd(ovf_n, 1u);
        if (i < ovf_cap) ovf[i] = sbase + ((unsigned long long)b << RG::LOW) + e;
    }
    // this lane's 8 entries (x) of a complete segment past its region, whose ring
    // LDS address is a & ~63
    __device__ __forceinline__ void ovf_seg(uint32_t a, uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) const {
        const uint32_t bt = ((a & ~63u) - (uint32_t)(uintptr_t)ring) / (2u * RG::RING);
        const uint32_t i8 = atomicAdd(ovf_n, 8u);
        const uint32_t w4[4] = {x0, x1, x2, x3};
        for (uint32_t e = 0; e < 8; ++e)
            if (i8 + e < ovf_cap)
                ovf[i8 + e] = sbase + ((unsigned long long)bt << RG::LOW) + ((w4[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
    }

    template <bool MASKED>
    __device__ __forceinline__ void tile(uint32_t l, uint32_t h, uint32_t Wm) {
        const uint32_t wb = (uint32_t)(uintptr_t)(W + par * RG::NBK);  // LDS byte address, 4 NBK-aligned
        uint32_t c[16], old[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) c[j] = __builtin_amdgcn_alignbit(h, l, 2 * j);  // low 2k bits: the window
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            // 4 * bucket of window j = bits [2j + LOW, 2j + 2k) of the tile at bit 2:
            // for even LOW that is in the window (LOW - 2) / 2 bases on when there is
            // one in this tile; v_bitop3 (x & mask) | wb keeps it one op (the ORed
            // base has zero low bits)
            constexpr int SH = RG::LOW - 2;
            const int sh = 2 * j + SH;
            uint32_t x;
            if ((SH & 1) == 0 && j + SH / 2 < 16) x = c[j + SH / 2];
            else x = sh < 32 ? __builtin_amdgcn_alignbit(h, l, sh) : h >> (sh - 32);
            const uint32_t wa = __builtin_amdgcn_bitop3_b32(x, (uint32_t)(4 * RG::NBK - 4), wb, 0xEA);
            old[j] = 0u;
            if (!MASKED || ((Wm >> j) & 1u))
                old[j] = __hip_atomic_fetch_add((__attribute__((address_space(3))) uint32_t *)(uintptr_t)wa, 2u,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        uint32_t any = 0u;  // OR of the returned words: low half >= 2 RING iff some entry did not fit
        // 2 RING, opaque to the compiler so the fit test stays one 16-bit compare
        uint32_t cap2;
        asm("s_mov_b32 %0, %1" : "=s"(cap2) : "i"(2 * RG::RING));
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t o = old[j];
            // byte offset: 2 * (b RING | swz) with the fill XORed into its low bits
            const uint32_t off = (o >> 15) ^ (o & (uint32_t)(2 * RG::RING - 1));
            bool ok = (uint16_t)o < (uint16_t)cap2;
            if (MASKED) ok = ok && ((Wm >> j) & 1u);
            uint16_t *dst = ok ? reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(ring) + off)
                               : dummy + 2 * lane;
            // the entry: the low LOW bits (ds_write_b16 drops the rest when LOW = 16)
            *dst = (uint16_t)(RG::LOW == 16 ? c[j] : c[j] & ((1u << RG::LOW) - 1u));
            any |= o;
        }
        if (__builtin_expect(__any((any & 0xFFFFu) >= (uint32_t)(2 * RG::RING)), 0)) {
            // ring full: straight to the list (skewed input)
            for (int j = 0; j < 16; ++j) {
                const uint32_t lo = (old[j] & 0xFFFFu) >> 1;
                if ((!MASKED || ((Wm >> j) & 1u)) && lo >= (uint32_t)RG::RING)
                {
                    const uint32_t bj = (c[j] >> RG::LOW) & (RG::NBK - 1);
                    const unsigned long long at = gH[bj] + lo;
                    const uint32_t e = c[j] & ((1u << RG::LOW) - 1u);
                    if (!SAMPLED || at < lim[bj]) ent[at] = (uint16_t)e;
                    else ovf_put(bj, e);
                }
            }
        }
    }

    // entry at relative list index g of bucket b, from the ring (h: ring slot 0's index)
    __device__ __forceinline__ uint16_t ring_entry(uint32_t b, uint32_t h, uint32_t g) const {
        if constexpr (ring_circ<K>()) return ring[b * RG::RING + ((g & (RG::RING - 1)) ^ ring_swz(b))];
        return ring[b * RG::RING + ((g - h) ^ ring_swz(b))];
    }

    // start of a piece: list (s, b)'s segment of this workgroup begins at F
    // (sampled mode: F is 32-aligned and the region holds capb entries; entries past
    // it are dropped and reported by finish())
    __device__ __forceinline__ void begin(uint32_t b, unsigned long long F, uint32_t capb, bool owner) {
        P0 = F & ~31ull;
        f = v = f0 = (uint32_t)(F - P0);
        cap = SAMPLED ? f0 + capb : ~0u;
        if (owner) {
            W[b] = ring_circ<K>() ? ring_word_circ<K>(b, f) : ring_word<K>(b, f);
            gH[b] = P0;
            if (SAMPLED) lim[b] = P0 + cap;
        }
    }

    // phase B for this thread's bucket; the caller brackets it with barriers.
    // Complete segments leave as whole 64-byte stores by lane quads (one lane per
    // segment issues 64 scattered 16-byte pieces per store, ~2x slower in HBM:
    // scripts/write_microbench.hip): in pass t every quad stores the segment of
    // its lane t, whose ring address and list index / 32 reach the quad by DPP
    // broadcasts (VALU, no LDS round trip).  All bookkeeping is 32-bit.
    __device__ __forceinline__ void flush() {
        const uint32_t b = (uint32_t)tid / RG::TPB, j = (uint32_t)tid % RG::TPB;
        const uint32_t h = f & ~31u;  // ring slot 0
        const uint32_t fill = (W[par * RG::NBK + b] & 0xFFFFu) >> 1;  // slots used (or wanted) this round
        const uint32_t f1 = h + fill;
        const uint32_t nseg = (fill < (uint32_t)RG::RING ? fill : (uint32_t)RG::RING) >> 5;
        const uint32_t x8 = ring_swz(b) >> 3;  // the swizzle in 16-byte chunks
        uint4 *row = reinterpret_cast<uint4 *>(ring + b * RG::RING);
        // the partial last segment moves to the ring's start at the end (after
        // this wave's reads of segment 0; no other thread reads segments 0 or
        // nseg); its chunks are read now, their latency hidden
        // (unconditional reads, inside the bucket's own ring: predicated ones
        // would each wait for the last)
        constexpr bool CIRC = ring_circ<K>();
        const uint32_t nq = (!CIRC && fill <= (uint32_t)RG::RING && j == 0 && nseg > 0) ? ((fill & 31u) + 7u) >> 3 : 0u;
        uint4 tl0, tl1, tl2, tl3;
        if constexpr (!CIRC) {
            tl0 = row[((4 * nseg + 0) ^ x8) & (RG::RING / 8 - 1)];
            tl1 = row[((4 * nseg + 1) ^ x8) & (RG::RING / 8 - 1)];
            tl2 = row[((4 * nseg + 2) ^ x8) & (RG::RING / 8 - 1)];
            tl3 = row[((4 * nseg + 3) ^ x8) & (RG::RING / 8 - 1)];
        }
        uint32_t i0 = j;
        if (h < v && j == 0 && nseg > 0) {  // segment 0 partly before v (piece start, after an overflow)
            for (uint32_t q = 0; q < 32; ++q)
                if (h + q >= v) {
                    const uint16_t e = ring_entry(b, h, h + q);
                    if (!SAMPLED || h + q < cap) ent[P0 + h + q] = e;
                    else ovf_put(b, e);
                }
            i0 = j + RG::TPB;
        }
        const uint32_t q = (uint32_t)lane & 3u;
        const uint32_t rowb = (uint32_t)(uintptr_t)row;                      // LDS byte address of the ring
        const uint32_t gs = (uint32_t)((P0 + h) >> 5);                        // list index / 32 of slot 0
        for (uint32_t i = i0; __any(i < nseg); i += RG::TPB) {  // mostly once: two segments are rare
            // bit 2: a segment to store, bit 3: one past its region (to the overflow
            // list); bits 0-1: the chunk swizzle
            const bool in = !SAMPLED || h + 32u * i + 32u <= cap;
            // the ring half of segment i (circular: it follows the list index)
            const uint32_t half = CIRC ? (((h >> 5) + i) & 1u) ^ (x8 >> 2) : (i ^ (x8 >> 2));
            const uint32_t A = (rowb + 64u * half) | (x8 & 3u) | (i < nseg ? (in ? 4u : 8u) : 0u);
            uint32_t a[4], g[4];
            quad_bcast4(A, a);
            quad_bcast4(gs + i, g);
            u32x4 val[4];  // (a quad without a segment reads a chunk of its own ring harmlessly)
#pragma unroll
            for (int t = 0; t < 4; ++t) val[t] = *(const lds_u32x4 *)(uintptr_t)((a[t] & ~63u) + 16u * (q ^ (a[t] & 3u)));
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (a[t] & 4u) reinterpret_cast<u32x4 *>(ent + 32ull * g[t])[q] = val[t];
            if (SAMPLED && __builtin_expect(__any(((a[0] | a[1] | a[2] | a[3]) & 8u) != 0u), 0)) {
                for (int t = 0; t < 4; ++t)  // this lane's 8 entries of the quad's segment t
                    if (a[t] & 8u) ovf_seg(a[t], val[t][0], val[t][1], val[t][2], val[t][3]);
            }
        }
        if (fill > (uint32_t)RG::RING) {
            v = f1;  // [h + RING, f1) went straight to the list
        } else if constexpr (!CIRC) {  // the partial last segment to the ring's start
            if (nq > 0) row[0 ^ x8] = tl0;
            if (nq > 1) row[1 ^ x8] = tl1;
            if (nq > 2) row[2 ^ x8] = tl2;
            if (nq > 3) row[3 ^ x8] = tl3;
        }
        f = f1;
        if (j == 0) {
            W[(par ^ 1u) * RG::NBK + b] = CIRC ? ring_word_circ<K>(b, f1) : ring_word<K>(b, f1 & 31u);
            gH[b] = P0 + (f1 & ~31u);
        }
        par ^= 1u;
    }

    __device__ void after_iter(int64_t, int64_t, bool) {  // one tile per wave per round
        lds_barrier();  // every window of the round is ranked and in its ring
        flush();
        lds_barrier();  // rings read, W set up: the next round may write
    }

    // end of a piece: the partial segment left in the ring, entry by entry (past the
    // region: to the overflow list); the piece's entries of the bucket -> *cnt_out
    // (sampled mode: R4 reads min(cnt, capacity) of them from the region)
    __device__ __forceinline__ void finish(uint32_t *cnt_out) {
        const uint32_t b = (uint32_t)tid / RG::TPB, j = (uint32_t)tid % RG::TPB;
        const uint32_t h = f & ~31u;
        const uint32_t lo = h > v ? h : v;
        for (uint32_t g = lo + j; g < f; g += RG::TPB) {
            const uint16_t e = ring_entry(b, h, g);
            if (!SAMPLED || g < cap) ent[P0 + g] = e;
            else ovf_put(b, e);
        }
        if (j == 0) *cnt_out = f - f0;
    }
};

// R3 launch: the piece walk of radix_count_kernel with the ring scatter (the whole
// LDS of a CU: one 1024-thread workgroup per CU).  SAMPLED: into the capacity
// regions (p.capv), entries past them to the overflow lists (p.ovf).
template <int K, class Idx, bool SAMPLED>
__global__ __launch_bounds__(1024) void radix_ring_kernel(RParams p) {
    using RG = RingGeom<K>;
    constexpr int NWAVES = RG::BLOCK / 64;
    __shared__ __attribute__((aligned(16))) uint16_t s_ring[RG::NBK * RG::RING];
    __shared__ uint32_t s_W[2 * RG::NBK];
    __shared__ unsigned long long s_gH[RG::NBK];
    __shared__ unsigned long long s_lim[RG::NBK];
    __shared__ uint16_t s_dummy[128];
    __shared__ int64_t s_first;
    __shared__ uint32_t s_ovf_n;

    const int tid = threadIdx.x, lane = tid & 63;
    if (gated_off(p)) return;
    // sampled mode: the capacities must fit the entry array (else the exact rerun)
    if (SAMPLED && p.off[p.n * RG::NBK * p.G] > p.ent_cap) {
        if (tid == 0) __hip_atomic_store(p.flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int w = blockIdx.x;
    const Geom g = make_geom<Idx>(p);
    const int64_t tb = g.T0 + (int64_t)w * g.tpw;
    const int64_t te = (tb + g.tpw) < g.T1 ? (tb + g.tpw) : g.T1;
    if (tb >= te) return;
    const int64_t R0 = (tb << kTileShift) > g.wl ? (tb << kTileShift) : g.wl;
    const int64_t R1 = (te << kTileShift) < g.wh ? (te << kTileShift) : g.wh;
    if (tid == 0) {
        s_first = first_record_at<Idx>(p, R0);
        s_ovf_n = 0u;
    }
    __syncthreads();
    const uint32_t b = (uint32_t)tid / RG::TPB;
    for (int64_t s = s_first; s < p.n; ++s) {
        if (rec_off<Idx>(p, s) >= R1) break;
        int64_t ca, ce;
        record_windows<K, Idx>(p, g, s, ca, ce);
        const int64_t ps = ca > R0 ? ca : R0;
        const int64_t pe = ce < R1 ? ce : R1;
        if (ps >= pe) continue;
        RRingOp<K, SAMPLED> op;
        op.ring = s_ring;
        op.W = s_W;
        op.gH = s_gH;
        op.dummy = s_dummy;
        op.ent = p.ent;
        op.tid = tid;
        op.lane = lane;
        op.par = 0;
        const int64_t li = ((s * RG::NBK) + b) * p.G + w;  // (s, b, w)
        op.lim = s_lim;
        op.ovf = p.ovf ? p.ovf + (int64_t)w * p.ovf_cap : nullptr;
        op.ovf_n = &s_ovf_n;
        op.ovf_cap = p.ovf_cap;
        op.sbase = (unsigned long long)s << (2 * K);
        op.begin(b, p.off[li], SAMPLED ? p.capv[li] : 0u, (uint32_t)tid % RG::TPB == 0);  // this workgroup's segment of list (s, b)
        __syncthreads();
        const int64_t tp0 = ps >> kTileShift;
        const int64_t tp1 = ((pe - 1) >> kTileShift) + 1;
        const int64_t per = (tp1 - tp0 + NWAVES - 1) / NWAVES;
        const int64_t a0 = tp0 + (int64_t)wave * per;
        const int64_t a1 = (a0 + per) < tp1 ? (a0 + per) : tp1;
        stream_tiles<K, RRingOp<K, SAMPLED>, kRScatPF, 0>(p.data, a0, a1, per, ps, pe, g.rl, g.rh, lane, op);
        op.finish(p.cnt + li);
        __syncthreads();
    }
    if (SAMPLED && tid == 0) {
        p.ovf_cnt[w] = s_ovf_n;
        if (s_ovf_n > p.ovf_cap) __hip_atomic_store(p.flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Sampled mode, after R4: the overflow lists' entries added into stage (device-scope
// atomics; skewed input only).  Nothing when the exact rerun ran.
__global__ __launch_bounds__(256) void radix_overflow_kernel(RParams p) {
    if (__hip_atomic_load(p.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    const int64_t w = blockIdx.x;
    const uint32_t c = p.ovf_cnt[w];
    const uint32_t n = c < p.ovf_cap ? c : p.ovf_cap;
    const unsigned long long *o = p.ovf + w * (int64_t)p.ovf_cap;
    for (uint32_t i = blockIdx.y * 256 + threadIdx.x; i < n; i += gridDim.y * 256)
        atomicAdd(&p.stage[o[i]], 1u);
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
        const auto add8 = [&](const uint4 x) {
            add(x.x & 0xFFFFu);
            add(x.x >> 16);
            add(x.y & 0xFFFFu);
            add(x.y >> 16);
            add(x.z & 0xFFFFu);
            add(x.z >> 16);
            add(x.w & 0xFFFFu);
            add(x.w >> 16);
        };
        // four 16-byte loads in flight per lane (64 KB per CU): one per iteration
        // left the loop waiting on HBM latency
        uint64_t i = threadIdx.x;
        const auto ld = [&](uint64_t k) { return v[k]; };  // (non-temporal loads: no gain, same-box A/B)
        for (; i + (kR4U - 1) * 1024 < nvec; i += kR4U * 1024) {
            uint4 x[kR4U];
#pragma unroll
            for (int u = 0; u < kR4U; ++u) x[u] = ld(i + 1024u * u);
#pragma unroll
            for (int u = 0; u < kR4U; ++u) add8(x[u]);
        }
        for (; i < nvec; i += 1024) add8(v[i]);
        const uint64_t t = a + nvec * 8;
        if (t + threadIdx.x < end) add(ent[t + threadIdx.x]);
    }
}

// Sampled mode: a list is the G regions [rb[r], rb[r] + rn[r]) of its workgroups,
// with gaps between them.  The regions' 16-byte vectors are numbered 0 .. V-1 in
// order (vpre: exclusive prefix of each region's vector count) and thread t takes
// vectors t, t + 1024, ..., kR4U in flight, walking its region cursor forward;
// a vector's entries outside its region are skipped.
constexpr int kMaxRegions = 256;  // workgroups of R1/R3 in sampled mode
template <int LOW>
__device__ __forceinline__ void hist_regions(const uint16_t *ent, const uint32_t *vpre, const unsigned long long *rb,
                                             const uint32_t *rn, uint32_t *h) {
    const uint32_t V = vpre[kMaxRegions];
    const uint4 *v = reinterpret_cast<const uint4 *>(ent);
    // the thread's current region r, cached in registers: flat vectors [vb, ve),
    // address of vector vb, and [jf, jl) the ones whose 8 entries all lie in it
    uint32_t r = 0, vb = 0, ve = 0, jf = 0, jl = 0;
    unsigned long long va0 = 0;
    const auto enter = [&](uint32_t q) {
        vb = vpre[q];
        ve = vpre[q + 1];
        const unsigned long long lo = rb[q], hi = lo + rn[q];
        va0 = lo >> 3;
        jf = vb + ((lo & 7u) ? 1u : 0u);
        jl = ve - (((hi & 7u) && ve > jf) ? 1u : 0u);
    };
    enter(0);
    for (uint32_t j0 = threadIdx.x; j0 < V; j0 += kR4U * 1024) {
        uint4 x[kR4U];
        uint32_t m[kR4U];  // valid entries of vector u (bit q: entry q)
#pragma unroll
        for (int u = 0; u < kR4U; ++u) {
            const uint32_t j = j0 + 1024u * u;
            m[u] = 0u;
            if (j < V) {
                while (j >= ve) enter(++r);
                const unsigned long long va = va0 + (j - vb);
                // non-temporal: the entries are read once (C3's R4 4.95 -> 4.52 ms, same
                // box; with eight loads in flight per lane instead of four: 4.60)
                typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(v + va));
                x[u] = make_uint4(t[0], t[1], t[2], t[3]);
                if (j >= jf && j < jl) {
                    m[u] = 0xFFu;
                } else {  // a region's first or last vector: entries [lo, lo + rn) of it
                    const int64_t dlo = (int64_t)(rb[r] - va * 8), dhi = dlo + (int64_t)rn[r];
                    const uint32_t mlo = dlo <= 0 ? 0xFFu : ((0xFFu << dlo) & 0xFFu);
                    const uint32_t mhi = dhi >= 8 ? 0xFFu : (dhi <= 0 ? 0u : ((1u << dhi) - 1u));
                    m[u] = mlo & mhi;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kR4U; ++u) {
            const uint32_t e[8] = {x[u].x & 0xFFFFu, x[u].x >> 16, x[u].y & 0xFFFFu, x[u].y >> 16,
                                   x[u].z & 0xFFFFu, x[u].z >> 16, x[u].w & 0xFFFFu, x[u].w >> 16};
            if (m[u] == 0xFFu) {
#pragma unroll
                for (int q = 0; q < 8; ++q) hist_add<LOW>(h, e[q]);
            } else if (m[u] != 0u) {
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if ((m[u] >> q) & 1u) hist_add<LOW>(h, e[q]);
            }
        }
    }
}

// Cold path of R4 (LOW = 16): the list [beg, end) recounted exactly in two 32 768-bin
// halves with 32-bit bins (kept out of line: the hot loop's registers).
template <int LOW>
__device__ __noinline__ void hist_recount(const uint16_t *ent, uint64_t beg, uint64_t end, uint32_t *h,
                                          uint32_t *dst) {
    constexpr int kWords = 1 << (LOW - 1);
    for (uint32_t half = 0; half < 2; ++half) {
        __syncthreads();
        for (int i = threadIdx.x; i < kWords; i += 1024) h[i] = 0u;
        __syncthreads();
        hist_list<LOW, true>(ent, beg, end, h, half);
        __syncthreads();
        for (int i = threadIdx.x; i < kWords; i += 1024) dst[half * kWords + i] = h[i];
    }
}

// The same for a list of nreg regions [rb[r], rb[r] + rn[r]) (sampled mode).
template <int LOW>
__device__ __noinline__ void hist_recount_regions(const uint16_t *ent, const unsigned long long *rb,
                                                  const uint32_t *rn, int nreg, uint32_t *h, uint32_t *dst) {
    constexpr int kWords = 1 << (LOW - 1);
    for (uint32_t half = 0; half < 2; ++half) {
        __syncthreads();
        for (int i = threadIdx.x; i < kWords; i += 1024) h[i] = 0u;
        __syncthreads();
        for (int r = 0; r < nreg; ++r) hist_list<LOW, true>(ent, rb[r], rb[r] + rn[r], h, half);
        __syncthreads();
        for (int i = threadIdx.x; i < kWords; i += 1024) dst[half * kWords + i] = h[i];
    }
}

// R4: one workgroup per list (s, b): 2^LOW-bin LDS histogram -> stage.  LOW = 16
// packs two 16-bit bins per word (128 KB); a bin that reaches 65 536 within the
// list wraps, which lowers the sum of the bins below the list length (a carry
// into the neighbour costs 65 535, one out of the word 65 536), and the list is
// then recounted exactly in two 32 768-bin halves.
// REG (sampled mode): the list is the G regions (off, min(cnt, capacity)) of the
// workgroups (all of cnt when the exact rerun ran: then the regions are contiguous).
template <int K, bool REG>
__global__ __launch_bounds__(1024) void radix_hist_kernel(RParams p, int64_t nbins) {
    constexpr int LOW = low_bits(K);
    constexpr int kBucketBins = 1 << LOW;
    constexpr int kWords = LOW <= 15 ? kBucketBins : kBucketBins / 2;
    __shared__ __attribute__((aligned(16))) uint32_t h[kWords];
    __shared__ unsigned long long s_sum;
    __shared__ uint32_t s_vpre[REG ? kMaxRegions + 1 : 1];
    __shared__ unsigned long long s_rb[REG ? kMaxRegions : 1];
    __shared__ uint32_t s_rn[REG ? kMaxRegions : 1];
    __shared__ uint64_t s_scan[kScanBlock / 64];
    const int64_t nlists = p.n * p.nbk;
    // sampled mode: did the exact rerun run (then every region is exact and whole)?
    const bool rerun = REG && __hip_atomic_load(p.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    // REG: thread t < G holds region t of the next list, loaded one list ahead so
    // that the loads' latency hides behind the current list's histogram
    unsigned long long nx_rb = 0;
    uint32_t nx_ne = 0;
    const auto fetch = [&](int64_t L) {
        if (REG && L < nlists && (int)threadIdx.x < p.G) {
            const int64_t li = L * p.G + threadIdx.x;
            nx_rb = p.off[li];
            const uint32_t c = p.cnt[li], cap = rerun ? c : p.capv[li];
            nx_ne = c < cap ? c : cap;  // past the capacity: in the overflow list
        }
    };
    fetch(blockIdx.x);
    bool dirty = true;  // (the list-end pass leaves the bins cleared, but for a recount)
    for (int64_t list = blockIdx.x; list < nlists; list += gridDim.x) {  // list = s*nbk + b
        const int64_t s = list / p.nbk, b = list % p.nbk;
        if (b == 0 && threadIdx.x == 0 && p.status) {  // int32 bins of >= 2^31 windows could wrap
            const Geom g = make_geom<int64_t>(p);
            int64_t ca, ce;
            record_windows<K, int64_t>(p, g, s, ca, ce);
            if (ce - ca >= ((int64_t)1 << 31))
                __hip_atomic_store(p.status, (uint32_t)KMC_ERR_RECORD_TOO_LONG, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (dirty)
            for (int i = threadIdx.x; i < kWords; i += 1024) h[i] = 0u;
        if (threadIdx.x == 0) s_sum = 0ull;
        uint64_t beg, end;  // entries of the list (REG: beg = 0, end = their number)
        const int nreg = p.G;
        if constexpr (REG) {
            // every workgroup's region of the list (a dependent search for the
            // workgroups that hold record s cost more); one block scan of (vectors,
            // entries) packed in 64 bits
            const int t = threadIdx.x;
            const unsigned long long rb = nx_rb;
            const uint32_t ne = nx_ne;
            fetch(list + gridDim.x);
            uint64_t nv = 0;
            if (t < nreg) {
                nv = ne ? ((rb + ne + 7) >> 3) - (rb >> 3) : 0;
                s_rb[t] = rb;
                s_rn[t] = ne;
            } else if (t < kMaxRegions) {
                s_rb[t] = 0;
                s_rn[t] = 0;
            }
            uint64_t tot;
            const uint64_t ex = block_excl_scan(t < nreg ? nv | ((uint64_t)ne << 32) : 0ull, s_scan, tot);
            if (t <= kMaxRegions) s_vpre[t] = (uint32_t)ex;
            beg = 0;
            end = tot >> 32;
            __syncthreads();
            hist_regions<LOW>(p.ent, s_vpre, s_rb, s_rn, h);
        } else {
            __syncthreads();
            beg = p.off[list * p.G];
            end = p.off[(list + 1) * p.G];
            hist_list<LOW, false>(p.ent, beg, end, h, 0u);
        }
        __syncthreads();
        uint32_t *dst = p.stage + s * nbins + b * kBucketBins;
        {
            // one pass (round 4, same box: R4 4.34 -> 4.19 ms against a sum pass, a
            // write pass and a clear pass): stage row written, bins summed (LOW = 16:
            // wrap check) and cleared
            uint32_t part = 0u;
            for (int i = threadIdx.x; i < kWords; i += 1024) {
                const uint32_t w = h[i];
                h[i] = 0u;
                if constexpr (LOW <= 15) {
                    dst[i] = w;
                } else {
                    part += (w & 0xFFFFu) + (w >> 16);
                    reinterpret_cast<uint2 *>(dst)[i] = make_uint2(w & 0xFFFFu, w >> 16);
                }
            }
            dirty = false;
            if constexpr (LOW > 15) {
                atomicAdd(&s_sum, (unsigned long long)part);
                __syncthreads();
                if (s_sum != end - beg) {  // a bin wrapped: the exact recount overwrites the row
                    if constexpr (REG) hist_recount_regions<LOW>(p.ent, s_rb, s_rn, nreg, h, dst);
                    else hist_recount<LOW>(p.ent, beg, end, h, dst);
                    dirty = true;
                }
            }
        }
        __syncthreads();  // h and s_sum are reused by the next list
    }
}

// R5: stage [n][nbins] -> sum[s + ld*code], transposed through LDS in tiles of
// kPlaceS records x kPlaceC codes: rows are read 16 bytes per lane, and the
// tile's output (kPlaceC codes x its records) is written in record-fastest order,
// i.e. contiguously when ld = n.  Grid (nbins / kPlaceC, record groups).
constexpr int kPlaceC = 512, kPlaceS = 16;
__global__ __launch_bounds__(256) void radix_place_kernel(RParams p, int64_t nbins) {
    __shared__ uint32_t t[kPlaceS][kPlaceC + 1];
    const int64_t c0 = (int64_t)blockIdx.x * kPlaceC;
    for (int64_t s0 = (int64_t)blockIdx.y * kPlaceS; s0 < p.n; s0 += (int64_t)gridDim.y * kPlaceS) {
        const int ts = (int)(p.n - s0 < kPlaceS ? p.n - s0 : kPlaceS);
        for (int q = threadIdx.x; q < ts * (kPlaceC / 4); q += 256) {
            const int r = q / (kPlaceC / 4), cc = (q % (kPlaceC / 4)) * 4;
            const uint4 v = *reinterpret_cast<const uint4 *>(p.stage + (s0 + r) * nbins + c0 + cc);
            t[r][cc] = v.x;
            t[r][cc + 1] = v.y;
            t[r][cc + 2] = v.z;
            t[r][cc + 3] = v.w;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < ts * kPlaceC; i += 256) {
            const int c = i / ts, r = i % ts;
            p.sum[s0 + r + p.ld * (c0 + c)] = (int32_t)t[r][c];
        }
        __syncthreads();
    }
}

// R5 when ld = n > 16 (the output matrix is one contiguous [nbins][n] array): each
// workgroup writes kPlaceO consecutive outputs (codes c_lo .. c_hi, every
// record), gathered through LDS from the n stage rows (each read contiguously).
// The 16-record tiles above split a code's row between workgroups when n is not a
// multiple of 16 (25 records: 6.8 ms instead of ~2).  n <= kPlaceMaxN.
constexpr int kPlaceO = 4096, kPlaceMaxN = 1024;
__global__ __launch_bounds__(256) void radix_place_contig_kernel(RParams p, int64_t nbins) {
    __shared__ uint32_t t[kPlaceO + 3 * kPlaceMaxN];
    const uint32_t n = (uint32_t)p.n;
    const int64_t total = nbins * (int64_t)n;
    for (int64_t o0 = (int64_t)blockIdx.x * kPlaceO; o0 < total; o0 += (int64_t)gridDim.x * kPlaceO) {
        const int64_t c_lo = o0 / n;
        const int64_t o1 = (o0 + kPlaceO < total ? o0 + kPlaceO : total);
        const uint32_t nc = (uint32_t)((o1 - 1) / n - c_lo + 1);  // codes touched
        const uint32_t sr = nc | 1u;                               // odd row stride: spread the banks
        for (uint32_t q = threadIdx.x; q < n * nc; q += 256) {
            const uint32_t r = q / nc, cc = q - r * nc;
            t[r * sr + cc] = p.stage[(int64_t)r * nbins + c_lo + cc];
        }
        __syncthreads();
        const uint32_t first = (uint32_t)(o0 - c_lo * n);  // record of output o0
        for (uint32_t i = threadIdx.x; i < (uint32_t)(o1 - o0); i += 256) {
            const uint32_t x = first + i, c = x / n, r = x - c * n;
            p.sum[o0 + i] = (int32_t)t[r * sr + c];
        }
        __syncthreads();
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
inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct RLayout {
    size_t cnt, off, bsum, capv, flag, ovf_cnt, ovf, ent, stage, total;
    int64_t m, nscan;
};

inline RLayout r_layout(int k, int64_t n, int G, int64_t ent_cap, bool sampled, uint32_t ovf_cap) {
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
    L.capv = o;
    o += sampled ? al256((size_t)L.m * 4) : 0;
    L.flag = o;
    o += sampled ? 256 : 0;
    L.ovf_cnt = o;
    o += sampled ? al256((size_t)G * 4) : 0;
    L.ovf = o;
    o += sampled ? al256((size_t)G * ovf_cap * 8) : 0;
    L.ent = o;
    o += al256((size_t)ent_cap * 2 + 16);
    L.stage = o;
    o += al256((size_t)n * ((size_t)1 << (2 * k)) * 4);
    L.total = o;
    return L;
}

std::mutex r_mu;
std::vector<int> r_cus;  // CUs per device

// Partition offsets (kmc_diag_radix_mode): 0 = auto, 1 = exact (R1 count + scan),
// 2 = sampled (regions sized from a 1-in-16 tile sample, exact rerun on overflow);
// cap_scale multiplies the sampled capacities (test hook: < 1 forces the rerun).
int g_radix_mode = 0;
float g_cap_scale = 1.0f;

// Sampled mode pays when the lists are long: it replaces R1's full read of the
// input by a 1-in-16 sample (C3: R1 1.95 -> 0.21 ms; 1-in-8 0.42, 1-in-32 0.12 ms
// but R3 + R4 +0.1-0.2 ms with the wider regions, same box), but R4 then sets up G regions
// per list and walks them (C3: +0.1-0.3 ms over 10 240 lists of ~1 M entries; C3R,
// 25 600 lists of ~120 K entries: +0.6 ms, more than its R1 saving).
constexpr double kSampledMinPerList = 256.0 * 1024.0;

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
int run_radix(const kmc_dense_args *a, int64_t ibias, hipStream_t st, bool size_only, size_t *size_out) {
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
    constexpr int64_t NBK = (int64_t)1 << (2 * K - low_bits(K));
    const double win = wh > wl ? (double)(wh - wl) : 0.0;       // >= valid windows in range
    const double regions = (double)(G + n) * (double)NBK;       // >= (s, b, w) with a piece
    int mode;
    float cap_scale;
    {
        std::lock_guard<std::mutex> lk(r_mu);
        mode = g_radix_mode;
        cap_scale = g_cap_scale;
    }
    const bool sampled = G <= kMaxRegions &&
                         (mode == 2 || (mode == 0 && win >= kSampledMinPerList * (double)n * (double)NBK));
    // sampled capacities: sum over regions of 1.05 c + 6 sqrt(16 c) + 64 (+ 31 rounding),
    // c summing to the windows; Cauchy-Schwarz bounds the square roots
    const int64_t ent_cap = sampled ? (int64_t)(1.05 * win + 95.0 * regions + 6.0 * std::sqrt((double)kSampleStride * win * regions) + 64.0)
                                    : (int64_t)win;
    // overflow lists: 1/32 of the windows in all (past that, the exact rerun)
    const uint32_t ovf_cap = (uint32_t)std::min<double>(std::max<double>(4096.0, win / 32.0 / G), 1 << 30);
    const RLayout L = r_layout(K, n, G, ent_cap, sampled, ovf_cap);
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
    p.ibias = ibias;
    p.n = n;
    p.wl = wl;
    p.wh = wh;
    p.rl = (int64_t)a->read_lo;
    p.rh = (int64_t)a->read_hi;
    p.derive = 0;
    p.G = G;
    p.nbk = 1 << (2 * K - low_bits(K));
    p.cnt = reinterpret_cast<uint32_t *>(base + L.cnt);
    p.off = reinterpret_cast<uint64_t *>(base + L.off);
    p.ent = reinterpret_cast<uint16_t *>(base + L.ent);
    p.stage = reinterpret_cast<uint32_t *>(base + L.stage);
    p.sum = a->sum;
    p.ld = a->sum_ld ? (int64_t)a->sum_ld : n;
    p.invalid = a->invalid;
    p.capv = nullptr;
    p.flag = nullptr;
    p.gate = nullptr;
    p.ovf = nullptr;
    p.ovf_cnt = nullptr;
    p.ovf_cap = 0;
    p.ent_cap = (uint64_t)ent_cap;
    p.cap_scale = cap_scale;
    p.status = reinterpret_cast<uint32_t *>(a->status);
    uint64_t *bsum = reinterpret_cast<uint64_t *>(base + L.bsum);
    const int64_t nbins = (int64_t)1 << (2 * K);
    const unsigned hist_grid = (unsigned)std::min<int64_t>(n * p.nbk, kMaxGridX);

    if (t_trace_before) {
        he = hipEventRecord(t_trace_before, st);
        if (he != hipSuccess) return (int)he;
    }
    if (sampled) {
        // S1 sample -> capacities -> region starts -> R3 into the regions; if one
        // overflowed (or they exceed ent_cap) the gated exact path reruns R1 + scan +
        // R3 on the device (no host sync); R4 reads (off, cnt) regions either way
        RParams ps = p;
        ps.capv = reinterpret_cast<uint32_t *>(base + L.capv);
        ps.flag = reinterpret_cast<uint32_t *>(base + L.flag);
        ps.ovf = reinterpret_cast<unsigned long long *>(base + L.ovf);
        ps.ovf_cnt = reinterpret_cast<uint32_t *>(base + L.ovf_cnt);
        ps.ovf_cap = ovf_cap;
        he = hipMemsetAsync(ps.flag, 0, sizeof(uint32_t), st);
        if (he == hipSuccess) he = hipMemsetAsync(ps.ovf_cnt, 0, (size_t)G * 4, st);
        if (he != hipSuccess) return (int)he;
        hipLaunchKernelGGL((radix_count_kernel<K, int64_t, true>), dim3(G), dim3(1024), 0, st, ps);
        const int64_t cap_blocks = std::min<int64_t>((L.m + 255) / 256, 4096);
        hipLaunchKernelGGL((radix_cap_kernel<K, int64_t>), dim3((unsigned)(cap_blocks > 0 ? cap_blocks : 1)), dim3(256),
                           0, st, ps);
        excl_scan_u32(ps.capv, L.m, bsum, p.off, st);
        hipLaunchKernelGGL((radix_ring_kernel<K, int64_t, true>), dim3(G), dim3(1024), 0, st, ps);
        RParams px = p;  // (no capacities, no overflow lists)
        px.gate = ps.flag;
        hipLaunchKernelGGL((radix_count_kernel<K, int64_t>), dim3(G), dim3(1024), 0, st, px);
        excl_scan_u32(p.cnt, L.m, bsum, p.off, st, ps.flag);
        hipLaunchKernelGGL((radix_ring_kernel<K, int64_t, false>), dim3(G), dim3(1024), 0, st, px);
        hipLaunchKernelGGL((radix_hist_kernel<K, true>), dim3(hist_grid), dim3(1024), 0, st, ps, nbins);
        hipLaunchKernelGGL(radix_overflow_kernel, dim3((unsigned)G, 16), dim3(256), 0, st, ps);
    } else {
        he = hipMemsetAsync(p.cnt, 0, (size_t)L.m * 4, st);
        if (he != hipSuccess) return (int)he;
        hipLaunchKernelGGL((radix_count_kernel<K, int64_t>), dim3(G), dim3(1024), 0, st, p);
        excl_scan_u32(p.cnt, L.m, bsum, p.off, st);
        hipLaunchKernelGGL((radix_ring_kernel<K, int64_t, false>), dim3(G), dim3(1024), 0, st, p);
        hipLaunchKernelGGL((radix_hist_kernel<K, false>), dim3(hist_grid), dim3(1024), 0, st, p, nbins);
    }
    if (p.ld == n && n > kPlaceS && n <= kPlaceMaxN) {  // n <= 16: one tile row covers every record
        const int64_t blocks = (nbins * n + kPlaceO - 1) / kPlaceO;
        hipLaunchKernelGGL(radix_place_contig_kernel, dim3((unsigned)std::min<int64_t>(blocks, kMaxGridX)), dim3(256),
                           0, st, p, nbins);
    } else {
        hipLaunchKernelGGL(radix_place_kernel,
                           dim3((unsigned)(nbins / kPlaceC),
                                (unsigned)std::min<int64_t>((n + kPlaceS - 1) / kPlaceS, kMaxGridY)),
                           dim3(256), 0, st, p, nbins);
    }
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

#ifdef KMC_DIAG_HOOKS
// Test hook (diagnostic library only, not in kmc.h): see g_radix_mode.
extern "C" KMC_DIAG_API int kmc_diag_radix_mode(int mode, float cap_scale) {
    if (mode < 0 || mode > 2 || !(cap_scale > 0.0f)) return KMC_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(r_mu);
    g_radix_mode = mode;
    g_cap_scale = cap_scale;
    return KMC_OK;
}
#endif

// Entry used by kmc_dense.hip for 9 <= k <= KMC_DENSE_MAX_K.
int radix_dense(const kmc_dense_args *a, int64_t ibias, hipStream_t st, bool size_only, size_t *size_out) {
    switch (a->k) {
        case 9: return run_radix<9>(a, ibias, st, size_only, size_out);
        case 10: return run_radix<10>(a, ibias, st, size_only, size_out);
        case 11: return run_radix<11>(a, ibias, st, size_only, size_out);
        case 12: return run_radix<12>(a, ibias, st, size_only, size_out);
        case 13: return run_radix<13>(a, ibias, st, size_only, size_out);
        default: return KMC_ERR_UNSUPPORTED_K;
    }
}

}  // namespace kmc
