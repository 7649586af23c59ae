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
// LOW = min(2k - 6, 15), 16 from k = 12 on (low_bits).  Bytes per k-mer: 1 (R1) +
// 1 (R3) input, 2 written + 2 read entries, plus the output twice; the LDS
// histograms see the same bank-conflict-bound atomic rate as the k <= 8 kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <vector>

#include "kmc.h"
#include "kmc_internal.h"
#include "kmc_scan.h"
#include "kmc_stream.h"

// tile prefetch depth and nt loads of the count (R1) and scatter (R3) walks, each
// from a same-box A/B: R1 PF 3 + nt 2.04-2.06 -> 1.95-2.01 ms; R3 PF 2-4 equal, and
// nt loads made it slower
#ifndef KMC_RSCAT_PF
#define KMC_RSCAT_PF 2
#endif
#ifndef KMC_RCOUNT_PF
#define KMC_RCOUNT_PF 3
#endif
#ifndef KMC_RCOUNT_NT
#define KMC_RCOUNT_NT 1
#endif
#ifndef KMC_R4_U
#define KMC_R4_U 4  // R4 16-byte entry loads in flight per lane (2 / 4 / 8 measured equal, same box)
#endif
#ifndef KMC_RING_RT
#define KMC_RING_RT 1
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
    const char *data;        // 16-byte aligned
    const void *indices;
    int64_t ibias;           // added to every indices[] value (kmc_stream.h rec_off)
    int64_t n;
    int64_t wl, wh, rl, rh;
    int derive;
    int G;           // workgroups of R1/R3
    int nbk;         // buckets per record
    uint32_t *cnt;   // [n][nbk][G]
    uint64_t *off;   // [n*nbk*G + 1] exclusive prefix of cnt
    uint16_t *ent;   // entries
    uint32_t *stage; // [n][4^k]
    int32_t *sum;
    int64_t ld;
    int32_t *invalid;
};

// R1 op: bucket counters with kCountRep replicas interleaved (counter b of lane l
// at word b*kCountRep + l % kCountRep), so the 32 lanes of an LDS lane group
// always hit 32 different banks (1 024 buckets x 32 replicas = 128 KB at k = 13).
constexpr int kCountRep = 32;
template <int K>
struct RCountOp {
    static constexpr int LOW = low_bits(K);
    uint32_t *c;  // LDS bucket counters (this lane's replica)
    __device__ void before_tile() {}
    template <bool MASKED>
    __device__ __forceinline__ void tile(uint32_t lo, uint32_t hi, uint32_t W) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t code = window_code_rt<K>(lo, hi, j);
            if (!MASKED || ((W >> j) & 1u))
                __hip_atomic_fetch_add(&c[(code >> LOW) * kCountRep], 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __device__ void after_iter(int64_t, int64_t, bool) {}
};

// R1: the piece walk of the dense kernel, counting per record piece the windows
// of each bucket in LDS -> cnt[(s*NBK + b)*G + w].
template <int K, class Idx>
__global__ __launch_bounds__(1024) void radix_count_kernel(RParams p) {
    constexpr int BLOCK = 1024;
    constexpr int NWAVES = BLOCK / 64;
    constexpr int NBK = 1 << (2 * K - low_bits(K));
    __shared__ uint32_t s_cnt[NBK * kCountRep];
    __shared__ int64_t s_first;

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
        const int64_t lbase = (s * NBK) * p.G + w;  // cnt index of (s, b=0, w); stride G per bucket
        for (int i = tid; i < NBK * kCountRep; i += BLOCK) s_cnt[i] = 0u;
        __syncthreads();
        const int64_t tp0 = ps >> kTileShift;
        const int64_t tp1 = ((pe - 1) >> kTileShift) + 1;
        const int64_t per = (tp1 - tp0 + NWAVES - 1) / NWAVES;
        const int64_t a0 = tp0 + (int64_t)wave * per;
        const int64_t a1 = (a0 + per) < tp1 ? (a0 + per) : tp1;
        RCountOp<K> op{s_cnt + (lane & (kCountRep - 1))};
        stream_tiles<K, RCountOp<K>, KMC_RCOUNT_PF, KMC_RCOUNT_NT>(p.data, a0, a1, per, ps, pe, g.rl, g.rh, lane, op);
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
    static_assert(2 * (BLOCK * 16 * KMC_RING_RT + 32) < 65536, "one tile per wave per round");
};

// o[t] = x of lane t of this lane's quad (DPP quad_perm broadcasts)
__device__ __forceinline__ void quad_bcast4(uint32_t x, uint32_t *o) {
    o[0] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x00, 0xF, 0xF, false);
    o[1] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x55, 0xF, 0xF, false);
    o[2] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xAA, 0xF, 0xF, false);
    o[3] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xFF, 0xF, 0xF, false);
}

// slot swizzle of bucket b (XOR mask, a multiple of 8 slots below 64)
__device__ __forceinline__ uint32_t ring_swz(uint32_t b) { return ((b >> 1) & 7u) * 8u; }

// W word of bucket b for a round whose first entry goes to ring slot f0 (< 32)
template <int K>
__device__ __forceinline__ uint32_t ring_word(uint32_t b, uint32_t f0) {
    return ((b * (uint32_t)RingGeom<K>::RING | ring_swz(b)) << 16) | (f0 << 1);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

template <int K>
struct RRingOp {
    using RG = RingGeom<K>;
    uint16_t *ring;        // LDS, NBK * RING entries
    uint32_t *W;           // LDS, [2][NBK]
    unsigned long long *gH;  // LDS, [NBK]: list index of every bucket's ring slot 0 this round
    uint16_t *dummy;       // LDS, 2 halfwords per lane
    uint16_t *ent;
    int tid, lane;
    uint32_t par;          // W buffer of this round
    // phase-B state of bucket tid / TPB (replicated over its TPB threads), list
    // indices relative to P0 = this piece's first list index rounded down to 32:
    // f = next entry, v = first entry still to be written from the ring
    unsigned long long P0;
    uint32_t f, v;
    int held = 0;          // tiles of this round taken (workgroup-uniform)

    __device__ void before_tile() {}

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
                    ent[gH[(c[j] >> RG::LOW) & (RG::NBK - 1)] + lo] = (uint16_t)(c[j] & ((1u << RG::LOW) - 1u));
            }
        }
    }

    // entry at relative list index g of bucket b, from the ring (h: ring slot 0's index)
    __device__ __forceinline__ uint16_t ring_entry(uint32_t b, uint32_t h, uint32_t g) const {
        return ring[b * RG::RING + ((g - h) ^ ring_swz(b))];
    }

    // start of a piece: list (s, b)'s segment of this workgroup begins at F
    __device__ __forceinline__ void begin(uint32_t b, unsigned long long F, bool owner) {
        P0 = F & ~31ull;
        f = v = (uint32_t)(F - P0);
        if (owner) {
            W[b] = ring_word<K>(b, f);
            gH[b] = P0;
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
        const uint32_t nq = (fill <= (uint32_t)RG::RING && j == 0 && nseg > 0) ? ((fill & 31u) + 7u) >> 3 : 0u;
        const uint4 tl0 = row[((4 * nseg + 0) ^ x8) & (RG::RING / 8 - 1)];
        const uint4 tl1 = row[((4 * nseg + 1) ^ x8) & (RG::RING / 8 - 1)];
        const uint4 tl2 = row[((4 * nseg + 2) ^ x8) & (RG::RING / 8 - 1)];
        const uint4 tl3 = row[((4 * nseg + 3) ^ x8) & (RG::RING / 8 - 1)];
        uint32_t i0 = j;
        if (h < v && j == 0 && nseg > 0) {  // segment 0 partly before v (piece start, after an overflow)
            for (uint32_t q = 0; q < 32; ++q)
                if (h + q >= v) ent[P0 + h + q] = ring_entry(b, h, h + q);
            i0 = j + RG::TPB;
        }
        const uint32_t q = (uint32_t)lane & 3u;
        const uint32_t rowb = (uint32_t)(uintptr_t)row;                      // LDS byte address of the ring
        const uint32_t gs = (uint32_t)((P0 + h) >> 5);                        // list index / 32 of slot 0
        for (uint32_t i = i0; __any(i < nseg); i += RG::TPB) {  // mostly once: two segments are rare
            // bit 2: a segment to store; bits 0-1: the chunk swizzle
            const uint32_t A = (rowb + 64u * (i ^ (x8 >> 2))) | (x8 & 3u) | (i < nseg ? 4u : 0u);
            uint32_t a[4], g[4];
            quad_bcast4(A, a);
            quad_bcast4(gs + i, g);
            u32x4 val[4];  // (a quad without a segment reads a chunk of its own ring harmlessly)
#pragma unroll
            for (int t = 0; t < 4; ++t) val[t] = *(const lds_u32x4 *)(uintptr_t)((a[t] & ~63u) + 16u * (q ^ (a[t] & 3u)));
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (a[t] & 4u) reinterpret_cast<u32x4 *>(ent + 32ull * g[t])[q] = val[t];
        }
        if (fill > (uint32_t)RG::RING) {
            v = f1;  // [h + RING, f1) went straight to the list
        } else {     // the partial last segment to the ring's start
            if (nq > 0) row[0 ^ x8] = tl0;
            if (nq > 1) row[1 ^ x8] = tl1;
            if (nq > 2) row[2 ^ x8] = tl2;
            if (nq > 3) row[3 ^ x8] = tl3;
        }
        f = f1;
        if (j == 0) {
            W[(par ^ 1u) * RG::NBK + b] = ring_word<K>(b, f1 & 31u);
            gH[b] = P0 + (f1 & ~31u);
        }
        par ^= 1u;
    }

    __device__ void after_iter(int64_t i, int64_t per, bool) {
        if (++held < KMC_RING_RT && i + 1 < per) return;
        held = 0;
        lds_barrier();  // every window of the round is ranked and in its ring
        flush();
        lds_barrier();  // rings read, W set up: the next round may write
    }

    // end of a piece: the partial segment left in the ring, entry by entry
    __device__ __forceinline__ void finish() {
        const uint32_t b = (uint32_t)tid / RG::TPB, j = (uint32_t)tid % RG::TPB;
        const uint32_t h = f & ~31u;
        const uint32_t lo = h > v ? h : v;
        for (uint32_t g = lo + j; g < f; g += RG::TPB) ent[P0 + g] = ring_entry(b, h, g);
    }
};

// R3 launch: the piece walk of radix_count_kernel with the ring scatter (the whole
// LDS of a CU: one 1024-thread workgroup per CU).
template <int K, class Idx>
__global__ __launch_bounds__(1024) void radix_ring_kernel(RParams p) {
    using RG = RingGeom<K>;
    constexpr int NWAVES = RG::BLOCK / 64;
    __shared__ __attribute__((aligned(16))) uint16_t s_ring[RG::NBK * RG::RING];
    __shared__ uint32_t s_W[2 * RG::NBK];
    __shared__ unsigned long long s_gH[RG::NBK];
    __shared__ uint16_t s_dummy[128];
    __shared__ int64_t s_first;

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
    const uint32_t b = (uint32_t)tid / RG::TPB;
    for (int64_t s = s_first; s < p.n; ++s) {
        if (rec_off<Idx>(p, s) >= R1) break;
        int64_t ca, ce;
        record_windows<K, Idx>(p, g, s, ca, ce);
        const int64_t ps = ca > R0 ? ca : R0;
        const int64_t pe = ce < R1 ? ce : R1;
        if (ps >= pe) continue;
        RRingOp<K> op;
        op.ring = s_ring;
        op.W = s_W;
        op.gH = s_gH;
        op.dummy = s_dummy;
        op.ent = p.ent;
        op.tid = tid;
        op.lane = lane;
        op.par = 0;
        op.begin(b, p.off[((s * RG::NBK) + b) * p.G + w], (uint32_t)tid % RG::TPB == 0);  // this workgroup's segment of list (s, b)
        __syncthreads();
        const int64_t tp0 = ps >> kTileShift;
        const int64_t tp1 = ((pe - 1) >> kTileShift) + 1;
        const int64_t per = (tp1 - tp0 + NWAVES - 1) / NWAVES;
        const int64_t a0 = tp0 + (int64_t)wave * per;
        const int64_t a1 = (a0 + per) < tp1 ? (a0 + per) : tp1;
        stream_tiles<K, RRingOp<K>, KMC_RSCAT_PF, 0>(p.data, a0, a1, per, ps, pe, g.rl, g.rh, lane, op);
        op.finish();
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
        for (; i + (KMC_R4_U - 1) * 1024 < nvec; i += KMC_R4_U * 1024) {
            uint4 x[KMC_R4_U];
#pragma unroll
            for (int u = 0; u < KMC_R4_U; ++u) x[u] = ld(i + 1024u * u);
#pragma unroll
            for (int u = 0; u < KMC_R4_U; ++u) add8(x[u]);
        }
        for (; i < nvec; i += 1024) add8(v[i]);
        const uint64_t t = a + nvec * 8;
        if (t + threadIdx.x < end) add(ent[t + threadIdx.x]);
    }
}

// Cold path of R4 (LOW = 16): the list recounted exactly in two 32 768-bin
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
                hist_recount<LOW>(p.ent, beg, end, h, dst);
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
    uint64_t *bsum = reinterpret_cast<uint64_t *>(base + L.bsum);
    const int64_t nbins = (int64_t)1 << (2 * K);

    if (t_trace_before) {
        he = hipEventRecord(t_trace_before, st);
        if (he != hipSuccess) return (int)he;
    }
    he = hipMemsetAsync(p.cnt, 0, (size_t)L.m * 4, st);
    if (he != hipSuccess) return (int)he;
    hipLaunchKernelGGL((radix_count_kernel<K, int64_t>), dim3(G), dim3(1024), 0, st, p);
    excl_scan_u32(p.cnt, L.m, bsum, p.off, st);
    hipLaunchKernelGGL((radix_ring_kernel<K, int64_t>), dim3(G), dim3(1024), 0, st, p);
    hipLaunchKernelGGL((radix_hist_kernel<low_bits(K)>), dim3((unsigned)std::min<int64_t>(n * p.nbk, kMaxGridX)),
                       dim3(1024), 0, st, p, nbins);
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
