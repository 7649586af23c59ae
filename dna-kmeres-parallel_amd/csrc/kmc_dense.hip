// kmc_dense.hip — dense k-mer histogram kernels for gfx950 (MI355X, CDNA4).
//
// Replaces sumKmereCoincidencesGlobalMemory (reference kernels.h:113-144), which
// gives one block per record and one thread per pattern, every thread rescanning
// its record with 3-byte compares.  Here one pass reads every byte once:
//
//   HBM --dwordx4--> lane registers: 16 ASCII bases per lane per tile (1 KiB/wave)
//       --SWAR-----> 32-bit 2-bit-packed codes (first base in the low bits, i.e.
//                    the reference's little-endian bin order) + 16-bit invalid mask
//       --shfl-----> the next lane's codes as the (k-1)-base halo
//       --bfe------> 16 window codes per lane, one LDS atomic each
//       --flush----> per-record histogram, written once (direct or via slab reduce)
//
// Layout of the work: the buffer is cut into 1 KiB tiles; workgroup w owns a
// contiguous tile range and walks the records intersecting it ("pieces").  A
// piece covering a whole record is written straight to sum[]; the (at most two)
// partial pieces of a workgroup go to a slab, summed per record by
// reduce_dense_kernel.  No global atomics on the hot path.
//
// Histogram storage per workgroup (LDS):
//   k <= 7 : 32-bit counters, R replicas interleaved (bin*R + lane%R) so lanes of a
//            32-lane LDS group never collide on small alphabets (k <= 4: R = 32).
//   k == 8 : 65 536 bins do not fit as 32-bit (256 KB > 160 KB LDS): two 16-bit
//            counters per word (bin c in the low half, c|0x8000 in the high
//            half), plain adds; periodic scans move hot halves to spill entries,
//            a piece whose halves wrapped anyway is recounted with returning adds
//            (every wrap recorded as a spill entry), and reduce_dense_kernel adds
//            the spill entries of every record back.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "kmc.h"
#include "kmc_internal.h"
#include "kmc_stream.h"

namespace kmc {
// k == 8, HM 3: tiles per wave between two scans that move hot 16-bit halves to
// spill entries (section 4.1 of DESIGN.md: 64 / 256 / 512 / 1 024 measured)
constexpr int kHm3Scan = 256;
// k >= 7: tiles per chunk of the workgroup's shared tile counter (stream_chunks,
// round 5).  Same box, kernel alone over 10 Gbase (profiles/r05o_chunk_ab.txt):
// k = 8 2.242 ms with one contiguous run per wave, 2.15 / 2.07-2.09 / 2.05-2.07 /
// 2.05-2.08 ms with chunks of 4 / 8 / 16 / 32 tiles; k = 7 2.14 -> 2.06 (16); k <= 6
// (HBM-bound, the more VGPRs of the chunked loop cost one wave per SIMD) keep the
// contiguous runs: k = 4 1.77-1.79 against 1.84-1.92 ms chunked.
constexpr int kChunk = 16;
thread_local hipEvent_t t_trace_before = nullptr;
thread_local hipEvent_t t_trace_after = nullptr;
namespace {

struct Spill {
    int64_t rec;
    int32_t code;
    int32_t amount;
};

struct Params {
    const char *data;        // 16-byte aligned (the caller's pointer rounded down)
    const void *indices;
    int64_t ibias;           // added to every indices[] value: the caller's misalignment
    int64_t n;
    int32_t *sum;
    int64_t ld;
    int32_t *invalid;
    int64_t wl, wh, rl, rh;  // window range, readable range (derive == 0)
    int derive;              // 1: both ranges = [indices[0], indices[n])
    int G;                   // workgroups of the count kernel
    uint32_t *slab;          // [G][2][4^k] (k = 8: the first 4^k / 2 words, packed 16-bit halves)
    int64_t *slot_rec;       // [G][2] record held by each slab slot, -1 = none
    Spill *spill;            // [G][spill_cap]
    uint32_t *spill_cnt;     // [G]
    uint32_t spill_cap;
    uint32_t *status;        // the call's status word (kmc_dense_args::status, or the device's host-mapped
                             // kmc_dense_status flag): a kmc_status code when the counts are not valid
};

// Store a kmc_status code in the call's status word (a plain system-scope store:
// the word may be host-mapped; any nonzero code marks the call failed).
__device__ __forceinline__ void raise_status(uint32_t *st, uint32_t code) {
    if (st) __hip_atomic_store(st, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// 1 or 0x10000 from bit `hb` (0/1): one v_mad_u32_u24 (hipcc otherwise emits
// and + cmp + cndmask for the same select).
__device__ __forceinline__ uint32_t half_inc(uint32_t hb) {
    uint32_t r;
    asm("v_mad_u32_u24 %0, %1, %2, 1" : "=v"(r) : "v"(hb), "s"(0xFFFFu));
    return r;
}

// Per-piece context of the k == 8 packed-16-bit histogram.
struct P16Ctx {
    uint32_t *h;
    uint32_t *spilled;  // LDS: increments moved to spill entries by scans (this piece)
    uint32_t *spill_n;  // LDS counter
    Spill *spill;       // this workgroup's slice
    uint32_t cap;
    int64_t rec;
};

__device__ __forceinline__ void p16_spill(const P16Ctx &c, int32_t code, int32_t amount) {
    const uint32_t i = atomicAdd(c.spill_n, 1u);
    if (i < c.cap) {
        Spill e;
        e.rec = c.rec;
        e.code = code;
        e.amount = amount;
        c.spill[i] = e;
    }
}

// A half of a packed word wrapped (the returned old value had 0xFFFF in the half
// that was incremented): record the exact correction, and undo a carry from the
// low half into the high half.  Every wrap of either 16-bit field is observed
// exactly once, by the atomic that caused it (forward: the add that saw 0xFFFF;
// backward: the carry removal that saw 0), so the spill entries plus the final
// field values reconstruct the true counts for any interleaving of the waves.
//   hb      1 if the window incremented the high half
//   hiwrap  the low-half add also found the high half at 0xFFFF (carry wrapped it)
__device__ __noinline__ void p16_fix(const P16Ctx &c, uint32_t word, uint32_t hb, uint32_t hiwrap) {
    if (hb == 0u) {
        p16_spill(c, (int32_t)word, 65536);
        if (hiwrap) p16_spill(c, (int32_t)(word | 0x8000u), 65536);
        const uint32_t o2 = __hip_atomic_fetch_add(&c.h[word], 0xFFFF0000u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((o2 >> 16) == 0u) p16_spill(c, (int32_t)(word | 0x8000u), -65536);
    } else {
        p16_spill(c, (int32_t)(word | 0x8000u), 65536);
    }
}

// Code of window j (0..15) of a lane whose bases are lo (own 16) : hi (next 16).
template <int K, int J>
__device__ __forceinline__ uint32_t window_code(uint32_t lo, uint32_t mid) {
    constexpr uint32_t M = (K == 16) ? 0xFFFFFFFFu : ((1u << (2 * K)) - 1u);
    if constexpr (J <= 16 - K)
        return (lo >> (2 * J)) & M;
    else
        return (mid >> (2 * (J - 8))) & M;
}

template <int K, int R, int J, bool MASKED>
__device__ __forceinline__ void add32(uint32_t lo, uint32_t mid, uint32_t W, uint32_t *h, uint32_t rep) {
    const uint32_t code = window_code<K, J>(lo, mid);
    if (!MASKED || ((W >> J) & 1u))
        __hip_atomic_fetch_add(&h[code * R + rep], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int K, int R, bool MASKED>
__device__ __forceinline__ void count_tile32(uint32_t lo, uint32_t hi, uint32_t W, uint32_t *h, int lane) {
    const uint32_t mid = __builtin_amdgcn_alignbit(hi, lo, 16);  // bases 8..23
    const uint32_t rep = (uint32_t)(lane & (R - 1));
    add32<K, R, 0, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 1, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 2, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 3, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 4, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 5, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 6, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 7, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 8, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 9, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 10, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 11, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 12, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 13, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 14, MASKED>(lo, mid, W, h, rep);
    add32<K, R, 15, MASKED>(lo, mid, W, h, rep);
}

// k == 8, packed 16-bit halves, plain adds (HM == 3): a half that reaches 32 768
// is moved to a spill entry by the periodic scans (p16_scan), a wrap between two
// scans is detected by the piece total and the piece recounted (recount_p16).
template <bool MASKED>
__device__ __forceinline__ void count_tile_p16_plain(uint32_t lo, uint32_t hi, uint32_t W, uint32_t *h) {
    const uint32_t mid = __builtin_amdgcn_alignbit(hi, lo, 16);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t src = (j <= 8) ? lo : mid;
        const int off = (j <= 8) ? 2 * j : 2 * (j - 8);
        const uint32_t word = (src >> off) & 0x7FFFu;
        const uint32_t hb = (src >> (off + 15)) & 1u;
        if (!MASKED || ((W >> j) & 1u))
            __hip_atomic_fetch_add(&h[word], half_inc(hb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

template <int K, int R, int HM, bool MASKED>
__device__ __forceinline__ void count_tile(uint32_t lo, uint32_t hi, uint32_t W, uint32_t *h, int lane) {
    if constexpr (HM == 3)
        count_tile_p16_plain<MASKED>(lo, hi, W, h);
    else
        count_tile32<K, R, MASKED>(lo, hi, W, h, lane);
}

// Cold path of the scan: move every half's multiple of T of 4 words into spills.
template <uint32_t T>
__device__ __noinline__ void p16_scan_fix(const P16Ctx &pc, int i4) {
    uint32_t *w = pc.h + 4 * i4;
    for (int q = 0; q < 4; ++q) {
        const uint32_t word = (uint32_t)(4 * i4 + q);
        const uint32_t x = w[q];
        const uint32_t lo = x & 0xFFFFu, hi = x >> 16;
        if (lo >= T) {
            p16_spill(pc, (int32_t)word, (int32_t)(lo & ~(T - 1)));
            atomicAdd(pc.spilled, lo & ~(T - 1));
        }
        if (hi >= T) {
            p16_spill(pc, (int32_t)(word | 0x8000u), (int32_t)(hi & ~(T - 1)));
            atomicAdd(pc.spilled, hi & ~(T - 1));
        }
        w[q] = (lo & (T - 1)) | ((hi & (T - 1)) << 16);
    }
}

template <int BLOCK, uint32_t T>
__device__ __forceinline__ void p16_scan(const P16Ctx &pc) {
    constexpr uint32_t HOT = (0xFFFFu & ~(T - 1)) * 0x00010001u;  // bits >= T in both halves
    constexpr int NW4 = (1 << 15) / 4;  // 32768 words as uint4
    const uint4 *h4 = reinterpret_cast<const uint4 *>(pc.h);
    uint32_t hot = 0u;  // bit i: chunk threadIdx.x + i*BLOCK has a half >= T
#pragma unroll
    for (int i = 0; i < NW4 / BLOCK; ++i) {
        const uint4 v = h4[threadIdx.x + i * BLOCK];
        hot |= (uint32_t)(((v.x | v.y | v.z | v.w) & HOT) != 0u) << i;
    }
    if (hot) {
        for (int i = 0; i < NW4 / BLOCK; ++i)
            if ((hot >> i) & 1u) p16_scan_fix<T>(pc, (int)threadIdx.x + i * BLOCK);
    }
}

// The dense histogram as a stream_tiles operation (HM 0: 32-bit bins, HM 3: k = 8
// packed 16-bit halves).
template <int K, int R, int HM, int BLOCK>
struct DenseOp {
    static_assert(HM == 0 || HM == 3, "histogram modes: 0 (32-bit bins) and 3 (k = 8 packed halves)");
    uint32_t *h;
    int lane;
    const P16Ctx &pc;
    uint32_t nwin = 0u;  // HM 3: windows this lane added

    __device__ DenseOp(uint32_t *h_, int lane_, const P16Ctx &pc_) : h(h_), lane(lane_), pc(pc_) {}

    __device__ __forceinline__ void before_tile() {}
    template <bool MASKED>
    __device__ __forceinline__ void tile(uint32_t lo, uint32_t hi, uint32_t W) {
        count_tile<K, R, HM, MASKED>(lo, hi, W, h, lane);
        if constexpr (HM == 3) nwin += MASKED ? (uint32_t)__builtin_popcount(W) : 16u;
    }
    // HM 3: hot halves (>= 32768) go to spill entries every kHm3Scan tiles per
    // wave (stream_chunks' segments), so a half wraps only if one k-mer takes
    // >= 32768 of the workgroup's NWAVES * kHm3Scan * 1024 windows in between (long
    // low-complexity runs); wraps stay detected by the piece total
    __device__ __forceinline__ void segment_end() {
        if constexpr (HM == 3) {
            lds_barrier();
            p16_scan<BLOCK, 32768u>(pc);
            lds_barrier();
        }
    }
    static constexpr int kSegChunks = HM == 3 ? BLOCK / 64 * kHm3Scan / kChunk : 0;
    __device__ __forceinline__ void after_iter(int64_t, int64_t, bool) {}  // (k <= 6: stream_tiles)
};

// HM 3's exact recount of the windows [ps, pe) of a piece whose 16-bit halves
// wrapped (skewed input only): returning adds, every wrap fixed up by p16_fix, over
// a plain rolling-code walk of a contiguous run of windows per thread, out of line
// (a returning-add tile stream inlined beside the hot loop made the kernel spill
// VGPRs).  Bytes outside [rl, rh) are invalid, as in load_lane.
template <int BLOCK>
__device__ __noinline__ void recount_p16(const char *data, int64_t ps, int64_t pe, int64_t rl, int64_t rh,
                                         const P16Ctx &pc) {
    constexpr int K = 8;
    const int64_t per = (pe - ps + BLOCK - 1) / BLOCK;
    const int64_t i0 = ps + (int64_t)threadIdx.x * per;
    const int64_t i1 = (i0 + per) < pe ? (i0 + per) : pe;
    uint32_t code = 0u, run = 0u;
    for (int64_t b = i0; b < i1 + K - 1; ++b) {
        const uint32_t c = (b >= rl && b < rh) ? (uint32_t)(uint8_t)data[b] : 0u;
        const uint32_t v = c == 'A' ? 0u : c == 'C' ? 1u : c == 'G' ? 2u : c == 'T' ? 3u : 4u;
        run = v < 4u ? run + 1u : 0u;
        code = (code >> 2) | ((v & 3u) << (2 * K - 2));  // base b at bits 14..15 (LE order)
        if (run >= (uint32_t)K) {                          // window b - K + 1 in [i0, i1)
            const uint32_t word = code & 0x7FFFu, hb = code >> 15;
            const uint32_t old = __hip_atomic_fetch_add(&pc.h[word], half_inc(hb), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t m = hb ? 0xFFFF0000u : 0x0000FFFFu;
            if ((old & m) == m) p16_fix(pc, word, hb, old >= 0xFFFF0000u ? 1u : 0u);
        }
    }
}

template <int K, int R, int HM, class Idx, int BLOCK>
__global__ __launch_bounds__(BLOCK) void count_dense_kernel(Params p) {
    constexpr bool P16 = HM != 0;
    constexpr int NB = 1 << (2 * K);
    constexpr int NW = P16 ? NB / 2 : NB * R;
    // static LDS: the histogram's address is a link-time constant, folded into the
    // ds_add offset (dynamic LDS costs one v_add per window)
    __shared__ __attribute__((aligned(16))) uint32_t smem[NW + 8];
    uint32_t *h = smem;
    uint32_t *misc = smem + NW;  // [0] spill count, [1],[2] first record, [3] windows added, [4] decoded sum

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = blockIdx.x;
    const Geom g = make_geom<Idx>(p);
    const int64_t tb = g.T0 + (int64_t)w * g.tpw;
    const int64_t te = (tb + g.tpw) < g.T1 ? (tb + g.tpw) : g.T1;
    int64_t slot0 = -1, slot1 = -1;

    if (tb < te) {
        const int64_t R0 = (tb << kTileShift) > g.wl ? (tb << kTileShift) : g.wl;
        const int64_t R1 = (te << kTileShift) < g.wh ? (te << kTileShift) : g.wh;
        int64_t s0 = 0;
        // (round 4: the first record found by one load per thread when n <= BLOCK,
        // the LDS cleared and the slab flushed 16 bytes per lane: the fixed part of a
        // launch, which an 8-way shard's step pays on 1/8 of the work)
        if (p.n <= BLOCK) {
            // last record s with indices[s] <= R0 (records before it end before R0;
            // the offsets are sorted): the number of such records, less one
            if (tid == 0) {
                misc[0] = 0u;
                misc[3] = 0u;
                misc[4] = 0u;
                misc[5] = 0u;
                misc[7] = 0u;
            }
            const bool le = tid < p.n && rec_off<Idx>(p, tid) <= R0;
            for (int i = tid; i < NW / 4; i += BLOCK) reinterpret_cast<uint4 *>(h)[i] = make_uint4(0u, 0u, 0u, 0u);
            const int cnt = __syncthreads_count(le);
            s0 = cnt > 0 ? cnt - 1 : 0;
        } else {
            if (tid == 0) {
                // last record s with indices[s] <= R0 (records before it end before R0)
                int64_t lo = 0, hi = p.n - 1;
                if (rec_off<Idx>(p, 0) <= R0) {
                    while (lo < hi) {
                        const int64_t mid = (lo + hi + 1) >> 1;
                        if (rec_off<Idx>(p, mid) <= R0) lo = mid;
                        else hi = mid - 1;
                    }
                }
                misc[0] = 0u;
                misc[3] = 0u;
                misc[4] = 0u;
                misc[5] = 0u;
                misc[7] = 0u;
                misc[1] = (uint32_t)lo;
                misc[2] = (uint32_t)((uint64_t)lo >> 32);
            }
            for (int i = tid; i < NW / 4; i += BLOCK) reinterpret_cast<uint4 *>(h)[i] = make_uint4(0u, 0u, 0u, 0u);
            __syncthreads();
            s0 = (int64_t)((uint64_t)misc[1] | ((uint64_t)misc[2] << 32));
        }

        P16Ctx pc;
        pc.h = h;
        pc.spilled = misc + 5;
        pc.spill_n = misc;
        pc.spill = p.spill ? p.spill + (int64_t)w * p.spill_cap : nullptr;
        pc.cap = p.spill_cap;

        int npieces = 0;
        for (int64_t s = s0; s < p.n; ++s) {
            if (rec_off<Idx>(p, s) >= R1) break;
            int64_t ca, ce;
            record_windows<K, Idx>(p, g, s, ca, ce);
            const int64_t ps = ca > R0 ? ca : R0;
            const int64_t pe = ce < R1 ? ce : R1;
            if (ps >= pe) continue;
            pc.rec = s;
            // this piece's tiles: k >= 7 in chunks taken by the waves as they go
            // (misc[7]: the chunk counter, zero at the piece's start), k <= 6 in one
            // contiguous run per wave
            const int64_t tp0 = ps >> kTileShift;
            const int64_t tp1 = ((pe - 1) >> kTileShift) + 1;
            using Op = DenseOp<K, R, HM, BLOCK>;
            Op op(h, lane, pc);
            if constexpr (K >= 7) {
                stream_chunks<K, kChunk, Op::kSegChunks>(p.data, tp0, tp1, ps, pe, g.rl, g.rh, lane, &misc[7], op);
            } else {
                constexpr int NWAVES = BLOCK / 64;
                const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
                const int64_t per = (tp1 - tp0 + NWAVES - 1) / NWAVES;
                const int64_t a0 = tp0 + (int64_t)wave * per;
                const int64_t a1 = (a0 + per) < tp1 ? (a0 + per) : tp1;
                stream_tiles<K>(p.data, a0, a1, per, ps, pe, g.rl, g.rh, lane, op);
            }
            if constexpr (HM == 3) {
                const uint32_t wsum = wave_sum(op.nwin);
                if (lane == 0) atomicAdd(&misc[3], wsum);
            }
            __syncthreads();
            const bool entire = (ps == ca) && (pe == ce);
            int slot = 0;
            if (!entire) {
                slot = (npieces == 0) ? 0 : 1;
                if (slot == 0) slot0 = s;
                else slot1 = s;
            }
            uint32_t *dst = p.slab + ((int64_t)w * 2 + slot) * NB;
            if constexpr (P16) {
                // the packed words to sum[] (whole record) or the slab (packed as in
                // LDS: the halves are exact, wraps live in spills); the LDS cleared
                const auto flush = [&]() {
                    uint32_t dsum = 0u;
                    if (!entire) {  // the slab: 16 bytes per lane
                        for (int i = tid; i < NW / 4; i += BLOCK) {
                            const uint4 v = reinterpret_cast<const uint4 *>(h)[i];
                            reinterpret_cast<uint4 *>(h)[i] = make_uint4(0u, 0u, 0u, 0u);
                            dsum += (v.x & 0xFFFFu) + (v.x >> 16) + (v.y & 0xFFFFu) + (v.y >> 16) + (v.z & 0xFFFFu) +
                                    (v.z >> 16) + (v.w & 0xFFFFu) + (v.w >> 16);
                            reinterpret_cast<uint4 *>(dst)[i] = v;
                        }
                        return dsum;
                    }
                    for (int i = tid; i < NW; i += BLOCK) {
                        const uint32_t v = h[i];
                        h[i] = 0u;
                        dsum += (v & 0xFFFFu) + (v >> 16);
                        if (entire) {
                            p.sum[s + p.ld * (int64_t)i] = (int32_t)(v & 0xFFFFu);
                            p.sum[s + p.ld * (int64_t)(i + NW)] = (int32_t)(v >> 16);
                        } else {
                            dst[i] = v;
                        }
                    }
                    return dsum;
                };
                const uint32_t dsum = flush();
                if constexpr (HM == 3) {
                    const uint32_t wsum = wave_sum(dsum);
                    if (lane == 0) atomicAdd(&misc[4], wsum);
                    // every 16-bit wrap only loses counts (low half: -65535 net, high
                    // half: -65536), so the decoded total plus the scans' spills equals
                    // the windows added iff none wrapped
                    __syncthreads();
                    if (tid == 0) {
                        misc[6] = misc[3] != misc[4] + misc[5] ? 1u : 0u;
                        misc[3] = 0u;
                        misc[4] = 0u;
                        misc[5] = 0u;
                    }
                    __syncthreads();
                    if (misc[6]) {
                        // a half wrapped (skewed input): recount the piece exactly with
                        // returning adds, in place of a second launch; its scan
                        // entries are superseded (zeroed), the recount's wrap entries
                        // appended after them
                        const uint32_t n0 = misc[0] < pc.cap ? misc[0] : pc.cap;
                        for (uint32_t i = tid; i < n0; i += BLOCK)
                            if (pc.spill[i].rec == s) pc.spill[i].amount = 0;
                        __syncthreads();
                        recount_p16<BLOCK>(p.data, ps, pe, g.rl, g.rh, pc);
                        __syncthreads();
                        (void)flush();
                    }
                }
            } else {
                for (int c = tid; c < NB; c += BLOCK) {
                    uint32_t v = 0;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        v += h[c * R + r];
                        h[c * R + r] = 0u;
                    }
                    if (entire) p.sum[s + p.ld * (int64_t)c] = (int32_t)v;
                    else dst[c] = v;
                }
            }
            if (tid == 0) misc[7] = 0u;  // (every wave's last take of this piece is behind the barrier after it)
            __syncthreads();
            ++npieces;
        }
    }
    if (tid == 0) {
        p.slot_rec[2 * w] = slot0;
        p.slot_rec[2 * w + 1] = slot1;
        if (p.spill_cnt) {
            p.spill_cnt[w] = (tb < te) ? misc[0] : 0u;
            // never expected (spill_cap_for bounds the entries), but a lost entry
            // would be a silent short count: raise the deferred status flag
            if (tb < te && misc[0] > p.spill_cap) raise_status(p.status, KMC_ERR_CAPACITY);
        }
    }
}

// Records that span several workgroups: sum their slab slots; records without a
// window in range get zeros.  Grid (NW / RW, ny): blockIdx.x picks RW = 4 * RC
// slab words (NW = 4^k words, or 4^k / 2 packed words at k = 8, each holding bins
// c and c | 0x8000), records s = blockIdx.y, blockIdx.y + ny, ...  RC columns of
// 16-byte loads x RR rows of slots sum a record's slots with no dependent load in
// the loop, and the rows meet in LDS.  The slots follow from the geometry: record s
// spans workgroups wf < wlast, each of wf + 1 .. wlast holds it as its first piece
// (slot 0: its range starts inside s), and wf in slot 0 or 1 as slot_rec says.
// (One thread per word walking the workgroups with a slot_rec test before every
// slab load was latency-bound: 72 us for the ~205 slots of an 8-way shard's
// record, against a 325 us histogram; listing the slots from slot_rec in LDS first
// cost a round trip and two barriers per record.)
template <int K, class Idx, bool P16>
__global__ __launch_bounds__(256) void reduce_dense_kernel(Params p) {
    constexpr int NB = 1 << (2 * K);
    constexpr int NW = P16 ? NB / 2 : NB;
    constexpr int RC = NW / 4 < 16 ? NW / 4 : 16;  // 16-byte columns
    constexpr int RR = 256 / RC;                   // rows over the slots
    constexpr int RW = 4 * RC;                     // words per block
    constexpr int NH = P16 ? 2 : 1;                // counters per word
    __shared__ uint32_t s_part[RR][RW * NH];
    __shared__ uint32_t s_out[RW * NH];
    const int tid = threadIdx.x, col = tid % RC, row = tid / RC;
    const int64_t c0 = (int64_t)blockIdx.x * RW;
    const Geom g = make_geom<Idx>(p);
    // k = 8: the spill entries (halves moved out of 16-bit counters, wrap fix-ups)
    // of record s that fall in this block's words, from the lists of the workgroups
    // [wf, wlast] that hold its pieces; f(index into s_out layout, amount).  Only
    // when one of those lists is non-empty (skewed input).  A workgroup walks its
    // pieces in record order and appends a piece's entries before the next piece
    // starts, so every list is sorted by rec: a binary search finds s's entries,
    // and a list holding many records' entries costs each record only its own.
    const auto for_spills = [&](int64_t s, int64_t wf, int64_t wlast, auto &&f) {
        for (int64_t l = wf; l <= wlast; ++l) {
            const uint32_t c = p.spill_cnt[l] < p.spill_cap ? p.spill_cnt[l] : p.spill_cap;
            const Spill *sp = p.spill + l * (int64_t)p.spill_cap;
            uint32_t lo = 0u, hi = c;  // first entry with rec >= s (wave-uniform search)
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (sp[mid].rec < s) lo = mid + 1u;
                else hi = mid;
            }
            for (uint32_t i = lo + tid; i < c; i += 256) {
                const Spill e = sp[i];
                if (e.rec != s) break;
                const int64_t wd = (int64_t)(e.code & (NW - 1)) - c0;
                if (e.amount != 0 && wd >= 0 && wd < RW) f((int)wd + (e.code / NW) * RW, e.amount);
            }
        }
    };
    for (int64_t s = blockIdx.y; s < p.n; s += gridDim.y) {
        int64_t ca, ce;
        record_windows<K, Idx>(p, g, s, ca, ce);
        // int32 bins (and invalid counts) of a record with >= 2^31 windows in range
        // could wrap (the reference's int counters, main.cu:637, never see one)
        if (blockIdx.x == 0 && tid == 0 && ce - ca >= ((int64_t)1 << 31)) raise_status(p.status, KMC_ERR_RECORD_TOO_LONG);
        if (ce <= ca) {
            for (int i = tid; i < RW * NH; i += 256) {
                const int64_t c = c0 + i % RW + (i / RW) * NW;
                p.sum[s + p.ld * c] = 0;
            }
            continue;
        }
        const int64_t wf = ((ca >> kTileShift) - g.T0) / g.tpw;
        const int64_t wlast = (((ce - 1) >> kTileShift) - g.T0) / g.tpw;
        bool spills = false;
        if constexpr (P16) {
            uint32_t any = 0u;
            for (int64_t l = wf + tid; l <= wlast; l += 256) any |= p.spill_cnt[l];
            spills = __syncthreads_or(any != 0u) != 0;
        }
        if (wf == wlast) {  // written directly by the count kernel: its spills on top
            if (spills)
                for_spills(s, wf, wlast, [&](int i, int32_t a) {
                    atomicAdd(&p.sum[s + p.ld * (c0 + i % RW + (i / RW) * (int64_t)NW)], a);
                });
            continue;
        }
        uint32_t acc[4 * NH] = {};
        // slot of workgroup wf + i: 2 (wf + i) for i > 0; wf's first or second
        const int64_t sf = 2 * wf + (p.slot_rec[2 * wf] == s ? 0 : 1);
        const int64_t n = wlast - wf + 1;
#pragma unroll 4
        for (int64_t i = row; i < n; i += RR) {
            const int64_t slot = i == 0 ? sf : 2 * (wf + i);
            const uint4 v = reinterpret_cast<const uint4 *>(p.slab + slot * NB + c0)[col];
            const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if constexpr (P16) {
                    acc[e] += x[e] & 0xFFFFu;  // bin c
                    acc[4 + e] += x[e] >> 16;  // bin c + NW
                } else {
                    acc[e] += x[e];
                }
            }
        }
#pragma unroll
        for (int e = 0; e < 4 * NH; ++e) s_part[row][(e / 4) * RW + col * 4 + e % 4] = acc[e];
        __syncthreads();
        for (int i = tid; i < RW * NH; i += 256) {
            uint32_t t = 0u;
#pragma unroll 8
            for (int r = 0; r < RR; ++r) t += s_part[r][i];
            s_out[i] = t;
        }
        if (spills) {
            __syncthreads();
            for_spills(s, wf, wlast, [&](int i, int32_t a) { atomicAdd(&s_out[i], (uint32_t)a); });
        }
        __syncthreads();
        for (int i = tid; i < RW * NH; i += 256) {
            const int64_t c = c0 + i % RW + (i / RW) * NW;
            p.sum[s + p.ld * c] = (int32_t)s_out[i];
        }
        __syncthreads();  // s_part and s_out are reused by the next record
    }
}


// invalid[s] = (#windows of s in range) - sum over codes (the CPU path's bin 0);
// records blockIdx.x, blockIdx.x + gridDim.x, ...
template <int K, class Idx>
__global__ __launch_bounds__(256) void invalid_kernel(Params p) {
    constexpr int NB = 1 << (2 * K);
    __shared__ int64_t red[256];
    for (int64_t s = blockIdx.x; s < p.n; s += gridDim.x) {
        int64_t acc = 0;
        for (int c = threadIdx.x; c < NB; c += 256) acc += p.sum[s + p.ld * (int64_t)c];
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
            p.invalid[s] = (int32_t)(nw - red[0]);
        }
        __syncthreads();  // red is reused by the next record
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
template <int K>
struct Cfg;
// R = replicas of each 32-bit bin; BLOCK = threads per workgroup
// HM = histogram mode: 0 = 32-bit bins; 3 = k == 8 packed 16-bit halves, plain adds
//   + periodic hot-half scans + wrap detection by total, pieces that wrapped
//   recounted with returning adds (round 1 also had returning adds throughout and
//   scans every 3 tiles as modes 1 and 2; both measured slower and were removed).
template <> struct Cfg<1> { static constexpr int R = 32, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<2> { static constexpr int R = 32, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<3> { static constexpr int R = 32, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<4> { static constexpr int R = 32, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<5> { static constexpr int R = 8, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<6> { static constexpr int R = 2, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<7> { static constexpr int R = 1, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<8> { static constexpr int R = 1, BLOCK = 1024, HM = 3; static constexpr bool P16 = true; };

struct DevInfo {
    int cus = 0;
    int occ[KMC_DENSE_MAX_K + 1][2] = {};  // [k][idx64]
    uint32_t *status_host = nullptr;       // kmc_dense_status flag (host-mapped, allocated on first use)
    uint32_t *status_dev = nullptr;
};

std::mutex g_mu;
std::vector<DevInfo> g_dev;


template <int K, class Idx>
void *kernel_ptr() {
    return reinterpret_cast<void *>(&count_dense_kernel<K, Cfg<K>::R, Cfg<K>::HM, Idx, Cfg<K>::BLOCK>);
}

// CUs left out of the dense grid (kmc_set_reserved_cus), per host thread
thread_local int t_reserved_cus = 0;

#ifdef KMC_DIAG_HOOKS
// test hook (diagnostic library only): spill list capacity per workgroup (0: the bound)
std::atomic<uint32_t> g_diag_spill_cap{0};
#endif

template <int K, class Idx>
int grid_size(int device, int &G) {
    std::lock_guard<std::mutex> lk(g_mu);
    if ((int)g_dev.size() <= device) g_dev.resize(device + 1);
    DevInfo &d = g_dev[device];
    if (d.cus == 0) {
        int v = 0;
        hipError_t e = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device);
        if (e != hipSuccess) return (int)e;
        d.cus = v;
    }
    const int ix = sizeof(Idx) == 8 ? 1 : 0;
    if (d.occ[K][ix] == 0) {
        const void *kp = kernel_ptr<K, Idx>();
        int nb = 0;  // the histogram is static LDS, accounted by the query itself
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kp, Cfg<K>::BLOCK, 0);
        if (e != hipSuccess) return (int)e;
        d.occ[K][ix] = nb > 0 ? nb : 1;
    }
    // kmc_set_reserved_cus: leave that many CUs to a concurrent kernel
    const int cus = d.cus - t_reserved_cus;
    G = (cus > 0 ? cus : 1) * d.occ[K][ix];
    return 0;
}

// The device's kmc_dense_status flag: host-mapped, written by the dense kernels of
// the calls that pass no status word of their own.
int status_flag(int device, uint32_t **host, uint32_t **dev) {
    std::lock_guard<std::mutex> lk(g_mu);
    if ((int)g_dev.size() <= device) g_dev.resize(device + 1);
    DevInfo &d = g_dev[device];
    if (!d.status_host) {
        void *h = nullptr;
        hipError_t e = hipHostMalloc(&h, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) return KMC_ERR_NOMEM;
        void *dp = nullptr;
        e = hipHostGetDevicePointer(&dp, h, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(h);
            return (int)e;
        }
        *static_cast<volatile uint32_t *>(h) = 0u;
        d.status_host = static_cast<uint32_t *>(h);
        d.status_dev = static_cast<uint32_t *>(dp);
    }
    *host = d.status_host;
    *dev = d.status_dev;
    return 0;
}

// Read and clear the flag of `device` (no device call).
int take_status(int device) {
    uint32_t *h = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if ((int)g_dev.size() > device && device >= 0) h = g_dev[device].status_host;
    }
    if (!h) return KMC_OK;
    const uint32_t v = __atomic_exchange_n(h, 0u, __ATOMIC_ACQ_REL);
    return (int)v;  // the code a kernel stored, KMC_OK if none
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct WsLayout {
    size_t slot_rec, spill_cnt, slab, spill, total;
};

inline WsLayout ws_layout(int k, int G, uint32_t spill_cap) {
    WsLayout L;
    const size_t nb = (size_t)1 << (2 * k);
    size_t o = 0;
    L.slot_rec = o;
    o += align256((size_t)G * 2 * sizeof(int64_t));
    L.spill_cnt = o;
    o += align256((size_t)G * sizeof(uint32_t));
    L.slab = o;
    o += align256((size_t)G * 2 * nb * sizeof(uint32_t));
    L.spill = o;
    o += align256((size_t)G * spill_cap * sizeof(Spill));
    L.total = o;
    return L;
}

// Upper bound of the spill entries one workgroup can emit for `tiles` tiles: a
// scan entry (HM 2) stands for >= T >= 4096 increments of one 16-bit field; a wrap
// entry (HM 1) for 65 536, or pairs with one.
// Entries per window, whatever the scan interval: a scan entry (HM 3 / HM 2) moves
// a multiple of its threshold T >= 32768 (HM 3) or >= 4096 (HM 2) out of one field,
// all of it increments of that field since its last scan; a wrap of the HM 1 recount
// costs 65 536 increments and emits at most 3 entries.  The recount keeps the first
// pass's scan entries (zeroed) beside its own, so HM 3 + recount emits at most
// windows * (1/32768 + 3/65536) = windows * 5/65536 <= windows / 4096 entries.
constexpr uint32_t kSpillWindowsPerEntry = 4096;
static_assert(5u * kSpillWindowsPerEntry <= 65536u, "HM 3 scan + HM 1 recount entries exceed the spill cap");
inline uint32_t spill_cap_for(int64_t tiles_per_wg) {
    const int64_t windows = tiles_per_wg * kTile;
    return (uint32_t)(windows / kSpillWindowsPerEntry + 64);
}

struct Plan {
    int G;
    uint32_t spill_cap;
    WsLayout L;
};

template <int K, class Idx>
int make_plan(int device, bool derive, int64_t wl, int64_t wh, Plan &pl) {
    int G = 0;
    int e = grid_size<K, Idx>(device, G);
    if (e) return e;
    pl.spill_cap = 0;
    if (!derive) {
        const int64_t tiles = wh > wl ? ((wh + kTile - 1) >> kTileShift) - (wl >> kTileShift) : 0;
        if (tiles < G) G = tiles > 0 ? (int)tiles : 1;
        const int64_t tpw = tiles > 0 ? (tiles + G - 1) / G : 1;
        if (Cfg<K>::P16) {
            pl.spill_cap = spill_cap_for(tpw);
#ifdef KMC_DIAG_HOOKS
            const uint32_t dc = g_diag_spill_cap.load();
            if (dc) pl.spill_cap = dc;
#endif
        }
    }
    pl.G = G;
    pl.L = ws_layout(K, G, pl.spill_cap);
    return 0;
}

// library-owned workspace, per device
struct WsCache {
    void *ptr = nullptr;
    size_t bytes = 0;
};
std::vector<WsCache> g_ws;

int cached_workspace(int device, size_t need, void **out) {
    std::lock_guard<std::mutex> lk(g_mu);
    if ((int)g_ws.size() <= device) g_ws.resize(device + 1);
    WsCache &c = g_ws[device];
    if (c.bytes < need) {
        if (c.ptr) {
            hipError_t e = hipFree(c.ptr);
            if (e != hipSuccess) return (int)e;
            c.ptr = nullptr;
            c.bytes = 0;
        }
        hipError_t e = hipMalloc(&c.ptr, need);
        if (e != hipSuccess) return KMC_ERR_NOMEM;
        c.bytes = need;
    }
    *out = c.ptr;
    return 0;
}

struct Request {
    const char *data;        // 16-byte aligned
    const void *indices;
    int64_t ibias;           // see Params
    int64_t n;
    int32_t *sum;
    int64_t ld;
    int32_t *invalid;
    bool derive;
    int64_t wl, wh, rl, rh;
    void *ws;
    size_t ws_bytes;
    uint32_t *status;        // the call's status word (NULL: the device's flag)
};

template <int K, class Idx>
int run_dense(const Request &q, hipStream_t st) {
    int device = 0;
    hipError_t he = hipGetDevice(&device);
    if (he != hipSuccess) return (int)he;
    bool derive = q.derive;
    int64_t wl = q.wl, wh = q.wh, rl = q.rl, rh = q.rh;
    if (derive && Cfg<K>::P16) {
        // the packed layout sizes its spill area from the range: read it once
        Idx ends[2];
        he = hipMemcpyAsync(&ends[0], q.indices, sizeof(Idx), hipMemcpyDeviceToHost, st);
        if (he == hipSuccess)
            he = hipMemcpyAsync(&ends[1], (const Idx *)q.indices + q.n, sizeof(Idx), hipMemcpyDeviceToHost, st);
        if (he == hipSuccess) he = hipStreamSynchronize(st);
        if (he != hipSuccess) return (int)he;
        wl = rl = (int64_t)ends[0] + q.ibias;
        wh = rh = (int64_t)ends[1] + q.ibias;
        derive = false;
    }
    Plan pl;
    int e = make_plan<K, Idx>(device, derive, wl, wh, pl);
    if (e) return e;
    void *ws = q.ws;
    if (ws == nullptr) {
        e = cached_workspace(device, pl.L.total, &ws);
        if (e) return e;
    } else if (q.ws_bytes < pl.L.total) {
        return KMC_ERR_WORKSPACE;
    }
    char *base = static_cast<char *>(ws);
    Params p;
    p.data = q.data;
    p.indices = q.indices;
    p.ibias = q.ibias;
    p.n = q.n;
    p.sum = q.sum;
    p.ld = q.ld;
    p.invalid = q.invalid;
    p.wl = wl;
    p.wh = wh;
    p.rl = rl;
    p.rh = rh;
    p.derive = derive ? 1 : 0;
    p.G = pl.G;
    p.slot_rec = reinterpret_cast<int64_t *>(base + pl.L.slot_rec);
    p.spill_cnt = Cfg<K>::P16 ? reinterpret_cast<uint32_t *>(base + pl.L.spill_cnt) : nullptr;
    p.slab = reinterpret_cast<uint32_t *>(base + pl.L.slab);
    p.spill = Cfg<K>::P16 ? reinterpret_cast<Spill *>(base + pl.L.spill) : nullptr;
    p.spill_cap = pl.spill_cap;
    p.status = q.status;
    if (!p.status) {
        uint32_t *sh = nullptr;
        e = status_flag(device, &sh, &p.status);
        if (e) return e;
    }

    constexpr int NB = 1 << (2 * K);
    if (t_trace_before) {
        he = hipEventRecord(t_trace_before, st);
        if (he != hipSuccess) return (int)he;
    }
    hipLaunchKernelGGL((count_dense_kernel<K, Cfg<K>::R, Cfg<K>::HM, Idx, Cfg<K>::BLOCK>), dim3(pl.G),
                       dim3(Cfg<K>::BLOCK), 0, st, p);
    he = hipGetLastError();
    if (he != hipSuccess) return (int)he;
    if (t_trace_after) {
        he = hipEventRecord(t_trace_after, st);
        if (he != hipSuccess) return (int)he;
    }
    // (HM 3: pieces whose 16-bit counters wrapped are recounted by the count kernel
    // itself, right after their flush)
    constexpr int NWR = Cfg<K>::P16 ? NB / 2 : NB;  // slab words per slot
    constexpr int RW = NWR / 4 < 16 ? NWR : 64;      // words per reduce block (its RW)
    const unsigned cb = (unsigned)(NWR / RW);
    hipLaunchKernelGGL((reduce_dense_kernel<K, Idx, Cfg<K>::P16>), dim3(cb, (unsigned)std::min<int64_t>(q.n, kMaxGridY)),
                       dim3(256), 0, st, p);
    he = hipGetLastError();
    if (he != hipSuccess) return (int)he;
    // (k = 8: the spill entries are added by the reduce, which reads the lists of
    // the workgroups that hold each record's pieces.  spill_cap_for bounds the
    // entries a workgroup can emit -- scan entries stand for >= 32 768 windows, wrap
    // entries for 65 536, at most 3 per wrap -- and p16_spill keeps counting past
    // the cap, so an overflow raises the kmc_dense_status flag instead of passing
    // silently.)
    if (q.invalid) {
        hipLaunchKernelGGL((invalid_kernel<K, Idx>), dim3((unsigned)std::min<int64_t>(q.n, kMaxGridX)), dim3(256), 0,
                           st, p);
        he = hipGetLastError();
        if (he != hipSuccess) return (int)he;
    }
    return 0;
}

template <class Idx>
int dispatch(int k, const Request &q, hipStream_t st) {
    switch (k) {
        case 1: return run_dense<1, Idx>(q, st);
        case 2: return run_dense<2, Idx>(q, st);
        case 3: return run_dense<3, Idx>(q, st);
        case 4: return run_dense<4, Idx>(q, st);
        case 5: return run_dense<5, Idx>(q, st);
        case 6: return run_dense<6, Idx>(q, st);
        case 7: return run_dense<7, Idx>(q, st);
        case 8: return run_dense<8, Idx>(q, st);
        default: return KMC_ERR_UNSUPPORTED_K;
    }
}

template <class Idx>
size_t workspace_for(int k, int device, bool derive, int64_t wl, int64_t wh) {
    Plan pl;
    int e = 0;
    switch (k) {
        case 1: e = make_plan<1, Idx>(device, derive, wl, wh, pl); break;
        case 2: e = make_plan<2, Idx>(device, derive, wl, wh, pl); break;
        case 3: e = make_plan<3, Idx>(device, derive, wl, wh, pl); break;
        case 4: e = make_plan<4, Idx>(device, derive, wl, wh, pl); break;
        case 5: e = make_plan<5, Idx>(device, derive, wl, wh, pl); break;
        case 6: e = make_plan<6, Idx>(device, derive, wl, wh, pl); break;
        case 7: e = make_plan<7, Idx>(device, derive, wl, wh, pl); break;
        case 8: e = make_plan<8, Idx>(device, derive, wl, wh, pl); break;
        default: return 0;
    }
    return e ? 0 : pl.L.total;
}

}  // namespace
}  // namespace kmc

using namespace kmc;

extern "C" int kmc_set_reserved_cus(int n) {
    if (n < 0 || n > 64) return KMC_ERR_INVALID_ARG;
    t_reserved_cus = n;
    return KMC_OK;
}

extern "C" int kmc_dense_status(int device) { return take_status(device); }

#ifdef KMC_DIAG_HOOKS
// Test hook (diagnostic library only, not in kmc.h): the k = 8 spill list
// capacity per workgroup, lowered so that an overflow raises the status flag.
extern "C" KMC_DIAG_API int kmc_diag_dense_spill_cap(unsigned cap) {
    g_diag_spill_cap.store(cap);
    return KMC_OK;
}
#endif

extern "C" int kmc_trace_set_events(hipEvent_t before, hipEvent_t after) {
    t_trace_before = before;
    t_trace_after = after;
    return KMC_OK;
}

extern "C" int sumKmereCoincidencesGlobalMemory_hip(char *data, int *indices, unsigned num_seqs, int *sum,
                                                    hipStream_t stream) {
    if (num_seqs == 0) return KMC_OK;
    if (!data || !indices || !sum) return KMC_ERR_INVALID_ARG;
    // kernels.h:113 takes any char *: a pointer inside a buffer (data + off) is
    // rounded down to 16 bytes and the offsets biased by the difference (the
    // aligned block holding data[0] lies in data's own page)
    const uintptr_t mis = reinterpret_cast<uintptr_t>(data) & 15u;
    Request q{};
    q.data = data - mis;
    q.ibias = (int64_t)mis;
    q.indices = indices;
    q.n = num_seqs;
    q.sum = sum;
    q.ld = num_seqs;
    q.derive = true;
    return dispatch<int>(KMC_DROPIN_K, q, stream);
}

// An unaligned data pointer (kernels.h:113 takes any char *): data rounded down to
// 16 bytes, every range and record offset moved up by the difference.
static kmc_dense_args aligned_args(const kmc_dense_args *a, int64_t &bias) {
    kmc_dense_args b = *a;
    const uintptr_t mis = reinterpret_cast<uintptr_t>(a->data) & 15u;
    b.data = a->data - mis;
    b.read_lo += mis;
    b.read_hi += mis;
    b.win_lo += mis;
    b.win_hi += mis;
    bias = (int64_t)mis;
    return b;
}

extern "C" size_t kmc_count_dense_ex_workspace_size(const kmc_dense_args *a0, int device) {
    if (!a0 || a0->k < 1 || a0->k > KMC_DENSE_MAX_K) return 0;
    int64_t bias = 0;
    const kmc_dense_args al = aligned_args(a0, bias);
    const kmc_dense_args *a = &al;
    if (a->k > 8) {
        size_t sz = 0;
        return radix_dense(a, bias, nullptr, true, &sz) == 0 ? sz : 0;
    }
    const int64_t wl = (int64_t)a->win_lo, wh = (int64_t)a->win_hi;
    return workspace_for<int64_t>(a->k, device, false, wl, wh);
}

extern "C" int kmc_count_dense_ex(const kmc_dense_args *a0, hipStream_t stream) {
    if (!a0) return KMC_ERR_INVALID_ARG;
    if (a0->k < 1 || a0->k > KMC_DENSE_MAX_K) return KMC_ERR_UNSUPPORTED_K;
    if (a0->num_seqs == 0) return KMC_OK;
    if (!a0->data || !a0->indices || !a0->sum) return KMC_ERR_INVALID_ARG;
    if (a0->read_hi < a0->read_lo || a0->win_hi < a0->win_lo) return KMC_ERR_INVALID_ARG;
    if (a0->sum_ld != 0 && a0->sum_ld < a0->num_seqs) return KMC_ERR_INVALID_ARG;
    int64_t bias = 0;
    kmc_dense_args al = aligned_args(a0, bias);
    const kmc_dense_args *a = &al;
    if (!al.status) {  // the device's flag (kmc_dense_status)
        int device = 0;
        hipError_t he = hipGetDevice(&device);
        if (he != hipSuccess) return (int)he;
        uint32_t *sh = nullptr, *sd = nullptr;
        const int e = status_flag(device, &sh, &sd);
        if (e) return e;
        al.status = reinterpret_cast<int32_t *>(sd);
    }
    if (a->k > 8) return radix_dense(a, bias, stream, false, nullptr);
    Request q{};
    q.data = a->data;
    q.ibias = bias;
    q.indices = a->indices;
    q.n = (int64_t)a->num_seqs;
    q.sum = a->sum;
    q.ld = a->sum_ld ? (int64_t)a->sum_ld : (int64_t)a->num_seqs;
    q.invalid = a->invalid;
    q.derive = false;
    q.wl = (int64_t)a->win_lo;
    q.wh = (int64_t)a->win_hi;
    q.rl = (int64_t)a->read_lo;
    q.rh = (int64_t)a->read_hi;
    q.ws = a->workspace;
    q.ws_bytes = a->workspace_bytes;
    q.status = reinterpret_cast<uint32_t *>(a->status);
    return dispatch<int64_t>(a->k, q, stream);
}

extern "C" size_t kmc_count_dense_workspace_size(int k, uint64_t num_seqs, uint64_t data_bytes, int device) {
    if (k < 1 || k > KMC_DENSE_MAX_K) return 0;
    // the size for the most demanding alignment (a misaligned pointer moves the
    // ranges up to 15 bytes, which can add a tile)
    if (k > 8) {
        kmc_dense_args a{};
        a.k = k;
        a.num_seqs = num_seqs;
        a.read_lo = a.win_lo = 15;
        a.read_hi = a.win_hi = data_bytes + 15;
        size_t sz = 0;
        return radix_dense(&a, 15, nullptr, true, &sz) == 0 ? sz : 0;
    }
    return workspace_for<int64_t>(k, device, false, 15, (int64_t)data_bytes + 15);
}

extern "C" int kmc_count_dense(const char *data, const int64_t *indices, uint64_t num_seqs, uint64_t data_bytes,
                               int k, int32_t *sum, int32_t *invalid, void *workspace, size_t workspace_bytes,
                               hipStream_t stream) {
    kmc_dense_args a{};
    a.data = data;
    a.indices = indices;
    a.num_seqs = num_seqs;
    a.k = k;
    a.sum = sum;
    a.sum_ld = num_seqs;
    a.invalid = invalid;
    a.read_lo = 0;
    a.read_hi = data_bytes;
    a.win_lo = 0;
    a.win_hi = data_bytes;
    a.workspace = workspace;
    a.workspace_bytes = workspace_bytes;
    return kmc_count_dense_ex(&a, stream);
}
