// kmc_dense.hip — dense k-mer histogram kernels for gfx950 (MI355X, CDNA4).
//
// Replaces sumKmereCoincidencesGlobalMemory (reference kernels.h:113-144), which
// gives one block per record and one thread per pattern, every thread rescanning
// its record with 3-byte compares.  Here one pass reads every byte once:
//
//   HBM --dwordx4--> lane registers: 16 ASCII bases per lane per tile (1 KiB/wave)
//       --SWAR-----> 32-bit 2-bit-packed codes (first base in the low bits, i.e.
//                    the reference's little-endian bin order) + 16-bit invalid mask
//       --DPP------> the next lane's codes as the (k-1)-base halo
//       --bfe------> 16 window codes per lane, one LDS atomic each
//       --flush----> per-record histogram, written once (direct or via slab reduce)
//
// Layout of the work: the buffer is cut into 1 KiB tiles; workgroup w has a home
// range of tiles and walks the records intersecting it ("pieces"), its 16 waves
// splitting each piece into contiguous per-wave runs.  The first and the last
// piece of a home range (the ones that can be cut by its ends) are claimed by
// their waves in chunks of kChunk tiles, front to back, through one 64-bit claim
// word per wave (front | back << 32); a workgroup done with its own range becomes
// a thief and claims chunks from the back of the pieces with the most work left,
// so a workgroup that starts late (its CU held by another kernel, e.g. the RCCL
// all-reduce that bench.py overlaps with the next step) or runs slow is helped
// instead of setting the kernel's end.  A piece covering a whole record is written
// straight to sum[]; the other pieces go to slab slots (two per home range, one per
// thief round), summed per record by reduce_dense_kernel.  No global atomics on the
// hot path.
//
// Histogram storage per workgroup (LDS):
//   k <= 7 : 32-bit counters, R replicas interleaved (bin*R + lane%R) so lanes of a
//            32-lane LDS group never collide on small alphabets (k <= 4: R = 32).
//   k == 8 : 65 536 bins do not fit as 32-bit (256 KB > 160 KB LDS): two 16-bit
//            counters per word (bin c in the low half, c|0x8000 in the high half),
//            plain adds.  Every KMC_HM3_SCAN tiles a wave moves the halves >= 32 768
//            of its 1/16 of the words to spill entries (atomic subtract, no
//            barrier); a 16-bit wrap can only lose counts, so a piece whose decoded
//            total plus spills differs from its windows wrapped, and its record is
//            recounted exactly by recount_dense_kernel (returning adds).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "kmc.h"
#include "kmc_internal.h"
#include "kmc_stream.h"

// k == 8: tiles per wave between two scans of its words (hot 16-bit halves to spill
// entries; 0: no scans)
#ifndef KMC_HM3_SCAN
#define KMC_HM3_SCAN 256
#endif

namespace kmc {
thread_local hipEvent_t t_trace_before = nullptr;
thread_local hipEvent_t t_trace_after = nullptr;
namespace {

constexpr int kChunk = 32;                  // tiles per claim of a stealable piece
constexpr int kClaimWaves = 16;             // claim words per piece (>= waves of any block size)
constexpr uint64_t kInitBit = 1ull << 63;   // epoch word being initialised
constexpr uint64_t kBackOne = 0xFFFFFFFF00000000ull;  // + this = back - 1

struct Spill {
    int64_t rec;
    int32_t code;
    int32_t amount;
};

// Slab slots: [0, 2G) the first / last piece of each home range, [2G, 2G + pool_cap)
// thief rounds, then (k = 8) [.., + 2G) the recount's first / last pieces.
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
    int G;                   // workgroups of the count kernel (home ranges)
    uint32_t *slab;          // [slots][words] (k = 8: 4^k / 2 words of packed 16-bit halves)
    int64_t *slot_rec;       // [slots] record held by each slab slot, -1 = none
    uint32_t pool_cap;       // thief slots
    Spill *spill;            // [G][spill_cap] first pass (k = 8)
    uint32_t *spill_cnt;     // [G]
    uint32_t spill_cap;
    Spill *fb_spill;         // [G][fb_spill_cap] recount pass
    uint32_t *fb_spill_cnt;  // [G]
    uint32_t fb_spill_cap;
    uint64_t *claims;        // [G][2][kClaimWaves] chunk claims of the first / last piece
    uint64_t *wg_ep;         // [G] epoch of a home range's claim words
    uint64_t *pool;          // [2] epoch, thief slots taken
    uint64_t *flags;         // [4] epoch words: any record failed, any spill, any recount spill
    uint64_t *rec_direct;    // [n] epoch: record written straight to sum
    uint64_t *rec_fail;      // [n] epoch: record's 16-bit counters wrapped (recounted)
    uint64_t epoch;          // this call's (non-zero, < 2^63)
    int steal;               // thieves enabled
    uint32_t owner_delay;    // test hook: owners of every third range wait this many 100 MHz ticks
};

enum { kFlagFail = 0, kFlagSpill = 1, kFlagFbSpill = 2 };

__device__ __forceinline__ uint64_t ld_acq(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rel(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t readfirstlane64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
    return (uint64_t)lo | ((uint64_t)hi << 32);
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

// k == 8, packed 16-bit halves with returning adds (HM == 1).  The 16 adds of a
// tile are issued, and their returned values are checked one tile later
// (p16_check), so the LDS return latency hides behind the next tile's decode.
struct P16Pending {
    uint32_t old[16];
    uint32_t lo, hi, W;
};

template <bool MASKED>
__device__ __forceinline__ void count_tile_p16(uint32_t lo, uint32_t hi, uint32_t W, const P16Ctx &pc,
                                               P16Pending &pd) {
    const uint32_t mid = __builtin_amdgcn_alignbit(hi, lo, 16);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t src = (j <= 8) ? lo : mid;
        const int off = (j <= 8) ? 2 * j : 2 * (j - 8);
        const uint32_t word = (src >> off) & 0x7FFFu;
        const uint32_t hb = (src >> (off + 15)) & 1u;
        pd.old[j] = 0u;
        if (!MASKED || ((W >> j) & 1u))
            pd.old[j] = __hip_atomic_fetch_add(&pc.h[word], half_inc(hb), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    pd.lo = lo;
    pd.hi = hi;
    pd.W = MASKED ? W : 0xFFFFu;
}

// Conservative precheck: a half can only have wrapped if some returned value had
// a half >= 0x8000; random input never gets there, skewed input takes the exact
// per-window path.
__device__ __forceinline__ void p16_check(const P16Ctx &pc, const P16Pending &pd) {
    uint32_t any = 0u;
#pragma unroll
    for (int j = 0; j < 16; ++j) any |= pd.old[j];
    if (__any((any & 0x80008000u) != 0u)) {
        const uint32_t mid = __builtin_amdgcn_alignbit(pd.hi, pd.lo, 16);
        uint32_t ovf = 0u, hw = 0u;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t src = (j <= 8) ? pd.lo : mid;
            const int off = (j <= 8) ? 2 * j : 2 * (j - 8);
            const uint32_t m = ((src >> (off + 15)) & 1u) ? 0xFFFF0000u : 0x0000FFFFu;
            ovf |= (uint32_t)((pd.old[j] & m) == m) << j;
            hw |= (uint32_t)(pd.old[j] >= 0xFFFF0000u) << j;
        }
        ovf &= pd.W;
        if (ovf != 0u) {
            const uint64_t both = (uint64_t)pd.lo | ((uint64_t)pd.hi << 32);
            for (int j = 0; j < 16; ++j) {
                if ((ovf >> j) & 1u) {
                    const uint32_t code = (uint32_t)(both >> (2 * j)) & 0xFFFFu;
                    p16_fix(pc, code & 0x7FFFu, code >> 15, (hw >> j) & 1u);
                }
            }
        }
    }
}

// k == 8, packed 16-bit halves, plain adds (HM == 2): overflow is excluded by the
// between-barrier scans of count_wave_range (p16_scan).
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
__device__ __forceinline__ void count_tile(uint32_t lo, uint32_t hi, uint32_t W, uint32_t *h, int lane,
                                           const P16Ctx &pc, P16Pending &pd) {
    if constexpr (HM == 1)
        count_tile_p16<MASKED>(lo, hi, W, pc, pd);
    else if constexpr (HM == 2 || HM == 3)
        count_tile_p16_plain<MASKED>(lo, hi, W, h);
    else
        count_tile32<K, R, MASKED>(lo, hi, W, h, lane);
}

// k == 8, HM 3, no barrier: wave `wave` of NWAVES scans its 1/NWAVES of the packed
// words and moves every half >= T to a spill entry, by an atomic subtract of the
// multiple of T it read (the other waves keep adding meanwhile; halves only grow,
// so the subtract never borrows unless the half wrapped in between, which the
// piece's total check catches).
template <uint32_t T>
__device__ __noinline__ void p16_scan_fix(const P16Ctx &pc, int i4) {
    for (int q = 0; q < 4; ++q) {
        const uint32_t word = (uint32_t)(4 * i4 + q);
        const uint32_t x = __hip_atomic_load(&pc.h[word], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t la = (x & 0xFFFFu) & ~(T - 1u), ha = (x >> 16) & ~(T - 1u);
        if (la | ha) {
            __hip_atomic_fetch_sub(&pc.h[word], la | (ha << 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (la) {
                p16_spill(pc, (int32_t)word, (int32_t)la);
                atomicAdd(pc.spilled, la);
            }
            if (ha) {
                p16_spill(pc, (int32_t)(word | 0x8000u), (int32_t)ha);
                atomicAdd(pc.spilled, ha);
            }
        }
    }
}

template <int NWAVES, uint32_t T>
__device__ __forceinline__ void p16_scan_wave(const P16Ctx &pc, int wave, int lane) {
    constexpr uint32_t HOT = (0xFFFFu & ~(T - 1)) * 0x00010001u;  // bits >= T in both halves
    constexpr int PER_WAVE = (1 << 15) / 4 / NWAVES;             // uint4 of this wave's words
    static_assert(PER_WAVE % 64 == 0, "scan slice");
    const uint4 *h4 = reinterpret_cast<const uint4 *>(pc.h) + wave * PER_WAVE;
    uint32_t hot = 0u;
#pragma unroll
    for (int i = 0; i < PER_WAVE / 64; ++i) {
        const uint4 v = h4[lane + 64 * i];
        hot |= (uint32_t)(((v.x | v.y | v.z | v.w) & HOT) != 0u) << i;
    }
    if (hot) {
        for (int i = 0; i < PER_WAVE / 64; ++i)
            if ((hot >> i) & 1u) p16_scan_fix<T>(pc, wave * PER_WAVE + lane + 64 * i);
    }
}

// The dense histogram as a stream_tiles operation.  HM 0: 32-bit bins; HM 3: packed
// 16-bit halves, plain adds, a per-wave scan every KMC_HM3_SCAN tiles; HM 1 (the
// recount): returning adds, every wrap fixed up exactly.
template <int K, int R, int HM, int BLOCK>
struct DenseOp {
    uint32_t *h;
    int lane, wave;
    const P16Ctx &pc;
    P16Pending pd;
    bool pending = false;
    uint32_t nwin = 0u;   // HM 3: windows this lane added
    uint32_t tiles = 0u;  // HM 3: tiles since this wave's last scan

    __device__ DenseOp(uint32_t *h_, int lane_, int wave_, const P16Ctx &pc_) : h(h_), lane(lane_), wave(wave_), pc(pc_) {}

    __device__ __forceinline__ void before_tile() {
        if constexpr (HM == 1) {
            if (pending) p16_check(pc, pd);
        }
    }
    template <bool MASKED>
    __device__ __forceinline__ void tile(uint32_t lo, uint32_t hi, uint32_t W) {
        count_tile<K, R, HM, MASKED>(lo, hi, W, h, lane, pc, pd);
        if constexpr (HM == 1) pending = true;
        if constexpr (HM == 3) nwin += MASKED ? (uint32_t)__builtin_popcount(W) : 16u;
    }
    __device__ __forceinline__ void after_iter(int64_t i, int64_t per, bool) {
        if constexpr (HM == 1) {
            if (pending && i + 1 == per) {
                p16_check(pc, pd);
                pending = false;
            }
        }
        if constexpr (HM == 3 && KMC_HM3_SCAN > 0) {
            // hot halves (>= 32768) go to spill entries every KMC_HM3_SCAN tiles of
            // this wave, so a half wraps only if one k-mer takes >= 32768 of the
            // windows added between two scans of its word (long low-complexity
            // runs); wraps stay detected by the piece total
            if (++tiles == (uint32_t)KMC_HM3_SCAN) {
                tiles = 0u;
                p16_scan_wave<BLOCK / 64, 32768u>(pc, wave, lane);
            }
        }
    }
};

// ---------------------------------------------------------------------------
// work distribution
// ---------------------------------------------------------------------------
// One-shot initialisation of an object shared by workgroups, tagged by this
// call's epoch: the first thread to move the epoch word from a stale value to
// epoch | kInitBit runs init() and publishes epoch; the others wait for it.  Stale
// values (an earlier call, never-written memory) are not this call's epoch.
template <class F>
__device__ __forceinline__ void ensure_epoch(uint64_t *ep, uint64_t epoch, F &&init) {
    for (;;) {
        uint64_t e = ld_acq(ep);
        if (e == epoch) return;
        if (e == (epoch | kInitBit)) {
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        if (__hip_atomic_compare_exchange_strong(ep, &e, epoch | kInitBit, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
            init();
            st_rel(ep, epoch);
            return;
        }
    }
}

struct Range {
    int64_t R0, R1;  // window positions of a home range (R0 >= R1: empty)
};

__device__ __forceinline__ Range home_range(const Geom &g, int64_t w) {
    const int64_t tb = g.T0 + w * g.tpw;
    const int64_t te = (tb + g.tpw) < g.T1 ? (tb + g.tpw) : g.T1;
    Range r;
    r.R0 = (tb << kTileShift) > g.wl ? (tb << kTileShift) : g.wl;
    r.R1 = (te << kTileShift) < g.wh ? (te << kTileShift) : g.wh;
    if (tb >= te) r.R1 = r.R0;
    return r;
}

struct Piece {
    int64_t s;       // record (-1: none)
    int64_t ca, ce;  // the record's windows in the counted range
    int64_t ps, pe;  // ... inside the home range
};

template <int K, class Idx, class P>
__device__ __forceinline__ bool piece_at(const P &p, const Geom &g, int64_t s, const Range &r, Piece &pc) {
    pc.s = s;
    record_windows<K, Idx>(p, g, s, pc.ca, pc.ce);
    pc.ps = pc.ca > r.R0 ? pc.ca : r.R0;
    pc.pe = pc.ce < r.R1 ? pc.ce : r.R1;
    return pc.ps < pc.pe;
}

// The first (which 0) or last (which 1) non-empty piece of home range w, the two
// that claims make stealable; s = -1 when there is none (which 1: also when the
// range has a single piece).  Pieces between them are whole records, counted by
// the owner alone and written straight to sum.
template <int K, class Idx>
__device__ __forceinline__ Piece stealable_piece(const Params &p, const Geom &g, int64_t w, int which) {
    Piece pc;
    pc.s = -1;
    const Range r = home_range(g, w);
    if (r.R0 >= r.R1) return pc;
    int64_t s = first_record_at<Idx>(p, r.R0);
    bool found = false;
#pragma unroll 1
    for (; s < p.n && rec_off<Idx>(p, s) < r.R1; ++s)
        if (piece_at<K, Idx>(p, g, s, r, pc)) {
            found = true;
            break;
        }
    if (!found) {
        pc.s = -1;
        return pc;
    }
    if (which == 0) return pc;
    const int64_t s0 = s;
#pragma unroll 1
    for (int64_t t = first_record_at<Idx>(p, r.R1 - 1); t > s0; --t)
        if (piece_at<K, Idx>(p, g, t, r, pc)) return pc;
    pc.s = -1;
    return pc;
}

// The contiguous tile run of wave v of a piece (as the static split: per = tiles/waves)
__device__ __forceinline__ void wave_run(const Piece &pc, int nwaves, int v, int64_t &a0, int64_t &a1) {
    const int64_t tp0 = pc.ps >> kTileShift, tp1 = ((pc.pe - 1) >> kTileShift) + 1;
    const int64_t per = (tp1 - tp0 + nwaves - 1) / nwaves;
    a0 = tp0 + (int64_t)v * per;
    a1 = (a0 + per) < tp1 ? (a0 + per) : tp1;
    if (a1 < a0) a1 = a0;
}
__device__ __forceinline__ int64_t chunks_of(int64_t a0, int64_t a1) { return (a1 - a0 + kChunk - 1) / kChunk; }

// window positions of piece pc inside tiles [t0, t1)
__device__ __forceinline__ int64_t covered(const Piece &pc, int64_t t0, int64_t t1) {
    const int64_t lo = (t0 << kTileShift) > pc.ps ? (t0 << kTileShift) : pc.ps;
    const int64_t hi = (t1 << kTileShift) < pc.pe ? (t1 << kTileShift) : pc.pe;
    return hi > lo ? hi - lo : 0;
}

__device__ __forceinline__ uint64_t *claim_word(const Params &p, int64_t w, int which, int v) {
    return p.claims + (w * 2 + which) * kClaimWaves + v;
}

// home range w's claim words: (front 0, back = chunks of the wave's run), once per call
template <int K, class Idx, int NWAVES>
__device__ __forceinline__ void ensure_claims(const Params &p, const Geom &g, int64_t w) {
    ensure_epoch(p.wg_ep + w, p.epoch, [&] {
#pragma unroll 1
        for (int which = 0; which < 2; ++which) {
            const Piece pc = stealable_piece<K, Idx>(p, g, w, which);
#pragma unroll 1
            for (int v = 0; v < kClaimWaves; ++v) {
                int64_t nch = 0;
                if (pc.s >= 0 && v < NWAVES) {
                    int64_t a0, a1;
                    wave_run(pc, NWAVES, v, a0, a1);
                    nch = chunks_of(a0, a1);
                }
                __hip_atomic_store(claim_word(p, w, which, v), (uint64_t)nch << 32, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    });
}

__device__ __forceinline__ bool claim_ok(uint64_t x) { return (int32_t)(uint32_t)x < (int32_t)(x >> 32); }

// Thief: the last unclaimed chunk of a wave's run (wave-uniform), -1 when none is left.
__device__ __forceinline__ int64_t claim_back(uint64_t *st, int lane) {
    int64_t ch = -1;
    if (lane == 0) {
        const uint64_t cur = __hip_atomic_load(st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (claim_ok(cur)) {
            const uint64_t old = __hip_atomic_fetch_add(st, kBackOne, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (claim_ok(old)) ch = (int64_t)(int32_t)(old >> 32) - 1;
        }
    }
    return (int64_t)readfirstlane64((uint64_t)ch);
}

// Chunks of a victim's piece nobody has claimed yet (all of them when the victim
// has not started and no thief initialised its words).
template <int K, class Idx, int NWAVES>
__device__ __forceinline__ int64_t unclaimed(const Params &p, const Geom &g, int64_t v, int which) {
    if (ld_acq(p.wg_ep + v) == p.epoch) {
        int64_t r = 0;
#pragma unroll 1
        for (int j = 0; j < NWAVES; ++j) {
            const uint64_t x = __hip_atomic_load(claim_word(p, v, which, j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int32_t f = (int32_t)(uint32_t)x, b = (int32_t)(x >> 32);
            r += b > f ? b - f : 0;
        }
        return r;
    }
    const Piece pc = stealable_piece<K, Idx>(p, g, v, which);
    if (pc.s < 0) return 0;
    int64_t r = 0;
#pragma unroll 1
    for (int j = 0; j < NWAVES; ++j) {
        int64_t a0, a1;
        wave_run(pc, NWAVES, j, a0, a1);
        r += chunks_of(a0, a1);
    }
    return r;
}

// A thief slab slot of this call, ~0u when the pool is used up.
__device__ __forceinline__ uint32_t pool_take(const Params &p) {
    ensure_epoch(p.pool, p.epoch,
                 [&] { __hip_atomic_store(p.pool + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); });
    const uint64_t i = __hip_atomic_fetch_add(p.pool + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return i < p.pool_cap ? (uint32_t)i : ~0u;
}

__device__ __forceinline__ uint32_t pool_used(const Params &p) {
    if (ld_acq(p.pool) != p.epoch) return 0u;
    const uint64_t n = __hip_atomic_load(p.pool + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return n < p.pool_cap ? (uint32_t)n : p.pool_cap;
}

// Owner: wave run [a0, a1) of a stealable piece, claimed front to back kChunk tiles at
// a time.  The claim of the next chunk is issued when a chunk starts and read when
// it ends, and the tile stream (prefetch ring included) runs on across chunks: the
// owner's chunks are contiguous, thieves take them from the back.  Returns the
// window positions covered.  (One flat loop: the same logic as a loop over chunks
// around a loop over tiles was miscompiled by this ROCm 7.2 hipcc: the tiles after
// the first chunk were counted from stale registers, scripts/diag_dense.py.)
template <int K, class Op>
__device__ __forceinline__ int64_t stream_owner(const char *__restrict__ data, const Piece &pp, int64_t a0, int64_t a1,
                                                int64_t rl, int64_t rh, int lane, Op &op, uint64_t *st) {
    using TS = TileStream<K>;
    static_assert(kChunk % TS::NS == 0, "chunks hold whole ring rounds");
    const int64_t nt = a1 - a0;
    if (nt <= 0) return 0;
    uint64_t c = 0;
    if (lane == 0) c = __hip_atomic_fetch_add(st, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!claim_ok(readfirstlane64(c))) return 0;  // the whole run was stolen
    TS ts;
    ts.start(data, a0, pp.ps, pp.pe, rl, rh, lane);
    int64_t lim = nt < kChunk ? nt : kChunk;
    uint64_t nx = 0;
    if (lane == 0 && lim < nt) nx = __hip_atomic_fetch_add(st, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int64_t i = 0; i < lim; i += TS::NS) {
        ts.template steps<0>(i, lim, lim, op);
        if (i + TS::NS >= lim && lim < nt) {  // a chunk done: the next one, if still ours
            if (claim_ok(readfirstlane64(nx))) {
                lim = (lim + kChunk) < nt ? (lim + kChunk) : nt;
                if (lane == 0 && lim < nt)
                    nx = __hip_atomic_fetch_add(st, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    return covered(pp, a0, a0 + lim);
}

// LDS words after the histogram: [0] spill entries of this workgroup's list,
// [1] windows added, [2] decoded total, [3] spilled, [4] spill entries before the
// piece, [5] thief slot, [6] verdict, [8..9] window positions (u64), [10..11]
// first record (u64), [12..13] first-piece record, [14..15] last-piece record,
// [16..17] victim pick (u64)
constexpr int kMisc = 32;

// End of a piece (the whole workgroup): its histogram goes to sum (the piece holds
// every window of the record) or to slab slot `slot`; k = 8 checks the piece for
// 16-bit wraps (then the record is flagged for the recount) and applies the spill
// entries of a direct write.  Returns 0 = slot used, 1 = written to sum, 2 = wrapped.
template <int K, int R, int HM, int BLOCK>
__device__ __forceinline__ uint32_t finish_piece(const Params &p, uint32_t *h, uint32_t *misc, const P16Ctx &pc, const Piece &pp,
                                 int64_t slot, uint32_t nwin, int64_t pos) {
    constexpr bool P16 = HM != 0;
    constexpr int NB = 1 << (2 * K);
    constexpr int NW = P16 ? NB / 2 : NB * R;
    const int tid = threadIdx.x, lane = tid & 63;
    unsigned long long *m64 = reinterpret_cast<unsigned long long *>(misc);
    if constexpr (HM == 3) {
        const uint32_t ws = wave_sum(nwin);
        if (lane == 0) atomicAdd(&misc[1], ws);
    }
    if (lane == 0) atomicAdd(&m64[4], (unsigned long long)pos);
    __syncthreads();
    const bool entire = m64[4] == (unsigned long long)(pp.ce - pp.ca);
    const int64_t s = pp.s;
    if constexpr (P16) {
        uint32_t *dst = p.slab + slot * (int64_t)(NB / 2);
        uint32_t dsum = 0u;
        for (int i = tid; i < NW; i += BLOCK) {
            const uint32_t v = h[i];
            h[i] = 0u;
            dsum += (v & 0xFFFFu) + (v >> 16);
            if (entire) {
                p.sum[s + p.ld * (int64_t)i] = (int32_t)(v & 0xFFFFu);
                p.sum[s + p.ld * (int64_t)(i + NW)] = (int32_t)(v >> 16);
            } else {
                dst[i] = v;  // packed as in LDS: the halves are exact (wraps live in spills)
            }
        }
        const uint32_t ws = wave_sum(dsum);
        if (lane == 0) atomicAdd(&misc[2], ws);
    } else {
        uint32_t *dst = p.slab + slot * (int64_t)NB;
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
    __syncthreads();
    if (tid == 0) {
        // every 16-bit wrap only loses counts (low half: -65535 net, high half:
        // -65536), so the decoded total plus the scans' spills equals the windows
        // added iff none wrapped; spill entries past the list's capacity were lost
        bool failed = false;
        if constexpr (HM == 3) failed = misc[1] != misc[2] + misc[3] || misc[0] > pc.cap;
        if (failed) {
            __hip_atomic_store(p.rec_fail + s, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(p.flags + kFlagFail, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (entire) {
            __hip_atomic_store(p.rec_direct + s, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        misc[6] = failed ? 2u : (entire ? 1u : 0u);
        misc[1] = 0u;
        misc[2] = 0u;
        misc[3] = 0u;
        m64[4] = 0ull;
    }
    __syncthreads();
    const uint32_t verdict = misc[6];
    if constexpr (HM == 3) {
        const uint32_t n0 = misc[4], n1 = misc[0] < pc.cap ? misc[0] : pc.cap;
        __syncthreads();  // every thread has read misc[4]
        if (tid == 0) misc[4] = misc[0];
        if (verdict == 1u) {
            // a direct write takes its spills now; a slab piece's are the reduce's
            for (uint32_t i = n0 + tid; i < n1; i += BLOCK) {
                const Spill e = pc.spill[i];
                atomicAdd(&p.sum[e.rec + p.ld * (int64_t)e.code], e.amount);
            }
        } else if (verdict == 0u && tid == 0 && n1 > n0) {
            __hip_atomic_store(p.flags + kFlagSpill, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    return verdict;
}

template <int K, int R, int HM, class Idx, int BLOCK>
__global__ __launch_bounds__(BLOCK) void count_dense_kernel(Params p) {
    static_assert(HM == 0 || HM == 3, "first pass: 32-bit bins or packed halves with scans");
    constexpr bool P16 = HM != 0;
    constexpr int NB = 1 << (2 * K);
    constexpr int NW = P16 ? NB / 2 : NB * R;
    constexpr int NWAVES = BLOCK / 64;
    static_assert(NWAVES <= kClaimWaves, "claim words per piece");
    // static LDS: the histogram's address is a link-time constant, folded into the
    // ds_add offset (dynamic LDS costs one v_add per window)
    __shared__ __attribute__((aligned(16))) uint32_t smem[NW + kMisc];
    uint32_t *h = smem;
    uint32_t *misc = smem + NW;
    unsigned long long *m64 = reinterpret_cast<unsigned long long *>(misc);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar tile bookkeeping
    const int64_t w = blockIdx.x;
    const Geom g = make_geom<Idx>(p);
    const Range r = home_range(g, w);
    if (p.owner_delay && (w % 3) == 0) {  // test hook: a late owner, its pieces stolen
        const uint64_t t0 = wall_clock64();
        while (wall_clock64() - t0 < p.owner_delay) __builtin_amdgcn_s_sleep(8);
    }
    for (int i = tid; i < NW; i += BLOCK) h[i] = 0u;
    if (tid < kMisc) misc[tid] = 0u;
    P16Ctx pc;
    pc.h = h;
    pc.spilled = misc + 3;
    pc.spill_n = misc;
    pc.spill = P16 ? p.spill + w * (int64_t)p.spill_cap : nullptr;
    pc.cap = p.spill_cap;
    pc.rec = -1;
    __syncthreads();
    if (tid == 0 && r.R0 < r.R1) {
        ensure_claims<K, Idx, NWAVES>(p, g, w);
        m64[5] = (unsigned long long)first_record_at<Idx>(p, r.R0);
        m64[6] = (unsigned long long)stealable_piece<K, Idx>(p, g, w, 0).s;
        m64[7] = (unsigned long long)stealable_piece<K, Idx>(p, g, w, 1).s;
    }
    __syncthreads();
    int64_t own_first = -1, own_last = -1;  // records in the owner's two slab slots
    if (r.R0 < r.R1) {
        const int64_t s_first = (int64_t)m64[6], s_last = (int64_t)m64[7];
        for (int64_t s = (int64_t)m64[5]; s < p.n; ++s) {
            if (rec_off<Idx>(p, s) >= r.R1) break;
            Piece pp;
            if (!piece_at<K, Idx>(p, g, s, r, pp)) continue;
            const int which = s == s_first ? 0 : (s == s_last ? 1 : 2);
            pc.rec = s;
            DenseOp<K, R, HM, BLOCK> op(h, lane, wave, pc);
            int64_t a0, a1, pos;
            wave_run(pp, NWAVES, wave, a0, a1);
            if (which < 2) {
                pos = stream_owner<K>(p.data, pp, a0, a1, g.rl, g.rh, lane, op, claim_word(p, w, which, wave));
            } else {  // a whole record inside the range: not stealable
                stream_tiles<K>(p.data, a0, a1, a1 - a0, pp.ps, pp.pe, g.rl, g.rh, lane, op);
                pos = covered(pp, a0, a1);
            }
            const int64_t slot = 2 * w + (which == 0 ? 0 : 1);
            const uint32_t verdict = finish_piece<K, R, HM, BLOCK>(p, h, misc, pc, pp, slot, op.nwin, pos);
            if (verdict == 0u && which == 0) own_first = s;
            if (verdict == 0u && which == 1) own_last = s;
        }
    }
    if (tid == 0) {
        p.slot_rec[2 * w] = own_first;
        p.slot_rec[2 * w + 1] = own_last;
    }
    // thief: chunks from the back of the stealable pieces with the most work left
    while (p.steal) {
        __syncthreads();
        if (tid == 0) m64[8] = 0ull;
        __syncthreads();
        for (int c = tid; c < 2 * p.G; c += BLOCK) {
            const int64_t v = c >> 1;
            if (v == w) continue;
            const int64_t rem = unclaimed<K, Idx, NWAVES>(p, g, v, c & 1);
            if (rem >= NWAVES)  // at least a chunk per wave: a round pays for its slab flush
                __hip_atomic_fetch_max(&m64[8], ((unsigned long long)rem << 24) | (unsigned long long)c,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        const unsigned long long pick = m64[8];
        if (pick == 0ull) break;
        const int c = (int)(pick & 0xFFFFFFull);
        const int64_t v = c >> 1;
        const int which = c & 1;
        if (tid == 0) {
            ensure_claims<K, Idx, NWAVES>(p, g, v);
            misc[5] = pool_take(p);
        }
        __syncthreads();
        const uint32_t ps_ = misc[5];
        if (ps_ == ~0u) break;  // no slab slot left: the owners finish their pieces
        const Piece pp = stealable_piece<K, Idx>(p, g, v, which);
        const int64_t slot = 2 * (int64_t)p.G + ps_;
        if (pp.s < 0) {
            if (tid == 0) p.slot_rec[slot] = -1;
            continue;
        }
        pc.rec = pp.s;
        DenseOp<K, R, HM, BLOCK> op(h, lane, wave, pc);
        int64_t pos = 0;
#pragma unroll 1
        for (int jj = 0; jj < NWAVES; ++jj) {  // this wave's twin run first, then the others
            const int j = (wave + jj) % NWAVES;
            uint64_t *st = claim_word(p, v, which, j);
            int64_t a0, a1;
            wave_run(pp, NWAVES, j, a0, a1);
            for (;;) {
                const int64_t ch = claim_back(st, lane);
                if (ch < 0) break;
                const int64_t c0 = a0 + ch * kChunk, c1 = (c0 + kChunk) < a1 ? (c0 + kChunk) : a1;
                stream_tiles<K>(p.data, c0, c1, c1 - c0, pp.ps, pp.pe, g.rl, g.rh, lane, op);
                pos += covered(pp, c0, c1);
            }
        }
        const uint32_t verdict = finish_piece<K, R, HM, BLOCK>(p, h, misc, pc, pp, slot, op.nwin, pos);
        if (tid == 0) p.slot_rec[slot] = verdict == 0u ? pp.s : -1;
    }
    if (P16 && tid == 0) p.spill_cnt[w] = misc[0];
}

// The exact recount of the records whose 16-bit counters wrapped in the first pass
// (k = 8; skewed input only): the static home ranges, returning adds (HM 1: every
// wrap recorded exactly), results to sum (whole records) or to the recount's slab
// slots and spill lists.  Exits at once when no record wrapped.
template <int K, class Idx, int BLOCK>
__global__ __launch_bounds__(BLOCK) void recount_dense_kernel(Params p) {
    constexpr int NB = 1 << (2 * K);
    constexpr int NW = NB / 2;
    constexpr int NWAVES = BLOCK / 64;
    if (ld_acq(p.flags + kFlagFail) != p.epoch) return;  // nothing wrapped (uniform)
    __shared__ __attribute__((aligned(16))) uint32_t smem[NW + kMisc];
    uint32_t *h = smem;
    uint32_t *misc = smem + NW;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int64_t w = blockIdx.x;
    const Geom g = make_geom<Idx>(p);
    const Range r = home_range(g, w);
    const int64_t base = 2 * (int64_t)p.G + p.pool_cap;  // the recount's slots
    int64_t slot_first = -1, slot_last = -1;
    for (int i = tid; i < NW; i += BLOCK) h[i] = 0u;
    if (tid < kMisc) misc[tid] = 0u;
    __shared__ int64_t s_first;
    if (tid == 0) s_first = r.R0 < r.R1 ? first_record_at<Idx>(p, r.R0) : p.n;
    __syncthreads();
    P16Ctx pc;
    pc.h = h;
    pc.spilled = misc + 3;
    pc.spill_n = misc;
    pc.spill = p.fb_spill + w * (int64_t)p.fb_spill_cap;
    pc.cap = p.fb_spill_cap;
    int npieces = 0;
    for (int64_t s = s_first; s < p.n && r.R0 < r.R1; ++s) {
        if (rec_off<Idx>(p, s) >= r.R1) break;
        Piece pp;
        if (!piece_at<K, Idx>(p, g, s, r, pp)) continue;
        const int k_piece = npieces++;
        if (ld_acq(p.rec_fail + s) != p.epoch) continue;
        pc.rec = s;
        const bool entire = pp.ps == pp.ca && pp.pe == pp.ce;
        const int64_t tp0 = pp.ps >> kTileShift, tp1 = ((pp.pe - 1) >> kTileShift) + 1;
        const int64_t per = (tp1 - tp0 + NWAVES - 1) / NWAVES;
        const int64_t a0 = tp0 + (int64_t)wave * per;
        const int64_t a1 = (a0 + per) < tp1 ? (a0 + per) : tp1;
        const uint32_t n0 = misc[0];
        DenseOp<K, 1, 1, BLOCK> op(h, lane, wave, pc);
        stream_tiles<K>(p.data, a0, a1, per, pp.ps, pp.pe, g.rl, g.rh, lane, op);
        __syncthreads();
        const int sl = k_piece == 0 ? 0 : 1;  // only the first and the last piece can be partial
        uint32_t *dst = p.slab + (base + 2 * w + sl) * (int64_t)NW;
        for (int i = tid; i < NW; i += BLOCK) {
            const uint32_t v = h[i];
            h[i] = 0u;
            if (entire) {
                p.sum[s + p.ld * (int64_t)i] = (int32_t)(v & 0xFFFFu);
                p.sum[s + p.ld * (int64_t)(i + NW)] = (int32_t)(v >> 16);
            } else {
                dst[i] = v;
            }
        }
        __syncthreads();
        const uint32_t n1 = misc[0] < pc.cap ? misc[0] : pc.cap;
        if (entire) {
            for (uint32_t i = n0 + tid; i < n1; i += BLOCK) {
                const Spill e = pc.spill[i];
                atomicAdd(&p.sum[e.rec + p.ld * (int64_t)e.code], e.amount);
            }
            if (tid == 0) __hip_atomic_store(p.rec_direct + s, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (sl == 0) slot_first = s;
            else slot_last = s;
            if (tid == 0 && n1 > n0)
                __hip_atomic_store(p.flags + kFlagFbSpill, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    }
    if (tid == 0) {
        p.slot_rec[base + 2 * w] = slot_first;
        p.slot_rec[base + 2 * w + 1] = slot_last;
        p.fb_spill_cnt[w] = misc[0];
    }
}

// Records cut between slab slots: sum their slots; records without a window in range
// get zeros.  Grid (NW / RW, ny): blockIdx.x picks RW = 4 * RC slab words (NW = 4^k
// words, or 4^k / 2 packed words at k = 8, each holding bins c and c | 0x8000),
// records s = blockIdx.y, blockIdx.y + ny, ...  A record's slots are the first /
// last slots of the home ranges it spans and the thief slots that hold it (or, when
// it wrapped, the recount's slots); the block lists them in LDS, then RC columns of
// 16-byte loads x RR rows of slots sum them with no dependent load in the loop, the
// rows meet in LDS, and the spill entries of the record's slab pieces are added.
// (One thread per word walking the workgroups with a slot_rec test before every
// slab load was latency-bound: 72 us for the ~205 slots of an 8-way shard's record,
// against a 325 us histogram; scripts/shardbench.py.)
constexpr int kRedList = 1024;  // slot candidates listed per chunk
template <int K, class Idx, bool P16>
__global__ __launch_bounds__(256) void reduce_dense_kernel(Params p) {
    constexpr int NB = 1 << (2 * K);
    constexpr int NW = P16 ? NB / 2 : NB;
    constexpr int RC = NW / 4 < 16 ? NW / 4 : 16;  // 16-byte columns
    constexpr int RR = 256 / RC;                   // rows over the slots
    constexpr int RW = 4 * RC;                     // words per block
    constexpr int NH = P16 ? 2 : 1;                // counters per word
    __shared__ uint32_t s_list[kRedList];
    __shared__ uint32_t s_n;
    __shared__ uint32_t s_part[RR][RW * NH];
    __shared__ uint32_t s_out[RW * NH];
    const int tid = threadIdx.x, col = tid % RC, row = tid / RC;
    const int64_t c0 = (int64_t)blockIdx.x * RW;
    const Geom g = make_geom<Idx>(p);
    const int64_t G2 = 2 * (int64_t)p.G;
    const int64_t thief_end = G2 + pool_used(p);
    const int64_t fb_base = G2 + p.pool_cap;
    for (int64_t s = blockIdx.y; s < p.n; s += gridDim.y) {
        int64_t ca, ce;
        record_windows<K, Idx>(p, g, s, ca, ce);
        if (ce <= ca) {
            for (int i = tid; i < RW * NH; i += 256) {
                const int64_t c = c0 + i % RW + (i / RW) * NW;
                p.sum[s + p.ld * c] = 0;
            }
            continue;
        }
        if (ld_acq(p.rec_direct + s) == p.epoch) continue;  // written by a count kernel
        const bool failed = P16 && ld_acq(p.rec_fail + s) == p.epoch;
        const int64_t wf = ((ca >> kTileShift) - g.T0) / g.tpw;
        const int64_t wlast = (((ce - 1) >> kTileShift) - g.T0) / g.tpw;
        // candidate slots: [A0, A1) = the spanned home ranges' two slots, then (first
        // pass) the thief slots [G2, thief_end)
        const int64_t A0 = (failed ? fb_base : 0) + 2 * wf, A1 = (failed ? fb_base : 0) + 2 * wlast + 2;
        const int64_t ncand = (A1 - A0) + (failed ? 0 : thief_end - G2);
        uint32_t acc[4 * NH] = {};
        for (int64_t cb = 0; cb < ncand; cb += kRedList) {
            const int64_t ce2 = (cb + kRedList) < ncand ? (cb + kRedList) : ncand;
            __syncthreads();  // the previous chunk's list is consumed
            if (tid == 0) s_n = 0u;
            __syncthreads();
            for (int64_t j = cb + tid; j < ce2; j += 256) {
                const int64_t sl = j < A1 - A0 ? A0 + j : G2 + (j - (A1 - A0));
                if (p.slot_rec[sl] == s) s_list[atomicAdd(&s_n, 1u)] = (uint32_t)sl;
            }
            __syncthreads();
            const uint32_t n = s_n;
#pragma unroll 4
            for (uint32_t i = row; i < n; i += RR) {
                const uint4 v = reinterpret_cast<const uint4 *>(p.slab + (int64_t)s_list[i] * NW + c0)[col];
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
        if constexpr (P16) {
            // spill entries of the record's slab pieces (first pass: any workgroup's
            // list, thieves included; recount: the spanned ranges' lists)
            const int fl = failed ? kFlagFbSpill : kFlagSpill;
            if (ld_acq(p.flags + fl) == p.epoch) {
                __syncthreads();
                const int64_t l0 = failed ? wf : 0, l1 = failed ? wlast + 1 : p.G;
                for (int64_t l = l0; l < l1; ++l) {
                    const uint32_t cnt0 = failed ? p.fb_spill_cnt[l] : p.spill_cnt[l];
                    const uint32_t cap = failed ? p.fb_spill_cap : p.spill_cap;
                    const uint32_t cnt = cnt0 < cap ? cnt0 : cap;
                    const Spill *sp = (failed ? p.fb_spill : p.spill) + l * (int64_t)cap;
                    for (uint32_t i = tid; i < cnt; i += 256) {
                        const Spill e = sp[i];
                        const int64_t wd = (int64_t)(e.code & (NW - 1)) - c0;
                        if (e.rec == s && wd >= 0 && wd < RW)
                            atomicAdd(&s_out[wd + (e.code >> 15) * RW], (uint32_t)e.amount);
                    }
                }
            }
        }
        __syncthreads();
        for (int i = tid; i < RW * NH; i += 256) {
            const int64_t c = c0 + i % RW + (i / RW) * NW;
            p.sum[s + p.ld * c] = (int32_t)s_out[i];
        }
        __syncthreads();  // s_part / s_out are reused by the next record
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
// HM = histogram mode: 0 = 32-bit bins; 3 = k == 8 packed 16-bit halves (plain adds,
// per-wave scans, wrapped records recounted with returning adds).
template <> struct Cfg<1> { static constexpr int R = 32, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<2> { static constexpr int R = 32, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<3> { static constexpr int R = 32, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<4> { static constexpr int R = 32, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
#ifndef KMC_R5
#define KMC_R5 8
#endif
#ifndef KMC_R6
#define KMC_R6 2
#endif
template <> struct Cfg<5> { static constexpr int R = KMC_R5, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<6> { static constexpr int R = KMC_R6, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<7> { static constexpr int R = 1, BLOCK = 512, HM = 0; static constexpr bool P16 = false; };
template <> struct Cfg<8> { static constexpr int R = 1, BLOCK = 1024, HM = 3; static constexpr bool P16 = true; };

struct DevInfo {
    int cus = 0;
    int occ[KMC_DENSE_MAX_K + 1][2] = {};  // [k][idx64]
};

std::mutex g_mu;
std::vector<DevInfo> g_dev;

// test hooks (kmc_diag_dense_steal): thieves on/off, owners of every third home
// range delayed (100 MHz ticks) so that thieves take their pieces
int g_steal = -1;  // -1: KMC_NO_STEAL decides
uint32_t g_owner_delay = 0;

bool steal_enabled() {
    if (g_steal >= 0) return g_steal != 0;
    static const bool off = [] {
        const char *e = std::getenv("KMC_NO_STEAL");
        return e != nullptr && e[0] == '1';
    }();
    return !off;
}

// A fresh epoch per call: every cross-workgroup word of the workspace (claims, the
// thief pool, record flags) is tagged with it, so no clearing pass is needed and
// values left by earlier calls (or never written) never match.
uint64_t next_epoch() {
    static std::atomic<uint64_t> ctr{(uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() * 2654435761ull};
    uint64_t e = ctr.fetch_add(1) & (kInitBit - 1);
    return e ? e : 1;
}

template <int K, class Idx>
void *kernel_ptr() {
    return reinterpret_cast<void *>(&count_dense_kernel<K, Cfg<K>::R, Cfg<K>::HM, Idx, Cfg<K>::BLOCK>);
}

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
    G = d.cus * d.occ[K][ix];
    return 0;
}

bool check_spill() {
    static const bool on = [] {
        const char *e = std::getenv("KMC_CHECK_SPILL");
        return e != nullptr && e[0] == '1';
    }();
    return on;
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct WsLayout {
    size_t slot_rec, spill_cnt, fb_spill_cnt, claims, wg_ep, pool, flags, rec_direct, rec_fail, slab, spill, fb_spill,
        total;
};

inline WsLayout ws_layout(int k, int G, int64_t n, uint32_t spill_cap, uint32_t fb_cap, uint32_t pool_cap) {
    WsLayout L;
    const bool p16 = k == 8;
    const size_t words = ((size_t)1 << (2 * k)) / (p16 ? 2 : 1);
    const size_t nslot = 2 * (size_t)G + pool_cap + (p16 ? 2 * (size_t)G : 0);
    size_t o = 0;
    L.slot_rec = o;
    o += align256(nslot * sizeof(int64_t));
    L.spill_cnt = o;
    o += align256((size_t)G * sizeof(uint32_t));
    L.fb_spill_cnt = o;
    o += align256((size_t)G * sizeof(uint32_t));
    L.claims = o;
    o += align256((size_t)G * 2 * kClaimWaves * sizeof(uint64_t));
    L.wg_ep = o;
    o += align256((size_t)G * sizeof(uint64_t));
    L.pool = o;
    o += align256(2 * sizeof(uint64_t));
    L.flags = o;
    o += align256(4 * sizeof(uint64_t));
    L.rec_direct = o;
    o += align256((size_t)n * sizeof(uint64_t));
    L.rec_fail = o;
    o += align256((size_t)n * sizeof(uint64_t));
    L.slab = o;
    o += align256(nslot * words * sizeof(uint32_t));
    L.spill = o;
    o += align256((size_t)G * spill_cap * sizeof(Spill));
    L.fb_spill = o;
    o += align256((size_t)G * fb_cap * sizeof(Spill));
    L.total = o;
    return L;
}

// Entries per window, whatever the scan interval: a scan entry moves a multiple of
// T = 32768 out of one field, all of it increments of that field since its last scan;
// a wrap of the recount (HM 1) costs 65 536 increments and emits at most 3 entries.
constexpr uint32_t kSpillWindowsPerEntry = 4096;
static_assert(3u * kSpillWindowsPerEntry <= 65536u && kSpillWindowsPerEntry <= 32768u, "spill capacity bound");
static_assert(KMC_HM3_SCAN >= 0, "scan interval");
inline uint32_t spill_cap_for(int64_t tiles_per_wg) {
    const int64_t windows = tiles_per_wg * kTile;
    return (uint32_t)(windows / kSpillWindowsPerEntry + 64);
}

struct Plan {
    int G;
    uint32_t spill_cap, fb_cap, pool_cap;
    WsLayout L;
};

template <int K, class Idx>
int make_plan(int device, bool derive, int64_t wl, int64_t wh, int64_t n, Plan &pl) {
    int G = 0;
    int e = grid_size<K, Idx>(device, G);
    if (e) return e;
    pl.spill_cap = pl.fb_cap = 0;
    if (!derive) {
        const int64_t tiles = wh > wl ? ((wh + kTile - 1) >> kTileShift) - (wl >> kTileShift) : 0;
        if (tiles < G) G = tiles > 0 ? (int)tiles : 1;
        const int64_t tpw = tiles > 0 ? (tiles + G - 1) / G : 1;
        if (Cfg<K>::P16) {
            pl.fb_cap = spill_cap_for(tpw);  // the recount's own home range: exact bound
            // first pass: thieves add windows beyond their own range; a list that
            // overflows flags its pieces' records for the recount (exact either way)
            pl.spill_cap = 2 * spill_cap_for(tpw);
        }
    }
    pl.G = G;
    pl.pool_cap = 2 * (uint32_t)G;
    pl.L = ws_layout(K, G, n, pl.spill_cap, pl.fb_cap, pl.pool_cap);
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
    int e = make_plan<K, Idx>(device, derive, wl, wh, q.n, pl);
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
    p.slab = reinterpret_cast<uint32_t *>(base + pl.L.slab);
    p.slot_rec = reinterpret_cast<int64_t *>(base + pl.L.slot_rec);
    p.pool_cap = pl.pool_cap;
    p.spill = reinterpret_cast<Spill *>(base + pl.L.spill);
    p.spill_cnt = reinterpret_cast<uint32_t *>(base + pl.L.spill_cnt);
    p.spill_cap = pl.spill_cap;
    p.fb_spill = reinterpret_cast<Spill *>(base + pl.L.fb_spill);
    p.fb_spill_cnt = reinterpret_cast<uint32_t *>(base + pl.L.fb_spill_cnt);
    p.fb_spill_cap = pl.fb_cap;
    p.claims = reinterpret_cast<uint64_t *>(base + pl.L.claims);
    p.wg_ep = reinterpret_cast<uint64_t *>(base + pl.L.wg_ep);
    p.pool = reinterpret_cast<uint64_t *>(base + pl.L.pool);
    p.flags = reinterpret_cast<uint64_t *>(base + pl.L.flags);
    p.rec_direct = reinterpret_cast<uint64_t *>(base + pl.L.rec_direct);
    p.rec_fail = reinterpret_cast<uint64_t *>(base + pl.L.rec_fail);
    p.epoch = next_epoch();
    p.steal = steal_enabled() ? 1 : 0;
    p.owner_delay = g_owner_delay;

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
    if constexpr (Cfg<K>::P16) {
        // exact recount of the records whose 16-bit counters wrapped (skewed input);
        // every workgroup exits at once when none did
        hipLaunchKernelGGL((recount_dense_kernel<K, Idx, Cfg<K>::BLOCK>), dim3(pl.G), dim3(Cfg<K>::BLOCK), 0, st, p);
        he = hipGetLastError();
        if (he != hipSuccess) return (int)he;
    }
    constexpr int NWR = Cfg<K>::P16 ? NB / 2 : NB;  // slab words per slot
    constexpr int RW = NWR / 4 < 16 ? NWR : 64;      // words per reduce block (its RW)
    const unsigned cb = (unsigned)(NWR / RW);
    hipLaunchKernelGGL((reduce_dense_kernel<K, Idx, Cfg<K>::P16>), dim3(cb, (unsigned)std::min<int64_t>(q.n, kMaxGridY)),
                       dim3(256), 0, st, p);
    he = hipGetLastError();
    if (he != hipSuccess) return (int)he;
    // the recount's spill lists are sized by the exact bound of spill_cap_for; with
    // KMC_CHECK_SPILL=1 (tests) the call synchronises and fails rather than return
    // counts that lost entries (the first pass flags its own overflows)
    if (Cfg<K>::P16 && check_spill()) {
        std::vector<uint32_t> cnt(pl.G);
        uint64_t fl = 0;
        he = hipMemcpyAsync(&fl, p.flags + kFlagFail, sizeof(fl), hipMemcpyDeviceToHost, st);
        if (he == hipSuccess)
            he = hipMemcpyAsync(cnt.data(), p.fb_spill_cnt, pl.G * sizeof(uint32_t), hipMemcpyDeviceToHost, st);
        if (he == hipSuccess) he = hipStreamSynchronize(st);
        if (he != hipSuccess) return (int)he;
        if (fl == p.epoch)
            for (uint32_t c : cnt)
                if (c > pl.fb_cap) return KMC_ERR_CAPACITY;
    }
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
size_t workspace_for(int k, int device, bool derive, int64_t wl, int64_t wh, int64_t n) {
    Plan pl;
    int e = 0;
    switch (k) {
        case 1: e = make_plan<1, Idx>(device, derive, wl, wh, n, pl); break;
        case 2: e = make_plan<2, Idx>(device, derive, wl, wh, n, pl); break;
        case 3: e = make_plan<3, Idx>(device, derive, wl, wh, n, pl); break;
        case 4: e = make_plan<4, Idx>(device, derive, wl, wh, n, pl); break;
        case 5: e = make_plan<5, Idx>(device, derive, wl, wh, n, pl); break;
        case 6: e = make_plan<6, Idx>(device, derive, wl, wh, n, pl); break;
        case 7: e = make_plan<7, Idx>(device, derive, wl, wh, n, pl); break;
        case 8: e = make_plan<8, Idx>(device, derive, wl, wh, n, pl); break;
        default: return 0;
    }
    return e ? 0 : pl.L.total;
}

}  // namespace
}  // namespace kmc

using namespace kmc;

// Test hook (not in kmc.h): steal 1/0 switches the thieves on/off (-1: KMC_NO_STEAL
// decides), owner_delay_ticks > 0 makes the owners of every third home range wait
// that many 100 MHz ticks first, so that thieves take their pieces.
extern "C" int kmc_diag_dense_steal(int steal, unsigned owner_delay_ticks) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_steal = steal < 0 ? -1 : (steal ? 1 : 0);
    g_owner_delay = owner_delay_ticks;
    return KMC_OK;
}

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
    return workspace_for<int64_t>(a->k, device, false, wl, wh, (int64_t)a->num_seqs);
}

extern "C" int kmc_count_dense_ex(const kmc_dense_args *a0, hipStream_t stream) {
    if (!a0) return KMC_ERR_INVALID_ARG;
    if (a0->k < 1 || a0->k > KMC_DENSE_MAX_K) return KMC_ERR_UNSUPPORTED_K;
    if (a0->num_seqs == 0) return KMC_OK;
    if (!a0->data || !a0->indices || !a0->sum) return KMC_ERR_INVALID_ARG;
    if (a0->read_hi < a0->read_lo || a0->win_hi < a0->win_lo) return KMC_ERR_INVALID_ARG;
    if (a0->sum_ld != 0 && a0->sum_ld < a0->num_seqs) return KMC_ERR_INVALID_ARG;
    int64_t bias = 0;
    const kmc_dense_args al = aligned_args(a0, bias);
    const kmc_dense_args *a = &al;
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
    return workspace_for<int64_t>(k, device, false, 15, (int64_t)data_bytes + 15, (int64_t)num_seqs);
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
