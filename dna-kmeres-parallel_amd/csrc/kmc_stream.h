// kmc_stream.h — the tile streaming loop shared by the HIP counting kernels.
//
// One wave streams a contiguous run of 1 KiB tiles of the ASCII record buffer
// (64 lanes x 16 B, global_load_dwordx4), decodes each lane's 16 bytes to 2-bit
// codes in registers, attaches the next lane's 16 bases as the (k-1)-base halo
// (lane 63: lane 0 of the next tile, already prefetched), and hands every tile
// to an operation functor: op.tile<MASKED>(lo, hi, W) with lo = the lane's 16
// bases, hi = the next 16, W = 16-bit mask of the windows to count (MASKED ==
// false: all 16).  The functor decides what a window does (LDS histogram add,
// bucket count, bucket scatter, ...).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kmc {

// Tiles kept in flight per wave ahead of the one being counted, and whether the
// once-read sequence stream uses non-temporal (nt) loads: defaults of the dense
// histogram kernels (round 2, same-box A/B: PF 2 -> 3 and nt loads took k = 8 from
// 2.32 to 2.24 ms and k = 1..7 down 2-4 %; profiles/r02_stream_pf_nt_ab.txt); the
// radix walks pass their own (PF 2, plain loads: PF 3 + nt made C3 4 % slower).
constexpr int kStreamPF = 3;
constexpr int kStreamNT = 1;

constexpr int kTileShift = 10;  // 1 KiB per wave per tile
constexpr int kTile = 1 << kTileShift;

// ---------------------------------------------------------------------------
// decode: 16 ASCII bytes (one lane's chunk) -> 32-bit word of 2-bit codes, base i
// at bits 2i (the reference's little-endian bin order), plus validity.
//
// The low 3 bits of A,C,G,T are 1,3,7,4 and distinct, so one v_perm_b32 on
// (w & 0x07070707) maps every byte to its code (a 4-entry table lookup per
// byte) and a second one to the letter that code stands for; a byte is valid
// iff it equals that letter (lowercase, N, '\r', '\0', ... never do).
// ---------------------------------------------------------------------------
constexpr uint32_t kCodeLo = 0x01000000u;   // table[0..3] = {-, A=0, -, C=1}
constexpr uint32_t kCodeHi = 0x02000003u;   // table[4..7] = {T=3, -, -, G=2}
constexpr uint32_t kCanonLo = 0x43FF41FFu;  // table[0..3] = {xx, 'A', xx, 'C'}
constexpr uint32_t kCanonHi = 0x47FFFF54u;  // table[4..7] = {'T', xx, xx, 'G'}

__device__ __forceinline__ uint32_t byte_codes(uint32_t w) {
    return __builtin_amdgcn_perm(kCodeHi, kCodeLo, w & 0x07070707u);
}
__device__ __forceinline__ uint32_t byte_mismatch(uint32_t w) {  // 0 in every valid byte
    return w ^ __builtin_amdgcn_perm(kCanonHi, kCanonLo, w & 0x07070707u);
}

// code = 16 packed 2-bit codes; bad = OR of the per-byte mismatches (0 iff all valid)
__device__ __forceinline__ void decode16(const uint4 r, uint32_t &code, uint32_t &bad) {
    const uint32_t c0 = byte_codes(r.x), c1 = byte_codes(r.y), c2 = byte_codes(r.z), c3 = byte_codes(r.w);
    bad = byte_mismatch(r.x) | byte_mismatch(r.y) | byte_mismatch(r.z) | byte_mismatch(r.w);
    // bytes -> nibbles -> one byte per dword (base 4d+i at bits 2(4d+i))
    const uint32_t u = __builtin_amdgcn_perm(c1, c0, 0x06040200u) | (__builtin_amdgcn_perm(c1, c0, 0x07050301u) << 2);
    const uint32_t v = __builtin_amdgcn_perm(c3, c2, 0x06040200u) | (__builtin_amdgcn_perm(c3, c2, 0x07050301u) << 2);
    code = __builtin_amdgcn_perm(v, u, 0x06040200u) | (__builtin_amdgcn_perm(v, u, 0x07050301u) << 4);
}

// 16-bit invalid-base mask of a chunk (slow path only)
__device__ __forceinline__ uint32_t bad_mask16(const uint4 r) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
    uint32_t bad = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t x = byte_mismatch(w[d]);
        const uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
        bad |= ((((nz >> 7) * 0x00204081u) >> 21) & 0xFu) << (4 * d);
    }
    return bad;
}

// One lane's 16 bytes of tile t; bytes outside [rl, rh) read as 0 (invalid).
__device__ __forceinline__ uint4 load_lane(const char *__restrict__ data, int64_t t, int lane, int64_t rl,
                                           int64_t rh) {
    const int64_t base = t << kTileShift;
    const int64_t q = base + (int64_t)lane * 16;
    if (base >= rl && base + kTile <= rh) {  // wave-uniform: whole tile readable
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(data + q));
        return make_uint4(x[0], x[1], x[2], x[3]);
    }
    uint32_t v[4] = {0u, 0u, 0u, 0u};
    if (q >= rl && q + 16 <= rh) {
        const uint4 x = *reinterpret_cast<const uint4 *>(data + q);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    } else {
#pragma unroll 1
        for (int i = 0; i < 16; ++i) {
            const int64_t b = q + i;
            if (b >= rl && b < rh) v[i >> 2] |= (uint32_t)(uint8_t)data[b] << (8 * (i & 3));
        }
    }
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// OR of x >> 0 .. x >> (K-1): bit j set iff any of bases j .. j+K-1 is invalid.
template <int K>
__device__ __forceinline__ uint32_t smear(uint32_t x) {
    uint32_t s = x;
    int c = 1;
#pragma unroll
    for (int it = 0; it < 6; ++it) {
        if (c < K) {
            const int st = (c < K - c) ? c : (K - c);
            s |= s >> st;
            c += st;
        }
    }
    return s;
}

// Value of lane+1 (lane 63 gets 0): DPP wave_shl:1, no LDS traffic (unlike
// __shfl_down, which is a ds_bpermute).
__device__ __forceinline__ uint32_t from_next_lane(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false);
}

// Inclusive prefix sum over the wave's 64 lanes in six DPP adds (row_shr 1/2/4/8
// within each row of 16, then row_bcast 15 and 31 carry the row totals up): VALU
// only, where a __shfl_up ladder is six ds_bpermute round trips through the LDS.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

// o[t] = x of lane t of this lane's quad (DPP quad_perm broadcasts: VALU, no LDS)
__device__ __forceinline__ void quad_bcast4(uint32_t x, uint32_t *o) {
    o[0] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x00, 0xF, 0xF, false);
    o[1] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x55, 0xF, 0xF, false);
    o[2] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xAA, 0xF, 0xF, false);
    o[3] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xFF, 0xF, 0xF, false);
}

// Workgroup barrier ordering LDS only: unlike __syncthreads() it does not wait for
// the wave's outstanding global loads, so the tile prefetch keeps streaming.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Geometry of a counting launch.  P carries indices, n, derive, wl/wh/rl/rh, G.
struct Geom {
    int64_t wl, wh, rl, rh;
    int64_t T0, T1, tpw;
};

// Record offset i as a position in p.data: indices[i] + p.ibias (the bias is the
// misalignment of the caller's data pointer, which the library rounds down to 16
// bytes: offsets and ranges move up by it, the bytes stay where they are).
template <class Idx, class P>
__device__ __forceinline__ int64_t rec_off(const P &p, int64_t i) {
    return (int64_t)((const Idx *)p.indices)[i] + p.ibias;
}

template <class Idx, class P>
__device__ __forceinline__ Geom make_geom(const P &p) {
    Geom g;
    if (p.derive) {
        g.wl = rec_off<Idx>(p, 0);
        g.wh = rec_off<Idx>(p, p.n);
        g.rl = g.wl;
        g.rh = g.wh;
    } else {
        g.wl = p.wl;
        g.wh = p.wh;
        g.rl = p.rl;
        g.rh = p.rh;
    }
    if (g.wh <= g.wl) {
        g.T0 = g.T1 = 0;
        g.tpw = 1;
    } else {
        g.T0 = g.wl >> kTileShift;
        g.T1 = (g.wh + kTile - 1) >> kTileShift;
        g.tpw = (g.T1 - g.T0 + p.G - 1) / p.G;
    }
    return g;
}

// Window range of record s clipped to the counted range: [ca, ce).
template <int K, class Idx, class P>
__device__ __forceinline__ void record_windows(const P &p, const Geom &g, int64_t s, int64_t &ca,
                                               int64_t &ce) {
    const int64_t a = rec_off<Idx>(p, s);
    const int64_t e = rec_off<Idx>(p, s + 1);
    const int64_t nw = e - a - K > 0 ? e - a - K : 0;  // kernels.h:133 generalised
    ca = a > g.wl ? a : g.wl;
    ce = (a + nw) < g.wh ? (a + nw) : g.wh;
}


// Last record s with indices[s] <= pos (records before it end at or before pos).
template <class Idx, class P>
__device__ __forceinline__ int64_t first_record_at(const P &p, int64_t pos) {
    int64_t lo = 0, hi = p.n - 1;
    if (rec_off<Idx>(p, 0) <= pos) {
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) >> 1;
            if (rec_off<Idx>(p, mid) <= pos) lo = mid;
            else hi = mid - 1;
        }
    }
    return lo;
}

// Prefetch form of load_lane, as a raw buffer load.  The resource covers the
// 16-byte blocks that hold readable bytes, [rl & ~15, (rh + 15) & ~15) (rebased
// at base_off as the wave moves: the range is capped at 2^31 bytes), and the
// hardware range check returns zeros for every lane whose block lies outside
// it (offsets below base_off wrap to huge unsigned values).  So the prefetch is
// one unconditional buffer_load_dwordx4 per lane and tile; in the (at most two)
// tiles holding rl or rh inside a block, mask_range then zeroes the bytes
// outside [rl, rh) in registers.  The blocks at rl and rh never cross a page.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const char *data, int64_t base_off, int64_t rh) {
    const int64_t rh16 = (rh + 15) & ~(int64_t)15;
    int64_t nrec = rh16 - base_off;
    nrec = nrec < 0 ? 0 : (nrec > (1ll << 31) ? (1ll << 31) : nrec);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(data) + base_off, (short)0, (int)nrec,
                                             0x00020000);
}

// base of the resource for tiles from t on
__device__ __forceinline__ int64_t tile_base(int64_t t, int64_t rl) {
    const int64_t b = t << kTileShift, rl16 = rl & ~(int64_t)15;
    return b > rl16 ? b : rl16;
}

template <int NT = kStreamNT>
__device__ __forceinline__ uint4 load_tile_fast(__amdgpu_buffer_rsrc_t rsrc, int64_t base_off, int64_t t,
                                                int lane) {
    const int64_t off = (t << kTileShift) - base_off + (int64_t)lane * 16;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)(uint32_t)off, 0, NT ? 2 : 0);
    return make_uint4(x[0], x[1], x[2], x[3]);
}

// rl or rh lies strictly inside a 16-byte block of tile t (scalar test)
__device__ __forceinline__ bool tile_straddles(int64_t t, int64_t rl, int64_t rh) {
    const int64_t b = t << kTileShift;
    return ((rl & 15) != 0 && rl > b && rl < b + kTile) || ((rh & 15) != 0 && rh > b && rh < b + kTile);
}

// zero the bytes of this lane's 16 (at offset q) that lie outside [rl, rh)
__device__ __forceinline__ uint4 mask_range(uint4 v, int64_t q, int64_t rl, int64_t rh) {
    const int64_t lo = rl - q, hi = rh - q;
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        int64_t a = lo - 4 * d, b = hi - 4 * d;
        a = a < 0 ? 0 : (a > 4 ? 4 : a);
        b = b < 0 ? 0 : (b > 4 ? 4 : b);
        uint32_t m = 0u;
        if (b > a) {
            const uint32_t upto = b == 4 ? 0xFFFFFFFFu : ((1u << (8 * (uint32_t)b)) - 1u);
            m = upto & ~((1u << (8 * (uint32_t)a)) - 1u);
        }
        w[d] &= m;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// One wave streams tiles [t0, t1) and counts the windows that start in [ps, pe),
// over `per` workgroup-uniform iterations (waves with fewer tiles keep calling
// op.after_iter, so workgroup barriers inside it stay matched).  Tile t+1 is
// decoded while tile t is counted (it is lane 63's halo of t).
//
// Prefetch: PF tiles ahead, in a ring of PF+1 register slots whose index
// is a compile-time constant in every step (the loop is unrolled by the ring
// size), issued unconditionally (load_tile_fast) so that no branch merges pending
// and completed loads.  Both matter: register moves between slots (r[q] =
// r[q+1]) or a load inside a branch make the compiler wait for the load it has
// just issued (s_waitcnt vmcnt(0)) before the next decode, which leaves one tile
// in flight per wave whatever PF says.
template <int K, int PF_ = kStreamPF, int NT_ = kStreamNT>
struct TileStream {
    static constexpr int PF = PF_;
    static constexpr int NT = NT_;
    static constexpr int NS = PF + 1;
    const char *__restrict__ data;
    int64_t t0, ps, pe, rl, rh;
    int lane;
    __amdgpu_buffer_rsrc_t rsrc;
    int64_t base_off;
    uint4 r[NS];
    uint32_t c_cur, v_cur;

    // step i (tile t0 + i < t1); S = i mod NS is the slot of tile t0 + i
    template <int S, class Op>
    __device__ __forceinline__ void step(int64_t i, int64_t per, Op &op) {
        const int64_t t = t0 + i;
        constexpr int SN = (S + 1) % NS, SL = (S + PF) % NS;
        r[SL] = load_tile_fast<NT>(rsrc, base_off, t + PF, lane);
        if (tile_straddles(t + 1, rl, rh))
            r[SN] = mask_range(r[SN], ((t + 1) << kTileShift) + (int64_t)lane * 16, rl, rh);
        const uint4 r_cur = r[S], r_nxt = r[SN];
        uint32_t c_nxt, v_nxt;
        decode16(r_nxt, c_nxt, v_nxt);
        // halo: next lane's 16 bases; lane 63 takes lane 0 of the next tile
        uint32_t hc = from_next_lane(c_cur);
        uint32_t hv = from_next_lane(v_cur);
        const uint32_t c0 = __builtin_amdgcn_readlane(c_nxt, 0);
        const uint32_t v0 = __builtin_amdgcn_readlane(v_nxt, 0);
        if (lane == 63) {
            hc = c0;
            hv = v0;
        }
        op.before_tile();
        const int64_t base = t << kTileShift;
        const bool interior = base >= ps && base + kTile <= pe;  // wave-uniform
        if (interior && !__any((v_cur | hv) != 0u)) {
            op.template tile<false>(c_cur, hc, 0xFFFFu);
        } else {
            // boundary tile or invalid bytes: exact per-window mask
            const int64_t pos = base + (int64_t)lane * 16;
            const int64_t dlo = ps - pos, dhi = pe - pos;
            const uint32_t mhi = dhi >= 16 ? 0xFFFFu : (dhi <= 0 ? 0u : ((1u << (uint32_t)dhi) - 1u));
            const uint32_t mlo = dlo <= 0 ? 0xFFFFu : (dlo >= 16 ? 0u : ((0xFFFFu << (uint32_t)dlo) & 0xFFFFu));
            const uint32_t b_own = bad_mask16(r_cur);
            uint32_t b_next = from_next_lane(b_own);
            const uint32_t b0 = __builtin_amdgcn_readlane(bad_mask16(r_nxt), 0);
            if (lane == 63) b_next = b0;
            const uint32_t W = ~smear<K>(b_own | (b_next << 16)) & mhi & mlo & 0xFFFFu;
            op.template tile<true>(c_cur, hc, W);
        }
        c_cur = c_nxt;
        v_cur = v_nxt;
        op.after_iter(i, per, true);
    }

    // steps i .. i+NS-1, stopping at n (the wave's tile count)
    template <int S, class Op>
    __device__ __forceinline__ void steps(int64_t i, int64_t n, int64_t per, Op &op) {
        if constexpr (S < NS) {
            if constexpr (S == 0) {
                base_off = tile_base(t0 + i, rl);
                rsrc = tile_rsrc(data, base_off, rh);
            }
            if (i + S < n) {
                step<S>(i + S, per, op);
                steps<S + 1>(i, n, per, op);
            }
        }
    }
};

template <int K, class Op, int PF = kStreamPF, int NT = kStreamNT>
__device__ __forceinline__ void stream_tiles(const char *__restrict__ data, int64_t t0, int64_t t1, int64_t per,
                                             int64_t ps, int64_t pe, int64_t rl, int64_t rh, int lane, Op &op) {
    using TS = TileStream<K, PF, NT>;
    const int64_t n = t1 > t0 ? t1 - t0 : 0;  // <= per
    if (n > 0) {
        TS ts;
        ts.data = data;
        ts.t0 = t0;
        ts.ps = ps;
        ts.pe = pe;
        ts.rl = rl;
        ts.rh = rh;
        ts.lane = lane;
#pragma unroll
        for (int q = 0; q < TS::NS; ++q) ts.r[q] = make_uint4(0u, 0u, 0u, 0u);
        ts.base_off = tile_base(t0, rl);
        ts.rsrc = tile_rsrc(data, ts.base_off, rh);
#pragma unroll
        for (int q = 0; q < TS::PF; ++q) ts.r[q] = load_tile_fast<NT>(ts.rsrc, ts.base_off, t0 + q, lane);
        if (tile_straddles(t0, rl, rh)) ts.r[0] = mask_range(ts.r[0], (t0 << kTileShift) + (int64_t)lane * 16, rl, rh);
        decode16(ts.r[0], ts.c_cur, ts.v_cur);
        for (int64_t i = 0; i < n; i += TS::NS) ts.template steps<0>(i, n, per, op);
    }
    for (int64_t i = n; i < per; ++i) op.after_iter(i, per, false);
}

// ---------------------------------------------------------------------------
// Chunked streaming (round 5, the dense histogram): the tiles of a piece are
// handed to the workgroup's waves in chunks of C tiles from an LDS counter instead
// of one contiguous run per wave.  Waves of one workgroup do not run at one speed
// on the LDS-bound k = 8 histogram: between two hot-half scans (256 tiles per wave)
// the fastest took 131 us and the slowest 239 us, and every scan barrier waits for
// the slowest (scripts/dense_phase_prof.py, profiles/r05m_dense_phase_prof.txt).
// Each wave takes its next chunk when it starts the current one, so the prefetch
// ring runs on into it without a break; the halo of a chunk's last tile (lane 0 of
// the physically next tile, which belongs to another chunk) is loaded by lane 0
// alone at the chunk's start.  SEGC > 0: after every SEGC chunks of the piece the
// waves meet for op.segment_end() (the k = 8 scans), each wave once per segment
// boundary whether or not it took a chunk in between.
template <int K, int C, int PF = kStreamPF, int NT = kStreamNT>
struct ChunkStream {
    static constexpr int NS = PF + 1;
    static_assert(C % NS == 0 && C > PF, "a chunk is whole turns of the prefetch ring");
    const char *__restrict__ data;
    int64_t ps, pe, rl, rh, tend;
    int lane;
    __amdgpu_buffer_rsrc_t rsrc;
    int64_t base_off;
    int64_t cb, nb;  // the current chunk's first tile; the next one's (-1: none)
    uint4 r[NS];
    uint4 hz;        // lane 0: the 16 bytes at tile cb + C (the halo of the chunk's last tile)
    uint32_t c_cur, v_cur;

    // tile t of this lane, or zeros (no memory access) when !valid
    __device__ __forceinline__ uint4 load_sel(int64_t t, bool valid) const {
        const int64_t off = (t << kTileShift) - base_off + (int64_t)lane * 16;
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, valid ? (int)(uint32_t)off : -16, 0, NT ? 2 : 0);
        return make_uint4(x[0], x[1], x[2], x[3]);
    }

    // a new current chunk: resource based at it, the halo of its last tile
    __device__ __forceinline__ void begin_chunk() {
        base_off = tile_base(cb, rl);
        rsrc = tile_rsrc(data, base_off, rh);
        const int64_t th = cb + C;
        hz = load_sel(th, lane == 0);
        if (tile_straddles(th, rl, rh)) hz = mask_range(hz, th << kTileShift, rl, rh);
    }

    // position j (j % NS == S) of the current chunk
    template <int S, class Op>
    __device__ __forceinline__ void step(int j, Op &op) {
        const int64_t t = cb + j;
        constexpr int SN = (S + 1) % NS, SL = (S + PF) % NS;
        const int jl = j + PF;  // the tile PF positions ahead: this chunk's, or the next one's
        r[SL] = jl < C ? load_sel(cb + jl, true) : load_sel(nb + (jl - C), nb >= 0);
        const int64_t tn = j + 1 < C ? t + 1 : nb;  // the tile after t in this wave's sequence
        if (tn >= 0 && tile_straddles(tn, rl, rh))
            r[SN] = mask_range(r[SN], (tn << kTileShift) + (int64_t)lane * 16, rl, rh);
        const uint4 r_cur = r[S], r_nxt = r[SN];
        uint32_t c_nxt, v_nxt;
        decode16(r_nxt, c_nxt, v_nxt);
        // halo: next lane's 16 bases; lane 63 takes lane 0 of tile t + 1 -- the next
        // in the sequence, except after the chunk's last tile
        const bool edge = S == NS - 1 && j == C - 1;  // (wave-uniform)
        uint32_t c_h = c_nxt, v_h = v_nxt;
        if (edge) decode16(hz, c_h, v_h);
        uint32_t hc = from_next_lane(c_cur);
        uint32_t hv = from_next_lane(v_cur);
        const uint32_t c0 = __builtin_amdgcn_readlane(c_h, 0);
        const uint32_t v0 = __builtin_amdgcn_readlane(v_h, 0);
        if (lane == 63) {
            hc = c0;
            hv = v0;
        }
        op.before_tile();
        const int64_t base = t << kTileShift;
        const bool interior = base >= ps && base + kTile <= pe;  // wave-uniform
        if (interior && !__any((v_cur | hv) != 0u)) {
            op.template tile<false>(c_cur, hc, 0xFFFFu);
        } else {
            const int64_t pos = base + (int64_t)lane * 16;
            const int64_t dlo = ps - pos, dhi = pe - pos;
            const uint32_t mhi = dhi >= 16 ? 0xFFFFu : (dhi <= 0 ? 0u : ((1u << (uint32_t)dhi) - 1u));
            const uint32_t mlo = dlo <= 0 ? 0xFFFFu : (dlo >= 16 ? 0u : ((0xFFFFu << (uint32_t)dlo) & 0xFFFFu));
            const uint32_t b_own = bad_mask16(r_cur);
            uint32_t b_next = from_next_lane(b_own);
            const uint32_t b0 = __builtin_amdgcn_readlane(bad_mask16(edge ? hz : r_nxt), 0);
            if (lane == 63) b_next = b0;
            const uint32_t W = ~smear<K>(b_own | (b_next << 16)) & mhi & mlo & 0xFFFFu;
            op.template tile<true>(c_cur, hc, W);
        }
        c_cur = c_nxt;
        v_cur = v_nxt;
    }

    // positions j .. j+NS-1 of the current chunk, stopping at the piece's end
    template <int S, class Op>
    __device__ __forceinline__ void steps(int j, Op &op) {
        if constexpr (S < NS) {
            if (cb + j + S < tend) {
                step<S>(j + S, op);
                steps<S + 1>(j, op);
            }
        }
    }
};

template <int K, int C, int SEGC, class Op, int PF = kStreamPF, int NT = kStreamNT>
__device__ __forceinline__ void stream_chunks(const char *__restrict__ data, int64_t tp0, int64_t tp1, int64_t ps,
                                              int64_t pe, int64_t rl, int64_t rh, int lane, uint32_t *ctr, Op &op) {
    using CS = ChunkStream<K, C, PF, NT>;
    const int64_t nch = tp1 > tp0 ? (tp1 - tp0 + C - 1) / C : 0;
    const auto grab = [&]() -> int64_t {  // the next chunk of the piece, or -1 (wave-uniform)
        uint32_t c = 0u;
        if (lane == 0) c = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        c = __builtin_amdgcn_readfirstlane(c);
        return (int64_t)c < nch ? (int64_t)c : -1;
    };
    int64_t seg = 0;  // segment boundaries this wave has passed
    int64_t c = grab();
    if (c >= 0) {
        CS cs;
        cs.data = data;
        cs.ps = ps;
        cs.pe = pe;
        cs.rl = rl;
        cs.rh = rh;
        cs.tend = tp1;
        cs.lane = lane;
        cs.cb = tp0 + c * C;
        cs.nb = -1;
        cs.begin_chunk();
#pragma unroll
        for (int q = 0; q < CS::NS; ++q) cs.r[q] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int q = 0; q < PF; ++q) cs.r[q] = cs.load_sel(cs.cb + q, true);
        if (tile_straddles(cs.cb, rl, rh))
            cs.r[0] = mask_range(cs.r[0], (cs.cb << kTileShift) + (int64_t)lane * 16, rl, rh);
        decode16(cs.r[0], cs.c_cur, cs.v_cur);
        int64_t nc = grab();
        for (;;) {
            cs.nb = nc >= 0 ? tp0 + nc * C : -1;
            for (int j = 0; j < C; j += CS::NS) cs.template steps<0>(j, op);
            if (nc < 0) break;
            if constexpr (SEGC > 0) {
                for (; seg < nc / SEGC; ++seg) op.segment_end();
            }
            cs.cb = cs.nb;
            cs.begin_chunk();
            nc = grab();
        }
    }
    if constexpr (SEGC > 0) {
        const int64_t nseg = (nch + SEGC - 1) / SEGC;
        for (; seg < nseg - 1; ++seg) op.segment_end();
    }
}

// Code of window j (bases j .. j+K-1, K <= 16) of a lane with bases lo : hi.
template <int K>
__device__ __forceinline__ uint32_t window_code_rt(uint32_t lo, uint32_t hi, int j) {
    constexpr uint32_t M = (K >= 16) ? 0xFFFFFFFFu : ((1u << (2 * K)) - 1u);
    return __builtin_amdgcn_alignbit(hi, lo, 2 * j) & M;
}

}  // namespace kmc
