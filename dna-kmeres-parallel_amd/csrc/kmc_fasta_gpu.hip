// kmc_fasta_gpu.hip — FASTA parsing on the GPU: the record
// rules of importSeqs / importSeqsNoNL (reference main.cu:474-545 / 401-473, as
// restated by kmc_fasta.cpp, uncapped) applied to the raw file bytes in HBM, so
// the host only moves bytes (the reference's getline parse runs at ~0.2 GB/s and
// dominates its end-to-end time).
//
// The reference's loop is a three-state machine over lines (split on '\n'):
//   OUT       between records                (empty / other lines: skipped)
//   OUT_NEW   a '>' header was seen          (the next non-empty, non-header line opens a record)
//   IN        inside a record                (lines are appended; an empty line, a line starting
//                                             with '\r', or with dialect 1 a '>' line closes it)
// Every line is a function state -> state of its class (empty, header, '\r', other),
// so the state before each line is an exclusive prefix of function compositions
// (associative, not commutative): a parallel scan.  Then every byte is kept or
// dropped from its line's action alone, and a byte-level stream compaction writes
// the record buffer: appended bytes ('|' -> '\0'), one '\0' at each closing line,
// one at end of input when a record is still open; record offsets at the opening
// lines.  Passes over the raw bytes (16 KiB tiles): newline count, line classes,
// kept-byte count, write.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <vector>

#include "kmc.h"
#include "kmc_scan.h"
#include "kmc_stream.h"

namespace kmc {
namespace {

constexpr int kFpBlock = 256;
constexpr int kFpPer = 64;                        // raw bytes per thread
constexpr int64_t kFpTile = kFpBlock * kFpPer;    // 16 KiB per block
constexpr int kLsPer = 16;                        // lines per thread in the line scan
constexpr int64_t kLsTile = (int64_t)kFpBlock * kLsPer;

// line classes, encoded as their state functions: f(s) = (f >> 2s) & 3
// states: 0 = OUT, 1 = OUT_NEW, 2 = IN
constexpr uint32_t kFnId = 0x24;       // s -> s
constexpr uint32_t kFnEmpty = 0x04;    // 0->0 1->1 2->0 (closes a record)
constexpr uint32_t kFnCr = 0x08;       // 0->0 1->2 2->0 (opens after a header; closes)
constexpr uint32_t kFnOther = 0x28;    // 0->0 1->2 2->2
constexpr uint32_t kFnHdr0 = 0x25;     // 0->1 1->1 2->2 (importSeqs: a '>' line inside a record is text)
constexpr uint32_t kFnHdr1 = 0x15;     // 0->1 1->1 2->1 (importSeqsNoNL: it closes and starts the next)

constexpr uint8_t kActAppend = 1, kActClose = 2, kActOpen = 4;

__device__ __forceinline__ uint32_t fthen(uint32_t a, uint32_t b) {  // a, then b
    uint32_t r = 0;
#pragma unroll
    for (int s = 0; s < 3; ++s) r |= ((b >> (2 * ((a >> (2 * s)) & 3))) & 3u) << (2 * s);
    return r;
}

__device__ __forceinline__ uint8_t line_action(uint32_t state, uint32_t fn) {
    if (state == 1) return (fn == kFnCr || fn == kFnOther) ? (kActOpen | kActAppend) : 0;
    if (state == 2) {
        if (fn == kFnEmpty || fn == kFnCr || fn == kFnHdr1) return kActClose;
        return kActAppend;  // other, or a header with dialect 0
    }
    return 0;
}

struct FParams {
    const uint8_t *raw;
    int64_t n;            // raw bytes
    int dialect;
    int64_t ntiles;       // raw tiles
    uint32_t *tile_nl;    // [ntiles] newlines per tile
    uint64_t *tile_lb;    // [ntiles + 1] first line of each tile
    uint8_t *fn;          // [lines] state function of each line
    uint8_t *act;         // [lines] action of each line
    int64_t nlines;
    int64_t ltiles;       // line-scan tiles
    uint32_t *lagg;       // [ltiles] composed function of each line tile, then its exclusive prefix
    uint32_t *lfinal;     // [1] composition of every line
    uint32_t *tile_keep;  // [ntiles]
    uint64_t *tile_ob;    // [ntiles + 1] output offset of each tile
    uint32_t *tile_open;  // [ntiles]
    uint64_t *tile_rb;    // [ntiles + 1] first record opened in each tile
    uint8_t *out;
    int64_t *idx;
    uint64_t *result;     // [2]: records, data bytes
};

// a thread's 64 raw bytes as 16 little-endian words (bytes past n read as 0)
__device__ __forceinline__ void load64(const FParams &p, int64_t q, uint32_t w[16]) {
    if (q + kFpPer <= p.n) {
        const uint4 *s = reinterpret_cast<const uint4 *>(p.raw + q);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 v = s[i];
            w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = 0u;
        for (int i = 0; i < kFpPer; ++i)
            if (q + i < p.n) w[i >> 2] |= (uint32_t)p.raw[q + i] << (8 * (i & 3));
    }
}

__device__ __forceinline__ uint32_t nl_bits(uint32_t x) {  // bit 8i+7 set iff byte i == '\n'
    const uint32_t y = x ^ 0x0A0A0A0Au;
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
}

__device__ __forceinline__ uint32_t count_nl(const uint32_t w[16]) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) c += __popc(nl_bits(w[i]));
    return c;
}

// block exclusive sum of a per-thread value (kFpBlock threads); total returned
__device__ __forceinline__ uint32_t block_excl_u32(uint32_t v, uint32_t *sh, uint32_t &total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
    for (int i = 0; i < kFpBlock / 64; ++i) {
        if (i < wid) before += sh[i];
        total += sh[i];
    }
    __syncthreads();
    return before + x - v;
}

// 1. newlines per tile
__global__ __launch_bounds__(kFpBlock) void fp_count_kernel(FParams p) {
    __shared__ uint32_t sh[kFpBlock / 64];
    uint32_t w[16];
    load64(p, (int64_t)blockIdx.x * kFpTile + (int64_t)threadIdx.x * kFpPer, w);
    uint32_t total;
    block_excl_u32(count_nl(w), sh, total);
    if (threadIdx.x == 0) p.tile_nl[blockIdx.x] = total;
}

// Walks a thread's bytes in order: f(pos, byte, line, is_line_start) for every
// byte below n; `line` counts the newlines before pos.
template <class F>
__device__ __forceinline__ void walk(const FParams &p, int64_t q, const uint32_t w[16], uint64_t line, F &&f) {
    if (q >= p.n) return;
    bool start = q == 0 || p.raw[q - 1] == '\n';
    for (int i = 0; i < kFpPer; ++i) {
        if (q + i >= p.n) break;
        const uint32_t b = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
        f(q + i, b, line, start);
        start = b == '\n';
        line += start;
    }
}

__device__ __forceinline__ uint64_t thread_first_line(const FParams &p, const uint32_t w[16], uint32_t *sh) {
    uint32_t total;
    const uint32_t before = block_excl_u32(count_nl(w), sh, total);
    return p.tile_lb[blockIdx.x] + before;
}

// 2. state function of every line (at its first byte)
__global__ __launch_bounds__(kFpBlock) void fp_class_kernel(FParams p) {
    __shared__ uint32_t sh[kFpBlock / 64];
    const int64_t q = (int64_t)blockIdx.x * kFpTile + (int64_t)threadIdx.x * kFpPer;
    uint32_t w[16];
    load64(p, q, w);
    const uint64_t l0 = thread_first_line(p, w, sh);
    const uint32_t hdr = p.dialect == 1 ? kFnHdr1 : kFnHdr0;
    walk(p, q, w, l0, [&](int64_t, uint32_t b, uint64_t line, bool start) {
        if (start)
            p.fn[line] = (uint8_t)(b == '\n' ? kFnEmpty : b == '>' ? hdr : b == '\r' ? kFnCr : kFnOther);
    });
}

// 3. exclusive composition scan over lines (three phases, kLsTile lines per block)
__device__ __forceinline__ uint32_t block_excl_fn(uint32_t v, uint32_t *sh, uint32_t &total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x = fthen(y, x);
    }
    uint32_t ex = __shfl_up(x, 1);
    if (lane == 0) ex = kFnId;
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    uint32_t before = kFnId;
    total = kFnId;
    for (int i = 0; i < kFpBlock / 64; ++i) {
        if (i < wid) before = fthen(before, sh[i]);
        total = fthen(total, sh[i]);
    }
    __syncthreads();
    return fthen(before, ex);
}

__device__ __forceinline__ uint32_t thread_fn(const FParams &p, int64_t l0) {
    uint32_t f = kFnId;
    for (int i = 0; i < kLsPer; ++i)
        if (l0 + i < p.nlines) f = fthen(f, p.fn[l0 + i]);
    return f;
}

__global__ __launch_bounds__(kFpBlock) void fp_lscan_reduce_kernel(FParams p) {
    __shared__ uint32_t sh[kFpBlock / 64];
    const int64_t l0 = (int64_t)blockIdx.x * kLsTile + (int64_t)threadIdx.x * kLsPer;
    uint32_t total;
    block_excl_fn(thread_fn(p, l0), sh, total);
    if (threadIdx.x == 0) p.lagg[blockIdx.x] = total;
}

__global__ __launch_bounds__(kFpBlock) void fp_lscan_top_kernel(FParams p) {
    __shared__ uint32_t sh[kFpBlock / 64];
    uint32_t carry = kFnId;
    for (int64_t base = 0; base < p.ltiles; base += kFpBlock) {
        const int64_t i = base + threadIdx.x;
        const uint32_t v = i < p.ltiles ? p.lagg[i] : kFnId;
        uint32_t total;
        const uint32_t ex = block_excl_fn(v, sh, total);
        if (i < p.ltiles) p.lagg[i] = fthen(carry, ex);
        carry = fthen(carry, total);
    }
    if (threadIdx.x == 0) p.lfinal[0] = carry;
}

__global__ __launch_bounds__(kFpBlock) void fp_lscan_apply_kernel(FParams p) {
    __shared__ uint32_t sh[kFpBlock / 64];
    const int64_t l0 = (int64_t)blockIdx.x * kLsTile + (int64_t)threadIdx.x * kLsPer;
    uint32_t total;
    uint32_t f = fthen(p.lagg[blockIdx.x], block_excl_fn(thread_fn(p, l0), sh, total));
    for (int i = 0; i < kLsPer; ++i) {
        const int64_t l = l0 + i;
        if (l >= p.nlines) break;
        const uint32_t fl = p.fn[l];
        p.act[l] = line_action(f & 3u, fl);  // state before line l = prefix(OUT)
        f = fthen(f, fl);
    }
}

// kept bytes and opened records of a thread
__device__ __forceinline__ void keep_counts(const FParams &p, int64_t q, const uint32_t w[16], uint64_t l0,
                                            uint32_t &kept, uint32_t &opens) {
    kept = 0;
    opens = 0;
    uint64_t cur = ~0ull;
    uint8_t a = 0;
    walk(p, q, w, l0, [&](int64_t, uint32_t b, uint64_t line, bool start) {
        if (line != cur) {
            cur = line;
            a = p.act[line];
        }
        if (start && (a & kActOpen)) ++opens;
        kept += (b == '\n') ? ((a & kActClose) ? 1u : 0u) : ((a & kActAppend) ? 1u : 0u);
    });
}

// 4. kept bytes and opened records per tile
__global__ __launch_bounds__(kFpBlock) void fp_keep_kernel(FParams p) {
    __shared__ uint32_t sh[kFpBlock / 64];
    const int64_t q = (int64_t)blockIdx.x * kFpTile + (int64_t)threadIdx.x * kFpPer;
    uint32_t w[16];
    load64(p, q, w);
    const uint64_t l0 = thread_first_line(p, w, sh);
    uint32_t kept, opens, tk, to;
    keep_counts(p, q, w, l0, kept, opens);
    block_excl_u32(kept, sh, tk);
    block_excl_u32(opens, sh, to);
    if (threadIdx.x == 0) {
        p.tile_keep[blockIdx.x] = tk;
        p.tile_open[blockIdx.x] = to;
    }
}

// 5. write: the tile's kept bytes are staged in LDS, then stored with whole
// dwords except the first and last partial dword of the tile's output range
__global__ __launch_bounds__(kFpBlock) void fp_write_kernel(FParams p) {
    __shared__ uint32_t sh[kFpBlock / 64];
    __shared__ __attribute__((aligned(16))) uint8_t stage[kFpTile + 8];
    const int64_t q = (int64_t)blockIdx.x * kFpTile + (int64_t)threadIdx.x * kFpPer;
    uint32_t w[16];
    load64(p, q, w);
    const uint64_t l0 = thread_first_line(p, w, sh);
    uint32_t kept, opens, tk, to;
    keep_counts(p, q, w, l0, kept, opens);
    const uint32_t kbefore = block_excl_u32(kept, sh, tk);
    const uint32_t obefore = block_excl_u32(opens, sh, to);
    const uint64_t ob = p.tile_ob[blockIdx.x];
    const uint32_t shift = (uint32_t)(ob & 3u);
    uint32_t o = kbefore;
    uint64_t rec = p.tile_rb[blockIdx.x] + obefore;
    uint64_t cur = ~0ull;
    uint8_t a = 0;
    walk(p, q, w, l0, [&](int64_t, uint32_t b, uint64_t line, bool start) {
        if (line != cur) {
            cur = line;
            a = p.act[line];
        }
        if (start && (a & kActOpen)) p.idx[rec++] = (int64_t)(ob + o);
        if (b == '\n') {
            if (a & kActClose) stage[shift + o++] = 0;
        } else if (a & kActAppend) {
            stage[shift + o++] = b == '|' ? 0 : (uint8_t)b;  // main.cu:538-540
        }
    });
    __syncthreads();
    // stage[shift + i] is output byte ob + i, i < tk
    const uint64_t gbeg = ob, gend = ob + tk;
    const uint64_t d0 = (gbeg + 3) >> 2, d1 = gend >> 2;  // whole output dwords [d0, d1)
    const uint32_t *st32 = reinterpret_cast<const uint32_t *>(stage);
    uint32_t *out32 = reinterpret_cast<uint32_t *>(p.out);
    const uint64_t sbase = gbeg & ~(uint64_t)3;  // output address of stage[0]
    for (uint64_t d = d0 + threadIdx.x; d < d1; d += kFpBlock) out32[d] = st32[(d * 4 - sbase) >> 2];
    if (threadIdx.x == 0) {
        const uint64_t hend = std::min<uint64_t>(d0 * 4, gend);
        for (uint64_t g = gbeg; g < hend; ++g) p.out[g] = stage[g - sbase];
        const uint64_t tbeg = std::max<uint64_t>(d1 * 4, hend);
        for (uint64_t g = tbeg; g < gend; ++g) p.out[g] = stage[g - sbase];
    }
}

// 6. end of input: close a record left open (or closed by a last line without
// '\n'), write the end offset
__global__ void fp_finish_kernel(FParams p, int has_tail) {
    uint64_t total = p.tile_ob[p.ntiles];
    const uint64_t nrec = p.tile_rb[p.ntiles];
    const bool open_at_end = (p.lfinal[0] & 3u) == 2u;
    const bool tail_close = has_tail && (p.act[p.nlines - 1] & kActClose);
    if (open_at_end || tail_close) p.out[total++] = 0;
    p.idx[nrec] = (int64_t)total;
    p.result[0] = nrec;
    p.result[1] = total;
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
struct FCache {
    void *ptr = nullptr;
    size_t bytes = 0;
};
std::mutex f_mu;
std::vector<FCache> f_ws[2];  // [0]: per-tile arrays (sized from the raw bytes), [1]: per-line arrays

inline size_t fal(size_t x) { return (x + 255) & ~(size_t)255; }

int f_workspace(int which, size_t need, char **out) {
    int device = 0;
    hipError_t he = hipGetDevice(&device);
    if (he != hipSuccess) return (int)he;
    std::lock_guard<std::mutex> lk(f_mu);
    std::vector<FCache> &v = f_ws[which];
    if ((int)v.size() <= device) v.resize(device + 1);
    FCache &c = v[device];
    if (c.bytes < need) {
        if (c.ptr && hipFree(c.ptr) != hipSuccess) return KMC_ERR_NOMEM;
        c.ptr = nullptr;
        c.bytes = 0;
        if (hipMalloc(&c.ptr, need) != hipSuccess) return KMC_ERR_NOMEM;
        c.bytes = need;
    }
    *out = static_cast<char *>(c.ptr);
    return 0;
}

// Parses raw[0, n) into out (capacity >= n + 1 always suffices) and the record
// offsets; `get_idx(num_records)` supplies the offsets buffer (num_records + 1
// entries) once the count is known, or returns null to stop with the counts only.
template <class GetIdx>
int parse_device(const char *raw, uint64_t n, int dialect, char *out, uint64_t out_cap, GetIdx &&get_idx,
                 uint64_t *num_seqs, uint64_t *data_bytes, hipStream_t st) {
    *num_seqs = 0;
    *data_bytes = 0;
    hipError_t he;
    if (n == 0) {
        int64_t *idx = get_idx((uint64_t)0);
        if (!idx) return KMC_ERR_NOMEM;
        const int64_t zero = 0;
        if ((he = hipMemcpyAsync(idx, &zero, 8, hipMemcpyHostToDevice, st)) || (he = hipStreamSynchronize(st)))
            return (int)he;
        return 0;
    }
    if (out_cap < n + 1) return KMC_ERR_CAPACITY;
    FParams p{};
    p.raw = reinterpret_cast<const uint8_t *>(raw);
    p.n = (int64_t)n;
    p.dialect = dialect;
    p.ntiles = (int64_t)((n + kFpTile - 1) / kFpTile);
    size_t o = 0;
    const size_t o_tnl = o; o += fal(p.ntiles * 4);
    const size_t o_tlb = o; o += fal((p.ntiles + 1) * 8);
    const size_t o_tk = o; o += fal(p.ntiles * 4);
    const size_t o_tob = o; o += fal((p.ntiles + 1) * 8);
    const size_t o_to = o; o += fal(p.ntiles * 4);
    const size_t o_trb = o; o += fal((p.ntiles + 1) * 8);
    const size_t o_bs = o; o += fal((scan_tiles(p.ntiles) + 1) * 8);
    const size_t o_res = o; o += fal(2 * 8);
    const size_t o_lfin = o; o += fal(4);
    char *ws = nullptr;
    int e = f_workspace(0, o, &ws);
    if (e) return e;
    p.tile_nl = reinterpret_cast<uint32_t *>(ws + o_tnl);
    p.tile_lb = reinterpret_cast<uint64_t *>(ws + o_tlb);
    p.tile_keep = reinterpret_cast<uint32_t *>(ws + o_tk);
    p.tile_ob = reinterpret_cast<uint64_t *>(ws + o_tob);
    p.tile_open = reinterpret_cast<uint32_t *>(ws + o_to);
    p.tile_rb = reinterpret_cast<uint64_t *>(ws + o_trb);
    uint64_t *bsum = reinterpret_cast<uint64_t *>(ws + o_bs);
    p.result = reinterpret_cast<uint64_t *>(ws + o_res);
    p.lfinal = reinterpret_cast<uint32_t *>(ws + o_lfin);
    // newlines -> line count
    hipLaunchKernelGGL(fp_count_kernel, dim3((unsigned)p.ntiles), dim3(kFpBlock), 0, st, p);
    excl_scan_u32(p.tile_nl, p.ntiles, bsum, p.tile_lb, st);
    uint64_t nl = 0;
    uint8_t last = 0;
    if ((he = hipGetLastError()) || (he = hipMemcpyAsync(&nl, p.tile_lb + p.ntiles, 8, hipMemcpyDeviceToHost, st)) ||
        (he = hipMemcpyAsync(&last, raw + n - 1, 1, hipMemcpyDeviceToHost, st)) || (he = hipStreamSynchronize(st)))
        return (int)he;
    const int has_tail = last != '\n';
    p.nlines = (int64_t)nl + has_tail;
    p.ltiles = (p.nlines + kLsTile - 1) / kLsTile;
    o = 0;
    const size_t o_fn = o; o += fal((size_t)p.nlines);
    const size_t o_act = o; o += fal((size_t)p.nlines);
    const size_t o_lagg = o; o += fal((size_t)(p.ltiles + 1) * 4);
    if ((e = f_workspace(1, o, &ws))) return e;
    p.fn = reinterpret_cast<uint8_t *>(ws + o_fn);
    p.act = reinterpret_cast<uint8_t *>(ws + o_act);
    p.lagg = reinterpret_cast<uint32_t *>(ws + o_lagg);
    // line states -> actions -> kept bytes and records per tile
    hipLaunchKernelGGL(fp_class_kernel, dim3((unsigned)p.ntiles), dim3(kFpBlock), 0, st, p);
    hipLaunchKernelGGL(fp_lscan_reduce_kernel, dim3((unsigned)p.ltiles), dim3(kFpBlock), 0, st, p);
    hipLaunchKernelGGL(fp_lscan_top_kernel, dim3(1), dim3(kFpBlock), 0, st, p);
    hipLaunchKernelGGL(fp_lscan_apply_kernel, dim3((unsigned)p.ltiles), dim3(kFpBlock), 0, st, p);
    hipLaunchKernelGGL(fp_keep_kernel, dim3((unsigned)p.ntiles), dim3(kFpBlock), 0, st, p);
    excl_scan_u32(p.tile_keep, p.ntiles, bsum, p.tile_ob, st);
    excl_scan_u32(p.tile_open, p.ntiles, bsum, p.tile_rb, st);
    uint64_t nrec = 0;
    if ((he = hipGetLastError()) || (he = hipMemcpyAsync(&nrec, p.tile_rb + p.ntiles, 8, hipMemcpyDeviceToHost, st)) ||
        (he = hipStreamSynchronize(st)))
        return (int)he;
    *num_seqs = nrec;
    p.idx = get_idx(nrec);
    if (!p.idx) return 0;  // counts only
    p.out = reinterpret_cast<uint8_t *>(out);
    hipLaunchKernelGGL(fp_write_kernel, dim3((unsigned)p.ntiles), dim3(kFpBlock), 0, st, p);
    hipLaunchKernelGGL(fp_finish_kernel, dim3(1), dim3(1), 0, st, p, has_tail);
    uint64_t res[2];
    if ((he = hipGetLastError()) || (he = hipMemcpyAsync(res, p.result, 16, hipMemcpyDeviceToHost, st)) ||
        (he = hipStreamSynchronize(st)))
        return (int)he;
    *num_seqs = res[0];
    *data_bytes = res[1];
    return 0;
}

}  // namespace
}  // namespace kmc

using namespace kmc;

extern "C" int kmc_fasta_parse_device(const char *raw, uint64_t raw_bytes, int dialect, char *data,
                                      uint64_t data_cap, int64_t *indices, uint64_t indices_cap,
                                      uint64_t *num_seqs, uint64_t *data_bytes, hipStream_t stream) {
    if (!num_seqs || !data_bytes || (dialect != 0 && dialect != 1)) return KMC_ERR_INVALID_ARG;
    if ((raw_bytes && (!raw || !data)) || !indices) return KMC_ERR_INVALID_ARG;
    if ((reinterpret_cast<uintptr_t>(raw) & 15u) || (reinterpret_cast<uintptr_t>(data) & 3u))
        return KMC_ERR_ALIGNMENT;
    bool too_small = false;
    auto get_idx = [&](uint64_t nrec) -> int64_t * {
        if (indices_cap < nrec + 1) {
            too_small = true;
            return nullptr;
        }
        return indices;
    };
    const int rc = parse_device(raw, raw_bytes, dialect, data, data_cap, get_idx, num_seqs, data_bytes, stream);
    if (!rc && too_small) return KMC_ERR_CAPACITY;
    return rc;
}

extern "C" int kmc_fasta_load_device(const char *path, int dialect, int64_t max_seqs, char **data,
                                     uint64_t *data_bytes, int64_t **indices, uint64_t *num_seqs,
                                     hipStream_t stream) {
    if (!path || !data || !data_bytes || !indices || !num_seqs || (dialect != 0 && dialect != 1))
        return KMC_ERR_INVALID_ARG;
    *data = nullptr;
    *indices = nullptr;
    *data_bytes = 0;
    *num_seqs = 0;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return KMC_ERR_IO;
    const off_t size = lseek(fd, 0, SEEK_END);
    if (size < 0 || lseek(fd, 0, SEEK_SET) != 0) {
        close(fd);
        return KMC_ERR_IO;
    }
    const uint64_t n = (uint64_t)size;
    // the raw bytes -> device through two pinned staging buffers (the read of
    // chunk i+1 overlaps the copy of chunk i)
    char *raw = nullptr;
    hipError_t he = hipMalloc(&raw, n + 16);
    if (he != hipSuccess) {
        close(fd);
        return KMC_ERR_NOMEM;
    }
    constexpr size_t kChunk = 64u << 20;
    char *pin[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    int rc = 0;
    for (int b = 0; b < 2 && !rc; ++b) {
        if (hipHostMalloc(&pin[b], kChunk, hipHostMallocDefault) != hipSuccess) rc = KMC_ERR_NOMEM;
        else if (hipEventCreateWithFlags(&done[b], hipEventDisableTiming) != hipSuccess) rc = KMC_ERR_NOMEM;
    }
    uint64_t i = 0;
    for (uint64_t off = 0; off < n && !rc; off += kChunk, ++i) {
        const int b = (int)(i & 1);
        if (i >= 2 && (he = hipEventSynchronize(done[b])) != hipSuccess) {
            rc = (int)he;
            break;
        }
        const size_t want = (size_t)std::min<uint64_t>(kChunk, n - off);
        size_t got = 0;
        while (got < want) {
            const ssize_t r = read(fd, pin[b] + got, want - got);
            if (r <= 0) {
                rc = KMC_ERR_IO;
                break;
            }
            got += (size_t)r;
        }
        if (rc) break;
        if ((he = hipMemcpyAsync(raw + off, pin[b], want, hipMemcpyHostToDevice, stream)) ||
            (he = hipEventRecord(done[b], stream)))
            rc = (int)he;
    }
    close(fd);
    if (!rc && (he = hipStreamSynchronize(stream))) rc = (int)he;
    for (int b = 0; b < 2; ++b) {
        if (done[b]) (void)hipEventDestroy(done[b]);
        if (pin[b]) (void)hipHostFree(pin[b]);
    }
    if (!rc && hipMalloc(data, n + 16) != hipSuccess) rc = KMC_ERR_NOMEM;
    bool capped = false;
    auto get_idx = [&](uint64_t nrec) -> int64_t * {
        if (max_seqs > 0 && nrec > (uint64_t)max_seqs) {
            capped = true;  // the reference's MAX_SEQS cut falls mid-record: host rule below
            return nullptr;
        }
        if (hipMalloc(indices, (nrec + 1) * 8) != hipSuccess) return nullptr;
        return *indices;
    };
    if (!rc) {
        rc = parse_device(raw, n, dialect, *data, n + 16, get_idx, num_seqs, data_bytes, stream);
        if (!rc && !capped && !*indices) rc = KMC_ERR_NOMEM;
    }
    (void)hipFree(raw);
    if (!rc && capped) {
        (void)hipFree(*data);
        *data = nullptr;
        kmc_fasta *f = nullptr;
        rc = kmc_fasta_load(path, dialect, max_seqs, &f);
        if (!rc) {
            const uint64_t fb = kmc_fasta_data_bytes(f), fn = kmc_fasta_num_seqs(f);
            if (hipMalloc(data, fb + 16) != hipSuccess || hipMalloc(indices, (fn + 1) * 8) != hipSuccess) {
                rc = KMC_ERR_NOMEM;
            } else {
                he = hipSuccess;
                if (fb) he = hipMemcpy(*data, kmc_fasta_data(f), fb, hipMemcpyHostToDevice);
                if (he == hipSuccess)
                    he = hipMemcpy(*indices, kmc_fasta_indices(f), (fn + 1) * 8, hipMemcpyHostToDevice);
                rc = (int)he;
                *data_bytes = fb;
                *num_seqs = fn;
            }
            kmc_fasta_free(f);
        }
    }
    if (rc) {
        if (*data) (void)hipFree(*data);
        if (*indices) (void)hipFree(*indices);
        *data = nullptr;
        *indices = nullptr;
        *num_seqs = 0;
        *data_bytes = 0;
    }
    return rc;
}
