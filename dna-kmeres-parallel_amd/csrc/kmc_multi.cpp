// kmc_multi.cpp — shard planning and the single-process multi-GPU driver.
//
// The reference is one process on one GPU (no NCCL/MPI).  Its
// records are independent, so the path partitions: every device counts the
// windows that start in its byte range (reading a k-1 byte halo past it), and
// one RCCL all-reduce of the int32 count matrix is the only exchange.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "kmc.h"

extern "C" int kmc_plan_shards(const int64_t *indices, uint64_t num_seqs, int k, int nshards, uint64_t align,
                               kmc_shard *out) {
    if (!indices || !out || nshards < 1 || k < 1) return KMC_ERR_INVALID_ARG;
    if (align == 0) align = 4096;
    const uint64_t lo = num_seqs ? (uint64_t)indices[0] : 0;
    const uint64_t hi = num_seqs ? (uint64_t)indices[num_seqs] : 0;
    if (hi < lo) return KMC_ERR_INVALID_ARG;
    std::vector<uint64_t> cut(nshards + 1);
    cut[0] = lo;
    cut[nshards] = hi;
    for (int i = 1; i < nshards; ++i) {
        const uint64_t ideal = lo + (uint64_t)((unsigned __int128)(hi - lo) * (uint64_t)i / (uint64_t)nshards);
        uint64_t c = (ideal / align) * align;  // inner cuts on `align` boundaries
        c = std::max(c, cut[i - 1]);
        c = std::min(c, hi);
        cut[i] = c;
    }
    for (int i = 0; i < nshards; ++i) {
        out[i].win_lo = cut[i];
        out[i].win_hi = cut[i + 1];
        out[i].read_lo = cut[i];
        out[i].read_hi = std::min<uint64_t>(cut[i + 1] + (uint64_t)(k - 1), hi);
        if (out[i].read_hi < out[i].read_lo) out[i].read_hi = out[i].read_lo;
    }
    return KMC_OK;
}

namespace {

struct DevBufs {
    int dev = 0;
    hipStream_t st = nullptr;
    char *data = nullptr;
    int64_t *idx = nullptr;
    int32_t *sum = nullptr;
    int32_t *inv = nullptr;
    void *ws = nullptr;
};

void release(std::vector<DevBufs> &b) {
    for (auto &d : b) {
        (void)hipSetDevice(d.dev);
        if (d.st) (void)hipStreamSynchronize(d.st);
        (void)hipFree(d.data);
        (void)hipFree(d.idx);
        (void)hipFree(d.sum);
        (void)hipFree(d.inv);
        (void)hipFree(d.ws);
        if (d.st) (void)hipStreamDestroy(d.st);
    }
}

}  // namespace

extern "C" int kmc_count_multi(const char *data, const int64_t *indices, uint64_t num_seqs, uint64_t data_bytes,
                               int k, int ndev, const int *devices, int32_t *sum, int32_t *invalid) {
    if (num_seqs == 0) return KMC_OK;
    if (!data || !indices || !sum || ndev < 1) return KMC_ERR_INVALID_ARG;
    if (k < 1 || k > KMC_DENSE_MAX_K) return KMC_ERR_UNSUPPORTED_K;
    if ((uint64_t)indices[num_seqs] > data_bytes) return KMC_ERR_INVALID_ARG;
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess || visible < 1) return KMC_ERR_NO_DEVICE;
    std::vector<int> devs(ndev);
    for (int i = 0; i < ndev; ++i) {
        devs[i] = devices ? devices[i] : i;
        if (devs[i] < 0 || devs[i] >= visible) return KMC_ERR_INVALID_ARG;
    }
    std::vector<kmc_shard> sh(ndev);
    int rc = kmc_plan_shards(indices, num_seqs, k, ndev, 4096, sh.data());
    if (rc) return rc;
    const uint64_t nb = (uint64_t)1 << (2 * k);
    const size_t sum_bytes = nb * num_seqs * sizeof(int32_t);
    int cur = 0;
    (void)hipGetDevice(&cur);

    std::vector<DevBufs> b(ndev);
    auto fail = [&](int code) {
        release(b);
        (void)hipSetDevice(cur);
        return code;
    };
    for (int i = 0; i < ndev; ++i) {
        DevBufs &d = b[i];
        d.dev = devs[i];
        if (hipSetDevice(d.dev) != hipSuccess) return fail(KMC_ERR_NO_DEVICE);
        if (hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking) != hipSuccess) return fail(KMC_ERR_NO_DEVICE);
        // the device holds [base, read_hi) with base = read_lo rounded down to 16 so that
        // the library's data pointer (device base - base) stays 16-byte aligned
        const uint64_t base = sh[i].read_lo & ~(uint64_t)15;
        const uint64_t len = sh[i].read_hi - base;
        if (hipMalloc(&d.data, len + 16) != hipSuccess) return fail(KMC_ERR_NOMEM);
        if (hipMalloc(&d.idx, (num_seqs + 1) * sizeof(int64_t)) != hipSuccess) return fail(KMC_ERR_NOMEM);
        if (hipMalloc(&d.sum, sum_bytes) != hipSuccess) return fail(KMC_ERR_NOMEM);
        if (invalid && hipMalloc(&d.inv, num_seqs * sizeof(int32_t)) != hipSuccess) return fail(KMC_ERR_NOMEM);
        kmc_dense_args a{};
        a.data = d.data - base;
        a.indices = d.idx;
        a.num_seqs = num_seqs;
        a.k = k;
        a.sum = d.sum;
        a.sum_ld = num_seqs;
        a.invalid = d.inv;
        a.read_lo = sh[i].read_lo;
        a.read_hi = sh[i].read_hi;
        a.win_lo = sh[i].win_lo;
        a.win_hi = sh[i].win_hi;
        const size_t wsb = kmc_count_dense_ex_workspace_size(&a, d.dev);
        if (wsb == 0 || hipMalloc(&d.ws, wsb) != hipSuccess) return fail(KMC_ERR_NOMEM);
        a.workspace = d.ws;
        a.workspace_bytes = wsb;
        if (hipMemcpyAsync(d.data, data + base, len, hipMemcpyHostToDevice, d.st) != hipSuccess ||
            hipMemcpyAsync(d.idx, indices, (num_seqs + 1) * sizeof(int64_t), hipMemcpyHostToDevice, d.st) !=
                hipSuccess)
            return fail(KMC_ERR_NOMEM);
        rc = kmc_count_dense_ex(&a, d.st);
        if (rc) return fail(rc);
    }
    // one all-reduce of the int32 matrix (and the invalid vector) over xGMI
    std::vector<ncclComm_t> comms(ndev);
    if (ncclCommInitAll(comms.data(), ndev, devs.data()) != ncclSuccess) return fail(KMC_ERR_RCCL);
    ncclResult_t nr = ncclGroupStart();
    for (int i = 0; i < ndev && nr == ncclSuccess; ++i) {
        nr = ncclAllReduce(b[i].sum, b[i].sum, nb * num_seqs, ncclInt32, ncclSum, comms[i], b[i].st);
        if (nr == ncclSuccess && invalid)
            nr = ncclAllReduce(b[i].inv, b[i].inv, num_seqs, ncclInt32, ncclSum, comms[i], b[i].st);
    }
    if (nr == ncclSuccess) nr = ncclGroupEnd();
    else ncclGroupEnd();
    if (nr == ncclSuccess) {
        (void)hipSetDevice(b[0].dev);
        if (hipMemcpyAsync(sum, b[0].sum, sum_bytes, hipMemcpyDeviceToHost, b[0].st) != hipSuccess) nr = ncclSystemError;
        if (invalid && hipMemcpyAsync(invalid, b[0].inv, num_seqs * sizeof(int32_t), hipMemcpyDeviceToHost,
                                      b[0].st) != hipSuccess)
            nr = ncclSystemError;
        if (hipStreamSynchronize(b[0].st) != hipSuccess) nr = ncclSystemError;
    }
    for (auto &c : comms) ncclCommDestroy(c);
    release(b);
    (void)hipSetDevice(cur);
    return nr == ncclSuccess ? KMC_OK : KMC_ERR_RCCL;
}
