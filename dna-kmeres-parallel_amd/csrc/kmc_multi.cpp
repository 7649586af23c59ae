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
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
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

// Communicators of one device set, created on first use (ncclCommInitAll is a
// collective setup of its own, far dearer than a 21 MB all-reduce) and kept until
// kmc_multi_release().  RCCL communicators are not thread-safe, so every entry
// carries its own mutex, held by a kmc_count_multi call from ncclGroupStart until
// its copy-back has synchronised: calls on the same device set serialise their
// collectives, calls on disjoint sets run concurrently.  An entry whose collective
// failed is dropped (and its communicators aborted), so the next call on that set
// builds fresh ones instead of reusing a communicator in an error state.
struct CommSet {
    std::mutex mu;
    std::vector<ncclComm_t> comms;
};
std::mutex g_comm_mu;
std::map<std::vector<int>, std::shared_ptr<CommSet>> g_comms;

int comms_for(const std::vector<int> &devs, std::shared_ptr<CommSet> &out) {
    std::lock_guard<std::mutex> lk(g_comm_mu);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        auto cs = std::make_shared<CommSet>();
        cs->comms.resize(devs.size());
        if (ncclCommInitAll(cs->comms.data(), (int)devs.size(), devs.data()) != ncclSuccess) return KMC_ERR_RCCL;
        it = g_comms.emplace(devs, std::move(cs)).first;
    }
    out = it->second;
    return KMC_OK;
}

// Remove a failed set from the cache (if it is still the cached one) and abort its
// communicators.  The caller holds cs->mu.
void drop_comms(const std::vector<int> &devs, const std::shared_ptr<CommSet> &cs) {
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        auto it = g_comms.find(devs);
        if (it != g_comms.end() && it->second == cs) g_comms.erase(it);
    }
    for (auto &c : cs->comms) (void)ncclCommAbort(c);
    cs->comms.clear();
}

struct DevBufs {
    int dev = 0;
    hipStream_t st = nullptr;
    char *data = nullptr;
    int64_t *idx = nullptr;
    int32_t *sum = nullptr;
    int32_t *inv = nullptr;
    void *ws = nullptr;
    char *pin[2] = {nullptr, nullptr};  // pinned staging of the host -> device copy
    hipEvent_t done[2] = {nullptr, nullptr};
    int rc = KMC_OK;
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
        for (int j = 0; j < 2; ++j) {
            if (d.pin[j]) (void)hipHostFree(d.pin[j]);
            if (d.done[j]) (void)hipEventDestroy(d.done[j]);
        }
        if (d.st) (void)hipStreamDestroy(d.st);
    }
}

constexpr size_t kStage = (size_t)32 << 20;  // bytes per pinned staging buffer

// Host thread of one device: allocate, stream the shard + halo through two pinned
// buffers (the host copy into one overlaps the DMA out of the other), count.  One
// thread per device, so every device loads at the same time.
void load_and_count(DevBufs &d, const char *data, const int64_t *indices, uint64_t num_seqs, int k,
                    const kmc_shard &sh, bool want_invalid, size_t sum_bytes) {
    auto bad = [&](int code) { d.rc = code; };
    if (hipSetDevice(d.dev) != hipSuccess) return bad(KMC_ERR_NO_DEVICE);
    if (hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking) != hipSuccess) return bad(KMC_ERR_NO_DEVICE);
    // the device holds [base, read_hi) with base = read_lo rounded down to 16 so that
    // the library's data pointer (device base - base) stays 16-byte aligned
    const uint64_t base = sh.read_lo & ~(uint64_t)15;
    const uint64_t len = sh.read_hi - base;
    if (hipMalloc(&d.data, len + 16) != hipSuccess) return bad(KMC_ERR_NOMEM);
    if (hipMalloc(&d.idx, (num_seqs + 1) * sizeof(int64_t)) != hipSuccess) return bad(KMC_ERR_NOMEM);
    if (hipMalloc(&d.sum, sum_bytes) != hipSuccess) return bad(KMC_ERR_NOMEM);
    if (want_invalid && hipMalloc(&d.inv, num_seqs * sizeof(int32_t)) != hipSuccess) return bad(KMC_ERR_NOMEM);
    for (int j = 0; j < 2; ++j) {
        if (hipHostMalloc(reinterpret_cast<void **>(&d.pin[j]), kStage, hipHostMallocDefault) != hipSuccess)
            return bad(KMC_ERR_NOMEM);
        if (hipEventCreateWithFlags(&d.done[j], hipEventDisableTiming) != hipSuccess) return bad(KMC_ERR_NOMEM);
    }
    kmc_dense_args a{};
    a.data = d.data - base;
    a.indices = d.idx;
    a.num_seqs = num_seqs;
    a.k = k;
    a.sum = d.sum;
    a.sum_ld = num_seqs;
    a.invalid = d.inv;
    a.read_lo = sh.read_lo;
    a.read_hi = sh.read_hi;
    a.win_lo = sh.win_lo;
    a.win_hi = sh.win_hi;
    const size_t wsb = kmc_count_dense_ex_workspace_size(&a, d.dev);
    if (wsb == 0 || hipMalloc(&d.ws, wsb) != hipSuccess) return bad(KMC_ERR_NOMEM);
    a.workspace = d.ws;
    a.workspace_bytes = wsb;
    // indices are small: one synchronous copy
    if (hipMemcpy(d.idx, indices, (num_seqs + 1) * sizeof(int64_t), hipMemcpyHostToDevice) != hipSuccess)
        return bad(KMC_ERR_NOMEM);
    uint64_t done = 0;
    for (int j = 0; done < len; j ^= 1) {
        const size_t c = (size_t)std::min<uint64_t>(kStage, len - done);
        if (hipEventSynchronize(d.done[j]) != hipSuccess) return bad(KMC_ERR_NOMEM);  // buffer j free again
        std::memcpy(d.pin[j], data + base + done, c);
        if (hipMemcpyAsync(d.data + done, d.pin[j], c, hipMemcpyHostToDevice, d.st) != hipSuccess ||
            hipEventRecord(d.done[j], d.st) != hipSuccess)
            return bad(KMC_ERR_NOMEM);
        done += c;
    }
    d.rc = kmc_count_dense_ex(&a, d.st);
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
        for (int j = 0; j < i; ++j)
            if (devs[j] == devs[i]) return KMC_ERR_INVALID_ARG;  // one communicator rank per device
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
    {
        std::vector<std::thread> th;
        th.reserve(ndev);
        for (int i = 0; i < ndev; ++i) {
            b[i].dev = devs[i];
            th.emplace_back(load_and_count, std::ref(b[i]), data, indices, num_seqs, k, std::cref(sh[i]),
                            invalid != nullptr, sum_bytes);
        }
        for (auto &t : th) t.join();
    }
    for (auto &d : b)
        if (d.rc) return fail(d.rc);
    // one all-reduce of the int32 matrix (and the invalid vector) over xGMI
    std::shared_ptr<CommSet> cs;
    rc = comms_for(devs, cs);
    if (rc) return fail(rc);
    std::unique_lock<std::mutex> use(cs->mu);  // this set's communicators, until the copy-back is done
    if (cs->comms.empty()) {                   // dropped by a failed call while we waited: build anew
        use.unlock();
        cs.reset();
        rc = comms_for(devs, cs);
        if (rc) return fail(rc);
        use = std::unique_lock<std::mutex>(cs->mu);
    }
    ncclResult_t nr = ncclGroupStart();
    for (int i = 0; i < ndev && nr == ncclSuccess; ++i) {
        nr = ncclAllReduce(b[i].sum, b[i].sum, nb * num_seqs, ncclInt32, ncclSum, cs->comms[i], b[i].st);
        if (nr == ncclSuccess && invalid)
            nr = ncclAllReduce(b[i].inv, b[i].inv, num_seqs, ncclInt32, ncclSum, cs->comms[i], b[i].st);
    }
    if (nr == ncclSuccess) nr = ncclGroupEnd();
    else ncclGroupEnd();
    bool comm_ok = nr == ncclSuccess;
    if (comm_ok) {
        for (auto &d : b) {  // the collective itself finished on every device
            (void)hipSetDevice(d.dev);
            if (hipStreamSynchronize(d.st) != hipSuccess) comm_ok = false;
        }
        if (!comm_ok) nr = ncclSystemError;
    }
    if (nr == ncclSuccess) {
        (void)hipSetDevice(b[0].dev);
        if (hipMemcpyAsync(sum, b[0].sum, sum_bytes, hipMemcpyDeviceToHost, b[0].st) != hipSuccess) nr = ncclSystemError;
        if (invalid && hipMemcpyAsync(invalid, b[0].inv, num_seqs * sizeof(int32_t), hipMemcpyDeviceToHost,
                                      b[0].st) != hipSuccess)
            nr = ncclSystemError;
        if (hipStreamSynchronize(b[0].st) != hipSuccess) nr = ncclSystemError;
    }
    if (!comm_ok) drop_comms(devs, cs);
    use.unlock();
    release(b);
    (void)hipSetDevice(cur);
    return nr == ncclSuccess ? KMC_OK : KMC_ERR_RCCL;
}

extern "C" int kmc_multi_release(void) {
    std::map<std::vector<int>, std::shared_ptr<CommSet>> all;
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        all.swap(g_comms);
    }
    for (auto &e : all) {
        std::lock_guard<std::mutex> use(e.second->mu);  // wait for a call still using the set
        for (auto &c : e.second->comms) ncclCommDestroy(c);
        e.second->comms.clear();
    }
    return KMC_OK;
}
