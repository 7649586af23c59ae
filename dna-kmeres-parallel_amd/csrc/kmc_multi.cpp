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

// Per-device state of kmc_count_multi, created on a device's first call and kept
// until kmc_multi_release(): the stream, two pinned staging buffers, and grow-only
// device buffers (shard + halo, offsets, count matrix, invalid vector, workspace),
// so a second call on the same device set allocates nothing (one-shot CLI use
// paid ~10 hipMalloc/hipHostMalloc per device and call before).  Each device has a
// mutex that a call holds from its first allocation to its copy-back; a call
// takes the mutexes of its devices in ascending device order, so calls on
// overlapping sets ({0,1} and {1,2}) serialise instead of running RCCL
// collectives concurrently on communicators that share a GPU, and cannot
// deadlock; calls on disjoint sets run concurrently.
struct DevState {
    std::mutex mu;
    int dev = 0;
    hipStream_t st = nullptr;
    char *pin[2] = {nullptr, nullptr};  // pinned staging of the host -> device copy
    hipEvent_t done[2] = {nullptr, nullptr};
    char *data = nullptr;
    size_t data_cap = 0;
    int64_t *idx = nullptr;
    size_t idx_cap = 0;
    int32_t *sum = nullptr;
    size_t sum_cap = 0;
    int32_t *inv = nullptr;
    size_t inv_cap = 0;
    void *ws = nullptr;
    size_t ws_cap = 0;
    int32_t *status = nullptr;  // this call's dense status word on the device (kmc_dense_args::status)
    size_t status_cap = 0;
    int rc = KMC_OK;  // result of this call's load + count (written by its worker thread)
};

std::mutex g_mu;                                       // guards the two maps below
std::map<int, std::unique_ptr<DevState>> g_dev;        // device -> state (stable addresses)
std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;  // sorted device set -> comms

DevState *dev_state(int dev) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto &p = g_dev[dev];
    if (!p) {
        p.reset(new DevState);
        p->dev = dev;
    }
    return p.get();
}

void free_state(DevState &d) {  // caller holds d.mu
    (void)hipSetDevice(d.dev);
    if (d.st) (void)hipStreamSynchronize(d.st);
    (void)hipFree(d.data);
    (void)hipFree(d.idx);
    (void)hipFree(d.sum);
    (void)hipFree(d.inv);
    (void)hipFree(d.ws);
    (void)hipFree(d.status);
    for (int j = 0; j < 2; ++j) {
        if (d.pin[j]) (void)hipHostFree(d.pin[j]);
        if (d.done[j]) (void)hipEventDestroy(d.done[j]);
        d.pin[j] = nullptr;
        d.done[j] = nullptr;
    }
    if (d.st) (void)hipStreamDestroy(d.st);
    d.st = nullptr;
    d.data = nullptr;
    d.idx = nullptr;
    d.sum = nullptr;
    d.inv = nullptr;
    d.ws = nullptr;
    d.status = nullptr;
    d.data_cap = d.idx_cap = d.sum_cap = d.inv_cap = d.ws_cap = d.status_cap = 0;
}

// Grow a cached device buffer to at least `bytes` (contents are not kept).
template <class T>
bool reserve(T *&p, size_t &cap, size_t bytes) {
    if (bytes <= cap && p) return true;
    (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(reinterpret_cast<void **>(&p), bytes ? bytes : 16) != hipSuccess) return false;
    cap = bytes;
    return true;
}

// The communicators of a sorted device set, created on first use (ncclCommInitAll
// is a collective setup of its own, far dearer than a 21 MB all-reduce).  The caller
// holds every device mutex of the set, so no other call uses these communicators.
int comms_for(const std::vector<int> &devs, std::vector<ncclComm_t> &out) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        std::vector<ncclComm_t> c(devs.size());
        if (ncclCommInitAll(c.data(), (int)devs.size(), devs.data()) != ncclSuccess) return KMC_ERR_RCCL;
        it = g_comms.emplace(devs, std::move(c)).first;
    }
    out = it->second;
    return KMC_OK;
}

// A set whose collective failed is dropped and its communicators aborted, so the
// next call builds fresh ones instead of reusing a communicator in an error state.
void drop_comms(const std::vector<int> &devs) {
    std::vector<ncclComm_t> c;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_comms.find(devs);
        if (it == g_comms.end()) return;
        c.swap(it->second);
        g_comms.erase(it);
    }
    for (auto &x : c) (void)ncclCommAbort(x);
}

constexpr size_t kStage = (size_t)32 << 20;  // bytes per pinned staging buffer

// Host thread of one device: (re)use its buffers, stream the shard + halo through
// two pinned buffers (the host copy into one overlaps the DMA out of the other),
// count.  One thread per device, so every device loads at the same time.
void load_and_count(DevState &d, const char *data, const int64_t *indices, uint64_t num_seqs, int k,
                    const kmc_shard &sh, bool want_invalid, size_t sum_bytes) {
    auto bad = [&](int code) { d.rc = code; };
    d.rc = KMC_OK;
    if (hipSetDevice(d.dev) != hipSuccess) return bad(KMC_ERR_NO_DEVICE);
    if (!d.st && hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking) != hipSuccess) return bad(KMC_ERR_NO_DEVICE);
    for (int j = 0; j < 2; ++j) {
        if (!d.pin[j] &&
            hipHostMalloc(reinterpret_cast<void **>(&d.pin[j]), kStage, hipHostMallocDefault) != hipSuccess)
            return bad(KMC_ERR_NOMEM);
        if (!d.done[j] && hipEventCreateWithFlags(&d.done[j], hipEventDisableTiming) != hipSuccess)
            return bad(KMC_ERR_NOMEM);
    }
    // the device holds [base, read_hi) with base = read_lo rounded down to 16 so that
    // the library's data pointer (device base - base) stays 16-byte aligned
    const uint64_t base = sh.read_lo & ~(uint64_t)15;
    const uint64_t len = sh.read_hi - base;
    if (!reserve(d.data, d.data_cap, len + 16)) return bad(KMC_ERR_NOMEM);
    if (!reserve(d.idx, d.idx_cap, (num_seqs + 1) * sizeof(int64_t))) return bad(KMC_ERR_NOMEM);
    if (!reserve(d.sum, d.sum_cap, sum_bytes)) return bad(KMC_ERR_NOMEM);
    if (want_invalid && !reserve(d.inv, d.inv_cap, num_seqs * sizeof(int32_t))) return bad(KMC_ERR_NOMEM);
    if (!reserve(d.status, d.status_cap, sizeof(int32_t))) return bad(KMC_ERR_NOMEM);
    kmc_dense_args a{};
    a.data = d.data - base;
    a.indices = d.idx;
    a.num_seqs = num_seqs;
    a.k = k;
    a.sum = d.sum;
    a.sum_ld = num_seqs;
    a.invalid = want_invalid ? d.inv : nullptr;
    a.read_lo = sh.read_lo;
    a.read_hi = sh.read_hi;
    a.win_lo = sh.win_lo;
    a.win_hi = sh.win_hi;
    a.status = d.status;  // this shard's own status: another caller's failure is never reported here
    const size_t wsb = kmc_count_dense_ex_workspace_size(&a, d.dev);
    if (wsb == 0 || !reserve(d.ws, d.ws_cap, wsb)) return bad(KMC_ERR_NOMEM);
    a.workspace = d.ws;
    a.workspace_bytes = d.ws_cap;
    // indices are small: one copy, ordered before the count on the same stream
    if (hipMemcpyAsync(d.idx, indices, (num_seqs + 1) * sizeof(int64_t), hipMemcpyHostToDevice, d.st) !=
            hipSuccess ||
        hipMemsetAsync(d.status, 0, sizeof(int32_t), d.st) != hipSuccess)
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
    // int32 counts of a record of 2^31 or more windows could wrap in the all-reduce:
    // each shard sees fewer than 2^31 of its windows (so no shard's device check
    // fires), but their int32 sum is the whole record's.  The offsets are on the
    // host here, so every record is checked before anything is planned.
    for (uint64_t s = 0; s < num_seqs; ++s) {
        if (indices[s + 1] < indices[s]) return KMC_ERR_INVALID_ARG;
        if (indices[s + 1] - indices[s] - k >= ((int64_t)1 << 31)) return KMC_ERR_RECORD_TOO_LONG;
    }
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess || visible < 1) return KMC_ERR_NO_DEVICE;
    std::vector<int> devs(ndev);
    for (int i = 0; i < ndev; ++i) {
        devs[i] = devices ? devices[i] : i;
        if (devs[i] < 0 || devs[i] >= visible) return KMC_ERR_INVALID_ARG;
    }
    // the set as a sorted list: the communicator cache key and the lock order
    std::sort(devs.begin(), devs.end());
    if (std::adjacent_find(devs.begin(), devs.end()) != devs.end())
        return KMC_ERR_INVALID_ARG;  // one communicator rank per device
    std::vector<kmc_shard> sh(ndev);
    int rc = kmc_plan_shards(indices, num_seqs, k, ndev, 4096, sh.data());
    if (rc) return rc;
    const uint64_t nb = (uint64_t)1 << (2 * k);
    const size_t sum_bytes = nb * num_seqs * sizeof(int32_t);
    int cur = 0;
    (void)hipGetDevice(&cur);

    std::vector<DevState *> b(ndev);
    std::vector<std::unique_lock<std::mutex>> locks;
    locks.reserve(ndev);
    for (int i = 0; i < ndev; ++i) {  // ascending device order: no lock cycles
        b[i] = dev_state(devs[i]);
        locks.emplace_back(b[i]->mu);
    }
    {
        std::vector<std::thread> th;
        th.reserve(ndev);
        for (int i = 0; i < ndev; ++i)
            th.emplace_back(load_and_count, std::ref(*b[i]), data, indices, num_seqs, k, std::cref(sh[i]),
                            invalid != nullptr, sum_bytes);
        for (auto &t : th) t.join();
    }
    for (auto *d : b)
        if (d->rc) {
            // the other devices' copies and counts may still run: let them finish
            // before the call returns (their buffers stay cached for the next call)
            for (auto *o : b)
                if (o->st) {
                    (void)hipSetDevice(o->dev);
                    (void)hipStreamSynchronize(o->st);
                }
            (void)hipSetDevice(cur);
            return d->rc;
        }
    // one all-reduce of the int32 matrix (and the invalid vector) over xGMI
    std::vector<ncclComm_t> comms;
    rc = comms_for(devs, comms);
    if (rc) {
        (void)hipSetDevice(cur);
        return rc;
    }
    ncclResult_t nr = ncclGroupStart();
    for (int i = 0; i < ndev && nr == ncclSuccess; ++i) {
        nr = ncclAllReduce(b[i]->sum, b[i]->sum, nb * num_seqs, ncclInt32, ncclSum, comms[i], b[i]->st);
        if (nr == ncclSuccess && invalid)
            nr = ncclAllReduce(b[i]->inv, b[i]->inv, num_seqs, ncclInt32, ncclSum, comms[i], b[i]->st);
    }
    if (nr == ncclSuccess) nr = ncclGroupEnd();
    else ncclGroupEnd();
    bool comm_ok = nr == ncclSuccess;
    // a HIP failure after the collective (a stream or copy error) is reported as its
    // hipError_t, not as an RCCL failure: no RCCL call failed
    hipError_t he = hipSuccess;
    if (comm_ok) {
        for (auto *d : b) {  // the collective itself finished on every device
            (void)hipSetDevice(d->dev);
            const hipError_t e = hipStreamSynchronize(d->st);
            if (e != hipSuccess && he == hipSuccess) he = e;
        }
        // (a stream that failed to drain may hold a collective in an error state)
        if (he != hipSuccess) comm_ok = false;
    }
    int st = KMC_OK;  // every device has synchronised: the shards' own status words
    if (nr == ncclSuccess && he == hipSuccess)
        for (auto *d : b) {
            int32_t v = 0;
            (void)hipSetDevice(d->dev);
            const hipError_t e = hipMemcpy(&v, d->status, sizeof(v), hipMemcpyDeviceToHost);
            if (e != hipSuccess) {
                if (he == hipSuccess) he = e;
            } else if (v != KMC_OK && st == KMC_OK) {
                st = v;
            }
        }
    if (nr == ncclSuccess && he == hipSuccess) {
        DevState &d = *b[0];
        (void)hipSetDevice(d.dev);
        he = hipMemcpyAsync(sum, d.sum, sum_bytes, hipMemcpyDeviceToHost, d.st);
        if (he == hipSuccess && invalid)
            he = hipMemcpyAsync(invalid, d.inv, num_seqs * sizeof(int32_t), hipMemcpyDeviceToHost, d.st);
        const hipError_t e = hipStreamSynchronize(d.st);
        if (he == hipSuccess) he = e;
    }
    if (!comm_ok) drop_comms(devs);
    (void)hipSetDevice(cur);
    if (nr != ncclSuccess) return KMC_ERR_RCCL;
    if (he != hipSuccess) return (int)he;
    return st;
}

extern "C" int kmc_multi_release(void) {
    // every device mutex, in ascending order, so no call is using a communicator or
    // a buffer while they are destroyed
    std::vector<DevState *> all;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (auto &e : g_dev) all.push_back(e.second.get());  // map order = ascending device
    }
    std::vector<std::unique_lock<std::mutex>> locks;
    for (auto *d : all) locks.emplace_back(d->mu);
    std::map<std::vector<int>, std::vector<ncclComm_t>> comms;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        comms.swap(g_comms);
    }
    for (auto &e : comms)
        for (auto &c : e.second) ncclCommDestroy(c);
    for (auto *d : all) free_state(*d);
    return KMC_OK;
}
