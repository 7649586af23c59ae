// kmc_internal.h — declarations shared by the translation units of libkmc.so.
#pragma once
#include <cstdint>

struct kmc_dense_args;
typedef struct ihipStream_t *hipStream_t;

// Test hooks (kmc_diag_*) exist only in the diagnostic library lib/libkmc_diag.so
// (built with -DKMC_DIAG_HOOKS for the tests that force an algorithm choice);
// libkmc.so exports exactly the entry points of kmc.h.
#define KMC_DIAG_API __attribute__((visibility("default")))

namespace kmc {
typedef struct ihipEvent_t *hipEvent_t;
// Grid extents of the per-record / per-list helper kernels, which loop over the
// rest (a launch must keep gridDim * blockDim below 2^32 per dimension).
constexpr int64_t kMaxGridX = 1 << 20;
constexpr int64_t kMaxGridY = 32768;
// kmc_trace_set_events: recorded around the histogram kernel (k <= 8) or the
// whole radix pipeline (k > 8) of the next dense count calls on this thread.
extern thread_local hipEvent_t t_trace_before, t_trace_after;

// 9 <= k <= KMC_DENSE_MAX_K: radix-partitioned dense counting (kmc_radix.hip).
// a->data is 16-byte aligned; ibias is added to every record offset (the caller's
// misalignment, already added to a's ranges).  size_only: report the workspace size
// in *size_out instead of launching.
int radix_dense(const ::kmc_dense_args *a, int64_t ibias, hipStream_t st, bool size_only, size_t *size_out);

// splitmix64 output n (0-based) of the stream seeded with `seed` (Steele et al.):
// z = seed + (n+1)*golden; two xor-shift-multiply rounds; final xor-shift.
__host__ __device__ inline uint64_t splitmix64_at(uint64_t seed, uint64_t n) {
    uint64_t z = seed + (n + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
}  // namespace kmc
