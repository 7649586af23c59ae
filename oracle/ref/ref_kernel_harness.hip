// ref_kernel_harness.hip — TEST INFRASTRUCTURE ONLY.
//
// Compiles the reference's OWN device code, /root/reference/kernels.h (included
// as-is, with the reference's compile-time K, default 3), for gfx950 with hipcc,
// and exposes its step-1 launch exactly as main.cu issues it:
//   c_perms filled from permutation() with one MemcpyToSymbol per pattern (main.cu:151-158)
//   sumKmereCoincidencesGlobalMemory<<<BLOCKS_STEP_1=54018, PERMS_KMERES>>>  (main.cu:290)
// and its step-2 launch minKmeres2<<<1000, 64>>> (main.cu:327).
// The GPU parity tests run it on the MI355X box next to the HIP product kernels.
#include <hip/hip_runtime.h>
#include <cstring>
#include <cmath>
#include <cstdlib>

#include "utils.h"    // /root/reference/utils.h
#include "kernels.h"  // /root/reference/kernels.h

extern "C" {

int ref_kernel_k() { return K; }

int ref_kernel_upload_patterns() {
    const int n = PERMS_KMERES;
    char **perms = (char **)malloc(n * sizeof(char *));
    for (int i = 0; i < n; ++i) perms[i] = (char *)calloc(K + 1, 1);
    permutation("ACGT", K, perms);
    int err = 0;
    for (int i = 0; i < n && !err; ++i)
        err = (int)hipMemcpyToSymbol(HIP_SYMBOL(c_perms), perms[i], K + 1, i * (K + 1));
    for (int i = 0; i < n; ++i) free(perms[i]);
    free(perms);
    return err;
}

// data/indices/sum are device pointers.  Synchronous like main.cu:290-294.
int ref_kernel_launch(char *data, int *indices, unsigned num_seqs, int *sum) {
    sumKmereCoincidencesGlobalMemory<<<54018, PERMS_KMERES>>>(data, indices, num_seqs, sum);
    int err = (int)hipDeviceSynchronize();
    if (!err) err = (int)hipGetLastError();
    return err;
}

// One step-2 launch as main.cu:327 issues it: minKmeres2<<<blocks=1000, THREADS=64>>>
// (main.cu:24, 41), then the sync + error check of main.cu:328-333.
int ref_min_kmeres2_launch(int *sums, float *mins, int num_seqs, int current_seq, int *indexes) {
    minKmeres2<<<1000, 64>>>(sums, mins, num_seqs, current_seq, indexes);
    int err = (int)hipDeviceSynchronize();
    if (!err) err = (int)hipGetLastError();
    return err;
}

}  // extern "C"
