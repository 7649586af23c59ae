// kmc_common.cpp — error strings and version of libkmc.so.
#include <hip/hip_runtime_api.h>

#include "kmc.h"

extern "C" const char *kmc_error_string(int code) {
    switch (code) {
        case KMC_OK: return "success";
        case KMC_ERR_INVALID_ARG: return "invalid argument";
        case KMC_ERR_UNSUPPORTED_K: return "k outside the supported range of this entry point";
        case KMC_ERR_ALIGNMENT: return "pointer not aligned as required (data: 16 bytes, workspace: 256 bytes)";
        case KMC_ERR_WORKSPACE: return "workspace smaller than the required size";
        case KMC_ERR_IO: return "file cannot be opened or read";
        case KMC_ERR_NOMEM: return "allocation failed";
        case KMC_ERR_RCCL: return "RCCL call failed";
        case KMC_ERR_NO_DEVICE: return "no HIP device visible";
        case KMC_ERR_CAPACITY: return "output capacity smaller than the result";
        case KMC_ERR_RECORD_TOO_LONG: return "a record has 2^31 or more windows in one call: int32 counts could wrap";
        case KMC_ERR_INTERNAL: return "a device-side bound check fired (library defect): outputs not valid";
        default: return hipGetErrorString(static_cast<hipError_t>(code));
    }
}

// 0.2.0: kmc_dense_args gained its trailing `status` field (round 5) and
// KMC_ERR_INTERNAL was added (round 6); a caller built against the 0.1 header
// passes the shorter struct and must check kmc_version() >= 200 first.
extern "C" int kmc_version(void) { return 200; }
