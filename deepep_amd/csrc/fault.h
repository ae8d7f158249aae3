// fault.h -- the device-side error record of the window paths (include/deepep_amd.h,
// DEEPEP_ERROR_RECORD_INTS): a flag word plus the first fault, written by whichever lane gets there
// first, so the host can say which unit / row / address went wrong instead of "something failed".
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/deepep_amd.h"

namespace deepep {

// Set `bit` in rec[0]; the first caller of any kind also fills rec[1..6] (vector stores).
__device__ __forceinline__ void record_fault(int32_t* rec, int bit, int kind, int64_t unit, int64_t rank,
                                             uint64_t addr, int64_t extra) {
    if (rec == nullptr) return;
    atomicOr(rec, bit);
    if (atomicCAS(rec + 1, 0, kind) == 0) {
        rec[2] = static_cast<int32_t>(unit);
        rec[3] = static_cast<int32_t>(rank);
        rec[4] = static_cast<int32_t>(addr & 0xffffffffull);
        rec[5] = static_cast<int32_t>(addr >> 32);
        rec[6] = static_cast<int32_t>(extra);
    }
}

}  // namespace deepep
