// xcd_probe.hip -- diagnostic kernels for tools/xgmi_xcd_probe.py (not part of the product).
//
// Fill / check a region of memory from the workgroups of chosen XCDs only (HW_REG_XCC_ID), so that a
// hand-off can be forced across XCDs: each kernel runs a grid-stride loop over the region in which
// only the workgroups whose XCD is in `xcd_mask` take part (the rest exit).  Loads come in three
// flavours: plain, non-temporal (nt) and system-scope (sc0 sc1).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11)) & 0xF; }

__global__ void __launch_bounds__(256) fill_kernel(int32_t* p, int64_t n, int32_t v, uint32_t xcd_mask, int32_t* wgs) {
    __shared__ int s_ok;
    __shared__ int64_t s_chunk;
    if (threadIdx.x == 0) s_ok = (xcd_mask >> xcc_id()) & 1;
    __syncthreads();
    if (!s_ok) return;
    constexpr int64_t kChunk = 256 * 16;
    for (;;) {                                   // work queue of chunks over the participating workgroups
        if (threadIdx.x == 0) s_chunk = atomicAdd(wgs, 1);
        __syncthreads();
        const int64_t lo = s_chunk * kChunk;
        __syncthreads();
        if (lo >= n) return;
        const int64_t hi = min(n, lo + kChunk);
        for (int64_t i = lo + threadIdx.x; i < hi; i += 256) p[i] = v;
    }
}

template <int kFlavour>
__global__ void __launch_bounds__(256) check_kernel(const int32_t* p, int64_t n, int32_t expect, uint32_t xcd_mask,
                                                    int32_t* wgs, unsigned long long* mismatches) {
    __shared__ int s_ok;
    if (threadIdx.x == 0) s_ok = (xcd_mask >> xcc_id()) & 1;
    __syncthreads();
    if (!s_ok) return;
    __shared__ int64_t s_chunk;
    constexpr int64_t kChunk = 256 * 16;
    unsigned long long bad = 0;
    for (;;) {
        if (threadIdx.x == 0) s_chunk = atomicAdd(wgs, 1);
        __syncthreads();
        const int64_t lo = s_chunk * kChunk;
        __syncthreads();
        if (lo >= n) break;
        const int64_t hi = min(n, lo + kChunk);
        for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
            int32_t v;
            if constexpr (kFlavour == 0) v = p[i];
            else if constexpr (kFlavour == 1) v = __builtin_nontemporal_load(p + i);
            else v = __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            bad += v != expect;
        }
    }
    if (bad) atomicAdd(mismatches, bad);
}

}  // namespace

extern "C" {

// xcd_mask: bit x = XCD x takes part.  wgs: int32 work-queue counter (zeroed by the caller).
int xcd_fill(int32_t* p, int64_t n, int32_t v, uint32_t xcd_mask, int32_t* wgs, void* stream) {
    hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), p, n, v, xcd_mask,
                       wgs);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int xcd_check(const int32_t* p, int64_t n, int32_t expect, uint32_t xcd_mask, int flavour, int32_t* wgs,
              unsigned long long* mismatches, void* stream) {
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (flavour == 0) hipLaunchKernelGGL(check_kernel<0>, dim3(2048), dim3(256), 0, s, p, n, expect, xcd_mask, wgs, mismatches);
    else if (flavour == 1) hipLaunchKernelGGL(check_kernel<1>, dim3(2048), dim3(256), 0, s, p, n, expect, xcd_mask, wgs, mismatches);
    else hipLaunchKernelGGL(check_kernel<2>, dim3(2048), dim3(256), 0, s, p, n, expect, xcd_mask, wgs, mismatches);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
