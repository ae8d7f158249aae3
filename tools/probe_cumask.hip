// CU-mask probe (diagnostic): which (XCC, SE, CU) slots run the workgroups of a stream created
// with hipExtStreamCreateWithCUMask, for a given logical-CU bit mask.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void where_kernel(uint32_t* out, int spin) {
    if (threadIdx.x != 0) return;
    // HW_REG_HW_ID (4), bits [0, 32); HW_REG_XCC_ID (20), bits [0, 16)
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11));
    for (volatile int i = 0; i < spin; ++i) {}
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
}

extern "C" int probe_cumask(const uint32_t* mask, int words, int blocks, uint32_t* out_host) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, words, mask) != hipSuccess) return -1;
    uint32_t* d;
    if (hipMalloc(&d, sizeof(uint32_t) * 2 * blocks) != hipSuccess) return -2;
    hipLaunchKernelGGL(where_kernel, dim3(blocks), dim3(64), 0, s, d, 2000);
    if (hipStreamSynchronize(s) != hipSuccess) return -3;
    hipMemcpy(out_host, d, sizeof(uint32_t) * 2 * blocks, hipMemcpyDeviceToHost);
    hipFree(d);
    hipStreamDestroy(s);
    return 0;
}
