// Test-only device clock probes (not product code): the barrier tests' device-side ordering evidence.
//   stamp_clock(dst, stream)        one thread stores wall_clock64() (the device's constant 100 MHz clock,
//                                   the same counter for every process on the GPU) at dst when the stream
//                                   reaches it
//   spin_ticks(ticks, dst, stream)  one thread spins until `ticks` of that clock have passed, then stores
//                                   the clock at dst: a device delay in wall-clock time, unlike
//                                   torch.cuda._sleep's shader-clock cycles
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void stamp_kernel(uint64_t* dst) { *dst = wall_clock64(); }

__global__ void spin_kernel(uint64_t ticks, uint64_t* dst) {
    const uint64_t t0 = wall_clock64();
    uint64_t t = t0;
    while (t - t0 < ticks) {                // every path ends: the clock only moves forward
        __builtin_amdgcn_s_sleep(8);
        t = wall_clock64();
    }
    *dst = t;
}

extern "C" {

int stamp_clock(uint64_t* dst, void* stream) {
    hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(1), 0, static_cast<hipStream_t>(stream), dst);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int spin_ticks(uint64_t ticks, uint64_t* dst, void* stream) {
    if (ticks > 100000000ull) return -1;    // at most 1 s
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(1), 0, static_cast<hipStream_t>(stream), ticks, dst);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int clock_rate_khz(void) {
    int khz = 0;
    return hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0) == hipSuccess ? khz : -1;
}

}
