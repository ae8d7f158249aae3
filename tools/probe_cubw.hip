// Per-CU HBM read rate under a CU mask (diagnostic for DESIGN.md section 6b): is the ~50 GB/s per CU
// seen by every combine kernel below 64 CUs a ceiling of register loads, or of the CU itself?
// Reads 2 KiB units (as the combine's row chunks) of a 1 GiB buffer, in order or in a scattered
// (bijective) order, either into VGPRs (global_load_dwordx4 nt) or into LDS by LDS-DMA
// (global_load_lds_dwordx4), L units in flight per wave, on a persistent grid of the masked CUs.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

template <int L, bool kLDS>
__global__ void __launch_bounds__(256) rd_kernel(const u32x4* src, int64_t nunits, int scattered, uint32_t* sink) {
    __shared__ u32x4 lds[kLDS ? 4 : 1][kLDS ? L : 1][2][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t gw = static_cast<int64_t>(blockIdx.x) * 4 + wave, nw = static_cast<int64_t>(gridDim.x) * 4;
    uint32_t x = 0;
    for (int64_t base = gw * L; base < nunits; base += nw * L) {
        u32x4 v[kLDS ? 1 : L][2];
#pragma unroll
        for (int j = 0; j < L; ++j) {
            const int64_t u = base + j;
            if (u < nunits) {
                const int64_t pu = scattered ? ((u * 0x9E3779B1ll) & (nunits - 1)) : u;
                const u32x4* p = src + pu * 128;
                if constexpr (kLDS) {
                    __builtin_amdgcn_global_load_lds((gbl_void_t*)(p + lane), (lds_void_t*)&lds[wave][j][0][0], 16, 0, 0);
                    __builtin_amdgcn_global_load_lds((gbl_void_t*)(p + 64 + lane), (lds_void_t*)&lds[wave][j][1][0], 16, 0, 0);
                } else {
                    v[j][0] = __builtin_nontemporal_load(p + lane);
                    v[j][1] = __builtin_nontemporal_load(p + 64 + lane);
                }
            }
        }
        if constexpr (kLDS) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            x ^= lds[wave][L - 1][1][lane][0];
        } else {
#pragma unroll
            for (int j = 0; j < L; ++j) x ^= v[j][0][0] ^ v[j][1][3];
        }
    }
    if (x == 0x9e3779b1u) sink[0] = x;
}

namespace {
u32x4* g_buf = nullptr;
uint32_t* g_sink = nullptr;
constexpr int64_t kUnits = int64_t(1) << 19;           // 2^19 units of 2 KiB = 1 GiB

template <int L, bool kLDS>
void launch(int grid, int scattered, hipStream_t s) {
    hipLaunchKernelGGL((rd_kernel<L, kLDS>), dim3(grid), dim3(256), 0, s, g_buf, kUnits, scattered, g_sink);
}
}  // namespace

int g_spread = 0;   // 0: the first `cus` bits; 1: per XCD, CU slots spread evenly over the XCD's CUs

extern "C" void probe_cubw_set_spread(int spread) { g_spread = spread; }

// cus: the first `cus` mask bits (bit b = CU b / 8 of XCD b % 8), 0 = the whole chip unmasked.
// Returns the average microseconds per launch in *us, GB/s in *gbps.
extern "C" int probe_cubw(int cus, int wg_per_cu, int L, int lds, int scattered, int iters, float* us, float* gbps) {
    if (g_buf == nullptr) {
        if (hipMalloc(&g_buf, kUnits * 2048) != hipSuccess) return -1;
        if (hipMemset(g_buf, 1, kUnits * 2048) != hipSuccess) return -1;
        if (hipMalloc(&g_sink, 64) != hipSuccess) return -1;
    }
    int dev = 0, n = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    hipStream_t s = nullptr;
    if (cus > 0 && cus < n) {
        uint32_t mask[64] = {};
        if (g_spread) {
            const int per_xcd = n / 8, k = (cus + 7) / 8;         // CU slots per XCD in the mask, wanted
            for (int x = 0; x < 8; ++x)
                for (int j = 0; j < k; ++j) {
                    const int b = (j * per_xcd / k) * 8 + x;
                    mask[b / 32] |= 1u << (b % 32);
                }
        } else {
            for (int b = 0; b < cus; ++b) mask[b / 32] |= 1u << (b % 32);
        }
        if (hipExtStreamCreateWithCUMask(&s, (n + 31) / 32, mask) != hipSuccess) return -2;
    } else {
        cus = n;
        if (hipStreamCreate(&s) != hipSuccess) return -2;
    }
    const int grid = cus * wg_per_cu;
    auto go = [&]() {
        if (lds) {
            if (L == 4) launch<4, true>(grid, scattered, s);
            else if (L == 8) launch<8, true>(grid, scattered, s);
            else launch<2, true>(grid, scattered, s);
        } else {
            if (L == 4) launch<4, false>(grid, scattered, s);
            else if (L == 8) launch<8, false>(grid, scattered, s);
            else if (L == 16) launch<16, false>(grid, scattered, s);
            else launch<2, false>(grid, scattered, s);
        }
    };
    for (int i = 0; i < 2; ++i) go();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, s);
    for (int i = 0; i < iters; ++i) go();
    hipEventRecord(e1, s);
    if (hipEventSynchronize(e1) != hipSuccess) return -3;
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    *us = ms * 1e3f / iters;
    *gbps = static_cast<float>(kUnits * 2048 / (*us * 1e3));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipStreamDestroy(s);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}
