// Load cache-policy probe (diagnostic): the fused combine's gather (per (token, 2 KiB chunk) item:
// the token's 8 rows, fp32 sum, one bf16 row stored with buffer_store sc1, 8-wave workgroups)
// with the row loads issued as raw buffer loads carrying each cache-policy combination.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

template <int kLoadAux, int kStoreAux, bool kGlobalNT>
__global__ void __launch_bounds__(512) gather_ld(const uint16_t* src, const int32_t* table, uint16_t* out, int T,
                                                 int hidden) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nvec = hidden / 8, nch = nvec / 128;
    const int64_t it = (int64_t)blockIdx.x * 8 + wave;
    if (it >= (int64_t)T * nch) return;
    const int64_t t = it / nch;
    const int c = (int)(it - t * nch);
    int32_t my = lane < 8 ? table[t * 8 + lane] : -1;
    float acc[2][8] = {};
    u32x4 v[8][2];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int32_t s = __builtin_amdgcn_readlane(my, j);
        const int off = (c * 128 + lane) * 16;
        if constexpr (kGlobalNT) {
            const u32x4* row = reinterpret_cast<const u32x4*>(src + (int64_t)s * hidden);
            v[j][0] = __builtin_nontemporal_load(row + c * 128 + lane);
            v[j][1] = __builtin_nontemporal_load(row + c * 128 + lane + 64);
        } else {
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(src + (int64_t)s * hidden), 0,
                                                              hidden * 2, 0x00020000);
            v[j][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kLoadAux);
            v[j][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 1024, 0, kLoadAux);
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                acc[q][2 * d] += __uint_as_float(v[j][q][d] << 16);
                acc[q][2 * d + 1] += __uint_as_float(v[j][q][d] & 0xffff0000u);
            }
    const auto orow = __builtin_amdgcn_make_buffer_rsrc(out + t * hidden, 0, hidden * 2, 0x00020000);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        u32x4 r;
#pragma unroll
        for (int d = 0; d < 4; ++d) r[d] = pack(acc[q][2 * d], acc[q][2 * d + 1]);
        __builtin_amdgcn_raw_buffer_store_b128(r, orow, (c * 128 + lane + 64 * q) * 16, 0, kStoreAux);
    }
}

extern "C" int probe_ld(int variant, const void* src, const int32_t* table, void* out, int T, int hidden,
                        hipStream_t s) {
    const int64_t items = (int64_t)T * (hidden / 8 / 128);
    const dim3 grid((unsigned)((items + 7) / 8)), block(512);
    const uint16_t* x = (const uint16_t*)src;
    uint16_t* o = (uint16_t*)out;
#define V(N, L, S, G) case N: hipLaunchKernelGGL((gather_ld<L, S, G>), grid, block, 0, s, x, table, o, T, hidden); break;
    switch (variant) {
        V(0, 0, 16, true)      // global_load nt (the kernel's loads)
        V(1, 0, 16, false)     // buffer_load plain
        V(2, 2, 16, false)     // nt
        V(3, 1, 16, false)     // sc0
        V(4, 16, 16, false)    // sc1
        V(5, 17, 16, false)    // sc0 sc1
        V(6, 18, 16, false)    // sc1 nt
        V(7, 3, 16, false)     // sc0 nt
        V(8, 19, 16, false)    // sc0 sc1 nt
        V(9, 2, 0, false)      // nt loads, plain stores
        V(10, 2, 17, false)    // nt loads, sc0 sc1 stores
        V(11, 2, 18, false)    // nt loads, sc1 nt stores
        default: return -1;
    }
#undef V
    return (int)hipGetLastError();
}
