// probe_tok.hip -- diagnostic: one wave streams whole tokens (all column chunks of its tokens, the
// loads of the next chunk in flight while the current one is summed and stored), against the
// product kernel's one-wave-per-(token, chunk) items.  Plain sum, K = 8 valid rows per token.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

namespace {

__device__ __forceinline__ float lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

constexpr int K = 8;

template <int kVPT, int kAux>
__global__ void __launch_bounds__(256) token_stream(const uint16_t* __restrict__ src, const int32_t* __restrict__ table,
                                                    uint16_t* __restrict__ out, int T, int hidden) {
    const int lane = threadIdx.x & 63;
    const int nvec = hidden / 8;
    const int nch = nvec / (64 * kVPT);                      // column chunks per token (exact here)
    const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * 4;
    const int64_t ntok = g < T ? (T - 1 - g) / nw + 1 : 0;  // tokens of this wave
    const int64_t nitems = ntok * nch;
    if (nitems == 0) return;

    auto issue = [&](int64_t j, u32x4 (&v)[K][kVPT]) {
        const int64_t t = g + (j / nch) * nw;
        const int c = (int)(j % nch);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            int32_t s = __builtin_amdgcn_readfirstlane(table[t * K + k]);
            s = s < 0 ? 0 : s;                                   // probe: no masked slots expected
            const u32x4* row = reinterpret_cast<const u32x4*>(src + (int64_t)s * hidden) + c * 64 * kVPT + lane;
#pragma unroll
            for (int q = 0; q < kVPT; ++q) v[k][q] = __builtin_nontemporal_load(row + 64 * q);
        }
    };
    auto finish = [&](int64_t j, u32x4 (&v)[K][kVPT]) {
        const int64_t t = g + (j / nch) * nw;
        const int c = (int)(j % nch);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + t * hidden, 0, hidden * 2, 0x00020000);
#pragma unroll
        for (int q = 0; q < kVPT; ++q) {
            float a[8] = {};
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    a[2 * d] += lo(v[k][q][d]);
                    a[2 * d + 1] += hi(v[k][q][d]);
                }
            u32x4 r;
#pragma unroll
            for (int d = 0; d < 4; ++d) r[d] = pack(a[2 * d], a[2 * d + 1]);
            __builtin_amdgcn_raw_buffer_store_b128(r, rs, (c * 64 * kVPT + 64 * q + lane) * 16, 0, kAux);
        }
    };
    u32x4 va[K][kVPT], vb[K][kVPT];
    issue(0, va);
    for (int64_t j = 0; j < nitems; j += 2) {
        if (j + 1 < nitems) issue(j + 1, vb);
        finish(j, va);
        if (j + 1 >= nitems) break;
        if (j + 2 < nitems) issue(j + 2, va);
        finish(j + 1, vb);
    }
}

}  // namespace

extern "C" int probe_token_stream(int vpt, int aux, const void* src, const int32_t* table, void* out, int T,
                                  int hidden, int grid, hipStream_t s) {
    const uint16_t* x = (const uint16_t*)src;
    uint16_t* o = (uint16_t*)out;
    if (hidden % (8 * 64 * vpt)) return -1;
#define L(V, A) hipLaunchKernelGGL((token_stream<V, A>), dim3(grid), dim3(256), 0, s, x, table, o, T, hidden)
    if (vpt == 1 && aux == 16) L(1, 16);
    else if (vpt == 2 && aux == 16) L(2, 16);
    else if (vpt == 1 && aux == 2) L(1, 2);
    else if (vpt == 2 && aux == 2) L(2, 2);
    else return -2;
#undef L
    return hipGetLastError();
}
