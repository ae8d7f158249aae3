// probe_prefetch.hip -- diagnostic (not product code): read a list of expanded rows in the given
// (address-sorted) order and discard them, so that a later gather of the same rows can be served
// from the Infinity Cache.  Used by tools/kprefetch.py to test whether a window-ordered sweep ahead
// of the fused combine turns its 256 concurrent expert-segment streams into one sequential sweep.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* row, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(row), 0, bytes, 0x00020000);
}

// One wave per row (14 x 16 B per lane at hidden 7168), consecutive waves on consecutive rows of the
// list; the loaded words are folded into one value that is stored only if it equals a magic number.
template <int kAux>
__global__ void __launch_bounds__(256) prefetch_rows(const uint16_t* x, int64_t stride, const int32_t* rows, int n,
                                                     int nvec, uint32_t* sink) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = static_cast<int64_t>(gridDim.x) * 4;
    uint32_t acc = 0;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); i < n; i += nw) {
        const int32_t r = rows[i];
        const __amdgpu_buffer_rsrc_t rs = row_rsrc(x + static_cast<int64_t>(r) * stride, nvec * 16);
        u32x4 v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j)
            v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (j * 64 + lane) * 16, 0, kAux);   // range-checked
#pragma unroll
        for (int j = 0; j < 16; ++j) acc ^= v[j][0] ^ v[j][3];
    }
    if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

}  // namespace

extern "C" int probe_prefetch(int policy, const void* x, int64_t stride, const int32_t* rows, int n, int hidden,
                              int grid, void* sink, void* stream) {
    if (n <= 0) return 0;
    const int nvec = hidden / 8;
    if (nvec > 16 * 64) return -1;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 g(static_cast<unsigned>(grid)), b(256);
    const auto* xs = static_cast<const uint16_t*>(x);
    auto* sk = static_cast<uint32_t*>(sink);
    if (policy == 1) hipLaunchKernelGGL(prefetch_rows<2>, g, b, 0, s, xs, stride, rows, n, nvec, sk);        // nt
    else if (policy == 2) hipLaunchKernelGGL(prefetch_rows<16>, g, b, 0, s, xs, stride, rows, n, nvec, sk);  // sc1
    else hipLaunchKernelGGL(prefetch_rows<0>, g, b, 0, s, xs, stride, rows, n, nvec, sk);                    // plain
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
