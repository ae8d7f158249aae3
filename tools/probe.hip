// tools/probe.hip -- diagnostic kernels for the combine's memory roofline (not product code).
//
// Each probe isolates one property of the fused combine's traffic on MI355X:
//   stream_read      sequential read of a buffer, 16 B/lane, sum kept live (read ceiling)
//   stream_copy      16 B/lane copy (read+write ceiling)
//   gather<...>      the combine's access pattern: per (token, column chunk) item, 8 source rows
//                    gathered through a slot table, fp32 sum, bf16 row written
//                    kStore    write the output row (else keep the sum live, no store)
//                    kSeq      ignore the table: row = token * 8 + k (sequential rows)
//                    kNT       non-temporal loads
//                    kPipe     software pipeline: issue the next item's loads before reducing
//                              the current one (persistent grid-stride over items)
// Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/libprobe.so tools/probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

template <bool kNT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if constexpr (kNT) return __builtin_nontemporal_load(p);
    else return *p;
}

__global__ void __launch_bounds__(256) stream_read(const u32x4* src, int64_t nvec, float* sink) {
    float acc = 0.f;
    for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256 * 4) {
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t k = i + (int64_t)j * gridDim.x * 256;
            v[j] = k < nvec ? __builtin_nontemporal_load(src + k) : (u32x4){0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += lo(v[j][0]) + hi(v[j][3]);
    }
    if (acc == 12345.f) sink[0] = acc;
}

__global__ void __launch_bounds__(256) stream_copy(const u32x4* src, u32x4* dst, int64_t nvec) {
    for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

template <bool kStore, bool kSeq, bool kNT, bool kPipe>
__global__ void __launch_bounds__(256) gather(const uint16_t* src, const int32_t* table, uint16_t* out,
                                              int T, int hidden, float* sink) {
    constexpr int K = 8;
    const int lane = threadIdx.x & 63;
    const int nvec = hidden / 8;
    const int nchunks = nvec / 128;                   // 64 lanes x 2 vectors per chunk
    const int64_t items = (int64_t)T * nchunks;
    const int64_t gwave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    float keep = 0.f;

    auto slot_of = [&](int64_t t, int k) -> int64_t {
        if constexpr (kSeq) return t * K + k;
        else return table[t * K + k];
    };
    auto issue = [&](int64_t it, u32x4 (&v)[K][2]) {
        const int64_t t = it / nchunks;
        const int c = (int)(it - t * nchunks);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t s = __builtin_amdgcn_readfirstlane((int)slot_of(t, k));
            const u32x4* row = reinterpret_cast<const u32x4*>(src + s * hidden) + c * 128 + lane;
            v[k][0] = ld<kNT>(row);
            v[k][1] = ld<kNT>(row + 64);
        }
    };
    auto finish = [&](int64_t it, u32x4 (&v)[K][2]) {
        const int64_t t = it / nchunks;
        const int c = (int)(it - t * nchunks);
        float a[2][8] = {};
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    a[h][2 * d] += lo(v[k][h][d]);
                    a[h][2 * d + 1] += hi(v[k][h][d]);
                }
        if constexpr (kStore) {
            u32x4* o = reinterpret_cast<u32x4*>(out + t * hidden) + c * 128 + lane;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                u32x4 r;
#pragma unroll
                for (int d = 0; d < 4; ++d) r[d] = pack(a[h][2 * d], a[h][2 * d + 1]);
                __builtin_nontemporal_store(r, o + 64 * h);
            }
        } else {
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int e = 0; e < 8; ++e) keep += a[h][e];
        }
    };

    if constexpr (kPipe) {
        u32x4 va[K][2], vb[K][2];
        int64_t it = gwave;
        if (it < items) issue(it, va);
        while (it < items) {
            const int64_t nx = it + nwaves;
            if (nx < items) issue(nx, vb);
            finish(it, va);
            it = nx;
            if (it >= items) break;
            const int64_t nx2 = it + nwaves;
            if (nx2 < items) issue(nx2, va);
            finish(it, vb);
            it = nx2;
        }
    } else {
        for (int64_t it = gwave; it < items; it += nwaves) {
            u32x4 v[K][2];
            issue(it, v);
            finish(it, v);
        }
    }
    if (!kStore && keep == 12345.f) sink[0] = keep;
}

extern "C" {

int probe_stream_read(const void* src, int64_t bytes, float* sink, int grid, hipStream_t s) {
    hipLaunchKernelGGL(stream_read, dim3(grid), dim3(256), 0, s, (const u32x4*)src, bytes / 16, sink);
    return hipGetLastError();
}

int probe_stream_copy(const void* src, void* dst, int64_t bytes, int grid, hipStream_t s) {
    hipLaunchKernelGGL(stream_copy, dim3(grid), dim3(256), 0, s, (const u32x4*)src, (u32x4*)dst, bytes / 16);
    return hipGetLastError();
}

int probe_gather(int variant, const void* src, const int32_t* table, void* out, int T, int hidden,
                 float* sink, int grid, hipStream_t s) {
    // variant bits: 1 store, 2 sequential rows, 4 nt loads, 8 pipelined
    const uint16_t* x = (const uint16_t*)src;
    uint16_t* o = (uint16_t*)out;
#define P(V, A, B, C, D) case V: hipLaunchKernelGGL((gather<A, B, C, D>), dim3(grid), dim3(256), 0, s, x, table, o, T, hidden, sink); break;
    switch (variant) {
        P(0, false, false, false, false) P(1, true, false, false, false) P(2, false, true, false, false)
        P(3, true, true, false, false) P(4, false, false, true, false) P(5, true, false, true, false)
        P(6, false, true, true, false) P(7, true, true, true, false) P(8, false, false, false, true)
        P(9, true, false, false, true) P(10, false, true, false, true) P(11, true, true, false, true)
        P(12, false, false, true, true) P(13, true, false, true, true) P(14, false, true, true, true)
        P(15, true, true, true, true)
        default: return -1;
    }
#undef P
    return hipGetLastError();
}

}

// ---- store-policy probes: gather (table, nt loads) + buffer stores with a given aux policy
//      aux bits (gfx950): 1 = sc0, 2 = nt, 16 = sc1.  kRegion > 0 wraps the output rows modulo
//      kRegion tokens (writes stay cache-resident), kNoLoad stores without loading (write only).
template <int kAux, int kRegion, bool kNoLoad>
__global__ void __launch_bounds__(256) gather_store(const uint16_t* src, const int32_t* table, uint16_t* out,
                                                    int T, int hidden) {
    constexpr int K = 8;
    const int lane = threadIdx.x & 63;
    const int nvec = hidden / 8;
    const int nchunks = nvec / 128;
    const int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (it >= (int64_t)T * nchunks) return;
    const int64_t t = it / nchunks;
    const int c = (int)(it - t * nchunks);
    float a[2][8] = {};
    if constexpr (!kNoLoad) {
        u32x4 v[K][2];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t s = __builtin_amdgcn_readfirstlane(table[t * K + k]);
            const u32x4* row = reinterpret_cast<const u32x4*>(src + s * hidden) + c * 128 + lane;
            v[k][0] = __builtin_nontemporal_load(row);
            v[k][1] = __builtin_nontemporal_load(row + 64);
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    a[h][2 * d] += lo(v[k][h][d]);
                    a[h][2 * d + 1] += hi(v[k][h][d]);
                }
    }
    const int64_t ot = kRegion > 0 ? (t % kRegion) : t;
    const int64_t base = (ot * hidden + (int64_t)c * 128 * 8) * 2;       // bytes
    __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        u32x4 r;
#pragma unroll
        for (int d = 0; d < 4; ++d) r[d] = pack(a[h][2 * d], a[h][2 * d + 1]);
        __builtin_amdgcn_raw_buffer_store_b128(r, rsrc, (int)(base + (h * 64 + lane) * 16), 0, kAux);
    }
}

// ---- write-burst probe: a workgroup of 8 waves reduces 8 consecutive items (16 KiB of contiguous
//      output at H = 7168: items are row-major chunks) into LDS, then stores the 16 KiB as one burst
//      with all 512 threads (sc1), instead of each wave storing its 2 KiB as soon as it is done.
//      kRounds > 1: a persistent workgroup buffers kRounds such groups (kRounds x 16 KiB) per burst.
template <int kRounds>
__global__ void __launch_bounds__(512) gather_burst(const uint16_t* src, const int32_t* table, uint16_t* out,
                                                    int T, int hidden) {
    constexpr int K = 8;
    __shared__ u32x4 s_out[kRounds][8][128];                 // [round][wave][2 x 64 lanes]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nvec = hidden / 8;
    const int nchunks = nvec / 128;
    const int64_t items = (int64_t)T * nchunks;
    for (int64_t g0 = (int64_t)blockIdx.x * 8 * kRounds; g0 < items; g0 += (int64_t)gridDim.x * 8 * kRounds) {
#pragma unroll
        for (int r = 0; r < kRounds; ++r) {
            const int64_t it = g0 + r * 8 + wave;
            if (it >= items) continue;
            const int64_t t = it / nchunks;
            const int c = (int)(it - t * nchunks);
            float a[2][8] = {};
            u32x4 v[K][2];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int64_t srow = __builtin_amdgcn_readfirstlane(table[t * K + k]);
                const u32x4* row = reinterpret_cast<const u32x4*>(src + srow * hidden) + c * 128 + lane;
                v[k][0] = __builtin_nontemporal_load(row);
                v[k][1] = __builtin_nontemporal_load(row + 64);
            }
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        a[h][2 * d] += lo(v[k][h][d]);
                        a[h][2 * d + 1] += hi(v[k][h][d]);
                    }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                u32x4 q;
#pragma unroll
                for (int d = 0; d < 4; ++d) q[d] = pack(a[h][2 * d], a[h][2 * d + 1]);
                s_out[r][wave][h * 64 + lane] = q;
            }
        }
        __syncthreads();
        // the group's items are consecutive, so its output is one contiguous run of 8 x kRounds x 2 KiB
        const int64_t n_it = min((int64_t)8 * kRounds, items - g0);
        const u32x4* flat = &s_out[0][0][0];
        u32x4* dst = reinterpret_cast<u32x4*>(out) + g0 * 128;
        __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(n_it * 2048), 0x00020000);
        for (int i = threadIdx.x; i < 8 * kRounds * 128; i += 512)
            __builtin_amdgcn_raw_buffer_store_b128(flat[i], rsrc, i * 16, 0, 16);
        __syncthreads();
    }
}

static int g_lds_pad = 0;      // extra dynamic LDS per workgroup (caps workgroups per CU: occupancy probe)
extern "C" void probe_set_lds_pad(int bytes) { g_lds_pad = bytes; }

extern "C" int probe_gather_burst(int rounds, int grid, const void* src, const int32_t* table, void* out, int T,
                                  int hidden, hipStream_t s) {
    const uint16_t* x = (const uint16_t*)src;
    uint16_t* o = (uint16_t*)out;
    const int64_t items = (int64_t)T * (hidden / 8 / 128);
    if (grid <= 0) grid = (int)((items + 8 * rounds - 1) / (8 * rounds));
    if (rounds == 1) hipLaunchKernelGGL((gather_burst<1>), dim3(grid), dim3(512), g_lds_pad, s, x, table, o, T, hidden);
    else if (rounds == 2) hipLaunchKernelGGL((gather_burst<2>), dim3(grid), dim3(512), g_lds_pad, s, x, table, o, T, hidden);
    else if (rounds == 4) hipLaunchKernelGGL((gather_burst<4>), dim3(grid), dim3(512), g_lds_pad, s, x, table, o, T, hidden);
    else return -1;
    return hipGetLastError();
}

extern "C" int probe_gather_store(int policy, int region, int noload, const void* src, const int32_t* table,
                                  void* out, int T, int hidden, hipStream_t s) {
    const uint16_t* x = (const uint16_t*)src;
    uint16_t* o = (uint16_t*)out;
    const int items = T * (hidden / 8 / 128);
    const dim3 g((items + 3) / 4), b(256);
#define Q(A, R, N) if (policy == A && region == R && noload == N) { hipLaunchKernelGGL((gather_store<A, R, N>), g, b, 0, s, x, table, o, T, hidden); return hipGetLastError(); }
    Q(0, 0, 0) Q(1, 0, 0) Q(2, 0, 0) Q(3, 0, 0) Q(16, 0, 0) Q(17, 0, 0) Q(18, 0, 0) Q(19, 0, 0)
    Q(2, 64, 0) Q(0, 64, 0) Q(16, 64, 0)
    Q(0, 0, 1) Q(2, 0, 1) Q(16, 0, 1)
#undef Q
    return -1;
}
