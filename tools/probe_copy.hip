// Dispatch-copy probes (diagnostic, not the product): the expanded copy x[T][H] -> out[N][H]
// source-major (one wave per (token, 2 KiB chunk), up to K scattered stores) vs destination-major
// (one wave per (kRows consecutive expanded rows, 2 KiB chunk), gathered loads, in-order stores).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) scatter_copy(const uint8_t* x, const int32_t* dst, int T, int K, int xb,
                                                    uint8_t* out) {
    const int lane = threadIdx.x & 63;
    const int nvec = xb / 16, nch = (nvec + 127) / 128;
    const int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (it >= (int64_t)T * nch) return;
    const int64_t t = it / nch;
    const int c = (int)(it - t * nch);
    int32_t my = lane < K ? dst[t * K + lane] : -1;
    const uint64_t m0 = __ballot(my >= 0);
    const int v0 = c * 128 + lane, v1 = v0 + 64;
    const u32x4 z = {0u, 0u, 0u, 0u};
    const u32x4 a0 = v0 < nvec ? __builtin_nontemporal_load((const u32x4*)(x + t * xb) + v0) : z;
    const u32x4 a1 = v1 < nvec ? __builtin_nontemporal_load((const u32x4*)(x + t * xb) + v1) : z;
    for (uint64_t m = m0; m; m &= m - 1) {
        const int64_t d = __builtin_amdgcn_readlane(my, __builtin_ctzll(m));
        auto rs = __builtin_amdgcn_make_buffer_rsrc(out + d * xb, 0, xb, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(a0, rs, v0 * 16, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(a1, rs, v1 * 16, 0, 16);
    }
}

template <int kRows, int kAux>
__global__ void __launch_bounds__(256) gather_copy(const uint8_t* x, const int32_t* inv, int N, int xb,
                                                   uint8_t* out) {
    const int lane = threadIdx.x & 63;
    const int nvec = xb / 16, nch = (nvec + 127) / 128;
    const int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t ngroups = ((int64_t)N + kRows - 1) / kRows;
    if (it >= ngroups * nch) return;
    // chunk-major inside a group so the 4 waves of a workgroup write 4 consecutive chunks
    const int64_t grp = it / nch;
    const int c = (int)(it - grp * nch);
    const int v0 = c * 128 + lane, v1 = v0 + 64;
    const u32x4 z = {0u, 0u, 0u, 0u};
    u32x4 a[kRows][2];
    int64_t rows[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int64_t j = grp * kRows + r;
        const int32_t t = j < N ? inv[j] : -1;
        rows[r] = t;
        const u32x4* src = (const u32x4*)(x + (int64_t)(t < 0 ? 0 : t) * xb);
        a[r][0] = (t >= 0 && v0 < nvec) ? src[v0] : z;
        a[r][1] = (t >= 0 && v1 < nvec) ? src[v1] : z;
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int64_t j = grp * kRows + r;
        if (j >= N || rows[r] < 0) continue;
        auto rs = __builtin_amdgcn_make_buffer_rsrc(out + j * xb, 0, xb, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(a[r][0], rs, v0 * 16, 0, kAux);
        __builtin_amdgcn_raw_buffer_store_b128(a[r][1], rs, v1 * 16, 0, kAux);
    }
}


// Generalised source-major scatter: kWaves waves per workgroup, item = (token, 64*kVPT-vector chunk).
template <int kWaves, int kVPT, int kAux>
__global__ void __launch_bounds__(64 * kWaves) scatter_copy_t(const uint8_t* x, const int32_t* dst, int T, int K,
                                                              int xb, uint8_t* out) {
    const int lane = threadIdx.x & 63;
    constexpr int kCh = 64 * kVPT;
    const int nvec = xb / 16, nch = (nvec + kCh - 1) / kCh;
    const int64_t it = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (it >= (int64_t)T * nch) return;
    const int64_t t = it / nch;
    const int c = (int)(it - t * nch);
    int32_t my = lane < K ? dst[t * K + lane] : -1;
    const uint64_t m0 = __ballot(my >= 0);
    const u32x4 z = {0u, 0u, 0u, 0u};
    u32x4 a[kVPT];
#pragma unroll
    for (int v = 0; v < kVPT; ++v) {
        const int vi = c * kCh + v * 64 + lane;
        a[v] = vi < nvec ? __builtin_nontemporal_load((const u32x4*)(x + t * xb) + vi) : z;
    }
    for (uint64_t m = m0; m; m &= m - 1) {
        const int64_t d = __builtin_amdgcn_readlane(my, __builtin_ctzll(m));
        auto rs = __builtin_amdgcn_make_buffer_rsrc(out + d * xb, 0, xb, 0x00020000);
#pragma unroll
        for (int v = 0; v < kVPT; ++v)
            __builtin_amdgcn_raw_buffer_store_b128(a[v], rs, (c * kCh + v * 64 + lane) * 16, 0, kAux);
    }
}

template <int kWaves, int kVPT, int kAux>
static void launch_t(const uint8_t* x, const int32_t* dst, int T, int K, int xb, uint8_t* o, hipStream_t s) {
    const int nch = (xb / 16 + 64 * kVPT - 1) / (64 * kVPT);
    const int64_t items = (int64_t)T * nch;
    hipLaunchKernelGGL((scatter_copy_t<kWaves, kVPT, kAux>), dim3((unsigned)((items + kWaves - 1) / kWaves)),
                       dim3(64 * kWaves), 0, s, x, dst, T, K, xb, o);
}


// Write-only scatter (no loads): the destination pattern of the copy with constant data.
__global__ void __launch_bounds__(256) scatter_write_only(const int32_t* dst, int T, int K, int xb, uint8_t* out) {
    const int lane = threadIdx.x & 63;
    const int nvec = xb / 16, nch = (nvec + 127) / 128;
    const int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (it >= (int64_t)T * nch) return;
    const int64_t t = it / nch;
    const int c = (int)(it - t * nch);
    int32_t my = lane < K ? dst[t * K + lane] : -1;
    const uint64_t m0 = __ballot(my >= 0);
    const int v0 = c * 128 + lane, v1 = v0 + 64;
    const u32x4 a = {(uint32_t)t, 1u, 2u, 3u};
    for (uint64_t m = m0; m; m &= m - 1) {
        const int64_t d = __builtin_amdgcn_readlane(my, __builtin_ctzll(m));
        auto rs = __builtin_amdgcn_make_buffer_rsrc(out + d * xb, 0, xb, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(a, rs, v0 * 16, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(a, rs, v1 * 16, 0, 16);
    }
}
// Write-only in address order: one wave per (row, 2 KiB chunk) of out.
__global__ void __launch_bounds__(256) seq_write_only(int N, int xb, uint8_t* out) {
    const int lane = threadIdx.x & 63;
    const int nvec = xb / 16, nch = (nvec + 127) / 128;
    const int64_t it = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (it >= (int64_t)N * nch) return;
    const int64_t j = it / nch;
    const int c = (int)(it - j * nch);
    const int v0 = c * 128 + lane, v1 = v0 + 64;
    const u32x4 a = {(uint32_t)j, 1u, 2u, 3u};
    auto rs = __builtin_amdgcn_make_buffer_rsrc(out + j * xb, 0, xb, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(a, rs, v0 * 16, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(a, rs, v1 * 16, 0, 16);
}

// One wave per token, its 2 KiB chunks in order with the next kAhead chunks' loads in flight while the
// current chunk is stored to every destination (the read latency hidden behind the store stream).
template <int kWaves, int kAhead>
__global__ void __launch_bounds__(64 * kWaves) scatter_copy_pf(const uint8_t* x, const int32_t* dst, int T, int K,
                                                               int xb, uint8_t* out) {
    const int lane = threadIdx.x & 63;
    const int nvec = xb / 16, nch = (nvec + 127) / 128;
    const int64_t t = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (t >= T) return;
    int32_t my = lane < K ? dst[t * K + lane] : -1;
    const uint64_t m0 = __ballot(my >= 0);
    const u32x4 z = {0u, 0u, 0u, 0u};
    const u32x4* src = (const u32x4*)(x + t * xb);
    u32x4 a[kAhead + 1][2];
#pragma unroll
    for (int j = 0; j <= kAhead; ++j) {
        const int v0 = j * 128 + lane, v1 = v0 + 64;
        a[j][0] = (j < nch && v0 < nvec) ? __builtin_nontemporal_load(src + v0) : z;
        a[j][1] = (j < nch && v1 < nvec) ? __builtin_nontemporal_load(src + v1) : z;
    }
    for (int c = 0; c < nch; ++c) {
        const int v0 = c * 128 + lane, v1 = v0 + 64;
        for (uint64_t m = m0; m; m &= m - 1) {
            const int64_t d = __builtin_amdgcn_readlane(my, __builtin_ctzll(m));
            auto rs = __builtin_amdgcn_make_buffer_rsrc(out + d * xb, 0, xb, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(a[0][0], rs, v0 * 16, 0, 16);
            __builtin_amdgcn_raw_buffer_store_b128(a[0][1], rs, v1 * 16, 0, 16);
        }
#pragma unroll
        for (int j = 0; j < kAhead; ++j) { a[j][0] = a[j + 1][0]; a[j][1] = a[j + 1][1]; }
        const int n = c + kAhead + 1, w0 = n * 128 + lane, w1 = w0 + 64;
        a[kAhead][0] = (n < nch && w0 < nvec) ? __builtin_nontemporal_load(src + w0) : z;
        a[kAhead][1] = (n < nch && w1 < nvec) ? __builtin_nontemporal_load(src + w1) : z;
    }
}

// Blocked destination-major: the tokens are cut into kTok-token blocks; inside a block, one wave per
// (expert, 2 KiB chunk) copies the block's rows of that expert -- consecutive destination rows, so
// every store run is an expert segment of the block -- reading x rows that the block keeps hot in
// cache (kTok x 14 KiB: 3.5 MB at 256 tokens).  kXcd: each block is owned by one XCD (workgroup w runs on
// XCD w % 8, so workgroups w = xcd (mod 8) take blocks xcd, xcd + 8, ...) and its x rows stay in
// that XCD's L2; otherwise blocks are dealt to the grid in order (re-reads from the Infinity Cache).
// off / cnt: [nblocks][E] first destination row and row count of expert e inside block b; inv[row] =
// the source token of destination row `row`.
template <int kAux, bool kXcd, bool kNT>
__global__ void __launch_bounds__(256) blocked_copy(const uint8_t* x, const int32_t* inv, const int32_t* off,
                                                    const int32_t* cnt, int nblocks, int E, int xb, uint8_t* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nvec = xb / 16, nch = (nvec + 127) / 128;
    const int64_t wg_per_block = ((int64_t)E * nch + 3) / 4;
    int64_t blk, k;
    if (kXcd) {
        const int64_t xcd = blockIdx.x % 8, kk = blockIdx.x / 8;
        blk = xcd + 8 * (kk / wg_per_block);
        k = kk % wg_per_block;
    } else {
        blk = blockIdx.x / wg_per_block;
        k = blockIdx.x % wg_per_block;
    }
    if (blk >= nblocks) return;
    const int64_t it = k * 4 + wave;
    const int e = (int)(it / nch), c = (int)(it - (int64_t)e * nch);
    if (e >= E) return;
    const int r0 = off[blk * E + e], n = cnt[blk * E + e];
    const int v0 = c * 128 + lane, v1 = v0 + 64;
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (int j = 0; j < n; j += 4) {
        u32x4 a[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (j + q < n) {
                const int64_t t = __builtin_amdgcn_readfirstlane(inv[r0 + j + q]);
                const u32x4* src = (const u32x4*)(x + t * xb);
                if constexpr (kNT) {
                    a[q][0] = v0 < nvec ? __builtin_nontemporal_load(src + v0) : z;
                    a[q][1] = v1 < nvec ? __builtin_nontemporal_load(src + v1) : z;
                } else {
                    a[q][0] = v0 < nvec ? src[v0] : z;
                    a[q][1] = v1 < nvec ? src[v1] : z;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (j + q < n) {
                auto rs = __builtin_amdgcn_make_buffer_rsrc(out + (int64_t)(r0 + j + q) * xb, 0, xb, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(a[q][0], rs, v0 * 16, 0, kAux);
                __builtin_amdgcn_raw_buffer_store_b128(a[q][1], rs, v1 * 16, 0, kAux);
            }
        }
    }
}

// Row-streaming variant of blocked_copy: one wave per (block, expert) walks the block's rows of the
// expert, each row whole (kVec 16-byte vectors per lane: all of a 14 KiB row at kVec = 14), so a
// wave's stores are whole consecutive rows -- one contiguous run per (block, expert).
template <int kAux, int kVec>
__global__ void __launch_bounds__(256) blocked_copy_rows(const uint8_t* x, const int32_t* inv, const int32_t* off,
                                                         const int32_t* cnt, int nblocks, int E, int xb, uint8_t* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nvec = xb / 16;
    const int64_t wg_per_block = ((int64_t)E + 3) / 4;
    const int64_t xcd = blockIdx.x % 8, kk = blockIdx.x / 8;
    const int64_t blk = xcd + 8 * (kk / wg_per_block);
    const int e = (int)((kk % wg_per_block) * 4 + wave);
    if (blk >= nblocks || e >= E) return;
    const int r0 = off[blk * E + e], n = cnt[blk * E + e];
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (int j = 0; j < n; ++j) {
        const int64_t t = __builtin_amdgcn_readfirstlane(inv[r0 + j]);
        const u32x4* src = (const u32x4*)(x + t * xb);
        u32x4 a[kVec];
#pragma unroll
        for (int q = 0; q < kVec; ++q) a[q] = q * 64 + lane < nvec ? src[q * 64 + lane] : z;
        auto rs = __builtin_amdgcn_make_buffer_rsrc(out + (int64_t)(r0 + j) * xb, 0, xb, 0x00020000);
#pragma unroll
        for (int q = 0; q < kVec; ++q) __builtin_amdgcn_raw_buffer_store_b128(a[q], rs, (q * 64 + lane) * 16, 0, kAux);
    }
}

// blocked_copy with kRows rows in flight per wave
template <int kAux, int kRows>
__global__ void __launch_bounds__(256) blocked_copy_r(const uint8_t* x, const int32_t* inv, const int32_t* off,
                                                      const int32_t* cnt, int nblocks, int E, int xb, uint8_t* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nvec = xb / 16, nch = (nvec + 127) / 128;
    const int64_t wg_per_block = ((int64_t)E * nch + 3) / 4;
    const int64_t xcd = blockIdx.x % 8, kk = blockIdx.x / 8;
    const int64_t blk = xcd + 8 * (kk / wg_per_block);
    const int64_t it = (kk % wg_per_block) * 4 + wave;
    const int e = (int)(it / nch), c = (int)(it - (int64_t)e * nch);
    if (blk >= nblocks || e >= E) return;
    const int r0 = off[blk * E + e], n = cnt[blk * E + e];
    const int v0 = c * 128 + lane, v1 = v0 + 64;
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (int j = 0; j < n; j += kRows) {
        u32x4 a[kRows][2];
#pragma unroll
        for (int q = 0; q < kRows; ++q) {
            if (j + q < n) {
                const int64_t t = __builtin_amdgcn_readfirstlane(inv[r0 + j + q]);
                const u32x4* src = (const u32x4*)(x + t * xb);
                a[q][0] = v0 < nvec ? src[v0] : z;
                a[q][1] = v1 < nvec ? src[v1] : z;
            }
        }
#pragma unroll
        for (int q = 0; q < kRows; ++q) {
            if (j + q < n) {
                auto rs = __builtin_amdgcn_make_buffer_rsrc(out + (int64_t)(r0 + j + q) * xb, 0, xb, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(a[q][0], rs, v0 * 16, 0, kAux);
                __builtin_amdgcn_raw_buffer_store_b128(a[q][1], rs, v1 * 16, 0, kAux);
            }
        }
    }
}

extern "C" int probe_blocked_copy(int variant, const void* x, const int32_t* inv, const int32_t* off,
                                  const int32_t* cnt, int nblocks, int E, int xb, void* out, hipStream_t s) {
    const int nch = (xb / 16 + 127) / 128;
    const int64_t wg_per_block = ((int64_t)E * nch + 3) / 4;
    const dim3 g_xcd((unsigned)(8 * wg_per_block * ((nblocks + 7) / 8))), g_lin((unsigned)(wg_per_block * nblocks));
    const uint8_t* xx = (const uint8_t*)x;
    uint8_t* o = (uint8_t*)out;
    switch (variant) {
        case 0: hipLaunchKernelGGL((blocked_copy<16, true, false>), g_xcd, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o); break;
        case 1: hipLaunchKernelGGL((blocked_copy<16, false, false>), g_lin, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o); break;
        case 2: hipLaunchKernelGGL((blocked_copy<0, true, false>), g_xcd, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o); break;
        case 3: hipLaunchKernelGGL((blocked_copy<2, true, false>), g_xcd, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o); break;
        case 4: hipLaunchKernelGGL((blocked_copy<16, true, true>), g_xcd, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o); break;
        case 5: hipLaunchKernelGGL((blocked_copy<2, false, false>), g_lin, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o); break;
        case 6: hipLaunchKernelGGL((blocked_copy_r<2, 8>), g_xcd, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o); break;
        case 7: hipLaunchKernelGGL((blocked_copy_r<2, 2>), g_xcd, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o); break;
        case 8: hipLaunchKernelGGL((blocked_copy_r<3, 4>), g_xcd, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o); break;
        case 9: hipLaunchKernelGGL((blocked_copy_r<18, 4>), g_xcd, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o); break;
        case 10: {
            const dim3 g((unsigned)(8 * ((E + 3) / 4) * ((nblocks + 7) / 8)));
            if (xb == 14336) hipLaunchKernelGGL((blocked_copy_rows<2, 14>), g, dim3(256), 0, s, xx, inv, off, cnt, nblocks, E, xb, o);
            else return -2;
            break;
        }
        default: return -1;
    }
    return (int)hipGetLastError();
}

template <int kWaves, int kAhead>
static void launch_pf(const uint8_t* x, const int32_t* dst, int T, int K, int xb, uint8_t* o, hipStream_t s) {
    hipLaunchKernelGGL((scatter_copy_pf<kWaves, kAhead>), dim3((unsigned)((T + kWaves - 1) / kWaves)),
                       dim3(64 * kWaves), 0, s, x, dst, T, K, xb, o);
}

extern "C" int probe_copy(int variant, const void* x, const int32_t* dst, const int32_t* inv, int T, int K, int N,
                          int xb, void* out, hipStream_t s) {
    const int nch = (xb / 16 + 127) / 128;
    auto grid = [&](int64_t items) { return dim3((unsigned)((items + 3) / 4)); };
    const uint8_t* xx = (const uint8_t*)x;
    uint8_t* o = (uint8_t*)out;
    switch (variant) {
        case 0: hipLaunchKernelGGL(scatter_copy, grid((int64_t)T * nch), dim3(256), 0, s, xx, dst, T, K, xb, o); break;
        case 1: hipLaunchKernelGGL((gather_copy<1, 16>), grid((int64_t)N * nch), dim3(256), 0, s, xx, inv, N, xb, o); break;
        case 2: hipLaunchKernelGGL((gather_copy<2, 16>), grid((int64_t)(N + 1) / 2 * nch), dim3(256), 0, s, xx, inv, N, xb, o); break;
        case 4: hipLaunchKernelGGL((gather_copy<4, 16>), grid((int64_t)(N + 3) / 4 * nch), dim3(256), 0, s, xx, inv, N, xb, o); break;
        case 8: hipLaunchKernelGGL((gather_copy<8, 16>), grid((int64_t)(N + 7) / 8 * nch), dim3(256), 0, s, xx, inv, N, xb, o); break;
        case 40: hipLaunchKernelGGL((gather_copy<4, 0>), grid((int64_t)(N + 3) / 4 * nch), dim3(256), 0, s, xx, inv, N, xb, o); break;
        case 42: hipLaunchKernelGGL((gather_copy<4, 2>), grid((int64_t)(N + 3) / 4 * nch), dim3(256), 0, s, xx, inv, N, xb, o); break;
        case 48: hipLaunchKernelGGL((gather_copy<4, 18>), grid((int64_t)(N + 3) / 4 * nch), dim3(256), 0, s, xx, inv, N, xb, o); break;
        case 88: hipLaunchKernelGGL((gather_copy<8, 18>), grid((int64_t)(N + 7) / 8 * nch), dim3(256), 0, s, xx, inv, N, xb, o); break;
        case 28: hipLaunchKernelGGL((gather_copy<2, 18>), grid((int64_t)(N + 1) / 2 * nch), dim3(256), 0, s, xx, inv, N, xb, o); break;
        case 100: launch_t<4, 2, 16>(xx, dst, T, K, xb, o, s); break;
        case 101: launch_t<8, 2, 16>(xx, dst, T, K, xb, o, s); break;
        case 102: launch_t<4, 4, 16>(xx, dst, T, K, xb, o, s); break;
        case 103: launch_t<8, 4, 16>(xx, dst, T, K, xb, o, s); break;
        case 104: launch_t<4, 7, 16>(xx, dst, T, K, xb, o, s); break;
        case 105: launch_t<4, 14, 16>(xx, dst, T, K, xb, o, s); break;
        case 106: launch_t<4, 2, 0>(xx, dst, T, K, xb, o, s); break;
        case 107: launch_t<4, 2, 2>(xx, dst, T, K, xb, o, s); break;
        case 108: launch_t<2, 2, 16>(xx, dst, T, K, xb, o, s); break;
        case 109: launch_t<4, 1, 16>(xx, dst, T, K, xb, o, s); break;
        case 110: launch_t<16, 2, 16>(xx, dst, T, K, xb, o, s); break;
        case 111: launch_t<8, 7, 16>(xx, dst, T, K, xb, o, s); break;
        case 300: launch_pf<4, 1>(xx, dst, T, K, xb, o, s); break;
        case 301: launch_pf<4, 2>(xx, dst, T, K, xb, o, s); break;
        case 302: launch_pf<2, 1>(xx, dst, T, K, xb, o, s); break;
        case 303: launch_pf<1, 1>(xx, dst, T, K, xb, o, s); break;
        case 304: launch_pf<1, 3>(xx, dst, T, K, xb, o, s); break;
        case 200: hipLaunchKernelGGL(scatter_write_only, grid((int64_t)T * nch), dim3(256), 0, s, dst, T, K, xb, o); break;
        case 201: hipLaunchKernelGGL(seq_write_only, grid((int64_t)N * nch), dim3(256), 0, s, N, xb, o); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}
