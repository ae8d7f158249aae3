// dispatch.hip -- the handle producer of the combine path (ElasticBuffer.dispatch) on MI355X.
//
// Reference (paths in /root/reference):
//   dispatch_impl                deep_ep/include/deep_ep/impls/dispatch.cuh:17-409
//     notify: per-rank / per-expert counts, slot per destination (:79-258, :336-351)
//     push:   [hidden | sf | topk_idx | weights | src_global_idx] per (token, destination) (:373-392)
//   dispatch_copy_epilogue_impl  deep_ep/include/deep_ep/impls/dispatch_copy_epilogue.cuh:11-323
//     recv_x / recv_sf / recv_topk_weights, expanded rows grouped by local expert (:112-123),
//     recv_src_metadata = {src_global_idx, src_rank * K + master_topk, slot_0..slot_{K-1}} (:188-207)
//
// Design (MI355X-first): the exchange between ranks is one RCCL all_to_all_single of packed byte
// rows (host side); these kernels are the byte work around it.  The slot a token gets inside a
// destination / an expert is its rank among earlier tokens (ascending token order), computed with
// block scans and per-wave ballot masks instead of atomics, so the receive order is deterministic:
// grouped by source rank, ascending source token -- refs.dispatch's order and the reference's
// deterministic mode -- which the combine plan relies on.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdio.h>

#include <algorithm>

#include "../../include/deepep_amd.h"
#include "fault.h"

extern "C" __attribute__((visibility("hidden"))) int deepep_amd_set_error(int code, const char* msg);

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Receive-side blocks: DEEPEP_DISPATCH_BLOCK_ROWS consecutive received rows (count / slots / the expanded
// copy).  128 rows x 14 KiB = 1.8 MB of source rows per block: what one XCD's L2 keeps for the
// expanded copy's re-reads (below).
constexpr int kBlockRows = DEEPEP_DISPATCH_BLOCK_ROWS;

// ---------------------------------------------------------------- route: token -> destination slots
// dst_slot[t][r] = #{t' < t : t' routed to r} or -1; send_counts[r] = #{t : t routed to r}
// (dispatch.cuh:79-258 notify + slot assignment).  Two passes over 256-token blocks, one thread
// per token: (1) per-block counts per destination rank; (2) each block sums the counts of the
// blocks before it and ranks its tokens with per-wave ballots -- deterministic, no atomics on
// global memory, and every launch spreads over ceil(T / 256) workgroups.
__device__ __forceinline__ uint64_t route_mask(const int64_t* __restrict__ topk_idx, int t, int T, int K, int epr) {
    uint64_t mask = 0;
    if (t < T)
        for (int k = 0; k < K; ++k) {
            const int64_t e = topk_idx[static_cast<int64_t>(t) * K + k];
            if (e >= 0) mask |= 1ull << static_cast<int>(e / epr);
        }
    return mask;
}

__global__ void __launch_bounds__(256)
route_count_kernel(const int64_t* __restrict__ topk_idx, int T, int K, int epr, int R,
                   int32_t* __restrict__ block_counts) {
    __shared__ int32_t s_cnt[4][64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint64_t mask = route_mask(topk_idx, blockIdx.x * 256 + tid, T, K, epr);
    for (int r = 0; r < R; ++r) {
        const int c = __popcll(__ballot((mask >> r) & 1ull));
        if (lane == 0) s_cnt[wave][r] = c;
    }
    __syncthreads();
    if (tid < R)
        block_counts[static_cast<int64_t>(blockIdx.x) * R + tid] = s_cnt[0][tid] + s_cnt[1][tid] + s_cnt[2][tid] +
                                                                   s_cnt[3][tid];
}

__global__ void __launch_bounds__(256)
route_assign_kernel(const int64_t* __restrict__ topk_idx, int T, int K, int epr, int R,
                    const int32_t* __restrict__ block_counts, int32_t* __restrict__ dst_slot,
                    int32_t* __restrict__ send_counts) {
    __shared__ int32_t s_base[64];
    __shared__ int32_t s_cnt[4][64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int b = blockIdx.x, nb = gridDim.x;
    if (tid < R) {
        int base = 0;
        for (int j = 0; j < b; ++j) base += block_counts[static_cast<int64_t>(j) * R + tid];
        s_base[tid] = base;
        if (b == nb - 1) send_counts[tid] = base + block_counts[static_cast<int64_t>(b) * R + tid];
    }
    const int t = b * 256 + tid;
    const uint64_t mask = route_mask(topk_idx, t, T, K, epr);
    for (int r = 0; r < R; ++r) {
        const int c = __popcll(__ballot((mask >> r) & 1ull));
        if (lane == 0) s_cnt[wave][r] = c;
    }
    __syncthreads();
    if (t >= T) return;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int r = 0; r < R; ++r) {
        const bool hit = (mask >> r) & 1ull;
        const uint64_t bal = __ballot(hit);
        int slot = -1;
        if (hit) {
            slot = s_base[r] + __popcll(bal & lt);
            for (int w = 0; w < wave; ++w) slot += s_cnt[w][r];
        }
        dst_slot[static_cast<int64_t>(t) * R + r] = slot;
    }
}

// ---------------------------------------------------------------- expert histogram (notify)
// counts[e] += #{(t, k) : topk_idx[t][k] == e}: the per-expert half of dispatch_impl's notify
// (dispatch.cuh:79-258), exchanged together with the per-rank counts so the receiver learns its
// expert sizes -- and the host both vectors -- in one sync.  LDS histogram per workgroup, then one
// global atomic per non-empty bin (integer adds: the result does not depend on their order).
constexpr int kHistEntries = 2048;                   // (t, k) entries per workgroup

__global__ void __launch_bounds__(256)
expert_hist_kernel(const int64_t* __restrict__ topk_idx, int64_t n, int E, int32_t* __restrict__ counts) {
    extern __shared__ int32_t s_hist[];              // [E]
    for (int e = threadIdx.x; e < E; e += 256) s_hist[e] = 0;
    __syncthreads();
    const int64_t base = static_cast<int64_t>(blockIdx.x) * kHistEntries;
    for (int j = threadIdx.x; j < kHistEntries; j += 256) {
        const int64_t i = base + j;
        if (i < n) {
            const int64_t e = topk_idx[i];
            if (e >= 0 && e < E) atomicAdd(&s_hist[e], 1);
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < E; e += 256)
        if (s_hist[e] != 0) atomicAdd(&counts[e], s_hist[e]);
}

// ---------------------------------------------------------------- notify: the send side in two launches
// Everything the send side of a fresh dispatch derives from topk_idx: dst_slot (as route_count +
// route_assign), and the record every destination d gets -- notify[d] = [tokens to d | tokens per expert
// of d (expert_hist's slice) | per-64-token-block tokens to d | per-block (token, lane) pairs to d
// (block_counts_kernel)] -- plus the exclusive prefix of the per-rank counts (the packed rows' send
// offsets).  Two launches over 256-token workgroups replace five launches and three torch ops between
// them (a fresh dispatch is launch-bound: each launch costs ~10 us of host time):
//   count:  per workgroup, tokens per destination and an expert histogram (LDS) into the workspace;
//           the per-64-token-block counts (one wave = one block) straight into notify;
//   assign: per workgroup, the destination slots of its tokens (base = the earlier workgroups' counts,
//           ballot ranks inside), and a grid-strided share of the totals: per-destination tokens,
//           expert counts summed over the workgroups' histograms, send offsets, zeroed tail blocks.
// No atomics on global memory and no zeroed inputs; deterministic.
constexpr int kNotifyTok = 256;                      // tokens per workgroup (4 waves)

__global__ void __launch_bounds__(kNotifyTok)
notify_count_kernel(const int64_t* __restrict__ topk_idx, int T, int K, int E, int R, int nb,
                    int32_t* __restrict__ notify, int32_t* __restrict__ ws_cnt, int32_t* __restrict__ ws_hist) {
    extern __shared__ int32_t s_hist[];              // [E]
    __shared__ int32_t s_cnt[4][64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int epr = E / R;
    const int64_t W = 1 + epr + 2 * static_cast<int64_t>(nb);
    for (int e = tid; e < E; e += kNotifyTok) s_hist[e] = 0;
    __syncthreads();
    const int t = blockIdx.x * kNotifyTok + tid;
    uint64_t mask = 0;
    int rk[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        rk[k] = -1;
        if (k < K && t < T) {
            const int64_t e = topk_idx[static_cast<int64_t>(t) * K + k];
            if (e >= 0 && e < E) {
                rk[k] = static_cast<int>(e) / epr;
                mask |= 1ull << rk[k];
                atomicAdd(&s_hist[static_cast<int>(e)], 1);
            }
        }
    }
    const int b = blockIdx.x * (kNotifyTok / 64) + wave;     // this wave's 64-token block
    for (int r = 0; r < R; ++r) {
        const uint64_t bal = __ballot((mask >> r) & 1ull);
        if (lane == 0) s_cnt[wave][r] = __popcll(bal);
        if (nb > 0) {
            int c = 0;
#pragma unroll
            for (int k = 0; k < 32; ++k) c += rk[k] == r;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
            if (lane == 0 && b < nb) {
                notify[r * W + 1 + epr + b] = __popcll(bal);
                notify[r * W + 1 + epr + nb + b] = c;
            }
        }
    }
    __syncthreads();
    if (tid < R)
        ws_cnt[static_cast<int64_t>(blockIdx.x) * R + tid] = s_cnt[0][tid] + s_cnt[1][tid] + s_cnt[2][tid] + s_cnt[3][tid];
    for (int e = tid; e < E; e += kNotifyTok) ws_hist[static_cast<int64_t>(blockIdx.x) * E + e] = s_hist[e];
}

__global__ void __launch_bounds__(kNotifyTok)
notify_assign_kernel(const int64_t* __restrict__ topk_idx, int T, int K, int E, int R, int nb, int nblk,
                     const int32_t* __restrict__ ws_cnt, const int32_t* __restrict__ ws_hist,
                     int32_t* __restrict__ dst_slot, int32_t* __restrict__ notify, int32_t* __restrict__ send_offsets) {
    __shared__ int32_t s_base[64];
    __shared__ int32_t s_cnt[4][64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int blk = blockIdx.x, grid = gridDim.x;
    const int epr = E / R;
    const int64_t W = 1 + epr + 2 * static_cast<int64_t>(nb);
    constexpr int kBatch = 16;                           // loads in flight per thread
    // sum of base[j * stride] over j < n
    auto column_sum = [&](const int32_t* __restrict__ base, int64_t stride, int n) {
        int c = 0;
        for (int j0 = 0; j0 < n; j0 += kBatch) {
            int v[kBatch];
#pragma unroll
            for (int j = 0; j < kBatch; ++j) v[j] = j0 + j < n ? base[static_cast<int64_t>(j0 + j) * stride] : 0;
#pragma unroll
            for (int j = 0; j < kBatch; ++j) c += v[j];
        }
        return c;
    };
    if (tid < R) s_base[tid] = column_sum(ws_cnt + tid, R, min(blk, nblk));
    const int t = blk * kNotifyTok + tid;
    uint64_t mask = 0;
    if (t < T)
        for (int k = 0; k < K; ++k) {
            const int64_t e = topk_idx[static_cast<int64_t>(t) * K + k];
            if (e >= 0 && e < E) mask |= 1ull << (static_cast<int>(e) / epr);
        }
    for (int r = 0; r < R; ++r) {
        const int c = __popcll(__ballot((mask >> r) & 1ull));
        if (lane == 0) s_cnt[wave][r] = c;
    }
    __syncthreads();
    if (blk < nblk && t < T) {
        const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        for (int r = 0; r < R; ++r) {
            const bool hit = (mask >> r) & 1ull;
            const uint64_t bal = __ballot(hit);
            int slot = -1;
            if (hit) {
                slot = s_base[r] + __popcll(bal & lt);
                for (int w = 0; w < wave; ++w) slot += s_cnt[w][r];
            }
            dst_slot[static_cast<int64_t>(t) * R + r] = slot;
        }
    }
    // the totals, grid-strided: expert counts (sum of the workgroups' histograms), per-destination
    // tokens and send offsets (workgroup 0), tail blocks no count workgroup covered (zeros)
    for (int e = blk * kNotifyTok + tid; e < E; e += grid * kNotifyTok) {
        const int r = e / epr;
        notify[r * W + 1 + (e - r * epr)] = column_sum(ws_hist + e, E, nblk);
    }
    if (blk == 0) {
        __syncthreads();                                 // s_base is free again
        if (tid < R) {
            const int total = column_sum(ws_cnt + tid, R, nblk);
            s_base[tid] = total;
            notify[tid * W] = total;
        }
        __syncthreads();
        if (tid < R) {
            int before = 0;
            for (int q = 0; q < tid; ++q) before += s_base[q];
            send_offsets[tid] = before;
        }
    }
    const int covered = nblk * (kNotifyTok / 64);
    for (int i = blk * kNotifyTok + tid; i < R * nb; i += grid * kNotifyTok) {
        const int r = i / nb, bb = i - r * nb;
        if (bb >= covered) {
            notify[r * W + 1 + epr + bb] = 0;
            notify[r * W + 1 + epr + nb + bb] = 0;
        }
    }
}

// ---------------------------------------------------------------- pack: one wave per token
// packed row layout (bytes): [x | sf @sf_off | topk_idx (int64) @idx_off | weights @w_off | src @src_off]
// Row of (token t, destination r): base_r + (send_offsets[r] + dst_slot[t][r]) * row_bytes, base_r =
// dest_bases[r] (a peer's symmetric window: the xGMI transport, system-scope write-through stores,
// dispatch.cuh:373-392's push) or `packed` for every r (one local buffer for the RCCL all-to-all).
template <bool kPeer>
__device__ __forceinline__ void put16(uint8_t* row, int off, const u32x4& v, int row_bytes) {
    if constexpr (kPeer) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row, 0, row_bytes, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 17);          // sc0 sc1: system scope
    } else {
        *reinterpret_cast<u32x4*>(row + off) = v;
    }
}

template <bool kPeer, typename V>
__device__ __forceinline__ void put(V* p, V v) {
    if constexpr (kPeer) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else *p = v;
}

template <bool kPeer>
__global__ void __launch_bounds__(64)
pack_kernel(const uint8_t* __restrict__ x, int64_t x_stride, int x_bytes,
            const uint8_t* __restrict__ sf, int64_t sf_stride, int sf_bytes,
            const int64_t* __restrict__ topk_idx, const float* __restrict__ topk_weights, int K,
            int32_t src_base, const int32_t* __restrict__ dst_slot, const int32_t* __restrict__ send_offsets, int R,
            uint8_t* __restrict__ packed, const uint64_t* __restrict__ dest_bases, int64_t row_bytes,
            int64_t dest_rows, int sf_off, int idx_off, int w_off, int src_off, int32_t* __restrict__ error_flag) {
    const int t = blockIdx.x, lane = threadIdx.x;
    // the window barrier before this push timed out (bit 2): the peers may still read their
    // windows, so nothing is stored into them (the call's results are invalid and the next call raises)
    if (kPeer && error_flag != nullptr &&
        (__hip_atomic_load(error_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2))
        return;
    // lane r holds the byte address of the destination row for rank r (0: not routed to r)
    // (a row index outside the destination buffer -- offsets or slots that disagree with its size -- is
    // never stored: bit 4 and the error record instead of a write past a window)
    uint64_t my_row = 0;
    if (lane < R) {
        const int32_t s = dst_slot[static_cast<int64_t>(t) * R + lane];
        if (s >= 0) {
            const uint64_t base = kPeer ? dest_bases[lane] : reinterpret_cast<uint64_t>(packed);
            const int64_t row = static_cast<int64_t>(send_offsets[lane]) + s;
            if (row >= 0 && row < dest_rows)
                my_row = base + static_cast<uint64_t>(row) * row_bytes;
            else
                deepep::record_fault(error_flag, DEEPEP_FLAG_BAD_ADDRESS, DEEPEP_FAULT_PACK_ROW, t, lane,
                                     base + static_cast<uint64_t>(row) * row_bytes, dest_rows);
        }
    }
    const uint64_t dmask = __ballot(my_row != 0);
    auto row_of = [&](int r) -> uint8_t* {
        const uint64_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(my_row & 0xffffffffu), r));
        const uint64_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(my_row >> 32), r));
        return reinterpret_cast<uint8_t*>((hi << 32) | lo);
    };
    const u32x4* xs = reinterpret_cast<const u32x4*>(x + t * x_stride);
    for (int v = lane; v < x_bytes / 16; v += 64) {
        const u32x4 val = __builtin_nontemporal_load(xs + v);
        for (uint64_t m = dmask; m; m &= m - 1)
            put16<kPeer>(row_of(__builtin_ctzll(m)), v * 16, val, static_cast<int>(row_bytes));
    }
    for (int v = lane; v < sf_bytes / 4; v += 64) {
        const uint32_t val = reinterpret_cast<const uint32_t*>(sf + t * sf_stride)[v];
        for (uint64_t m = dmask; m; m &= m - 1)
            put<kPeer>(reinterpret_cast<uint32_t*>(row_of(__builtin_ctzll(m)) + sf_off) + v, val);
    }
    int64_t e = 0;
    float w = 0.0f;
    if (lane < K) {
        e = topk_idx[static_cast<int64_t>(t) * K + lane];
        w = topk_weights != nullptr ? topk_weights[static_cast<int64_t>(t) * K + lane] : 0.0f;
    }
    for (uint64_t m = dmask; m; m &= m - 1) {
        uint8_t* row = row_of(__builtin_ctzll(m));
        if (lane < K) {
            put<kPeer>(reinterpret_cast<int64_t*>(row + idx_off) + lane, e);
            put<kPeer>(reinterpret_cast<float*>(row + w_off) + lane, w);
        }
        if (lane == 0) put<kPeer>(reinterpret_cast<int32_t*>(row + src_off), static_cast<int32_t>(src_base + t));
    }
}

// ---------------------------------------------------------------- receive side
__device__ __forceinline__ int local_expert(int64_t e, int rank, int epr) {
    return (e >= static_cast<int64_t>(rank) * epr && e < static_cast<int64_t>(rank + 1) * epr)
               ? static_cast<int>(e - static_cast<int64_t>(rank) * epr) : -1;
}

// One thread per received row, kBlockRows rows per workgroup: metadata columns 0-1, the local top-k
// indices (non-expanded recv_topk_idx) and per-workgroup expert histograms.  N is the host's row
// count; the rows actually received are rank_psum[R - 1] (the same number after a host-synced notify;
// fewer when the host sized the launch for the worst case, dispatch(do_cpu_sync=False)).  Rows past
// the received ones get metadata -1 (and recv_topk_idx -1): the later kernels skip them.
__global__ void __launch_bounds__(kBlockRows)
count_kernel(const uint8_t* __restrict__ packed, int64_t row_bytes, int idx_off, int src_off, int N, int K,
             int rank, int epr, const int32_t* __restrict__ recv_counts, int counts_stride, int32_t* __restrict__ psum_out,
             int R, int pad_rows, int own_first, int32_t* __restrict__ row_map,
             int32_t* __restrict__ meta, int64_t* __restrict__ recv_topk_idx, int32_t* __restrict__ block_counts,
             int fill_slots) {
    extern __shared__ int32_t s_hist[];                 // [epr]
    __shared__ int32_t rank_psum[64];                   // inclusive prefix of rows per source rank
    for (int e = threadIdx.x; e < epr; e += kBlockRows) s_hist[e] = 0;
    if (threadIdx.x < R)
        rank_psum[threadIdx.x] = recv_counts[static_cast<int64_t>(threadIdx.x) * (counts_stride > 0 ? counts_stride : 1)];
    __syncthreads();
    if (counts_stride > 0) {                            // counts -> inclusive prefix (R <= 64)
        if (threadIdx.x == 0)
            for (int s = 1; s < R; ++s) rank_psum[s] += rank_psum[s - 1];
        __syncthreads();
        if (psum_out != nullptr && blockIdx.x == 0 && threadIdx.x < R) psum_out[threadIdx.x] = rank_psum[threadIdx.x];
    }
    const int i = blockIdx.x * kBlockRows + threadIdx.x;
    const int received = min(N, rank_psum[R - 1]);
    if (i >= received && i < N) {
        const int64_t mrow = static_cast<int64_t>(i) * (K + 2);
        meta[mrow] = -1;
        meta[mrow + 1] = -1;
        if (recv_topk_idx != nullptr)
            for (int k = 0; k < K; ++k) recv_topk_idx[static_cast<int64_t>(i) * K + k] = -1;
    }
    if (i < received) {
        int src_rank = 0;
        while (src_rank < R - 1 && i >= rank_psum[src_rank]) ++src_rank;
        // padded receive buffer (a worst-case-sized exchange): source s's rows start at s * pad_rows;
        // own rows first (the local bypass): [rows from this rank | rows from the others, rank order]
        const int start = src_rank > 0 ? rank_psum[src_rank - 1] : 0;
        const int own_start = rank > 0 ? rank_psum[rank - 1] : 0, own_rows = rank_psum[rank] - own_start;
        int64_t prow = i;
        if (pad_rows > 0) {
            // own first: the slots in receive order [rank, 0, .., rank - 1, rank + 1, ..]
            const int slot = !own_first ? src_rank : (src_rank == rank ? 0 : (src_rank < rank ? src_rank + 1 : src_rank));
            prow = static_cast<int64_t>(slot) * pad_rows + i - start;
        } else if (own_first) {
            prow = src_rank == rank ? i - own_start : (src_rank < rank ? i + own_rows : i);
        }
        if (row_map != nullptr) row_map[i] = static_cast<int32_t>(prow);
        const uint8_t* row = packed + prow * row_bytes;
        const int64_t* idx = reinterpret_cast<const int64_t*>(row + idx_off);
        int master = -1;
        for (int k = 0; k < K; ++k) {
            const int le = local_expert(idx[k], rank, epr);
            if (le >= 0) {
                master = k;
                atomicAdd(&s_hist[le], 1);
            }
            if (recv_topk_idx != nullptr) recv_topk_idx[static_cast<int64_t>(i) * K + k] = le;
        }
        const int64_t mrow = static_cast<int64_t>(i) * (K + 2);
        meta[mrow] = *reinterpret_cast<const int32_t*>(row + src_off);
        meta[mrow + 1] = src_rank * K + master;
    }
    if (fill_slots && i < N)                            // non-expanded: no expanded slots
        for (int k = 0; k < K; ++k) meta[static_cast<int64_t>(i) * (K + 2) + 2 + k] = -1;
    __syncthreads();
    if (blockIdx.x * kBlockRows < N)                    // (N == 0: the one workgroup formed psum_out only)
        for (int e = threadIdx.x; e < epr; e += kBlockRows)
            block_counts[static_cast<int64_t>(blockIdx.x) * epr + e] = s_hist[e];
}

// Thread (expert e, block group g) of 1024 threads: G = 1024 / epr groups of consecutive blocks, so a
// warp-row of threads reads one block's counts for consecutive experts (coalesced) and every thread walks
// ceil(nblocks / G) blocks with 16 loads in flight.  Pass 1: each group's partial count; then the experts'
// totals, a workgroup scan of the aligned totals (expert group starts aligned to expert_alignment) and the
// handle's prefix sums (elastic.py:36-45 semantics); pass 2: each block's first slot inside its expert
// group = the group start + the earlier groups' partials + a running sum over the thread's blocks.
// (Round 2 had one thread per expert walk every block: 32 busy threads and ~340 blocks at EP = 8.)
__global__ void __launch_bounds__(1024)
scan_kernel(int32_t* __restrict__ block_counts, int nblocks, int epr, int align, int expanded,
            int32_t* __restrict__ expert_counts, int32_t* __restrict__ psum_expert) {
    constexpr int kBatch = 16;
    __shared__ int32_t s_part[1024];                     // [g][e]
    __shared__ int32_t s_aligned[1024];
    const int tid = threadIdx.x;
    const int G = 1024 / epr;
    const int e = tid % epr, g = tid / epr;
    const bool active = g < G;
    const int per = (nblocks + G - 1) / G;
    const int b_lo = min(nblocks, g * per), b_hi = min(nblocks, b_lo + per);
    int part = 0;
    if (active)
        for (int b0 = b_lo; b0 < b_hi; b0 += kBatch) {
            int c[kBatch];
#pragma unroll
            for (int j = 0; j < kBatch; ++j)
                c[j] = b0 + j < b_hi ? block_counts[static_cast<int64_t>(b0 + j) * epr + e] : 0;
#pragma unroll
            for (int j = 0; j < kBatch; ++j) part += c[j];
        }
    if (active) s_part[tid] = part;
    __syncthreads();
    int total = 0;
    if (tid < epr)
        for (int q = 0; q < G; ++q) total += s_part[q * epr + tid];
    const int aligned = tid < epr ? (total + align - 1) / align * align : 0;
    s_aligned[tid] = aligned;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {          // inclusive scan of the aligned group sizes
        const int v = tid >= off ? s_aligned[tid - off] : 0;
        __syncthreads();
        s_aligned[tid] += v;
        __syncthreads();
    }
    if (tid < epr) {
        const int start = s_aligned[tid] - aligned;
        expert_counts[tid] = total;
        psum_expert[tid] = expanded ? start + total : start + aligned;
        s_aligned[tid] = start;                           // read below by every group of expert tid
    }
    __syncthreads();
    if (!active) return;
    int run = s_aligned[e];
    for (int q = 0; q < g; ++q) run += s_part[q * epr + e];
    for (int b0 = b_lo; b0 < b_hi; b0 += kBatch) {
        int c[kBatch];
#pragma unroll
        for (int j = 0; j < kBatch; ++j)
            c[j] = b0 + j < b_hi ? block_counts[static_cast<int64_t>(b0 + j) * epr + e] : 0;
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
            if (b0 + j < b_hi) block_counts[static_cast<int64_t>(b0 + j) * epr + e] = run;
            run += c[j];
        }
    }
}

// Expanded slot of every (row, local lane): the expert group's offset for this workgroup plus the
// number of earlier rows of the workgroup holding the same expert (per-wave 64-bit ballot masks in
// LDS).  A token never holds one expert twice, so this is the ascending-token order.  Rows whose
// metadata count_kernel marked -1 (past the received rows) get no slots.  inv (optional): the inverse
// map, inv[slot] = row * K + lane, read by the expanded copy.
constexpr int kSlotWaves = kBlockRows / 64;

__global__ void __launch_bounds__(kBlockRows)
slots_kernel(const uint8_t* __restrict__ packed, int64_t row_bytes, int idx_off, int N, int K, int rank, int epr,
             const int32_t* __restrict__ block_offsets, int32_t* __restrict__ meta, int32_t* __restrict__ inv,
             const int32_t* __restrict__ row_map) {
    extern __shared__ uint64_t s_bits[];                // [epr][kSlotWaves]
    for (int j = threadIdx.x; j < epr * kSlotWaves; j += kBlockRows) s_bits[j] = 0ull;
    __syncthreads();
    const int i = blockIdx.x * kBlockRows + threadIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool valid = i < N && meta[static_cast<int64_t>(i) * (K + 2)] >= 0;
    const int64_t prow = valid && row_map != nullptr ? row_map[i] : i;
    const int64_t* idx = reinterpret_cast<const int64_t*>(packed + prow * row_bytes + idx_off);
    if (valid)
        for (int k = 0; k < K; ++k) {
            const int le = local_expert(idx[k], rank, epr);
            if (le >= 0) atomicOr(reinterpret_cast<unsigned long long*>(&s_bits[le * kSlotWaves + wave]), 1ull << lane);
        }
    __syncthreads();
    if (i >= N) return;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int k = 0; k < K; ++k) {
        const int le = valid ? local_expert(idx[k], rank, epr) : -1;
        int slot = -1;
        if (le >= 0) {
            slot = block_offsets[static_cast<int64_t>(blockIdx.x) * epr + le];
            for (int w = 0; w < wave; ++w) slot += __popcll(s_bits[le * kSlotWaves + w]);
            slot += __popcll(s_bits[le * kSlotWaves + wave] & lt);
            if (inv != nullptr) inv[slot] = i * K + k;
        }
        meta[static_cast<int64_t>(i) * (K + 2) + 2 + k] = slot;
    }
}

// x (and sf) of received row i to recv_x[i] (non-expanded) or to every local slot (expanded);
// weights to recv_topk_weights[i][k] or [slot].  Work item = (row, 2 KiB column chunk): one wave
// per item, 4 items per 256-thread workgroup (the combine kernel's tiling, mirrored: one load, up
// to K stores per lane and vector).  The x rows come from the packed receive row, or -- one rank,
// nothing exchanged -- straight from the sender's x / sf (x_direct: row = src_global_idx %
// num_max_tokens), so x is read once.  Row stores are write-through buffer stores (sc1).
__global__ void __launch_bounds__(256)
copy_kernel(const uint8_t* __restrict__ packed, int64_t row_bytes, int x_bytes, int sf_off, int sf_bytes, int w_off,
            int N, int K, const int32_t* __restrict__ meta, int expanded,
            const uint8_t* __restrict__ x_direct, int64_t x_direct_stride,
            const uint8_t* __restrict__ sf_direct, int64_t sf_direct_stride, int num_max_tokens,
            uint8_t* __restrict__ recv_x, uint8_t* __restrict__ recv_sf, float* __restrict__ recv_w,
            int64_t num_out_rows, const int32_t* __restrict__ row_map, int32_t* __restrict__ error_flag) {
    constexpr int kChunkVecs = 128;                        // 64 lanes x 2 x 16 B
    const int lane = threadIdx.x & 63;
    // a timed-out window barrier (bit 2): the received rows are not trustworthy, store nothing
    if (error_flag != nullptr && (__hip_atomic_load(error_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2))
        return;
    const int nvec = x_bytes / 16;
    const int nchunks = max(1, (nvec + kChunkVecs - 1) / kChunkVecs);
    const int64_t it = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (it >= static_cast<int64_t>(N) * nchunks) return;
    const int64_t i = it / nchunks;
    const int c = static_cast<int>(it - i * nchunks);
    if (meta[i * (K + 2)] < 0) return;                     // past the received rows (count_kernel)
    const uint8_t* row = packed + (row_map != nullptr ? static_cast<int64_t>(row_map[i]) : i) * row_bytes;
    const uint8_t* xs = row;
    const uint8_t* sfs = row + sf_off;
    if (x_direct != nullptr) {
        const int64_t t = meta[i * (K + 2)] % num_max_tokens;
        xs = x_direct + t * x_direct_stride;
        sfs = sf_direct != nullptr ? sf_direct + t * sf_direct_stride : nullptr;
    }
    // lane k holds the destination row of lane k's slot (expanded) or lane 0 holds i
    int32_t my_dst = -1;
    if (expanded) {
        if (lane < K) my_dst = meta[i * (K + 2) + 2 + lane];
    } else if (lane == 0) {
        my_dst = static_cast<int32_t>(i);
    }
    if (my_dst >= num_out_rows) {                          // never store past the outputs
        if (error_flag != nullptr) atomicOr(error_flag, 1);
        my_dst = -1;
    }
    const uint64_t dmask = __ballot(my_dst >= 0);
    const int v0 = c * kChunkVecs + lane, v1 = v0 + 64;
    const u32x4 zero = {0u, 0u, 0u, 0u};
    const u32x4 a0 = v0 < nvec ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(xs) + v0) : zero;
    const u32x4 a1 = v1 < nvec ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(xs) + v1) : zero;
    for (uint64_t m = dmask; m; m &= m - 1) {
        const int64_t d = __builtin_amdgcn_readlane(my_dst, __builtin_ctzll(m));
        // the descriptor's range check drops the lanes past the row end
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(recv_x + d * x_bytes, 0, x_bytes,
                                                                            0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(a0, rs, v0 * 16, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(a1, rs, v1 * 16, 0, 16);
    }
    if (c != 0) return;
    if (recv_sf != nullptr && sfs != nullptr)
        for (int v = lane; v < sf_bytes / 4; v += 64) {
            const uint32_t val = reinterpret_cast<const uint32_t*>(sfs)[v];
            for (uint64_t m = dmask; m; m &= m - 1) {
                const int64_t d = __builtin_amdgcn_readlane(my_dst, __builtin_ctzll(m));
                reinterpret_cast<uint32_t*>(recv_sf + d * sf_bytes)[v] = val;
            }
        }
    if (recv_w != nullptr && lane < K) {
        const float w = reinterpret_cast<const float*>(row + w_off)[lane];
        if (expanded) {
            if (my_dst >= 0) recv_w[my_dst] = w;
        } else {
            recv_w[i * K + lane] = w;
        }
    }
}

// Expanded copy, destination-major inside blocks of received rows.  The rows of
// block b (kBlockRows received rows) that go to local expert e are the consecutive expanded rows
// [block_offsets[b][e], block_offsets[b + 1][e]) (the slots kernel numbers them in row order), so one
// wave per (block, expert, 2 KiB column chunk) writes a run of whole consecutive destination rows
// and reads their sources through inv.  The block's source rows (1.8 MB) are read once from HBM and
// re-read -- once per local expert of each row -- from the L2 of the one XCD that owns the block
// (workgroups w = x (mod 8) run on XCD x and take blocks x, x + 8, ...).  Stores are streaming
// write-through (sc1 nt).  Measured at BASELINE config 2 (round-3 probe, CHANGELOG.md; two boxes): 151.4 vs
// 163.5 us and 182.0 vs 213.6 us for the source-major copy (one load, up to K scattered stores).
constexpr int kCopyAux = 18;                          // sc1 | nt

template <bool kDirect>
__global__ void __launch_bounds__(256)
copy_expanded_kernel(const uint8_t* __restrict__ packed, int64_t row_bytes, int x_bytes, int sf_off, int sf_bytes,
                     int w_off, int N, int K, const int32_t* __restrict__ meta,
                     const uint8_t* __restrict__ x_direct, int64_t x_direct_stride,
                     const uint8_t* __restrict__ sf_direct, int64_t sf_direct_stride, int num_max_tokens,
                     const int32_t* __restrict__ inv, const int32_t* __restrict__ block_offsets,
                     const int32_t* __restrict__ expert_end, int nb, int epr,
                     uint8_t* __restrict__ recv_x, uint8_t* __restrict__ recv_sf, float* __restrict__ recv_w,
                     int64_t num_out_rows, const int32_t* __restrict__ row_map, int32_t* __restrict__ error_flag) {
    constexpr int kChunkVecs = 128;                        // 64 lanes x 2 x 16 B
    constexpr int kRows = 4;                               // destination rows in flight per wave
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (error_flag != nullptr && (__hip_atomic_load(error_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2))
        return;                                            // a timed-out window barrier: store nothing
    const int nvec = x_bytes / 16;
    const int nch = max(1, (nvec + kChunkVecs - 1) / kChunkVecs);
    const int64_t wg_per_block = (static_cast<int64_t>(epr) * nch + 3) / 4;
    const int64_t xcd = blockIdx.x % 8, kk = blockIdx.x / 8;
    const int64_t b = xcd + 8 * (kk / wg_per_block);
    const int64_t it = (kk % wg_per_block) * 4 + wave;
    const int e = static_cast<int>(it / nch), c = static_cast<int>(it - static_cast<int64_t>(e) * nch);
    if (b >= nb || e >= epr) return;
    const int r0 = block_offsets[b * epr + e];
    const int r1 = b + 1 < nb ? block_offsets[(b + 1) * epr + e] : expert_end[e];
    const int v0 = c * kChunkVecs + lane, v1 = v0 + 64;
    const u32x4 zero = {0u, 0u, 0u, 0u};
    for (int j = r0; j < r1; j += kRows) {
        const uint8_t* rows[kRows];
        int32_t src_i[kRows], src_k[kRows];
        u32x4 a[kRows][2];
#pragma unroll
        for (int q = 0; q < kRows; ++q) {
            src_i[q] = -1;
            src_k[q] = 0;
            rows[q] = nullptr;
            if (j + q < r1) {
                const int32_t code = __builtin_amdgcn_readfirstlane(inv[j + q]);
                const int32_t i = code >= 0 ? code / K : -1;
                if (i >= 0 && i < N) {
                    src_i[q] = i;
                    src_k[q] = code - i * K;
                    if constexpr (kDirect) {
                        const int64_t t = meta[static_cast<int64_t>(i) * (K + 2)] % num_max_tokens;
                        rows[q] = x_direct + t * x_direct_stride;
                    } else {
                        rows[q] = packed + (row_map != nullptr ? static_cast<int64_t>(row_map[i]) : i) * row_bytes;
                    }
                    const u32x4* xs = reinterpret_cast<const u32x4*>(rows[q]);
                    a[q][0] = v0 < nvec ? xs[v0] : zero;
                    a[q][1] = v1 < nvec ? xs[v1] : zero;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < kRows; ++q) {
            if (src_i[q] < 0) continue;
            const int64_t d = j + q;
            if (d >= num_out_rows) {                       // never store past the outputs
                if (lane == 0 && error_flag != nullptr) atomicOr(error_flag, 1);
                continue;
            }
            // the descriptor's range check drops the lanes past the row end
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(recv_x + d * x_bytes, 0, x_bytes,
                                                                                0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(a[q][0], rs, v0 * 16, 0, kCopyAux);
            __builtin_amdgcn_raw_buffer_store_b128(a[q][1], rs, v1 * 16, 0, kCopyAux);
            if (c != 0) continue;
            if (recv_sf != nullptr) {
                const uint8_t* sfs;
                if constexpr (kDirect) {
                    const int64_t t = meta[static_cast<int64_t>(src_i[q]) * (K + 2)] % num_max_tokens;
                    sfs = sf_direct != nullptr ? sf_direct + t * sf_direct_stride : nullptr;
                } else {
                    sfs = rows[q] + sf_off;
                }
                if (sfs != nullptr)
                    for (int v = lane; v < sf_bytes / 4; v += 64)
                        reinterpret_cast<uint32_t*>(recv_sf + d * sf_bytes)[v] = reinterpret_cast<const uint32_t*>(sfs)[v];
            }
            if (recv_w != nullptr && lane == 0) {
                const int64_t prow = row_map != nullptr ? static_cast<int64_t>(row_map[src_i[q]]) : src_i[q];
                recv_w[d] = reinterpret_cast<const float*>(packed + prow * row_bytes + w_off)[src_k[q]];
            }
        }
    }
}

int launch_status(const char* what) {
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        char buf[256];
        snprintf(buf, sizeof(buf), "%s launch failed: %s", what, hipGetErrorString(err));
        return deepep_amd_set_error(DEEPEP_ERR_HIP, buf);
    }
    return DEEPEP_OK;
}

bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

extern "C" {

int deepep_dispatch_route(const int64_t* topk_idx, int num_tokens, int num_topk, int num_experts, int num_ranks,
                          int32_t* dst_slot, int32_t* send_counts, int32_t* block_counts, deepep_stream_t stream) {
    if (num_tokens < 0 || num_topk < 1 || num_topk > 32 || num_ranks < 1 || num_ranks > 64 ||
        num_experts % num_ranks != 0 || send_counts == nullptr ||
        (num_tokens > 0 && (dst_slot == nullptr || topk_idx == nullptr || block_counts == nullptr)))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "dispatch_route: invalid arguments");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (num_tokens == 0) {
        const hipError_t e = hipMemsetAsync(send_counts, 0, sizeof(int32_t) * num_ranks, s);
        return e == hipSuccess ? DEEPEP_OK : launch_status("dispatch_route memset");
    }
    const int nb = (num_tokens + 255) / 256;
    const int epr = num_experts / num_ranks;
    hipLaunchKernelGGL(route_count_kernel, dim3(nb), dim3(256), 0, s, topk_idx, num_tokens, num_topk, epr, num_ranks,
                       block_counts);
    hipLaunchKernelGGL(route_assign_kernel, dim3(nb), dim3(256), 0, s, topk_idx, num_tokens, num_topk, epr, num_ranks,
                       block_counts, dst_slot, send_counts);
    return launch_status("dispatch_route");
}

int64_t deepep_dispatch_notify_workspace(int num_tokens, int num_experts, int num_ranks) {
    const int64_t nblk = (static_cast<int64_t>(std::max(num_tokens, 0)) + kNotifyTok - 1) / kNotifyTok;
    return nblk * (num_ranks + num_experts) * 4;
}

int deepep_dispatch_notify(const int64_t* topk_idx, int num_tokens, int num_topk, int num_experts, int num_ranks,
                           int num_blocks, int32_t* dst_slot, int32_t* notify, int32_t* send_offsets,
                           void* workspace, int64_t workspace_bytes, deepep_stream_t stream) {
    if (num_tokens < 0 || num_topk < 1 || num_topk > 32 || num_ranks < 1 || num_ranks > 64 ||
        num_experts < num_ranks || num_experts % num_ranks != 0 || num_experts > 32768 ||
        num_blocks < 0 || (num_ranks > 1 && num_blocks < (num_tokens + 63) / 64) ||
        notify == nullptr || send_offsets == nullptr || (num_tokens > 0 && (dst_slot == nullptr || topk_idx == nullptr)) ||
        workspace_bytes < deepep_dispatch_notify_workspace(num_tokens, num_experts, num_ranks) ||
        (num_tokens > 0 && workspace == nullptr))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "dispatch_notify: invalid arguments");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int nblk = (num_tokens + kNotifyTok - 1) / kNotifyTok;
    int32_t* ws_cnt = static_cast<int32_t*>(workspace);
    int32_t* ws_hist = ws_cnt + static_cast<int64_t>(nblk) * num_ranks;
    if (nblk > 0)
        hipLaunchKernelGGL(notify_count_kernel, dim3(nblk), dim3(kNotifyTok), static_cast<size_t>(num_experts) * 4, s,
                           topk_idx, num_tokens, num_topk, num_experts, num_ranks, num_blocks, notify, ws_cnt, ws_hist);
    hipLaunchKernelGGL(notify_assign_kernel, dim3(std::max(nblk, 1)), dim3(kNotifyTok), 0, s, topk_idx, num_tokens,
                       num_topk, num_experts, num_ranks, num_blocks, nblk, ws_cnt, ws_hist, dst_slot, notify,
                       send_offsets);
    return launch_status("dispatch_notify");
}

int deepep_dispatch_expert_counts(const int64_t* topk_idx, int num_tokens, int num_topk, int num_experts,
                                  int32_t* counts, deepep_stream_t stream) {
    if (num_tokens < 0 || num_topk < 1 || num_topk > 32 || num_experts < 1 || num_experts > 32768 ||
        counts == nullptr || (num_tokens > 0 && topk_idx == nullptr))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "dispatch_expert_counts: invalid arguments");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const hipError_t e = hipMemsetAsync(counts, 0, sizeof(int32_t) * num_experts, s);
    if (e != hipSuccess) return launch_status("dispatch_expert_counts memset");
    const int64_t n = static_cast<int64_t>(num_tokens) * num_topk;
    if (n > 0)
        hipLaunchKernelGGL(expert_hist_kernel, dim3(static_cast<unsigned>((n + kHistEntries - 1) / kHistEntries)),
                           dim3(256), num_experts * 4, s, topk_idx, n, num_experts, counts);
    return launch_status("dispatch_expert_counts");
}

int deepep_dispatch_pack(const void* x, int64_t x_row_stride_bytes, int x_bytes,
                         const void* sf, int64_t sf_row_stride_bytes, int sf_bytes,
                         const int64_t* topk_idx, const float* topk_weights, int num_tokens, int num_topk,
                         int32_t src_base, const int32_t* dst_slot, const int32_t* send_offsets, int num_ranks,
                         void* packed, const uint64_t* dest_bases, int64_t row_bytes, int64_t dest_rows,
                         int sf_off, int idx_off, int w_off, int src_off, int32_t* error_flag,
                         deepep_stream_t stream) {
    if (num_tokens == 0) return DEEPEP_OK;
    if (num_tokens < 0 || num_topk < 1 || num_topk > 32 || num_ranks < 1 || num_ranks > 64 || x_bytes % 16 ||
        dest_rows < 0 || row_bytes < src_off + 4 ||
        sf_bytes % 4 || row_bytes % 16 || !a16(x) || (dest_bases == nullptr && !a16(packed)) ||
        x_row_stride_bytes % 16 || idx_off % 8 || w_off % 4 || src_off % 4 || (sf_bytes > 0 && sf == nullptr) ||
        (dest_bases == nullptr && packed == nullptr))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "dispatch_pack: invalid arguments or alignment");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (dest_bases != nullptr)
        hipLaunchKernelGGL(pack_kernel<true>, dim3(num_tokens), dim3(64), 0, s,
                           static_cast<const uint8_t*>(x), x_row_stride_bytes, x_bytes,
                           static_cast<const uint8_t*>(sf), sf_row_stride_bytes, sf_bytes,
                           topk_idx, topk_weights, num_topk, src_base, dst_slot, send_offsets, num_ranks,
                           static_cast<uint8_t*>(packed), dest_bases, row_bytes, dest_rows, sf_off, idx_off, w_off, src_off,
                           error_flag);
    else
        hipLaunchKernelGGL(pack_kernel<false>, dim3(num_tokens), dim3(64), 0, s,
                           static_cast<const uint8_t*>(x), x_row_stride_bytes, x_bytes,
                           static_cast<const uint8_t*>(sf), sf_row_stride_bytes, sf_bytes,
                           topk_idx, topk_weights, num_topk, src_base, dst_slot, send_offsets, num_ranks,
                           static_cast<uint8_t*>(packed), dest_bases, row_bytes, dest_rows, sf_off, idx_off, w_off, src_off,
                           error_flag);
    return launch_status("dispatch_pack");
}

int deepep_dispatch_count(const void* packed, int64_t row_bytes, int idx_off, int src_off, int num_recv, int num_topk,
                          int rank, int num_local_experts, const int32_t* recv_rank_psum, int num_ranks,
                          int recv_counts_stride, int32_t* psum_out, int pad_rows, int own_first, int32_t* row_map,
                          int32_t* src_metadata, int64_t* recv_topk_idx, int32_t* block_counts,
                          deepep_stream_t stream) {
    // a rank that receives nothing: no rows, but one workgroup still forms psum_out
    if (num_recv == 0 && (psum_out == nullptr || recv_counts_stride == 0)) return DEEPEP_OK;
    if (num_recv < 0 || num_topk < 1 || num_topk > 32 || num_local_experts < 1 || num_local_experts > 1024 ||
        num_ranks < 1 || num_ranks > 64 || recv_counts_stride < 0 || rank < 0 || rank >= num_ranks ||
        (num_recv > 0 && (src_metadata == nullptr || block_counts == nullptr || packed == nullptr)) ||
        recv_rank_psum == nullptr || pad_rows < 0 || (num_recv > 0 && (pad_rows > 0 || own_first) && row_map == nullptr) ||
        static_cast<int64_t>(pad_rows) * num_ranks >= (int64_t(1) << 31))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "dispatch_count: invalid arguments");
    const int nblocks = std::max(1, (num_recv + kBlockRows - 1) / kBlockRows);
    hipLaunchKernelGGL(count_kernel, dim3(nblocks), dim3(kBlockRows), num_local_experts * 4,
                       reinterpret_cast<hipStream_t>(stream), static_cast<const uint8_t*>(packed), row_bytes,
                       idx_off, src_off, num_recv, num_topk, rank, num_local_experts, recv_rank_psum,
                       recv_counts_stride, psum_out, num_ranks, pad_rows, own_first ? 1 : 0, row_map, src_metadata,
                       recv_topk_idx, block_counts, 0);
    return launch_status("dispatch_count");
}

int deepep_dispatch_receive(const void* packed, int64_t row_bytes, int idx_off, int src_off, int num_recv,
                            int num_topk, int rank, int num_local_experts, const int32_t* recv_counts,
                            int num_ranks, int recv_counts_stride, int32_t* psum_out, int pad_rows, int own_first,
                            int32_t* row_map, int32_t* src_metadata, int64_t* recv_topk_idx, int32_t* block_counts,
                            int expert_alignment, int expanded, int32_t* expert_counts, int32_t* psum_expert,
                            int32_t* inv, deepep_stream_t stream) {
    if (num_recv < 0 || num_topk < 1 || num_topk > 32 || num_local_experts < 1 || num_local_experts > 1024 ||
        num_ranks < 1 || num_ranks > 64 || recv_counts_stride < 1 || recv_counts == nullptr || psum_out == nullptr ||
        rank < 0 || rank >= num_ranks ||
        (num_recv > 0 && (src_metadata == nullptr || block_counts == nullptr || packed == nullptr)) ||
        pad_rows < 0 || (num_recv > 0 && (pad_rows > 0 || own_first) && row_map == nullptr) ||
        static_cast<int64_t>(pad_rows) * num_ranks >= (int64_t(1) << 31) || expert_alignment < 1 ||
        expert_counts == nullptr || psum_expert == nullptr ||
        static_cast<int64_t>(num_recv) * num_topk >= (int64_t(1) << 31))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "dispatch_receive: invalid arguments");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int nblocks = (num_recv + kBlockRows - 1) / kBlockRows;
    hipLaunchKernelGGL(count_kernel, dim3(std::max(nblocks, 1)), dim3(kBlockRows), num_local_experts * 4, s,
                       static_cast<const uint8_t*>(packed), row_bytes, idx_off, src_off, num_recv, num_topk, rank,
                       num_local_experts, recv_counts, recv_counts_stride, psum_out, num_ranks, pad_rows,
                       own_first ? 1 : 0, row_map, src_metadata, recv_topk_idx, block_counts, expanded ? 0 : 1);
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, s, block_counts, nblocks, num_local_experts,
                       expert_alignment, expanded, expert_counts, psum_expert);
    if (expanded && nblocks > 0)
        hipLaunchKernelGGL(slots_kernel, dim3(nblocks), dim3(kBlockRows), num_local_experts * kSlotWaves * 8, s,
                           static_cast<const uint8_t*>(packed), row_bytes, idx_off, num_recv, num_topk, rank,
                           num_local_experts, block_counts, src_metadata, inv, row_map);
    return launch_status("dispatch_receive");
}

int deepep_dispatch_scan(int32_t* block_counts, int num_blocks, int num_local_experts, int expert_alignment,
                         int expanded, int32_t* expert_counts, int32_t* psum_expert, deepep_stream_t stream) {
    if (num_blocks < 0 || num_local_experts < 1 || num_local_experts > 1024 || expert_alignment < 1 ||
        expert_counts == nullptr || psum_expert == nullptr || (num_blocks > 0 && block_counts == nullptr))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "dispatch_scan: invalid arguments");
    hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream),
                       block_counts, num_blocks, num_local_experts, expert_alignment, expanded,
                       expert_counts, psum_expert);
    return launch_status("dispatch_scan");
}

int deepep_dispatch_slots(const void* packed, int64_t row_bytes, int idx_off, int num_recv, int num_topk,
                          int rank, int num_local_experts, const int32_t* block_offsets, int32_t* src_metadata,
                          int32_t* inv, const int32_t* row_map, deepep_stream_t stream) {
    if (num_recv == 0) return DEEPEP_OK;
    if (num_recv < 0 || num_topk < 1 || num_topk > 32 || num_local_experts < 1 || num_local_experts > 1024 ||
        packed == nullptr || block_offsets == nullptr || src_metadata == nullptr ||
        static_cast<int64_t>(num_recv) * num_topk >= (int64_t(1) << 31))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "dispatch_slots: invalid arguments");
    const int nblocks = (num_recv + kBlockRows - 1) / kBlockRows;
    hipLaunchKernelGGL(slots_kernel, dim3(nblocks), dim3(kBlockRows), num_local_experts * kSlotWaves * 8,
                       reinterpret_cast<hipStream_t>(stream), static_cast<const uint8_t*>(packed), row_bytes,
                       idx_off, num_recv, num_topk, rank, num_local_experts, block_offsets, src_metadata, inv,
                       row_map);
    return launch_status("dispatch_slots");
}

int deepep_dispatch_copy(const void* packed, int64_t row_bytes, int x_bytes, int sf_off, int sf_bytes, int w_off,
                         int num_recv, int num_topk, const int32_t* src_metadata, int expanded,
                         const void* x_direct, int64_t x_direct_stride_bytes,
                         const void* sf_direct, int64_t sf_direct_stride_bytes, int num_max_tokens,
                         void* recv_x, void* recv_sf, float* recv_topk_weights, int64_t num_out_rows,
                         const int32_t* inv, const int32_t* block_offsets, const int32_t* expert_end,
                         int num_local_experts, const int32_t* row_map, int32_t* error_flag, deepep_stream_t stream) {
    if (num_recv == 0) return DEEPEP_OK;
    if (num_recv < 0 || num_topk < 1 || num_topk > 32 || x_bytes % 16 || row_bytes % 16 || !a16(packed) ||
        num_out_rows < 0 ||
        !a16(recv_x) || (recv_sf != nullptr && sf_bytes % 4) || src_metadata == nullptr ||
        (x_direct != nullptr && (!a16(x_direct) || x_direct_stride_bytes % 16 || num_max_tokens < 1 ||
                                 (recv_sf != nullptr && sf_direct == nullptr))) ||
        (inv != nullptr && (!expanded || block_offsets == nullptr || expert_end == nullptr || num_local_experts < 1 ||
                            num_local_experts > 1024)))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "dispatch_copy: invalid arguments or alignment");
    if (inv != nullptr) {
        // the blocked destination-major copy (expanded layout)
        const int nb = (num_recv + kBlockRows - 1) / kBlockRows;
        const int nch = std::max(1, (x_bytes / 16 + 127) / 128);
        const int64_t wg_per_block = (static_cast<int64_t>(num_local_experts) * nch + 3) / 4;
        const int64_t grid = 8 * wg_per_block * ((nb + 7) / 8);
        auto launch = [&](auto kernel) {
            hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0,
                               reinterpret_cast<hipStream_t>(stream),
                               static_cast<const uint8_t*>(packed), row_bytes, x_bytes, sf_off, sf_bytes, w_off,
                               num_recv, num_topk, src_metadata, static_cast<const uint8_t*>(x_direct),
                               x_direct_stride_bytes, static_cast<const uint8_t*>(sf_direct), sf_direct_stride_bytes,
                               num_max_tokens, inv, block_offsets, expert_end, nb, num_local_experts,
                               static_cast<uint8_t*>(recv_x), static_cast<uint8_t*>(recv_sf), recv_topk_weights,
                               num_out_rows, row_map, error_flag);
        };
        if (x_direct != nullptr) launch(copy_expanded_kernel<true>);
        else launch(copy_expanded_kernel<false>);
        return launch_status("dispatch_copy");
    }
    const int64_t nchunks = std::max<int64_t>(1, (x_bytes / 16 + 127) / 128);
    const int64_t items = static_cast<int64_t>(num_recv) * nchunks;
    hipLaunchKernelGGL(copy_kernel, dim3(static_cast<unsigned>((items + 3) / 4)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream),
                       static_cast<const uint8_t*>(packed), row_bytes, x_bytes, sf_off, sf_bytes, w_off,
                       num_recv, num_topk, src_metadata, expanded,
                       static_cast<const uint8_t*>(x_direct), x_direct_stride_bytes,
                       static_cast<const uint8_t*>(sf_direct), sf_direct_stride_bytes, num_max_tokens,
                       static_cast<uint8_t*>(recv_x), static_cast<uint8_t*>(recv_sf), recv_topk_weights,
                       num_out_rows, row_map, error_flag);
    return launch_status("dispatch_copy");
}

}  // extern "C"
