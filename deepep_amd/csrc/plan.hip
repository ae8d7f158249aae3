// plan.hip -- the EP > 1 combine plan, built on the device (gfx950), with no host synchronisation.
//
// The reference's combine re-derives its addressing inside every launch: combine_impl walks
// recv_src_metadata to find each partial's owner row (deep_ep/include/deep_ep/impls/combine.cuh:96-106)
// and combine_reduce_epilogue_impl walks topk_idx, deduplicating ranks by their highest top-k lane
// (combine_reduce_epilogue.cuh:62-95, common/ptx.cuh:412-421).  This build splits the EP > 1 combine
// into source-token chunks (pipelined exchange) and materialises that addressing
// once per handle as small int32 tables.  Everything here is computed from device data: the handle's
// metadata / routing and the per-64-token-block counts the dispatch's notify already carries (its one
// host sync also gave the host the same counts, which size the exchange), so a first combine on a
// fresh handle issues kernels only -- it can run under torch.cuda.set_sync_debug_mode("error") and be
// captured into a HIP graph.
//
// Counting unit: a block = 64 consecutive tokens of a source rank (one wave).  A pipeline chunk is a
// whole number of blocks, so every chunk's exchange sizes are sums of block counts.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>
#include <stdio.h>

#include "../../include/deepep_amd.h"
#include "fault.h"

extern "C" __attribute__((visibility("hidden"))) int deepep_amd_set_error(int code, const char* msg);

namespace {

constexpr int kBlk = DEEPEP_PLAN_BLOCK_TOKENS;      // 64 tokens = one wave
constexpr int kMaxRanks = 64;
constexpr int kMaxTopk = 32;

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int n = __shfl_up(v, off, 64);
        if (lane >= off) v += n;
    }
    return v;
}

__device__ __forceinline__ int rank_of_expert(int64_t e, int epr) { return e >= 0 ? static_cast<int>(e / epr) : -1; }

// ---------------------------------------------------------------- block counts (notify)
// tok[r][b] = tokens of block b routed to rank r, pairs[r][b] = (token, lane) entries routed to r.
__global__ void __launch_bounds__(64)
block_counts_kernel(const int64_t* __restrict__ topk_idx, int T, int K, int epr, int R, int nb,
                    int32_t* __restrict__ tok, int32_t* __restrict__ pairs) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const int t = b * kBlk + lane;
    int rk[kMaxTopk];
#pragma unroll
    for (int k = 0; k < kMaxTopk; ++k)
        rk[k] = (t < T && k < K) ? rank_of_expert(topk_idx[static_cast<int64_t>(t) * K + k], epr) : -1;
    for (int r = 0; r < R; ++r) {
        int c = 0;
#pragma unroll
        for (int k = 0; k < kMaxTopk; ++k) c += rk[k] == r;
        const int ntok = __popcll(__ballot(c > 0));
        const int npair = wave_sum(c);
        if (lane == 0) {
            tok[static_cast<int64_t>(r) * nb + b] = ntok;
            pairs[static_cast<int64_t>(r) * nb + b] = npair;
        }
    }
}

// Order of the peer groups inside a chunk's rows.  Without the local bypass: rank order.  With it
// (DEEPEP_PLAN_LOCAL_BYPASS, the RCCL transport): the expert side puts its own rank's units last -- the
// send rows of the other ranks stay one contiguous, rank-ordered all-to-all input with a zero diagonal
// split, and the own units land right after them -- and the source side puts the rows of its own rank
// first, followed by the all-to-all output in rank order; the two layouts meet in one allocation
// [send rows | own rows | received rows], so phase B reads the own partials where phase A wrote them
// (the reference's own-slot store is local too, combine.cuh:96-101).
__device__ __forceinline__ int send_order(int l, int rank, int R, bool bypass) {
    return !bypass ? l : (l == rank ? R - 1 : (l > rank ? l - 1 : l));
}
__device__ __forceinline__ int recv_order(int l, int rank, bool bypass) {
    return !bypass ? l : (l == rank ? 0 : (l < rank ? l + 1 : l));
}

// ---------------------------------------------------------------- expert side
// One wave per segment (source rank s, block b): the received rows of s's tokens [64 b, 64 b + 64),
// contiguous in receive order (grouped by source rank, ascending token).  Unit order inside chunk c:
// grouped by source rank in send_order (the RCCL send buffer), or round-robin over the source ranks
// (interleave: the xGMI stores then reach every peer at once) -- unit p of source s goes to position
// sum_{s'} min(n_{s'}, p + [s' < s]), the stable sort of (p * R + s).
__global__ void __launch_bounds__(64)
plan_expert_kernel(const int32_t* __restrict__ meta, int num_recv, int K, int R, int rank, int t_max,
                   const int32_t* __restrict__ recv_tok, const int32_t* __restrict__ recv_pairs, int nb, int bpc,
                   int flags, int32_t* __restrict__ table_a, int32_t* __restrict__ wtable_a,
                   const uint64_t* __restrict__ bases, int64_t row_bytes, int64_t window_bytes,
                   uint64_t* __restrict__ out_rows, int32_t* __restrict__ err, int padded) {
    __shared__ int s_n[kMaxRanks];
    const int lane = threadIdx.x;
    const int s = blockIdx.x / nb, b = blockIdx.x - s * nb;
    const int seg_len = recv_tok[static_cast<int64_t>(s) * nb + b];
    if (seg_len == 0) return;                                   // wave-uniform
    const bool single = flags & DEEPEP_PLAN_SINGLE, expanded = flags & DEEPEP_PLAN_EXPANDED;
    const bool interleave = flags & DEEPEP_PLAN_INTERLEAVE, rank_layout = flags & DEEPEP_PLAN_RANK_LAYOUT;
    const bool bypass = (flags & DEEPEP_PLAN_LOCAL_BYPASS) && !interleave;
    const int32_t* cnt = single ? recv_pairs : recv_tok;
    const int cb0 = (b / bpc) * bpc, cb1 = min(cb0 + bpc, nb);
    // lane l < R: rows received from l (all blocks), units of l before the chunk, units of l in it
    int rows_l = 0, before_l = 0, n_l = 0, rows_s_before = 0, p0 = 0;
    if (lane < R) {
        const int32_t* tl = recv_tok + static_cast<int64_t>(lane) * nb;
        const int32_t* cl = cnt + static_cast<int64_t>(lane) * nb;
        for (int j = 0; j < nb; ++j) rows_l += tl[j];
        for (int j = 0; j < cb0; ++j) before_l += cl[j];
        for (int j = cb0; j < cb1; ++j) n_l += cl[j];
        if (lane == s) {
            for (int j = 0; j < b; ++j) rows_s_before += tl[j];
            for (int j = cb0; j < b; ++j) p0 += cl[j];
        }
        s_n[lane] = n_l;
    }
    __syncthreads();
    const int seg_row0 = wave_sum(lane < s ? rows_l : 0) + __shfl(rows_s_before, s, 64);
    // padded (a sync-free dispatch's handle: the host knows no counts): every chunk holds R x `padded`
    // unit positions, source s's units at s * padded + p (or p * R + s interleaved); positions past a
    // source's count stay the caller's fill and are skipped
    const int chunk_base = padded > 0 ? (b / bpc) * R * padded : wave_sum(before_l);
    const int chunk_units = padded > 0 ? R * padded : wave_sum(n_l);     // units of the whole chunk
    const int os = send_order(s, rank, R, bypass);
    const int grouped_base = padded > 0 ? os * padded
                                        : wave_sum(lane < R && send_order(lane, rank, R, bypass) < os ? n_l : 0);
    p0 = __shfl(p0, s, 64);
    auto position = [&](int p) -> int {                         // unit p of source s inside the chunk
        if (padded > 0) return interleave ? p * R + s : grouped_base + p;
        if (!interleave) return grouped_base + p;
        int pos = 0;
        for (int l = 0; l < R; ++l) pos += min(s_n[l], p + (l < s ? 1 : 0));
        return pos;
    };
    const int i = seg_row0 + lane;                              // this lane's received row
    // counts that disagree with the metadata (a row past the received ones) write nothing for the lane:
    // its units keep the caller's -1 / 0 fill and are skipped by phase A.  The lane stays in the wave
    // (the single reduction's scan below needs every lane).
    const bool past_recv = lane < seg_len && i >= num_recv;
    if (past_recv) deepep::record_fault(err, DEEPEP_FLAG_BAD_SLOT, DEEPEP_FAULT_PLAN_UNIT, i, s, 0, num_recv);
    const bool active = lane < seg_len && !past_recv;
    const int32_t* m = meta + static_cast<int64_t>(active ? i : 0) * (K + 2);
    // the window row of (source, slot, token), or 0 unless all of its bytes lie inside that window
    auto window_row = [&](int64_t u, int slot) -> uint64_t {
        const int src = m[1] / K, st = m[0] % t_max;
        if (m[0] < 0 || m[1] < 0 || src >= R) {                 // metadata no correct dispatch produces
            deepep::record_fault(err, DEEPEP_FLAG_BAD_SLOT, DEEPEP_FAULT_PLAN_ROW, u, src, 0, m[0]);
            return 0ull;
        }
        const int64_t off = (static_cast<int64_t>(slot) * t_max + st) * row_bytes;
        if (slot < 0 || off + row_bytes > window_bytes) {
            deepep::record_fault(err, DEEPEP_FLAG_BAD_SLOT, DEEPEP_FAULT_PLAN_ROW, u, src, bases[src] + off,
                                 window_bytes >> 4);
            return 0ull;
        }
        return bases[src] + static_cast<uint64_t>(off);
    };
    // A unit is stored only inside its chunk and -- padded -- inside its own source's `padded` positions:
    // counts that disagree with the metadata (or a token whose lanes on this rank exceed the padding,
    // handle.build_ep_plan) must never overwrite another source's units.
    auto in_chunk = [&](int p, int64_t pos) -> bool {
        if (pos >= 0 && pos < chunk_units && (padded == 0 || p < padded)) return true;
        deepep::record_fault(err, DEEPEP_FLAG_BAD_SLOT, DEEPEP_FAULT_PLAN_UNIT, chunk_base + pos, s, 0, chunk_units);
        return false;
    };
    if (!single) {
        if (!active) return;
        const int pos = position(p0 + lane);
        if (!in_chunk(p0 + lane, pos)) return;
        const int64_t u = chunk_base + pos;
        if (expanded) {
            for (int k = 0; k < K; ++k) table_a[u * K + k] = m[2 + k];
        } else {
            table_a[u] = i;
            if (wtable_a != nullptr)
                for (int k = 0; k < K; ++k) wtable_a[u * K + k] = i * K + k;
        }
        // a row that is not provably inside its window is 0: phase A skips the unit and flags the call
        if (out_rows != nullptr) out_rows[u] = window_row(u, rank_layout ? rank : m[1] % K);
        return;
    }
    // single reduction: one unit per valid (row, lane), (row, lane) order
    int v = 0;
    if (active)
        for (int k = 0; k < K; ++k) v += m[2 + k] >= 0;
    const int q = wave_incl_scan(v, lane) - v;
    if (!active) return;
    int p = p0 + q;
    for (int k = 0; k < K; ++k) {
        const int32_t slot = m[2 + k];
        if (slot < 0) continue;
        const int pos = position(p);
        if (!in_chunk(p++, pos)) return;
        const int64_t u = chunk_base + pos;
        table_a[u] = slot;
        if (out_rows != nullptr) out_rows[u] = window_row(u, k);
    }
}

// ---------------------------------------------------------------- source side
// One wave per 64-token block of the owned tokens.  Multiple reduction: the rows of the token's
// partials in ascending dedup-master-lane order (a rank's master is its highest lane,
// combine_reduce_epilogue.cuh:74-95), then -1; the weight table points at each lane's weight inside
// the packed row of its rank's partial.  Single reduction: the row of every (t, k).
__global__ void __launch_bounds__(64)
plan_source_kernel(const int64_t* __restrict__ topk_idx, int T, int K, int epr, int R, int rank, int t_max,
                   const int32_t* __restrict__ dst_slot, const int32_t* __restrict__ send_tok,
                   const int32_t* __restrict__ send_pairs, int nb, int bpc, int flags, int64_t row_floats,
                   int64_t w_off, int32_t* __restrict__ table_b, int width, int32_t* __restrict__ wtable, int padded) {
    __shared__ int s_base[kMaxRanks];
    const int lane = threadIdx.x, b = blockIdx.x;
    const int t = b * kBlk + lane;
    const bool single = flags & DEEPEP_PLAN_SINGLE, window = flags & DEEPEP_PLAN_WINDOW;
    const bool rank_layout = flags & DEEPEP_PLAN_RANK_LAYOUT;
    const bool bypass = (flags & DEEPEP_PLAN_LOCAL_BYPASS) && !window;
    const int cb0 = (b / bpc) * bpc, cb1 = min(cb0 + bpc, nb);
    if (!window) {
        // receive buffer of chunk c: grouped by expert rank d in recv_order, each group in ascending
        // (token[, lane])
        int n_l = 0, extra = 0;
        if (lane < R) {
            const int32_t* cl = (single ? send_pairs : send_tok) + static_cast<int64_t>(lane) * nb;
            for (int j = cb0; j < cb1; ++j) n_l += cl[j];
            if (single) {
                for (int j = cb0; j < b; ++j) extra += cl[j];                 // earlier blocks of the chunk
            } else {
                for (int j = 0; j < cb0; ++j) extra -= cl[j];                 // dst_slot counts from token 0
            }
        }
        // rows of the expert ranks before this lane's rank in recv_order (a wave-uniform loop)
        const int me = recv_order(lane, rank, bypass);
        int before = 0;
        for (int l = 0; l < R; ++l) {
            const int nl = __shfl(n_l, l, 64);
            if (recv_order(l, rank, bypass) < me) before += nl;
        }
        // padded: expert rank d's rows of the chunk start at recv_order(d) * padded (a worst-case-padded
        // exchange)
        if (lane < R) s_base[lane] = (padded > 0 ? me * padded : before) + extra;
        __syncthreads();
    }
    int rk[kMaxTopk];
#pragma unroll
    for (int k = 0; k < kMaxTopk; ++k)
        rk[k] = (t < T && k < K) ? rank_of_expert(topk_idx[static_cast<int64_t>(t) * K + k], epr) : -1;
    if (single) {
        int32_t row[kMaxTopk];
#pragma unroll
        for (int k = 0; k < kMaxTopk; ++k) row[k] = -1;
        if (window) {
#pragma unroll
            for (int k = 0; k < kMaxTopk; ++k)
                if (rk[k] >= 0) row[k] = k * t_max + t;
        } else {
            for (int d = 0; d < R; ++d) {                           // wave-uniform loop: scans stay converged
                int c = 0;
#pragma unroll
                for (int k = 0; k < kMaxTopk; ++k) c += rk[k] == d;
                int off = s_base[d] + wave_incl_scan(c, lane) - c;
                // padded: rows past destination d's `padded` rows of the chunk belong to the next
                // destination -- a unit plan_expert rejected (flagged there); such a lane reads nothing
                const int lim = padded > 0 ? recv_order(d, rank, bypass) * padded + padded : INT32_MAX;
#pragma unroll
                for (int k = 0; k < kMaxTopk; ++k)
                    if (rk[k] == d) {
                        row[k] = off < lim ? off : -1;
                        ++off;
                    }
            }
        }
        if (t < T)
            for (int k = 0; k < K; ++k) table_b[static_cast<int64_t>(t) * width + k] = row[k];
        return;
    }
    if (t >= T) return;
    auto row_of = [&](int d, int master) -> int32_t {
        if (window) return (rank_layout ? d : master) * t_max + t;
        return s_base[d] + dst_slot[static_cast<int64_t>(t) * R + d];
    };
    auto master_of = [&](int d) -> int {
        int m = -1;
        for (int k = 0; k < K; ++k)
            if (rk[k] == d) m = k;
        return m;
    };
    int n = 0;
    for (int k = 0; k < K; ++k) {
        const int d = rk[k];
        if (d < 0 || master_of(d) != k) continue;                 // k is d's master lane: ascending order
        if (n < width) table_b[static_cast<int64_t>(t) * width + n] = row_of(d, k);
        ++n;
    }
    for (; n < width; ++n) table_b[static_cast<int64_t>(t) * width + n] = -1;
    if (wtable != nullptr)
        for (int k = 0; k < K; ++k) {
            const int d = rk[k];
            wtable[static_cast<int64_t>(t) * K + k] =
                d >= 0 ? static_cast<int32_t>(static_cast<int64_t>(row_of(d, master_of(d))) * row_floats + w_off + k)
                       : -1;
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

}  // namespace

extern "C" {

int deepep_route_block_counts(const int64_t* topk_idx, int num_tokens, int num_topk, int num_experts, int num_ranks,
                              int num_blocks, int32_t* tok_counts, int32_t* pair_counts, deepep_stream_t stream) {
    if (num_tokens < 0 || num_topk < 1 || num_topk > kMaxTopk || num_ranks < 1 || num_ranks > kMaxRanks ||
        num_experts < num_ranks || num_experts % num_ranks != 0 || num_blocks < (num_tokens + kBlk - 1) / kBlk ||
        (num_blocks > 0 && (tok_counts == nullptr || pair_counts == nullptr)) || (num_tokens > 0 && topk_idx == nullptr))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "route_block_counts: invalid arguments");
    if (num_blocks == 0) return DEEPEP_OK;
    hipLaunchKernelGGL(block_counts_kernel, dim3(num_blocks), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                       topk_idx, num_tokens, num_topk, num_experts / num_ranks, num_ranks, num_blocks,
                       tok_counts, pair_counts);
    return launch_status("route_block_counts");
}

int deepep_plan_expert(const int32_t* src_metadata, int num_recv, int num_topk, int num_ranks, int rank,
                       int num_max_tokens, const int32_t* recv_tok, const int32_t* recv_pairs, int num_blocks,
                       int blocks_per_chunk, int flags, int32_t* table_a, int32_t* wtable_a,
                       const uint64_t* window_bases, int64_t window_row_bytes, int64_t window_bytes,
                       uint64_t* out_rows, int32_t* error_flag, int padded_stride, deepep_stream_t stream) {
    const bool single = flags & DEEPEP_PLAN_SINGLE;
    if (num_recv < 0 || padded_stride < 0 ||
        static_cast<int64_t>(padded_stride) * num_ranks * ((num_blocks + blocks_per_chunk - 1) /
                                                           (blocks_per_chunk > 0 ? blocks_per_chunk : 1)) >=
            (int64_t(1) << 31) || num_topk < 1 || num_topk > kMaxTopk || num_ranks < 1 || num_ranks > kMaxRanks || rank < 0 ||
        rank >= num_ranks || num_max_tokens < 1 || num_blocks < 0 || blocks_per_chunk < 1 ||
        (num_blocks > 0 && (recv_tok == nullptr || (single && recv_pairs == nullptr))) ||
        (num_recv > 0 && src_metadata == nullptr) ||
        (out_rows != nullptr && (window_bases == nullptr || window_row_bytes <= 0 || window_row_bytes % 16 ||
                                 window_bytes < window_row_bytes)) ||
        (single && (flags & DEEPEP_PLAN_EXPANDED) == 0))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "plan_expert: invalid arguments");
    if (num_blocks == 0) return DEEPEP_OK;
    hipLaunchKernelGGL(plan_expert_kernel, dim3(num_ranks * num_blocks), dim3(64), 0,
                       reinterpret_cast<hipStream_t>(stream), src_metadata, num_recv, num_topk, num_ranks, rank,
                       num_max_tokens, recv_tok, recv_pairs, num_blocks, blocks_per_chunk, flags, table_a, wtable_a,
                       window_bases, window_row_bytes, window_bytes, out_rows, error_flag, padded_stride);
    return launch_status("plan_expert");
}

int deepep_plan_source(const int64_t* topk_idx, int num_tokens, int num_topk, int num_experts, int num_ranks,
                       int rank, int num_max_tokens, const int32_t* dst_slot, const int32_t* send_tok,
                       const int32_t* send_pairs, int num_blocks, int blocks_per_chunk, int flags,
                       int64_t row_floats, int64_t weights_offset, int32_t* table_b, int table_b_width,
                       int32_t* wtable, int padded_stride, deepep_stream_t stream) {
    const bool single = flags & DEEPEP_PLAN_SINGLE, window = flags & DEEPEP_PLAN_WINDOW;
    const int need_width = single ? num_topk : (num_ranks < num_topk ? num_ranks : num_topk);
    if (num_tokens < 0 || padded_stride < 0 || (window && padded_stride > 0) || num_topk < 1 || num_topk > kMaxTopk || num_ranks < 1 || num_ranks > kMaxRanks ||
        num_experts % num_ranks != 0 || rank < 0 || rank >= num_ranks || num_tokens > num_max_tokens || blocks_per_chunk < 1 ||
        num_blocks < (num_tokens + kBlk - 1) / kBlk || table_b_width != need_width ||
        (num_tokens > 0 && (topk_idx == nullptr || table_b == nullptr)) ||
        (!window && num_tokens > 0 && (send_tok == nullptr || (single ? send_pairs == nullptr : dst_slot == nullptr))) ||
        (wtable != nullptr && (single || row_floats < 1 || weights_offset < 0)))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "plan_source: invalid arguments");
    if (num_tokens == 0) return DEEPEP_OK;
    hipLaunchKernelGGL(plan_source_kernel, dim3((num_tokens + kBlk - 1) / kBlk), dim3(64), 0,
                       reinterpret_cast<hipStream_t>(stream), topk_idx, num_tokens, num_topk,
                       num_experts / num_ranks, num_ranks, rank, num_max_tokens, dst_slot, send_tok, send_pairs, num_blocks,
                       blocks_per_chunk, flags, row_floats, weights_offset, table_b, table_b_width, wtable,
                       padded_stride);
    return launch_status("plan_source");
}

}  // extern "C"
