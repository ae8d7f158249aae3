// combine.hip -- the combine reduction for MI355X (gfx950, CDNA4), exported through
// the C-ABI declared in include/deepep_amd.h.
//
// What is computed (semantics of the reference, /root/reference paths):
//   DEEPEP_MODE_LOCAL    combine_impl's local reduce       deep_ep/include/deep_ep/impls/combine.cuh:114-213
//   DEEPEP_MODE_EPILOGUE combine_reduce_epilogue_impl      deep_ep/include/deep_ep/impls/combine_reduce_epilogue.cuh:62-125
//   arithmetic core      combine_reduce                    deep_ep/include/deep_ep/impls/combine_utils.cuh:55-170
//   weighted variant     legacy low-latency combine        csrc/kernels/legacy/internode_ll.cu:1072-1135
//
// How (MI355X-first, not a translation of the TMA/warp design):
//   * the work is split into items = (output row, column chunk of 64 lanes x vpt x 16 B); one wave64
//     owns one item and a workgroup of 4 or 8 waves owns that many consecutive items, so the grid is
//     tens of thousands of workgroups with no tail imbalance;
//   * the item's row of the slot table (and, weighted, the gating weights) is staged once per
//     workgroup in LDS, one entry per lane; the valid slots are visited in ascending order through
//     the wave's ballot mask (= the reference's compacted slot order);
//   * each lane keeps 2-8 rows x vpt x 16 B of non-temporal global_load_dwordx4 in flight (every
//     expanded row is read exactly once), accumulates bf16 -> fp32 in registers in the reference's
//     order, rounds once with v_cvt_pk_bf16_f32 (RNE) and writes vpt x 16 B with a write-through
//     buffer store.
//   No MFMA: this is an HBM-bound gather + elementwise add (roofline and measurements in DESIGN.md).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>

#include "../../include/deepep_amd.h"
#include "fault.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kMaxWidth = 32;          // top-k <= 32, as the reference (combine_reduce_epilogue.cuh:64)

thread_local char g_last_error[512] = "";

int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
    return code;
}

__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// Round-to-nearest-even pack of two floats (v_cvt_pk_bf16_f32), = __float22bfloat162_rn.
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    const bf16x2 r = __builtin_convertvector((f32x2){a, b}, bf16x2);
    return __builtin_bit_cast(uint32_t, r);
}

template <bool kNT>
__device__ __forceinline__ u32x4 load16(const u32x4* p) {
    if constexpr (kNT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

struct Params {
    const uint16_t* src;
    int64_t num_src_rows;
    int64_t src_stride;          // elements
    const int32_t* table;
    int64_t table_stride;
    int table_width;
    const float* row_weights;
    const uint16_t* bias0;
    const uint16_t* bias1;
    uint16_t* out;
    int64_t out_stride;          // elements
    int num_units;
    int hidden;
    const int32_t* wtable;
    int64_t wtable_stride;
    const float* wsrc;
    float* out_weights;
    int num_weights;
    int weights_pad;             // floats written per unit's weight row (>= num_weights; zeros past them)
    int64_t out_weights_stride;  // floats between consecutive units' weight rows
    int units_per_block;
    int32_t* error_flag;
    const uint64_t* out_rows;    // scatter (phase A over xGMI): byte address of unit u's output row, or NULL
    int64_t weights_offset;      // scatter: byte offset of the weights inside the output row
    const uint64_t* win_bases;   // scatter: the windows every out_rows[u] must lie in (lane l < win_count: window l)
    int win_count;
    uint64_t win_limit;          // scatter: largest offset of a row start inside a window (extent - row bytes)
};

// Scatter (phase A into the owners' windows): the byte address of unit u's row, or 0 when the unit must
// not be stored -- a row plan_expert rejected (0, bit 1) or one not wholly inside any window (bit 4 and
// the error record: a wild store through a bad address is never issued).  Wave-uniform.
__device__ __forceinline__ uint64_t checked_row(const Params& p, int64_t u, int lane, bool report) {
    const uint64_t a = p.out_rows[u];
    if (a == 1ull) return 0ull;                          // a padding position of a padded plan: no unit
    if (a == 0ull) {
        if (report && lane == 0 && p.error_flag != nullptr) atomicOr(p.error_flag, DEEPEP_FLAG_BAD_SLOT);
        return 0ull;
    }
    const uint64_t base = lane < p.win_count ? p.win_bases[lane] : 0ull;
    const bool inside = lane < p.win_count && (a & 15ull) == 0ull && a >= base && a - base <= p.win_limit;
    if (__ballot(inside) != 0ull) return a;
    if (report && lane == 0)
        deepep::record_fault(p.error_flag, DEEPEP_FLAG_BAD_ADDRESS, DEEPEP_FAULT_SCATTER_ROW, u, -1, a,
                             static_cast<int64_t>(p.win_limit >> 4));
    return 0ull;
}

// acc[8*v + e] += element e of the 16-byte vector (8 bf16)
__device__ __forceinline__ void acc_add(float* acc, const u32x4& v) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        acc[2 * d] += bf16_lo(v[d]);
        acc[2 * d + 1] += bf16_hi(v[d]);
    }
}

__device__ __forceinline__ void acc_fma(float* acc, const u32x4& v, float w) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        acc[2 * d] = __builtin_fmaf(bf16_lo(v[d]), w, acc[2 * d]);
        acc[2 * d + 1] = __builtin_fmaf(bf16_hi(v[d]), w, acc[2 * d + 1]);
    }
}

__device__ __forceinline__ u32x4 acc_pack(const float* acc) {
    u32x4 r;
#pragma unroll
    for (int d = 0; d < 4; ++d)
        r[d] = pack_bf16x2(acc[2 * d], acc[2 * d + 1]);
    return r;
}

// Output stores: buffer_store_dwordx4 with a per-row descriptor (the hardware range check drops the
// lanes past the row end).  Three cache policies ship, one per kind of output:
//   sc1     (write-through, line not kept in L2): the fused and epilogue reduces, whose output is
//           written in token order -- best or tied in every cache state measured;
//   sc1 nt  (write-through streaming): phase A's send rows, written once and read back only by the
//           exchange -- within 2 % of the best policy in every cache state at EP = 2 / 4 / 8;
//   sc0 sc1 (system scope): phase A into a peer's symmetric window over xGMI, visible to the owning
//           GPU once the kernel has completed, whatever MTYPE the importing process maps it with.
// (plain, nt and a per-unit sc1 / sc1 nt mix lost or were cache-state dependent; their measurements
// are in CHANGELOG.md, the code in git history.)
constexpr int kAuxSC1 = 16, kAuxSys = 17, kAuxSC1NT = 18;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* row, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(row), 0, bytes, 0x00020000);
}

// The pass-through weight of lane k of unit u: wsrc[wtable[u][k]] (or wsrc[u * num_weights + k]), 0
// for masked lanes and for lanes past num_weights (the zeros of a padded tail line).  When the slot
// table doubles as the weight table (the expanded layouts) the lane's slot is already in hand -- and
// so is its weight when the reduction is weighted by the same array -- so no dependent gather
// delays the wave's row loads.
template <bool kWeighted>
__device__ __forceinline__ float pass_through_weight(const Params& p, int64_t u, int lane, int32_t my_slot, float my_w) {
    if (lane >= p.num_weights) return 0.0f;
    if (p.table != nullptr && p.wtable == p.table && p.wtable_stride == p.table_stride && lane < p.table_width) {
        if (kWeighted && p.wsrc == p.row_weights) return my_w;
        return my_slot >= 0 ? p.wsrc[my_slot] : 0.0f;
    }
    const int64_t i = p.wtable == nullptr ? u * p.num_weights + lane
                                          : static_cast<int64_t>(p.wtable[u * p.wtable_stride + lane]);
    return i >= 0 ? p.wsrc[i] : 0.0f;
}

// Store it: into the unit's weight row, or the row tail of a peer's window (system scope, as the
// row stores).  weights_pad > num_weights writes a packed row's whole 128-byte tail line.
__device__ __forceinline__ void store_weight(const Params& p, int64_t u, uint16_t* out_row, int lane, float v) {
    if (p.out_rows != nullptr) {
        float* const ow = reinterpret_cast<float*>(reinterpret_cast<char*>(out_row) + p.weights_offset);
        __hip_atomic_store(ow + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        p.out_weights[u * p.out_weights_stride + lane] = v;
    }
}

// One wave per item = (unit u, column chunk c): the chunk is 64 lanes x kVPT x 16 B of every
// source row of u.  The unit's slot table row (and its gating weights) arrive in my_slot / my_w, one
// entry per lane; the valid slots are then visited in ascending order through the ballot mask,
// which is exactly the compacted order of compute_topk_slots (combine_utils.cuh:41-53).
template <int kMode, bool kWeighted, int kVPT, bool kFull, int kStoreAux, int kGroup>
__device__ __forceinline__ void combine_item(const Params& p, int64_t it, int nchunks, int nvec, int lane,
                                             int32_t my_slot, float my_w) {
    constexpr int kChunkVecs = 64 * kVPT;
    const int64_t u = it / nchunks;
    const int c = static_cast<int>(it - u * nchunks);
    // A barrier of this window timed out (bit 2 of the error flag, set by deepep_sym_barrier /
    // _wait): the rows in flight are not trustworthy, so no store reaches a peer and the output is
    // poisoned with NaN instead of holding a silently wrong sum.
    const bool aborted = p.error_flag != nullptr && (__hip_atomic_load(p.error_flag, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT) & 2);
    if (aborted && p.out_rows != nullptr) return;
    if (aborted) my_slot = -1;
    const uint64_t valid = __ballot(my_slot >= 0);
    const int n = __popcll(valid);

    // ---- top-k weight pass-through (combine.cuh:215-226, combine_reduce_epilogue.cuh:127-141),
    //      written once per unit by the wave owning chunk 0: gathered here, stored after the row
    uint16_t* const out_row = p.out_rows != nullptr ? reinterpret_cast<uint16_t*>(checked_row(p, u, lane, c == 0))
                                                     : p.out + u * p.out_stride;
    if (out_row == nullptr) return;                      // rejected / outside every window: flagged above
    const bool wlane = c == 0 && p.num_weights > 0 && lane < p.weights_pad;
    const float wv = wlane ? pass_through_weight<kWeighted>(p, u, lane, my_slot, my_w) : 0.0f;

    int vidx[kVPT];
    bool vok[kVPT];
#pragma unroll
    for (int v = 0; v < kVPT; ++v) {
        vidx[v] = c * kChunkVecs + v * 64 + lane;
        vok[v] = kFull || vidx[v] < nvec;
    }
    const bool has_bias0 = p.bias0 != nullptr, has_bias1 = p.bias1 != nullptr;
    const bool has_bias = has_bias0 || has_bias1;

    // Initial value: -0.0f where the reference adds two sources in bf16 without an fp32 zero in
    // front (the hadd bypass, combine_utils.cuh:79-110: -0 + a == a exactly), +0.0f where it
    // starts from `float2 reduced = {}` (combine_utils.cuh:114).
    bool copy_row = false;
    float init;
    if constexpr (kMode == DEEPEP_MODE_LOCAL || kMode == DEEPEP_MODE_FUSED) {
        copy_row = !kWeighted && n == 1;                      // no_local_reduce (combine.cuh:134-156)
        init = (!kWeighted && n == 2) ? -0.0f : 0.0f;
    } else {
        // epilogue: bypass only without bias; weighted (single reduction, legacy semantics): from +0
        init = (!kWeighted && !has_bias && n == 2) ? -0.0f : 0.0f;
    }
    float acc[kVPT][8];
#pragma unroll
    for (int v = 0; v < kVPT; ++v)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[v][e] = init;
    if constexpr (kMode == DEEPEP_MODE_EPILOGUE) {
        // bias0 then bias1 before the partials (combine_utils.cuh:113-127)
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            if (has_bias0 && vok[v]) acc_add(acc[v], *(reinterpret_cast<const u32x4*>(p.bias0 + u * p.hidden) + vidx[v]));
            if (has_bias1 && vok[v]) acc_add(acc[v], *(reinterpret_cast<const u32x4*>(p.bias1 + u * p.hidden) + vidx[v]));
        }
    }

    // The valid lanes, lowest first, kGroup at a time: every row of a group is loaded before any is
    // accumulated (kGroup rows x kVPT x 16 B in flight per lane), and the accumulation order is the
    // ascending lane order of compute_topk_slots whatever the group size.  `rem` is wave-uniform.
    u32x4 result[kVPT];
    uint64_t rem = valid;
    while (rem != 0ull) {
        int lane_of[kGroup];
#pragma unroll
        for (int j = 0; j < kGroup; ++j) {
            lane_of[j] = rem != 0ull ? static_cast<int>(__builtin_ctzll(rem)) : -1;
            rem &= rem - 1ull;                              // (no-op once empty)
        }
        u32x4 vals[kGroup][kVPT];
#pragma unroll
        for (int j = 0; j < kGroup; ++j) {
            if (lane_of[j] >= 0) {
                const int32_t sj = __builtin_amdgcn_readlane(my_slot, lane_of[j]);
                const u32x4* row = reinterpret_cast<const u32x4*>(p.src + static_cast<int64_t>(sj) * p.src_stride);
#pragma unroll
                for (int v = 0; v < kVPT; ++v)
                    vals[j][v] = vok[v] ? load16<true>(row + vidx[v]) : (u32x4){0u, 0u, 0u, 0u};
            }
        }
        if (copy_row) {
#pragma unroll
            for (int v = 0; v < kVPT; ++v) result[v] = vals[0][v];        // n == 1: lane_of[0] is it
        } else {
#pragma unroll
            for (int j = 0; j < kGroup; ++j) {
                if (lane_of[j] >= 0) {
                    if constexpr (kWeighted) {
                        const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_w), lane_of[j]));
#pragma unroll
                        for (int v = 0; v < kVPT; ++v) acc_fma(acc[v], vals[j][v], w);
                    } else {
#pragma unroll
                        for (int v = 0; v < kVPT; ++v) acc_add(acc[v], vals[j][v]);
                    }
                }
            }
        }
    }
    if (!copy_row) {
#pragma unroll
        for (int v = 0; v < kVPT; ++v) result[v] = acc_pack(acc[v]);
    }

    if constexpr (kMode == DEEPEP_MODE_FUSED) {
        // Phase B over the single per-rank partial (EP = 1): epilogue with one slot.
        // No bias: hadd bypass with a zero second operand -> +0 + partial.
        // Bias: fp32 +0 + bias0 + bias1 + partial, one rounding (combine_utils.cuh:111-165).
        const bool present = n > 0;
#pragma unroll
        for (int v = 0; v < kVPT; ++v) {
            float a[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] = 0.0f;
            if (has_bias0 && vok[v]) acc_add(a, *(reinterpret_cast<const u32x4*>(p.bias0 + u * p.hidden) + vidx[v]));
            if (has_bias1 && vok[v]) acc_add(a, *(reinterpret_cast<const u32x4*>(p.bias1 + u * p.hidden) + vidx[v]));
            if (present) acc_add(a, result[v]);
            result[v] = acc_pack(a);
        }
    }

    if (aborted) {
#pragma unroll
        for (int v = 0; v < kVPT; ++v) result[v] = (u32x4){0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u};
    }
    const __amdgpu_buffer_rsrc_t orow = row_rsrc(out_row, p.hidden * 2);
#pragma unroll
    for (int v = 0; v < kVPT; ++v)
        __builtin_amdgcn_raw_buffer_store_b128(result[v], orow, vidx[v] * 16, 0, kStoreAux);
    if (wlane) store_weight(p, u, out_row, lane, wv);
}

// A workgroup of kWaves waves takes kWaves consecutive items; the slot-table rows of the units those
// items belong to (and their gating weights) are staged once per workgroup in LDS, one entry per lane.
// One workgroup per kWaves items: 28,672 workgroups at config 2, no tail imbalance.
template <int kMode, bool kWeighted, int kVPT, bool kFull, int kStoreAux, int kWaves, int kGroup>
__global__ void __launch_bounds__(64 * kWaves)
combine_rows_kernel(const Params p) {
    constexpr int kChunkVecs = 64 * kVPT;
    __shared__ int32_t s_slot[kWaves][kMaxWidth];
    __shared__ float s_w[kWaves][kMaxWidth];
    const int tid = static_cast<int>(threadIdx.x), lane = tid & 63, wave = tid >> 6;
    const int nvec = p.hidden >> 3;                          // 16-byte vectors per row
    const int nchunks = (nvec + kChunkVecs - 1) / kChunkVecs;
    const int64_t items = static_cast<int64_t>(p.num_units) * nchunks;
    const int width = p.table == nullptr ? 1 : p.table_width;
    const int64_t it0 = static_cast<int64_t>(blockIdx.x) * kWaves;
    const int64_t it = it0 + wave;
    const int64_t u_first = it0 / nchunks;
    const int nu = static_cast<int>(min(it0 + kWaves - 1, items - 1) / nchunks - u_first) + 1;
    if (tid < nu * width) {                                  // nu * width <= kWaves * 32 threads
        const int ul = tid / width, j = tid - ul * width;
        const int64_t u = u_first + ul;
        int32_t s = p.table == nullptr ? static_cast<int32_t>(u) : p.table[u * p.table_stride + j];
        if (s >= p.num_src_rows) {                           // never dereference a bad slot
            if (p.error_flag != nullptr) atomicOr(p.error_flag, DEEPEP_FLAG_BAD_SLOT);
            s = -1;
        }
        s_slot[ul][j] = s;
        if constexpr (kWeighted) s_w[ul][j] = s >= 0 ? p.row_weights[s] : 0.0f;
    }
    __syncthreads();
    if (it >= items) return;
    int32_t my_slot = -1;
    float my_w = 0.0f;
    if (lane < width) {
        const int ul = static_cast<int>(it / nchunks - u_first);
        my_slot = s_slot[ul][lane];
        if constexpr (kWeighted) my_w = s_w[ul][lane];
    }
    combine_item<kMode, kWeighted, kVPT, kFull, kStoreAux, kGroup>(p, it, nchunks, nvec, lane, my_slot, my_w);
}

// CU-budget streams created by deepep_stream_create_cu_budget (symmetric.hip) and their CU counts: a
// launch on one keeps its full grid (the CU mask alone holds it to the budget) with at most 4 rows in
// flight per lane -- 64 VGPRs, 8 waves per SIMD, more bytes in flight per budgeted CU than 8 rows at 5
// waves (config 2: 128 CUs 208 vs 235 us, 32 CUs 603 vs 661 us, profiles/archive/r02n_kcu2.jsonl).
std::mutex g_budget_mutex;
std::map<hipStream_t, int> g_budget_cus;

int budget_cus_of(hipStream_t s) {
    if (s == nullptr) return 0;
    std::lock_guard<std::mutex> lock(g_budget_mutex);
    const auto it = g_budget_cus.find(s);
    return it == g_budget_cus.end() ? 0 : it->second;
}

// The one tuning knob left (diagnostics; deepep_set_launch_config): vectors per lane (bits 0-3) and rows
// in flight (bits 4-7), 0 = automatic.  One atomic word, read once per launch, so a launch never sees
// half of another thread's update.
std::atomic<uint32_t> g_launch_config{0};

struct Shape {
    int vpt, waves, group;
};

template <int kMode, bool kWeighted, int kVPT, bool kFull, int kAux, int kWaves>
void launch_group(const Params& p, int group, hipStream_t stream) {
    const int nvec = p.hidden / 8;
    const int64_t items = static_cast<int64_t>(p.num_units) * ((nvec + 64 * kVPT - 1) / (64 * kVPT));
    const dim3 grid(static_cast<unsigned>((items + kWaves - 1) / kWaves)), block(64 * kWaves);
    if (group == 2)
        hipLaunchKernelGGL((combine_rows_kernel<kMode, kWeighted, kVPT, kFull, kAux, kWaves, 2>), grid, block, 0, stream, p);
    else if (group == 4)
        hipLaunchKernelGGL((combine_rows_kernel<kMode, kWeighted, kVPT, kFull, kAux, kWaves, 4>), grid, block, 0, stream, p);
    else
        hipLaunchKernelGGL((combine_rows_kernel<kMode, kWeighted, kVPT, kFull, kAux, kWaves, 8>), grid, block, 0, stream, p);
}

template <int kMode, bool kWeighted, int kAux>
void launch_shape(const Params& p, const Shape& sh, hipStream_t stream) {
    const int nvec = p.hidden / 8;
#define DEEPEP_WAVES(VPT, FULL)                                                            \
    (sh.waves == 4 ? launch_group<kMode, kWeighted, VPT, FULL, kAux, 4>(p, sh.group, stream) \
                   : launch_group<kMode, kWeighted, VPT, FULL, kAux, 8>(p, sh.group, stream))
    if (sh.vpt == 1) {
        if (nvec % 64 == 0) DEEPEP_WAVES(1, true);
        else DEEPEP_WAVES(1, false);
    } else {
        if (nvec % 128 == 0) DEEPEP_WAVES(2, true);
        else DEEPEP_WAVES(2, false);
    }
#undef DEEPEP_WAVES
}

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0; }

// ---------------------------------------------------------------- plan builder
__global__ void fill_kernel(int32_t* dst, int64_t n, int32_t value) {
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        dst[i] = value;
}

__global__ void local_plan_kernel(const int32_t* meta, int num_recv, int num_topk, int t_max, int expanded,
                                  int32_t* plan, int plan_width, int num_tokens,
                                  const int64_t* topk_idx, int32_t* wtable) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= num_recv) return;
    const int stride = num_topk + 2;
    const int t = meta[static_cast<int64_t>(i) * stride] % t_max;
    if (t < 0 || t >= num_tokens) return;
    if (expanded) {
        for (int k = 0; k < plan_width; ++k)
            plan[static_cast<int64_t>(t) * plan_width + k] = meta[static_cast<int64_t>(i) * stride + 2 + k];
    } else {
        plan[static_cast<int64_t>(t) * plan_width] = i;
    }
    if (wtable != nullptr)
        for (int k = 0; k < num_topk; ++k)
            wtable[static_cast<int64_t>(t) * num_topk + k] =
                topk_idx[static_cast<int64_t>(t) * num_topk + k] >= 0 ? i * num_topk + k : -1;
}

int launch_combine(int mode, int weighted, const Params& p, deepep_stream_t stream);

}  // namespace

extern "C" {

// Error reporting shared with dispatch.hip (not part of the public C-ABI).
__attribute__((visibility("hidden"))) int deepep_amd_set_error(int code, const char* msg) {
    return set_error(code, "%s", msg);
}

// Budget streams (shared with symmetric.hip; not part of the public C-ABI): cus <= 0 forgets one.
__attribute__((visibility("hidden"))) void deepep_amd_register_budget(void* stream, int cus) {
    std::lock_guard<std::mutex> lock(g_budget_mutex);
    if (cus > 0) g_budget_cus[static_cast<hipStream_t>(stream)] = cus;
    else g_budget_cus.erase(static_cast<hipStream_t>(stream));
}

int deepep_amd_abi_version(void) { return DEEPEP_AMD_ABI_VERSION; }

#ifndef DEEPEP_BUILD_ID
#define DEEPEP_BUILD_ID "unknown-build-id"
#endif
// The build id (hash of sources, header and flags, deepep_amd/_lib.py) stored with a marker so that
// it can be read from the file without loading it.
__attribute__((used)) static const char g_build_id[] = "DEEPEP_BUILD_ID=" DEEPEP_BUILD_ID;
const char* deepep_amd_build_id(void) { return g_build_id + 16; }

const char* deepep_amd_last_error(void) { return g_last_error; }

int deepep_combine_reduce(int mode, int weighted,
                          const void* src, int64_t num_src_rows, int64_t src_row_stride,
                          const int32_t* table, int64_t table_stride, int table_width,
                          const float* row_weights,
                          const void* bias0, const void* bias1,
                          void* out, int64_t out_row_stride,
                          int num_units, int hidden,
                          const int32_t* wtable, int64_t wtable_stride,
                          const float* wsrc, float* out_weights, int num_weights,
                          int64_t out_weights_stride, int weights_pad,
                          int units_per_block, int32_t* error_flag,
                          deepep_stream_t stream) {
    if (mode < DEEPEP_MODE_LOCAL || mode > DEEPEP_MODE_FUSED)
        return set_error(DEEPEP_ERR_INVALID_ARG, "invalid mode %d", mode);
    if (num_units < 0 || hidden < 0)
        return set_error(DEEPEP_ERR_INVALID_ARG, "negative size (num_units=%d, hidden=%d)", num_units, hidden);
    if (num_units == 0) return DEEPEP_OK;
    if (hidden % 8 != 0)
        return set_error(DEEPEP_ERR_INVALID_ARG, "hidden (%d) * sizeof(bf16) must be a multiple of 16 bytes", hidden);
    if (out == nullptr || (hidden > 0 && src == nullptr && num_src_rows > 0))
        return set_error(DEEPEP_ERR_INVALID_ARG, "null src/out");
    if (!aligned16(src) || !aligned16(out) || !aligned16(bias0) || !aligned16(bias1))
        return set_error(DEEPEP_ERR_INVALID_ARG, "src/out/bias must be 16-byte aligned");
    if (src_row_stride % 8 != 0 || out_row_stride % 8 != 0 || src_row_stride < hidden || out_row_stride < hidden)
        return set_error(DEEPEP_ERR_INVALID_ARG, "row strides must be >= hidden and multiples of 8 elements");
    if (table != nullptr && (table_width < 1 || table_width > kMaxWidth || table_stride < table_width))
        return set_error(DEEPEP_ERR_INVALID_ARG, "table width %d outside [1, %d] or stride too small", table_width, kMaxWidth);
    if (weighted && row_weights == nullptr)
        return set_error(DEEPEP_ERR_INVALID_ARG, "weighted reduction needs row weights");
    if (mode == DEEPEP_MODE_LOCAL && (bias0 != nullptr || bias1 != nullptr))
        return set_error(DEEPEP_ERR_INVALID_ARG, "bias is applied by the epilogue, not the local reduce");
    if (out_weights != nullptr && (wsrc == nullptr || num_weights < 1 || num_weights > kMaxWidth))
        return set_error(DEEPEP_ERR_INVALID_ARG, "weight pass-through needs wsrc and 1 <= num_weights <= %d", kMaxWidth);
    if (out_weights_stride == 0) out_weights_stride = num_weights;
    if (weights_pad < num_weights) weights_pad = num_weights;
    if (out_weights != nullptr && (out_weights_stride < weights_pad || weights_pad > 64))
        return set_error(DEEPEP_ERR_INVALID_ARG, "out_weights_stride (%lld) < weights_pad (%d) or weights_pad > 64",
                         static_cast<long long>(out_weights_stride), weights_pad);
    Params p;
    p.src = static_cast<const uint16_t*>(src);
    p.num_src_rows = num_src_rows;
    p.src_stride = src_row_stride;
    p.table = table;
    p.table_stride = table_stride;
    p.table_width = table_width;
    p.row_weights = row_weights;
    p.bias0 = static_cast<const uint16_t*>(bias0);
    p.bias1 = static_cast<const uint16_t*>(bias1);
    p.out = static_cast<uint16_t*>(out);
    p.out_stride = out_row_stride;
    p.num_units = num_units;
    p.hidden = hidden;
    p.wtable = wtable;
    p.wtable_stride = wtable_stride;
    p.wsrc = wsrc;
    p.out_weights = out_weights;
    p.num_weights = out_weights != nullptr ? num_weights : 0;
    p.weights_pad = weights_pad;
    p.out_weights_stride = out_weights_stride;
    p.units_per_block = units_per_block;
    p.error_flag = error_flag;
    p.out_rows = nullptr;
    p.weights_offset = 0;
    p.win_bases = nullptr;
    p.win_count = 0;
    p.win_limit = 0;

    return launch_combine(mode, weighted, p, stream);
}

int deepep_combine_reduce_scatter(int weighted,
                                  const void* src, int64_t num_src_rows, int64_t src_row_stride,
                                  const int32_t* table, int64_t table_stride, int table_width,
                                  const float* row_weights,
                                  const uint64_t* out_rows, int num_units, int hidden,
                                  const int32_t* wtable, int64_t wtable_stride,
                                  const float* wsrc, int num_weights, int64_t weights_offset, int weights_pad,
                                  const uint64_t* window_bases, int num_windows, int64_t window_bytes,
                                  int32_t* error_flag, deepep_stream_t stream) {
    if (num_units < 0 || hidden < 0)
        return set_error(DEEPEP_ERR_INVALID_ARG, "negative size (num_units=%d, hidden=%d)", num_units, hidden);
    if (num_units == 0) return DEEPEP_OK;
    if (hidden % 8 != 0)
        return set_error(DEEPEP_ERR_INVALID_ARG, "hidden (%d) * sizeof(bf16) must be a multiple of 16 bytes", hidden);
    if (out_rows == nullptr || (src == nullptr && num_src_rows > 0) || !aligned16(src))
        return set_error(DEEPEP_ERR_INVALID_ARG, "null out_rows / unaligned src");
    if (src_row_stride % 8 != 0 || src_row_stride < hidden)
        return set_error(DEEPEP_ERR_INVALID_ARG, "src row stride must be >= hidden and a multiple of 8 elements");
    if (table != nullptr && (table_width < 1 || table_width > kMaxWidth || table_stride < table_width))
        return set_error(DEEPEP_ERR_INVALID_ARG, "table width %d outside [1, %d] or stride too small", table_width, kMaxWidth);
    if (weighted && row_weights == nullptr)
        return set_error(DEEPEP_ERR_INVALID_ARG, "weighted reduction needs row weights");
    if (num_weights > 0 && (wsrc == nullptr || num_weights > kMaxWidth || weights_offset < int64_t(hidden) * 2 ||
                            weights_offset % 4 != 0))
        return set_error(DEEPEP_ERR_INVALID_ARG, "weights need wsrc, num_weights <= %d and an offset past the row", kMaxWidth);
    if (weights_pad < num_weights) weights_pad = num_weights;
    if (weights_pad > 64) return set_error(DEEPEP_ERR_INVALID_ARG, "weights_pad > 64");
    // the bytes one unit stores: the bf16 row, then (with weights) weights_pad floats at weights_offset
    const int64_t row_extent = num_weights > 0 ? std::max<int64_t>(int64_t(hidden) * 2, weights_offset + 4 * weights_pad)
                                               : int64_t(hidden) * 2;
    if (window_bases == nullptr || num_windows < 1 || num_windows > 64 || window_bytes < row_extent)
        return set_error(DEEPEP_ERR_INVALID_ARG, "scatter needs 1..64 windows of at least one row (%lld bytes)",
                         static_cast<long long>(row_extent));
    Params p;
    p.src = static_cast<const uint16_t*>(src);
    p.num_src_rows = num_src_rows;
    p.src_stride = src_row_stride;
    p.table = table;
    p.table_stride = table_stride;
    p.table_width = table_width;
    p.row_weights = row_weights;
    p.bias0 = nullptr;
    p.bias1 = nullptr;
    p.out = nullptr;
    p.out_stride = 0;
    p.num_units = num_units;
    p.hidden = hidden;
    p.wtable = wtable;
    p.wtable_stride = wtable_stride;
    p.wsrc = wsrc;
    p.out_weights = nullptr;
    p.num_weights = num_weights > 0 ? num_weights : 0;
    p.weights_pad = weights_pad;
    p.out_weights_stride = 0;
    p.units_per_block = 0;
    p.error_flag = error_flag;
    p.out_rows = out_rows;
    p.weights_offset = weights_offset;
    p.win_bases = window_bases;
    p.win_count = num_windows;
    p.win_limit = static_cast<uint64_t>(window_bytes - row_extent);
    return launch_combine(DEEPEP_MODE_LOCAL, weighted, p, stream);
}

}  // extern "C"

namespace {

int launch_combine(int mode, int weighted, const Params& p, deepep_stream_t stream) {
    // Launch shape: one wave per (unit, 64 x vpt x 16-byte column chunk) item, `waves` items per
    // workgroup, `group` source rows loaded per lane before any is accumulated.  Measured per shape
    // class (launch-shape sweeps of rounds 2-4: DESIGN.md section 3, CHANGELOG.md):
    //   fused reduce over top-k >= 5, rows >= 256 vectors: 1 KiB chunks, 2 rows, 4 waves -- few registers,
    //     many waves (config 2: -0.9 to -1.6 % against 2 KiB / 8 rows / 8 waves on three boxes);
    //   fused over top-k >= 5, rows of 128-255 vectors: 2 KiB chunks, 4 rows, 8 waves;
    //   epilogue (phase B) and the other fused shapes: 2 KiB chunks, 8 rows, 8 waves;
    //   phase A (LOCAL, ~1.5 local rows per received token at EP = 8): 2 KiB chunks, 4 rows, 4 waves
    //     (64 VGPRs, 8 waves per SIMD; 1 KiB chunks lose there, 297-330 vs 249.6 us);
    // rows in flight are capped at the slot table's width rounded up to 2 / 4 (top-2: 33.7 vs 40.1 us),
    // and at 4 on a CU-budget stream.
    const uint32_t cfg = g_launch_config.load(std::memory_order_relaxed);
    const int cfg_vpt = static_cast<int>(cfg & 15u), cfg_rows = static_cast<int>((cfg >> 4) & 15u);
    const int nvec = p.hidden / 8;
    const int width = p.table == nullptr ? 1 : p.table_width;
    const int width_cap = width <= 2 ? 2 : (width <= 4 ? 4 : 8);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int budget = budget_cus_of(s);
    Shape sh;
    sh.vpt = nvec >= 128 ? 2 : 1;
    sh.waves = mode == DEEPEP_MODE_LOCAL ? 4 : 8;
    sh.group = std::min(mode == DEEPEP_MODE_LOCAL || budget > 0 ? 4 : 8, width_cap);
    const bool automatic = cfg == 0 && p.units_per_block == 0 && budget == 0;
    if (automatic && mode == DEEPEP_MODE_FUSED && width >= 5 && nvec >= 256) {
        sh.vpt = 1;
        sh.group = 2;
        sh.waves = 4;
    } else if (automatic && mode == DEEPEP_MODE_FUSED && width >= 5 && nvec >= 128) {
        sh.group = 4;
    }
    if (cfg_vpt != 0) sh.vpt = cfg_vpt;
    if (cfg_rows != 0) sh.group = cfg_rows;
    if (p.units_per_block == 4 || p.units_per_block == 8) sh.waves = p.units_per_block;

#define DEEPEP_POLICY(M, AUX) \
    (weighted ? launch_shape<M, true, AUX>(p, sh, s) : launch_shape<M, false, AUX>(p, sh, s))
    if (mode == DEEPEP_MODE_LOCAL && p.out_rows != nullptr) DEEPEP_POLICY(DEEPEP_MODE_LOCAL, kAuxSys);
    else if (mode == DEEPEP_MODE_LOCAL) DEEPEP_POLICY(DEEPEP_MODE_LOCAL, kAuxSC1NT);
    else if (mode == DEEPEP_MODE_EPILOGUE) DEEPEP_POLICY(DEEPEP_MODE_EPILOGUE, kAuxSC1);
    else DEEPEP_POLICY(DEEPEP_MODE_FUSED, kAuxSC1);
#undef DEEPEP_POLICY
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess)
        return set_error(DEEPEP_ERR_HIP, "combine launch failed: %s", hipGetErrorString(err));
    return DEEPEP_OK;
}

}  // namespace

extern "C" {

int deepep_build_local_plan(const int32_t* src_metadata, int num_recv_tokens, int num_topk,
                            int num_max_tokens_per_rank, int expanded,
                            int32_t* plan, int plan_width, int num_tokens,
                            const int64_t* topk_idx, int32_t* wtable,
                            deepep_stream_t stream) {
    if (num_recv_tokens < 0 || num_tokens < 0 || num_topk < 1 || num_topk > kMaxWidth || num_max_tokens_per_rank < 1)
        return set_error(DEEPEP_ERR_INVALID_ARG, "invalid plan sizes");
    if ((num_tokens > 0 && plan == nullptr) || (num_recv_tokens > 0 && src_metadata == nullptr))
        return set_error(DEEPEP_ERR_INVALID_ARG, "null plan/metadata");
    if (plan_width != (expanded ? num_topk : 1))
        return set_error(DEEPEP_ERR_INVALID_ARG, "plan width must be num_topk (expanded) or 1");
    if (wtable != nullptr && topk_idx == nullptr)
        return set_error(DEEPEP_ERR_INVALID_ARG, "wtable needs topk_idx");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t n_plan = static_cast<int64_t>(num_tokens) * plan_width;
    if (n_plan > 0)
        hipLaunchKernelGGL(fill_kernel, dim3(static_cast<unsigned>(std::min<int64_t>((n_plan + 255) / 256, 1024))), dim3(256), 0, s,
                           plan, n_plan, -1);
    if (wtable != nullptr && num_tokens > 0) {
        const int64_t n_w = static_cast<int64_t>(num_tokens) * num_topk;
        hipLaunchKernelGGL(fill_kernel, dim3(static_cast<unsigned>(std::min<int64_t>((n_w + 255) / 256, 1024))), dim3(256), 0, s,
                           wtable, n_w, -1);
    }
    if (num_recv_tokens > 0)
        hipLaunchKernelGGL(local_plan_kernel, dim3((num_recv_tokens + 255) / 256), dim3(256), 0, s,
                           src_metadata, num_recv_tokens, num_topk, num_max_tokens_per_rank, expanded,
                           plan, plan_width, num_tokens, topk_idx, wtable);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess)
        return set_error(DEEPEP_ERR_HIP, "plan launch failed: %s", hipGetErrorString(err));
    return DEEPEP_OK;
}

int deepep_set_launch_config(int vec_per_lane, int rows_in_flight) {
    if (vec_per_lane < 0 || vec_per_lane > 2 ||
        (rows_in_flight != 0 && rows_in_flight != 2 && rows_in_flight != 4 && rows_in_flight != 8))
        return set_error(DEEPEP_ERR_INVALID_ARG, "invalid launch configuration (vec_per_lane 0-2, rows_in_flight 0/2/4/8)");
    g_launch_config.store(static_cast<uint32_t>(vec_per_lane) | (static_cast<uint32_t>(rows_in_flight) << 4),
                          std::memory_order_relaxed);
    return DEEPEP_OK;
}

int64_t deepep_combine_buffer_size(int num_max_tokens_per_rank, int hidden, int num_topk,
                                   int num_ranks, int allow_multiple_reduction) {
    // TokenLayout(hidden * 2, 0, num_topk, false) with 32-byte alignment (layout.cuh:179-209),
    // receive slots = min(R, K) with multiple reduction else K (buffer.hpp:616-633); the
    // xGMI fabric is load/store reachable, so no separate send buffer (is_scaleup_nvlink).
    if (num_max_tokens_per_rank <= 0 || hidden <= 0 || num_ranks <= 0)
        return set_error(DEEPEP_ERR_INVALID_ARG, "invalid buffer size arguments");
    if (num_topk == 0) num_topk = 32;
    auto align = [](int64_t x, int64_t a) { return (x + a - 1) / a * a; };
    const int64_t token_bytes = align(int64_t(hidden) * 2, 32) + align(int64_t(num_topk) * 8, 32);
    const int64_t slots = allow_multiple_reduction ? std::min(num_ranks, num_topk) : num_topk;
    return slots * num_max_tokens_per_rank * token_bytes;
}

}  // extern "C"
