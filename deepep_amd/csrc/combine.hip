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
//   * the work is split into items = (output row, column chunk of 64 lanes x 2 x 16 B); one wave64
//     owns one item and a 512-thread workgroup owns 8 consecutive items (7 items per token at
//     hidden 7168), so the grid is ~7K workgroups with no tail imbalance;
//   * the item's row of the slot table (and, weighted, the gating weights) is staged once per
//     workgroup in LDS, one entry per lane; the valid slots are visited in ascending order through
//     the wave's ballot mask (= the reference's compacted slot order);
//   * each lane keeps 8 rows x 2 x 16 B of non-temporal global_load_dwordx4 in flight (every
//     expanded row is read exactly once), accumulates bf16 -> fp32 in registers in the reference's
//     order, rounds once with v_cvt_pk_bf16_f32 (RNE) and writes 2 x 16 B with a write-through
//     (sc1) buffer store.
//   No MFMA: this is an HBM-bound gather + elementwise add (roofline and measurements in DESIGN.md).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include <algorithm>
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

template <bool kNT>
__device__ __forceinline__ void store16(u32x4* p, const u32x4& v) {
    if constexpr (kNT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
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
    int xcd_blocks;              // item kernel: 1 = XCD-contiguous workgroup order (see xcd_block)
    int cap_cus;                 // > 0: persistent grid, at most the workgroups this many CUs hold at once
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

// Workgroups are dealt round-robin to the 8 XCDs (workgroup b runs on XCD b % 8).  With
// xcd_blocks, workgroup b takes block xcd_block(b) instead, so each XCD works through one
// contiguous eighth of the items (its L2 and its share of the memory traffic stay on neighbouring
// tokens) -- a bijection on [0, n) for any n.
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t n) {
    const int64_t per = n / 8, rem = n % 8, xcd = b % 8, idx = b / 8;
    return xcd * per + (xcd < rem ? xcd : rem) + idx;
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

// Output stores: buffer_store_dwordx4 with a per-row descriptor (the hardware range check
// drops the lanes past the row end).  The cache policy is a template parameter; measured on
// MI355X (a round-1 gather probe, 8192 x 7168 x top-8): sc1 (write-through, line dropped from L2)
// 164.6 us, plain 166.2 us, nt 171.8 us for the gather + store pattern; write-only 8.0 / 7.4 /
// 5.9 TB/s.  sc1 is the default.
constexpr int kAuxNT = 2, kAuxSC1 = 16;      // (sc0 = 1)
// Stores into a peer's symmetric window (the xGMI transport) are system-scope write-through
// (sc0 sc1): they must be visible to another GPU once the kernel has completed, whatever MTYPE the
// importing process maps the window with.  Same speed as sc1 (a round-1 load/store policy probe).
constexpr int kAuxSys = 17;
// Write-through streaming (sc1 nt): what the dispatch's blocked expanded copy stores with (dispatch.hip);
// a launch-config option here (store_policy 3), measured against sc1 in tools/kbisect.py.
constexpr int kAuxSC1NT = 18;
// Per unit (launch-config store policy 4): sc1 when the unit reduces >= 3 rows, sc1 nt otherwise.  Phase A at
// EP = 2 / 4 / 8 (tools/kphase_a.py, profiles/r04g_kphasea_*, r04i_kphasea_cache_state.jsonl): back to back
// into the same send rows it beats sc1 nt everywhere by 3.5-12 %, but how much depends on what the caches
// hold: after a 512 MB write flush (dirty lines, as a GEMM that has just written the expert rows leaves them)
// it is 7 % slower at EP = 2 and 4 and equal at EP = 8; sc1 nt is within 2 % in every state.  So phase A keeps
// sc1 nt by default.  Never passed to the store builtin itself.
constexpr int kAuxPerUnit = 1003;     // 1000 + the row threshold

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
    if constexpr (kStoreAux > 1000) {
        if (n >= kStoreAux - 1000) {
#pragma unroll
            for (int v = 0; v < kVPT; ++v)
                __builtin_amdgcn_raw_buffer_store_b128(result[v], orow, vidx[v] * 16, 0, kAuxSC1);
        } else {
#pragma unroll
            for (int v = 0; v < kVPT; ++v)
                __builtin_amdgcn_raw_buffer_store_b128(result[v], orow, vidx[v] * 16, 0, kAuxSC1NT);
        }
    } else {
#pragma unroll
        for (int v = 0; v < kVPT; ++v)
            __builtin_amdgcn_raw_buffer_store_b128(result[v], orow, vidx[v] * 16, 0, kStoreAux);
    }
    if (wlane) store_weight(p, u, out_row, lane, wv);
}

// A workgroup of kWaves waves takes kWaves consecutive items (a virtual block); the unit's slot table
// row (and its gating weights) is staged once per workgroup in LDS (kLDS) or per wave in registers.
// The grid is one workgroup per virtual block, or -- on a CU-budget stream, or when forced -- capped
// at the workgroups the (budgeted) CUs hold at once, each walking virtual blocks grid-stride
// (p.persistent): the waves then stay resident instead of a launch per 2 KiB item.
template <int kMode, bool kWeighted, int kVPT, bool kFull, int kStoreAux, bool kLDS, int kWaves = 4, int kGroup = 8,
          bool kPersistent = false>
__global__ void __launch_bounds__(64 * kWaves)
combine_rows_kernel(const Params p) {
    constexpr int kChunkVecs = 64 * kVPT;
    __shared__ int32_t s_slot[kWaves][kMaxWidth];
    __shared__ float s_w[kWaves][kMaxWidth];
    const int tid = static_cast<int>(threadIdx.x), lane = tid & 63, wave = tid >> 6;
    const int nvec = p.hidden >> 3;                          // 16-byte vectors per row
    const int nchunks = (nvec + kChunkVecs - 1) / kChunkVecs;
    const int64_t items = static_cast<int64_t>(p.num_units) * nchunks;
    const int64_t nblocks = (items + kWaves - 1) / kWaves;
    const int width = p.table == nullptr ? 1 : p.table_width;

    auto load_slot = [&](int64_t u, int j) -> int32_t {
        int32_t s = p.table == nullptr ? static_cast<int32_t>(u) : p.table[u * p.table_stride + j];
        if (s >= p.num_src_rows) {                           // never dereference a bad slot
            if (p.error_flag != nullptr) atomicOr(p.error_flag, 1);
            s = -1;
        }
        return s;
    };

    auto block = [&](int64_t vb) {
        const int64_t blk = p.xcd_blocks ? xcd_block(vb, nblocks) : vb;
        const int64_t it0 = blk * kWaves;
        const int64_t it = it0 + wave;
        int32_t my_slot = -1;
        float my_w = 0.0f;
        if constexpr (kLDS) {
            if (vb != blockIdx.x) __syncthreads();          // the previous block's waves read s_slot
            const int64_t u_first = it0 / nchunks;
            const int nu = static_cast<int>(min(it0 + kWaves - 1, items - 1) / nchunks - u_first) + 1;
            if (tid < nu * width) {                         // nu * width <= kWaves * 32 threads
                const int ul = tid / width, j = tid - ul * width;
                const int32_t s = load_slot(u_first + ul, j);
                s_slot[ul][j] = s;
                if constexpr (kWeighted) s_w[ul][j] = s >= 0 ? p.row_weights[s] : 0.0f;
            }
            __syncthreads();
            if (it < items && lane < width) {
                const int ul = static_cast<int>(it / nchunks - u_first);
                my_slot = s_slot[ul][lane];
                if constexpr (kWeighted) my_w = s_w[ul][lane];
            }
        } else {
            if (it < items && lane < width) {
                my_slot = load_slot(it / nchunks, lane);
                if constexpr (kWeighted) my_w = my_slot >= 0 ? p.row_weights[my_slot] : 0.0f;
            }
        }
        if (it < items)
            combine_item<kMode, kWeighted, kVPT, kFull, kStoreAux, kGroup>(p, it, nchunks, nvec, lane, my_slot, my_w);
    };
    if constexpr (kPersistent && !kLDS) {
        // per-wave items, grid-stride, with the NEXT item's slots loading while this item's rows are
        // gathered: a wave never waits on a slot-table load between two rounds of row loads
        const int64_t stride = static_cast<int64_t>(gridDim.x) * kWaves;
        int64_t it = static_cast<int64_t>(blockIdx.x) * kWaves + wave;
        int32_t next = (it < items && lane < width) ? load_slot(it / nchunks, lane) : -1;
        for (; it < items; it += stride) {
            const int32_t my_slot = next;
            float my_w = 0.0f;
            if constexpr (kWeighted) my_w = my_slot >= 0 ? p.row_weights[my_slot] : 0.0f;
            next = (it + stride < items && lane < width) ? load_slot((it + stride) / nchunks, lane) : -1;
            combine_item<kMode, kWeighted, kVPT, kFull, kStoreAux, kGroup>(p, it, nchunks, nvec, lane, my_slot, my_w);
        }
    } else if constexpr (kPersistent) {
        for (int64_t vb = blockIdx.x; vb < nblocks; vb += gridDim.x) block(vb);
    } else {
        block(blockIdx.x);                          // one virtual block per workgroup
    }
}

// Streaming variant: one wave owns a whole unit (all of its column chunks), for slot tables of at
// most kStreamWidth entries and hidden sizes that are a whole number of chunks.  The unit's slots,
// weights and weight pass-through are handled once; then the chunks are walked in order with the
// loads of chunk c + 1 (every valid row, kVPT x 16 B per lane) issued before chunk c is summed and
// stored, so each wave keeps its rows streaming and writes its output row front to back.  The
// arithmetic per chunk is exactly combine_rows_kernel's (same init, order, rounding), so the two
// kernels give identical bits; measured on config 2: 161.3 us vs 171.3 us on one box
// (DESIGN.md section 3).
constexpr int kStreamWidth = 8;

template <int kMode, bool kWeighted, int kVPT, int kStoreAux>
__global__ void __launch_bounds__(256)
combine_stream_kernel(const Params p) {
    constexpr int kChunkVecs = 64 * kVPT;
    const int lane = static_cast<int>(threadIdx.x) & 63;
    const int nchunks = (p.hidden >> 3) / kChunkVecs;
    const int width = p.table == nullptr ? 1 : p.table_width;
    // one unit per wave, or (a grid capped at the resident capacity) units strided over the waves
    const int64_t stride = static_cast<int64_t>(gridDim.x) * 4;
    // a timed-out barrier (see combine_rows_kernel): no peer stores, NaN output
    const bool aborted = p.error_flag != nullptr && (__hip_atomic_load(p.error_flag, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT) & 2);
    if (aborted && p.out_rows != nullptr) return;
    for (int64_t u = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); u < p.num_units; u += stride) {
    int32_t my_slot = -1;
    float my_w = 0.0f;
    if (lane < width) {
        my_slot = p.table == nullptr ? static_cast<int32_t>(u) : p.table[u * p.table_stride + lane];
        if (my_slot >= p.num_src_rows) {                     // never dereference a bad slot
            if (p.error_flag != nullptr) atomicOr(p.error_flag, 1);
            my_slot = -1;
        }
        if constexpr (kWeighted) my_w = my_slot >= 0 ? p.row_weights[my_slot] : 0.0f;
    }
    if (aborted) my_slot = -1;
    const uint64_t valid = __ballot(my_slot >= 0);
    const int n = __popcll(valid);

    uint16_t* const out_row = p.out_rows != nullptr ? reinterpret_cast<uint16_t*>(checked_row(p, u, lane, true))
                                                     : p.out + u * p.out_stride;
    if (out_row == nullptr) continue;                    // rejected / outside every window: flagged

    const bool wlane = p.num_weights > 0 && lane < p.weights_pad;     // top-k weight pass-through, once per unit
    const float wv = wlane ? pass_through_weight<kWeighted>(p, u, lane, my_slot, my_w) : 0.0f;

    // the valid lanes in ascending order (n <= kStreamWidth) with their row pointers and weights
    const u32x4* rows[kStreamWidth];
    float wj[kStreamWidth];
    {
        uint64_t rem = valid;
#pragma unroll
        for (int j = 0; j < kStreamWidth; ++j) {
            const int l = rem != 0ull ? static_cast<int>(__builtin_ctzll(rem)) : 0;
            const int32_t sj = __builtin_amdgcn_readlane(my_slot, l);
            rows[j] = reinterpret_cast<const u32x4*>(p.src + static_cast<int64_t>(sj < 0 ? 0 : sj) * p.src_stride);
            wj[j] = kWeighted ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_w), l)) : 0.0f;
            rem &= rem - 1ull;
        }
    }
    const bool has_bias0 = p.bias0 != nullptr, has_bias1 = p.bias1 != nullptr;
    const bool has_bias = has_bias0 || has_bias1;
    bool copy_row = false;
    float init;
    if constexpr (kMode == DEEPEP_MODE_LOCAL || kMode == DEEPEP_MODE_FUSED) {
        copy_row = !kWeighted && n == 1;
        init = (!kWeighted && n == 2) ? -0.0f : 0.0f;
    } else {
        init = (!kWeighted && !has_bias && n == 2) ? -0.0f : 0.0f;
    }
    const __amdgpu_buffer_rsrc_t orow = row_rsrc(out_row, p.hidden * 2);

    auto issue = [&](int c, u32x4 (&v)[kStreamWidth][kVPT]) {
#pragma unroll
        for (int j = 0; j < kStreamWidth; ++j)
            if (j < n) {
#pragma unroll
                for (int q = 0; q < kVPT; ++q) v[j][q] = load16<true>(rows[j] + c * kChunkVecs + q * 64 + lane);
            }
    };
    auto finish = [&](int c, u32x4 (&v)[kStreamWidth][kVPT]) {
        u32x4 result[kVPT];
#pragma unroll
        for (int q = 0; q < kVPT; ++q) {
            const int vi = c * kChunkVecs + q * 64 + lane;
            float acc[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = init;
            if constexpr (kMode == DEEPEP_MODE_EPILOGUE) {     // bias0 then bias1 before the partials
                if (has_bias0) acc_add(acc, *(reinterpret_cast<const u32x4*>(p.bias0 + u * p.hidden) + vi));
                if (has_bias1) acc_add(acc, *(reinterpret_cast<const u32x4*>(p.bias1 + u * p.hidden) + vi));
            }
            if (copy_row) {
                result[q] = v[0][q];
            } else {
#pragma unroll
                for (int j = 0; j < kStreamWidth; ++j)
                    if (j < n) {
                        if constexpr (kWeighted) acc_fma(acc, v[j][q], wj[j]);
                        else acc_add(acc, v[j][q]);
                    }
                result[q] = acc_pack(acc);
            }
            if constexpr (kMode == DEEPEP_MODE_FUSED) {
                float a[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) a[e] = 0.0f;
                if (has_bias0) acc_add(a, *(reinterpret_cast<const u32x4*>(p.bias0 + u * p.hidden) + vi));
                if (has_bias1) acc_add(a, *(reinterpret_cast<const u32x4*>(p.bias1 + u * p.hidden) + vi));
                if (n > 0) acc_add(a, result[q]);
                result[q] = acc_pack(a);
            }
            if (aborted) result[q] = (u32x4){0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u};
            __builtin_amdgcn_raw_buffer_store_b128(result[q], orow, vi * 16, 0, kStoreAux);
        }
    };
    u32x4 va[kStreamWidth][kVPT], vb[kStreamWidth][kVPT];
    issue(0, va);
    for (int c = 0; c < nchunks; c += 2) {
        if (c + 1 < nchunks) issue(c + 1, vb);
        finish(c, va);
        if (c + 1 >= nchunks) break;
        if (c + 2 < nchunks) issue(c + 2, va);
        finish(c + 1, vb);
    }
    if (wlane) store_weight(p, u, out_row, lane, wv);
    }
}

int device_cus() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                    hipSuccess)
            cus = 256;
    }
    return cus;
}

// CU-budget streams created by deepep_stream_create_cu_budget (symmetric.hip) and their CU counts:
// a launch on one takes a persistent grid sized to the budget.
std::mutex g_budget_mutex;
std::map<hipStream_t, int> g_budget_cus;

int budget_cus_of(hipStream_t s) {
    if (s == nullptr) return 0;
    std::lock_guard<std::mutex> lock(g_budget_mutex);
    const auto it = g_budget_cus.find(s);
    return it == g_budget_cus.end() ? 0 : it->second;
}

// persistent: the grid is capped at the workgroups the chip holds at once (occupancy x CUs), so
// there is no partial last round of long-lived waves; otherwise one unit per wave
template <int kMode, bool kWeighted, int kVPT, int kAux>
void launch_stream_policy(const Params& p, bool persistent, hipStream_t stream) {
    const auto kernel = combine_stream_kernel<kMode, kWeighted, kVPT, kAux>;
    int64_t blocks = (p.num_units + 3) / 4;
    if (persistent || p.cap_cus > 0) {
        static int per_cu = 0;                    // per template instance
        if (per_cu == 0 && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess)
            per_cu = 1;
        blocks = std::min<int64_t>(blocks, std::max(1, per_cu) * static_cast<int64_t>(p.cap_cus > 0 ? p.cap_cus
                                                                                                    : device_cus()));
    }
    hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream, p);
}

template <int kMode, bool kWeighted, int kVPT>
void launch_stream(const Params& p, int policy, bool persistent, hipStream_t stream) {
    if (policy == 0) launch_stream_policy<kMode, kWeighted, kVPT, 0>(p, persistent, stream);
    else if (policy == 1) launch_stream_policy<kMode, kWeighted, kVPT, kAuxNT>(p, persistent, stream);
    else if (policy == 3) launch_stream_policy<kMode, kWeighted, kVPT, kAuxSys>(p, persistent, stream);
    else launch_stream_policy<kMode, kWeighted, kVPT, kAuxSC1>(p, persistent, stream);
}

struct LaunchConfig {
    int vec_per_lane = 0;        // 0: auto (16-byte vectors per lane per source row and item)
    int stage_lds = -1;          // -1: auto (1 = LDS staging per workgroup, 0 = per-wave registers)
    int store_policy = -1;       // -1: auto (0 plain, 1 nt, 2 sc1)
    int rows_in_flight = 0;      // 0: auto (source rows loaded per lane before accumulating: 2, 4 or 8)
};
LaunchConfig g_config;

// Item kernel vs streaming kernel.  Both give identical bits; which is faster depends on the box
// (config 2: the streaming kernel ran 161 us against 171 us on one MI355X and 187-197 us against
// 175 us on most others).  The item kernel is the default; nothing is timed
// inside a call (a per-shape autotune used to, with a host sync in the call path).
// deepep_set_kernel_choice forces another candidate.
int g_kernel_choice = -1;        // -1 default (the item kernel), else a candidate of launch_combine
int g_last_choice = 0;

template <int kMode, bool kWeighted, int kVPT, bool kFull, int kAux, bool kLDS, int kWaves, int kGroup>
void launch_shape(const Params& p, int64_t items, hipStream_t stream) {
    const int64_t blocks = (items + kWaves - 1) / kWaves;
    if constexpr (kGroup == 8) {
        if (p.cap_cus > 0) {                      // persistent: what the (budgeted) CUs hold at once
            const auto kernel = combine_rows_kernel<kMode, kWeighted, kVPT, kFull, kAux, kLDS, kWaves, kGroup, true>;
            static int per_cu = 0;                // per template instance
            if (per_cu == 0 &&
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 64 * kWaves, 0) != hipSuccess)
                per_cu = 1;
            const int64_t grid = std::min<int64_t>(blocks, static_cast<int64_t>(std::max(1, per_cu)) * p.cap_cus);
            hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(grid)), dim3(64 * kWaves), 0, stream, p);
            return;
        }
    }
    hipLaunchKernelGGL((combine_rows_kernel<kMode, kWeighted, kVPT, kFull, kAux, kLDS, kWaves, kGroup, false>),
                       dim3(static_cast<unsigned>(blocks)), dim3(64 * kWaves), 0, stream, p);
}

// Workgroup shape and rows in flight.  The fused / epilogue reduces (8 rows per token at EP = 1):
// 8 waves x 8 rows in flight (measured on two boxes: 157.5-159.7 us vs 159.6-161.1 us with 4 waves,
// 169 us with 16, 180 us with 12).  Phase A of EP > 1 (1.5 local rows per received token at EP = 8)
// gains from occupancy instead: see launch_combine for the automatic choice.
template <int kMode, bool kWeighted, int kVPT, bool kFull, int kAux>
void launch_lds(const Params& p, bool lds, int waves, int group, hipStream_t stream) {
    const int nvec = p.hidden / 8;
    const int64_t items = static_cast<int64_t>(p.num_units) * ((nvec + 64 * kVPT - 1) / (64 * kVPT));
    if constexpr (kAux == kAuxSC1 || kAux == kAuxSys || kAux == kAuxSC1NT || kAux > 1000) {
        if (lds) {
            if (waves == 8) {
                if (group == 2) launch_shape<kMode, kWeighted, kVPT, kFull, kAux, true, 8, 2>(p, items, stream);
                else if (group == 4) launch_shape<kMode, kWeighted, kVPT, kFull, kAux, true, 8, 4>(p, items, stream);
                else launch_shape<kMode, kWeighted, kVPT, kFull, kAux, true, 8, 8>(p, items, stream);
            } else {
                if (group == 2) launch_shape<kMode, kWeighted, kVPT, kFull, kAux, true, 4, 2>(p, items, stream);
                else if (group == 4) launch_shape<kMode, kWeighted, kVPT, kFull, kAux, true, 4, 4>(p, items, stream);
                else launch_shape<kMode, kWeighted, kVPT, kFull, kAux, true, 4, 8>(p, items, stream);
            }
            return;
        }
    }
    if (lds) launch_shape<kMode, kWeighted, kVPT, kFull, kAux, true, 4, 8>(p, items, stream);
    else launch_shape<kMode, kWeighted, kVPT, kFull, kAux, false, 4, 8>(p, items, stream);
}

struct Shape {
    int vpt, policy, waves, group;
    bool lds;
};

template <int kMode, bool kWeighted, int kVPT, bool kFull>
void launch_aux(const Params& p, const Shape& sh, hipStream_t stream) {
    if (sh.policy == 0) launch_lds<kMode, kWeighted, kVPT, kFull, 0>(p, sh.lds, sh.waves, sh.group, stream);
    else if (sh.policy == 1) launch_lds<kMode, kWeighted, kVPT, kFull, kAuxNT>(p, sh.lds, sh.waves, sh.group, stream);
    else if (sh.policy == 3) launch_lds<kMode, kWeighted, kVPT, kFull, kAuxSys>(p, sh.lds, sh.waves, sh.group, stream);
    else if (sh.policy == 4) launch_lds<kMode, kWeighted, kVPT, kFull, kAuxSC1NT>(p, sh.lds, sh.waves, sh.group, stream);
    else if (sh.policy == 5) {
        if constexpr (kMode == DEEPEP_MODE_LOCAL) launch_lds<kMode, kWeighted, kVPT, kFull, kAuxPerUnit>(p, sh.lds, sh.waves, sh.group, stream);
        else launch_lds<kMode, kWeighted, kVPT, kFull, kAuxSC1>(p, sh.lds, sh.waves, sh.group, stream);
    }
    else launch_lds<kMode, kWeighted, kVPT, kFull, kAuxSC1>(p, sh.lds, sh.waves, sh.group, stream);
}

template <int kMode, bool kWeighted>
void launch_vpt(const Params& p, const Shape& sh, hipStream_t stream) {
    const int nvec = p.hidden / 8;
    if (sh.vpt == 1) {
        if (nvec % 64 == 0) launch_aux<kMode, kWeighted, 1, true>(p, sh, stream);
        else launch_aux<kMode, kWeighted, 1, false>(p, sh, stream);
    } else {
        if (nvec % 128 == 0) launch_aux<kMode, kWeighted, 2, true>(p, sh, stream);
        else launch_aux<kMode, kWeighted, 2, false>(p, sh, stream);
    }
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
    p.xcd_blocks = 0;
    p.cap_cus = 0;
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
    p.xcd_blocks = 0;
    p.cap_cus = 0;
    p.win_bases = window_bases;
    p.win_count = num_windows;
    p.win_limit = static_cast<uint64_t>(window_bytes - row_extent);
    return launch_combine(DEEPEP_MODE_LOCAL, weighted, p, stream);
}

}  // extern "C"

namespace {

int launch_combine(int mode, int weighted, const Params& p_in, deepep_stream_t stream) {
    Params p = p_in;
    // Launch shape: one wave per (unit, 64 x vpt x 16-byte column chunk) item; at hidden 7168 a
    // token is 7 items of 2 KiB per source row.
    const int nvec = p.hidden / 8;
    Shape sh;
    sh.vpt = g_config.vec_per_lane > 0 ? g_config.vec_per_lane : (nvec >= 128 ? 2 : 1);
    if (sh.vpt != 1 && sh.vpt != 2) sh.vpt = 2;
    sh.lds = g_config.stage_lds >= 0 ? g_config.stage_lds != 0 : true;
    // store policies: 0 plain, 1 nt, 2 sc1 (fused / epilogue default), 3 system scope (peer windows),
    // 4 sc1 nt (phase A default), 5 per unit (kAuxPerUnit; opt-in).  Phase A's packed send rows are written
    // once and read back only by the exchange, so they stream past L2 (sc1 nt): EP = 8, back to back, 248.9 vs
    // 251.4 us with sc1 (profiles/r04a_kphasea.jsonl), and the only policy within 2 % of the best in every
    // cache state measured (r04i_kphasea_cache_state.jsonl).  The fused and epilogue reduces keep sc1 (their
    // output is written in token order; sc1 is best or tied in every cache state, r04i_kshapes_cache_state.jsonl).
    const int auto_policy = mode == DEEPEP_MODE_LOCAL ? 4 : 2;
    sh.policy = p.out_rows != nullptr ? 3 : (g_config.store_policy == 4 ? 5 : g_config.store_policy == 3 ? 4 :
                                              (g_config.store_policy >= 0 ? g_config.store_policy : auto_policy));
    // units_per_block 4 / 8 forces the workgroup shape; 0 = automatic
    sh.waves = p.units_per_block == 4 ? 4 : (p.units_per_block == 8 ? 8 : (mode == DEEPEP_MODE_LOCAL ? 4 : 8));
    // rows in flight per lane: 8 for the fused / epilogue reduces (8 rows per token at EP = 1), 4 for
    // phase A (about 1.5 local rows per received token at EP = 8: 64 VGPRs and 8 waves per SIMD beat
    // deeper per-wave loads, tools/kphase.py 252-254 vs 256-260 us)
    // A unit never has more valid rows than its table is wide, so the rows in flight are capped at the
    // width rounded up to 2 / 4: registers for rows that never come only cost occupancy (top-2, config-2
    // shape otherwise: 33.7 vs 40.1 us; top-4: 93.5 vs 95.9 us; tools/kshapes.py, profiles/r04e_kshapes_*, r04f_kshapes_*).
    const int width = p.table == nullptr ? 1 : p.table_width;
    const int width_cap = width <= 2 ? 2 : (width <= 4 ? 4 : 8);
    sh.group = g_config.rows_in_flight > 0 ? g_config.rows_in_flight
                                           : std::min(mode == DEEPEP_MODE_LOCAL ? 4 : 8, width_cap);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // A forced streaming kernel (one wave per unit, chunks pipelined) applies only when the shape is
    // automatic: an explicit units_per_block / LDS / rows-in-flight setting selects the item kernel
    // (which also serves tables wider than kStreamWidth and ragged hidden sizes).
    const bool stream_ok = (p.table == nullptr || p.table_width <= kStreamWidth) && nvec % (64 * sh.vpt) == 0 &&
                           p.units_per_block == 0 && g_config.stage_lds < 0 && g_config.rows_in_flight == 0;
    auto launch_items = [&]() {
        if (mode == DEEPEP_MODE_LOCAL) {
            if (weighted) launch_vpt<DEEPEP_MODE_LOCAL, true>(p, sh, s);
            else launch_vpt<DEEPEP_MODE_LOCAL, false>(p, sh, s);
        } else if (mode == DEEPEP_MODE_EPILOGUE) {
            if (weighted) launch_vpt<DEEPEP_MODE_EPILOGUE, true>(p, sh, s);
            else launch_vpt<DEEPEP_MODE_EPILOGUE, false>(p, sh, s);
        } else {
            if (weighted) launch_vpt<DEEPEP_MODE_FUSED, true>(p, sh, s);
            else launch_vpt<DEEPEP_MODE_FUSED, false>(p, sh, s);
        }
    };
    auto launch_streaming = [&](int vpt, bool persistent) {
#define DEEPEP_STREAM(M, W) \
        (vpt == 1 ? launch_stream<M, W, 1>(p, sh.policy, persistent, s) \
                  : launch_stream<M, W, 2>(p, sh.policy, persistent, s))
        if (mode == DEEPEP_MODE_LOCAL) {
            if (weighted) DEEPEP_STREAM(DEEPEP_MODE_LOCAL, true); else DEEPEP_STREAM(DEEPEP_MODE_LOCAL, false);
        } else if (mode == DEEPEP_MODE_EPILOGUE) {
            if (weighted) DEEPEP_STREAM(DEEPEP_MODE_EPILOGUE, true); else DEEPEP_STREAM(DEEPEP_MODE_EPILOGUE, false);
        } else {
            if (weighted) DEEPEP_STREAM(DEEPEP_MODE_FUSED, true); else DEEPEP_STREAM(DEEPEP_MODE_FUSED, false);
        }
#undef DEEPEP_STREAM
    };
    // candidates: 0 item kernel, 1 streaming kernel (sh.vpt vectors per lane), 2 streaming kernel with
    // 1 vector per lane (half the registers, more waves per SIMD), 3 streaming kernel on a persistent
    // grid (sh.vpt vectors per lane)
    // 4: the item kernel with XCD-contiguous workgroup order -- it lost
    // on every measurement (config 2 188.4 vs 175.3 us, EP = 8 phase A 318 vs 301, phase B 126 vs
    // 115): neighbouring items spread over all XCDs stream better
    // 5: the item kernel on a persistent grid (as many workgroups as the chip holds at once)
    // 6: the item kernel on its full grid (what the default does on a CU-budget stream too)
    // On a CU-budget stream the item kernel keeps its full grid (the CU mask alone holds it to the
    // budget) with 4 rows in flight per lane: 64 VGPRs, 8 waves per SIMD, so a budgeted CU keeps more
    // bytes in flight than with 8 rows at 5 waves (config 2, profiles/r02n_kcu2.jsonl:
    // 128 CUs 208 vs 235 us on a persistent grid, 32 CUs 603 vs 661 us; the whole chip is unchanged);
    // the streaming kernels and the forced persistent item kernel take a persistent grid sized to it.
    const int budget = budget_cus_of(s);
    if (budget > 0 && g_config.rows_in_flight == 0) sh.group = std::min(4, width_cap);
    // The EP = 1 fused reduce over wide tables (top-k >= 5) and rows of at least 256 vectors: 1 vector per
    // lane (1 KiB chunks), 2 rows in flight, 4-wave workgroups -- few registers, many waves.  Three boxes,
    // same output buffer, medians of 3-5 interleaved rounds (tools/kshapes.py, profiles/r04e_kshapes_*, r04f_kshapes_*):
    // config 2 172.4 / 171.1 / 173.9 us vs 175.1 / 173.9 / 175.5 (-0.9 to -1.6 %), hidden 4096 -0.9 to
    // -2.8 %, hidden 2048 -1.4 to -2.2 %, hidden 5120 x top-6 -1.7 to -2.5 %.  Not for phase A (LOCAL:
    // 295 vs 247 us, tools/kphase_a.py) nor narrower rows (hidden 1024: 2 vectors, 4 rows, 8 waves win).
    const bool fused_wide = mode == DEEPEP_MODE_FUSED && width >= 5 && nvec >= 256 && budget == 0 &&
                            g_config.vec_per_lane == 0 && g_config.rows_in_flight == 0 && g_config.stage_lds < 0 &&
                            p.units_per_block == 0;
    // hidden 1024 (one 2 KiB item per row): 4 rows in flight, 23.7 / 23.6 vs 25.1 / 25.2 us on two boxes
    const bool fused_narrow = mode == DEEPEP_MODE_FUSED && width >= 5 && nvec >= 128 && nvec < 256 && budget == 0 &&
                              g_config.vec_per_lane == 0 && g_config.rows_in_flight == 0 && g_config.stage_lds < 0 &&
                              p.units_per_block == 0;
    auto launch_choice = [&](int c) {
        if (c == 0 && fused_wide) {
            sh.vpt = 1;
            sh.group = 2;
            sh.waves = 4;
        } else if (c == 0 && fused_narrow) {
            sh.group = 4;
        }
        p.xcd_blocks = c == 4 ? 1 : 0;
        p.cap_cus = (c == 0 || c == 4 || c == 6) ? 0 : (budget > 0 ? budget : (c == 5 ? device_cus() : 0));
        // the persistent item grid exists for 8 rows in flight only (launch_shape): a capped launch always
        // takes it, so a forced choice 5 never silently runs the full grid
        if (p.cap_cus > 0 && (c == 0 || c == 4 || c == 5 || c == 6)) sh.group = 8;
        // a persistent grid stages slots per wave (no workgroup barrier between a wave's items), so
        // each wave streams at its own pace
        sh.lds = g_config.stage_lds >= 0 ? g_config.stage_lds != 0 : p.cap_cus == 0;
        if (c == 0 || c == 4 || c == 5 || c == 6) launch_items();
        else launch_streaming(c == 2 ? 1 : sh.vpt, c == 3);
    };
    const int forced = g_kernel_choice;
    const int choice = (forced == 5 || forced == 6) ? forced : ((stream_ok && forced >= 0) ? forced : 0);
    g_last_choice = choice;
    launch_choice(choice);
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

int deepep_set_kernel_choice(int choice) {
    if (choice < -1 || choice > 6) return set_error(DEEPEP_ERR_INVALID_ARG, "kernel choice must be -1 or 0..6");
    g_kernel_choice = choice;
    return DEEPEP_OK;
}

int deepep_last_kernel_choice(void) { return g_last_choice; }

int deepep_set_launch_config(int vec_per_lane, int stage_lds, int store_policy, int rows_in_flight) {
    if (vec_per_lane < 0 || vec_per_lane > 2 || stage_lds < -1 || stage_lds > 1 || store_policy < -1 ||
        store_policy > 4 || (rows_in_flight != 0 && rows_in_flight != 2 && rows_in_flight != 4 && rows_in_flight != 8))
        return set_error(DEEPEP_ERR_INVALID_ARG, "invalid launch configuration");
    g_config.vec_per_lane = vec_per_lane;
    g_config.stage_lds = stage_lds;
    g_config.store_policy = store_policy;
    g_config.rows_in_flight = rows_in_flight;
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
