/*
 * oracle/combine_ref.c -- CPU restatement of DeepEP's combine reduction.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in deepep_amd/ links, loads or calls this
 * file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * it, and only as the checker.  Parity of this restatement is pinned against
 * golden vectors produced by the reference's own pure-torch oracle
 * (deep_ep/utils/refs.py), see tests/golden/gen_golden.py and
 * tests/test_oracle_golden.py.
 *
 * The arithmetic restated here is the one the reference CUDA kernels perform
 * (all paths relative to /root/reference):
 *
 *   phase A  deep_ep/include/deep_ep/impls/combine.cuh:114-213
 *            (per received token: copy when exactly one local top-k slot is
 *            valid, otherwise combine_reduce over the compacted valid slots)
 *   phase B  deep_ep/include/deep_ep/impls/combine_reduce_epilogue.cuh:62-142
 *            (per output token: dedup ranks with the highest top-k lane as
 *            master, reduce the per-rank partials plus bias, gather weights)
 *   core     deep_ep/include/deep_ep/impls/combine_utils.cuh:55-170
 *            (bf16 "hadd bypass" when no bias and <= 2 valid sources,
 *            otherwise fp32 accumulate bias0, bias1, then sources in
 *            ascending order, one round-to-nearest-even to bf16)
 *   weighted csrc/kernels/legacy/internode_ll.cu:1072-1135 and :704-711
 *            (legacy low-latency combine: acc = sum_k fma(y_k, w_k, acc) over
 *            valid k ascending, starting from 0.0f, one rounding to bf16)
 *
 * Compiled with -O2 -ffp-contract=off so that every float '+' is one IEEE
 * binary32 addition; fmaf() is the correctly rounded fused multiply-add.
 */
#include <stdint.h>
#include <string.h>
#include <math.h>

/* ------------------------------------------------------------------ bf16 */

static inline float bf16_to_f32(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* Round-to-nearest-even, the rounding of __float22bfloat162_rn
 * (combine_utils.cuh:162).  NaNs are quieted (payload kept), which is what
 * gfx950's v_cvt_pk_bf16_f32 does; CUDA returns a canonical NaN instead, so
 * NaN payloads are outside the parity contract. */
static inline uint16_t f32_to_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u)
        return (uint16_t)((u >> 16) | 0x0040u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

/* bf16 + bf16 as __hadd2 on nv_bfloat162 (combine_utils.cuh:88-95): the exact
 * sum rounded once to bf16.  Rounding the binary32 sum instead is identical
 * because 24 >= 2*8 + 2 (double rounding is innocuous for addition). */
static inline uint16_t bf16_hadd(uint16_t a, uint16_t b) {
    return f32_to_bf16(bf16_to_f32(a) + bf16_to_f32(b));
}

uint16_t oracle_f32_to_bf16(float f) { return f32_to_bf16(f); }
float oracle_bf16_to_f32(uint16_t h) { return bf16_to_f32(h); }

/* ---------------------------------------------------------- combine_reduce
 * Reduce `n` source rows (already compacted, ascending order) of `hidden`
 * bf16 into dst, with optional bias rows.  Restates combine_utils.cuh:55-170
 * with kNumValidTopk = `width` (the size of the compacted slot array, which
 * decides whether the hadd bypass applies: `width <= 2 or slot[2] < 0`). */
static void combine_reduce_row(const uint16_t* const* src, int n, int width,
                               const uint16_t* bias0, const uint16_t* bias1,
                               int hidden, uint16_t* dst) {
    const int bypass = (bias0 == NULL && bias1 == NULL) && (width <= 2 || n <= 2);
    if (bypass) {
        /* values_0/values_1 are loaded with a >= 0 predicate, zeros otherwise
         * (ptx::ldg_with_gez_pred, ptx.cuh:176-188). */
        for (int h = 0; h < hidden; ++h) {
            uint16_t v0 = n > 0 ? src[0][h] : 0;
            uint16_t v1 = (width > 1 && n > 1) ? src[1][h] : 0;
            dst[h] = bf16_hadd(v0, v1);
        }
        return;
    }
    for (int h = 0; h < hidden; ++h) {
        float acc = 0.0f;                       /* float2 reduced[...] = {} */
        if (bias0) acc += bf16_to_f32(bias0[h]);
        if (bias1) acc += bf16_to_f32(bias1[h]);
        for (int j = 0; j < n; ++j)
            acc += bf16_to_f32(src[j][h]);
        dst[h] = f32_to_bf16(acc);
    }
}

/* Weighted reduction, legacy low-latency semantics (internode_ll.cu:704-711,
 * 1080-1125): combined_values start at 0.0f and accumulate
 * float(y) * weight; nvcc contracts that into one FMA (default
 * -fmad=true), restated here with fmaf(). */
static void weighted_reduce_row_bias(const uint16_t* const* src, const float* w, int n,
                                     const uint16_t* bias0, const uint16_t* bias1,
                                     int hidden, uint16_t* dst) {
    for (int h = 0; h < hidden; ++h) {
        float acc = 0.0f;
        if (bias0) acc += bf16_to_f32(bias0[h]);
        if (bias1) acc += bf16_to_f32(bias1[h]);
        for (int j = 0; j < n; ++j)
            acc = fmaf(bf16_to_f32(src[j][h]), w[j], acc);
        dst[h] = f32_to_bf16(acc);
    }
}

static void weighted_reduce_row(const uint16_t* const* src, const float* w, int n,
                                int hidden, uint16_t* dst) {
    weighted_reduce_row_bias(src, w, n, NULL, NULL, hidden, dst);
}

/* ------------------------------------------------------------- phase A
 * For each received token i (combine.cuh:86-237):
 *   expanded:   slots = src_metadata[i*(K+2) + 2 + k], k < K
 *               popc(valid) == 1 -> copy that row         (:136-156 no_local_reduce)
 *               otherwise        -> combine_reduce over the valid slots in
 *                                   ascending k (:157-176, width = K)
 *   not expanded: copy x[i]                                 (:134-156)
 * The result row is written to out[i].  Weights (pass-through, :215-226):
 *   expanded:   out_w[i*K + k] = slot_k >= 0 ? topk_weights[slot_k] : 0
 *   otherwise:  out_w[i*K + k] = topk_weights[i*K + k]
 * `weighted` = 1 selects the legacy weighted arithmetic for the reduction
 * (expanded only): row_k is scaled by topk_weights[slot_k].
 * Returns 0, or -1 on an out-of-range slot. */
int oracle_combine_phase_a(const uint16_t* x, int64_t num_x_rows, int hidden,
                           const int32_t* src_metadata, int num_recv_tokens, int num_topk,
                           int expanded, const float* topk_weights, int weighted,
                           uint16_t* out, float* out_w) {
    const int K = num_topk, stride = K + 2;
    const uint16_t* src[64];
    float w[64];
    if (K > 64) return -1;
    for (int i = 0; i < num_recv_tokens; ++i) {
        uint16_t* dst = out + (int64_t)i * hidden;
        if (!expanded) {
            if (i >= num_x_rows) return -1;
            memcpy(dst, x + (int64_t)i * hidden, (size_t)hidden * 2);
            if (out_w && topk_weights)
                for (int k = 0; k < K; ++k) out_w[(int64_t)i * K + k] = topk_weights[(int64_t)i * K + k];
            continue;
        }
        int n = 0;
        for (int k = 0; k < K; ++k) {
            const int32_t s = src_metadata[(int64_t)i * stride + 2 + k];
            if (s >= 0) {
                if (s >= num_x_rows) return -1;
                src[n] = x + (int64_t)s * hidden;
                w[n] = topk_weights ? topk_weights[s] : 0.0f;
                ++n;
            }
            if (out_w && topk_weights)
                out_w[(int64_t)i * K + k] = s >= 0 ? topk_weights[s] : 0.0f;
        }
        if (weighted) {
            weighted_reduce_row(src, w, n, hidden, dst);
        } else if (n == 1) {
            memcpy(dst, src[0], (size_t)hidden * 2);
        } else {
            combine_reduce_row(src, n, K, NULL, NULL, hidden, dst);
        }
    }
    return 0;
}

/* ------------------------------------------------------------- phase B
 * combine_reduce_epilogue_impl (combine_reduce_epilogue.cuh:62-142) for the
 * single-node case (kNumScaleoutRanks == 1).
 *   recv:       [num_slots][num_max_tokens][hidden] bf16, the symmetric
 *               receive buffer, slot = rank (rank layout) or top-k lane
 *   recv_w:     [num_slots][num_max_tokens][K] fp32 (may be NULL)
 *   rank_layout: use_rank_layout() (combine_utils.cuh:8-13)
 *   dedup:      0 only for expanded + !allow_multiple_reduction (:66-68)
 * Returns 0, or -1 on inconsistent arguments. */
int oracle_combine_phase_b(const uint16_t* recv, const float* recv_w,
                           int num_slots, int num_max_tokens,
                           const int64_t* topk_idx, int num_tokens, int num_topk,
                           int num_experts, int num_ranks, int rank_layout, int dedup,
                           const uint16_t* bias0, const uint16_t* bias1, int hidden,
                           uint16_t* combined, float* combined_w) {
    const int K = num_topk;
    if (K > 32 || num_experts % num_ranks) return -1;
    const int experts_per_rank = num_experts / num_ranks;
    const int width = rank_layout ? (num_ranks < K ? num_ranks : K) : K;   /* kNumTokensInLayout */
    const uint16_t* src[64];
    int rank_of[32], valid[32];
    for (int t = 0; t < num_tokens; ++t) {
        for (int k = 0; k < K; ++k) {
            const int64_t e = topk_idx[(int64_t)t * K + k];
            rank_of[k] = e >= 0 ? (int)(e / experts_per_rank) : -1;
        }
        /* reduce_valid_mask: lanes that are the highest lane holding their
         * key (ptx::deduplicate = get_master_lane_idx(match) == lane), and a
         * valid rank.  Lanes >= K hold -1 and never win for a valid key. */
        for (int k = 0; k < K; ++k) {
            int is_master = 1;
            if (dedup)
                for (int j = k + 1; j < K; ++j)
                    if (rank_of[j] == rank_of[k]) { is_master = 0; break; }
            valid[k] = is_master && rank_of[k] >= 0;
        }
        /* compute_topk_slots (combine_utils.cuh:41-53): ascending lanes,
         * slot = rank (rank layout) or the lane itself. */
        int n = 0;
        for (int k = 0; k < K && n < width; ++k) {
            if (!valid[k]) continue;
            const int slot = rank_layout ? rank_of[k] : k;
            if (slot >= num_slots) return -1;
            src[n++] = recv + ((int64_t)slot * num_max_tokens + t) * hidden;
        }
        combine_reduce_row(src, n, width,
                           bias0 ? bias0 + (int64_t)t * hidden : NULL,
                           bias1 ? bias1 + (int64_t)t * hidden : NULL,
                           hidden, combined + (int64_t)t * hidden);
        if (combined_w) {
            for (int k = 0; k < K; ++k) {
                float value = 0.0f;
                if (rank_of[k] >= 0 && recv_w) {
                    int master = k;   /* highest lane with the same rank value */
                    for (int j = K - 1; j > k; --j)
                        if (rank_of[j] == rank_of[k]) { master = j; break; }
                    const int slot = rank_layout ? rank_of[k] : master;
                    value = recv_w[((int64_t)slot * num_max_tokens + t) * K + k];
                }
                combined_w[(int64_t)t * K + k] = value;
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------ legacy weighted
 * low_latency_combine's reduction (internode_ll.cu:1072-1135): y is
 * [num_tokens][num_topk][hidden] (the expert outputs of each token, as the
 * source rank receives them), w is [num_tokens][num_topk]. */
int oracle_combine_weighted_ll(const uint16_t* y, const int64_t* topk_idx, const float* w,
                               int num_tokens, int num_topk, int hidden, uint16_t* out) {
    const uint16_t* src[64];
    float ws[64];
    if (num_topk > 64) return -1;
    for (int t = 0; t < num_tokens; ++t) {
        int n = 0;
        for (int k = 0; k < num_topk; ++k) {
            if (topk_idx[(int64_t)t * num_topk + k] < 0) continue;
            src[n] = y + ((int64_t)t * num_topk + k) * hidden;
            ws[n] = w[(int64_t)t * num_topk + k];
            ++n;
        }
        weighted_reduce_row(src, ws, n, hidden, out + (int64_t)t * hidden);
    }
    return 0;
}

/* --------------------------------------------------- table-driven rows
 * The same per-row arithmetic, driven by the slot tables the product's C-ABI
 * takes (include/deepep_amd.h, deepep_combine_reduce) instead of the
 * reference's receive buffer.  Used by the CPU orchestration tests as a
 * stand-in kernel provider; its semantics are the phase-A/phase-B rules above
 * (mode 0 = phase A, 1 = phase B with width = table width, 2 = phase A then
 * phase B over one slot).  Pointers are host pointers.
 * Weighted mode 1 (the single-reduction weighted combine: every expanded row
 * sent unreduced, one reduction at the source rank) is the legacy low-latency
 * sum with the bias in front: acc = 0 + bias0 + bias1, then acc = fma(y_j, w_j,
 * acc) over the valid rows, one rounding -- without bias exactly
 * internode_ll.cu:1072-1135. */
int oracle_combine_rows(int mode, int weighted,
                        const uint16_t* src, int64_t num_src_rows, int64_t src_stride,
                        const int32_t* table, int64_t table_stride, int table_width,
                        const float* row_weights,
                        const uint16_t* bias0, const uint16_t* bias1,
                        uint16_t* out, int64_t out_stride, int num_units, int hidden,
                        const int32_t* wtable, int64_t wtable_stride,
                        const float* wsrc, float* out_weights, int num_weights,
                        int64_t out_weights_stride) {
    const uint16_t* rows[64];
    float w[64];
    uint16_t partial[65536];
    if (table_width > 64 || hidden > 65536) return -1;
    const int width = table ? table_width : 1;
    for (int u = 0; u < num_units; ++u) {
        int n = 0;
        for (int j = 0; j < width; ++j) {
            const int64_t s = table ? table[(int64_t)u * table_stride + j] : u;
            if (s < 0) continue;
            if (s >= num_src_rows) return -1;
            rows[n] = src + s * src_stride;
            w[n] = weighted ? row_weights[s] : 0.0f;
            ++n;
        }
        uint16_t* dst = out + (int64_t)u * out_stride;
        const uint16_t* b0 = bias0 ? bias0 + (int64_t)u * hidden : NULL;
        const uint16_t* b1 = bias1 ? bias1 + (int64_t)u * hidden : NULL;
        if (mode == 1) {
            if (weighted) weighted_reduce_row_bias(rows, w, n, b0, b1, hidden, dst);
            else combine_reduce_row(rows, n, width, b0, b1, hidden, dst);
        } else {
            uint16_t* a = mode == 2 ? partial : dst;
            if (weighted) weighted_reduce_row(rows, w, n, hidden, a);
            else if (n == 1) memcpy(a, rows[0], (size_t)hidden * 2);
            else combine_reduce_row(rows, n, width, NULL, NULL, hidden, a);
            if (mode == 2) {
                const uint16_t* one[1] = {partial};
                combine_reduce_row(one, n > 0 ? 1 : 0, 1, b0, b1, hidden, dst);
            }
        }
        if (out_weights) {
            for (int k = 0; k < num_weights; ++k) {
                const int64_t i = wtable ? wtable[(int64_t)u * wtable_stride + k] : (int64_t)u * num_weights + k;
                out_weights[(int64_t)u * (out_weights_stride ? out_weights_stride : num_weights) + k] =
                    i >= 0 ? wsrc[i] : 0.0f;
            }
        }
    }
    return 0;
}
