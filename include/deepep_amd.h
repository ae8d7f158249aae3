/*
 * deepep_amd.h -- C-ABI of libdeepep_amd.so, the MI355X (gfx950) combine reduction.
 *
 * Plain C: raw device pointers, sizes and a hipStream_t; no torch types.  Every
 * entry point returns DEEPEP_OK (0) or a negative DEEPEP_ERR_* code; the message
 * of the last failure on the calling thread is available from
 * deepep_amd_last_error().  The Python host layer (deepep_amd/_lib.py) turns a
 * non-zero code into RuntimeError, which is what the reference raises for a
 * failed EP_HOST_ASSERT (EPException -> RuntimeError,
 * deep_ep/include/deep_ep/common/exception.cuh:11-37 in /root/reference).
 *
 * Reference interfaces replaced (paths relative to /root/reference):
 *   deepep_combine_reduce(mode = DEEPEP_MODE_LOCAL)
 *       launch_combine / combine_impl, the per-received-token local reduce
 *       (csrc/kernels/elastic/combine.hpp:114-193,
 *        deep_ep/include/deep_ep/impls/combine.cuh:28-243)
 *   deepep_combine_reduce(mode = DEEPEP_MODE_EPILOGUE)
 *       launch_combine_reduce_epilogue / combine_reduce_epilogue_impl
 *       (csrc/kernels/elastic/combine.hpp:248-287,
 *        deep_ep/include/deep_ep/impls/combine_reduce_epilogue.cuh:24-143)
 *   deepep_combine_reduce(mode = DEEPEP_MODE_FUSED)
 *       both of the above at EP = 1, fused into one pass (no receive buffer)
 *   deepep_build_local_plan
 *       the token -> slot lookup that combine_reduce_epilogue_impl performs per
 *       token through the symmetric receive buffer (combine_reduce_epilogue.cuh:62-95),
 *       materialised once per handle
 *   deepep_combine_buffer_size
 *       ElasticBuffer::get_combine_buffer_size (csrc/elastic/buffer.hpp:616-650)
 * The Python-facing runtime call these serve is _C.ElasticBuffer.combine
 * (csrc/elastic/buffer.hpp:1179-1343), re-implemented in deepep_amd/buffer.py.
 */
#ifndef DEEPEP_AMD_H
#define DEEPEP_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* deepep_stream_t;   /* == hipStream_t */

#define DEEPEP_AMD_ABI_VERSION 2

#define DEEPEP_OK               0
#define DEEPEP_ERR_INVALID_ARG  (-1)
#define DEEPEP_ERR_UNSUPPORTED  (-2)
#define DEEPEP_ERR_HIP          (-3)

/* Reduction modes of deepep_combine_reduce. */
#define DEEPEP_MODE_LOCAL     0   /* phase A: copy if 1 valid slot, hadd if 2, else fp32 sum   */
#define DEEPEP_MODE_EPILOGUE  1   /* phase B: bias0 + bias1 + partials (hadd bypass w/o bias)    */
#define DEEPEP_MODE_FUSED     2   /* phase A then phase B over the single partial (EP = 1)       */

int deepep_amd_abi_version(void);
const char* deepep_amd_last_error(void);

/*
 * Per unit u in [0, num_units): gather the source rows listed in
 * table[u * table_stride + j] (j < table_width, entries < 0 are skipped; a NULL
 * table means the single row u), reduce them in ascending j in fp32 with the
 * reference's rounding rules for `mode`, and write one bf16 row to
 * out + u * out_row_stride.
 *
 *   src            bf16 [num_src_rows][src_row_stride], rows 16-byte aligned
 *   hidden         elements per row; hidden % 8 == 0
 *   weighted       0: plain sum (ElasticBuffer semantics);
 *                  1: row j scaled by row_weights[slot_j] with an fp32 fma chain
 *                     (legacy low_latency_combine semantics, csrc/kernels/legacy/
 *                     internode_ll.cu:1072-1135); modes LOCAL and FUSED only
 *   bias0, bias1   bf16 [num_units][hidden] or NULL (modes EPILOGUE and FUSED)
 *   out_weights    fp32 rows of out_weights_stride floats (0 = num_weights) or NULL: top-k
 *                  weight pass-through, written once per unit:
 *                  out_weights[u*out_weights_stride + k] = (i = wtable ? wtable[u*wtable_stride + k]
 *                                                             : u*num_weights + k) >= 0 ? wsrc[i] : 0
 *                  (a stride lets the weights ride in the tail of packed exchange rows)
 *   units_per_block  reserved (0); the launch tiles (row, column-chunk) items, 4 per workgroup
 *   error_flag     device int or NULL; set to 1 when a slot is >= num_src_rows
 *                  (such slots are skipped, never dereferenced)
 */
int deepep_combine_reduce(int mode, int weighted,
                          const void* src, int64_t num_src_rows, int64_t src_row_stride,
                          const int32_t* table, int64_t table_stride, int table_width,
                          const float* row_weights,
                          const void* bias0, const void* bias1,
                          void* out, int64_t out_row_stride,
                          int num_units, int hidden,
                          const int32_t* wtable, int64_t wtable_stride,
                          const float* wsrc, float* out_weights, int num_weights,
                          int64_t out_weights_stride,
                          int units_per_block, int32_t* error_flag,
                          deepep_stream_t stream);

/*
 * Token-major slot table for the EP = 1 fused path, from the handle's
 * recv_src_metadata ([num_recv_tokens][num_topk + 2] int32, column 0 =
 * src_rank * num_max_tokens_per_rank + src_token, columns 2.. = expanded slots).
 *   expanded = 1: plan[t][k] = metadata slot k of the token received from t, else -1
 *   expanded = 0: plan[t][0] = i (the received row of t), else -1
 * plan is [num_tokens][plan_width] int32 (plan_width = num_topk or 1) and is fully
 * written.  When wtable is not NULL ([num_tokens][num_topk]) it receives the
 * weight-source index of the non-expanded pass-through: i*num_topk + k where
 * topk_idx[t][k] >= 0, else -1 (topk_idx is int64 [num_tokens][num_topk]).
 */
int deepep_build_local_plan(const int32_t* src_metadata, int num_recv_tokens, int num_topk,
                            int num_max_tokens_per_rank, int expanded,
                            int32_t* plan, int plan_width, int num_tokens,
                            const int64_t* topk_idx, int32_t* wtable,
                            deepep_stream_t stream);

/*
 * Tuning / diagnostics (process-global; 0 or -1 = automatic, the default):
 *   vec_per_lane   16-byte vectors each lane loads per source row and item (1 or 2)
 *   stage_lds      1: stage the slot table / weights per workgroup in LDS; 0: per wave in registers
 *   store_policy   output store cache policy: 0 plain, 1 nt, 2 sc1 (write-through)
 * The results are identical for every configuration; only the speed changes.
 */
int deepep_set_launch_config(int vec_per_lane, int stage_lds, int store_policy);

/* ElasticBuffer::get_combine_buffer_size for one node (num_scaleout_ranks == 1). */
int64_t deepep_combine_buffer_size(int num_max_tokens_per_rank, int hidden, int num_topk,
                                   int num_ranks, int allow_multiple_reduction);

#ifdef __cplusplus
}
#endif

#endif /* DEEPEP_AMD_H */
