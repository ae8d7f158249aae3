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
 *   deepep_dispatch_notify (or _route / _expert_counts) / _pack   (the handle producer, send side)
 *       dispatch_impl's notify, slot assignment and token push
 *       (deep_ep/include/deep_ep/impls/dispatch.cuh:79-258, 336-392)
 *   deepep_dispatch_count / _scan / _slots / _copy   (receive side)
 *       dispatch_copy_epilogue_impl (deep_ep/include/deep_ep/impls/dispatch_copy_epilogue.cuh:11-323)
 *   deepep_route_block_counts / deepep_plan_expert / deepep_plan_source   (EP > 1 combine plan)
 *       the addressing combine_impl and combine_reduce_epilogue_impl derive inside every launch
 *       (combine.cuh:96-106, combine_reduce_epilogue.cuh:62-95), built once per handle on the device
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

#define DEEPEP_AMD_ABI_VERSION 14

#define DEEPEP_OK               0
#define DEEPEP_ERR_INVALID_ARG  (-1)
#define DEEPEP_ERR_UNSUPPORTED  (-2)
#define DEEPEP_ERR_HIP          (-3)

/* Error record: the error_flag of the window paths (the scatter, plan_expert, the xGMI dispatch pack)
 * points at DEEPEP_ERROR_RECORD_INTS device ints.  [0] = flag bits: 1 = a slot / unit was rejected
 * (skipped, never dereferenced), 2 = a window barrier timed out, 4 = a computed window address fell
 * outside every window (nothing stored there).  [1..7] = the first fault with bit 4 or a rejected plan
 * entry: [1] kind (DEEPEP_FAULT_*), [2] unit / token / row, [3] rank / lane, [4] address low 32 bits,
 * [5] address high 32 bits, [6] an extra value (the extent it exceeded, in 16-byte units).  The host
 * layer raises RuntimeError with this record at the next call.  The other entry points that take an
 * error_flag use [0] only. */
#define DEEPEP_ERROR_RECORD_INTS 8
#define DEEPEP_FLAG_BAD_SLOT     1
#define DEEPEP_FLAG_TIMEOUT      2
#define DEEPEP_FLAG_BAD_ADDRESS  4
#define DEEPEP_FAULT_SCATTER_ROW 1   /* deepep_combine_reduce_scatter: out_rows[u] outside every window  */
#define DEEPEP_FAULT_PLAN_ROW    2   /* deepep_plan_expert: window row past the window's data extent     */
#define DEEPEP_FAULT_PLAN_UNIT   3   /* deepep_plan_expert: unit position / received row out of range     */
#define DEEPEP_FAULT_PACK_ROW    4   /* deepep_dispatch_pack: destination row past the destination buffer */

/* Reduction modes of deepep_combine_reduce. */
#define DEEPEP_MODE_LOCAL     0   /* phase A: copy if 1 valid slot, hadd if 2, else fp32 sum   */
#define DEEPEP_MODE_EPILOGUE  1   /* phase B: bias0 + bias1 + partials (hadd bypass w/o bias)    */
#define DEEPEP_MODE_FUSED     2   /* phase A then phase B over the single partial (EP = 1)       */

int deepep_amd_abi_version(void);
const char* deepep_amd_last_error(void);
/* 16 hex digits: sha256 of the sources, this header and the compile flags the library was built
 * from (deepep_amd/_lib.py source_build_id); the Python loader refuses a binary whose id does not
 * match the sources next to it. */
const char* deepep_amd_build_id(void);

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
 *                     internode_ll.cu:1072-1135); in mode EPILOGUE (the single-reduction
 *                     combine) the chain starts from +0 + bias0 + bias1
 *   bias0, bias1   bf16 [num_units][hidden] or NULL (modes EPILOGUE and FUSED)
 *   out_weights    fp32 rows of out_weights_stride floats (0 = num_weights) or NULL: top-k
 *                  weight pass-through, written once per unit:
 *                  out_weights[u*out_weights_stride + k] = (i = wtable ? wtable[u*wtable_stride + k]
 *                                                             : u*num_weights + k) >= 0 ? wsrc[i] : 0
 *                  (a stride lets the weights ride in the tail of packed exchange rows)
 *   weights_pad    floats written per weight row (<= 64; values below num_weights mean num_weights):
 *                  the entries past num_weights are zeros.  32 writes a packed row's whole 128-byte
 *                  tail line at once: a partial-line store costs the memory side a read-modify-write
 *   units_per_block  workgroup shape: 4 = 4 (row, column-chunk) items per 256-thread workgroup,
 *                  8 = 8 items per 512-thread workgroup, 0 = automatic (4 for LOCAL, else 8)
 *   error_flag     device int or NULL; bit 1 is set when a slot is >= num_src_rows (such slots are
 *                  skipped, never dereferenced).  When bit 2 is already set (a symmetric-window
 *                  barrier timed out, deepep_sym_barrier) the launch stores NaN rows instead of sums
 *                  (and deepep_combine_reduce_scatter stores nothing into the peers' windows)
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
                          int64_t out_weights_stride, int weights_pad,
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
 * Tuning / diagnostics: vec_per_lane = 16-byte vectors each lane loads per source row and item (1 or 2),
 * rows_in_flight = source rows each lane loads before accumulating them (2, 4 or 8); 0 = automatic, the
 * default.  Process-wide, stored as one atomic word that every launch reads once.  Automatic shape: 2 KiB
 * chunks (1 KiB for rows under 128 vectors); rows in flight at most the slot table's width rounded up to
 * 2 / 4 / 8, and 2 (with 1 KiB chunks and 4-wave workgroups) for the fused reduce over top-k >= 5, 8 for
 * the epilogue, 4 for phase A (DEEPEP_MODE_LOCAL) and for every launch on a CU-budget stream.  The store
 * policy follows the output: sc1 nt for phase A's send rows, system scope for peer windows
 * (deepep_combine_reduce_scatter), sc1 otherwise.  The results are identical for every configuration;
 * only the speed changes.
 */
int deepep_set_launch_config(int vec_per_lane, int rows_in_flight);

/* ------------------------------------------------------------------ dispatch
 * Packed token row exchanged between ranks (byte offsets, all 16-byte aligned except as noted):
 *   [x: x_bytes | sf @sf_off: sf_bytes | topk_idx int64[K] @idx_off | weights fp32[K] @w_off |
 *    src_global_idx int32 @src_off], row_bytes % 16 == 0.
 * Receive order: grouped by source rank, ascending source token (deterministic).
 */

/* dst_slot[t][r] = #{t' < t routed to rank r} or -1 (int32 [num_tokens][num_ranks]);
 * send_counts[r] = tokens routed to rank r.  A token is routed to r when one of its top-k experts
 * lives on r (experts_per_rank = num_experts / num_ranks).  block_counts: int32 scratch of
 * ceil(num_tokens / 256) * num_ranks entries. */
int deepep_dispatch_route(const int64_t* topk_idx, int num_tokens, int num_topk, int num_experts, int num_ranks,
                          int32_t* dst_slot, int32_t* send_counts, int32_t* block_counts, deepep_stream_t stream);

/* counts[e] = #{(t, k) : topk_idx[t][k] == e} (int32 [num_experts], zeroed first; entries < 0 are
 * masked slots).  The per-expert half of dispatch_impl's notify (dispatch.cuh:79-258): each sender
 * sends slice [r * experts_per_rank, (r + 1) * experts_per_rank) to rank r with its per-rank count, so
 * one exchange and one host sync give the receiver both its row count per source rank and its
 * rows per local expert. */
int deepep_dispatch_expert_counts(const int64_t* topk_idx, int num_tokens, int num_topk, int num_experts,
                                  int32_t* counts, deepep_stream_t stream);

/* The send side of a fresh dispatch in two launches: dst_slot as deepep_dispatch_route; notify int32
 * [num_ranks][W], W = 1 + experts_per_rank + 2 * num_blocks, row d = [tokens routed to d |
 * deepep_dispatch_expert_counts' slice of d's experts | per-64-token-block tokens routed to d
 * (deepep_route_block_counts' tok) | per-block (token, lane) pairs routed to d (its pairs)] -- the record
 * dispatch_impl's notify sends to d (dispatch.cuh:79-258); send_offsets int32 [num_ranks] = the exclusive
 * prefix of the per-rank token counts.  num_blocks may be 0 (no block counts, one rank) or >=
 * ceil(num_tokens / 64); blocks past the tokens hold 0.  No output needs zeroing.  workspace: device
 * scratch of at least deepep_dispatch_notify_workspace(...) bytes. */
int64_t deepep_dispatch_notify_workspace(int num_tokens, int num_experts, int num_ranks);
int deepep_dispatch_notify(const int64_t* topk_idx, int num_tokens, int num_topk, int num_experts, int num_ranks,
                           int num_blocks, int32_t* dst_slot, int32_t* notify, int32_t* send_offsets,
                           void* workspace, int64_t workspace_bytes, deepep_stream_t stream);

/* Write packed row send_offsets[r] + dst_slot[t][r] for every (token t, destination r), in `packed`
 * (dest_bases NULL: one local buffer for an all-to-all) or in rank r's buffer at dest_bases[r] (device
 * uint64 [num_ranks]: the peers' symmetric windows, system-scope stores -- the xGMI push of
 * dispatch.cuh:373-392); src_global_idx = src_base + t.  topk_weights may be NULL (zeros are sent).
 * dest_rows: rows every destination buffer holds (`packed`, or each peer window); a row index
 * send_offsets[r] + dst_slot[t][r] outside [0, dest_rows) is not stored: bit 4 of error_flag is set and
 * the fault recorded (DEEPEP_FAULT_PACK_ROW).  error_flag (device, DEEPEP_ERROR_RECORD_INTS ints, or
 * NULL): with dest_bases, nothing is stored once bit 2 is set (the window barrier before the push timed
 * out). */
int deepep_dispatch_pack(const void* x, int64_t x_row_stride_bytes, int x_bytes,
                         const void* sf, int64_t sf_row_stride_bytes, int sf_bytes,
                         const int64_t* topk_idx, const float* topk_weights, int num_tokens, int num_topk,
                         int32_t src_base, const int32_t* dst_slot, const int32_t* send_offsets, int num_ranks,
                         void* packed, const uint64_t* dest_bases, int64_t row_bytes, int64_t dest_rows,
                         int sf_off, int idx_off, int w_off, int src_off, int32_t* error_flag,
                         deepep_stream_t stream);

/* Receive-side block: DEEPEP_DISPATCH_BLOCK_ROWS consecutive received rows. */
#define DEEPEP_DISPATCH_BLOCK_ROWS 128

/* Receive side, pass 1: src_metadata columns 0-1 ({src_global_idx, src_rank * K + master lane}),
 * recv_topk_idx (local expert or -1, int64 [num_recv][K], may be NULL) and per-block expert
 * histograms block_counts [ceil(num_recv / DEEPEP_DISPATCH_BLOCK_ROWS)][num_local_experts]. recv_counts_stride
 * 0: recv_rank_psum is the inclusive prefix sum of rows per source rank (device memory);
 * recv_counts_stride > 0: recv_rank_psum[s * recv_counts_stride] is the row count of source rank s (the
 * notify records' first column) and the prefix sum is formed here, and written to psum_out (int32
 * [num_ranks], may be NULL).  num_ranks <= 64.  Rows from the last prefix sum
 * up to num_recv (a launch sized for the worst case, dispatch(do_cpu_sync=False)) get src_metadata
 * columns 0-1 = -1 and recv_topk_idx -1; passes 3 and 4 skip them.
 * pad_rows > 0: the packed rows come from a worst-case-sized exchange, source s's rows at s * pad_rows
 * (not contiguous); row_map (int32 [num_recv]) then receives the packed row of every received row i,
 * which passes 3 and 4 take as their row_map.  own_first (the local bypass): packed = [rows from `rank`
 * itself | rows from the other sources in rank order] -- the sender packed its own rows straight behind
 * its send rows, so they never enter the all-to-all -- and row_map is written the same way; with pad_rows
 * the padded slots are in that order too (`rank`'s at 0, source s < rank at (s + 1) * pad_rows, s > rank at
 * s * pad_rows).  Neither: packed row i is row i (row_map may be NULL). */
int deepep_dispatch_count(const void* packed, int64_t row_bytes, int idx_off, int src_off, int num_recv, int num_topk,
                          int rank, int num_local_experts, const int32_t* recv_rank_psum, int num_ranks,
                          int recv_counts_stride, int32_t* psum_out, int pad_rows, int own_first, int32_t* row_map,
                          int32_t* src_metadata, int64_t* recv_topk_idx, int32_t* block_counts,
                          deepep_stream_t stream);

/* Passes 1-3 in one call (the launches back to back, no host work between them): deepep_dispatch_count in
 * counts mode (recv_counts_stride >= 1, psum_out required), deepep_dispatch_scan, and -- expanded -- the
 * slots pass (inv optional); non-expanded, src_metadata columns 2.. are set to -1. */
int deepep_dispatch_receive(const void* packed, int64_t row_bytes, int idx_off, int src_off, int num_recv,
                            int num_topk, int rank, int num_local_experts, const int32_t* recv_counts,
                            int num_ranks, int recv_counts_stride, int32_t* psum_out, int pad_rows, int own_first,
                            int32_t* row_map,
                            int32_t* src_metadata, int64_t* recv_topk_idx, int32_t* block_counts,
                            int expert_alignment, int expanded, int32_t* expert_counts, int32_t* psum_expert,
                            int32_t* inv, deepep_stream_t stream);

/* Pass 2: block_counts becomes each block's first slot inside its expert group (expert
 * groups start at aligned offsets); expert_counts = rows per expert; psum_expert as the reference
 * handle's psum_num_recv_tokens_per_expert (expanded: aligned start + count; else inclusive aligned). */
int deepep_dispatch_scan(int32_t* block_counts, int num_blocks, int num_local_experts, int expert_alignment,
                         int expanded, int32_t* expert_counts, int32_t* psum_expert, deepep_stream_t stream);

/* Pass 3 (expanded only): src_metadata columns 2.. = expanded row of every local slot, -1 elsewhere
 * (all -1 for a row whose column 0 is -1).  inv (int32 [expanded rows], or NULL): the inverse map,
 * inv[slot] = row * num_topk + lane for every slot written (alignment padding rows are not written). */
int deepep_dispatch_slots(const void* packed, int64_t row_bytes, int idx_off, int num_recv, int num_topk,
                          int rank, int num_local_experts, const int32_t* block_offsets, int32_t* src_metadata,
                          int32_t* inv, const int32_t* row_map, deepep_stream_t stream);

/* Pass 4: recv_x / recv_sf rows (row i, or every local slot when expanded) and top-k weights
 * ([num_recv][K] or, expanded, [slot]).  recv_sf / recv_topk_weights may be NULL.  With x_direct
 * (one rank: nothing was exchanged, the packed rows carry only metadata) the x / sf bytes of row i
 * are read from x_direct / sf_direct at row src_metadata[i][0] % num_max_tokens.  Destination rows
 * >= num_out_rows (the rows recv_x holds) are skipped and set bit 1 of error_flag (device int or
 * NULL); once bit 2 is set (a timed-out window barrier) nothing is stored.  Rows whose
 * src_metadata[i][0] is -1 (past the received rows, pass 1) are skipped.
 * inv (expanded only, or NULL): pass 3's inverse map; then the copy runs destination-major inside
 * blocks of received rows -- expert e's rows of block b are [block_offsets[b][e], block_offsets[b+1][e])
 * (pass 2's offsets; the last block ends at expert_end[e], pass 2's psum_expert) -- each block owned
 * by one XCD, whose L2 serves its rows' re-reads.  Same bytes as with inv NULL
 * (source-major: one load of each received row, a store per local slot). */
int deepep_dispatch_copy(const void* packed, int64_t row_bytes, int x_bytes, int sf_off, int sf_bytes, int w_off,
                         int num_recv, int num_topk, const int32_t* src_metadata, int expanded,
                         const void* x_direct, int64_t x_direct_stride_bytes,
                         const void* sf_direct, int64_t sf_direct_stride_bytes, int num_max_tokens,
                         void* recv_x, void* recv_sf, float* recv_topk_weights, int64_t num_out_rows,
                         const int32_t* inv, const int32_t* block_offsets, const int32_t* expert_end,
                         int num_local_experts, const int32_t* row_map, int32_t* error_flag, deepep_stream_t stream);

/* ------------------------------------------------------------------ EP > 1 combine plan
 * The EP > 1 combine runs in pipeline chunks of source tokens: chunk c = tokens
 * [c * B, (c + 1) * B) of every rank, B = blocks_per_chunk * DEEPEP_PLAN_BLOCK_TOKENS.  Phase A on an
 * expert rank reduces the chunk's received rows into partials; they travel to their source ranks
 * (RCCL all-to-all of the chunk's rows grouped by source rank, or xGMI stores into the source rank's
 * window); phase B on the source rank reduces each token's partials.  These three calls build every
 * table of that schedule on the device from the dispatch's counts, so a first combine needs no host
 * synchronisation.  Counts are per block of DEEPEP_PLAN_BLOCK_TOKENS consecutive tokens of a source
 * rank, int32 [num_ranks][num_blocks] (num_blocks >= ceil(num_max_tokens / 64)).
 */
#define DEEPEP_PLAN_BLOCK_TOKENS 64
#define DEEPEP_PLAN_EXPANDED     1    /* x is the expanded layout (metadata columns 2.. are rows)       */
#define DEEPEP_PLAN_SINGLE       2    /* single reduction: every valid (row, lane) travels unreduced     */
#define DEEPEP_PLAN_INTERLEAVE   4    /* phase-A units round-robin over source ranks (xGMI stores)      */
#define DEEPEP_PLAN_RANK_LAYOUT  8    /* receive slot = expert rank (R <= K), else the master lane        */
#define DEEPEP_PLAN_WINDOW      16    /* source side: rows are window rows slot * T_max + t               */
#define DEEPEP_PLAN_LOCAL_BYPASS 32   /* RCCL exchange without the own-rank diagonal (below)              */

/* Sender side of the notify: tok_counts[r][b] = tokens of block b routed to rank r, pair_counts[r][b] =
 * (token, lane) entries of block b routed to r (blocks past num_tokens are zero). */
int deepep_route_block_counts(const int64_t* topk_idx, int num_tokens, int num_topk, int num_experts, int num_ranks,
                              int num_blocks, int32_t* tok_counts, int32_t* pair_counts, deepep_stream_t stream);

/* Expert side: phase-A units of every chunk, concatenated in chunk order.  recv_tok / recv_pairs are
 * the counts received from every source rank (rows received per source block).  Inside a chunk, units
 * are grouped by source rank (the send buffer of an all-to-all), or round-robin over the source ranks
 * with DEEPEP_PLAN_INTERLEAVE.  Multiple reduction: one unit per received row i; table_a[u] = the
 * metadata slots of i (expanded, K wide) or i (1 wide), wtable_a[u][k] = i * K + k (non-expanded,
 * may be NULL).  Single reduction: one unit per valid (row, lane) in (row, lane) order, table_a[u] =
 * the expanded row (1 wide).  out_rows (optional, the xGMI transport): byte address of unit u's row,
 * window_bases[src_rank] + (slot * num_max_tokens + src_token) * window_row_bytes, slot = rank (rank
 * layout) or the master lane (multiple reduction), the lane (single reduction) -- combine.cuh:96-106.
 * Bounds: a received row index >= num_recv (src_metadata rows) or a unit position past its chunk's unit
 * count (counts that disagree with the metadata) writes nothing for that unit (DEEPEP_FAULT_PLAN_UNIT);
 * a window row whose bytes do not lie inside [0, window_bytes) of its window, or metadata no correct
 * dispatch produces, gives out_rows[u] = 0 (DEEPEP_FAULT_PLAN_ROW), which the scatter skips.  Callers
 * pre-fill table_a / wtable_a with -1 and out_rows with 0, so an unwritten unit is never an address.
 * error_flag: DEEPEP_ERROR_RECORD_INTS device ints or NULL (bit 1 and the record are set on a fault).
 * padded_stride > 0 (a handle whose counts only the device knows: dispatch without a CPU sync): chunk c
 * holds num_ranks * padded_stride unit positions starting at c * num_ranks * padded_stride; unit p of
 * source s sits at s * padded_stride + p (or p * num_ranks + s with DEEPEP_PLAN_INTERLEAVE).  The positions
 * no unit takes keep the caller's fill: -1 slots (a zero partial) and, for out_rows, the value 1, which
 * the scatter skips silently.  A unit p >= padded_stride of its source (more (token, lane) pairs on this
 * rank than the padding allows) is rejected like a unit past its chunk, so it never lands in another
 * source's positions.
 * DEEPEP_PLAN_LOCAL_BYPASS (grouped order only): inside every chunk the groups follow the ranks in order
 * except this rank's, which comes last -- [units of the other sources, rank order | units of `rank`] -- so
 * the first part is an all-to-all input whose split for `rank` is 0 and the own units can be written
 * straight into the receive rows deepep_plan_source lays out with the same flag (the reference's own
 * receive slot is local memory, combine.cuh:96-101). */
int deepep_plan_expert(const int32_t* src_metadata, int num_recv, int num_topk, int num_ranks, int rank,
                       int num_max_tokens, const int32_t* recv_tok, const int32_t* recv_pairs, int num_blocks,
                       int blocks_per_chunk, int flags, int32_t* table_a, int32_t* wtable_a,
                       const uint64_t* window_bases, int64_t window_row_bytes, int64_t window_bytes,
                       uint64_t* out_rows, int32_t* error_flag, int padded_stride, deepep_stream_t stream);

/* Source side, per owned token t (chunk c = t / B).  Multiple reduction: table_b [T][min(R, K)] = the
 * rows of t's partials in ascending dedup-master-lane order (a rank's master is its highest top-k
 * lane; combine_reduce_epilogue.cuh:74-95), then -1; wtable [T][K] (or NULL) = row(rank of lane k) *
 * row_floats + weights_offset + k, or -1: the float index of lane k's weight in the packed receive rows.
 * A row is the partial's row in chunk c's receive buffer (grouped by expert rank, ascending token:
 * dst_slot [T][R] from deepep_dispatch_route gives the rank among earlier tokens) or, with
 * DEEPEP_PLAN_WINDOW, the window row slot * num_max_tokens + t.  Single reduction: table_b [T][K] = the
 * row of (t, k): receive-buffer order (expert rank, then (token, lane)) or window row k * T_max + t.
 * padded_stride > 0 (not with DEEPEP_PLAN_WINDOW): the receive buffer of a chunk is worst-case padded,
 * expert rank d's rows from d * padded_stride (the plan_expert layout above, after the exchange); a row
 * past d's padded_stride rows (a unit plan_expert rejects) is -1.
 * DEEPEP_PLAN_LOCAL_BYPASS (not with DEEPEP_PLAN_WINDOW): the chunk's receive rows are [rows from `rank`
 * (phase A's own units, written in place) | rows received from the other ranks, rank order], i.e. the
 * rows of `rank` come first. */
int deepep_plan_source(const int64_t* topk_idx, int num_tokens, int num_topk, int num_experts, int num_ranks,
                       int rank, int num_max_tokens, const int32_t* dst_slot, const int32_t* send_tok,
                       const int32_t* send_pairs, int num_blocks, int blocks_per_chunk, int flags,
                       int64_t row_floats, int64_t weights_offset, int32_t* table_b, int table_b_width,
                       int32_t* wtable, int padded_stride, deepep_stream_t stream);

/* ------------------------------------------------------------------ symmetric buffer over xGMI
 * Replaces the reference's NCCLSymmetricMemoryContext (csrc/elastic/nccl.cu:62-153, buffer.hpp:181-208)
 * and its device barrier (deep_ep/include/deep_ep/common/comm.cuh:88-129).  One uncached device
 * allocation per rank, exported/imported with HIP IPC; kernels on any rank load/store a peer's
 * window over xGMI. */
#define DEEPEP_IPC_HANDLE_BYTES 64

int deepep_sym_alloc(int64_t bytes, void** ptr);            /* zero-filled, hipDeviceMallocUncached */
int deepep_sym_free(void* ptr);
int deepep_sym_export(void* ptr, void* handle);             /* handle: DEEPEP_IPC_HANDLE_BYTES bytes */
int deepep_sym_import(const void* handle, void** ptr);      /* a peer's window, mapped into this process */
int deepep_sym_close(void* ptr);

/* Window header, DEEPEP_SYM_HEADER_BYTES from the window base (zero at allocation): the int64 flag
 * table [DEEPEP_SYM_FLAG_SLOTS][64], then int64 counters [3][DEEPEP_SYM_FLAG_SLOTS] (publishes, waits,
 * workgroup arrivals), then from DEEPEP_SYM_NOTIFY_OFFSET the notify area the dispatch's counts are
 * exchanged through (deepep_sym_put); the data region starts at DEEPEP_SYM_HEADER_BYTES. */
#define DEEPEP_SYM_NOTIFY_OFFSET 65536
#define DEEPEP_SYM_HEADER_BYTES 1048576

/* Store src + d * bytes (bytes % 16 == 0) at dest_bases[d] + dest_offset for every d < num_ranks:
 * system-scope write-through stores into the peers' windows (dest_bases: device uint64 [num_ranks],
 * e.g. the window bases, so dest_offset addresses the header's notify area).  dest_extent: the bytes
 * every destination window spans from its base (header + data); a put whose [dest_offset, dest_offset
 * + bytes) does not lie inside it is rejected (DEEPEP_ERR_INVALID_ARG) before anything is launched.
 * The dispatch notify's transport: rank r puts its count record for every destination into slot r of
 * that destination's area, then a barrier makes them visible (dispatch.cuh:79-258's notify over
 * NVLink).  Nothing is stored once bit 2 of error_flag (device int or NULL) is set. */
int deepep_sym_put(const void* src, int64_t bytes, const uint64_t* dest_bases, int num_ranks, int64_t dest_offset,
                   int64_t dest_extent, const int32_t* error_flag, deepep_stream_t stream);

/* Group barrier on the stream: peer_flags (device, uint64 [num_ranks]) holds the address of every
 * rank's window header (above).  Every XCD's L2 is first written back (the stores into peer windows before
 * the call may sit in any of them).  Rank r then stores
 * the epoch into entry [r] of slot 0 of every rank's table (system-scope release) and waits until
 * its own entries all reach it (system-scope acquire).  epoch <= 0: the next epoch is counted on
 * the device (this rank's counter), so a captured HIP graph replays with fresh epochs -- use it
 * for every call of a window, or host epochs (growing by one per call) for every call, not both.
 * After timeout_us (<= 0: 100 s) the wait gives up and sets bit 2 of *error_flag (comm.cuh:30-54
 * traps instead). */
int deepep_sym_barrier(const uint64_t* peer_flags, int rank, int num_ranks, int64_t epoch, int64_t timeout_us,
                       int32_t* error_flag, deepep_stream_t stream);

/* Split barrier for pipelined phases, on flag slot 1 <= slot < DEEPEP_SYM_FLAG_SLOTS of the same
 * tables (slot 0 is deepep_sym_barrier's): deepep_sym_signal stores `value` into slot `slot`, entry
 * [rank], of every rank's table after the stream's earlier work (system-scope release);
 * deepep_sym_wait waits until every entry of slot `slot` of this rank's table reaches `value`
 * (timeout as deepep_sym_barrier).  value <= 0: counted on the device, signals and waits each
 * with their own per-slot counter (the n-th wait of a slot waits for every rank's n-th signal). */
#define DEEPEP_SYM_FLAG_SLOTS 64
int deepep_sym_signal(const uint64_t* peer_flags, int rank, int num_ranks, int slot, int64_t value,
                      deepep_stream_t stream);
int deepep_sym_wait(const uint64_t* peer_flags, int rank, int num_ranks, int slot, int64_t value, int64_t timeout_us,
                    int32_t* error_flag, deepep_stream_t stream);

/* Phase A writing straight into the owners' receive rows (combine_impl's NVLink push,
 * combine.cuh:96-106, 125-176, 215-226): the reduce of deepep_combine_reduce(DEEPEP_MODE_LOCAL, ...)
 * with unit u's bf16 row stored at byte address out_rows[u] (any rank's window, 16-byte aligned)
 * and, when num_weights > 0, its top-k weights (the wtable / wsrc pass-through rule above, weights_pad
 * floats) at out_rows[u] + weights_offset.  All these stores are system-scope write-through (sc0 sc1),
 * so they are visible to the owning GPU once the kernel has completed.
 * Windows: window_bases (device uint64 [num_windows]) and window_bytes, the data extent of each.  Every
 * row is checked before it is stored: unless all its bytes (the bf16 row and, with weights, the weight
 * tail) lie inside one window, the unit is skipped, bit 4 of error_flag is set and the fault recorded
 * (DEEPEP_FAULT_SCATTER_ROW); out_rows[u] == 0 (a unit plan_expert rejected) is skipped with bit 1,
 * out_rows[u] == 1 (a padding position of a padded plan) silently.
 * error_flag: DEEPEP_ERROR_RECORD_INTS device ints or NULL. */
int deepep_combine_reduce_scatter(int weighted,
                                  const void* src, int64_t num_src_rows, int64_t src_row_stride,
                                  const int32_t* table, int64_t table_stride, int table_width,
                                  const float* row_weights,
                                  const uint64_t* out_rows, int num_units, int hidden,
                                  const int32_t* wtable, int64_t wtable_stride,
                                  const float* wsrc, int num_weights, int64_t weights_offset, int weights_pad,
                                  const uint64_t* window_bases, int num_windows, int64_t window_bytes,
                                  int32_t* error_flag, deepep_stream_t stream);

/* A CU budget: a stream whose kernels run on `num_cus` compute units only, rounded up to a multiple
 * of 8 (hipExtStreamCreateWithCUMask, the first num_cus mask bits = num_cus / 8 CUs on every XCD),
 * leaving the rest to overlapping
 * compute.  It is how this build honours an explicit num_sms (the reference sizes combine_impl's
 * grid with it, csrc/kernels/elastic/combine.hpp:135, elastic.py:1086-1088). */
int deepep_stream_create_cu_budget(int num_cus, deepep_stream_t* stream);
int deepep_stream_destroy(deepep_stream_t stream);
/* Diagnostic: how many distinct CUs (and XCDs) a stream's workgroups run on (8192 one-wave workgroups
 * recording their hardware ids; synchronises the stream). */
int deepep_stream_probe_cus(deepep_stream_t stream, int* num_cus, int* num_xcds);

/* ElasticBuffer::get_combine_buffer_size for one node (num_scaleout_ranks == 1). */
int64_t deepep_combine_buffer_size(int num_max_tokens_per_rank, int hidden, int num_topk,
                                   int num_ranks, int allow_multiple_reduction);

#ifdef __cplusplus
}
#endif

#endif /* DEEPEP_AMD_H */
