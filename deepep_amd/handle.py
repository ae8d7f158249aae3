"""EPHandle and the per-handle combine plan.

EPHandle keeps the attributes of the reference's handle
(deep_ep/buffers/elastic.py:25-98 in /root/reference) so user code that reads them
keeps working.  What is new is `CombinePlan`: the token -> source-row tables the
combine kernels read, derived once from the handle's routing and cached on it
(the reference re-derives them inside every combine_reduce_epilogue_impl launch,
combine_reduce_epilogue.cuh:62-95, by walking topk_idx and the symmetric receive
buffer; here they are small int32 tables, 4*K bytes per token).

Invariant the plan relies on for EP > 1 (guaranteed by ElasticBuffer.dispatch):
on every expert rank the received tokens are grouped by source rank and ascending
source token inside a rank -- the order of refs.dispatch (deep_ep/utils/refs.py:10-123)
and of the reference's deterministic mode (elastic.py:117-131).  The source rank can
then compute where each of its tokens' partials lands after the exchange without
any extra communication.
"""
from dataclasses import dataclass, field
from typing import List, Optional

import torch


@dataclass
class ChunkPlan:
    """One pipeline chunk of the EP > 1 combine: the source tokens [lo, hi) of every rank."""
    lo: int
    hi: int
    table_a: Optional[torch.Tensor]          # expert side: [n, K] expanded slots, or [n, 1] received rows
    wtable_a: Optional[torch.Tensor]         # expert side: [n, K] weight-source index
    send_counts: List[int]                   # expert side: rows sent back to every source rank
    back_counts: List[int]                   # source side: rows received from every expert rank
    table_b: torch.Tensor                    # source side: [hi - lo, min(R, K)] rows of the chunk's receive buffer
    row_of_lane: torch.Tensor                # source side: [hi - lo, K]
    wtables: dict = field(default_factory=dict)
    out_rows: Optional[torch.Tensor] = None  # xGMI transport, expert side: [n] window row address per unit


@dataclass
class CombinePlan:
    num_ranks: int
    num_tokens: int
    num_topk: int
    expanded: bool
    # EP == 1: token-major source-row table for the fused kernel
    local_table: Optional[torch.Tensor] = None        # [T, K] (expanded) or [T, 1] int32
    local_wtable: Optional[torch.Tensor] = None       # [T, K] int32, non-expanded weight pass-through
    # EP > 1, multiple reduction
    recv_counts: Optional[List[int]] = None           # rows this rank holds per source rank (phase A output)
    back_counts: Optional[List[int]] = None           # partial rows this rank receives per expert rank
    table_b: Optional[torch.Tensor] = None            # [T, min(R, K)] rows of the receive buffer, master order
    row_of_lane: Optional[torch.Tensor] = None        # [T, K] receive row holding lane k's weight, or -1
    wtables: Optional[dict] = None                    # packed-row weight tables, keyed by (row floats, offset)
    chunks: Optional[List[ChunkPlan]] = None          # pipelined exchange (phase A | all-to-all | phase B)
    # EP > 1 over the xGMI symmetric windows
    out_rows: Optional[torch.Tensor] = None           # [N_recv] int64 byte address of each partial's row
    window_row_bytes: int = 0
    # EP > 1, single reduction (allow_multiple_reduction=False, expanded): rows sent unreduced
    send_slots1: Optional[torch.Tensor] = None        # [N_send, 1] expanded rows in send order
    send_counts1: Optional[List[int]] = None
    back_counts1: Optional[List[int]] = None
    table_b1: Optional[torch.Tensor] = None           # [T, K] rows of the receive buffer per (t, k)


def epilogue_tables(topk_idx: torch.Tensor, num_experts: int, num_ranks: int):
    """Source-side tables for EP > 1 (multiple reduction).

    For token t and expert rank r (r owns an expert of t), the partial of t computed
    on r arrives at row offset[r] + pos_r(t) of the exchange receive buffer, where
    pos_r(t) counts the earlier tokens routed to r.  Rows are listed in ascending
    order of the highest top-k lane that maps to r (the dedup master lane,
    deep_ep/include/deep_ep/common/ptx.cuh:412-421, combine_reduce_epilogue.cuh:74-95).
    """
    T, K = topk_idx.shape
    R = num_ranks
    dev = topk_idx.device
    epr = num_experts // R
    rank_of = torch.where(topk_idx >= 0, torch.div(topk_idx, epr, rounding_mode='floor'),
                          torch.full_like(topk_idx, -1))
    ranks = torch.arange(R, device=dev)
    hit = rank_of.unsqueeze(-1) == ranks.view(1, 1, R)                 # [T, K, R]
    is_to = hit.any(dim=1)                                              # [T, R]
    back_counts = is_to.sum(dim=0)                                      # [R]
    pos = torch.cumsum(is_to.to(torch.int64), dim=0) - 1
    offsets = torch.cumsum(back_counts, dim=0) - back_counts
    row = torch.where(is_to, offsets.view(1, R) + pos, torch.full_like(pos, -1))
    lanes = torch.arange(K, device=dev).view(1, K, 1)
    master = torch.where(hit, lanes, torch.full_like(lanes, -1)).amax(dim=1)      # [T, R]
    key = torch.where(is_to, master, K + ranks.view(1, R))
    order = torch.argsort(key, dim=1, stable=True)[:, :min(R, K)]
    table_b = row.gather(1, order).to(torch.int32).contiguous()
    row_of_lane = torch.where(rank_of >= 0, row.gather(1, rank_of.clamp(min=0)), torch.full_like(rank_of, -1))
    return table_b, row_of_lane.contiguous(), [int(v) for v in back_counts.tolist()]


def weight_table(row_of_lane: torch.Tensor, row_floats: int, offset: int) -> torch.Tensor:
    """[T, K] int32 index of lane k's weight in a float view of packed receive rows
    (row r's weights start at r * row_floats + offset), or -1."""
    K = row_of_lane.shape[1]
    k_idx = torch.arange(K, device=row_of_lane.device).view(1, K)
    idx = torch.where(row_of_lane >= 0, row_of_lane * row_floats + offset + k_idx, torch.full_like(row_of_lane, -1))
    assert int(idx.max().item()) < 2 ** 31 if idx.numel() else True
    return idx.to(torch.int32).contiguous()


def window_tables(topk_idx: torch.Tensor, num_experts: int, num_ranks: int, num_max_tokens: int,
                  rank_layout: bool):
    """Source-side tables for the xGMI transport, where partials land in this rank's symmetric
    window at row slot * T_max + t (slot = expert rank under the rank layout, else the dedup
    master lane; combine.cuh:96-106, combine_utils.cuh:8-13).  Returns table_b [T, min(R, K)]
    (rows in ascending dedup-master-lane order, combine_reduce_epilogue.cuh:74-95) and
    row_of_lane [T, K] (the row holding lane k's weight, or -1)."""
    T, K = topk_idx.shape
    R = num_ranks
    dev = topk_idx.device
    epr = num_experts // R
    rank_of = torch.where(topk_idx >= 0, torch.div(topk_idx, epr, rounding_mode='floor'),
                          torch.full_like(topk_idx, -1))
    ranks = torch.arange(R, device=dev)
    hit = rank_of.unsqueeze(-1) == ranks.view(1, 1, R)                 # [T, K, R]
    is_to = hit.any(dim=1)                                              # [T, R]
    lanes = torch.arange(K, device=dev).view(1, K, 1)
    master = torch.where(hit, lanes, torch.full_like(lanes, -1)).amax(dim=1)      # [T, R]
    slot = ranks.view(1, R).expand(T, R) if rank_layout else master
    t_idx = torch.arange(T, device=dev).view(T, 1)
    row = torch.where(is_to, slot * num_max_tokens + t_idx, torch.full_like(master, -1))
    key = torch.where(is_to, master, K + ranks.view(1, R))
    order = torch.argsort(key, dim=1, stable=True)[:, :min(R, K)]
    table_b = row.gather(1, order).to(torch.int32).contiguous()
    row_of_lane = torch.where(rank_of >= 0, row.gather(1, rank_of.clamp(min=0)), torch.full_like(rank_of, -1))
    return table_b, row_of_lane.contiguous()


def chunk_plans(meta: torch.Tensor, recv_counts: List[int], topk_idx: torch.Tensor, num_experts: int,
                num_ranks: int, num_max_tokens: int, num_chunks: int, expanded: bool) -> List[ChunkPlan]:
    """Split the EP > 1 combine into chunks of source tokens so that phase A of chunk c+1, the
    all-to-all of chunk c and phase B of chunk c-1 overlap.  Chunk c holds the source tokens
    [c * B, (c + 1) * B) of every rank, B = ceil(num_max_tokens / num_chunks); on the expert side
    those are, for every source rank, a contiguous run of its received rows (receive order is
    (source rank, ascending token)), so the chunk's send buffer is again grouped by source rank."""
    T, K = topk_idx.shape
    R = num_ranks
    dev = meta.device
    n_recv = sum(recv_counts)
    B = (num_max_tokens + num_chunks - 1) // num_chunks
    m = meta[:n_recv]
    chunk_of_row = torch.div(m[:, 0] % num_max_tokens, B, rounding_mode='floor')
    src_rank = torch.div(m[:, 1], K, rounding_mode='floor')
    plans = []
    for c in range(num_chunks):
        lo, hi = c * B, min((c + 1) * B, T)
        rows = (chunk_of_row == c).nonzero().view(-1)
        if expanded:
            table_a = m[rows, 2:].contiguous()
            wtable_a = table_a
        elif num_chunks == 1:
            table_a, wtable_a = None, None               # received row i is unit i
        else:
            table_a = rows.to(torch.int32).view(-1, 1).contiguous()
            wtable_a = (rows.view(-1, 1) * K + torch.arange(K, device=dev).view(1, K)).to(torch.int32).contiguous()
        send_counts = [int(v) for v in torch.bincount(src_rank[rows], minlength=R).tolist()]
        if hi > lo:
            table_b, row_of_lane, back_counts = epilogue_tables(topk_idx[lo:hi], num_experts, R)
        else:
            table_b = torch.empty((0, min(R, K)), dtype=torch.int32, device=dev)
            row_of_lane = torch.empty((0, K), dtype=topk_idx.dtype, device=dev)
            back_counts = [0] * R
        plans.append(ChunkPlan(lo, max(lo, hi), table_a, wtable_a, send_counts, back_counts, table_b, row_of_lane))
    return plans


def single_reduction_tables(topk_idx: torch.Tensor, num_experts: int, num_ranks: int):
    """Source-side table for unreduced sends: row of (t, k) in the receive buffer.

    Expert ranks send every valid (token, lane) row in (ascending token, ascending
    lane) order per source rank, so row(t, k) = offset[r] + #{(t', k') < (t, k) on r}.
    """
    T, K = topk_idx.shape
    R = num_ranks
    dev = topk_idx.device
    epr = num_experts // R
    rank_of = torch.where(topk_idx >= 0, torch.div(topk_idx, epr, rounding_mode='floor'),
                          torch.full_like(topk_idx, -1)).reshape(-1)
    onehot = rank_of.unsqueeze(-1) == torch.arange(R, device=dev).view(1, R)    # [T*K, R]
    counts = onehot.sum(dim=0)
    pos = torch.cumsum(onehot.to(torch.int64), dim=0) - 1
    offsets = torch.cumsum(counts, dim=0) - counts
    row_all = offsets.view(1, R) + pos
    row = torch.where(rank_of >= 0, row_all.gather(1, rank_of.clamp(min=0).view(-1, 1)).view(-1),
                      torch.full_like(rank_of, -1))
    return row.view(T, K).to(torch.int32).contiguous(), [int(v) for v in counts.tolist()]


class EPHandle:
    """Communication handle returned by `ElasticBuffer.dispatch` (same attributes as the reference)."""

    def __init__(self,
                 do_expand: bool,
                 num_experts: int, expert_alignment: int,
                 num_max_tokens_per_rank: int,
                 num_sms: int,
                 topk_idx: torch.Tensor,
                 num_recv_tokens: int,
                 num_expanded_tokens: int,
                 num_recv_tokens_per_expert_list: list,
                 psum_num_recv_tokens_per_scaleup_rank: torch.Tensor,
                 psum_num_recv_tokens_per_expert: torch.Tensor,
                 num_unaligned_recv_tokens_per_expert: torch.Tensor,
                 recv_src_metadata: torch.Tensor,
                 dst_buffer_slot_idx: torch.Tensor,
                 token_metadata_at_forward: Optional[torch.Tensor],
                 channel_linked_list: Optional[torch.Tensor]):
        assert topk_idx is not None
        self.do_expand = do_expand
        self.num_experts = num_experts
        self.expert_alignment = expert_alignment
        self.num_max_tokens_per_rank = num_max_tokens_per_rank
        self.num_sms = num_sms
        self.topk_idx = topk_idx
        self.psum_num_recv_tokens_per_scaleup_rank = psum_num_recv_tokens_per_scaleup_rank
        self.psum_num_recv_tokens_per_expert = psum_num_recv_tokens_per_expert
        self.num_unaligned_recv_tokens_per_expert = num_unaligned_recv_tokens_per_expert
        self.num_recv_tokens_per_expert_list = num_recv_tokens_per_expert_list
        self.recv_src_metadata = recv_src_metadata
        self.dst_buffer_slot_idx = dst_buffer_slot_idx
        self.token_metadata_at_forward = token_metadata_at_forward
        self.channel_linked_list = channel_linked_list
        self.num_recv_tokens = num_recv_tokens
        self.num_expanded_tokens = num_expanded_tokens
        self.cached_recv_src_metadata_before_sort = None
        # Host-side copies captured at dispatch (counts per source rank), and the combine plan cache
        self._recv_counts: Optional[List[int]] = None
        self._send_counts: Optional[List[int]] = None         # cached dispatch: no host sync needed
        self._send_offsets: Optional[torch.Tensor] = None
        self._recv_topk_idx: Optional[torch.Tensor] = None    # non-expanded recv_topk_idx (int64, N rows)
        self._combine_plans = {}

    def deterministic_sort(self, *args, **kwargs) -> None:
        """The dispatch of this build is deterministic by construction (received tokens sorted by
        source global index, expanded rows by (expert, source index)), which is the order the
        reference's deterministic_sort produces (elastic.py:100-192); nothing to do."""
        return None


def single_chunk_plans(meta: torch.Tensor, recv_counts: List[int], topk_idx: torch.Tensor, num_experts: int,
                       num_ranks: int, num_max_tokens: int, num_chunks: int) -> List[ChunkPlan]:
    """The single-reduction exchange (every valid expanded row unreduced) split into the same source-
    token chunks as chunk_plans.  Expert side: chunk c's rows are, per source rank, a contiguous run
    of received rows, and their valid lanes in (row, lane) order are the chunk's send buffer, grouped
    by source rank (`table_a` = [n, 1] expanded rows).  Source side: `table_b` [hi - lo, K] is
    single_reduction_tables over the chunk's tokens."""
    T, K = topk_idx.shape
    R = num_ranks
    dev = meta.device
    n_recv = sum(recv_counts)
    B = (num_max_tokens + num_chunks - 1) // num_chunks
    m = meta[:n_recv]
    chunk_of_row = torch.div(m[:, 0] % num_max_tokens, B, rounding_mode='floor')
    src_rank = torch.div(m[:, 1], K, rounding_mode='floor')
    plans = []
    for c in range(num_chunks):
        lo, hi = c * B, min((c + 1) * B, T)
        rows = (chunk_of_row == c).nonzero().view(-1)
        slots = m[rows, 2:]
        valid = slots >= 0
        send_slots = slots[valid].view(-1, 1).to(torch.int32).contiguous()
        lanes_per_row = valid.sum(dim=1)
        send_counts = [int(v) for v in torch.bincount(src_rank[rows], weights=lanes_per_row.to(torch.float64),
                                                      minlength=R).round().to(torch.int64).tolist()]
        if hi > lo:
            table_b, back_counts = single_reduction_tables(topk_idx[lo:hi], num_experts, R)
        else:
            table_b, back_counts = torch.empty((0, K), dtype=torch.int32, device=dev), [0] * R
        plans.append(ChunkPlan(lo, max(lo, hi), send_slots, None, send_counts, back_counts, table_b, table_b))
    return plans
