"""Tensor-level wrappers over the C-ABI (deepep_amd/_lib.py).

`HipKernels` is the only kernel provider the product uses.  It accepts torch
tensors, checks dtypes/shapes/devices on the host (the checks of
csrc/elastic/buffer.hpp:1200-1247 in the reference that concern the kernels), and
passes raw device pointers plus the stream handle to libdeepep_amd.so.
"""
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib
from ._lib import MODE_EPILOGUE, MODE_FUSED, MODE_LOCAL, ptr
from .utils import align

__all__ = ['HipKernels', 'RowLayout', 'MODE_LOCAL', 'MODE_EPILOGUE', 'MODE_FUSED']


@dataclass(frozen=True)
class RowLayout:
    """Byte layout of one packed dispatch row (include/deepep_amd.h, dispatch section)."""
    x_bytes: int
    sf_bytes: int
    num_topk: int
    sf_off: int
    idx_off: int
    w_off: int
    src_off: int
    row_bytes: int

    @staticmethod
    def make(x_bytes: int, sf_bytes: int, num_topk: int) -> 'RowLayout':
        sf_off = x_bytes
        idx_off = align(sf_off + sf_bytes, 16)
        w_off = idx_off + align(num_topk * 8, 16)
        src_off = w_off + align(num_topk * 4, 16)
        # rows are whole 128-byte lines, so every row (and its x bytes) starts on a line
        return RowLayout(x_bytes, sf_bytes, num_topk, sf_off, idx_off, w_off, src_off, align(src_off + 16, 128))


def _require(cond: bool, msg: str) -> None:
    if not cond:
        raise RuntimeError(f'deepep_amd: {msg}')


def _stream_handle(stream) -> int:
    return stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream


def _table_view(table: Optional[torch.Tensor]):
    """(tensor, row stride in elements, width) of a 2-D int32 table view (rows may be strided)."""
    if table is None:
        return None, 0, 1
    _require(table.dim() == 2 and table.dtype == torch.int32 and table.stride(1) == 1,
             'slot tables must be 2-D int32 with unit column stride')
    return table, table.stride(0), table.shape[1]


class HipKernels:
    """The HIP implementation of the combine primitives (gfx950)."""

    name = 'hip'

    def __init__(self):
        self.lib = _lib.load()

    def combine_reduce(self, mode: int, src: torch.Tensor, out: torch.Tensor, num_units: int,
                       table: Optional[torch.Tensor] = None,
                       row_weights: Optional[torch.Tensor] = None,
                       bias0: Optional[torch.Tensor] = None, bias1: Optional[torch.Tensor] = None,
                       wtable: Optional[torch.Tensor] = None, wsrc: Optional[torch.Tensor] = None,
                       out_weights: Optional[torch.Tensor] = None,
                       units_per_block: int = 0, error_flag: Optional[torch.Tensor] = None,
                       weights_pad: int = 0, stream=None) -> None:
        """weights_pad: floats written per weight row (zeros past the weights); 32 fills a packed
        row's 128-byte tail line, so no partial line reaches the memory side."""
        _require(src.is_cuda and out.is_cuda, 'combine tensors must be on the GPU')
        _require(src.dtype == torch.bfloat16 and out.dtype == torch.bfloat16, 'combine rows must be bfloat16')
        _require(src.dim() == 2 and out.dim() == 2 and (src.numel() == 0 or src.stride(1) == 1) and
                 (out.numel() == 0 or out.stride(1) == 1), 'combine rows must be 2-D with unit column stride')
        hidden = out.shape[1]
        _require(src.shape[1] == hidden or src.shape[0] == 0, 'source and output hidden sizes differ')
        _require(out.shape[0] >= num_units, 'output has fewer rows than units')
        for b in (bias0, bias1):
            if b is not None:
                _require(b.is_cuda and b.dtype == torch.bfloat16 and b.is_contiguous() and
                         tuple(b.shape) == (num_units, hidden), 'bias must be contiguous bf16 [num_tokens, hidden]')
        t, t_stride, t_width = _table_view(table)
        if t is not None:
            _require(t.shape[0] >= num_units, 'slot table has fewer rows than units')
        w, w_stride, _ = _table_view(wtable)
        num_weights = 0
        ow_stride = 0
        if out_weights is not None:
            _require(out_weights.dtype == torch.float32 and out_weights.dim() == 2 and out_weights.stride(1) == 1,
                     'weights must be float32 [units, k] with unit column stride')
            _require(out_weights.shape[0] >= num_units, 'weight output has fewer rows than units')
            num_weights = out_weights.shape[1]
            ow_stride = out_weights.stride(0)
            _require(wsrc is not None and wsrc.dtype == torch.float32 and wsrc.dim() == 1 and
                     (wsrc.stride(0) == 1 or wsrc.numel() <= 1), 'weight source must be a 1-D float32 view')
        weighted = row_weights is not None
        if weighted:
            _require(row_weights.dtype == torch.float32 and row_weights.is_contiguous(),
                     'row weights must be contiguous float32')
        rc = self.lib.deepep_combine_reduce(
            mode, int(weighted),
            ptr(src), src.shape[0], src.stride(0) if src.shape[0] > 0 else hidden,
            ptr(t), t_stride, t_width,
            ptr(row_weights),
            ptr(bias0), ptr(bias1),
            ptr(out), out.stride(0) if out.shape[0] > 0 else hidden,
            num_units, hidden,
            ptr(w), w_stride,
            ptr(wsrc), ptr(out_weights), num_weights, ow_stride, weights_pad,
            units_per_block, ptr(error_flag),
            _stream_handle(stream))
        _lib.check(rc, 'combine_reduce')

    def combine_reduce_scatter(self, src: torch.Tensor, num_units: int, out_rows: torch.Tensor,
                               table: Optional[torch.Tensor] = None, row_weights: Optional[torch.Tensor] = None,
                               wtable: Optional[torch.Tensor] = None, wsrc: Optional[torch.Tensor] = None,
                               num_weights: int = 0, weights_offset: int = 0, weights_pad: int = 0,
                               error_flag: Optional[torch.Tensor] = None, *, windows, stream=None) -> None:
        """Phase A storing unit u's row at byte address out_rows[u] (a peer window over xGMI).
        windows = (bases, bytes): int64 [n] device tensor of window data addresses and the extent of each;
        a row not wholly inside one of them is skipped and flagged (error_flag: an error record of
        _lib.ERROR_RECORD_INTS ints)."""
        _require(src.is_cuda and src.dtype == torch.bfloat16 and src.dim() == 2 and
                 (src.numel() == 0 or src.stride(1) == 1), 'combine rows must be 2-D bf16 on the GPU with unit column stride')
        _require(out_rows.is_cuda and out_rows.dtype == torch.int64 and out_rows.is_contiguous() and
                 out_rows.shape[0] >= num_units, 'out_rows must be int64 [num_units] on the GPU')
        win_bases, win_bytes = windows
        _require(win_bases.is_cuda and win_bases.dtype == torch.int64 and win_bases.is_contiguous() and
                 win_bases.dim() == 1, 'window bases must be int64 [num_windows] on the GPU')
        _require(error_flag is None or error_flag.numel() >= 1, 'error flag')
        t, t_stride, t_width = _table_view(table)
        w, w_stride, _ = _table_view(wtable)
        if num_weights:
            _require(wsrc is not None and wsrc.dtype == torch.float32 and wsrc.dim() == 1, 'weight source')
        if row_weights is not None:
            _require(row_weights.dtype == torch.float32 and row_weights.is_contiguous(), 'row weights')
        hidden = src.shape[1]
        rc = self.lib.deepep_combine_reduce_scatter(
            int(row_weights is not None), ptr(src), src.shape[0], src.stride(0) if src.shape[0] > 0 else hidden,
            ptr(t), t_stride, t_width, ptr(row_weights), ptr(out_rows), num_units, hidden,
            ptr(w), w_stride, ptr(wsrc), num_weights, weights_offset, weights_pad,
            ptr(win_bases), win_bases.shape[0], int(win_bytes), ptr(error_flag), _stream_handle(stream))
        _lib.check(rc, 'combine_reduce_scatter')

    def build_local_plan(self, src_metadata: torch.Tensor, num_recv_tokens: int, num_topk: int,
                         num_max_tokens_per_rank: int, expanded: bool, plan: torch.Tensor,
                         num_tokens: int, topk_idx: Optional[torch.Tensor] = None,
                         wtable: Optional[torch.Tensor] = None, stream=None) -> None:
        _require(src_metadata.is_cuda and src_metadata.dtype == torch.int32 and src_metadata.is_contiguous(),
                 'recv_src_metadata must be contiguous int32 on the GPU')
        _require(plan.is_contiguous() and plan.dtype == torch.int32, 'plan must be contiguous int32')
        rc = self.lib.deepep_build_local_plan(
            ptr(src_metadata), num_recv_tokens, num_topk, num_max_tokens_per_rank, int(expanded),
            ptr(plan), plan.shape[1], num_tokens, ptr(topk_idx), ptr(wtable), _stream_handle(stream))
        _lib.check(rc, 'build_local_plan')

    # ------------------------------------------------------------------ dispatch (handle producer)
    def dispatch_route(self, topk_idx, num_experts, num_ranks, dst_slot, send_counts, stream=None):
        _require(topk_idx.is_cuda and topk_idx.dtype == torch.int64 and topk_idx.is_contiguous(), 'topk_idx int64')
        T, K = topk_idx.shape
        block_counts = torch.empty((max(1, (T + 255) // 256) * num_ranks,), dtype=torch.int32, device=topk_idx.device)
        rc = self.lib.deepep_dispatch_route(ptr(topk_idx), T, K, num_experts, num_ranks, ptr(dst_slot),
                                            ptr(send_counts), ptr(block_counts), _stream_handle(stream))
        _lib.check(rc, 'dispatch_route')

    def dispatch_notify(self, topk_idx, num_experts, num_ranks, num_blocks, dst_slot, notify, send_offsets,
                        stream=None):
        """The send side in two launches: dst_slot [T, R], notify int32 [R, 1 + E/R + 2 * num_blocks] (per
        destination: tokens | tokens per expert | per-block tokens | per-block pairs), send_offsets [R]."""
        _require(topk_idx.is_cuda and topk_idx.dtype == torch.int64 and topk_idx.is_contiguous(), 'topk_idx int64')
        T, K = topk_idx.shape
        W = 1 + num_experts // num_ranks + 2 * num_blocks
        _require(notify.dtype == torch.int32 and notify.is_contiguous() and tuple(notify.shape) == (num_ranks, W),
                 'notify must be contiguous int32 [num_ranks, 1 + experts_per_rank + 2 * num_blocks]')
        _require(dst_slot.dtype == torch.int32 and dst_slot.is_contiguous() and dst_slot.numel() == T * num_ranks,
                 'dst_slot must be contiguous int32 [num_tokens, num_ranks]')
        _require(send_offsets.dtype == torch.int32 and send_offsets.is_contiguous() and
                 send_offsets.numel() == num_ranks, 'send_offsets must be contiguous int32 [num_ranks]')
        ws_bytes = int(self.lib.deepep_dispatch_notify_workspace(T, num_experts, num_ranks))
        ws = torch.empty((max(ws_bytes, 16),), dtype=torch.uint8, device=topk_idx.device)
        rc = self.lib.deepep_dispatch_notify(ptr(topk_idx), T, K, num_experts, num_ranks, num_blocks, ptr(dst_slot),
                                             ptr(notify), ptr(send_offsets), ptr(ws), ws.numel(),
                                             _stream_handle(stream))
        _lib.check(rc, 'dispatch_notify')

    def dispatch_expert_counts(self, topk_idx, num_experts, counts, stream=None):
        """counts[e] = (t, k) entries routed to expert e (int32 [num_experts])."""
        _require(topk_idx.is_cuda and topk_idx.dtype == torch.int64 and topk_idx.is_contiguous(), 'topk_idx int64')
        _require(counts.dtype == torch.int32 and counts.is_contiguous() and counts.numel() == num_experts,
                 'expert counts must be contiguous int32 [num_experts]')
        T, K = topk_idx.shape
        rc = self.lib.deepep_dispatch_expert_counts(ptr(topk_idx), T, K, num_experts, ptr(counts),
                                                    _stream_handle(stream))
        _lib.check(rc, 'dispatch_expert_counts')

    # ------------------------------------------------------------------ EP > 1 combine plan (plan.hip)
    def route_block_counts(self, topk_idx, num_experts, num_ranks, num_blocks, tok, pairs, stream=None):
        """tok / pairs: int32 [num_ranks, num_blocks] (64-token blocks of this rank's tokens)."""
        _require(topk_idx.is_cuda and topk_idx.dtype == torch.int64 and topk_idx.is_contiguous(), 'topk_idx int64')
        for t in (tok, pairs):
            _require(t.dtype == torch.int32 and t.is_contiguous() and t.numel() == num_ranks * num_blocks,
                     'block counts must be contiguous int32 [num_ranks, num_blocks]')
        T, K = topk_idx.shape
        rc = self.lib.deepep_route_block_counts(ptr(topk_idx), T, K, num_experts, num_ranks, num_blocks, ptr(tok),
                                                ptr(pairs), _stream_handle(stream))
        _lib.check(rc, 'route_block_counts')

    def plan_expert(self, meta, num_topk, num_ranks, rank, num_max_tokens, recv_tok, recv_pairs, num_blocks,
                    blocks_per_chunk, flags, table_a, wtable_a, window_bases, window_row_bytes, out_rows,
                    window_bytes: int = 0, error_flag=None, padded_stride: int = 0, stream=None):
        """window_bytes: the data extent of every window (out_rows rows are bounded by it); error_flag:
        an error record (_lib.ERROR_RECORD_INTS ints) or None.  table_a / wtable_a / out_rows should be
        pre-filled with -1 / -1 / 0: a unit the kernel rejects is left as it was."""
        _require(meta.is_cuda and meta.dtype == torch.int32 and meta.is_contiguous(), 'recv_src_metadata int32')
        _require(table_a.dtype == torch.int32 and table_a.is_contiguous(), 'table_a int32')
        _require(wtable_a is None or (wtable_a.dtype == torch.int32 and wtable_a.is_contiguous()), 'wtable_a int32')
        _require(out_rows is None or (out_rows.dtype == torch.int64 and out_rows.is_contiguous() and
                                      window_bases is not None and window_bytes > 0),
                 'out_rows int64 with window bases and extent')
        rc = self.lib.deepep_plan_expert(ptr(meta), meta.shape[0], num_topk, num_ranks, rank, num_max_tokens,
                                         ptr(recv_tok), ptr(recv_pairs), num_blocks, blocks_per_chunk, flags,
                                         ptr(table_a), ptr(wtable_a), ptr(window_bases), window_row_bytes,
                                         int(window_bytes), ptr(out_rows), ptr(error_flag), int(padded_stride),
                                         _stream_handle(stream))
        _lib.check(rc, 'plan_expert')

    def plan_source(self, topk_idx, num_experts, num_ranks, rank, num_max_tokens, dst_slot, send_tok, send_pairs,
                    num_blocks, blocks_per_chunk, flags, row_floats, weights_offset, table_b, wtable,
                    padded_stride: int = 0, stream=None):
        _require(topk_idx.is_cuda and topk_idx.dtype == torch.int64 and topk_idx.is_contiguous(), 'topk_idx int64')
        _require(table_b.dtype == torch.int32 and table_b.is_contiguous(), 'table_b int32')
        _require(wtable is None or (wtable.dtype == torch.int32 and wtable.is_contiguous()), 'wtable int32')
        T, K = topk_idx.shape
        rc = self.lib.deepep_plan_source(ptr(topk_idx), T, K, num_experts, num_ranks, rank, num_max_tokens, ptr(dst_slot),
                                         ptr(send_tok), ptr(send_pairs), num_blocks, blocks_per_chunk, flags,
                                         row_floats, weights_offset, ptr(table_b), table_b.shape[1], ptr(wtable),
                                         int(padded_stride), _stream_handle(stream))
        _lib.check(rc, 'plan_source')

    def dispatch_pack(self, x_bytes, sf_bytes, topk_idx, topk_weights, src_base, dst_slot, send_offsets,
                      packed, layout: RowLayout, dest_bases=None, dest_rows: Optional[int] = None, error_flag=None,
                      stream=None):
        """x_bytes / sf_bytes: [T, bytes] uint8 views (rows may be strided).  dest_bases: optional
        int64 [R] device tensor of per-destination buffer addresses (peer windows) instead of `packed`;
        dest_rows: the rows each destination holds (default: the rows of `packed`); a row past it is
        not stored (flagged in error_flag, an error record of _lib.ERROR_RECORD_INTS ints)."""
        T, K = topk_idx.shape
        if dest_bases is not None:
            _require(dest_bases.is_cuda and dest_bases.dtype == torch.int64 and dest_bases.is_contiguous() and
                     dest_bases.numel() == dst_slot.shape[1], 'dest_bases must be int64 [num_ranks] on the GPU')
            _require(dest_rows is not None, 'dest_rows (rows per destination window) is required with dest_bases')
        else:
            dest_rows = packed.shape[0] if dest_rows is None else min(dest_rows, packed.shape[0])
        rc = self.lib.deepep_dispatch_pack(
            ptr(x_bytes), x_bytes.stride(0) if T else layout.x_bytes, layout.x_bytes,
            ptr(sf_bytes), sf_bytes.stride(0) if sf_bytes is not None and T else 0, layout.sf_bytes,
            ptr(topk_idx), ptr(topk_weights), T, K, src_base, ptr(dst_slot), ptr(send_offsets),
            dst_slot.shape[1], ptr(packed), ptr(dest_bases), layout.row_bytes, int(dest_rows), layout.sf_off,
            layout.idx_off,
            layout.w_off, layout.src_off, ptr(error_flag), _stream_handle(stream))
        _lib.check(rc, 'dispatch_pack')

    def dispatch_count(self, packed, layout: RowLayout, num_recv, rank, num_local_experts, rank_psum, meta,
                       recv_topk_idx, block_counts, pad_rows: int = 0, row_map=None, rank_counts=None,
                       psum_out=None, own_first: bool = False, stream=None):
        """rank_psum: inclusive prefix of rows per source rank (int32 [R]); or, with rank_psum None,
        rank_counts: rows per source rank (an int32 [R] view of any stride, e.g. the notify records'
        first column), whose prefix the kernel forms and writes to psum_out (int32 [R]).
        pad_rows > 0: `packed` is a worst-case-sized receive buffer, source s's rows at s * pad_rows;
        row_map (int32 [num_recv]) receives each received row's packed row (for slots / copy).
        own_first: `packed` = [rows from this rank | rows from the others, rank order] (the local bypass);
        row_map is written the same way."""
        src = rank_psum if rank_psum is not None else rank_counts
        _require(src is not None and src.dim() == 1 and src.dtype == torch.int32 and src.stride(0) >= 1,
                 'dispatch_count needs rank_psum or rank_counts (int32 [num_ranks])')
        R = src.shape[0]
        stride = 0 if rank_psum is not None else src.stride(0)
        _require(psum_out is None or (psum_out.dtype == torch.int32 and psum_out.is_contiguous() and
                                      psum_out.numel() == R), 'psum_out must be contiguous int32 [num_ranks]')
        _require(pad_rows == 0 or (row_map is not None and row_map.dtype == torch.int32 and
                                   row_map.numel() >= num_recv and packed.shape[0] >= pad_rows * R),
                 'padded receive rows need a row map and R * pad_rows packed rows')
        _require(not own_first or (row_map is not None and row_map.dtype == torch.int32 and
                                   row_map.numel() >= num_recv), 'own-first receive rows need a row map')
        rc = self.lib.deepep_dispatch_count(
            ptr(packed), layout.row_bytes, layout.idx_off, layout.src_off, num_recv, layout.num_topk, rank,
            num_local_experts, ptr(src), R, stride, ptr(psum_out), pad_rows, int(own_first), ptr(row_map), ptr(meta),
            ptr(recv_topk_idx), ptr(block_counts), _stream_handle(stream))
        _lib.check(rc, 'dispatch_count')

    def dispatch_receive(self, packed, layout: RowLayout, num_recv, rank, num_local_experts, rank_counts, psum_out,
                         meta, recv_topk_idx, block_counts, expert_alignment, expanded, expert_counts, psum_expert,
                         inv=None, pad_rows: int = 0, row_map=None, own_first: bool = False, stream=None):
        """count (counts mode) -> scan -> slots (expanded) in one call: the receive side's launches back to
        back.  Non-expanded: meta columns 2.. become -1."""
        _require(rank_counts.dim() == 1 and rank_counts.dtype == torch.int32 and rank_counts.stride(0) >= 1,
                 'rank_counts must be an int32 [num_ranks] view')
        R = rank_counts.shape[0]
        _require(psum_out.dtype == torch.int32 and psum_out.is_contiguous() and psum_out.numel() == R,
                 'psum_out must be contiguous int32 [num_ranks]')
        _require(pad_rows == 0 or (row_map is not None and row_map.dtype == torch.int32 and
                                   row_map.numel() >= num_recv and packed.shape[0] >= pad_rows * R),
                 'padded receive rows need a row map and R * pad_rows packed rows')
        _require(not own_first or (row_map is not None and row_map.dtype == torch.int32 and
                                   row_map.numel() >= num_recv), 'own-first receive rows need a row map')
        _require(inv is None or (inv.dtype == torch.int32 and inv.is_contiguous()), 'inv int32')
        rc = self.lib.deepep_dispatch_receive(
            ptr(packed), layout.row_bytes, layout.idx_off, layout.src_off, num_recv, layout.num_topk, rank,
            num_local_experts, ptr(rank_counts), R, rank_counts.stride(0), ptr(psum_out), pad_rows, int(own_first),
            ptr(row_map),
            ptr(meta), ptr(recv_topk_idx), ptr(block_counts), expert_alignment, int(expanded), ptr(expert_counts),
            ptr(psum_expert), ptr(inv), _stream_handle(stream))
        _lib.check(rc, 'dispatch_receive')

    def dispatch_scan(self, block_counts, num_local_experts, expert_alignment, expanded, expert_counts,
                      psum_expert, stream=None):
        rc = self.lib.deepep_dispatch_scan(ptr(block_counts), block_counts.shape[0], num_local_experts,
                                           expert_alignment, int(expanded), ptr(expert_counts), ptr(psum_expert),
                                           _stream_handle(stream))
        _lib.check(rc, 'dispatch_scan')

    def dispatch_slots(self, packed, layout: RowLayout, num_recv, rank, num_local_experts, block_offsets, meta,
                       inv=None, row_map=None, stream=None):
        """inv: optional int32 [expanded rows]: inv[slot] = row * K + lane (the expanded copy's map)."""
        _require(inv is None or (inv.dtype == torch.int32 and inv.is_contiguous()), 'inv int32')
        rc = self.lib.deepep_dispatch_slots(ptr(packed), layout.row_bytes, layout.idx_off, num_recv,
                                            layout.num_topk, rank, num_local_experts, ptr(block_offsets),
                                            ptr(meta), ptr(inv), ptr(row_map), _stream_handle(stream))
        _lib.check(rc, 'dispatch_slots')

    def dispatch_copy(self, packed, layout: RowLayout, num_recv, meta, expanded, recv_x_bytes, recv_sf_bytes,
                      recv_w, x_direct=None, sf_direct=None, num_max_tokens: int = 0, error_flag=None,
                      inv=None, block_offsets=None, expert_end=None, row_map=None, stream=None):
        """x_direct / sf_direct: [T, bytes] uint8 views of the sender's rows (one rank: the packed rows
        then carry only metadata and row i's x is x_direct[src_metadata[i][0] % num_max_tokens]).
        inv / block_offsets / expert_end (expanded): the blocked destination-major copy (dispatch_slots'
        inverse map, dispatch_scan's per-block offsets [blocks, local experts] and psum_expert)."""
        if inv is not None:
            _require(expanded and block_offsets is not None and expert_end is not None and
                     block_offsets.dim() == 2 and block_offsets.shape[0] ==
                     (num_recv + _lib.DISPATCH_BLOCK_ROWS - 1) // _lib.DISPATCH_BLOCK_ROWS and
                     expert_end.numel() == block_offsets.shape[1], 'blocked copy tables')
        x_bytes = x_direct.shape[1] if x_direct is not None else layout.x_bytes
        sf_bytes = sf_direct.shape[1] if sf_direct is not None else layout.sf_bytes
        rc = self.lib.deepep_dispatch_copy(ptr(packed), layout.row_bytes, x_bytes, layout.sf_off,
                                           sf_bytes, layout.w_off, num_recv, layout.num_topk, ptr(meta),
                                           int(expanded),
                                           ptr(x_direct), x_direct.stride(0) if x_direct is not None else 0,
                                           ptr(sf_direct), sf_direct.stride(0) if sf_direct is not None else 0,
                                           num_max_tokens,
                                           ptr(recv_x_bytes), ptr(recv_sf_bytes), ptr(recv_w),
                                           recv_x_bytes.shape[0], ptr(inv), ptr(block_offsets), ptr(expert_end),
                                           block_offsets.shape[1] if block_offsets is not None else 0,
                                           ptr(row_map), ptr(error_flag), _stream_handle(stream))
        _lib.check(rc, 'dispatch_copy')

    def combine_buffer_size(self, num_max_tokens_per_rank: int, hidden: int, num_topk: int,
                            num_ranks: int, allow_multiple_reduction: bool) -> int:
        v = self.lib.deepep_combine_buffer_size(num_max_tokens_per_rank, hidden, num_topk, num_ranks,
                                                int(allow_multiple_reduction))
        _lib.check(0 if v >= 0 else int(v), 'combine_buffer_size')
        return int(v)
