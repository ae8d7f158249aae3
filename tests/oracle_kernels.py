"""A CPU kernel provider backed by the oracle -- TEST INFRASTRUCTURE ONLY.

It has the interface of deepep_amd.kernels.HipKernels and is injected by the CPU
tests into ElasticBuffer (`buffer._kernels = OracleKernels()`) to exercise the host
orchestration (plans, dispatch, RCCL/gloo exchange, stream bookkeeping) without a
GPU.  The product never selects it.
"""
from typing import Optional

import torch

import oracle
from deepep_amd._lib import DISPATCH_BLOCK_ROWS
from tests import plan_ref


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


class OracleKernels:
    name = 'oracle'

    def combine_reduce(self, mode, src, out, num_units, table=None, row_weights=None, bias0=None, bias1=None,
                       wtable=None, wsrc=None, out_weights=None, units_per_block=0, error_flag=None, weights_pad=0,
                       stream=None):
        assert src.device.type == 'cpu' and out.device.type == 'cpu'
        for t in (src, out, table, row_weights, bias0, bias1, wtable, wsrc, out_weights):
            assert t is None or t.dim() == 1 or t.stride(-1) == 1
        hidden = out.shape[1]
        rc = oracle.rows_lib().oracle_combine_rows(
            mode, int(row_weights is not None),
            _p(src), src.shape[0], src.stride(0) if src.shape[0] else hidden,
            _p(table), table.stride(0) if table is not None else 0, table.shape[1] if table is not None else 1,
            _p(row_weights), _p(bias0), _p(bias1),
            _p(out), out.stride(0) if out.shape[0] else hidden, num_units, hidden,
            _p(wtable), wtable.stride(0) if wtable is not None else 0,
            _p(wsrc), _p(out_weights), out_weights.shape[1] if out_weights is not None else 0,
            out_weights.stride(0) if out_weights is not None else 0)
        assert rc == 0, 'oracle_combine_rows failed'
        if out_weights is not None and weights_pad > out_weights.shape[1] and num_units:
            wide = torch.as_strided(out_weights, (num_units, weights_pad), (out_weights.stride(0), 1))
            wide[:, out_weights.shape[1]:] = 0                  # the rest of the row's tail line

    def build_local_plan(self, src_metadata, num_recv_tokens, num_topk, num_max_tokens_per_rank, expanded,
                         plan, num_tokens, topk_idx=None, wtable=None, stream=None):
        meta = src_metadata[:num_recv_tokens]
        plan.fill_(-1)
        rows = (meta[:, 0] >= 0).nonzero(as_tuple=True)[0]     # metadata -1: not a received row (C: -1 % n < 0)
        t = (meta[rows, 0] % num_max_tokens_per_rank).long()
        if expanded:
            plan[t] = meta[rows, 2:2 + plan.shape[1]]
        else:
            plan[t, 0] = rows.to(torch.int32)
        if wtable is not None:
            wtable.fill_(-1)
            inv = torch.full((num_tokens,), -1, dtype=torch.int64)
            inv[t] = rows
            k = torch.arange(num_topk).view(1, -1)
            ok = (topk_idx >= 0) & (inv.view(-1, 1) >= 0)
            wtable.copy_(torch.where(ok, inv.view(-1, 1) * num_topk + k, torch.full_like(topk_idx, -1)).to(torch.int32))

    # ------------------------------------------------------------------ EP > 1 plan (tests/plan_ref.py)
    def route_block_counts(self, topk_idx, num_experts, num_ranks, num_blocks, tok, pairs, stream=None):
        t, p = plan_ref.route_block_counts(topk_idx, num_experts, num_ranks, num_blocks)
        tok.copy_(t)
        pairs.copy_(p)

    def plan_expert(self, meta, num_topk, num_ranks, rank, num_max_tokens, recv_tok, recv_pairs, num_blocks,
                    blocks_per_chunk, flags, table_a, wtable_a, window_bases, window_row_bytes, out_rows,
                    window_bytes=0, error_flag=None, padded_stride=0, stream=None):
        plan_ref.plan_expert(meta, num_topk, num_ranks, rank, num_max_tokens, recv_tok, recv_pairs, num_blocks,
                             blocks_per_chunk, flags, table_a, wtable_a, window_bases, window_row_bytes, out_rows,
                             padded=padded_stride)

    def plan_source(self, topk_idx, num_experts, num_ranks, rank, num_max_tokens, dst_slot, send_tok, send_pairs,
                    num_blocks, blocks_per_chunk, flags, row_floats, weights_offset, table_b, wtable,
                    padded_stride=0, stream=None):
        plan_ref.plan_source(topk_idx, num_experts, num_ranks, rank, num_max_tokens, dst_slot, send_tok, send_pairs,
                             num_blocks, blocks_per_chunk, flags, row_floats, weights_offset, table_b, wtable,
                             padded=padded_stride)

    # ------------------------------------------------------------------ dispatch primitives (CPU stand-ins)
    def dispatch_route(self, topk_idx, num_experts, num_ranks, dst_slot, send_counts, stream=None):
        epr = num_experts // num_ranks
        rank_of = torch.where(topk_idx >= 0, torch.div(topk_idx, epr, rounding_mode='floor'),
                              torch.full_like(topk_idx, -1))
        is_to = (rank_of.unsqueeze(-1) == torch.arange(num_ranks).view(1, 1, -1)).any(dim=1)
        dst_slot.copy_(torch.where(is_to, torch.cumsum(is_to.to(torch.int64), 0) - 1,
                                   torch.full(is_to.shape, -1, dtype=torch.int64)).to(torch.int32))
        send_counts.copy_(is_to.sum(dim=0).to(torch.int32))

    def dispatch_notify(self, topk_idx, num_experts, num_ranks, num_blocks, dst_slot, notify, send_offsets,
                        stream=None):
        R, epr = num_ranks, num_experts // num_ranks
        send_counts = torch.empty((R,), dtype=torch.int32)
        self.dispatch_route(topk_idx, num_experts, R, dst_slot, send_counts)
        hist = torch.empty((num_experts,), dtype=torch.int32)
        self.dispatch_expert_counts(topk_idx, num_experts, hist)
        notify[:, 0] = send_counts
        notify[:, 1:1 + epr] = hist.view(R, epr)
        if num_blocks:
            tok = torch.empty((R, num_blocks), dtype=torch.int32)
            pairs = torch.empty((R, num_blocks), dtype=torch.int32)
            self.route_block_counts(topk_idx, num_experts, R, num_blocks, tok, pairs)
            notify[:, 1 + epr:1 + epr + num_blocks] = tok
            notify[:, 1 + epr + num_blocks:] = pairs
        send_offsets.copy_((torch.cumsum(send_counts, 0) - send_counts).to(torch.int32))

    def dispatch_expert_counts(self, topk_idx, num_experts, counts, stream=None):
        valid = topk_idx[topk_idx >= 0].view(-1)
        counts.copy_(torch.bincount(valid, minlength=num_experts)[:num_experts].to(torch.int32))

    def dispatch_pack(self, x_bytes, sf_bytes, topk_idx, topk_weights, src_base, dst_slot, send_offsets,
                      packed, layout, dest_bases=None, dest_rows=None, error_flag=None, stream=None):
        assert dest_bases is None, 'the CPU stand-in packs into one local buffer'
        t_idx, r_idx = (dst_slot >= 0).nonzero(as_tuple=True)
        dest = (send_offsets[r_idx] + dst_slot[t_idx, r_idx]).long()
        K = layout.num_topk
        packed[dest, :layout.x_bytes] = x_bytes[t_idx]
        if sf_bytes is not None:
            packed[dest, layout.sf_off:layout.sf_off + layout.sf_bytes] = sf_bytes[t_idx]
        packed[dest, layout.idx_off:layout.idx_off + 8 * K] = topk_idx[t_idx].contiguous().view(torch.uint8).view(-1, 8 * K)
        w = topk_weights if topk_weights is not None else torch.zeros(topk_idx.shape, dtype=torch.float32)
        packed[dest, layout.w_off:layout.w_off + 4 * K] = w[t_idx].contiguous().view(torch.uint8).view(-1, 4 * K)
        src = (src_base + t_idx).to(torch.int32)
        packed[dest, layout.src_off:layout.src_off + 4] = src.view(torch.uint8).view(-1, 4)

    @staticmethod
    def _rows(packed, N, row_map):
        """The packed rows of received rows 0..N-1 (a padded receive buffer reads through row_map)."""
        return packed[:N] if row_map is None else packed[row_map[:N].long()]

    @staticmethod
    def _local(packed, layout, N, rank, epr, row_map=None):
        K = layout.num_topk
        packed = OracleKernels._rows(packed, N, row_map)
        idx = packed[:N, layout.idx_off:layout.idx_off + 8 * K].contiguous().view(torch.int64).view(N, K)
        inr = (idx >= rank * epr) & (idx < (rank + 1) * epr)
        return torch.where(inr, idx - rank * epr, torch.full_like(idx, -1))

    def dispatch_count(self, packed, layout, num_recv, rank, num_local_experts, rank_psum, meta, recv_topk_idx,
                       block_counts, pad_rows=0, row_map=None, rank_counts=None, psum_out=None, own_first=False,
                       stream=None):
        K, epr = layout.num_topk, num_local_experts
        if rank_psum is None:
            rank_psum = torch.cumsum(rank_counts, 0).to(torch.int32)
            if psum_out is not None:
                psum_out.copy_(rank_psum)
        if num_recv == 0:
            return
        N = min(num_recv, int(rank_psum[-1]))          # rows received; the rest get metadata -1
        meta[N:num_recv, :2] = -1
        if recv_topk_idx is not None:
            recv_topk_idx[N:num_recv] = -1
        src_rank = torch.searchsorted(rank_psum.to(torch.int64), torch.arange(N), right=True).clamp(max=rank_psum.numel() - 1)
        start = torch.cat([torch.zeros(1, dtype=torch.int64), rank_psum.to(torch.int64)])[src_rank]
        if pad_rows:
            slot = src_rank
            if own_first:                                # receive order [rank, 0, .., rank - 1, rank + 1, ..]
                slot = torch.where(src_rank == rank, torch.zeros_like(src_rank),
                                   torch.where(src_rank < rank, src_rank + 1, src_rank))
            row_map[:N] = (slot * pad_rows + torch.arange(N) - start).to(torch.int32)
        elif own_first:
            # [rows from this rank | the other sources' rows in rank order] (the local bypass)
            psum = rank_psum.to(torch.int64)
            own_start = int(psum[rank - 1]) if rank > 0 else 0
            own_rows = int(psum[rank]) - own_start
            i = torch.arange(N)
            row_map[:N] = torch.where(src_rank == rank, i - own_start,
                                      torch.where(src_rank < rank, i + own_rows, i)).to(torch.int32)
        rm = row_map if pad_rows or own_first else None
        le = self._local(packed, layout, N, rank, epr, rm)
        src = self._rows(packed, N, rm)[:, layout.src_off:layout.src_off + 4].contiguous().view(torch.int32).view(N)
        master = torch.where(le >= 0, torch.arange(K).view(1, K), torch.full_like(le, -1)).amax(dim=1)
        meta[:N, 0] = src
        meta[:N, 1] = (src_rank * K + master).to(torch.int32)
        if recv_topk_idx is not None:
            recv_topk_idx[:N].copy_(le)
        block_counts.zero_()
        rows = DISPATCH_BLOCK_ROWS
        for b in range(block_counts.shape[0]):
            chunk = le[b * rows:(b + 1) * rows]
            chunk = chunk[chunk >= 0]
            block_counts[b] += torch.bincount(chunk, minlength=epr).to(torch.int32)

    def dispatch_receive(self, packed, layout, num_recv, rank, num_local_experts, rank_counts, psum_out, meta,
                         recv_topk_idx, block_counts, expert_alignment, expanded, expert_counts, psum_expert,
                         inv=None, pad_rows=0, row_map=None, own_first=False, stream=None):
        self.dispatch_count(packed, layout, num_recv, rank, num_local_experts, None, meta, recv_topk_idx, block_counts,
                            pad_rows=pad_rows, row_map=row_map, rank_counts=rank_counts, psum_out=psum_out,
                            own_first=own_first)
        self.dispatch_scan(block_counts, num_local_experts, expert_alignment, expanded, expert_counts, psum_expert)
        if expanded:
            self.dispatch_slots(packed, layout, num_recv, rank, num_local_experts, block_counts, meta, inv=inv,
                                row_map=row_map)
        else:
            meta[:num_recv, 2:] = -1

    def dispatch_scan(self, block_counts, num_local_experts, expert_alignment, expanded, expert_counts, psum_expert,
                      stream=None):
        counts = block_counts.sum(dim=0).to(torch.int64)
        excl = torch.cumsum(block_counts.to(torch.int64), dim=0) - block_counts
        aligned = (counts + expert_alignment - 1) // expert_alignment * expert_alignment
        start = torch.cumsum(aligned, 0) - aligned
        block_counts.copy_((excl + start.view(1, -1)).to(torch.int32))
        expert_counts.copy_(counts.to(torch.int32))
        psum_expert.copy_((start + counts if expanded else start + aligned).to(torch.int32))

    def dispatch_slots(self, packed, layout, num_recv, rank, num_local_experts, block_offsets, meta, inv=None,
                       row_map=None, stream=None):
        n = int((meta[:num_recv, 0] >= 0).sum())         # the received rows come first
        le = torch.full((num_recv, layout.num_topk), -1, dtype=torch.int64)
        le[:n] = self._local(packed, layout, n, rank, num_local_experts, row_map)
        meta[:num_recv, 2:] = -1
        rows = DISPATCH_BLOCK_ROWS
        for b in range(block_offsets.shape[0]):
            run = block_offsets[b].clone()
            for i in range(b * rows, min(num_recv, (b + 1) * rows)):
                if int(meta[i, 0]) < 0:                  # past the received rows
                    continue
                for k in range(layout.num_topk):
                    e = int(le[i, k])
                    if e >= 0:
                        meta[i, 2 + k] = run[e]
                        if inv is not None:
                            inv[run[e]] = i * layout.num_topk + k
                        run[e] += 1

    def dispatch_copy(self, packed, layout, num_recv, meta, expanded, recv_x_bytes, recv_sf_bytes, recv_w,
                      x_direct=None, sf_direct=None, num_max_tokens=0, error_flag=None, inv=None,
                      block_offsets=None, expert_end=None, row_map=None, stream=None):
        K = layout.num_topk
        N = int((meta[:num_recv, 0] >= 0).sum())         # the received rows come first
        packed = self._rows(packed, N, row_map)
        if x_direct is not None:
            t = (meta[:N, 0].long() % num_max_tokens)
            xs = x_direct[t]
            sfs = sf_direct[t] if sf_direct is not None else None
        else:
            xs = packed[:N, :layout.x_bytes]
            sfs = packed[:N, layout.sf_off:layout.sf_off + layout.sf_bytes]
        w = packed[:N, layout.w_off:layout.w_off + 4 * K].contiguous().view(torch.float32).view(N, K)
        if not expanded:
            recv_x_bytes[:N] = xs
            if recv_sf_bytes is not None:
                recv_sf_bytes[:N] = sfs
            if recv_w is not None:
                recv_w[:N] = w
            return
        ii, kk = (meta[:N, 2:] >= 0).nonzero(as_tuple=True)
        rows = meta[ii, 2 + kk].long()
        recv_x_bytes[rows] = xs[ii]
        if recv_sf_bytes is not None:
            recv_sf_bytes[rows] = sfs[ii]
        if recv_w is not None:
            recv_w[rows] = w[ii, kk]
