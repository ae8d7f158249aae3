"""CPU restatement of the EP > 1 combine plan -- TEST INFRASTRUCTURE ONLY.

The product builds these tables with HIP kernels (deepep_amd/csrc/plan.hip, C-ABI
deepep_route_block_counts / deepep_plan_expert / deepep_plan_source).  This module states the
same tables from their definitions with plain torch on the CPU, straight from the reference's
addressing rules, so that

* tests/oracle_kernels.py can run the whole EP > 1 host orchestration on gloo ranks without a GPU,
* tests/test_sync_free_gpu.py can check the HIP plan kernels against it bit for bit.

Reference rules restated (paths in /root/reference):
* the partial of received token i goes to its source rank's receive slot
  `use_rank_layout ? my_rank : master_topk` at token row src_token (combine.cuh:96-106,
  combine_utils.cuh:8-13);
* phase B visits a token's partials in ascending order of each rank's dedup master lane (its
  highest top-k lane, combine_reduce_epilogue.cuh:74-95, ptx.cuh:412-421);
* the single reduction (kDoExpandedSend, combine.cuh:177-213) sends every valid (row, lane)
  unreduced, into per-top-k slots (buffer.hpp:616-633).
The exchange geometry (64-token blocks, chunks of whole blocks, send buffers grouped by peer
rank in ascending (token, lane) order, round-robin unit order for the xGMI stores) is this
build's, DESIGN.md section 5.
"""
import torch

BLOCK = 64
EXPANDED, SINGLE, INTERLEAVE, RANK_LAYOUT, WINDOW, LOCAL_BYPASS = 1, 2, 4, 8, 16, 32


def _rank_of(topk_idx: torch.Tensor, num_experts: int, num_ranks: int) -> torch.Tensor:
    epr = num_experts // num_ranks
    return torch.where(topk_idx >= 0, torch.div(topk_idx, epr, rounding_mode='floor'), torch.full_like(topk_idx, -1))


def route_block_counts(topk_idx, num_experts, num_ranks, num_blocks):
    """(tok, pairs) int32 [R, nb]: tokens / (token, lane) pairs of every 64-token block routed to each rank."""
    T = topk_idx.shape[0]
    R = num_ranks
    rank_of = _rank_of(topk_idx.long(), num_experts, R)
    pairs_t = (rank_of.unsqueeze(-1) == torch.arange(R).view(1, 1, R)).sum(dim=1)          # [T, R]
    blk = torch.arange(T) // BLOCK
    tok = torch.zeros((R, num_blocks), dtype=torch.int64)
    pairs = torch.zeros((R, num_blocks), dtype=torch.int64)
    tok.index_add_(1, blk, (pairs_t > 0).to(torch.int64).T)
    pairs.index_add_(1, blk, pairs_t.T)
    return tok.to(torch.int32), pairs.to(torch.int32)


def send_order(l: int, rank: int, R: int, bypass: bool) -> int:
    """Place of peer l's group in a chunk's send rows: rank order, or with the local bypass rank order
    without `rank`, whose own units come last (include/deepep_amd.h, DEEPEP_PLAN_LOCAL_BYPASS)."""
    if not bypass:
        return l
    return R - 1 if l == rank else (l - 1 if l > rank else l)


def recv_order(l: int, rank: int, bypass: bool) -> int:
    """Place of peer l's group in a chunk's receive rows: rank order, or with the local bypass `rank`'s
    own rows first, then the other ranks in order."""
    if not bypass:
        return l
    return 0 if l == rank else (l + 1 if l < rank else l)


def _positions(unit_src, unit_chunk, counts, R, interleave, padded=0, rank=0, bypass=False):
    """Unit index of every unit (given in receive order) inside the concatenated chunk tables:
    chunk base + position inside the chunk (grouped by source rank in send_order, or round-robin).
    padded > 0: every chunk holds R * padded positions, unit p of source s at send_order(s) * padded + p
    (p * R + s); a unit p >= padded is rejected (-1: not stored)."""
    n = unit_src.numel()                                       # counts: [chunks, R]
    base = torch.cumsum(counts.sum(dim=1), 0) - counts.sum(dim=1)
    if padded:
        base = torch.arange(counts.shape[0]) * R * padded
    # p = rank of the unit among the units of its (source, chunk) group, in receive order
    key = unit_chunk * R + unit_src
    order = torch.argsort(key, stable=True)
    sorted_key = key[order]
    first = torch.searchsorted(sorted_key, sorted_key, right=False)
    p = torch.empty(n, dtype=torch.int64)
    p[order] = torch.arange(n) - first
    out = torch.empty(n, dtype=torch.int64)
    for i in range(n):
        c, s, pi = int(unit_chunk[i]), int(unit_src[i]), int(p[i])
        if padded and pi >= padded:
            out[i] = -1
            continue
        if padded:
            pos = pi * R + s if interleave else send_order(s, rank, R, bypass) * padded + pi
        elif interleave:
            pos = sum(min(int(counts[c, l]), pi + (1 if l < s else 0)) for l in range(R))
        else:
            os_ = send_order(s, rank, R, bypass)
            pos = sum(int(counts[c, l]) for l in range(R) if send_order(l, rank, R, bypass) < os_) + pi
        out[i] = int(base[c]) + pos
    return out


def plan_expert(meta, num_topk, num_ranks, rank, num_max_tokens, recv_tok, recv_pairs, num_blocks,
                blocks_per_chunk, flags, table_a, wtable_a, window_bases, window_row_bytes, out_rows, padded=0):
    K, R, T_max, bpc = num_topk, num_ranks, num_max_tokens, blocks_per_chunk
    single, expanded = bool(flags & SINGLE), bool(flags & EXPANDED)
    bypass = bool(flags & LOCAL_BYPASS) and not flags & INTERLEAVE
    n_recv = int(recv_tok.sum())
    m = meta[:n_recv].long()
    src = torch.div(m[:, 1], K, rounding_mode='floor')
    st = m[:, 0] % T_max
    chunk = torch.div(torch.div(st, BLOCK, rounding_mode='floor'), bpc, rounding_mode='floor')
    C = (num_blocks + bpc - 1) // bpc
    cnt = (recv_pairs if single else recv_tok).long()
    counts = torch.stack([cnt[:, c * bpc:(c + 1) * bpc].sum(dim=1) for c in range(C)])    # [C, R]
    if single:
        ii, kk = (m[:, 2:] >= 0).nonzero(as_tuple=True)         # (row, lane) order
        u = _positions(src[ii], chunk[ii], counts, R, bool(flags & INTERLEAVE), padded, rank, bypass)
        keep = u >= 0
        u, ii, kk = u[keep], ii[keep], kk[keep]
        table_a[u, 0] = m[ii, 2 + kk].to(torch.int32)
        if out_rows is not None:
            bases = window_bases.long().cpu()
            ok = (m[ii, 0] >= 0) & (m[ii, 1] >= 0) & (src[ii] < R)        # else a null row (plan.hip)
            addr = bases[src[ii].clamp(0, R - 1)] + (kk * T_max + st[ii]) * window_row_bytes
            out_rows[u] = torch.where(ok, addr, torch.zeros_like(addr)).to(out_rows.dtype)
        return
    u = _positions(src, chunk, counts, R, bool(flags & INTERLEAVE), padded, rank, bypass)
    rows = torch.arange(n_recv)
    if expanded:
        table_a[u] = m[:, 2:2 + K].to(torch.int32)
    else:
        table_a[u, 0] = rows.to(torch.int32)
        if wtable_a is not None:
            wtable_a[u] = (rows.view(-1, 1) * K + torch.arange(K).view(1, K)).to(torch.int32)
    if out_rows is not None:
        slot = torch.full_like(src, rank) if flags & RANK_LAYOUT else m[:, 1] % K
        bases = window_bases.long().cpu()
        ok = (m[:, 0] >= 0) & (m[:, 1] >= 0) & (src < R)                 # else a null row (plan.hip)
        addr = bases[src.clamp(0, R - 1)] + (slot * T_max + st) * window_row_bytes
        out_rows[u] = torch.where(ok, addr, torch.zeros_like(addr)).to(out_rows.dtype)


def plan_source(topk_idx, num_experts, num_ranks, rank, num_max_tokens, dst_slot, send_tok, send_pairs, num_blocks,
                blocks_per_chunk, flags, row_floats, weights_offset, table_b, wtable, padded=0):
    """Per owned token, from the routing alone (running counters, not dst_slot)."""
    T, K = topk_idx.shape
    R, T_max, bpc = num_ranks, num_max_tokens, blocks_per_chunk
    single, window, rank_layout = bool(flags & SINGLE), bool(flags & WINDOW), bool(flags & RANK_LAYOUT)
    bypass = bool(flags & LOCAL_BYPASS) and not window

    def base(c, d):
        """First row of expert rank d's group in chunk c's receive rows (recv_order)."""
        o = recv_order(d, rank, bypass)
        if padded:
            return o * padded
        return sum(int(counts[c, l]) for l in range(R) if recv_order(l, rank, bypass) < o)
    rank_of = _rank_of(topk_idx.long().cpu(), num_experts, R)
    C = (num_blocks + bpc - 1) // bpc
    cnt = (send_pairs if single else send_tok).long().cpu()
    counts = torch.stack([cnt[:, c * bpc:(c + 1) * bpc].sum(dim=1) for c in range(C)])    # [C, R]
    running = torch.zeros((C, R), dtype=torch.int64)
    width = table_b.shape[1]
    tb = torch.full((T, width), -1, dtype=torch.int64)
    wt = torch.full((T, K), -1, dtype=torch.int64)
    for t in range(T):
        c = (t // BLOCK) // bpc
        ranks = rank_of[t].tolist()
        if single:
            for k, d in enumerate(ranks):
                if d < 0:
                    continue
                if window:
                    tb[t, k] = k * T_max + t
                else:
                    ok = not padded or int(running[c, d]) < padded     # past d's padded rows: rejected
                    tb[t, k] = base(c, d) + int(running[c, d]) if ok else -1
                    running[c, d] += 1
            continue
        master = {d: k for k, d in enumerate(ranks) if d >= 0}            # highest lane wins
        row = {}
        for d, mk in master.items():
            if window:
                row[d] = (d if rank_layout else mk) * T_max + t
            else:
                row[d] = base(c, d) + int(running[c, d])
                running[c, d] += 1
        for j, d in enumerate(sorted(master, key=lambda d: master[d])[:width]):
            tb[t, j] = row[d]
        for k, d in enumerate(ranks):
            if d >= 0:
                wt[t, k] = row[d] * row_floats + weights_offset + k
    table_b.copy_(tb.to(torch.int32))
    if wtable is not None:
        wtable.copy_(wt.to(torch.int32))


def interleave_by_rank(units: torch.Tensor, dest_rank: torch.Tensor, num_ranks: int) -> torch.Tensor:
    """Round-robin unit order over the destination ranks (the xGMI phase-A order): the stable sort
    of (position inside its destination's run) * R + destination."""
    if units.numel() == 0 or num_ranks == 1:
        return units
    d = dest_rank[units]
    counts = torch.bincount(d, minlength=num_ranks)
    start = torch.cumsum(counts, 0) - counts
    pos = torch.arange(units.numel(), device=units.device) - start[d]
    return units[torch.argsort(pos * num_ranks + d)]


def epilogue_tables(topk_idx: torch.Tensor, num_experts: int, num_ranks: int):
    """One-chunk RCCL source-side tables (table_b [T, min(R, K)], row_of_lane [T, K], rows per expert
    rank) for the diagnostics in tools/ that drive phase B directly."""
    T, K = topk_idx.shape
    R = num_ranks
    dev = topk_idx.device
    rank_of = _rank_of(topk_idx, num_experts, R)
    ranks = torch.arange(R, device=dev)
    hit = rank_of.unsqueeze(-1) == ranks.view(1, 1, R)
    is_to = hit.any(dim=1)
    back_counts = is_to.sum(dim=0)
    pos = torch.cumsum(is_to.to(torch.int64), dim=0) - 1
    offsets = torch.cumsum(back_counts, dim=0) - back_counts
    row = torch.where(is_to, offsets.view(1, R) + pos, torch.full_like(pos, -1))
    lanes = torch.arange(K, device=dev).view(1, K, 1)
    master = torch.where(hit, lanes, torch.full_like(lanes, -1)).amax(dim=1)
    key = torch.where(is_to, master, K + ranks.view(1, R))
    order = torch.argsort(key, dim=1, stable=True)[:, :min(R, K)]
    table_b = row.gather(1, order).to(torch.int32).contiguous()
    row_of_lane = torch.where(rank_of >= 0, row.gather(1, rank_of.clamp(min=0)), torch.full_like(rank_of, -1))
    return table_b, row_of_lane.contiguous(), [int(v) for v in back_counts.tolist()]
