"""Shared test helpers: fixture loading and construction of the combine inputs the
reference test builds (tests/elastic/test_ep.py:185-206 in the reference)."""
import os
from typing import Dict, List

import numpy as np

from oracle import bf16_to_f32, f32_to_bf16, simulate_dispatch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
POISON = np.uint16(0x7fc1)       # a NaN: any read of a padding row shows up in the output


def load(name: str) -> Dict[str, np.ndarray]:
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def ranks_of(fx) -> List[Dict[str, np.ndarray]]:
    """Per-rank views of a fixture (single-rank fixtures have un-prefixed keys)."""
    T, H, K, E, R = (int(v) for v in fx['meta'])
    if 'topk_idx' in fx:
        return [dict(topk_idx=fx['topk_idx'], topk_weights=fx['topk_weights'], y=fx['y'],
                     bias0=fx['bias0'], bias1=fx['bias1'],
                     **{k: v for k, v in fx.items() if k.startswith('combined_')})]
    out = []
    for r in range(R):
        p = f'r{r}_'
        out.append({k[len(p):]: v for k, v in fx.items() if k.startswith(p)})
    return out


def ordered_accumulate(rows: np.ndarray) -> np.ndarray:
    """refs.ordered_accumulate (deep_ep/utils/refs.py:156-174): fp32 zeros, += each slot, one rounding."""
    acc = np.zeros(rows.shape[0:1] + rows.shape[2:], dtype=np.float32)
    for k in range(rows.shape[1]):
        acc = acc + bf16_to_f32(rows[:, k])
    return f32_to_bf16(acc)


def build_combine_inputs(fx, expert_alignment: int = 1):
    """For every expert rank: the received-token metadata, the expanded input rows
    (test_ep.py:201-206) and the non-expanded pre-reduced rows (test_ep.py:187-195)."""
    T, H, K, E, R = (int(v) for v in fx['meta'])
    ranks = ranks_of(fx)
    idx = [r['topk_idx'] for r in ranks]
    disp = simulate_dispatch(idx, E, T, expert_alignment)
    epr = E // R
    per_rank = []
    for r, d in enumerate(disp):
        meta = d['src_metadata']
        # expanded rows: y[src_rank][src_tok, k]
        x_exp = np.full((d['num_expanded'], H), POISON, dtype=np.uint16)
        w_exp = np.zeros((d['num_expanded'],), dtype=np.float32)
        for row, (g, k) in enumerate(d['expanded_src']):
            if g < 0:
                continue
            s, t = divmod(int(g), T)
            x_exp[row] = ranks[s]['y'][t, k]
            w_exp[row] = ranks[s]['topk_weights'][t, k]
        # non-expanded: caller pre-reduces the local slots (test_ep.py:191-195)
        n = meta.shape[0]
        local = np.zeros((n, K, H), dtype=np.uint16)
        w2d = np.zeros((n, K), dtype=np.float32)
        for i in range(n):
            s, t = divmod(int(meta[i, 0]), T)
            e = ranks[s]['topk_idx'][t]
            on_r = (e >= r * epr) & (e < (r + 1) * epr)
            local[i][on_r] = ranks[s]['y'][t][on_r]
            w2d[i] = ranks[s]['topk_weights'][t]
        x_red = ordered_accumulate(local) if n else np.zeros((0, H), dtype=np.uint16)
        per_rank.append(dict(meta=meta, x_exp=x_exp, w_exp=w_exp, x_red=x_red, w2d=w2d,
                             num_expanded=d['num_expanded'], src_global_idx=d['src_global_idx']))
    return ranks, per_rank


def weighted_multi_expected(fx, rank: int, bias=(None, None)) -> np.ndarray:
    """Expected bits of this build's gating-weighted combine with multiple reduction
    (`combine(..., apply_topk_weights=True)` on an expanded handle) for rank `rank` of a fixture: the
    oracle's restatement (oracle.combine_ep, weighted) -- on every expert rank an fp32 fma chain over the
    token's local lanes from +0 (internode_ll.cu:704-711), rounded to bf16, then phase B over the
    partials with the bias in front (combine_reduce_epilogue.cuh:62-125).  The reference has no such
    two-level weighted recipe, so its bits are this build's definition; `exact_weighted` pins them to
    the reference's tolerance.  bias: (bias0, bias1) bf16 bit arrays of this rank or None."""
    from oracle import combine_ep
    T, H, K, E, R = (int(v) for v in fx['meta'])
    ranks, per = build_combine_inputs(fx)
    biases = [(None, None)] * R
    biases[rank] = bias
    res = combine_ep([p['x_exp'] for p in per], [p['meta'] for p in per], [r['topk_idx'] for r in ranks], E, T,
                     expanded=True, topk_weights_per_rank=[p['w_exp'] for p in per], bias_per_rank=biases,
                     weighted=True)
    return res[rank][0]


def exact_weighted(me) -> np.ndarray:
    """float64 sum over the valid top-k lanes of weight x expert row, [T, H] -- the reference's weighted
    check compares combined_x with this exact value (tests/legacy/test_low_latency.py:178-181)."""
    y = bf16_to_f32(me['y']).astype(np.float64)
    w = np.where(me['topk_idx'] >= 0, me['topk_weights'], 0).astype(np.float64)
    return (y * w[..., None]).sum(axis=1)


WEIGHTED_TOLERANCE = 1e-5         # calc_diff bound of test_low_latency.py:178-181 (BF16 dispatch)


def dispatch_mode_checks(buf, x, topk_idx, topk_weights, num_experts: int, num_max_tokens: int,
                         expert_alignment: int, do_cpu_sync: bool, do_handle_copy: bool) -> List[str]:
    """The dispatch-mode checks of the reference test (tests/elastic/test_ep.py:143-177, 355-466):
    cached dispatch (handle reuse), cached expanded dispatch with zero padding, handle copy,
    deterministic repeat, the cumulative per-expert counter, per-expert prefix sums, and
    do_cpu_sync=False worst-case shapes.  Works for any kernel provider and device; returns the
    list of failed checks."""
    import torch
    fails = []
    args = dict(topk_idx=topk_idx, topk_weights=topk_weights, num_experts=num_experts,
                num_max_tokens_per_rank=num_max_tokens, expert_alignment=expert_alignment,
                do_handle_copy=do_handle_copy, do_cpu_sync=do_cpu_sync)
    recv_x, recv_idx, recv_w, handle, _ = buf.dispatch(x, **args)
    ex_x, ex_idx, ex_w, ex_handle, _ = buf.dispatch(x, do_expand=True, **args)
    c_x, c_idx, c_w, c_handle, _ = buf.dispatch(x, handle=handle)
    ce_x, _, ce_w, _, _ = buf.dispatch(x, topk_weights=topk_weights, do_expand=True, do_zero_padding=True,
                                       handle=ex_handle)

    def rows(t):
        return t[0] if isinstance(t, tuple) else t

    def same(a, b):
        if isinstance(a, tuple):
            return all(torch.equal(p, q) for p, q in zip(a, b))
        return torch.equal(a.view(torch.uint8) if a.dtype != torch.bool else a,
                           b.view(torch.uint8) if b.dtype != torch.bool else b)

    def head(t, n):
        return tuple(p[:n] for p in t) if isinstance(t, tuple) else t[:n]

    n = int(handle.psum_num_recv_tokens_per_scaleup_rank[-1].item())
    if (topk_idx.data_ptr() != handle.topk_idx.data_ptr()) != do_handle_copy:
        fails.append('handle copy')
    if handle.topk_idx.data_ptr() != c_handle.topk_idx.data_ptr():
        fails.append('cached handle does not share topk_idx')
    if ex_idx is not None:
        fails.append('expanded dispatch returned recv_topk_idx')
    if not do_cpu_sync:
        worst = num_max_tokens * buf.num_ranks
        if rows(recv_x).shape[0] != worst or handle.recv_src_metadata.shape[0] != worst:
            fails.append('do_cpu_sync=False shapes are not worst-case')
    recv_w_full = recv_w
    if not do_cpu_sync:
        # cached calls over a no-CPU-sync handle return the handle's worst-case shapes, and the same bits
        # as its first call (rows past the received ones: zeros / -1, as the first call's)
        if not (same(c_x, recv_x) and torch.equal(c_idx, recv_idx)):
            fails.append('cached dispatch over a no-CPU-sync handle differs from its first call')
        if rows(ce_x).shape[0] != rows(ex_x).shape[0] or ce_w.shape != ex_w.shape:
            fails.append('cached expanded dispatch over a no-CPU-sync handle changed shape')
    recv_x, recv_idx, recv_w = head(recv_x, n), recv_idx[:n], recv_w[:n]
    meta, ex_meta = handle.recv_src_metadata[:n], ex_handle.recv_src_metadata[:n]
    if not (same(head(c_x, n), recv_x) and torch.equal(c_idx[:n], recv_idx) and c_w is None):
        fails.append('cached dispatch differs')
    if not torch.equal(handle.dst_buffer_slot_idx, c_handle.dst_buffer_slot_idx) or \
            handle.num_recv_tokens_per_expert_list != c_handle.num_recv_tokens_per_expert_list:
        fails.append('cached handle differs')
    slots = ex_meta[:, 2:]
    valid = slots[slots >= 0].long()
    def pick(t, idx):
        return tuple(p[idx] for p in t) if isinstance(t, tuple) else t[idx]

    if not (same(pick(ce_x, valid), pick(ex_x, valid)) and torch.equal(ce_w[valid], ex_w[valid])):
        fails.append('cached expanded dispatch differs on valid rows')
    epr = num_experts // buf.num_ranks
    psum = [0] + [int(v) for v in ex_handle.psum_num_recv_tokens_per_expert.tolist()]
    for e in range(epr):
        start = psum[e + 1]
        end = (start + expert_alignment - 1) // expert_alignment * expert_alignment
        if bool((rows(ce_x)[start:end].float() != 0).any()) or bool((ce_w[start:end] != 0).any()):
            fails.append(f'zero padding of expert {e}')
            break
    # deterministic repeat
    r2 = buf.dispatch(x, **args)
    if not (same(head(r2[0], n), recv_x) and torch.equal(r2[1][:n], recv_idx) and
            torch.equal(r2[3].recv_src_metadata[:n], meta)):
        fails.append('dispatch is not deterministic')
    # cumulative per-expert counter and prefix sums (test_ep.py:446-462)
    stats = torch.zeros((epr,), dtype=torch.int32, device=recv_idx.device)
    buf.dispatch(x, cumulative_local_expert_recv_stats=stats, **args)
    npsum = [0] + [int(v) for v in handle.psum_num_recv_tokens_per_expert.tolist()]
    for e in range(epr):
        ref = int((recv_idx == e).sum().item())
        aligned = (ref + expert_alignment - 1) // expert_alignment * expert_alignment
        if do_cpu_sync and (int(stats[e].item()) != ref or handle.num_recv_tokens_per_expert_list[e] != aligned):
            fails.append(f'expert {e} counter')
            break
        al_prev = (psum[e] + expert_alignment - 1) // expert_alignment * expert_alignment
        if npsum[e + 1] - npsum[e] != aligned or psum[e + 1] - al_prev != ref:
            fails.append(f'expert {e} prefix sums')
            break
    if ex_handle.recv_src_metadata.shape[0] != (n if do_cpu_sync else num_max_tokens * buf.num_ranks):
        fails.append('expanded metadata rows')
    if not do_cpu_sync:
        # a handle made without a CPU sync combines exactly like a host-synced one (same slots, same rows)
        s_ex_x, _, s_ex_w, s_handle, _ = buf.dispatch(x, do_expand=True, **dict(args, do_cpu_sync=True))
        if not torch.equal(s_handle.recv_src_metadata, ex_handle.recv_src_metadata[:s_handle.recv_src_metadata.shape[0]]):
            fails.append('no-CPU-sync expanded metadata differs from the synced one')
        g = torch.Generator(device=rows(ex_x).device).manual_seed(3)
        y = torch.randn((ex_handle.num_expanded_tokens, rows(ex_x).shape[1]), generator=g,
                        device=rows(ex_x).device).to(torch.bfloat16)
        n_ex = s_handle.num_expanded_tokens
        out_f, w_f, _ = buf.combine(y, ex_handle, topk_weights=ex_w)
        out_s, w_s, _ = buf.combine(y[:n_ex].contiguous(), s_handle, topk_weights=s_ex_w)
        if not (torch.equal(out_f.view(torch.int16), out_s.view(torch.int16)) and torch.equal(w_f, w_s)):
            fails.append('combine over a no-CPU-sync handle differs')
        # the same for the received-token layout: one row per received token, worst-case padded
        s_x, _, s_w, s_rhandle, _ = buf.dispatch(x, **dict(args, do_cpu_sync=True))
        n_s = s_rhandle.recv_src_metadata.shape[0]
        y_r = torch.randn((handle.recv_src_metadata.shape[0], rows(ex_x).shape[1]), generator=g,
                          device=rows(ex_x).device).to(torch.bfloat16)
        out_f, w_f, _ = buf.combine(y_r, handle, topk_weights=recv_w_full)
        out_s, w_s, _ = buf.combine(y_r[:n_s].contiguous(), s_rhandle, topk_weights=s_w)
        if not (torch.equal(out_f.view(torch.int16), out_s.view(torch.int16)) and torch.equal(w_f, w_s)):
            fails.append('non-expanded combine over a no-CPU-sync handle differs')
    return fails
