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
