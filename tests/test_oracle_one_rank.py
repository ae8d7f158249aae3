"""CPU: oracle.combine_ep_one (one source rank's combine, threaded -- the full-output check of the
full-size EP = 8 GPU tests) equals oracle.combine_ep (pinned to refs.combine by the golden fixtures)."""
import numpy as np
import pytest

import oracle


@pytest.mark.parametrize('R,K,T,weighted,with_bias,threads', [
    (4, 8, 40, False, True, 3), (8, 8, 33, True, False, 4), (4, 2, 24, False, False, 1), (3, 4, 17, False, True, 8)])
def test_one_rank_equals_all_ranks(R, K, T, weighted, with_bias, threads):
    rng = np.random.default_rng(R * 100 + K * 10 + T)
    E, H = 8 * R, 64
    idx_all = []
    for _ in range(R):
        idx = np.array([rng.permutation(E)[:K] for _ in range(T)], dtype=np.int64)
        idx[rng.random((T, K)) < 0.2] = -1
        idx_all.append(idx)
    w_all = [rng.random((T, K)).astype(np.float32) * (i >= 0) for i in idx_all]
    disp = oracle.simulate_dispatch(idx_all, E, T)
    x_all, we_all = [], []
    for d in disp:
        x_all.append(oracle.f32_to_bf16(rng.standard_normal((d['num_expanded'], H)).astype(np.float32)))
        we = np.zeros((d['num_expanded'],), np.float32)
        for row, (g, k) in enumerate(d['expanded_src']):
            s, t = divmod(int(g), T)
            we[row] = w_all[s][t, k]
        we_all.append(we)
    bias = [(oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)) if with_bias else None, None)
            for _ in range(R)]
    metas = [d['src_metadata'] for d in disp]
    full = oracle.combine_ep(x_all, metas, idx_all, E, T, expanded=True, topk_weights_per_rank=we_all,
                             bias_per_rank=bias, weighted=weighted)
    for r in range(R):
        out, out_w = oracle.combine_ep_one(r, x_all, metas, idx_all[r], E, T, expanded=True,
                                           topk_weights_per_rank=we_all, bias=bias[r], weighted=weighted,
                                           threads=threads)
        assert np.array_equal(out, full[r][0]) and np.array_equal(out_w, full[r][1]), r


@pytest.mark.parametrize('R,K,T,threads', [(4, 8, 40, 3), (3, 4, 17, 8)])
def test_one_rank_equals_all_ranks_non_expanded(R, K, T, threads):
    """The received-token (non-expanded) layout: one pre-reduced row per received token, all K weights."""
    rng = np.random.default_rng(R * 7 + T)
    E, H = 8 * R, 64
    idx_all = []
    for _ in range(R):
        idx = np.array([rng.permutation(E)[:K] for _ in range(T)], dtype=np.int64)
        idx[rng.random((T, K)) < 0.2] = -1
        idx_all.append(idx)
    disp = oracle.simulate_dispatch(idx_all, E, T)
    metas = [d['src_metadata'].copy() for d in disp]
    for m in metas:
        m[:, 2:] = -1
    x_all = [oracle.f32_to_bf16(rng.standard_normal((m.shape[0], H)).astype(np.float32)) for m in metas]
    w_all = [rng.random((m.shape[0], K)).astype(np.float32) for m in metas]
    bias = [(oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)), None) for _ in range(R)]
    full = oracle.combine_ep(x_all, metas, idx_all, E, T, expanded=False, topk_weights_per_rank=w_all,
                             bias_per_rank=bias)
    for r in range(R):
        out, out_w = oracle.combine_ep_one(r, x_all, metas, idx_all[r], E, T, expanded=False,
                                           topk_weights_per_rank=w_all, bias=bias[r], threads=threads)
        assert np.array_equal(out, full[r][0]) and np.array_equal(out_w, full[r][1]), r
