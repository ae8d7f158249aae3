"""Pin the CPU oracle against the reference's own pure-torch oracle outputs.

The golden fixtures were produced by deep_ep/utils/refs.py (see
tests/golden/gen_golden.py).  The bar is the reference test's: bitwise equality
of combined_x and of the passed-through top-k weights (tests/elastic/test_ep.py:502-511),
and calc_diff < 1e-5 for the weighted variant (tests/legacy/test_low_latency.py:178-181).
"""
import numpy as np
import pytest

import oracle
from tests.helpers import build_combine_inputs, load, ordered_accumulate, ranks_of

FIXTURES = ['f1_ep1_t128_h1024_k2.npz', 'f2_ep8_t64_h256_k8.npz',
            'f3_ep8_skew_t128_h64_k8.npz', 'f4_ep4_t96_h256_k2.npz']


def _bias(rank, nb):
    if nb == 0:
        return (None, None)
    if nb == 1:
        return (rank['bias0'], None)
    return (rank['bias0'], rank['bias1'])


@pytest.mark.parametrize('name', FIXTURES)
@pytest.mark.parametrize('nb', [0, 1, 2])
def test_expanded_multi_reduction_matches_refs(name, nb):
    fx = load(name)
    T, H, K, E, R = (int(v) for v in fx['meta'])
    ranks, per_rank = build_combine_inputs(fx)
    res = oracle.combine_ep([p['x_exp'] for p in per_rank], [p['meta'] for p in per_rank],
                            [r['topk_idx'] for r in ranks], E, T, expanded=True,
                            allow_multiple_reduction=True,
                            topk_weights_per_rank=[p['w_exp'] for p in per_rank],
                            bias_per_rank=[_bias(r, nb) for r in ranks])
    for r, (out, out_w) in enumerate(res):
        assert np.array_equal(out, ranks[r][f'combined_multi_b{nb}']), f'rank {r}'
        assert np.array_equal(out_w, ranks[r]['topk_weights']), f'rank {r} weights'


@pytest.mark.parametrize('name', FIXTURES)
@pytest.mark.parametrize('nb', [0, 1, 2])
def test_non_expanded_matches_refs(name, nb):
    fx = load(name)
    T, H, K, E, R = (int(v) for v in fx['meta'])
    ranks, per_rank = build_combine_inputs(fx)
    res = oracle.combine_ep([p['x_red'] for p in per_rank], [p['meta'] for p in per_rank],
                            [r['topk_idx'] for r in ranks], E, T, expanded=False,
                            allow_multiple_reduction=True,
                            topk_weights_per_rank=[p['w2d'] for p in per_rank],
                            bias_per_rank=[_bias(r, nb) for r in ranks])
    for r, (out, out_w) in enumerate(res):
        assert np.array_equal(out, ranks[r][f'combined_multi_b{nb}']), f'rank {r}'
        assert np.array_equal(out_w, ranks[r]['topk_weights']), f'rank {r} weights'


@pytest.mark.parametrize('name', FIXTURES)
@pytest.mark.parametrize('nb', [0, 1, 2])
def test_expanded_single_reduction_matches_refs(name, nb):
    """allow_multiple_reduction=False: every top-k row is sent unreduced (kDoExpandedSend)."""
    fx = load(name)
    T, H, K, E, R = (int(v) for v in fx['meta'])
    ranks, per_rank = build_combine_inputs(fx)
    res = oracle.combine_ep([p['x_exp'] for p in per_rank], [p['meta'] for p in per_rank],
                            [r['topk_idx'] for r in ranks], E, T, expanded=True,
                            allow_multiple_reduction=False,
                            bias_per_rank=[_bias(r, nb) for r in ranks])
    for r, (out, _) in enumerate(res):
        assert np.array_equal(out, ranks[r][f'combined_single_b{nb}']), f'rank {r}'


def test_f1_ordered_accumulate_restatement():
    fx = load('f1_ep1_t128_h1024_k2.npz')
    assert np.array_equal(ordered_accumulate(fx['y']), fx['ordered_accumulate'])


def test_weighted_ll_within_reference_tolerance():
    fx = load('f1_ep1_t128_h1024_k2.npz')
    out = oracle.weighted_ll(fx['y'], fx['topk_idx'], fx['topk_weights'])
    diff = oracle.calc_diff(oracle.bf16_to_f32(out), fx['weighted_f64'])
    assert diff < 1e-5, diff
    # and it is the correctly rounded value of the fp32 fma chain: never more than 1 bf16 ulp
    ref = oracle.f32_to_bf16(fx['weighted_f64'].astype(np.float32))
    ulp = np.abs(out.astype(np.int32) - ref.astype(np.int32))
    assert ulp.max() <= 1


@pytest.mark.parametrize('name', ['f2_ep8_t64_h256_k8.npz', 'f4_ep4_t96_h256_k2.npz'])
def test_dispatch_order_matches_refs_dispatch(name):
    """The receive order the oracle (and the product's dispatch) assumes is refs.dispatch's."""
    fx = load(name)
    T, H, K, E, R = (int(v) for v in fx['meta'])
    ranks = ranks_of(fx)
    disp = oracle.simulate_dispatch([r['topk_idx'] for r in ranks], E, T)
    epr = E // R
    for r in range(R):
        assert np.array_equal(disp[r]['src_global_idx'], ranks[r]['dispatch_recv_src_token_idx'])
        # recv_topk_idx: local expert index or -1 (refs.py:113-118)
        ref_idx = ranks[r]['dispatch_recv_topk_idx']
        for i, g in enumerate(disp[r]['src_global_idx']):
            s, t = divmod(int(g), T)
            e = ranks[s]['topk_idx'][t]
            local = np.where((e >= r * epr) & (e < (r + 1) * epr), e - r * epr, -1)
            assert np.array_equal(local, ref_idx[i])
