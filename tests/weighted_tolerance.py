"""calc_diff of the gating-weighted multiple-reduction combine (the N > 1 bench recipe) against the exact
float64 sum, per rank of every golden fixture: the oracle's restatement, which the GPU path equals bit for
bit (tests/test_combine_gpu.py).  The reference's bound is 1e-5 (tests/legacy/test_low_latency.py:178-181)."""
import sys, json
ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import oracle
from tests.helpers import load, ranks_of, weighted_multi_expected, exact_weighted
out = {}
for fx_name in ['f1_ep1_t128_h1024_k2.npz', 'f4_ep4_t96_h256_k2.npz', 'f2_ep8_t64_h256_k8.npz', 'f3_ep8_skew_t128_h64_k8.npz']:
    fx = load(fx_name)
    ranks = ranks_of(fx)
    ds = []
    for r, me in enumerate(ranks):
        got = weighted_multi_expected(fx, r)
        ds.append(oracle.calc_diff(oracle.bf16_to_f32(got), exact_weighted(me)))
    out[fx_name] = [float('%.3g' % d) for d in ds]
print(json.dumps(out))
