"""BASELINE configs 3, 4 and 5 at full size: 8 EP ranks, each simulated by a thread on the one GPU
(exchange with ProcessGroupNCCL's stream semantics, tests/sim.py), through ElasticBuffer's HIP
dispatch and the pipelined (4-chunk) combine.

  C3  8 x 8192 tokens, hidden 7168, top-8, 256 experts, uniform routing: plain + bias, and the
      gating-weighted combine (apply_topk_weights: bitwise vs the oracle AND calc_diff < 1e-5 against the
      exact float64 sum on every rank, the reference's weighted tolerance); and both again with 10 %
      masked top-k slots and ragged batches (8192 - rank tokens)
  C4  the same with the FP8 dispatch (per-128 e4m3 + fp32 scales) chained into the BF16 combine:
      every expanded FP8 row is checked against its source token, the dequantised rows are the
      expert outputs the combine reduces
  C5  8 x 16384 tokens, skewed routing (get_unbalanced_scores, rank 0's experts ~4x the tokens)
  the reference test's default: 8 x 4096 ragged tokens, top-6 (fewer top-k lanes than ranks: the top-k
      receive layout), 0 or 2 biases, both layouts

The reference's own test checks every rank's whole output bitwise at 4096 tokens x 7168 x top-6
across 8 ranks (tests/elastic/test_ep.py:502-511, 577-580).  Here too: EVERY rank's whole combined_x
(all its tokens, with every expert rank's rows of them) is checked bitwise against the oracle
(oracle.combine_ep_one: the arithmetic of oracle.combine_ep, pinned to refs.combine, restricted to one
source rank; the 8 ranks' checks run concurrently, 2 host threads each), and the top-k weight
pass-through for every token of every rank.
"""
import numpy as np
import pytest
import torch

import oracle
from tests.sim import FakeGroup, ThreadComm, run_threads

pytestmark = pytest.mark.gpu



def _u16(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _calc_diff(a: torch.Tensor, b: torch.Tensor) -> float:
    """deep_ep/utils/math.py:5-9, in float64 on the GPU."""
    a, b = a.double() + 1, b.double() + 1
    return float(1 - 2 * (a * b).sum() / (a * a + b * b).sum())


def _rank(rank, world, T_max, H, K, E, skew, fp8, weighted, masked, ragged, expanded, num_bias, comm, shared, results):
    try:
        torch.cuda.set_device(0)
        from deepep_amd import ElasticBuffer
        from workloads import get_unbalanced_scores, per_token_cast_back, per_token_cast_to_fp8
        g = torch.Generator(device='cuda').manual_seed(4242 + rank)
        # ragged: rank r holds T_max - r tokens (the reference's test, tests/elastic/test_ep.py:62)
        T = T_max - rank if ragged else T_max
        if skew != 1.0:
            with comm.lock:                                   # the bisection uses torch's global generator
                torch.manual_seed(4242 + rank)
                scores = get_unbalanced_scores(T, E, world, K, skew, device='cuda')
        else:
            scores = torch.rand((T, E), device='cuda', generator=g)
        w, idx = torch.topk(scores, K, dim=-1, sorted=False)
        idx = idx.to(torch.int64).contiguous()
        if masked:
            # --masked-ratio (tests/elastic/test_ep.py:78-81): a share of the top-k slots -1, their weights 0
            idx.masked_fill_(torch.rand(idx.shape, device='cuda', generator=g) < masked, -1)
            w = w.masked_fill(idx < 0, 0)
        w = w.contiguous()
        x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
        biases = [torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16) for _ in range(num_bias)]
        buf = ElasticBuffer(FakeGroup(rank, world, comm), num_max_tokens_per_rank=T_max, hidden=H, num_topk=K)
        comm.install(buf, rank)
        failures = []
        if fp8:
            xq = per_token_cast_to_fp8(x)
            shared[('xq', rank)] = xq
            (ex_q, ex_sf), _, ex_w, handle, _ = buf.dispatch(xq, topk_idx=idx, topk_weights=w, num_experts=E,
                                                             do_expand=True)
            comm.bar.wait()
            # every expanded FP8 row (and its scales) is its source token's, bit for bit
            q_all = torch.cat([shared[('xq', s)][0].view(torch.uint8) for s in range(world)])
            sf_all = torch.cat([shared[('xq', s)][1] for s in range(world)])
            meta = handle.recv_src_metadata
            src = meta[:, 0].long()
            for k in range(K):
                rows = meta[:, 2 + k]
                ok = rows >= 0
                if not torch.equal(ex_q.view(torch.uint8)[rows[ok].long()], q_all[src[ok]]) or \
                        not torch.equal(ex_sf[rows[ok].long()], sf_all[src[ok]]):
                    failures.append(f'fp8 dispatch rows of lane {k}')
            y = per_token_cast_back(ex_q, ex_sf)                  # the expert outputs
        elif expanded:
            _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
            y = torch.randn((handle.num_expanded_tokens, H), device='cuda', generator=g).to(torch.bfloat16)
        else:
            # the received-token layout: one row per received token, which the caller has pre-reduced over its
            # local lanes (test_ep.py:187-195), and its K weights
            _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E)
            y = torch.randn((handle.num_recv_tokens, H), device='cuda', generator=g).to(torch.bfloat16)
        b = None if weighted or fp8 or not biases else (biases[0] if len(biases) == 1 else tuple(biases))
        out, out_w, _ = buf.combine(y, handle, topk_weights=ex_w, bias=b, apply_topk_weights=weighted)
        torch.cuda.synchronize()
        if getattr(buf, '_stream_b', None) is None:          # made by the pipelined schedule only
            failures.append('the combine did not take the pipelined schedule')
        if not torch.equal(out_w, w):
            failures.append('combined_topk_weights (all tokens)')
        shared[rank] = dict(meta=handle.recv_src_metadata.cpu().numpy(), y=y, ex_w=ex_w, idx=idx.cpu().numpy(),
                            out=out, bias=b)
        comm.bar.wait()
        # ---- the oracle on ALL of this rank's tokens, with every expert rank's rows of them
        n_s = T
        S = np.arange(T)
        pos = np.arange(T, dtype=np.int64)
        x_sub, m_sub, w_sub = [], [], []
        exact = torch.zeros((T, H), dtype=torch.float64, device='cuda') if weighted else None
        for r in range(world):
            m = shared[r]['meta']
            sel = m[:, 0] // T_max == rank
            mr = m[sel].copy()
            slots = mr[:, 2:]
            valid = slots >= 0
            if expanded:
                src_rows = torch.from_numpy(slots[valid].astype(np.int64)).cuda()
                new = np.full(slots.shape, -1, np.int32)
                new[valid] = np.arange(int(valid.sum()), dtype=np.int32)
                mr[:, 2:] = new
            else:                                             # row i of the received tokens is x row i
                src_rows = torch.from_numpy(np.nonzero(sel)[0].astype(np.int64)).cuda()
            x_sub.append(_u16(shared[r]['y'][src_rows]) if src_rows.numel() else np.zeros((0, H), np.uint16))
            w_sub.append(shared[r]['ex_w'][src_rows].cpu().numpy())
            mr[:, 0] = rank * n_s + pos[mr[:, 0] % T_max]
            m_sub.append(mr)
            if weighted:
                # the exact float64 gating-weighted sum of every token over all its expert ranks' rows
                tok = np.broadcast_to((m[sel, 0] % T_max)[:, None], slots.shape)[valid]
                if src_rows.numel():
                    exact.index_add_(0, torch.from_numpy(tok.astype(np.int64)).cuda(),
                                     shared[r]['y'][src_rows].double() * shared[r]['ex_w'][src_rows].double()[:, None])
        bl = [] if b is None else ([b] if isinstance(b, torch.Tensor) else list(b))
        bias_sub = tuple(_u16(t[torch.from_numpy(S).cuda()]) for t in bl) + (None,) * (2 - len(bl))
        exp, exp_w = oracle.combine_ep_one(rank, x_sub, m_sub, shared[rank]['idx'][S], E, n_s, expanded=expanded,
                                           topk_weights_per_rank=w_sub, bias=bias_sub, weighted=weighted,
                                           threads=2)
        got = _u16(out[torch.from_numpy(S).cuda()])
        if not np.array_equal(got, exp):
            bad = np.argwhere(got != exp)
            failures.append(f'combined_x differs on {len(bad)} elements of {n_s} tokens, first {bad[:3].tolist()}')
        shared[('full_checked', rank)] = got.shape[0]
        if not np.array_equal(exp_w, w.cpu().numpy()[S]):
            failures.append('oracle weights of the sample')
        if weighted:
            # the reference's weighted tolerance (tests/legacy/test_low_latency.py:178-181): calc_diff < 1e-5
            # against the exact sum, on every rank's whole output
            d = _calc_diff(out.double(), exact)
            shared[('calc_diff', rank)] = d
            if not d < 1e-5:
                failures.append(f'calc_diff {d:.3g} >= 1e-5 vs the exact float64 weighted sum')
            del exact
            if bool(torch.isnan(out.float()).any()):
                failures.append('NaN in combined_x')
        comm.bar.wait()
        results[rank] = failures
    except Exception:
        import traceback
        results[rank] = [traceback.format_exc()]
        comm.bar.abort()


def _run(T, skew=1.0, fp8=False, weighted=False, masked=0.0, ragged=False, expanded=True, K=8, num_bias=1):
    import threading
    world, H, E = 8, 7168, 256
    torch.cuda.init()                                   # not lazily from 8 threads at once
    torch.cuda.get_device_properties(0)
    comm = ThreadComm(world)
    comm.lock = threading.Lock()
    shared = {}
    results = run_threads(world, _rank, (world, T, H, K, E, skew, fp8, weighted, masked, ragged, expanded, num_bias,
                                         comm, shared), timeout=600)
    full = [shared.get(('full_checked', r)) for r in range(world)]
    diffs = [shared.get(('calc_diff', r)) for r in range(world)]
    del shared
    torch.cuda.empty_cache()
    assert len(results) == world, results
    bad = {r: f for r, f in results.items() if f}
    assert not bad, bad
    want = [T - r if ragged else T for r in range(world)]
    assert full == want, f'tokens checked per rank {full}, expected {want}'
    if weighted:
        assert all(d is not None and d < 1e-5 for d in diffs), diffs
        print(f'calc_diff per rank vs the exact weighted sum: {["%.2e" % d for d in diffs]}')


@pytest.mark.parametrize('weighted', [False, True], ids=['plain_bias', 'gating_weighted'])
def test_config3_ep8_8192_tokens(weighted):
    _run(8192, weighted=weighted)


@pytest.mark.parametrize('weighted', [False, True], ids=['plain_bias', 'gating_weighted'])
def test_config3_ep8_masked_ragged(weighted):
    """Config 3 with 10 % of the top-k slots masked (-1, weight 0; the reference's --masked-ratio) and
    ragged batches (rank r holds 8192 - r tokens of T_max = 8192, the reference's num_tokens)."""
    _run(8192, weighted=weighted, masked=0.1, ragged=True)


def test_config3_ep8_received_token_layout():
    """Config 3 in the received-token (non-expanded) layout with bias: one pre-reduced row per received token
    and its K weights (the reference's combine of a `do_expand=False` handle, test_ep.py:187-217)."""
    _run(8192, expanded=False)


@pytest.mark.parametrize('expanded,num_bias', [(True, 0), (True, 2), (False, 2)],
                         ids=['expanded_no_bias', 'expanded_two_biases', 'received_token_two_biases'])
def test_reference_default_ep8_4096_top6(expanded, num_bias):
    """The reference's own test at its default size (tests/elastic/test_ep.py:577-580: 4096 tokens x 7168 x
    top-6 over 256 experts, 8 ranks, rank r holding max(1, 4096 - r) tokens, :62) with 0 or 2 biases (:96-98):
    top-6 < 8 ranks, so the receive slots are per top-k lane (use_rank_layout false, combine_utils.cuh:8-18)
    -- the top-k layout at full size."""
    _run(4096, ragged=True, expanded=expanded, K=6, num_bias=num_bias)


def test_config4_ep8_fp8_dispatch_bf16_combine():
    _run(8192, fp8=True)


@pytest.mark.parametrize('weighted', [False, True], ids=['plain_bias', 'gating_weighted'])
def test_config5_ep8_16384_tokens_skewed(weighted):
    _run(16384, skew=4.0, weighted=weighted)
