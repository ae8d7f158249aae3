"""The reference's weighted-combine test (tests/legacy/test_low_latency.py) replayed through this build's
ElasticBuffer at that test's default size: 8 ranks (threads on the one GPU, tests/sim.py), 128 tokens per
rank x hidden 7168, top-8 over 288 experts (36 per rank), |randn| gating weights, 10 random top-k
positions masked to -1 (:70-77).

  dispatch   the expanded rows each rank receives are the inputs of its tokens: for the structured input
             (:60-61; every element of rank r's rows is r - 128 except the last 128 columns, which hold
             the source token index) every received row is constant over its first hidden - 128 columns,
             equal to its source rank - 128, and its last 128 columns equal its source token (:129-144);
             every local expert receives exactly the (token, lane) pairs of all ranks that route to it
             (:118-124)
  combine    the experts are the identity (the dispatched rows, dequantised after an FP8 dispatch, :108),
             so the gating-weighted combine must return x * sum of the token's unmasked weights:
             calc_diff < 1e-5 with a BF16 dispatch, < 9e-4 with an FP8 one, and no NaN (:178-181)

Both the structured input and the 0.1 x randn one (:68) run, with both dispatch dtypes.
"""
import numpy as np
import pytest
import torch

from tests.sim import FakeGroup, ThreadComm, run_threads

pytestmark = pytest.mark.gpu

WORLD, T, H, K, E = 8, 128, 7168, 8, 288
RANK_OFFSET = 128


def _calc_diff(a: torch.Tensor, b: torch.Tensor) -> float:
    """deep_ep/utils/math.py:5-9, in float64."""
    a, b = a.double() + 1, b.double() + 1
    return float(1 - 2 * (a * b).sum() / (a * a + b * b).sum())


def _rank(rank, fp8, structured, comm, shared, results):
    try:
        torch.cuda.set_device(0)
        from deepep_amd import ElasticBuffer
        from workloads import per_token_cast_back, per_token_cast_to_fp8
        g = torch.Generator(device='cuda').manual_seed(77 + rank)
        rng = np.random.default_rng(1000 + rank)
        if structured:
            x = torch.full((T, H), float(rank - RANK_OFFSET), dtype=torch.bfloat16, device='cuda')
            x[:, -128:] = torch.arange(T, device='cuda').to(torch.bfloat16).view(-1, 1)
        else:
            x = (torch.randn((T, H), device='cuda', generator=g) * 0.1).to(torch.bfloat16)
        scores = torch.randn((T, E), device='cuda', generator=g).abs() + 1
        idx = torch.topk(scores, K, dim=-1, largest=True, sorted=True)[1].to(torch.int64)
        w = torch.randn((T, K), device='cuda', generator=g).abs()
        for _ in range(10):
            idx[int(rng.integers(0, T)), int(rng.integers(0, K))] = -1
        shared[('idx', rank)] = idx
        buf = ElasticBuffer(FakeGroup(rank, WORLD, comm), num_max_tokens_per_rank=T, hidden=H, num_topk=K)
        comm.install(buf, rank)
        failures = []
        inp = per_token_cast_to_fp8(x) if fp8 else x
        recv, _, ex_w, handle, _ = buf.dispatch(inp, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
        torch.cuda.synchronize()
        comm.bar.wait()
        # ---- dispatch: expert counts of all ranks' routing, and (structured) the content of every row
        epr = E // WORLD
        all_idx = torch.stack([shared[('idx', s)] for s in range(WORLD)])
        want = [(all_idx == rank * epr + i).sum().item() for i in range(epr)]
        psum = handle.psum_num_recv_tokens_per_expert.tolist()
        got = [psum[0]] + [psum[i] - psum[i - 1] for i in range(1, epr)]
        if got != want:
            failures.append(f'received (token, lane) pairs per local expert {got} != {want}')
        y = per_token_cast_back(*recv) if fp8 else recv              # the identity experts' outputs
        if structured:
            meta = handle.recv_src_metadata
            n_recv = sum(handle._recv_counts)
            src = meta[:n_recv, 0].long()
            for k in range(K):
                rows = meta[:n_recv, 2 + k].long()
                ok = rows >= 0
                r = y[rows[ok]].float()
                s = src[ok]
                body = r[:, :-128]
                if not torch.equal(body.amin(dim=-1), body.amax(dim=-1)) or \
                        not torch.equal(body[:, 0], (s // T - RANK_OFFSET).float()):
                    failures.append(f'lane {k}: a received row is not its source rank - {RANK_OFFSET}')
                if not torch.equal(r[:, -128:], (s % T).float().view(-1, 1).expand(-1, 128)):
                    failures.append(f'lane {k}: a received row does not carry its source token index')
        # ---- combine: identity experts, gating-weighted -> x * sum of the unmasked weights
        out, out_w, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
        torch.cuda.synchronize()
        expected = x.double() * w.masked_fill(idx < 0, 0).double().sum(dim=1, keepdim=True)
        d = _calc_diff(out, expected)
        bound = 9e-4 if fp8 else 1e-5
        if not d < bound:
            failures.append(f'calc_diff {d:.3g} >= {bound}')
        if bool(torch.isnan(out.float()).any()):
            failures.append('NaN in combined_x')
        if not torch.equal(out_w, w.masked_fill(idx < 0, 0)):
            failures.append('combined_topk_weights')
        shared[('diff', rank)] = d
        comm.bar.wait()
        results[rank] = failures
    except Exception:
        import traceback
        results[rank] = [traceback.format_exc()]
        comm.bar.abort()


@pytest.mark.parametrize('structured', [True, False], ids=['structured_x', 'randn_x'])
@pytest.mark.parametrize('fp8', [False, True], ids=['bf16_dispatch', 'fp8_dispatch'])
def test_reference_low_latency_weighted_combine(fp8, structured):
    torch.cuda.init()
    torch.cuda.get_device_properties(0)
    comm = ThreadComm(WORLD)
    shared = {}
    results = run_threads(WORLD, _rank, (fp8, structured, comm, shared), timeout=300)
    assert len(results) == WORLD, results
    bad = {r: f for r, f in results.items() if f}
    assert not bad, bad
    print(f'calc_diff per rank: {["%.2e" % shared[("diff", r)] for r in range(WORLD)]}')
