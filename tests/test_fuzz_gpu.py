"""Randomised EP = 1 parity sweep on the GPU: ElasticBuffer dispatch + combine over seeded random
shapes (ragged hidden sizes, top-k 1..16, expert counts, masked slots, empty batches), every
combine flavour (expanded / non-expanded, multiple / single reduction, plain / gating-weighted,
bias 0/1/2) against the oracle, bitwise.  Mirrors the reference's mode matrix
(tests/elastic/test_ep.py:22-31) on shapes its fixed configs do not reach."""
import os

import numpy as np
import pytest
import torch

import oracle
from tests.test_buffer_cpu import _weighted_single

pytestmark = pytest.mark.gpu

HIDDENS = [8, 64, 520, 1024, 2056, 4104, 7168]
TOPKS = [1, 2, 3, 4, 6, 8, 12, 16, 24, 32]          # 32: the reference maximum


def _u16(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _bf16(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16).cuda()


def _case(seed: int):
    rng = np.random.default_rng(seed)
    T = int(rng.choice([0, 1, 7, 64, 129, 300]))
    H = int(rng.choice(HIDDENS))
    K = int(rng.choice(TOPKS))
    E = int(K * rng.integers(1, 9))
    masked = float(rng.choice([0.0, 0.1, 0.4]))
    return rng, T, H, K, E, masked


@pytest.fixture(params=[(0, 0), (1, 8), (2, 2)], ids=['auto', 'vpt1_rows8', 'vpt2_rows2'])
def launch_shape(request):
    """The automatic launch shape and two forced ones (deepep_set_launch_config: vectors per lane, rows in
    flight): every shape gives the same bits."""
    from deepep_amd import _lib
    lib = _lib.load()
    assert lib.deepep_set_launch_config(*request.param) == 0
    yield request.param
    lib.deepep_set_launch_config(0, 0)


@pytest.fixture(scope='module')
def group():
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29547')
        dist.init_process_group('gloo', rank=0, world_size=1)
    return dist.group.WORLD


@pytest.mark.parametrize('seed', range(32))
def test_random_shapes_ep1(group, seed, launch_shape):
    from deepep_amd import ElasticBuffer
    rng, T, H, K, E, masked = _case(seed)
    idx = np.array([rng.permutation(E)[:K] for _ in range(T)], dtype=np.int64).reshape(T, K)
    idx[rng.random((T, K)) < masked] = -1
    w = (rng.random((T, K)).astype(np.float32) * (idx >= 0)).astype(np.float32)
    biases = [oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)) for _ in range(2)]
    T_max = max(T, 1)
    x = torch.zeros((T, H), dtype=torch.bfloat16, device='cuda')
    g_idx, g_w = torch.from_numpy(idx).cuda(), torch.from_numpy(w).cuda()
    failures = []
    for amr in (True, False):
        buf = ElasticBuffer(group, num_max_tokens_per_rank=T_max, hidden=H, num_topk=K, allow_multiple_reduction=amr)
        _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=g_idx, topk_weights=g_w, num_experts=E,
                                             num_max_tokens_per_rank=T_max, do_expand=True)
        meta = handle.recv_src_metadata.cpu().numpy()
        n_exp = handle.num_expanded_tokens
        y = oracle.f32_to_bf16((rng.standard_normal((n_exp, H)) * rng.choice([1e-2, 1.0, 50.0])).astype(np.float32))
        # the token-major view of the same rows: y3[t, k] = y[slot of (t, k)]
        y3 = np.zeros((T, K, H), np.uint16)
        for i in range(meta.shape[0]):
            for k in range(K):
                if meta[i, 2 + k] >= 0:
                    y3[meta[i, 0] % T_max, k] = y[meta[i, 2 + k]]
        for nb in (0, 1, 2):
            b = [biases[0] if nb >= 1 else None, biases[1] if nb >= 2 else None]
            g_bias = None if nb == 0 else (_bf16(b[0]) if nb == 1 else (_bf16(b[0]), _bf16(b[1])))
            for weighted in (False, True):
                out, out_w, _ = buf.combine(_bf16(y), handle, topk_weights=ex_w if (weighted or amr) else None,
                                            bias=g_bias, apply_topk_weights=weighted)
                torch.cuda.synchronize()
                if amr:
                    part, _ = oracle.phase_a(y, meta, K, True, ex_w.cpu().numpy(), weighted=weighted)
                    recv = np.zeros((1, T_max, H), np.uint16)
                    recv[0, meta[:, 0] % T_max] = part
                    exp, _ = oracle.phase_b(recv, None, idx, E, 1, True, True, b[0], b[1])
                elif weighted:
                    cb = None if nb == 0 else (torch.from_numpy(b[0].view(np.int16)).view(torch.bfloat16) if nb == 1
                                               else tuple(torch.from_numpy(v.view(np.int16)).view(torch.bfloat16)
                                                          for v in b))
                    exp = _u16(_weighted_single(y3, torch.from_numpy(idx), torch.from_numpy(w), cb))
                else:
                    exp = oracle.combine_ep([y], [meta], [idx], E, T_max, expanded=True,
                                            allow_multiple_reduction=False, bias_per_rank=[tuple(b)])[0][0][:T]
                if not np.array_equal(_u16(out), exp):
                    failures.append(f'amr={amr} nb={nb} weighted={weighted}')
                if out_w is not None and not np.array_equal(out_w.cpu().numpy(), w):
                    failures.append(f'weights amr={amr} nb={nb} weighted={weighted}')
        if amr:
            # non-expanded: the caller pre-reduced its local experts; the combine copies/epilogues
            _, _, recv_w, nh, _ = buf.dispatch(x, topk_idx=g_idx, topk_weights=g_w, num_experts=E,
                                               num_max_tokens_per_rank=T_max)
            n = nh.num_recv_tokens
            x_red = oracle.f32_to_bf16(rng.standard_normal((n, H)).astype(np.float32))
            out, out_w, _ = buf.combine(_bf16(x_red), nh, topk_weights=recv_w, bias=_bf16(biases[0]) if T else None)
            torch.cuda.synchronize()
            recv = np.zeros((1, T_max, H), np.uint16)
            recv[0, nh.recv_src_metadata.cpu().numpy()[:n, 0] % T_max] = x_red
            exp, _ = oracle.phase_b(recv, None, idx, E, 1, True, True, biases[0] if T else None)
            if not np.array_equal(_u16(out), exp):
                failures.append('non-expanded')
            if not np.array_equal(out_w.cpu().numpy(), w):
                failures.append('non-expanded weights')
    assert not failures, (seed, T, H, K, E, masked, failures)


def _ep_thread(rank, world, seed, comm, results):
    """One simulated rank of a random EP = `world` case (threads on the one GPU, all-to-all by copies)."""
    try:
        from deepep_amd import ElasticBuffer
        from tests.sim import FakeGroup as _FakeGroup
        torch.cuda.set_device(0)
        rng = np.random.default_rng(seed)            # same stream in every thread: same global case
        K = int(rng.choice([1, 2, 4, 6, 8]))
        E = int(world * rng.integers(max(1, (K + world - 1) // world), 5))
        H = int(rng.choice([64, 520, 2056]))
        T = int(rng.choice([33, 96]))
        Ts = [int(rng.integers(0, T + 1)) for _ in range(world)]
        idx_all, w_all, y_all, b_all = [], [], [], []
        for r in range(world):
            idx = np.array([rng.permutation(E)[:K] for _ in range(Ts[r])], dtype=np.int64).reshape(Ts[r], K)
            idx[rng.random((Ts[r], K)) < 0.15] = -1
            idx_all.append(idx)
            w_all.append((rng.random((Ts[r], K)).astype(np.float32) * (idx >= 0)).astype(np.float32))
            y = oracle.f32_to_bf16(rng.standard_normal((Ts[r], K, H)).astype(np.float32))
            y[idx < 0] = 0
            y_all.append(y)
            b_all.append(oracle.f32_to_bf16(rng.standard_normal((Ts[r], H)).astype(np.float32)))
        disp = oracle.simulate_dispatch(idx_all, E, T)
        x_exp_all, w_exp_all = [], []
        for d in disp:
            xe = np.zeros((d['num_expanded'], H), np.uint16)
            we = np.zeros((d['num_expanded'],), np.float32)
            for row, (g, k) in enumerate(d['expanded_src']):
                s, t = divmod(int(g), T)
                xe[row], we[row] = y_all[s][t, k], w_all[s][t, k]
            x_exp_all.append(xe), w_exp_all.append(we)
        metas = [d['src_metadata'] for d in disp]
        grp = _FakeGroup(rank, world, comm)
        failures = []
        bias = _bf16(b_all[rank])
        x = torch.zeros((Ts[rank], H), dtype=torch.bfloat16, device='cuda')
        g_idx, g_w = torch.from_numpy(idx_all[rank]).cuda(), torch.from_numpy(w_all[rank]).cuda()
        for amr in (True, False):
            buf = ElasticBuffer(grp, num_max_tokens_per_rank=T, hidden=H, num_topk=K, allow_multiple_reduction=amr)
            comm.install(buf, rank)
            _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=g_idx, topk_weights=g_w, num_experts=E, do_expand=True)
            if not np.array_equal(handle.recv_src_metadata.cpu().numpy(), metas[rank]):
                failures.append(f'amr={amr}: recv_src_metadata')
                continue
            xin = _bf16(x_exp_all[rank])
            for weighted in (False, True):
                if amr:
                    exp = oracle.combine_ep(x_exp_all, metas, idx_all, E, T, expanded=True,
                                            topk_weights_per_rank=w_exp_all,
                                            bias_per_rank=[(b, None) for b in b_all], weighted=weighted)[rank]
                    out, out_w, _ = buf.combine(xin, handle, topk_weights=ex_w, bias=bias, apply_topk_weights=weighted)
                    ok_w = np.array_equal(out_w.cpu().numpy(), exp[1])
                    exp = exp[0]
                elif weighted:
                    cb = torch.from_numpy(b_all[rank].view(np.int16)).view(torch.bfloat16)
                    exp = _u16(_weighted_single(y_all[rank], torch.from_numpy(idx_all[rank]),
                                                torch.from_numpy(w_all[rank]), cb))
                    out, out_w, _ = buf.combine(xin, handle, topk_weights=ex_w, bias=bias, apply_topk_weights=True)
                    ok_w = np.array_equal(out_w.cpu().numpy(), w_all[rank])
                else:
                    exp = oracle.combine_ep(x_exp_all, metas, idx_all, E, T, expanded=True,
                                            allow_multiple_reduction=False,
                                            bias_per_rank=[(b, None) for b in b_all])[rank][0]
                    out, out_w, _ = buf.combine(xin, handle, bias=bias)
                    ok_w = out_w is None
                torch.cuda.synchronize()
                if not np.array_equal(_u16(out), exp):
                    failures.append(f'amr={amr} weighted={weighted}: combined_x')
                if not ok_w:
                    failures.append(f'amr={amr} weighted={weighted}: weights')
        results[rank] = failures
    except Exception:
        import traceback
        results[rank] = [traceback.format_exc()]
        comm.bar.abort()


@pytest.mark.parametrize('case', range(16))
def test_random_shapes_ep_sim(case, monkeypatch, launch_shape):
    """Random EP = 2..8 cases (ragged per-rank batches incl. empty ranks, top-k 1..8, R > K and
    R <= K layouts, chunked and one-shot exchange), all ranks simulated by threads on the GPU."""
    import threading
    from tests.sim import ThreadComm as _ThreadComm
    rng = np.random.default_rng(1000 + case)
    world = int(rng.choice([2, 3, 4, 5, 8]))
    if rng.random() < 0.5:
        monkeypatch.setenv('DEEPEP_COMBINE_CHUNKS', str(int(rng.choice([2, 3]))))
    comm = _ThreadComm(world)
    results = {}
    threads = [threading.Thread(target=_ep_thread, args=(r, world, 2000 + case, comm, results)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=150)
    assert len(results) == world, results
    bad = {r: f for r, f in results.items() if f}
    assert not bad, (case, world, bad)
