"""The ElasticBuffer host orchestration on CPU, across 1, 2, 4 and 8 gloo ranks.

Dispatch (handle producer), combine planning, the all-to-all exchange and the
stream-free bookkeeping run exactly as on the GPU; the row kernels are the
oracle's (tests/oracle_kernels.py, injected).  Expected outputs are the reference
oracle's golden fixtures (bitwise), mirroring tests/elastic/test_ep.py:185-231 and
:502-511 in the reference: combine of the caller-pre-reduced non-expanded input,
"reduced" (expanded) combine, bias 0/1/2, weight pass-through, and the
allow_multiple_reduction=False variant.
"""
import os
import socket
import traceback

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import (WEIGHTED_TOLERANCE, exact_weighted, load, ordered_accumulate, ranks_of,
                           weighted_multi_expected)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _u16_to_bf16(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16)


def _bf16_to_u16(t: torch.Tensor) -> np.ndarray:
    return t.contiguous().view(torch.int16).numpy().view(np.uint16)


def _weighted_single(y_u16: np.ndarray, idx: torch.Tensor, w: torch.Tensor, bias) -> torch.Tensor:
    """Expected single-reduction weighted combine of one source rank: acc = 0 + bias0 + bias1, then
    the legacy low-latency fma chain over the valid top-k rows (oracle_combine_rows, mode 1 weighted)."""
    from tests.oracle_kernels import OracleKernels
    T, K, H = y_u16.shape
    if T == 0:
        return torch.empty((0, H), dtype=torch.bfloat16)
    src = _u16_to_bf16(y_u16.reshape(T * K, H))
    table = torch.where(idx >= 0, torch.arange(T * K).view(T, K), torch.full((T, K), -1)).to(torch.int32)
    b0, b1 = (None, None) if bias is None else ((bias, None) if isinstance(bias, torch.Tensor) else bias)
    out = torch.empty((T, H), dtype=torch.bfloat16)
    OracleKernels().combine_reduce(1, src, out, T, table=table, row_weights=w.reshape(-1).contiguous(),
                                   bias0=b0, bias1=b1)
    return out


def _worker(rank, world, port, fixture, queue, env=None):
    import sys
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        os.environ.update(env or {})
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from deepep_amd import ElasticBuffer
        import oracle
        from tests.oracle_kernels import OracleKernels
        fx = load(fixture)
        T, H, K, E, R = (int(v) for v in fx['meta'])
        assert R == world
        ranks = ranks_of(fx)
        me = ranks[rank]
        topk_idx = torch.from_numpy(me['topk_idx'].copy())
        topk_w = torch.from_numpy(me['topk_weights'].copy())
        x = (_u16_to_bf16(me['x']) if 'x' in me else
             torch.randn((T, H), generator=torch.Generator().manual_seed(rank)).to(torch.bfloat16))
        biases = [_u16_to_bf16(me['bias0']), _u16_to_bf16(me['bias1'])]
        failures = []

        def y_of(g: int) -> np.ndarray:
            s, t = divmod(int(g), T)
            return ranks[s]['y'][t]

        for amr in (True, False):
            buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                                allow_multiple_reduction=amr, explicitly_destroy=True)
            buf._kernels = OracleKernels()
            # ---- non-expanded dispatch + combine (test_ep.py:143-149, 185-217)
            recv_x, recv_idx, recv_w, handle, _ = buf.dispatch(x, topk_idx=topk_idx, topk_weights=topk_w,
                                                               num_experts=E, num_max_tokens_per_rank=T)
            n = handle.num_recv_tokens
            src = handle.recv_src_metadata[:n, 0].numpy()
            if 'dispatch_recv_src_token_idx' in me:
                if not np.array_equal(src, me['dispatch_recv_src_token_idx']):
                    failures.append('dispatch order != refs.dispatch')
                if not np.array_equal(recv_idx.numpy(), me['dispatch_recv_topk_idx']):
                    failures.append('recv_topk_idx != refs.dispatch')
                if not np.array_equal(_bf16_to_u16(recv_x), me['dispatch_recv_x']):
                    failures.append('recv_x != refs.dispatch')
            local = np.stack([y_of(g) for g in src]) if n else np.zeros((0, K, H), np.uint16)
            local = np.where((recv_idx.numpy() == -1)[..., None], np.uint16(0), local)
            x_red = _u16_to_bf16(ordered_accumulate(local)) if n else torch.empty((0, H), dtype=torch.bfloat16)
            # ---- expanded dispatch + "reduced" combine input (test_ep.py:151-206)
            ex_x, ex_idx, ex_w, ex_handle, _ = buf.dispatch(x, topk_idx=topk_idx, topk_weights=topk_w,
                                                            num_experts=E, num_max_tokens_per_rank=T,
                                                            do_expand=True)
            assert ex_idx is None
            meta = ex_handle.recv_src_metadata.numpy()
            x_exp = np.full((ex_x.shape[0], H), 0x7fc1, dtype=np.uint16)
            for i in range(meta.shape[0]):
                y = y_of(meta[i, 0])
                for k in range(K):
                    if meta[i, 2 + k] >= 0:
                        x_exp[meta[i, 2 + k]] = y[k]
            x_exp = _u16_to_bf16(x_exp)
            for nb in (0, 1, 2):
                bias = None if nb == 0 else (biases[0] if nb == 1 else (biases[0], biases[1]))
                if amr:
                    out, out_w, _ = buf.combine(x_red, handle, topk_weights=recv_w, bias=bias)
                    if not np.array_equal(_bf16_to_u16(out), me[f'combined_multi_b{nb}']):
                        failures.append(f'non-expanded combine b{nb}')
                    if not torch.equal(out_w, topk_w):
                        failures.append(f'non-expanded weights b{nb}')
                    out, out_w, _ = buf.combine(x_exp, ex_handle, topk_weights=ex_w, bias=bias)
                    if not np.array_equal(_bf16_to_u16(out), me[f'combined_multi_b{nb}']):
                        failures.append(f'expanded combine b{nb}')
                    if not torch.equal(out_w, topk_w):
                        failures.append(f'expanded weights b{nb}')
                    # gating-weighted with multiple reduction (the N > 1 bench recipe): bitwise vs the oracle's
                    # restatement, and within the reference's weighted tolerance of the exact sum
                    out, out_w, _ = buf.combine(x_exp, ex_handle, topk_weights=ex_w, bias=bias,
                                                apply_topk_weights=True)
                    bias_u16 = (None, None) if nb == 0 else (me['bias0'], me['bias1'] if nb == 2 else None)
                    if not np.array_equal(_bf16_to_u16(out), weighted_multi_expected(fx, rank, bias_u16)):
                        failures.append(f'weighted multi-reduction combine b{nb}')
                    if not torch.equal(out_w, topk_w):
                        failures.append(f'weighted multi-reduction weights b{nb}')
                    if nb == 0:
                        d = oracle.calc_diff(oracle.bf16_to_f32(_bf16_to_u16(out)), exact_weighted(me))
                        if not d < WEIGHTED_TOLERANCE:
                            failures.append(f'weighted multi-reduction calc_diff {d} >= {WEIGHTED_TOLERANCE}')
                else:
                    out, out_w, _ = buf.combine(x_exp, ex_handle, bias=bias)
                    if not np.array_equal(_bf16_to_u16(out), me[f'combined_single_b{nb}']):
                        failures.append(f'single-reduction expanded combine b{nb}')
                    assert out_w is None
                    out, _, _ = buf.combine(x_red, handle, topk_weights=recv_w, bias=bias)
                    if not np.array_equal(_bf16_to_u16(out), me[f'combined_multi_b{nb}']):
                        failures.append(f'single-reduction non-expanded combine b{nb}')
                    # gating-weighted: every row unreduced to its source rank, one fma chain there
                    out, out_w, _ = buf.combine(x_exp, ex_handle, topk_weights=ex_w, bias=bias,
                                                apply_topk_weights=True)
                    if not torch.equal(out, _weighted_single(me['y'], topk_idx, topk_w, bias)):
                        failures.append(f'single-reduction weighted combine b{nb}')
                    if nb == 0 and not np.array_equal(_bf16_to_u16(out),
                                                      oracle.weighted_ll(me['y'], me['topk_idx'], me['topk_weights'])):
                        failures.append('single-reduction weighted != legacy low-latency restatement')
                    if not torch.equal(out_w, topk_w):
                        failures.append(f'single-reduction weighted pass-through b{nb}')
            buf.destroy()
        queue.put((rank, failures))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, [traceback.format_exc()]))


def _spawn(fixture, world, env=None):
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fixture, queue, env)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, failures = queue.get(timeout=240)
            results[rank] = failures
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return results


@pytest.mark.parametrize('fixture,world', [
    ('f1_ep1_t128_h1024_k2.npz', 1),
    ('f4_ep4_t96_h256_k2.npz', 4),
    ('f2_ep8_t64_h256_k8.npz', 8),
    ('f3_ep8_skew_t128_h64_k8.npz', 8),
])
def test_elastic_buffer_matches_golden(fixture, world):
    results = _spawn(fixture, world)
    assert len(results) == world
    bad = {r: f for r, f in results.items() if f}
    assert not bad, bad


@pytest.mark.parametrize('fixture,world,chunks', [
    ('f4_ep4_t96_h256_k2.npz', 4, 3),
    ('f3_ep8_skew_t128_h64_k8.npz', 8, 5),
])
def test_chunked_combine_matches_golden(fixture, world, chunks):
    """The EP > 1 combine split into source-token chunks (the pipelined schedule's plans) gives
    the same bits as the one-shot exchange."""
    results = _spawn(fixture, world, {'DEEPEP_COMBINE_CHUNKS': str(chunks)})
    assert len(results) == world
    bad = {r: f for r, f in results.items() if f}
    assert not bad, bad


def _random_worker(rank, world, port, seed, queue, env=None):
    import sys
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        os.environ.update(env or {})
        dist.init_process_group('gloo', rank=rank, world_size=world)
        import oracle
        from deepep_amd import ElasticBuffer
        from tests.oracle_kernels import OracleKernels
        T, H, K, E = (200 if env else 48), 136, 8, 8 * world     # hidden 136: a ragged number of 16-byte vectors
        rng = np.random.default_rng(seed)
        idx_all, w_all, y_all, b_all = [], [], [], []
        for r in range(world):
            idx = np.stack([rng.permutation(E)[:K] for _ in range(T)]).astype(np.int64)
            idx[rng.random((T, K)) < 0.2] = -1
            idx[0] = -1                              # a token routed nowhere
            w = rng.random((T, K)).astype(np.float32) * (idx >= 0)
            y = oracle.f32_to_bf16(rng.standard_normal((T, K, H)).astype(np.float32))
            y[idx < 0] = 0
            idx_all.append(idx), w_all.append(w), y_all.append(y)
            b_all.append(oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)))
        disp = oracle.simulate_dispatch(idx_all, E, T)
        x_exp_all, w_exp_all = [], []
        for r, d in enumerate(disp):
            xe = np.zeros((d['num_expanded'], H), np.uint16)
            we = np.zeros((d['num_expanded'],), np.float32)
            for row, (g, k) in enumerate(d['expanded_src']):
                s, t = divmod(int(g), T)
                xe[row], we[row] = y_all[s][t, k], w_all[s][t, k]
            x_exp_all.append(xe), w_exp_all.append(we)
        expect = oracle.combine_ep(x_exp_all, [d['src_metadata'] for d in disp], idx_all, E, T, expanded=True,
                                   topk_weights_per_rank=w_exp_all,
                                   bias_per_rank=[(b, None) for b in b_all])
        failures = []
        x = torch.zeros((T, H), dtype=torch.bfloat16)
        diagonals = {}
        for bypass in (True, False):
            buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
            buf._kernels = OracleKernels()
            buf.local_bypass = bypass
            # every row all-to-all of this buffer (dispatch rows, combine partials): this rank's own split
            splits = []
            a2a = buf._a2a

            def spy(out, inp, out_splits=None, in_splits=None, _a2a=a2a, _splits=splits):
                if in_splits is not None:
                    _splits.append((in_splits[rank], out_splits[rank]))
                return _a2a(out, inp, out_splits, in_splits)
            buf._a2a = spy
            _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=torch.from_numpy(idx_all[rank]),
                                                 topk_weights=torch.from_numpy(w_all[rank]),
                                                 num_experts=E, do_expand=True)
            if not np.array_equal(handle.recv_src_metadata.numpy(), disp[rank]['src_metadata']):
                failures.append(f'recv_src_metadata differs from the oracle dispatch (bypass {bypass})')
            out, out_w, _ = buf.combine(_u16_to_bf16(x_exp_all[rank]), handle, topk_weights=ex_w,
                                        bias=_u16_to_bf16(b_all[rank]))
            if not np.array_equal(_bf16_to_u16(out), expect[rank][0]):
                failures.append(f'combined_x (bypass {bypass})')
            if not np.array_equal(out_w.numpy(), expect[rank][1]):
                failures.append(f'combined_topk_weights (bypass {bypass})')
            diagonals[bypass] = splits
        # the local bypass: no row exchange carries this rank's own rows; without it they travel
        if not diagonals[True] or any(a or b for a, b in diagonals[True]):
            failures.append(f'own rows in the all-to-all with the local bypass: {diagonals[True]}')
        if not any(a for a, _ in diagonals[False]):
            failures.append(f'no own rows without the bypass (test routing too sparse?): {diagonals[False]}')
        queue.put((rank, failures))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, [traceback.format_exc()]))


@pytest.mark.parametrize('world,chunks', [(2, 0), (3, 0), (2, 4)])
def test_random_routing_world(world, chunks):
    """world_size 2 (and 3: a rank count that does not divide top-k) against oracle.combine_ep;
    (2, 4): the same exchange split into 4 source-token chunks."""
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    env = {'DEEPEP_COMBINE_CHUNKS': str(chunks)} if chunks else None
    procs = [ctx.Process(target=_random_worker, args=(r, world, port, 7 + world, queue, env))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, failures = queue.get(timeout=240)
            results[rank] = failures
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert len(results) == world and not any(results.values()), results


def _modes_worker(rank, world, port, alignment, do_cpu_sync, do_handle_copy, queue, t_max_extra=0):
    import sys
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from deepep_amd import ElasticBuffer
        from tests.helpers import dispatch_mode_checks
        from tests.oracle_kernels import OracleKernels
        T, H, K, E = 40, 64, 4, 4 * world
        g = torch.Generator().manual_seed(rank + 11)
        scores = torch.rand((T, E), generator=g)
        w, idx = torch.topk(scores, K, dim=-1, sorted=False)
        idx = idx.to(torch.int64)
        idx[torch.rand(idx.shape, generator=g) < 0.2] = -1
        idx[0] = -1                                        # tokens routed nowhere: fewer rows received than T
        idx[T // 2] = -1
        w = w.masked_fill(idx < 0, 0)
        x = torch.randn((T, H), generator=g).to(torch.bfloat16)
        T_max = T + t_max_extra
        buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T_max, hidden=H, num_topk=K)
        buf._kernels = OracleKernels()
        queue.put((rank, dispatch_mode_checks(buf, x, idx, w, E, T_max, alignment, do_cpu_sync, do_handle_copy)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, [traceback.format_exc()]))


@pytest.mark.parametrize('world,alignment,do_cpu_sync,do_handle_copy,t_max_extra', [
    (2, 1, True, True, 0), (2, 4, True, False, 0), (2, 8, False, True, 0), (1, 8, False, True, 0),
    (1, 1, False, False, 0), (1, 1, False, True, 200), (2, 4, False, True, 200), (2, 1, True, True, 200)])
def test_dispatch_modes(world, alignment, do_cpu_sync, do_handle_copy, t_max_extra):
    """Cached / cached-expanded-zero-padded / deterministic / counter / no-CPU-sync dispatch
    (tests/elastic/test_ep.py:143-177, 355-466) over 1 and 2 gloo ranks (one rank without a CPU sync
    sizes its launches for the worst case and bounds them by the device count).  t_max_extra: a
    num_max_tokens_per_rank well above the batch (ceil(T / 128) != ceil(T_max / 128)), so a cached
    dispatch over a no-CPU-sync handle must reuse the handle's worst-case tables."""
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_modes_worker, args=(r, world, port, alignment, do_cpu_sync, do_handle_copy, queue,
                                                     t_max_extra))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, failures = queue.get(timeout=240)
            results[rank] = failures
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert len(results) == world and not any(results.values()), results


def _empty_rank_worker(rank, world, port, queue):
    import sys
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        import oracle
        from deepep_amd import ElasticBuffer
        from tests.oracle_kernels import OracleKernels
        T_max, H, K, E = 32, 72, 4, 4 * world
        Ts = [0, T_max, 5][:world]                    # rank 0 sends nothing; the others do
        rng = np.random.default_rng(3)
        idx_all, w_all, y_all = [], [], []
        for r in range(world):
            idx = np.array([rng.permutation(E)[:K] for _ in range(Ts[r])], dtype=np.int64).reshape(Ts[r], K)
            w = rng.random((Ts[r], K)).astype(np.float32)
            y = oracle.f32_to_bf16(rng.standard_normal((Ts[r], K, H)).astype(np.float32))
            idx_all.append(idx), w_all.append(w), y_all.append(y)
        disp = oracle.simulate_dispatch(idx_all, E, T_max)
        x_exp_all, w_exp_all = [], []
        for r, d in enumerate(disp):
            xe = np.zeros((d['num_expanded'], H), np.uint16)
            we = np.zeros((d['num_expanded'],), np.float32)
            for row, (g, k) in enumerate(d['expanded_src']):
                s, t = divmod(int(g), T_max)
                xe[row], we[row] = y_all[s][t, k], w_all[s][t, k]
            x_exp_all.append(xe), w_exp_all.append(we)
        expect = oracle.combine_ep(x_exp_all, [d['src_metadata'] for d in disp], idx_all, E, T_max, expanded=True,
                                   topk_weights_per_rank=w_exp_all, bias_per_rank=[(None, None)] * world)
        buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T_max, hidden=H, num_topk=K)
        buf._kernels = OracleKernels()
        x = torch.zeros((Ts[rank], H), dtype=torch.bfloat16)
        _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=torch.from_numpy(idx_all[rank]),
                                             topk_weights=torch.from_numpy(w_all[rank]), num_experts=E,
                                             do_expand=True)
        failures = []
        out, out_w, _ = buf.combine(_u16_to_bf16(x_exp_all[rank]), handle, topk_weights=ex_w)
        if tuple(out.shape) != (Ts[rank], H) or not np.array_equal(_bf16_to_u16(out), expect[rank][0]):
            failures.append('combined_x')
        if not np.array_equal(out_w.numpy(), expect[rank][1]):
            failures.append('combined_topk_weights')
        queue.put((rank, failures))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, [traceback.format_exc()]))


@pytest.mark.parametrize('world', [2, 3])
def test_rank_with_no_tokens(world):
    """A rank that sends no tokens (num_tokens = 0) still takes part in dispatch and combine."""
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_rank_worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, failures = queue.get(timeout=240)
            results[rank] = failures
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert len(results) == world and not any(results.values()), results


def test_interleave_by_rank_is_a_round_robin_permutation():
    """xGMI phase-A units are reordered round-robin over destination ranks (every link busy at once)."""
    from tests.plan_ref import interleave_by_rank as _interleave_by_rank
    dest = torch.tensor([0] * 5 + [1] * 2 + [3] * 4)           # per received row, grouped by rank
    units = torch.tensor([0, 1, 2, 4, 5, 6, 7, 9, 10])          # a chunk's rows (ascending)
    out = _interleave_by_rank(units, dest, 4)
    assert sorted(out.tolist()) == units.tolist()
    assert out.tolist() == [0, 5, 7, 1, 6, 9, 2, 10, 4]
    assert _interleave_by_rank(units, dest, 1).tolist() == units.tolist()
    assert _interleave_by_rank(units[:0], dest, 4).numel() == 0


def test_notify_layout_matches_brute_force():
    """The dispatch notify on the host: per-rank view and the all-gathered view (xGMI push) agree,
    and every source's rows land in disjoint, packed, source-ordered ranges of each destination."""
    from deepep_amd.buffer import notify_layout
    rng = np.random.default_rng(5)
    for R, epr in ((1, 4), (2, 3), (3, 1), (8, 32)):
        counts = rng.integers(0, 50, size=(R, R, epr))            # [source][destination][local expert]
        rec = np.concatenate([counts.sum(-1, keepdims=True), counts], axis=-1)   # [tokens | per expert]
        # a token counts once per destination in `tokens` even if it hits several of its experts
        rec[..., 0] = np.minimum(rec[..., 0], rng.integers(0, 60, size=(R, R)))
        everyone = [int(v) for v in rec.reshape(-1)]
        spans = {}
        for r in range(R):
            mine = [int(v) for v in rec[:, r].reshape(-1)]
            _, recv_a, exp_a, off_none, _ = notify_layout(mine, R, r, epr, all_gathered=False)
            sends, recv_b, exp_b, offs, _ = notify_layout(everyone, R, r, epr, all_gathered=True)
            assert off_none is None and recv_a == recv_b and exp_a == exp_b
            assert recv_a == [int(v) for v in rec[:, r, 0]]
            assert exp_a == [int(v) for v in rec[:, r, 1:].sum(0)]
            assert sends == [int(v) for v in rec[r, :, 0]]
            for d in range(R):
                spans.setdefault(d, []).append((offs[d], offs[d] + sends[d], r))
        for d, sp in spans.items():                               # packed by source rank, no overlap
            sp.sort()
            assert [s[2] for s in sp] == list(range(R)) and sp[0][0] == 0
            assert all(a[1] == b[0] for a, b in zip(sp, sp[1:]))
            assert sp[-1][1] == int(rec[:, d, 0].sum())


def _sf_worker(rank, world, port, queue):
    import sys
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from deepep_amd import ElasticBuffer
        from tests.oracle_kernels import OracleKernels
        T, H, K, E = 37, 256, 4, 8 * world
        g = torch.Generator().manual_seed(rank)
        idx = torch.stack([torch.randperm(E, generator=g)[:K] for _ in range(T)])
        w = torch.rand((T, K), generator=g)
        xq = torch.randn((T, H), generator=g).to(torch.float8_e4m3fn)
        sf = torch.rand((T, H // 128), generator=g)
        buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
        buf._kernels = OracleKernels()
        failures = []
        (rq, rsf), _, _, h, _ = buf.dispatch((xq, sf), topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
        for hh in (None, h):
            args = dict(topk_weights=w, do_expand=True, use_tma_aligned_col_major_sf=True)
            args.update(handle=hh) if hh is not None else args.update(topk_idx=idx, num_experts=E)
            (cq, csf), _, _, _, _ = buf.dispatch((xq, sf), **args)
            n = csf.shape[0]
            if csf.stride() != (1, (n + 3) // 4 * 4):
                failures.append(f'scale-factor strides {csf.stride()} (cached {hh is not None})')
            if not (torch.equal(csf, rsf) and torch.equal(cq.view(torch.uint8), rq.view(torch.uint8))):
                failures.append(f'column-major dispatch differs (cached {hh is not None})')
        queue.put((rank, failures))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, [traceback.format_exc()]))


@pytest.mark.parametrize('world', [1, 2])
def test_tma_aligned_col_major_scale_factors(world):
    """dispatch(..., use_tma_aligned_col_major_sf=True) (the reference's layout for the next GEMM,
    buffer.hpp:1090-1096): the received scale factors are column-major with each pack column 16-byte
    aligned, and hold the same values as the row-major ones, fresh and cached."""
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sf_worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, failures = queue.get(timeout=240)
            results[rank] = failures
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert len(results) == world and not any(results.values()), results


def _barrier_worker(rank, world, port, queue):
    import sys
    import time
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from deepep_amd import ElasticBuffer
        buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=16, hidden=64, num_topk=2)
        waited = []
        for kw in (dict(), dict(use_comm_stream=False), dict(with_cpu_sync=True), dict(sequential=False)):
            dist.barrier()
            if rank == 0:
                time.sleep(0.4)                            # the last rank to arrive
            t0 = time.perf_counter()
            buf.barrier(**kw)
            waited.append(time.perf_counter() - t0)
        queue.put((rank, waited))
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, traceback.format_exc()))


def test_barrier_waits_for_every_rank():
    """ElasticBuffer.barrier (elastic.py:497-508) on a host-side group: every argument form returns on a rank
    only once the last rank has arrived."""
    world = 3
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_barrier_worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(queue.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
    assert all(isinstance(v, list) for v in res.values()), res
    for r in range(1, world):
        assert all(t > 0.3 for t in res[r]), (r, res[r])
