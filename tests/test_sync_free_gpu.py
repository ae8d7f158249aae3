"""The combine needs no host synchronisation, and its EP > 1 schedule is ordered by streams alone.

* The EP > 1 plan kernels (deepep_plan_expert / _source, deepep_route_block_counts) against their CPU
  restatement (tests/plan_ref.py), bit for bit, over rank counts, top-k, chunking, both reduction
  recipes, both layouts and both transports' addressing.
* A FIRST combine on a fresh handle (EP = 1, and EP = 4 / 8 simulated by threads whose exchange has
  ProcessGroupNCCL's stream semantics, tests/sim.py) runs under torch.cuda.set_sync_debug_mode("error")
  -- any host sync raises -- and is bitwise equal to the oracle; the reference's combine has no CPU
  sync either (csrc/elastic/buffer.hpp:1179-1343).
* The first combine on a fresh handle is captured into a HIP graph with no eager call before it.
* The pipelined EP > 1 schedule (phase A(c) | exchange(c) | phase B(c) on a second stream) is correct
  only because of its stream waits: with the exchange delayed on its stream, dropping the wait for it
  makes the result wrong, which this test detects.
"""
import os

import numpy as np
import pytest
import torch

import oracle
from tests import plan_ref
from tests.sim import FakeGroup, ThreadComm, run_threads

pytestmark = pytest.mark.gpu


def _u16(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _bf16(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16).cuda()


def _routing(world, T, K, E, seed, masked=0.1):
    rng = np.random.default_rng(seed)
    idx_all, w_all = [], []
    for _ in range(world):
        scores = rng.random((T, E))
        idx = np.argsort(-scores, axis=1)[:, :K].astype(np.int64)
        idx[rng.random((T, K)) < masked] = -1
        idx_all.append(idx)
        w_all.append((rng.random((T, K)).astype(np.float32) * (idx >= 0)).astype(np.float32))
    return rng, idx_all, w_all


def _expanded_inputs(rng, disp, idx_all, w_all, T, H):
    """Per expert rank: expanded rows (random bf16, one per (token, lane) received) and their weights."""
    x_all, wexp_all = [], []
    for d in disp:
        n = d['num_expanded']
        x_all.append(oracle.f32_to_bf16(rng.standard_normal((n, H)).astype(np.float32)))
        we = np.zeros((n,), np.float32)
        for row, (g, k) in enumerate(d['expanded_src']):
            s, t = divmod(int(g), T)
            we[row] = w_all[s][t, k]
        wexp_all.append(we)
    return x_all, wexp_all


@pytest.fixture(scope='module')
def kern():
    from deepep_amd.kernels import HipKernels
    return HipKernels()


# ----------------------------------------------------------------------------- plan kernels
@pytest.mark.parametrize('world,K,T,chunks', [(2, 8, 200, 3), (3, 4, 130, 1), (4, 2, 333, 4), (8, 8, 700, 4),
                                              (8, 8, 64, 1), (5, 1, 97, 2)])
def test_plan_kernels_match_reference(kern, world, K, T, chunks):
    from deepep_amd import _lib
    from deepep_amd.handle import chunk_geometry
    E = world * max(2, (K + world - 1) // world + 1)
    _, idx_all, _ = _routing(world, T, K, E, seed=world * 100 + K)
    nb, bpc, _ = chunk_geometry(T, chunks)
    disp = oracle.simulate_dispatch(idx_all, E, T)
    # per-source block counts: HIP vs the restatement
    tok_all, pairs_all = [], []
    for s in range(world):
        idx = torch.from_numpy(idx_all[s]).cuda()
        tok = torch.empty((world, nb), dtype=torch.int32, device='cuda')
        pairs = torch.empty_like(tok)
        kern.route_block_counts(idx, E, world, nb, tok, pairs)
        rt, rp = plan_ref.route_block_counts(torch.from_numpy(idx_all[s]), E, world, nb)
        assert torch.equal(tok.cpu(), rt) and torch.equal(pairs.cpu(), rp)
        tok_all.append(rt)
        pairs_all.append(rp)
    bases = torch.tensor([(1 << 40) * (s + 1) for s in range(world)], dtype=torch.int64)
    epr = E // world
    C = (nb + bpc - 1) // bpc
    for r in range(world):
        meta = torch.from_numpy(disp[r]['src_metadata']).cuda()
        recv_tok = torch.stack([tok_all[s][r] for s in range(world)])        # [source, block]
        recv_pairs = torch.stack([pairs_all[s][r] for s in range(world)])
        for single in (False, True):
            for expanded in ((True,) if single else (True, False)):
                # (transport, padded): RCCL with and without the local bypass, xGMI windows; exact counts and
                # the worst-case padding of a dispatch without a CPU sync
                for window, bypass in ((False, False), (False, True), (True, False)):
                    for padded in (0, bpc * 64 * (min(K, epr) if single else 1)):
                        flags = ((_lib.PLAN_EXPANDED if expanded else 0) | (_lib.PLAN_SINGLE if single else 0) |
                                 (_lib.PLAN_RANK_LAYOUT if world <= K and not single else 0) |
                                 (_lib.PLAN_INTERLEAVE if window else 0) | (_lib.PLAN_LOCAL_BYPASS if bypass else 0))
                        total = C * world * padded if padded else int((recv_pairs if single else recv_tok).sum())
                        width = K if expanded and not single else 1
                        outs = []
                        for dev in ('cuda', 'cpu'):
                            ta = torch.full((total, width), -7, dtype=torch.int32, device=dev)
                            wa = torch.full((total, K), -7, dtype=torch.int32, device=dev) if not expanded else None
                            orow = torch.full((total,), -7, dtype=torch.int64, device=dev) if window else None
                            args = (K, world, r, T, recv_tok.to(dev), recv_pairs.to(dev), nb, bpc, flags, ta, wa,
                                    bases.to(dev) if window else None, 14400 if window else 0, orow)
                            if dev == 'cuda':
                                kern.plan_expert(meta, *args, window_bytes=K * T * 14400 if window else 0,
                                                 padded_stride=padded)
                            else:
                                plan_ref.plan_expert(meta.cpu(), *args, padded=padded)
                            outs.append([t.cpu() if t is not None else None for t in (ta, wa, orow)])
                        for g, c, name in zip(outs[0], outs[1], ('table_a', 'wtable_a', 'out_rows')):
                            assert (g is None) == (c is None)
                            assert g is None or torch.equal(g, c), (r, single, expanded, window, bypass, padded, name)
        # source side (this rank's own tokens)
        idx = torch.from_numpy(idx_all[r]).cuda()
        dst = torch.empty((T, world), dtype=torch.int32, device='cuda')
        send_counts = torch.empty((world,), dtype=torch.int32, device='cuda')
        kern.dispatch_route(idx, E, world, dst, send_counts)
        for single in (False, True):
            for window, bypass in ((False, False), (False, True), (True, False)):
                for padded in ((0,) if window else (0, bpc * 64 * (min(K, epr) if single else 1))):
                    flags = ((_lib.PLAN_SINGLE if single else 0) | (_lib.PLAN_WINDOW if window else 0) |
                             (_lib.PLAN_RANK_LAYOUT if world <= K and not single else 0) |
                             (_lib.PLAN_LOCAL_BYPASS if bypass else 0))
                    width = K if single else min(world, K)
                    outs = []
                    for dev in ('cuda', 'cpu'):
                        tb = torch.full((T, width), -7, dtype=torch.int32, device=dev)
                        wt = None if single else torch.full((T, K), -7, dtype=torch.int32, device=dev)
                        args = (E, world, r, T, dst.to(dev), tok_all[r].to(dev), pairs_all[r].to(dev), nb, bpc, flags,
                                0 if single else 3600, 0 if single else 3584, tb, wt)
                        if dev == 'cuda':
                            kern.plan_source(idx, *args, padded_stride=padded)
                        else:
                            plan_ref.plan_source(idx.cpu(), *args, padded=padded)
                        outs.append((tb.cpu(), wt.cpu() if wt is not None else None))
                    assert torch.equal(outs[0][0], outs[1][0]), (r, single, window, bypass, padded, 'table_b')
                    assert (outs[0][1] is None and outs[1][1] is None) or torch.equal(outs[0][1], outs[1][1]), \
                        (r, single, window, bypass, padded, 'wtable')


# ----------------------------------------------------------------------------- sync-free first combine
def _group1():
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29561')
        dist.init_process_group('gloo', rank=0, world_size=1)
    return dist.group.WORLD


def _sync_free_rank(rank, world, T, H, K, E, comm, results):
    try:
        torch.cuda.set_device(0)
        from deepep_amd import ElasticBuffer
        rng, idx_all, w_all = _routing(world, T, K, E, seed=77 + world)
        disp = oracle.simulate_dispatch(idx_all, E, T)
        x_all, wexp_all = _expanded_inputs(rng, disp, idx_all, w_all, T, H)
        bias = [oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)) for _ in range(world)]
        metas = [d['src_metadata'] for d in disp]
        expect = oracle.combine_ep(x_all, metas, idx_all, E, T, expanded=True, topk_weights_per_rank=wexp_all,
                                   bias_per_rank=[(b, None) for b in bias])[rank]
        expect_single = oracle.combine_ep(x_all, metas, idx_all, E, T, expanded=True, allow_multiple_reduction=False,
                                          bias_per_rank=[(b, None) for b in bias])[rank][0]
        grp = FakeGroup(rank, world, comm) if world > 1 else _group1()
        failures = []
        for amr in (True, False):
            buf = ElasticBuffer(grp, num_max_tokens_per_rank=T, hidden=H, num_topk=K, allow_multiple_reduction=amr)
            if world > 1:
                comm.install(buf, rank)
            x = torch.zeros((T, H), dtype=torch.bfloat16, device='cuda')
            _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=torch.from_numpy(idx_all[rank]).cuda(),
                                                 topk_weights=torch.from_numpy(w_all[rank]).cuda(), num_experts=E,
                                                 do_expand=True)
            if not np.array_equal(handle.recv_src_metadata.cpu().numpy(), metas[rank]):
                failures.append(f'amr={amr}: metadata')
            xin, b = _bf16(x_all[rank]), _bf16(bias[rank])
            assert not handle._combine_plans                 # the combine below is the handle's first
            torch.cuda.synchronize()
            if world > 1:
                comm.bar.wait()
            if rank == 0:
                torch.cuda.set_sync_debug_mode('error')
            if world > 1:
                comm.bar.wait()
            try:
                if amr:
                    out, out_w, _ = buf.combine(xin, handle, topk_weights=ex_w, bias=b)
                else:
                    out, out_w, _ = buf.combine(xin, handle, bias=b)
            finally:
                if world > 1:
                    comm.bar.wait()
                if rank == 0:
                    torch.cuda.set_sync_debug_mode(0)
            torch.cuda.synchronize()
            if not np.array_equal(_u16(out), expect[0] if amr else expect_single):
                failures.append(f'amr={amr}: combined_x')
            if amr and not np.array_equal(out_w.cpu().numpy(), expect[1]):
                failures.append('combined_topk_weights')
        results[rank] = failures
    except Exception:
        import traceback
        results[rank] = [traceback.format_exc()]
        if comm is not None:
            comm.bar.abort()


def _dispatch_sync_free_rank(rank, world, T, H, K, E, comm, results):
    """A fresh dispatch(do_cpu_sync=False) and the handle's first combine, both under
    set_sync_debug_mode('error'): the worst-case-padded RCCL exchange (equal splits, no host sizes)
    and the padded combine plan."""
    try:
        torch.cuda.set_device(0)
        from deepep_amd import ElasticBuffer
        rng, idx_all, w_all = _routing(world, T, K, E, seed=313 + world)
        disp = oracle.simulate_dispatch(idx_all, E, T)
        x_all = [oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)) for _ in range(world)]
        bias = [oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)) for _ in range(world)]
        x_exp_all, w_exp_all = [], []
        for d in disp:
            xe = np.zeros((d['num_expanded'], H), np.uint16)
            we = np.zeros((d['num_expanded'],), np.float32)
            for row, (g, k) in enumerate(d['expanded_src']):
                s, t = divmod(int(g), T)
                xe[row], we[row] = x_all[s][t], w_all[s][t, k]
            x_exp_all.append(xe), w_exp_all.append(we)
        metas = [d['src_metadata'] for d in disp]
        failures = []
        for amr in (True, False):
            expect = oracle.combine_ep(x_exp_all, metas, idx_all, E, T, expanded=True, allow_multiple_reduction=amr,
                                       topk_weights_per_rank=w_exp_all if amr else None,
                                       bias_per_rank=[(b, None) for b in bias])[rank]
            buf = ElasticBuffer(FakeGroup(rank, world, comm), num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                                allow_multiple_reduction=amr)
            comm.install(buf, rank)
            x, b = _bf16(x_all[rank]), _bf16(bias[rank])
            idx, w = torch.from_numpy(idx_all[rank]).cuda(), torch.from_numpy(w_all[rank]).cuda()
            torch.cuda.synchronize()
            comm.bar.wait()
            if rank == 0:
                torch.cuda.set_sync_debug_mode('error')
            comm.bar.wait()
            try:
                ex_x, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E,
                                                        do_expand=True, do_cpu_sync=False)
                if amr:
                    out, out_w, _ = buf.combine(ex_x, handle, topk_weights=ex_w, bias=b)
                else:
                    out, out_w, _ = buf.combine(ex_x, handle, bias=b)
            finally:
                comm.bar.wait()
                if rank == 0:
                    torch.cuda.set_sync_debug_mode(0)
            torch.cuda.synchronize()
            n = int(handle.psum_num_recv_tokens_per_scaleup_rank[-1].item())
            meta = handle.recv_src_metadata.cpu().numpy()
            if meta.shape[0] != world * T or not np.array_equal(meta[:n], metas[rank]) or not (meta[n:] == -1).all():
                failures.append(f'amr={amr}: metadata')
            if not np.array_equal(_u16(out), expect[0]):
                failures.append(f'amr={amr}: combined_x')
            if amr and not np.array_equal(out_w.cpu().numpy(), expect[1]):
                failures.append(f'amr={amr}: combined_topk_weights')
            # a cached dispatch over the no-CPU-sync handle (the padded exchange again, the handle's tables):
            # the same bits as its first call on every received row
            comm.bar.wait()
            c_x, _, c_w, _, _ = buf.dispatch(x, topk_weights=w, do_expand=True, handle=handle)
            torch.cuda.synchronize()
            valid = torch.from_numpy(meta[:n, 2:]).cuda()
            valid = valid[valid >= 0].long()
            if c_x.shape != ex_x.shape or not torch.equal(c_x[valid].view(torch.int16), ex_x[valid].view(torch.int16)) \
                    or not torch.equal(c_w[valid], ex_w[valid]):
                failures.append(f'amr={amr}: cached dispatch over the no-CPU-sync handle')
            comm.bar.wait()
        results[rank] = failures
    except Exception:
        import traceback
        results[rank] = [traceback.format_exc()]
        if comm is not None:
            comm.bar.abort()


@pytest.mark.parametrize('world,T,E', [(4, 128, 64), (8, 1088, 64), (8, 1088, 32)])
def test_dispatch_without_cpu_sync_ep_gt_1(world, T, E):
    """EP > 1 dispatch(do_cpu_sync=False) + first combine over the (simulated) RCCL transport with no
    host synchronisation (csrc/elastic/buffer.hpp:1065-1070); T = 1088 gives a pipelined (multi-chunk)
    padded combine; E = 32 at EP = 8: 4 experts per rank < top-8, so the single reduction's padded
    chunks hold min(K, experts per rank) rows per token.  Bitwise vs the oracle, plain and single
    reduction; then a cached dispatch over the same handle."""
    H, K = 256, 8
    comm = ThreadComm(world)
    results = run_threads(world, _dispatch_sync_free_rank, (world, T, H, K, E, comm))
    assert len(results) == world, results
    bad = {r: f for r, f in results.items() if f}
    assert not bad, bad


@pytest.mark.parametrize('world,T', [(1, 1024), (4, 1024), (8, 1088)])
def test_first_combine_has_no_host_sync(world, T):
    """Fresh dispatch, then the handle's FIRST combine (plan built on the device, pipelined exchange at
    EP > 1: T >= 1024 gives 4 chunks) under set_sync_debug_mode('error'); bitwise vs the oracle."""
    H, K, E = 256, 8, 64
    comm = ThreadComm(world) if world > 1 else None
    results = run_threads(world, _sync_free_rank, (world, T, H, K, E, comm))
    assert len(results) == world, results
    bad = {r: f for r, f in results.items() if f}
    assert not bad, bad


def test_first_combine_captured_into_a_graph():
    """The first combine on a fresh handle (its plan is built by kernels inside the capture) is captured
    into a HIP graph and replays bitwise; an eager call afterwards agrees."""
    from deepep_amd import ElasticBuffer
    T, H, K, E = 640, 2048, 8, 64
    rng, idx_all, w_all = _routing(1, T, K, E, seed=5)
    buf = ElasticBuffer(_group1(), num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    x = torch.zeros((T, H), dtype=torch.bfloat16, device='cuda')
    _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=torch.from_numpy(idx_all[0]).cuda(),
                                         topk_weights=torch.from_numpy(w_all[0]).cuda(), num_experts=E, do_expand=True)
    y = _bf16(oracle.f32_to_bf16(rng.standard_normal((handle.num_expanded_tokens, H)).astype(np.float32)))
    bias = _bf16(oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)))
    assert not handle._combine_plans
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out, out_w, _ = buf.combine(y, handle, topk_weights=ex_w, bias=bias, apply_topk_weights=True)
    assert not handle._combine_plans                 # the captured plan belongs to the graph
    graph.replay()
    torch.cuda.synchronize()
    meta = handle.recv_src_metadata.cpu().numpy()
    part, _ = oracle.phase_a(_u16(y), meta, K, True, ex_w.cpu().numpy(), weighted=True)
    recv = np.zeros((1, T, H), np.uint16)
    recv[0, meta[:, 0] % T] = part
    ref, _ = oracle.phase_b(recv, None, idx_all[0], E, 1, True, True, _u16(bias))
    assert np.array_equal(_u16(out), ref)
    assert np.array_equal(out_w.cpu().numpy(), w_all[0])
    eager, eager_w, _ = buf.combine(y, handle, topk_weights=ex_w, bias=bias, apply_topk_weights=True)
    torch.cuda.synchronize()
    assert torch.equal(eager, out) and torch.equal(eager_w, out_w)


def _dispatch_combine_free(buf, x, idx, w, E, y, bias):
    """A fresh dispatch without CPU sync (EP = 1) and the first combine over its handle."""
    _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True,
                                         do_cpu_sync=False)
    out, out_w, _ = buf.combine(y, handle, topk_weights=ex_w, bias=bias, apply_topk_weights=True)
    return out, out_w, handle


@pytest.mark.parametrize('capture', [False, True])
def test_dispatch_without_cpu_sync_then_combine(capture):
    """dispatch(do_cpu_sync=False) on one rank issues kernels only (the reference's no-sync mode,
    csrc/elastic/buffer.hpp:1065-1070): with its first combine it runs under
    set_sync_debug_mode('error') and, with no eager call before it, inside a HIP graph capture.
    Tokens routed nowhere make the received count smaller than the launches' worst case; the
    combined rows are bitwise equal to the oracle and to a host-synced dispatch's."""
    from deepep_amd import ElasticBuffer
    T, H, K, E = 768, 1024, 8, 64
    rng, idx_all, w_all = _routing(1, T, K, E, seed=17)
    idx_all[0][[0, 5, T - 1]] = -1                       # three tokens routed nowhere
    w_all[0][[0, 5, T - 1]] = 0
    buf = ElasticBuffer(_group1(), num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    idx, w = torch.from_numpy(idx_all[0]).cuda(), torch.from_numpy(w_all[0]).cuda()
    x = _bf16(oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)))
    worst = T * min(K, E)
    y = _bf16(oracle.f32_to_bf16(rng.standard_normal((worst, H)).astype(np.float32)))
    bias = _bf16(oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)))
    torch.cuda.synchronize()
    if capture:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out, out_w, handle = _dispatch_combine_free(buf, x, idx, w, E, y, bias)
        graph.replay()
    else:
        torch.cuda.set_sync_debug_mode('error')
        try:
            out, out_w, handle = _dispatch_combine_free(buf, x, idx, w, E, y, bias)
        finally:
            torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    assert handle.num_expanded_tokens == worst and handle.recv_src_metadata.shape[0] == T
    assert handle.num_recv_tokens_per_expert_list == []
    meta = handle.recv_src_metadata.cpu().numpy()
    n = int(handle.psum_num_recv_tokens_per_scaleup_rank[-1].item())
    assert n == T - 3 and (meta[n:] == -1).all()
    # the same batch through a host-synced dispatch: same metadata rows, same combine bits
    _, _, s_w, s_handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    assert np.array_equal(s_handle.recv_src_metadata.cpu().numpy(), meta[:n])
    s_out, s_out_w, _ = buf.combine(y[:s_handle.num_expanded_tokens].contiguous(), s_handle, topk_weights=s_w,
                                    bias=bias, apply_topk_weights=True)
    torch.cuda.synchronize()
    assert torch.equal(s_out, out) and torch.equal(s_out_w, out_w)
    ex_w = np.zeros((worst,), np.float32)
    slots = meta[:n, 2:]
    tok = meta[:n, 0] % T
    ex_w[slots[slots >= 0]] = w_all[0][tok][slots >= 0]
    part, _ = oracle.phase_a(_u16(y), meta[:n], K, True, ex_w, weighted=True)
    recv = np.zeros((1, T, H), np.uint16)
    recv[0, tok] = part
    ref, _ = oracle.phase_b(recv, None, idx_all[0], E, 1, True, True, _u16(bias))
    assert np.array_equal(_u16(out), ref)
    assert np.array_equal(out_w.cpu().numpy(), w_all[0])


def test_plan_expert_rejects_impossible_metadata(kern):
    """Window addresses come only from metadata a correct dispatch can produce: a received row whose
    source index or master lane is negative, or whose source rank is out of range, gets a null window
    row (phase A then skips it and flags the call) -- never an address computed from garbage."""
    from deepep_amd.handle import PLAN_EXPANDED, PLAN_RANK_LAYOUT
    R, K, T_max, rank, row_bytes = 2, 2, 64, 1, 1024
    meta = torch.tensor([[0, 0 * K + 1, 0, -1],          # source rank 0, token 0, master lane 1: valid
                         [-5, 0 * K + 0, 1, -1],         # negative source index
                         [64 + 3, 1 * K + 0, 2, -1],     # source rank 1, token 3: valid
                         [64 + 9, 7 * K + 0, 3, -1]],    # source rank 7 of 2
                        dtype=torch.int32, device='cuda')
    recv_tok = torch.tensor([[2], [2]], dtype=torch.int32, device='cuda')
    bases = torch.tensor([1 << 40, 2 << 40], dtype=torch.int64, device='cuda')
    table_a = torch.empty((4, K), dtype=torch.int32, device='cuda')
    out_rows = torch.empty((4,), dtype=torch.int64, device='cuda')
    err = torch.zeros((8,), dtype=torch.int32, device='cuda')
    kern.plan_expert(meta, K, R, rank, T_max, recv_tok, recv_tok, 1, 1, PLAN_EXPANDED | PLAN_RANK_LAYOUT,
                     table_a, None, bases, row_bytes, out_rows, window_bytes=K * T_max * row_bytes, error_flag=err)
    torch.cuda.synchronize()
    expect = [(1 << 40) + (rank * T_max + 0) * row_bytes, 0, (2 << 40) + (rank * T_max + 3) * row_bytes, 0]
    assert out_rows.tolist() == expect
    assert table_a.tolist() == meta[:, 2:].tolist()
    rec = err.tolist()
    assert rec[0] == 1 and rec[1] == 2, rec                # bit 1, DEEPEP_FAULT_PLAN_ROW recorded


# ----------------------------------------------------------------------------- stream ordering
def _ordering_rank(rank, world, T, H, K, E, comm, drop_wait, results):
    try:
        torch.cuda.set_device(0)
        from deepep_amd import ElasticBuffer
        rng, idx_all, w_all = _routing(world, T, K, E, seed=31)
        disp = oracle.simulate_dispatch(idx_all, E, T)
        x_all, _ = _expanded_inputs(rng, disp, idx_all, w_all, T, H)
        metas = [d['src_metadata'] for d in disp]
        expect = oracle.combine_ep(x_all, metas, idx_all, E, T, expanded=True)[rank][0]
        buf = ElasticBuffer(FakeGroup(rank, world, comm), num_max_tokens_per_rank=T, hidden=H, num_topk=K)
        comm.install(buf, rank)
        x = torch.zeros((T, H), dtype=torch.bfloat16, device='cuda')
        _, _, _, handle, _ = buf.dispatch(x, topk_idx=torch.from_numpy(idx_all[rank]).cuda(), num_experts=E,
                                          do_expand=True)
        xin = _bf16(x_all[rank])
        buf.combine(xin * 3, handle)                     # warm: plan cached, receive buffers of this size freed
        torch.cuda.synchronize()
        comm.bar.wait()
        if drop_wait:                                   # a schedule that forgets to wait for the exchange
            import tests.sim as sim
            real = buf._a2a_async

            def no_wait(out, inp, os_, is_):
                real(out, inp, os_, is_)                 # the exchange still runs, on its own stream
                return sim.Work(torch.cuda.Event())      # never recorded: waiting on it orders nothing
            buf._a2a_async = no_wait
        comm.delay_cycles = 20_000_000                  # the exchange lands ~10 ms after it is queued
        out, _, _ = buf.combine(xin, handle)
        torch.cuda.synchronize()
        results[rank] = np.array_equal(_u16(out), expect)
    except Exception:
        import traceback
        results[rank] = traceback.format_exc()
        comm.bar.abort()


def _ordering_child(queue):
    """Both schedules in a fresh process (see the test): {drop_wait: {rank: bool or traceback}}."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        T, H, K, E, world = 1024, 256, 8, 32, 4
        out = {}
        for drop_wait in (False, True):
            comm = ThreadComm(world)
            out[drop_wait] = run_threads(world, _ordering_rank, (world, T, H, K, E, comm, drop_wait))
        queue.put(out)
    except Exception:
        import traceback
        queue.put(traceback.format_exc())


def test_pipelined_schedule_is_ordered_by_its_stream_waits():
    """EP = 4, 4 chunks, the exchange delayed on its own stream: the real schedule is bitwise right;
    the same schedule with the exchange's wait dropped is caught (phase B reads receive rows that
    have not landed).  The 4 simulated ranks use 12 streams; HIP deals streams round-robin onto
    GPU_MAX_HW_QUEUES hardware queues (4 by default), and a phase-B stream that shares a queue with a
    delayed exchange stream is serialised behind it, which would hide the race.  So the schedules
    run in a fresh process with 16 hardware queues: every stream of it gets its own."""
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    saved = os.environ.get('GPU_MAX_HW_QUEUES')
    os.environ['GPU_MAX_HW_QUEUES'] = '16'
    try:
        proc = ctx.Process(target=_ordering_child, args=(queue,))
        proc.start()
    finally:
        if saved is None:
            os.environ.pop('GPU_MAX_HW_QUEUES')
        else:
            os.environ['GPU_MAX_HW_QUEUES'] = saved
    try:
        out = queue.get(timeout=150)
    finally:
        proc.join(timeout=30)
        if proc.is_alive():
            proc.kill()
    assert isinstance(out, dict), out
    world = 4
    for drop_wait, results in out.items():
        assert len(results) == world and all(isinstance(v, bool) for v in results.values()), results
        if drop_wait:
            assert not all(results.values()), 'a schedule without the exchange wait went undetected'
        else:
            assert all(results.values()), results
