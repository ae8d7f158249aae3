"""GPU parity of the HIP dispatch (the combine path's handle producer) against the CPU
stand-in primitives and the reference's refs.dispatch fixtures, bitwise.

Every rank of an R-rank dispatch is run on the one GPU; the all-to-all between the
send and receive halves is done with device copies.  Checked: destination slots and
counts, packed rows, recv_src_metadata, recv_topk_idx, expert counts / prefix sums,
the expanded layout and the copied rows, weights and FP8 scale factors.
"""
import numpy as np
import pytest
import torch

from tests.oracle_kernels import OracleKernels

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def hip():
    from deepep_amd.kernels import HipKernels
    return HipKernels()


def _routing(T, E, K, R, masked, skew, gen):
    scores = torch.rand((T, E), generator=gen)
    if skew:
        scores[:, :E // R] *= 3.0                       # rank 0's experts are hot
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    if masked:
        idx[torch.rand(idx.shape, generator=gen) < masked] = -1
        w = w.masked_fill(idx < 0, 0)
    return idx, w


def _run_dispatch(kern, dev, ranks, E, K, H, T_max, expanded, alignment, fp8, direct=False, blocked=True):
    """Both halves of the dispatch for every rank with `kern`; returns per-rank outputs on the CPU.
    direct (one rank): metadata-only packed rows, the copy reads x / sf from the sender's tensors.
    blocked (expanded): the destination-major blocked copy (slots' inverse map), else source-major."""
    from deepep_amd._lib import DISPATCH_BLOCK_ROWS
    from deepep_amd.kernels import RowLayout
    R = len(ranks)
    epr = E // R
    sends = []
    for r, (x, sf, idx, w) in enumerate(ranks):
        T = idx.shape[0]
        x, idx, w = x.to(dev), idx.to(dev), w.to(dev)
        sf = sf.to(dev) if sf is not None else None
        dst = torch.empty((T, R), dtype=torch.int32, device=dev)
        cnt = torch.empty((R,), dtype=torch.int32, device=dev)
        kern.dispatch_route(idx, E, R, dst, cnt)
        cl = [int(v) for v in cnt.tolist()]
        xb = x.view(torch.uint8).view(T, -1)
        sb = sf.view(torch.uint8).view(T, -1) if sf is not None else None
        layout = (RowLayout.make(0, 0, K) if direct else
                  RowLayout.make(xb.shape[1], sb.shape[1] if sb is not None else 0, K))
        offs = torch.tensor([sum(cl[:i]) for i in range(R)], dtype=torch.int32, device=dev)
        packed = torch.zeros((sum(cl), layout.row_bytes), dtype=torch.uint8, device=dev)
        kern.dispatch_pack(xb[:, :0] if direct else xb, None if direct else sb, idx, w, r * T_max, dst, offs,
                           packed, layout)
        hist = torch.empty((E,), dtype=torch.int32, device=dev)
        kern.dispatch_expert_counts(idx, E, hist)
        sends.append((dst.cpu(), cl, packed, layout, xb, sb, hist.cpu()))
    outs = []
    for r in range(R):
        parts = [sends[s][2][sum(sends[s][1][:r]):sum(sends[s][1][:r + 1])] for s in range(R)]
        layout = sends[r][3]
        recv = torch.cat(parts) if parts else torch.zeros((0, layout.row_bytes), dtype=torch.uint8, device=dev)
        N = recv.shape[0]
        counts = [p.shape[0] for p in parts]
        psum = torch.tensor(np.cumsum(counts), dtype=torch.int32, device=dev)
        meta = torch.full((N, K + 2), -7, dtype=torch.int32, device=dev)
        ridx = None if expanded else torch.empty((N, K), dtype=torch.int64, device=dev)
        nb = (N + DISPATCH_BLOCK_ROWS - 1) // DISPATCH_BLOCK_ROWS
        bc = torch.empty((nb, epr), dtype=torch.int32, device=dev)
        kern.dispatch_count(recv, layout, N, r, epr, psum, meta, ridx, bc)
        ec = torch.empty((epr,), dtype=torch.int32, device=dev)
        pe = torch.empty((epr,), dtype=torch.int32, device=dev)
        kern.dispatch_scan(bc, epr, alignment, expanded, ec, pe)
        aligned = [(int(c) + alignment - 1) // alignment * alignment for c in ec.tolist()]
        inv = None
        if expanded:
            rows = sum(aligned)
            inv = torch.full((max(rows, 1),), -9, dtype=torch.int32, device=dev) if blocked else None
            kern.dispatch_slots(recv, layout, N, r, epr, bc, meta, inv=inv)
        else:
            meta[:, 2:] = -1
            rows = N
        x0 = ranks[0][0]
        rx = torch.zeros((rows, x0.shape[1]), dtype=x0.dtype, device=dev)
        rsf = torch.zeros((rows, ranks[0][1].shape[1]), dtype=torch.float32, device=dev) if fp8 else None
        rw = torch.zeros((rows,) if expanded else (N, K), dtype=torch.float32, device=dev)
        kern.dispatch_copy(recv, layout, N, meta, expanded, rx.view(torch.uint8),
                           rsf.view(torch.uint8) if rsf is not None else None, rw,
                           x_direct=sends[r][4] if direct else None, sf_direct=sends[r][5] if direct else None,
                           num_max_tokens=T_max, inv=inv, block_offsets=bc if inv is not None else None,
                           expert_end=pe if inv is not None else None)
        outs.append(dict(meta=meta.cpu(), ridx=None if ridx is None else ridx.cpu(), ec=ec.cpu(), pe=pe.cpu(),
                         rx=rx.cpu(), rsf=None if rsf is None else rsf.cpu(), rw=rw.cpu(), dst=sends[r][0],
                         cnt=sends[r][1],
                         notify_ec=sum(sends[s][6][r * epr:(r + 1) * epr] for s in range(R))))
    return outs


@pytest.mark.parametrize('R,K,E,T,H,expanded,alignment,fp8,masked,skew', [
    (1, 8, 64, 300, 7168, True, 1, False, 0.1, False),
    (1, 2, 8, 128, 1024, False, 1, False, 0.1, False),
    (4, 2, 16, 96, 512, True, 128, False, 0.15, False),
    (8, 8, 64, 200, 256, True, 1, True, 0.1, False),
    (8, 8, 256, 600, 7168, False, 1, False, 0.0, True),
    (3, 6, 24, 257, 128, True, 4, False, 0.2, True),
])
def test_dispatch_primitives_match_cpu(hip, R, K, E, T, H, expanded, alignment, fp8, masked, skew):
    from workloads import per_token_cast_to_fp8
    gen = torch.Generator().manual_seed(R * 1000 + K)
    ranks = []
    for r in range(R):
        idx, w = _routing(T - r, E, K, R, masked, skew, gen)
        x = torch.randn((T - r, H), generator=gen).to(torch.bfloat16)
        sf = None
        if fp8:
            x, sf = per_token_cast_to_fp8(x)
        ranks.append((x, sf, idx, w))
    got = _run_dispatch(hip, 'cuda', ranks, E, K, H, T, expanded, alignment, fp8)
    exp = _run_dispatch(OracleKernels(), 'cpu', ranks, E, K, H, T, expanded, alignment, fp8)
    # the source-major copy (no inverse map) gives the same rows as the blocked destination-major one
    src_major = _run_dispatch(hip, 'cuda', ranks, E, K, H, T, expanded, alignment, fp8, blocked=False)
    for r in range(R):
        assert torch.equal(got[r]['rx'].view(torch.uint8), src_major[r]['rx'].view(torch.uint8)), f'rank {r} copies'
        assert torch.equal(got[r]['rw'], src_major[r]['rw'])
        if fp8:
            assert torch.equal(got[r]['rsf'], src_major[r]['rsf'])
    for r in range(R):
        g, e = got[r], exp[r]
        assert torch.equal(g['dst'], e['dst']) and g['cnt'] == e['cnt'], f'rank {r} route'
        assert torch.equal(g['meta'], e['meta']), f'rank {r} recv_src_metadata'
        if not expanded:
            assert torch.equal(g['ridx'], e['ridx']), f'rank {r} recv_topk_idx'
        assert torch.equal(g['ec'], e['ec']) and torch.equal(g['pe'], e['pe']), f'rank {r} expert counts'
        # the notify histogram (senders' slices for rank r) predicts the receive side's counts
        assert torch.equal(g['notify_ec'], g['ec']) and torch.equal(e['notify_ec'], e['ec']), f'rank {r} notify'
        assert torch.equal(g['rx'].view(torch.uint8), e['rx'].view(torch.uint8)), f'rank {r} recv_x'
        assert torch.equal(g['rw'], e['rw']), f'rank {r} weights'
        if fp8:
            assert torch.equal(g['rsf'], e['rsf']), f'rank {r} scale factors'


@pytest.mark.parametrize('K,E,T,H,expanded,fp8', [
    (8, 64, 300, 7168, True, False),
    (2, 8, 128, 1024, False, False),
    (8, 32, 257, 512, True, True),
    (4, 16, 200, 256, False, True),
])
def test_dispatch_direct_copy_one_rank(hip, K, E, T, H, expanded, fp8):
    """One rank: the metadata-only pack + direct copy gives the same handle and rows as the packed path."""
    from workloads import per_token_cast_to_fp8
    gen = torch.Generator().manual_seed(K * 100 + T)
    idx, w = _routing(T, E, K, 1, 0.1, False, gen)
    x = torch.randn((T, H), generator=gen).to(torch.bfloat16)
    sf = None
    if fp8:
        x, sf = per_token_cast_to_fp8(x)
    ranks = [(x, sf, idx, w)]
    got = _run_dispatch(hip, 'cuda', ranks, E, K, H, T, expanded, 1, fp8, direct=True)[0]
    exp = _run_dispatch(OracleKernels(), 'cpu', ranks, E, K, H, T, expanded, 1, fp8)[0]
    assert torch.equal(got['meta'], exp['meta'])
    assert torch.equal(got['rx'].view(torch.uint8), exp['rx'].view(torch.uint8))
    assert torch.equal(got['rw'], exp['rw'])
    if fp8:
        assert torch.equal(got['rsf'], exp['rsf'])


@pytest.mark.parametrize('alignment,do_cpu_sync,do_handle_copy,fp8,t_max_extra', [
    (1, True, True, False, 0), (128, True, False, False, 0), (4, False, True, False, 0), (1, True, True, True, 0),
    (1, False, False, True, 0), (128, False, True, False, 0), (1, False, True, False, 300),
    (4, False, True, True, 300), (1, True, True, False, 300)])
def test_dispatch_modes_on_gpu(alignment, do_cpu_sync, do_handle_copy, fp8, t_max_extra):
    """ElasticBuffer.dispatch modes with the HIP kernels (EP = 1): cached, cached expanded with zero
    padding, handle copy, deterministic repeat, the per-expert counter, no CPU sync
    (tests/elastic/test_ep.py:143-177, 355-466).  t_max_extra > 0: num_max_tokens_per_rank above the
    batch, so the worst-case tables of a no-CPU-sync handle have more 128-row blocks than the batch
    (a cached dispatch must reuse them)."""
    import os
    import torch.distributed as dist
    from deepep_amd import ElasticBuffer
    from workloads import per_token_cast_to_fp8
    from tests.helpers import dispatch_mode_checks
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29544')
        dist.init_process_group('gloo', rank=0, world_size=1)
    T, H, K, E = 1000, 2048, 8, 64
    g = torch.Generator(device='cuda').manual_seed(alignment + 7)
    scores = torch.rand((T, E), device='cuda', generator=g)
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    idx[torch.rand(idx.shape, device='cuda', generator=g) < 0.1] = -1
    idx[0] = -1                                            # tokens routed nowhere: fewer rows received than T
    idx[T - 300] = -1
    w = w.masked_fill(idx < 0, 0)
    x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
    if fp8:
        x = per_token_cast_to_fp8(x)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T + t_max_extra, hidden=H, num_topk=K)
    fails = dispatch_mode_checks(buf, x, idx, w, E, T + t_max_extra, alignment, do_cpu_sync, do_handle_copy)
    assert not fails, fails


@pytest.mark.parametrize('R,K,E,T,T_max,masked', [
    (1, 8, 256, 8192, 8192, 0.0),          # config 2's send side
    (1, 2, 8, 1, 128, 0.5),
    (1, 16, 64, 3000, 4096, 0.1),
    (8, 8, 256, 8192, 8192, 0.05),         # config 3's
    (8, 8, 256, 5000, 16384, 0.0),         # blocks past the batch hold zeros
    (2, 3, 6, 1025, 1100, 0.3),
    (64, 4, 128, 700, 700, 0.1),
    (4, 8, 32, 0, 256, 0.0),               # an empty batch
    (3, 6, 24, 32768, 32768, 0.2),
    (8, 32, 256, 4000, 4096, 0.1),         # top-32
])
def test_dispatch_notify_matches_multi_launch_send_side(hip, R, K, E, T, T_max, masked):
    """deepep_dispatch_notify (two launches) == route + expert counts + block counts + prefix, bitwise,
    and the count kernel's counts mode (prefix formed in the kernel, psum_out) == its prefix-sum mode."""
    from deepep_amd.handle import chunk_geometry
    gen = torch.Generator().manual_seed(T + R * 7 + K)
    idx, _ = _routing(T, E, K, R, masked, False, gen) if T else (torch.zeros((0, K), dtype=torch.int64), None)
    idx = idx.cuda().contiguous()
    nb = chunk_geometry(T_max, 1)[0] if R > 1 else 0
    epr = E // R
    W = 1 + epr + 2 * nb
    dst = torch.full((T, R), -5, dtype=torch.int32, device='cuda')
    notify = torch.full((R, W), -5, dtype=torch.int32, device='cuda')
    offs = torch.full((R,), -5, dtype=torch.int32, device='cuda')
    hip.dispatch_notify(idx, E, R, nb, dst, notify, offs)
    dst_ref = torch.empty((T, R), dtype=torch.int32, device='cuda')
    cnt = torch.empty((R,), dtype=torch.int32, device='cuda')
    hist = torch.empty((E,), dtype=torch.int32, device='cuda')
    if T:
        hip.dispatch_route(idx, E, R, dst_ref, cnt)
    else:
        cnt.zero_()
    hip.dispatch_expert_counts(idx, E, hist)
    ref = [cnt.view(R, 1), hist.view(R, epr)]
    if nb:
        tok = torch.empty((R, nb), dtype=torch.int32, device='cuda')
        pairs = torch.empty((R, nb), dtype=torch.int32, device='cuda')
        hip.route_block_counts(idx, E, R, nb, tok, pairs)
        ref += [tok, pairs]
    torch.cuda.synchronize()
    assert torch.equal(dst, dst_ref), 'dst_slot'
    assert torch.equal(notify, torch.cat(ref, dim=1)), 'notify record'
    assert torch.equal(offs, (torch.cumsum(cnt, 0) - cnt).to(torch.int32)), 'send offsets'
    # count kernel fed with the notify column (strided counts) == fed with the host-formed prefix
    from deepep_amd._lib import DISPATCH_BLOCK_ROWS
    from deepep_amd.kernels import RowLayout
    layout = RowLayout.make(0, 0, K)
    n = int(cnt.sum())
    packed = torch.zeros((max(n, 1), layout.row_bytes), dtype=torch.uint8, device='cuda')
    if n:
        hip.dispatch_pack(torch.empty((T, 16), dtype=torch.uint8, device='cuda')[:, :0], None, idx, None, 0, dst, offs, packed,
                          layout)
    outs = []
    for mode in ('psum', 'counts'):
        meta = torch.full((n, K + 2), -3, dtype=torch.int32, device='cuda')
        bc = torch.full(((n + DISPATCH_BLOCK_ROWS - 1) // DISPATCH_BLOCK_ROWS, epr), -3, dtype=torch.int32,
                        device='cuda')
        psum_out = torch.full((R,), -3, dtype=torch.int32, device='cuda')
        if mode == 'psum':
            hip.dispatch_count(packed, layout, n, 0, epr, torch.cumsum(cnt, 0).to(torch.int32), meta, None, bc)
            psum_out = torch.cumsum(cnt, 0).to(torch.int32)
        else:
            hip.dispatch_count(packed, layout, n, 0, epr, None, meta, None, bc, rank_counts=notify[:, 0],
                               psum_out=psum_out)
        torch.cuda.synchronize()
        outs.append((meta, bc, psum_out))
    for a, b in zip(*outs):
        assert torch.equal(a, b), 'count kernel: counts mode differs from psum mode'
