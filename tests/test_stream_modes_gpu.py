"""The stream modes of the reference test (tests/elastic/test_ep.py:22-41): with / without
previous_event, async_with_compute_stream, allocate_on_comm_stream (and
previous_event_before_epilogue), for dispatch and combine, on the GPU.  Every mode must give the
sync-mode bits.  The inputs are produced on the compute stream right before each call, so a
missing stream dependency would read stale data, and the outputs are overwritten on the compute
stream right after the (awaited) call.  EP = 1 on the real device and EP = 4 with ranks simulated by
threads (the pipelined multi-chunk path, whose phase B runs on a second stream)."""
import os
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _modes():
    """enumerate_ep_modes' stream axes (test_ep.py:22-31) plus a previous_event_before_epilogue."""
    for with_previous_event in (0, 1):
        for async_with_compute_stream in (0, 1):
            for allocate_on_comm_stream in ((1,) if with_previous_event else (0, 1)):
                yield with_previous_event, async_with_compute_stream, allocate_on_comm_stream, 0
    yield 0, 1, 0, 1
    yield 1, 1, 1, 1


def _launch(buf, name, with_previous_event, async_with_compute_stream, before_epilogue, params):
    """test_ep.py:34-41: capture the previous event, call, wait on the returned event if async."""
    if with_previous_event:
        params['previous_event'] = buf.capture()
    if before_epilogue:
        params['previous_event_before_epilogue'] = buf.capture()
    values = getattr(buf, name)(**params)
    hooked = []
    if async_with_compute_stream:
        values[-1].register_hook_after_wait(lambda: hooked.append(1))
        values[-1].current_stream_wait()
        assert hooked == [1]
    return values


def _run_modes(buf, x_src, idx, w, E, T, H, tag):
    """All modes for one buffer; returns the list of mismatches."""
    fails = []
    biases = [torch.randn((T, H), device='cuda').to(torch.bfloat16) for _ in range(2)]

    def fresh(t):
        # produced on the compute stream right before the call (a slow multiply chain, so a
        # comm-stream kernel that does not wait reads unfinished data)
        out = t
        for _ in range(3):
            out = out * 1
        return out

    ref = {}
    for mode in [(0, 0, 0, 0)] + list(_modes()):
        prev, asyn, alloc, before = mode
        common = dict(async_with_compute_stream=bool(asyn), allocate_on_comm_stream=bool(alloc))
        recv_x, recv_idx, recv_w, handle, _ = _launch(
            buf, 'dispatch', prev, asyn, 0, dict(x=fresh(x_src), topk_idx=idx, topk_weights=w, num_experts=E,
                                                 **common))
        ex_x, _, ex_w, ex_handle, _ = _launch(
            buf, 'dispatch', prev, asyn, 0, dict(x=fresh(x_src), topk_idx=idx, topk_weights=w, num_experts=E,
                                                 do_expand=True, **common))
        got = {'recv_x': recv_x.clone(), 'ex_x': ex_x.clone(), 'recv_w': recv_w.clone(), 'ex_w': ex_w.clone()}
        g = torch.Generator(device='cuda').manual_seed(7)
        y_red = torch.randn((handle.num_recv_tokens, H), device='cuda', generator=g).to(torch.bfloat16)
        y_exp = torch.randn(ex_x.shape, device='cuda', generator=g).to(torch.bfloat16)
        for nb in (0, 1, 2):
            bias = None if nb == 0 else (fresh(biases[0]) if nb == 1 else (fresh(biases[0]), fresh(biases[1])))
            out, out_w, _ = _launch(buf, 'combine', prev, asyn, before,
                                    dict(x=fresh(y_red), handle=handle, topk_weights=recv_w, bias=bias, **common))
            got[f'combine_b{nb}'], got[f'combine_w_b{nb}'] = out.clone(), out_w.clone()
            out.fill_(0)                                   # the caller reuses the memory right away
            out, out_w, _ = _launch(buf, 'combine', prev, asyn, before,
                                    dict(x=fresh(y_exp), handle=ex_handle, topk_weights=ex_w, bias=bias, **common))
            got[f'expanded_b{nb}'], got[f'expanded_w_b{nb}'] = out.clone(), out_w.clone()
            out.fill_(0)
        out, _, _ = _launch(buf, 'combine', prev, asyn, before,
                            dict(x=fresh(y_exp), handle=ex_handle, topk_weights=ex_w, apply_topk_weights=True,
                                 **common))
        got['weighted'] = out.clone()
        # an explicit num_sms below the CU count: the kernels run on a CU-budget stream
        for cus in (40, 100):
            out, out_w, _ = _launch(buf, 'combine', prev, asyn, before,
                                    dict(x=fresh(y_exp), handle=ex_handle, topk_weights=ex_w, num_sms=cus, **common))
            got[f'budget{cus}'], got[f'budget{cus}_w'] = out.clone(), out_w.clone()
            out.fill_(0)
        torch.cuda.synchronize()
        if mode == (0, 0, 0, 0):
            ref = got
            for cus in (40, 100):
                if not (torch.equal(got[f'budget{cus}'], got['expanded_b0']) and
                        torch.equal(got[f'budget{cus}_w'], got['expanded_w_b0'])):
                    fails.append(f'{tag}: num_sms={cus} differs from the whole-chip combine')
            continue
        for k, v in got.items():
            if not torch.equal(v, ref[k]):
                fails.append(f'{tag} mode {mode}: {k}')
    return fails


def _inputs(T, H, K, E, seed):
    g = torch.Generator(device='cuda').manual_seed(seed)
    w, idx = torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    idx[torch.rand(idx.shape, device='cuda', generator=g) < 0.1] = -1
    w = w.masked_fill(idx < 0, 0)
    x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
    return x, idx, w


@pytest.mark.parametrize('avoid_record_stream', [0, 1])
def test_stream_modes_ep1(monkeypatch, avoid_record_stream):
    """avoid_record_stream: EP_AVOID_RECORD_STREAM=1 (event.py:17-30), the async tensors are kept
    alive by the returned event instead of record_stream."""
    monkeypatch.setenv('EP_AVOID_RECORD_STREAM', str(avoid_record_stream))
    import torch.distributed as dist
    from deepep_amd import ElasticBuffer
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29551')
        dist.init_process_group('gloo', rank=0, world_size=1)
    T, H, K, E = 777, 2048, 8, 64
    x, idx, w = _inputs(T, H, K, E, 1)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    fails = _run_modes(buf, x, idx, w, E, T, H, 'ep1')
    assert not fails, fails


def _sim_rank(rank, world, comm, results):
    try:
        from deepep_amd import ElasticBuffer
        from tests.sim import FakeGroup as _FakeGroup
        torch.cuda.set_device(0)
        T, H, K, E = 1100, 1024, 8, 32
        x, idx, w = _inputs(T, H, K, E, 100 + rank)
        buf = ElasticBuffer(_FakeGroup(rank, world, comm), num_max_tokens_per_rank=T, hidden=H, num_topk=K)
        comm.install(buf, rank)
        results[rank] = _run_modes(buf, x, idx, w, E, T, H, f'ep{world} rank {rank}')
    except Exception:
        import traceback
        results[rank] = [traceback.format_exc()]
        comm.bar.abort()


def test_stream_modes_ep4_pipelined(monkeypatch):
    """EP = 4, 1100 tokens per rank -> the 4-chunk pipelined exchange (phase B on a second stream)."""
    from tests.sim import ThreadComm as _ThreadComm
    monkeypatch.setenv('DEEPEP_COMBINE_CHUNKS', '4')
    world = 4
    comm = _ThreadComm(world)
    results = {}
    threads = [threading.Thread(target=_sim_rank, args=(r, world, comm, results)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=160)
    assert len(results) == world, results
    bad = {r: f for r, f in results.items() if f}
    assert not bad, bad


@pytest.mark.parametrize('num_sms,expect_cus', [(4, 8), (8, 8), (12, 16), (64, 64)])
def test_cu_budget_is_honoured_and_bitwise(num_sms, expect_cus):
    """An explicit num_sms is rounded up to whole CUs per XCD (a CU mask without bits on an XCD would
    leave that XCD unrestricted): the budget stream's workgroups run on exactly that many CUs, spread
    over all 8 XCDs; the combine on it -- from the default stream, and issued from the budget stream
    itself (no stream hops) -- is bitwise the whole-chip combine; so is a dispatch with that num_sms."""
    import ctypes
    import torch.distributed as dist
    from deepep_amd import ElasticBuffer
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29563')
        dist.init_process_group('gloo', rank=0, world_size=1)
    T, H, K, E = 512, 2048, 8, 64
    g = torch.Generator(device='cuda').manual_seed(num_sms)
    w, idx = torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1, sorted=False)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                         topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda', generator=g).to(torch.bfloat16)
    ref, ref_w, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
    bs = buf.get_cu_budget_stream(num_sms)
    n, x = ctypes.c_int(), ctypes.c_int()
    assert buf.kernels.lib.deepep_stream_probe_cus(ctypes.c_void_p(bs.cuda_stream), ctypes.byref(n), ctypes.byref(x)) == 0
    assert (n.value, x.value) == (expect_cus, 8), (n.value, x.value)
    out, out_w, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True, num_sms=num_sms)
    with torch.cuda.stream(bs):
        out2, out2_w, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True, num_sms=num_sms)
    torch.cuda.synchronize()
    assert torch.equal(out, ref) and torch.equal(out_w, ref_w)
    assert torch.equal(out2, ref) and torch.equal(out2_w, ref_w)
    # the dispatch honours an explicit num_sms the same way (the reference sizes its dispatch grids with it):
    # fresh and cached, bitwise the whole-chip dispatch
    x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
    args = dict(topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E, do_expand=True)
    rx, _, rw, rh, _ = buf.dispatch(x, **args)
    bx, _, bw, bh, _ = buf.dispatch(x, num_sms=num_sms, **args)
    cx, _, cw, _, _ = buf.dispatch(x, topk_weights=w, do_expand=True, handle=rh, num_sms=num_sms)
    torch.cuda.synchronize()
    assert torch.equal(bx, rx) and torch.equal(bw, rw) and torch.equal(bh.recv_src_metadata, rh.recv_src_metadata)
    assert torch.equal(cx, rx) and torch.equal(cw, rw)


@pytest.mark.parametrize('world', [1, 4])
def test_reference_cu_confined_default_is_bitwise(monkeypatch, world):
    """DEEPEP_COMBINE_CUS=handle: a combine called with num_sms=0 runs on a stream confined to the
    handle's num_sms (the reference's bandwidth-model default, elastic.py:1086 -> combine_impl's grid,
    combine.hpp:135), bitwise equal to the whole-chip default.  EP = 1's model value is the whole
    chip, so the handle's value is lowered to 16 there; EP = 4 keeps the model's value."""
    from deepep_amd import ElasticBuffer
    from tests.sim import FakeGroup, ThreadComm
    import torch.distributed as dist
    T, H, K, E = 256, 1024, 8, 64
    monkeypatch.setenv('DEEPEP_COMBINE_CUS', 'bogus')
    if world == 1:
        if not dist.is_initialized():
            os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
            os.environ.setdefault('MASTER_PORT', '29567')
            dist.init_process_group('gloo', rank=0, world_size=1)
        with pytest.raises(RuntimeError):
            ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    monkeypatch.setenv('DEEPEP_COMBINE_CUS', 'handle')
    comm = ThreadComm(world) if world > 1 else None
    if world == 1 and not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29567')
        dist.init_process_group('gloo', rank=0, world_size=1)
    results = {}

    def rank_fn(rank):
        try:
            torch.cuda.set_device(0)
            g = torch.Generator(device='cuda').manual_seed(100 + rank)
            w, idx = torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1, sorted=False)
            grp = FakeGroup(rank, world, comm) if world > 1 else dist.group.WORLD
            bufs = {}
            for mode in ('chip', 'handle'):
                bufs[mode] = ElasticBuffer(grp, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
                bufs[mode].combine_cu_mode = mode          # what DEEPEP_COMBINE_CUS sets at construction
                if comm is not None:
                    comm.install(bufs[mode], rank)
            _, _, ex_w, handle, _ = bufs['chip'].dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                                         topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E,
                                                         do_expand=True)
            if world == 1:
                handle.num_sms = 16
            y = torch.randn((handle.num_expanded_tokens, H), device='cuda', generator=g).to(torch.bfloat16)
            outs = {m: b.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True) for m, b in bufs.items()}
            torch.cuda.synchronize()
            fails = []
            if not (torch.equal(outs['chip'][0], outs['handle'][0]) and torch.equal(outs['chip'][1], outs['handle'][1])):
                fails.append('confined combine differs')
            cus = torch.cuda.get_device_properties(0).multi_processor_count
            if handle.num_sms < cus and bufs['handle']._cu_budget_stream(handle.num_sms) is None:
                fails.append('no budget stream for the handle num_sms')
            results[rank] = fails
        except Exception:
            import traceback
            results[rank] = [traceback.format_exc()]
            if comm is not None:
                comm.bar.abort()

    threads = [threading.Thread(target=rank_fn, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=160)
    assert len(results) == world and not any(results.values()), results
