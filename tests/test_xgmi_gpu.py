"""The xGMI transport (symmetric windows + device barrier, deepep_amd/symmetric.py) on the GPU.

World-size 2 and 4 run as separate processes sharing the box's one GPU: every rank opens its
peers' windows through HIP IPC, phase A stores partial rows straight into the owners' windows
and the device barrier orders the phases -- the same code path as on an 8-GPU node, with the
peer stores landing in the same HBM instead of crossing xGMI.  Results are compared bitwise with
oracle.combine_ep (the CPU restatement pinned to refs.combine) and with the RCCL-path combine.
"""
import os
import socket
import sys
import traceback

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _u16(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _bf16(a: np.ndarray, dev) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16).to(dev)


def _worker(rank, world, port, seed, T, H, K, queue, empty_rank=-1, chunks=0):
    sys.path.insert(0, ROOT)
    try:
        if chunks:
            os.environ['DEEPEP_COMBINE_CHUNKS'] = str(chunks)
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        import oracle
        from deepep_amd import ElasticBuffer
        dev = torch.device('cuda', 0)
        E = 8 * world
        rng = np.random.default_rng(seed)
        idx_all, w_all, y_all, b_all = [], [], [], []
        Ts = [0 if r == empty_rank else T for r in range(world)]     # empty_rank sends no tokens
        for r in range(world):
            Tr = Ts[r]
            idx = np.array([rng.permutation(E)[:K] for _ in range(Tr)], dtype=np.int64).reshape(Tr, K)
            idx[rng.random((Tr, K)) < 0.15] = -1
            if Tr:
                idx[0] = -1                               # a token routed nowhere
            w = rng.random((Tr, K)).astype(np.float32) * (idx >= 0)
            y = oracle.f32_to_bf16(rng.standard_normal((Tr, K, H)).astype(np.float32))
            y[idx < 0] = 0
            idx_all.append(idx), w_all.append(w), y_all.append(y)
            b_all.append(oracle.f32_to_bf16(rng.standard_normal((Tr, H)).astype(np.float32)))
        disp = oracle.simulate_dispatch(idx_all, E, T)
        x_exp_all, w_exp_all = [], []
        for r, d in enumerate(disp):
            xe = np.zeros((d['num_expanded'], H), np.uint16)
            we = np.zeros((d['num_expanded'],), np.float32)
            for row, (g, k) in enumerate(d['expanded_src']):
                s, t = divmod(int(g), T)
                xe[row], we[row] = y_all[s][t, k], w_all[s][t, k]
            x_exp_all.append(xe), w_exp_all.append(we)
        failures = []
        bufs = {}
        for transport in ('xgmi', 'rccl'):
            os.environ['DEEPEP_TRANSPORT'] = transport
            bufs[transport] = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                                            explicitly_destroy=True, num_gpu_timeout_secs=20)
        # dispatch over xGMI (rows pushed into the peers' windows) == dispatch over RCCL, bit for bit:
        # bf16 and fp8 + scale-factor payloads, reduced / expanded layouts, fresh and cached handles
        idx_t, w_t = torch.from_numpy(idx_all[rank]).to(dev), torch.from_numpy(w_all[rank]).to(dev)

        def as_bytes(v):
            if isinstance(v, tuple):
                return [as_bytes(u) for u in v]
            return None if v is None else v.contiguous().view(torch.uint8).cpu()

        def same(a, b):
            a, b = as_bytes(a), as_bytes(b)
            if isinstance(a, list):
                return all(same(u, v) for u, v in zip(a, b))
            return (a is None and b is None) or (a is not None and b is not None and torch.equal(a, b))

        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        payloads = []
        for _ in range(2):
            xb = torch.randn((Ts[rank], H), device=dev, generator=g).to(torch.bfloat16)
            x8 = torch.randn((Ts[rank], H), device=dev, generator=g).to(torch.float8_e4m3fn)
            sf = torch.rand((Ts[rank], H // 128), device=dev, generator=g)
            payloads.append((xb, (x8, sf)))
        for kind in (0, 1):
            for do_expand in (False, True):
                res = {t: b.dispatch(payloads[0][kind], topk_idx=idx_t, topk_weights=w_t, num_experts=E,
                                     do_expand=do_expand) for t, b in bufs.items()}
                cached = {t: b.dispatch(payloads[1][kind], handle=res[t][3], do_expand=do_expand) for t, b in bufs.items()}
                for tag, got in (('fresh', res), ('cached', cached)):
                    a, b = got['xgmi'], got['rccl']
                    for i, name in enumerate(('recv_x', 'recv_topk_idx', 'recv_topk_weights')):
                        if not same(a[i], b[i]):
                            failures.append(f'dispatch {tag} kind {kind} expand {do_expand}: {name} xgmi != rccl')
                    ha, hb = a[3], b[3]
                    for name in ('recv_src_metadata', 'psum_num_recv_tokens_per_scaleup_rank',
                                 'psum_num_recv_tokens_per_expert', 'num_unaligned_recv_tokens_per_expert'):
                        if not same(getattr(ha, name), getattr(hb, name)):
                            failures.append(f'dispatch {tag} kind {kind} expand {do_expand}: {name} xgmi != rccl')
                    if ha.num_recv_tokens_per_expert_list != hb.num_recv_tokens_per_expert_list:
                        failures.append(f'dispatch {tag} kind {kind} expand {do_expand}: expert list')
                # a cached-handle xGMI dispatch (no host sync) captured into a HIP graph, replayed
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    g_res = bufs['xgmi'].dispatch(payloads[1][kind], handle=res['xgmi'][3], do_expand=do_expand)
                for it in range(2):
                    graph.replay()
                    torch.cuda.synchronize()
                    if not all(same(g_res[i], cached['xgmi'][i]) for i in (0, 2)):
                        failures.append(f'dispatch graph replay {it} kind {kind} expand {do_expand}')
                del graph, g_res
        if bufs['xgmi']._sym is None:
            failures.append('xgmi dispatch did not create its window')
        x = torch.zeros((Ts[rank], H), dtype=torch.bfloat16, device=dev)
        buf = bufs['xgmi']
        _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=torch.from_numpy(idx_all[rank]).to(dev),
                                             topk_weights=torch.from_numpy(w_all[rank]).to(dev),
                                             num_experts=E, do_expand=True)
        if not np.array_equal(handle.recv_src_metadata.cpu().numpy(), disp[rank]['src_metadata']):
            failures.append('recv_src_metadata differs from the oracle dispatch')
        for nb in (0, 1):
            expect = oracle.combine_ep(x_exp_all, [d['src_metadata'] for d in disp], idx_all, E, T, expanded=True,
                                       topk_weights_per_rank=w_exp_all,
                                       bias_per_rank=[(b if nb else None, None) for b in b_all])
            bias = _bf16(b_all[rank], dev) if nb else None
            for it in range(3):                           # repeated calls reuse the windows (epochs)
                for transport, b in bufs.items():
                    out, out_w, _ = b.combine(_bf16(x_exp_all[rank], dev), handle, topk_weights=ex_w, bias=bias)
                    torch.cuda.current_stream().synchronize()
                    if not np.array_equal(_u16(out), expect[rank][0]):
                        failures.append(f'{transport} combined_x (bias {nb}, call {it})')
                    if not np.array_equal(out_w.cpu().numpy(), expect[rank][1]):
                        failures.append(f'{transport} combined_topk_weights (bias {nb}, call {it})')
        # phase A on a 64-CU budget stream (DEEPEP_PHASE_A_CUS): same bits
        bufs['xgmi'].phase_a_cus = 64
        out, out_w, _ = bufs['xgmi'].combine(_bf16(x_exp_all[rank], dev), handle, topk_weights=ex_w,
                                             bias=_bf16(b_all[rank], dev))
        torch.cuda.synchronize()
        if not (np.array_equal(_u16(out), expect[rank][0]) and np.array_equal(out_w.cpu().numpy(), expect[rank][1])):
            failures.append('xgmi combine with a phase-A CU budget')
        bufs['xgmi'].phase_a_cus = 0
        # HIP graph: the whole xGMI combine (device barrier, phase A stores into the peers' windows,
        # split signal / wait, phase B) captured once and replayed; the barrier epochs are counted on
        # the device, so every replay -- and eager calls in between -- synchronise correctly
        xb = bufs['xgmi']
        g_in, g_bias = _bf16(x_exp_all[rank], dev), _bf16(b_all[rank], dev)
        xb.combine(g_in, handle, topk_weights=ex_w, bias=g_bias)          # plans cached outside capture
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g_out, g_w, _ = xb.combine(g_in, handle, topk_weights=ex_w, bias=g_bias)
        for it in range(4):
            g_out.zero_()
            graph.replay()
            torch.cuda.synchronize()
            if not (np.array_equal(_u16(g_out), expect[rank][0]) and np.array_equal(g_w.cpu().numpy(), expect[rank][1])):
                failures.append(f'xgmi combine graph replay {it}')
            if it == 1:                                                  # an eager call between replays
                out, _, _ = xb.combine(g_in, handle, topk_weights=ex_w, bias=g_bias)
                torch.cuda.synchronize()
                if not np.array_equal(_u16(out), expect[rank][0]):
                    failures.append('xgmi eager combine between graph replays')
        xb._sym.check()
        del graph
        # An async combine (comm stream) followed at once by a sync-mode combine on the caller's stream
        # with other inputs, no wait on the first call's event: both use the one window, so the second
        # call's barrier must not pass before the first call's phase B has read it.
        x2_all = [oracle.f32_to_bf16(oracle.bf16_to_f32(v) * 2) for v in x_exp_all]
        expect2 = oracle.combine_ep(x2_all, [d['src_metadata'] for d in disp], idx_all, E, T, expanded=True,
                                    topk_weights_per_rank=w_exp_all, bias_per_rank=[(b, None) for b in b_all])
        g_in2 = _bf16(x2_all[rank], dev)
        for it in range(2):
            a_out, a_w, ev = xb.combine(g_in, handle, topk_weights=ex_w, bias=g_bias, async_with_compute_stream=True)
            s_out, s_w, _ = xb.combine(g_in2, handle, topk_weights=ex_w, bias=g_bias)
            ev.current_stream_wait()
            torch.cuda.synchronize()
            if not np.array_equal(_u16(a_out), expect[rank][0]):
                failures.append(f'async xgmi combine overtaken by the next sync call ({it})')
            if not np.array_equal(_u16(s_out), expect2[rank][0]):
                failures.append(f'sync xgmi combine after an async one ({it})')
        # A timed-out barrier poisons the launches behind it (bit 2 of the window's error flag): no
        # partial reaches a peer and the output is NaN, not a silently wrong sum; the next call raises.
        torch.cuda.synchronize()
        xb._sym.error_flag.fill_(2)
        p_out, _, _ = xb.combine(g_in, handle, topk_weights=ex_w, bias=g_bias)
        torch.cuda.synchronize()
        if not bool(torch.isnan(p_out.float()).all()):
            failures.append('combine after a timed-out barrier is not poisoned')
        xb._sym.error_flag.zero_()
        try:
            xb.combine(g_in, handle, topk_weights=ex_w, bias=g_bias)
            failures.append('the call after a timed-out barrier did not raise')
        except RuntimeError as e:
            if 'did not arrive' not in str(e):
                raise
        out, _, _ = xb.combine(g_in, handle, topk_weights=ex_w, bias=g_bias)        # usable again
        torch.cuda.synchronize()
        if not np.array_equal(_u16(out), expect[rank][0]):
            failures.append('xgmi combine after the poisoned call')
        # A corrupted plan entry (a window row address pointing into local memory outside every window):
        # phase A stores nothing through it, the window's error record names the unit and the address, and
        # the host raises.  Every rank corrupts one unit, so every rank's check sees it at the same call.
        key = [k for k in handle._combine_plans if k[0] == 'xgmi' and not k[1] and k[-1] == xb._sym_gen]
        chunk = next((ch for ch in handle._combine_plans[key[0]].chunks if ch.out_rows.numel()), None) if key else None
        if chunk is None:
            failures.append(f'no cached xgmi plan with units to corrupt (keys {list(handle._combine_plans)})')
        else:
            canary = torch.zeros((4 << 20,), dtype=torch.uint8, device=dev)
            saved = chunk.out_rows[0].clone()
            chunk.out_rows[0] = canary.data_ptr() + (1 << 20)
            xb.combine(g_in, handle, topk_weights=ex_w, bias=g_bias)
            torch.cuda.synchronize()
            chunk.out_rows[0] = saved
            rec = xb._sym.error_record.tolist()
            if int(canary.count_nonzero()) != 0:
                failures.append('a phase-A store escaped through a corrupted window address')
            addr = (rec[5] & 0xffffffff) << 32 | (rec[4] & 0xffffffff)
            if not (rec[0] & 4 and rec[1] == 1 and addr == canary.data_ptr() + (1 << 20)):
                failures.append(f'corrupted window address not recorded: {rec}')
            try:
                xb._sym.check()
                failures.append('check() did not raise after a rejected window address')
            except RuntimeError as e:
                if 'outside every window' not in str(e):
                    failures.append(f'unexpected error text: {e}')
            xb._sym.reset_error()
            out, _, _ = xb.combine(g_in, handle, topk_weights=ex_w, bias=g_bias)
            torch.cuda.synchronize()
            if not np.array_equal(_u16(out), expect[rank][0]) or xb._sym.error_record.tolist()[0]:
                failures.append('xgmi combine after the rejected window address')
        # The FIRST combine on a fresh handle captured into a HIP graph, no eager call before it: its
        # plan (window row addresses included) is built by kernels inside the capture.
        _, _, ex_w2, handle2, _ = xb.dispatch(x, topk_idx=torch.from_numpy(idx_all[rank]).to(dev),
                                              topk_weights=torch.from_numpy(w_all[rank]).to(dev),
                                              num_experts=E, do_expand=True)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            f_out, f_w, _ = xb.combine(g_in, handle2, topk_weights=ex_w2, bias=g_bias)
        for it in range(2):
            f_out.zero_()
            graph.replay()
            torch.cuda.synchronize()
            if not (np.array_equal(_u16(f_out), expect[rank][0]) and np.array_equal(f_w.cpu().numpy(), expect[rank][1])):
                failures.append(f'first xgmi combine captured, replay {it}')
        del graph
        xb._sym.check()
        # gating-weighted variant: xGMI and RCCL paths agree bit for bit
        outs = {}
        for transport, b in bufs.items():
            outs[transport], _, _ = b.combine(_bf16(x_exp_all[rank], dev), handle, topk_weights=ex_w,
                                              apply_topk_weights=True)
        if not torch.equal(outs['xgmi'], outs['rccl']):
            failures.append('weighted: xgmi != rccl')
        # non-expanded layout (the caller pre-reduces its local experts): both transports agree
        _, _, recv_w, nh, _ = buf.dispatch(x, topk_idx=torch.from_numpy(idx_all[rank]).to(dev),
                                            topk_weights=torch.from_numpy(w_all[rank]).to(dev), num_experts=E)
        g = torch.Generator(device=dev).manual_seed(rank)
        x_red = torch.randn((nh.num_recv_tokens, H), device=dev, generator=g).to(torch.bfloat16)
        bias = _bf16(b_all[rank], dev)
        o = {t: b.combine(x_red, nh, topk_weights=recv_w, bias=bias) for t, b in bufs.items()}
        if not (torch.equal(o['xgmi'][0], o['rccl'][0]) and torch.equal(o['xgmi'][1], o['rccl'][1])):
            failures.append('non-expanded: xgmi != rccl')
        if not torch.equal(o['xgmi'][1].cpu(), torch.from_numpy(w_all[rank])):
            failures.append('non-expanded: weight pass-through')
        # allow_multiple_reduction=False: every expanded row pushed unreduced into the source rank's
        # window (per-top-k slots), one reduction there -- plain vs the reference oracle, gating-weighted
        # vs the legacy low-latency fma chain (bias in front); both transports
        from tests.test_buffer_cpu import _weighted_single
        sbufs = {}
        # num_bytes just fits the multiple-reduction layout, so the single reduction's K-slot window
        # forces a re-allocation (where K > min(R, K))
        mb = 2 << 20
        multi_bytes = min(world, K) * T * ((2 * H + 15) // 16 * 16 + (4 * K + 15) // 16 * 16)
        for transport in ('xgmi', 'rccl'):
            os.environ['DEEPEP_TRANSPORT'] = transport
            sbufs[transport] = ElasticBuffer(dist.group.WORLD, num_bytes=(multi_bytes + mb - 1) // mb * mb,
                                             num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                                             allow_multiple_reduction=False, explicitly_destroy=True,
                                             num_gpu_timeout_secs=5)
        # the non-expanded handle takes the multiple-reduction path on this buffer too: its window
        # (min(R, K) slots) is outgrown by the expanded single reduction's (K slots) below, so the
        # buffer re-allocates and plans addressing the old window must not be reused
        nb_bias = _bf16(b_all[rank], dev)

        def non_expanded_check(tag):
            r = sbufs['xgmi'].combine(x_red, nh, topk_weights=recv_w, bias=nb_bias)
            if not (torch.equal(r[0], o['rccl'][0]) and torch.equal(r[1], o['rccl'][1])):
                failures.append(f'non-expanded on the single-reduction buffer ({tag})')
        non_expanded_check('before')
        for nb in (0, 1):
            expect = oracle.combine_ep(x_exp_all, [d['src_metadata'] for d in disp], idx_all, E, T, expanded=True,
                                       allow_multiple_reduction=False,
                                       bias_per_rank=[(b if nb else None, None) for b in b_all])
            bias = _bf16(b_all[rank], dev) if nb else None
            bias_cpu = torch.from_numpy(b_all[rank].view(np.int16)).view(torch.bfloat16) if nb else None
            exp_w = _weighted_single(y_all[rank], torch.from_numpy(idx_all[rank]), torch.from_numpy(w_all[rank]),
                                     bias_cpu)
            for it in range(2):
                for transport, b in sbufs.items():
                    out, out_w, _ = b.combine(_bf16(x_exp_all[rank], dev), handle, bias=bias)
                    torch.cuda.current_stream().synchronize()
                    if not np.array_equal(_u16(out), expect[rank][0]) or out_w is not None:
                        failures.append(f'{transport} single-reduction (bias {nb}, call {it})')
                    out, out_w, _ = b.combine(_bf16(x_exp_all[rank], dev), handle, topk_weights=ex_w, bias=bias,
                                              apply_topk_weights=True)
                    torch.cuda.current_stream().synchronize()
                    if os.environ.get('DEEPEP_TEST_TRACE'):
                        flag = int(b._sym.error_flag.item()) if b._sym is not None else -1
                        print(f'rank {rank} {transport} nb={nb} it={it} flag={flag} epoch='
                              f'{b._sym.epoch if b._sym is not None else -1}', file=sys.stderr, flush=True)
                    if not torch.equal(out.cpu(), exp_w):
                        failures.append(f'{transport} single-reduction weighted (bias {nb}, call {it})')
                    if not np.array_equal(out_w.cpu().numpy(), w_all[rank]):
                        failures.append(f'{transport} single-reduction weighted pass-through (bias {nb}, call {it})')
        non_expanded_check('after re-allocation')
        if sbufs['xgmi']._sym is None:
            failures.append('xgmi single-reduction transport did not create its window')
        else:
            sbufs['xgmi']._sym.check()
        for b in sbufs.values():
            b.destroy()
        if bufs['xgmi']._sym is None:
            failures.append('xgmi transport did not create its window')
        else:
            bufs['xgmi']._sym.check()
        for b in bufs.values():
            b.destroy()
        queue.put((rank, failures))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, [traceback.format_exc()]))


@pytest.mark.parametrize('world,T,H,K,empty_rank,chunks', [
    (2, 96, 1024, 8, -1, 0), (4, 64, 7168, 8, -1, 0), (4, 80, 256, 2, -1, 0), (3, 40, 512, 4, 1, 0),
    (2, 96, 1024, 8, -1, 3), (4, 80, 256, 2, -1, 5), (3, 40, 512, 4, 1, 4),
    (8, 48, 512, 8, -1, 2)])                                  # the node's full EP = 8 (8 processes)
def test_xgmi_transport_matches_oracle(world, T, H, K, empty_rank, chunks):
    """chunks > 0: the pipelined schedule (phase A per source-token chunk + split barrier, phase B
    of each chunk on a second stream)."""
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 100 + world + K, T, H, K, queue, empty_rank, chunks))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, failures = queue.get(timeout=150)
            results[rank] = failures
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    if len(results) != world or any(results.values()):
        # the root cause is usually one rank's exception; its peers then fail with a closed connection
        tails = {r: [f[-1500:] for f in fl] for r, fl in results.items()}
        pytest.fail(f'{len(results)}/{world} ranks reported; failures: {tails}', pytrace=False)


def _sync_free_worker(rank, world, port, T, H, K, chunks, queue):
    """dispatch(do_cpu_sync=False) + the handle's first combine over xGMI, with no host sync: the notify
    goes through the windows, every launch is sized for the worst case and bounded on the device, the
    combine plan is worst-case padded.  Run under set_sync_debug_mode('error') and, on a second buffer,
    captured whole into one HIP graph (no eager call before it) and replayed; bitwise vs the oracle."""
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        os.environ['DEEPEP_TRANSPORT'] = 'xgmi'
        if chunks:
            os.environ['DEEPEP_COMBINE_CHUNKS'] = str(chunks)
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        import oracle
        from deepep_amd import ElasticBuffer
        dev = torch.device('cuda', 0)
        E = 8 * world
        rng = np.random.default_rng(700 + world)
        idx_all = []
        for r in range(world):
            idx = np.array([rng.permutation(E)[:K] for _ in range(T)], dtype=np.int64).reshape(T, K)
            idx[rng.random((T, K)) < 0.15] = -1
            idx[0] = -1                                   # a token routed nowhere
            idx_all.append(idx)
        w_all = [rng.random((T, K)).astype(np.float32) * (i >= 0) for i in idx_all]
        x_all = [oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)) for _ in range(world)]
        b_all = [oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)) for _ in range(world)]
        disp = oracle.simulate_dispatch(idx_all, E, T)
        # the combine reduces the dispatched rows themselves (expert outputs = their inputs)
        x_exp_all, w_exp_all = [], []
        for d in disp:
            xe = np.zeros((d['num_expanded'], H), np.uint16)
            we = np.zeros((d['num_expanded'],), np.float32)
            for row, (g, k) in enumerate(d['expanded_src']):
                s, t = divmod(int(g), T)
                xe[row], we[row] = x_all[s][t], w_all[s][t, k]
            x_exp_all.append(xe), w_exp_all.append(we)
        expect = oracle.combine_ep(x_exp_all, [d['src_metadata'] for d in disp], idx_all, E, T, expanded=True,
                                   topk_weights_per_rank=w_exp_all,
                                   bias_per_rank=[(b, None) for b in b_all])[rank]
        x, bias = _bf16(x_all[rank], dev), _bf16(b_all[rank], dev)
        idx, w = torch.from_numpy(idx_all[rank]).to(dev), torch.from_numpy(w_all[rank]).to(dev)
        failures = []

        def step(buf):
            ex_x, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True,
                                                    do_cpu_sync=False)
            out, out_w, _ = buf.combine(ex_x, handle, topk_weights=ex_w, bias=bias)
            return out, out_w, handle

        def check(tag, out, out_w, handle):
            n = int(handle.psum_num_recv_tokens_per_scaleup_rank[-1].item())
            meta = handle.recv_src_metadata.cpu().numpy()
            if handle.recv_src_metadata.shape[0] != world * T or not (meta[n:] == -1).all():
                failures.append(f'{tag}: metadata is not worst-case shaped')
            if not np.array_equal(meta[:n], disp[rank]['src_metadata']):
                failures.append(f'{tag}: recv_src_metadata differs from the oracle dispatch')
            if not np.array_equal(_u16(out), expect[0]):
                failures.append(f'{tag}: combined_x differs from the oracle')
            if not np.array_equal(out_w.cpu().numpy(), expect[1]):
                failures.append(f'{tag}: combined_topk_weights differ from the oracle')

        buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                            explicitly_destroy=True, num_gpu_timeout_secs=30)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.set_sync_debug_mode('error')
        try:
            out, out_w, handle = step(buf)
        finally:
            torch.cuda.set_sync_debug_mode(0)
        torch.cuda.synchronize()
        check('sync-debug', out, out_w, handle)
        buf._sym.check()
        # the whole dispatch + first combine captured (plans and window traffic inside the graph)
        gbuf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                             explicitly_destroy=True, num_gpu_timeout_secs=30)
        torch.cuda.synchronize()
        dist.barrier()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g_out, g_w, g_handle = step(gbuf)
        for it in range(2):
            g_out.zero_()
            torch.cuda.synchronize()
            dist.barrier()
            graph.replay()
            torch.cuda.synchronize()
            check(f'graph replay {it}', g_out, g_w, g_handle)
        del graph
        gbuf._sym.check()
        for b in (buf, gbuf):
            b.destroy()
        queue.put((rank, failures))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, [traceback.format_exc()]))


@pytest.mark.parametrize('world,T,H,K,chunks', [(4, 64, 512, 8, 2), (8, 40, 256, 8, 0)])
def test_xgmi_dispatch_without_cpu_sync_then_combine(world, T, H, K, chunks):
    """EP > 1 without any host synchronisation (the reference's do_cpu_sync=False,
    csrc/elastic/buffer.hpp:1065-1070): processes sharing the GPU over HIP-IPC windows."""
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sync_free_worker, args=(r, world, port, T, H, K, chunks, queue))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, failures = queue.get(timeout=150)
            results[rank] = failures
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    if len(results) != world or any(results.values()):
        tails = {r: [f[-1500:] for f in fl] for r, fl in results.items()}
        pytest.fail(f'{len(results)}/{world} ranks reported; failures: {tails}', pytrace=False)


def test_lost_peer_times_out_instead_of_hanging():
    """Failure detection (comm.cuh:30-54, num_gpu_timeout_secs): rank 0 of a 2-rank window whose
    peer never arrives.  The device barrier and the split-barrier wait give up after the timeout,
    set the error flag and let the stream continue; check() raises.  (The reference traps.)"""
    import ctypes
    import time
    sys.path.insert(0, ROOT)
    from deepep_amd import _lib
    from deepep_amd.symmetric import HEADER_BYTES, SymmetricBuffer
    torch.cuda.set_device(0)
    lib = _lib.load()
    dead = ctypes.c_void_p()                    # the lost peer's window: allocated, never served
    _lib.check(lib.deepep_sym_alloc(HEADER_BYTES + 4096, ctypes.byref(dead)), 'sym_alloc')
    sym = SymmetricBuffer(None, 0, 2, 4096, torch.device('cuda', 0),
                          exchange=lambda base: [base, int(dead.value)], timeout_s=0.3)
    try:
        s = torch.cuda.current_stream()
        t0 = time.perf_counter()
        sym.barrier(s)
        torch.cuda.synchronize()
        assert int(sym.error_flag.item()) & 2, 'barrier did not report the timeout'
        with pytest.raises(RuntimeError, match='barrier timeout'):
            sym.check()
        sym.error_flag.zero_()
        sym.signal(1, s)                        # our own signal lands; the peer's never does
        sym.wait(1, s)
        torch.cuda.synchronize()
        assert int(sym.error_flag.item()) & 2, 'split-barrier wait did not report the timeout'
        assert time.perf_counter() - t0 < 30
        # what ElasticBuffer does around every xGMI call: publish the flag (no sync), poll it at
        # the next call -> RuntimeError there
        sym.publish(s)
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError, match='did not arrive'):
            sym.poll()
    finally:
        sym.destroy()
        _lib.check(lib.deepep_sym_free(dead), 'sym_free')


_ROW_TABLE_ROWS = 4093        # prime: the expert-output row of (source token g, lane k) is table[hash(g, k)]


def _row_table(H: int) -> np.ndarray:
    """The rows every expert output is drawn from: [4093, H] random bf16 (bits), the same in every
    process, so a rank can rebuild the expert outputs of its own tokens on every expert rank without
    moving any rows (and check its combined output against the oracle)."""
    rng = np.random.default_rng(20260)
    import oracle
    return oracle.f32_to_bf16(rng.standard_normal((_ROW_TABLE_ROWS, H)).astype(np.float32))


def _row_of(key):
    """Table row of key = global source token * K + lane (numpy or torch int64)."""
    return (key * 2654435761) % _ROW_TABLE_ROWS


def _full_worker(rank, world, port, queue, t_start):
    """BASELINE config 3 at full size over the xGMI transport: 8 processes sharing the GPU, HIP-IPC
    windows, the pipelined combine (4 chunks).  Each rank's WHOLE combined_x (and weight pass-through)
    is compared bitwise with oracle.combine_ep_one (the CPU restatement pinned to refs.combine) AND with
    the RCCL-path combine of the same handle and inputs.  The expert outputs are rows of a shared table
    picked by (source token, lane), so every rank rebuilds the rows of its own tokens on every expert
    rank from the gathered metadata, without moving rows between processes.  Every stage is reported
    with its wall-clock time since the test started (a stuck child names where it stopped)."""
    import time

    def stage(what: str) -> None:
        queue.put((rank, 'stage', f'{what} @{time.time() - t_start:.1f}s'))
    stage('started (torch imported)')
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        import torch.distributed as dist
        import oracle
        torch.cuda.set_device(0)
        stage('device set')
        dist.init_process_group('gloo', rank=rank, world_size=world)
        stage('gloo up')
        from deepep_amd import ElasticBuffer
        dev = torch.device('cuda', 0)
        T, H, K, E = 8192, 7168, 8, 256
        g = torch.Generator(device=dev).manual_seed(500 + rank)
        w, idx = torch.topk(torch.rand((T, E), device=dev, generator=g), K, dim=-1, sorted=False)
        idx = idx.to(torch.int64)
        x = torch.randn((T, H), device=dev, generator=g).to(torch.bfloat16)
        bias = torch.randn((T, H), device=dev, generator=g).to(torch.bfloat16)
        table = _row_table(H)
        bufs = {}
        for transport in ('xgmi', 'rccl'):
            os.environ['DEEPEP_TRANSPORT'] = transport
            bufs[transport] = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                                            explicitly_destroy=True, num_gpu_timeout_secs=60)
        failures = []
        stage('buffers built')
        ex_x, _, ex_w, handle, _ = bufs['xgmi'].dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E,
                                                         do_expand=True)
        _, _, ex_w_r, handle_r, _ = bufs['rccl'].dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E,
                                                          do_expand=True)
        if not torch.equal(handle.recv_src_metadata, handle_r.recv_src_metadata) or not torch.equal(ex_w, ex_w_r):
            meta_x, meta_r = handle.recv_src_metadata, handle_r.recv_src_metadata
            bad = (meta_x != meta_r).any(dim=1).nonzero().flatten() if meta_x.shape == meta_r.shape else None
            failures.append(f'xgmi dispatch != rccl dispatch: metadata shapes {tuple(meta_x.shape)} / '
                            f'{tuple(meta_r.shape)}, differing rows '
                            f'{None if bad is None else (bad.numel(), bad[:4].tolist())}, error flag '
                            f'{int(bufs["xgmi"]._sym.error_flag.item())}')
            queue.put((rank, failures))               # the combine would run on that metadata: stop here
            return
        # expert outputs: expanded row meta[j, 2 + k] holds table[_row_of(meta[j, 0] * K + k)]
        meta = handle.recv_src_metadata
        slots = meta[:, 2:].long()
        valid = slots >= 0
        keys = (meta[:, :1].long() * K + torch.arange(K, device=dev).view(1, K))[valid]
        tab = torch.from_numpy(table.view(np.int16)).to(dev).view(torch.bfloat16)
        y = torch.zeros((handle.num_expanded_tokens, H), dtype=torch.bfloat16, device=dev)
        y[slots[valid]] = tab[_row_of(keys)]
        del tab, keys
        # every expert rank's metadata rows of this rank's tokens (small: ~2 MB per rank)
        meta_np = meta.cpu().numpy()
        mine = {d: meta_np[meta_np[:, 1] // K == d] for d in range(world)}
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        idx_np, w_np = idx.cpu().numpy(), w.cpu().numpy()
        x_sub, m_sub, w_sub = [], [], []
        for e in range(world):
            m = gathered[e][rank].copy()
            sl = m[:, 2:]
            ok = sl >= 0
            tok = np.broadcast_to((m[:, :1] % T), sl.shape)[ok]
            lane = np.broadcast_to(np.arange(K), sl.shape)[ok]
            x_sub.append(table[_row_of((rank * T + tok).astype(np.int64) * K + lane)])
            w_sub.append(w_np[tok, lane].astype(np.float32))
            new = np.full(sl.shape, -1, np.int32)
            new[ok] = np.arange(int(ok.sum()), dtype=np.int32)
            m[:, 2:] = new
            m_sub.append(m)
        del gathered, mine
        stage('dispatched, rows built')
        for weighted in (False, True):
            b = None if weighted else bias
            outs = {t: bf.combine(y, handle, topk_weights=ex_w, bias=b, apply_topk_weights=weighted)
                    for t, bf in bufs.items()}
            torch.cuda.synchronize()
            stage(f'combined weighted={weighted}')
            exp, exp_w = oracle.combine_ep_one(rank, x_sub, m_sub, idx_np, E, T, expanded=True,
                                               topk_weights_per_rank=w_sub,
                                               bias=(_u16(b) if b is not None else None, None),
                                               weighted=weighted, threads=2)
            stage(f'oracle weighted={weighted}')
            for t in bufs:
                got = _u16(outs[t][0])
                if not np.array_equal(got, exp):
                    bad_rows = np.nonzero((got != exp).any(axis=1))[0]
                    failures.append(f'weighted={weighted}: {t} combined_x != oracle on {bad_rows.size} of {T} '
                                    f'tokens, first {bad_rows[:4].tolist()}')
                if not np.array_equal(outs[t][1].cpu().numpy(), exp_w):
                    failures.append(f'weighted={weighted}: {t} weight pass-through != oracle')
            if bufs['xgmi']._num_chunks(handle) < 2:
                failures.append('not pipelined')
            if not torch.equal(outs['xgmi'][0], outs['rccl'][0]):
                flag = int(bufs['xgmi']._sym.error_flag.item())
                bufs['xgmi']._sym.error_flag.zero_()
                bufs['xgmi']._sym._flag_event = None
                again = {t: bf.combine(y, handle, topk_weights=ex_w, bias=b, apply_topk_weights=weighted)[0]
                         for t, bf in bufs.items()}
                torch.cuda.synchronize()
                rows = (outs['xgmi'][0].float() != outs['rccl'][0].float()).any(dim=1)
                per_chunk = [int(rows[c * 2048:(c + 1) * 2048].sum()) for c in range(T // 2048)]
                failures.append(f'weighted={weighted}: xgmi combined_x != rccl on {int(rows.sum())} rows '
                                f'(per 2048-token chunk {per_chunk}); '
                                f'repeated: xgmi stable {torch.equal(again["xgmi"], outs["xgmi"][0])}, '
                                f'rccl stable {torch.equal(again["rccl"], outs["rccl"][0])}, '
                                f'repeated xgmi == rccl {torch.equal(again["xgmi"], again["rccl"])}, '
                                f'error flag after the first combine {flag}, after the repeat '
                                f'{int(bufs["xgmi"]._sym.error_flag.item())}')
            for t in bufs:
                if not torch.equal(outs[t][1], w):
                    bad_t = (outs[t][1] != w).any(dim=1).nonzero().flatten()
                    t0 = int(bad_t[0])
                    failures.append(f'weighted={weighted}: {t} weight pass-through on {bad_t.numel()} tokens, '
                                    f'first {bad_t[:4].tolist()}; token {t0} got {outs[t][1][t0].tolist()} '
                                    f'expected {w[t0].tolist()} routed to ranks {(idx[t0] // (E // 8)).tolist()}')
        bufs['xgmi']._sym.check()
        for bf in bufs.values():
            bf.destroy()
        queue.put((rank, failures))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, [traceback.format_exc()]))


@pytest.mark.timeout(300)
def test_xgmi_transport_full_size_config3():
    world = 8
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    import queue as queue_mod
    import time
    t_start = time.time()
    procs = [ctx.Process(target=_full_worker, args=(r, world, port, queue, t_start)) for r in range(world)]
    for p in procs:
        p.start()
    results, stages = {}, {r: 'not started (no marker yet)' for r in range(world)}
    deadline = time.time() + 240
    try:
        while len(results) < world and time.time() < deadline:
            try:
                msg = queue.get(timeout=5)
            except queue_mod.Empty:
                # a rank that died without reporting (its peers would wait out their barriers)
                dead = {r: [f'exited with code {p.exitcode} before reporting'] for r, p in enumerate(procs)
                        if p.exitcode is not None and r not in results}
                if dead:
                    results.update(dead)
                    break
                continue
            if len(msg) == 3:                 # progress marker
                stages[msg[0]] = msg[2]
                continue
            rank, failures = msg
            results[rank] = failures
            if failures:              # the other ranks may now wait out their barriers: stop early
                break
    finally:
        for p in procs:
            p.join(timeout=2 if len(results) != world or any(results.values()) else 30)
            if p.is_alive():
                p.kill()
    if len(results) != world or any(results.values()):
        tails = {r: [f[-1500:] for f in fl] for r, fl in results.items()}
        pytest.fail(f'{len(results)}/{world} ranks reported after {time.time() - t_start:.0f} s; last stage per '
                    f'rank (wall clock since the start) {stages}; failures: {tails}', pytrace=False)
