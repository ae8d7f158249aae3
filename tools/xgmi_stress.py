"""Stress the visibility of peer-window stores (xGMI transport) across processes sharing the GPU.

8 processes (gloo group) build an xgmi and an rccl ElasticBuffer at BASELINE config 3, dispatch once
over xGMI, take the RCCL-path combine of y as the reference, then run the xGMI combine ITERS times
alternating y and -y (every value and every rounding is exactly negated, so stale partials from
the previous call show up as sign flips).  Each rank reports per call the rows that differ from
+ref / -ref; the dispatch is repeated ITERS_D times and its handle compared with the first.
Env: XSTRESS_ITERS (default 40), XSTRESS_DISPATCH (default 10), XSTRESS_WEIGHTED (0/1), XSTRESS_T
(tokens per rank, default 8192: small T keeps the window L2-resident between calls)."""
import json
import os
import socket
import sys
import traceback

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, queue):
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from deepep_amd import ElasticBuffer
        dev = torch.device('cuda', 0)
        T, H, K, E = int(os.environ.get('XSTRESS_T', 8192)), 7168, 8, 256
        iters = int(os.environ.get('XSTRESS_ITERS', 40))
        iters_d = int(os.environ.get('XSTRESS_DISPATCH', 10))
        weighted = bool(int(os.environ.get('XSTRESS_WEIGHTED', 0)))
        g = torch.Generator(device=dev).manual_seed(900 + rank)
        w, idx = torch.topk(torch.rand((T, E), device=dev, generator=g), K, dim=-1, sorted=False)
        idx = idx.to(torch.int64)
        x = torch.randn((T, H), device=dev, generator=g).to(torch.bfloat16)
        bufs = {}
        for transport in ('xgmi', 'rccl'):
            os.environ['DEEPEP_TRANSPORT'] = transport
            bufs[transport] = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                                            explicitly_destroy=True, num_gpu_timeout_secs=20)
        xb = bufs['xgmi']
        # dispatch: repeated, alternating x and -x
        res = dict(dispatch_bad=[], combine_bad=[])
        r_x, _, r_w, r_handle, _ = bufs['rccl'].dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E,
                                                         do_expand=True)
        first = (r_x, r_w, r_handle.recv_src_metadata, None)
        for i in range(iters_d):
            xi = x if i % 2 == 0 else -x
            ex_x, _, ex_w, handle, _ = xb.dispatch(xi, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
            torch.cuda.synchronize()
            if first[3] is None:
                first = first[:3] + (handle,)
            exp_x = first[0] if i % 2 == 0 else -first[0]
            bad = dict(it=i, meta=not torch.equal(handle.recv_src_metadata, first[2]),
                       w=not torch.equal(ex_w, first[1]),
                       x_rows=int((ex_x.float() != exp_x.float()).any(dim=1).sum()))
            if bad['meta'] or bad['w'] or bad['x_rows']:
                res['dispatch_bad'].append(bad)
        handle, ex_w = first[3], first[1]
        y = torch.randn((handle.num_expanded_tokens, H), device=dev, generator=g).to(torch.bfloat16)
        ref, ref_w, _ = bufs['rccl'].combine(y, handle, topk_weights=ex_w, apply_topk_weights=weighted)
        ref = ref.clone()
        ny = -y
        for i in range(iters):
            yi = y if i % 2 == 0 else ny
            out, out_w, _ = xb.combine(yi, handle, topk_weights=ex_w, apply_topk_weights=weighted)
            torch.cuda.synchronize()
            exp = ref if i % 2 == 0 else -ref
            rows = (out.float() != exp.float()).any(dim=1)      # +0 == -0: x + (-x) is +0 either way
            n = int(rows.sum())
            wbad = int((out_w != ref_w).any(dim=1).sum())
            if n or wbad:
                stale = int(((out.float() == -exp.float()).any(dim=1) & rows).sum())
                blocks = sorted(set((rows.nonzero().flatten() // 64).tolist()))[:16]
                res['combine_bad'].append(dict(it=i, rows=n, stale_rows=stale, w_rows=wbad, blocks=blocks))
        res['error_flag'] = int(xb._sym.error_flag.item())
        for bf in bufs.values():
            bf.destroy()
        queue.put((rank, res))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, dict(exc=traceback.format_exc())))


def main():
    world = 8
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    import queue as _q
    import time
    t0 = time.time()
    try:
        got = 0
        while got < world and time.time() - t0 < 300:
            try:
                rank, res = queue.get(timeout=20)
            except _q.Empty:
                print(json.dumps(dict(waiting_s=round(time.time() - t0))), flush=True)
                continue
            got += 1
            if 'exc' in res:
                print(json.dumps(dict(rank=rank, exc=res['exc'][-2000:])), flush=True)
                break
            print(json.dumps(dict(rank=rank, error_flag=res['error_flag'], dispatch_bad=res['dispatch_bad'][:8],
                                  n_dispatch_bad=len(res['dispatch_bad']), n_combine_bad=len(res['combine_bad']),
                                  combine_bad=res['combine_bad'][:8])), flush=True)
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()


if __name__ == '__main__':
    main()
