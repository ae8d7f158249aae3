"""Repeat the config-3 xGMI test's sequence many times in one process group, to make a rare race
frequent: per round, a fresh xgmi dispatch (new handle), the rccl dispatch, the first xgmi combine on
the new handle (its plan is built in that call), the rccl combine; compare.  No host syncs inside a
round except the comparisons at its end (XROUNDS_SYNC=<points> adds torch.cuda.synchronize() at
named points to bisect: 'd' after the xgmi dispatch, 'r' after the rccl dispatch, 'p' before the
xgmi combine).  Env: XROUNDS (default 8), XROUNDS_T (default 8192)."""
import json
import os
import socket
import sys
import time
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
        T, H, K, E = int(os.environ.get('XROUNDS_T', 8192)), 7168, 8, 256
        rounds = int(os.environ.get('XROUNDS', 8))
        sync = os.environ.get('XROUNDS_SYNC', '')
        g = torch.Generator(device=dev).manual_seed(700 + rank)
        bufs = {}
        for transport in ('xgmi', 'rccl'):
            os.environ['DEEPEP_TRANSPORT'] = transport
            bufs[transport] = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                                            explicitly_destroy=True, num_gpu_timeout_secs=20)
        bad = []
        for i in range(rounds):
            w, idx = torch.topk(torch.rand((T, E), device=dev, generator=g), K, dim=-1, sorted=False)
            idx = idx.to(torch.int64)
            x = torch.randn((T, H), device=dev, generator=g).to(torch.bfloat16)
            bias = torch.randn((T, H), device=dev, generator=g).to(torch.bfloat16)
            _, _, ex_w, handle, _ = bufs['xgmi'].dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E,
                                                          do_expand=True)
            if 'd' in sync:
                torch.cuda.synchronize()
            _, _, ex_w_r, handle_r, _ = bufs['rccl'].dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E,
                                                              do_expand=True)
            if 'r' in sync:
                torch.cuda.synchronize()
            y = torch.randn((handle.num_expanded_tokens, H), device=dev, generator=g).to(torch.bfloat16)
            if 'p' in sync:
                torch.cuda.synchronize()
            ox, ow, _ = bufs['xgmi'].combine(y, handle, topk_weights=ex_w, bias=bias)
            rx, rw, _ = bufs['rccl'].combine(y, handle, topk_weights=ex_w, bias=bias)
            torch.cuda.synchronize()
            flag = int(bufs['xgmi']._sym.error_flag.item())
            ent = dict(round=i, flag=flag,
                       dispatch=not (torch.equal(handle.recv_src_metadata, handle_r.recv_src_metadata) and
                                     torch.equal(ex_w, ex_w_r)),
                       rows=int((ox.float() != rx.float()).any(dim=1).sum()),
                       w_tokens=int((ow != w).any(dim=1).sum()), rw_tokens=int((rw != w).any(dim=1).sum()))
            if ent['flag'] or ent['dispatch'] or ent['rows'] or ent['w_tokens'] or ent['rw_tokens']:
                bad.append(ent)
                bufs['xgmi']._sym.error_flag.zero_()
                bufs['xgmi']._sym._flag_event = None
        for bf in bufs.values():
            bf.destroy()
        queue.put((rank, dict(bad=bad, rounds=rounds)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, dict(exc=traceback.format_exc())))


def main():
    import queue as _q
    world = 8
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    t0 = time.time()
    try:
        got = 0
        while got < world and time.time() - t0 < 280:
            try:
                rank, res = queue.get(timeout=20)
            except _q.Empty:
                print(json.dumps(dict(waiting_s=round(time.time() - t0))), flush=True)
                continue
            got += 1
            if 'exc' in res:
                print(json.dumps(dict(rank=rank, exc=res['exc'][-1500:])), flush=True)
                break
            print(json.dumps(dict(rank=rank, rounds=res['rounds'], n_bad=len(res['bad']), bad=res['bad'][:8])),
                  flush=True)
    finally:
        for p in procs:
            p.join(timeout=3)
            if p.is_alive():
                p.kill()


if __name__ == '__main__':
    main()
