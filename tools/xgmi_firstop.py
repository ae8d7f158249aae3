"""Stress the FIRST operations over freshly imported xGMI windows (8 processes sharing the GPU).

The sporadic xGMI failures seen so far (a wrong first combine, a bad-slot flag in a first dispatch)
all came from the first call after the windows were created.  Here every rank builds one rccl
ElasticBuffer for the reference, then NEW xgmi ElasticBuffers ROUNDS times (fresh windows, fresh IPC
imports): dispatch + combine on each, compared with the rccl path (x rows, metadata, weights,
combined_x; float compares, so +0 == -0), then destroy.  Env: XFIRST_ROUNDS (default 12), XFIRST_T
(tokens per rank, default 4096)."""
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
        T, H, K, E = int(os.environ.get('XFIRST_T', 4096)), 7168, 8, 256
        rounds = int(os.environ.get('XFIRST_ROUNDS', 12))
        g = torch.Generator(device=dev).manual_seed(1300 + rank)
        w, idx = torch.topk(torch.rand((T, E), device=dev, generator=g), K, dim=-1, sorted=False)
        idx = idx.to(torch.int64)
        x = torch.randn((T, H), device=dev, generator=g).to(torch.bfloat16)
        os.environ['DEEPEP_TRANSPORT'] = 'rccl'
        rb = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K, explicitly_destroy=True)
        r_x, _, r_w, handle, _ = rb.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
        y = torch.randn((handle.num_expanded_tokens, H), device=dev, generator=g).to(torch.bfloat16)
        ref, ref_w, _ = rb.combine(y, handle, topk_weights=r_w)
        torch.cuda.synchronize()
        bad = []
        for i in range(rounds):
            os.environ['DEEPEP_TRANSPORT'] = 'xgmi'
            xb = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                               explicitly_destroy=True, num_gpu_timeout_secs=20)
            e_x, _, e_w, e_h, _ = xb.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
            torch.cuda.synchronize()
            flag_d = int(xb._sym.error_flag.item())
            ent = dict(round=i, flag_dispatch=flag_d,
                       meta=not torch.equal(e_h.recv_src_metadata, handle.recv_src_metadata),
                       x_rows=int((e_x.float() != r_x.float()).any(dim=1).sum()),
                       w=not torch.equal(e_w, r_w))
            out, out_w, _ = xb.combine(y, handle, topk_weights=r_w)     # the reference handle: same inputs
            torch.cuda.synchronize()
            ent['flag_combine'] = int(xb._sym.error_flag.item())
            ent['out_rows'] = int((out.float() != ref.float()).any(dim=1).sum())
            ent['out_w'] = not torch.equal(out_w, ref_w)
            if ent['flag_dispatch'] or ent['meta'] or ent['x_rows'] or ent['w'] or ent['flag_combine'] or \
                    ent['out_rows'] or ent['out_w']:
                bad.append(ent)
            xb._sym.error_flag.zero_()
            xb.destroy()
        rb.destroy()
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
            print(json.dumps(dict(rank=rank, rounds=res['rounds'], n_bad=len(res['bad']), bad=res['bad'][:6])),
                  flush=True)
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()


if __name__ == '__main__':
    main()
