"""xGMI transport preflight for bench.py at N > 1 (run as a child process, one per rank).

The xGMI transport (DEEPEP_TRANSPORT=xgmi: HIP IPC symmetric windows, system-scope stores into the
peers' windows, device barriers) has only ever run with every rank on ONE GPU.  On a node of
distinct GPUs a store through a mis-mapped window is a GPU fault that ends the process -- and
with it bench.py's whole line.  So before bench.py touches the GPU, every rank starts this script
as a child; the children form their own gloo world (port = the bench's MASTER_PORT + 1), each on
its rank's GPU, and run a small dispatch + combine over xGMI next to the same calls over the
default transport: dispatch outputs and handle metadata, combined_x and the weight pass-through
must match bit for bit, and no window error bit may be set.  bench.py times its xGMI legs only
when every child exited 0; otherwise the line says why they were skipped.

Prints one JSON line: {"ok": bool, "rank": r, "world": n, "device": d, "seconds": s, "error": ...}.
Exit status 0 = pass, 1 = mismatch or exception.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

TOKENS, HIDDEN, TOPK = 512, 7168, 8


def main() -> int:
    t0 = time.perf_counter()
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    res = dict(ok=False, rank=rank, world=world, device=None, error=None)
    try:
        import torch
        import torch.distributed as dist
        local = int(os.environ.get('LOCAL_RANK', rank))
        dev_i = local % torch.cuda.device_count()
        torch.cuda.set_device(dev_i)
        res['device'] = dev_i
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from deepep_amd import ElasticBuffer
        dev = torch.device('cuda', dev_i)
        E = 32 * world
        g = torch.Generator(device=dev).manual_seed(7 + rank)
        scores = torch.rand((TOKENS, E), device=dev, generator=g)
        w, idx = torch.topk(scores, TOPK, dim=-1, sorted=False)
        idx = idx.to(torch.int64)
        idx[torch.rand((TOKENS, TOPK), device=dev, generator=g) < 0.1] = -1
        x = torch.randn((TOKENS, HIDDEN), device=dev, generator=g).to(torch.bfloat16)
        bufs = {}
        for transport in ('rccl', 'xgmi'):
            bufs[transport] = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=TOKENS, hidden=HIDDEN,
                                            num_topk=TOPK, explicitly_destroy=True, num_gpu_timeout_secs=10)
            bufs[transport].transport = transport
        failures = []
        disp = {t: b.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
                for t, b in bufs.items()}
        torch.cuda.synchronize()
        a, b = disp['xgmi'], disp['rccl']
        for i, name in ((0, 'recv_x'), (2, 'recv_topk_weights')):
            if not torch.equal(a[i].view(torch.uint8), b[i].view(torch.uint8)):
                failures.append(f'dispatch {name}')
        if not torch.equal(a[3].recv_src_metadata, b[3].recv_src_metadata):
            failures.append('dispatch recv_src_metadata')
        y = torch.randn(a[0].shape, device=dev, generator=g).to(torch.bfloat16)
        outs = {}
        for t, buf in bufs.items():
            for _ in range(2):                          # the second call reuses the windows (epochs)
                outs[t] = buf.combine(y, disp[t][3], topk_weights=disp[t][2], apply_topk_weights=True)
            torch.cuda.synchronize()
        if not torch.equal(outs['xgmi'][0], outs['rccl'][0]):
            failures.append('combined_x')
        if not torch.equal(outs['xgmi'][1], outs['rccl'][1]):
            failures.append('combined_topk_weights')
        bufs['xgmi']._sym.check()                       # raises on a window error bit
        t = torch.tensor([0 if failures else 1], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        if failures:
            res['error'] = 'xgmi != rccl: ' + ', '.join(failures)
        elif not int(t.item()):
            res['error'] = 'mismatch on another rank'
        else:
            res['ok'] = True
        for buf in bufs.values():
            buf.destroy()
        dist.destroy_process_group()
    except Exception as e:                              # noqa: BLE001 -- reported to the parent
        res['error'] = f'{type(e).__name__}: {e}'[:300]
    res['seconds'] = round(time.perf_counter() - t0, 2)
    print(json.dumps(res), flush=True)
    return 0 if res['ok'] else 1


if __name__ == '__main__':
    sys.exit(main())
