"""RCCL transport preflight for bench.py at N > 1 (run as a child process, one per rank).

The N > 1 headline is the combine over RCCL's all_to_all_single (async, waited on the stream).  RCCL has
never run with more than one rank in this code base's measured history; an init failure, an all-to-all
failure or a hang in the headline would cost the whole line.  So before bench.py touches the GPU, every
rank starts this script as a child; the children form their own RCCL world (port = the bench's
MASTER_PORT + 2, each on its rank's GPU) plus a gloo group of the same ranks, and run a small dispatch +
combine twice: over the RCCL group (the headline's transport: row all-to-alls, pipelined chunks) and over
the gloo group (the same kernels, the exchange through host memory).  Dispatch outputs and handle
metadata, combined_x and the weight pass-through must match bit for bit; every rank's verdict is
combined over gloo.  bench.py uses RCCL for the headline only when every child exited 0.

DEEPEP_BENCH_FAIL_RCCL_PREFLIGHT=1 makes the child fail on purpose (the CPU tests of the fallback).
Prints one JSON line: {"ok": bool, "rank": r, "world": n, "device": d, "seconds": s, "error": ...}.
Exit status 0 = pass, 1 = mismatch or exception.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

TOKENS, HIDDEN, TOPK = 1024, 7168, 8          # 1024 tokens: the combine runs its 4-chunk pipeline


def main() -> int:
    t0 = time.perf_counter()
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    res = dict(ok=False, rank=rank, world=world, device=None, error=None)
    try:
        if os.environ.get('DEEPEP_BENCH_FAIL_RCCL_PREFLIGHT', '0') == '1':
            raise RuntimeError('failure injected (DEEPEP_BENCH_FAIL_RCCL_PREFLIGHT=1)')
        import torch
        import torch.distributed as dist
        local = int(os.environ.get('LOCAL_RANK', rank))
        dev_i = local % torch.cuda.device_count()
        torch.cuda.set_device(dev_i)
        res['device'] = dev_i
        dev = torch.device('cuda', dev_i)
        dist.init_process_group('nccl', rank=rank, world_size=world, device_id=dev)
        host_group = dist.new_group(backend='gloo')
        from deepep_amd import ElasticBuffer
        E = 32 * world
        g = torch.Generator(device=dev).manual_seed(11 + rank)
        scores = torch.rand((TOKENS, E), device=dev, generator=g)
        w, idx = torch.topk(scores, TOPK, dim=-1, sorted=False)
        idx = idx.to(torch.int64)
        idx[torch.rand((TOKENS, TOPK), device=dev, generator=g) < 0.1] = -1
        x = torch.randn((TOKENS, HIDDEN), device=dev, generator=g).to(torch.bfloat16)
        bufs = {name: ElasticBuffer(group, num_max_tokens_per_rank=TOKENS, hidden=HIDDEN, num_topk=TOPK,
                                    explicitly_destroy=True)
                for name, group in (('rccl', dist.group.WORLD), ('gloo', host_group))}
        for b in bufs.values():
            b.transport = 'rccl'
        failures = []
        disp = {t: b.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
                for t, b in bufs.items()}
        torch.cuda.synchronize()
        a, b = disp['rccl'], disp['gloo']
        for i, name in ((0, 'recv_x'), (2, 'recv_topk_weights')):
            if not torch.equal(a[i].view(torch.uint8), b[i].view(torch.uint8)):
                failures.append(f'dispatch {name}')
        if not torch.equal(a[3].recv_src_metadata, b[3].recv_src_metadata):
            failures.append('dispatch recv_src_metadata')
        y = torch.randn(a[0].shape, device=dev, generator=g).to(torch.bfloat16)
        outs = {}
        for t, buf in bufs.items():
            for _ in range(2):                          # the second call reuses the cached plan
                outs[t] = buf.combine(y, disp[t][3], topk_weights=disp[t][2], apply_topk_weights=True)
            torch.cuda.synchronize()
        res['chunks'] = bufs['rccl']._num_chunks(disp['rccl'][3])
        if not torch.equal(outs['rccl'][0], outs['gloo'][0]):
            failures.append('combined_x')
        if not torch.equal(outs['rccl'][1], outs['gloo'][1]):
            failures.append('combined_topk_weights')
        # the barrier the bench brackets its timed loop with, over RCCL
        bufs['rccl'].barrier()
        torch.cuda.synchronize()
        t = torch.tensor([0 if failures else 1], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=host_group)
        if failures:
            res['error'] = 'rccl != gloo: ' + ', '.join(failures)
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
