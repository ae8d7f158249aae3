"""Is a freshly allocated symmetric window's header (barrier flags and counters) really zero?

8 processes share the GPU (gloo); each builds an xgmi ElasticBuffer (its window is allocated and
zeroed at construction, deepep_sym_alloc), synchronises, host-barriers, then reads its own window
header (HEADER_BYTES) and reports every nonzero int64 entry (flag table [slot][rank], counter rows).
Nonzero entries before the first barrier would let a first barrier / split-barrier wait pass early.
Env: XHDR_ROUNDS (default 3): buffers built and destroyed per process."""
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
        os.environ['DEEPEP_TRANSPORT'] = 'xgmi'
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from deepep_amd import ElasticBuffer
        from deepep_amd.symmetric import HEADER_BYTES, _DeviceArray
        res = []
        for i in range(int(os.environ.get('XHDR_ROUNDS', 3))):
            buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=8192, hidden=7168, num_topk=8,
                                explicitly_destroy=True)
            torch.cuda.synchronize()
            dist.barrier()
            hdr = torch.as_tensor(_DeviceArray(buf._sym.base, HEADER_BYTES), device='cuda').view(torch.int64)
            nz = (hdr != 0).nonzero().flatten().tolist()
            ent = dict(round=i, nonzero=len(nz))
            if nz:
                ent['first'] = [(j // 64, j % 64, int(hdr[j])) if j < 64 * 64 else ('cnt', j - 64 * 64, int(hdr[j]))
                                for j in nz[:12]]
            # the data region right after the header: zero too?
            data = torch.as_tensor(_DeviceArray(buf._sym.base + HEADER_BYTES, 1 << 20), device='cuda').view(torch.int64)
            ent['data_nonzero_first_MB'] = int((data != 0).sum())
            res.append(ent)
            dist.barrier()
            buf.destroy()
        queue.put((rank, res))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, [dict(exc=traceback.format_exc()[-1500:])]))


def main():
    world = 8
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        for _ in range(world):
            rank, res = queue.get(timeout=150)
            print(json.dumps(dict(rank=rank, res=res)), flush=True)
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()


if __name__ == '__main__':
    main()
