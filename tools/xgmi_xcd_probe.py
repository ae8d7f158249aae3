"""Cross-XCD hand-off through a symmetric window between two processes sharing the GPU.

Builds on tools/_xcd_probe.so (hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/xcd_probe.hip -o
tools/_xcd_probe.so): fill / check kernels that run on chosen XCDs only.  Per case and trial:
  owner (rank 1): fill its window region with P0 from XCD a, read it back from XCD a (lines cached
  there if the owner's mapping is cacheable);  host barrier;
  peer (rank 0): fill the same region with P1 through its IPC mapping from XCD b (b != a); sync;
  host barrier;  owner: check the region for P1 from XCD a with plain / nt / sc0-sc1 loads.
Any mismatch is a stale line in the owner's XCD-a L2: its view of its own window is cached and a
peer's writes through another XCD do not reach it.  Also run: the owner's memory from a plain
hipMalloc (torch) buffer shared the same way, as a control."""
import ctypes
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
        from deepep_amd.symmetric import HEADER_BYTES, SymmetricBuffer
        lib = ctypes.CDLL(os.path.join(ROOT, 'tools', '_xcd_probe.so'))
        lib.xcd_fill.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32, ctypes.c_void_p,
                                 ctypes.c_void_p]
        lib.xcd_check.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        dev = torch.device('cuda', 0)
        sym = SymmetricBuffer(dist.group.WORLD, rank, world, 64 << 20, dev)
        owner = 1
        s = torch.cuda.current_stream().cuda_stream
        wgs = torch.zeros((4,), dtype=torch.int32, device=dev)
        mism = torch.zeros((1,), dtype=torch.int64, device=dev)
        res = []
        trials = int(os.environ.get('XPROBE_TRIALS', 6))
        for size_mb in (1, 8):
            n = (size_mb << 20) // 4
            own_ptr = sym.base + HEADER_BYTES
            peer_ptr = sym.bases[owner] + HEADER_BYTES
            for a, b in ((0, 4), (2, 5), (7, 1)):
                for flavour in (0, 1, 2):
                    for t in range(trials):
                        p0, p1 = 5000 + 2 * t + 100 * flavour, 5001 + 2 * t + 100 * flavour
                        if rank == owner:
                            wgs.zero_()
                            lib.xcd_fill(ctypes.c_void_p(own_ptr), n, p0, 1 << a, ctypes.c_void_p(wgs.data_ptr()), s)
                            wgs.zero_()
                            mism.zero_()
                            lib.xcd_check(ctypes.c_void_p(own_ptr), n, p0, 1 << a, 0, ctypes.c_void_p(wgs.data_ptr()),
                                          ctypes.c_void_p(mism.data_ptr()), s)
                            torch.cuda.synchronize()
                            first = int(mism.item())
                        dist.barrier()
                        if rank == 0:
                            wgs.zero_()
                            lib.xcd_fill(ctypes.c_void_p(peer_ptr), n, p1, 1 << b, ctypes.c_void_p(wgs.data_ptr()), s)
                            torch.cuda.synchronize()
                        dist.barrier()
                        if rank == owner:
                            wgs.zero_()
                            mism.zero_()
                            lib.xcd_check(ctypes.c_void_p(own_ptr), n, p1, 1 << a, flavour,
                                          ctypes.c_void_p(wgs.data_ptr()), ctypes.c_void_p(mism.data_ptr()), s)
                            torch.cuda.synchronize()
                            res.append(dict(size_mb=size_mb, owner_xcd=a, peer_xcd=b, flavour=flavour, trial=t,
                                            first_read_bad=first, stale_words=int(mism.item())))
                        dist.barrier()
        queue.put((rank, res))
        dist.barrier()
        sym.destroy()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, [dict(exc=traceback.format_exc()[-2000:])]))


def main():
    world = 2
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        for _ in range(world):
            rank, res = queue.get(timeout=200)
            if rank == 1 or any('exc' in r for r in res):
                bad = [r for r in res if 'exc' in r or r.get('stale_words') or r.get('first_read_bad')]
                summary = {}
                for r in res:
                    if 'exc' in r:
                        continue
                    k = f"flavour{r['flavour']}_{r['size_mb']}MB"
                    summary.setdefault(k, [0, 0])
                    summary[k][0] += 1
                    summary[k][1] += bool(r['stale_words'])
                print(json.dumps(dict(rank=rank, trials=len(res), bad=len(bad), stale_trials=summary,
                                      examples=bad[:6])), flush=True)
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()


if __name__ == '__main__':
    main()
