"""Can a window owner read STALE lines of its own symmetric window after a peer wrote it?

2 processes share the GPU (gloo), each with a SymmetricBuffer (deepep_sym_alloc: uncached).  Per trial:
  1. the owner (rank 1) fills a region of its window with pattern P0 (plain stores) and reads it back
     with plain loads (so the lines would sit in its L2s if the mapping were cacheable);
  2. host barrier; rank 0 fills the same region through its IPC mapping with P1 and synchronises;
  3. host barrier; the owner reads the region again (a new kernel, plain loads) and counts P0 words.
  mode 'device': steps 2-3 ordered only by the device barrier (sym.barrier), no host sync between.
Any P0 word is a stale line: the owner's view of its own window is then cached and a peer's writes do
not invalidate it.  Variants: region size, and whether the owner runs an L2-evicting read in between.
Env: XPROBE_TRIALS (default 20)."""
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
        from deepep_amd.symmetric import SymmetricBuffer, _DeviceArray
        dev = torch.device('cuda', 0)
        sym = SymmetricBuffer(dist.group.WORLD, rank, world, 64 << 20, dev)
        owner = 1
        peer_view = torch.as_tensor(_DeviceArray(sym.bases[owner] + (64 << 10), 64 << 20), device=dev).view(torch.int32)
        own = sym.data.view(torch.int32)
        trials = int(os.environ.get('XPROBE_TRIALS', 20))
        res = []
        for mode, size_mb in [(m, z) for m in ('host', 'device') for z in (1, 4, 16)]:
            n = (size_mb << 20) // 4
            for t in range(trials):
                p0, p1 = 1000 + 2 * t, 1001 + 2 * t
                if rank == owner:
                    own[:n].fill_(p0)
                    s0 = int((own[:n] == p0).sum())          # plain loads: caches the lines if cacheable
                    torch.cuda.synchronize()
                dist.barrier()
                if mode == 'device':
                    # hand-off ordered only by the device barrier: no host sync between the peer's write
                    # and the owner's read
                    if rank == 0:
                        peer_view[:n].fill_(p1)
                    sym.barrier(torch.cuda.current_stream())
                    if rank == owner:
                        v = own[:n].clone()
                    torch.cuda.synchronize()
                else:
                    if rank == 0:
                        peer_view[:n].fill_(p1)
                        torch.cuda.synchronize()
                    dist.barrier()
                if rank == owner:
                    if mode != 'device':
                        v = own[:n].clone()
                    torch.cuda.synchronize()
                    stale = int((v == p0).sum())
                    other = int(((v != p0) & (v != p1)).sum())
                    res.append(dict(mode=mode, size_mb=size_mb, trial=t, first_read_ok=s0 == n, stale_words=stale,
                                    other_words=other))
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
                bad = [r for r in res if 'exc' in r or r['stale_words'] or r['other_words'] or not r['first_read_ok']]
                print(json.dumps(dict(rank=rank, trials=len(res), bad=len(bad), examples=bad[:6])), flush=True)
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()


if __name__ == '__main__':
    main()
