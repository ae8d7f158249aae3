"""Does a symmetric window leak device memory when it is freed?  (round 6: tests/test_pressure_gpu.py saw the
device's free memory fall ~6.5 MiB per xGMI buffer created and destroyed per process.)  Through the library's
own C-ABI (deepep_sym_alloc / _export / _import / _close / _free), per iteration, device free memory after it:

  python tools/probe_ipc_leak.py alloc      alloc + free
  python tools/probe_ipc_leak.py export     alloc + hipIpcGetMemHandle + free
  python tools/probe_ipc_leak.py reexport   one allocation, exported again every iteration
  python tools/probe_ipc_leak.py streams    a new torch.cuda.Stream() per iteration, used once (torch's stream pool
                                            creates its HIP streams lazily: each new one takes runtime resources)
  python tools/probe_ipc_leak.py buffers    a new ElasticBuffer per iteration (one rank), combine, destroy
  python tools/probe_ipc_leak.py pair       2 processes (gloo): alloc, export, exchange, import the peer's,
                                            close, free
  python tools/probe_ipc_leak.py pairpool   the same with ONE allocation per process kept across iterations
                                            (exported, imported and closed every iteration, never freed)
One JSON line per mode: the free-memory drop per iteration (MiB) after a warm-up iteration.
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
N_ITER, BYTES = 12, 3 << 20


def _free():
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info()[0]


def single(mode):
    from deepep_amd import _lib
    lib = _lib.load()
    torch.cuda.set_device(0)
    torch.zeros(1, device='cuda')
    frees = []
    keep = ctypes.c_void_p()
    if mode == 'reexport':
        assert lib.deepep_sym_alloc(BYTES, ctypes.byref(keep)) == 0
    streams = []
    for i in range(N_ITER):
        if mode == 'streams':
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                torch.zeros(1, device='cuda').add_(1)
            streams.append(st)
            frees.append(_free())
            continue
        if mode == 'buffers':
            import torch.distributed as dist
            if not dist.is_initialized():
                os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
                os.environ.setdefault('MASTER_PORT', '29571')
                dist.init_process_group('gloo', rank=0, world_size=1)
            from deepep_amd import ElasticBuffer
            b = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=64, hidden=256, num_topk=2,
                              explicitly_destroy=True)
            idx = torch.topk(torch.rand((64, 8), device='cuda'), 2, dim=-1)[1]
            ex, _, _, h, _ = b.dispatch(torch.randn((64, 256), device='cuda').to(torch.bfloat16), topk_idx=idx,
                                        num_experts=8, do_expand=True)
            b.combine(ex, h)
            b.destroy()
            del b, ex, h
            frees.append(_free() + torch.cuda.memory_reserved())
            continue
        if mode == 'reexport':
            h = ctypes.create_string_buffer(64)
            assert lib.deepep_sym_export(keep, h) == 0
            frees.append(_free())
            continue
        p = ctypes.c_void_p()
        assert lib.deepep_sym_alloc(BYTES, ctypes.byref(p)) == 0
        if mode == 'export':
            h = ctypes.create_string_buffer(64)
            assert lib.deepep_sym_export(p, h) == 0
        assert lib.deepep_sym_free(p) == 0
        frees.append(_free())
    drops = [(frees[1] - f) / 2 ** 20 for f in frees[1:]]
    print(json.dumps(dict(mode=mode, bytes=BYTES, drop_mib_after_iteration=[round(d, 2) for d in drops])), flush=True)


def _pair_worker(rank, port, q, pool=False):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=2)
    from deepep_amd import _lib
    lib = _lib.load()
    torch.zeros(1, device='cuda')
    frees = []
    keep = ctypes.c_void_p()
    if pool:
        assert lib.deepep_sym_alloc(BYTES, ctypes.byref(keep)) == 0
    for _ in range(N_ITER):
        p = keep
        if not pool:
            p = ctypes.c_void_p()
            assert lib.deepep_sym_alloc(BYTES, ctypes.byref(p)) == 0
        h = ctypes.create_string_buffer(64)
        assert lib.deepep_sym_export(p, h) == 0
        hs = [None, None]
        dist.all_gather_object(hs, h.raw)
        q_ = ctypes.c_void_p()
        assert lib.deepep_sym_import(ctypes.create_string_buffer(hs[1 - rank], 64), ctypes.byref(q_)) == 0
        dist.barrier()
        assert lib.deepep_sym_close(q_) == 0
        dist.barrier()
        if not pool:
            assert lib.deepep_sym_free(p) == 0
        dist.barrier()
        frees.append(_free())
        dist.barrier()
    q.put((rank, [(frees[1] - f) / 2 ** 20 for f in frees[1:]]))
    dist.destroy_process_group()


def pair(pool=False):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_pair_worker, args=(r, port, q, pool)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=30)
    print(json.dumps(dict(mode='pairpool' if pool else 'pair', bytes=BYTES, drop_mib_after_iteration={r: [round(d, 2) for d in v]
                                                                               for r, v in res.items()})), flush=True)


if __name__ == '__main__':
    m = sys.argv[1] if len(sys.argv) > 1 else 'alloc'
    pair(m == 'pairpool') if m.startswith('pair') else single(m)
