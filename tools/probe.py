"""Memory-roofline probes for the combine (diagnostic; see tools/probe.hip)."""
import ctypes
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, iters=20, warm=3):
    s = torch.cuda.current_stream()
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    torch.cuda.set_device(0)
    lib = ctypes.CDLL(os.path.join(ROOT, 'tools', 'libprobe.so'))
    P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    lib.probe_stream_read.argtypes = [P, I64, P, I, P]
    lib.probe_stream_copy.argtypes = [P, P, I64, I, P]
    lib.probe_gather.argtypes = [I, P, P, P, I, I, P, I, P]
    lib.probe_gather_store.argtypes = [I, I, I, P, P, P, I, I, P]
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29612')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    scores = torch.rand((T, E), device='cuda')
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                         topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w)
    table = handle._combine_plans[('multi', 1)].local_table
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    sink = torch.zeros(4, device='cuda')
    st = torch.cuda.current_stream().cuda_stream
    nb = y.numel() * 2
    res = []
    for grid in (1024, 2048, 4096, 16384):
        us = timeit(lambda: lib.probe_stream_read(y.data_ptr(), nb, sink.data_ptr(), grid, st))
        res.append(dict(probe=f'stream_read grid{grid}', us=round(us, 1), gbps=round(nb / us / 1e3, 1)))
    dst = torch.empty_like(y)
    for grid in (2048, 8192):
        us = timeit(lambda: lib.probe_stream_copy(y.data_ptr(), dst.data_ptr(), nb, grid, st))
        res.append(dict(probe=f'stream_copy grid{grid}', us=round(us, 1), gbps=round(2 * nb / us / 1e3, 1)))
    del dst
    items = T * (H // 8 // 128)
    gb_read = T * K * H * 2
    for policy, region, noload in ((2, 0, 0), (0, 0, 0), (1, 0, 0), (3, 0, 0), (16, 0, 0), (17, 0, 0), (18, 0, 0),
                                   (19, 0, 0), (2, 64, 0), (0, 64, 0), (16, 64, 0), (0, 0, 1), (2, 0, 1), (16, 0, 1)):
        us = timeit(lambda: lib.probe_gather_store(policy, region, noload, y.data_ptr(), table.data_ptr(),
                                                   out.data_ptr(), T, H, st))
        nbytes = (0 if noload else gb_read) + T * H * 2
        res.append(dict(probe=f'gather_store aux{policy} region{region} noload{noload}', us=round(us, 1),
                        gbps=round(nbytes / us / 1e3, 1)))
    for variant in (5, 4):
        for grid in ((items + 3) // 4,):
            if not (variant & 8) and grid != (items + 3) // 4:
                continue
            us = timeit(lambda: lib.probe_gather(variant, y.data_ptr(), table.data_ptr(), out.data_ptr(), T, H,
                                                 sink.data_ptr(), grid, st))
            nbytes = gb_read + (T * H * 2 if variant & 1 else 0)
            name = ('store ' if variant & 1 else 'nostore ') + ('seq ' if variant & 2 else 'table ') + \
                   ('nt ' if variant & 4 else 'plain ') + ('pipe' if variant & 8 else 'flat')
            res.append(dict(probe=f'gather {name} grid{grid}', us=round(us, 1), gbps=round(nbytes / us / 1e3, 1)))
    if os.environ.get('PROBE_BURST'):
        from deepep_amd.kernels import MODE_FUSED
        res = []
        lib.probe_gather_burst.argtypes = [I, I, P, P, P, I, I, P]
        ref = torch.empty_like(out)
        lib.probe_gather_store(16, 0, 0, y.data_ptr(), table.data_ptr(), ref.data_ptr(), T, H, st)
        for rep in range(2):
            for name, fn in [('gather_store sc1 (per-wave stores)',
                              lambda: lib.probe_gather_store(16, 0, 0, y.data_ptr(), table.data_ptr(), out.data_ptr(),
                                                             T, H, st))] + \
                            [(f'gather_burst rounds{r} grid{g}',
                              (lambda r=r, g=g: lib.probe_gather_burst(r, g, y.data_ptr(), table.data_ptr(),
                                                                       out.data_ptr(), T, H, st)))
                             for r, g in ((1, 0), (4, 0), (4, 512))] + \
                            [(f'gather_burst rounds1 grid0 lds_pad{pad}',
                              (lambda pad=pad: (lib.probe_set_lds_pad(pad), lib.probe_gather_burst(
                                  1, 0, y.data_ptr(), table.data_ptr(), out.data_ptr(), T, H, st))[1]))
                             for pad in (32768, 49152, 65536, 98304)] + \
                            [('gather_burst rounds4 grid0 lds_pad0', (lambda: (lib.probe_set_lds_pad(0), lib.probe_gather_burst(
                                  4, 0, y.data_ptr(), table.data_ptr(), out.data_ptr(), T, H, st))[1]))] + \
                            [('product fused kernel, plain sum (8-wave workgroups, per-wave stores)',
                              lambda: buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=table,
                                                                 stream=torch.cuda.current_stream()) or 0)]:
                out.zero_()
                assert fn() == 0
                torch.cuda.synchronize()
                same = bool(torch.equal(out, ref)) if not name.startswith('product') else None
                us = timeit(fn)
                res.append(dict(probe=name, rep=rep, us=round(us, 1), gbps=round((gb_read + T * H * 2) / us / 1e3, 1),
                                equal=same))
    for r in res:
        print(json.dumps(r), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
