"""Does the placement of the OUTPUT rows change the fused combine's time?  (diagnostic, config 2)

tools/kshapes.py timed the same kernel and launch shape at 163-175 us depending only on which freshly
allocated output it wrote.  Here one input (the expanded rows, expert layout) and one slot table are
reduced into outputs placed at several byte offsets inside one large allocation and into separate
allocations, interleaved over rounds (medians); the input is also cloned once to separate input from
output effects.  Every output is checked bitwise against the first.
"""
import json
import os
import statistics
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29637')
    dist.init_process_group('gloo', rank=0, world_size=1)
    import socket
    props = torch.cuda.get_device_properties(0)
    print(json.dumps(dict(box=socket.gethostname(), uuid=str(getattr(props, 'uuid', '')), gcn=getattr(props, 'gcnArchName', ''))), flush=True)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                         topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
    table = handle._combine_plans[('multi', 1)].local_table
    kern = buf.kernels
    s = torch.cuda.current_stream()
    nbytes = T * (K * H * 2 + H * 2 + K * 8)
    n = T * H
    MiB = 1 << 20
    offsets = [0, 4096, 65536, 256 * 1024, MiB, 2 * MiB, 3 * MiB, 4 * MiB, 6 * MiB, 8 * MiB, 16 * MiB, 24 * MiB,
               32 * MiB, 48 * MiB, 64 * MiB]
    pool = torch.empty((n + (offsets[-1] + 2 * MiB) // 2,), dtype=torch.bfloat16, device='cuda')
    outs = {f'pool+{o // 1024}K': pool[o // 2:o // 2 + n].view(T, H) for o in offsets}
    for i in range(6):
        outs[f'alloc{i}'] = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    y2 = y.clone()
    if os.environ.get('KOUT_INPUTS') == '1':
        # input placement: the same rows cloned into fresh allocations, one output (round 1 saw up to 10 %)
        clones = [y] + [y.clone() for _ in range(7)]
        times = {i: [] for i in range(len(clones))}
        out = outs['alloc0']
        ow0 = torch.empty((T, K), dtype=torch.float32, device='cuda')
        for _ in range(int(os.environ.get('KOUT_ROUNDS', 4))):
            for i, yy in enumerate(clones):
                times[i].append(timeit(lambda yy=yy: kern.combine_reduce(MODE_FUSED, yy, out, T, table=table,
                                                                         row_weights=ex_w, wtable=table, wsrc=ex_w,
                                                                         out_weights=ow0, stream=s), s, iters=30))
        for i in times:
            print(json.dumps(dict(input_clone=i, us=round(statistics.median(times[i]), 2),
                                  frac=round(nbytes / statistics.median(times[i]) / 8e6, 4),
                                  addr_mod_1G=clones[i].data_ptr() % (1 << 30))), flush=True)
        del clones
    ow = torch.empty((T, K), dtype=torch.float32, device='cuda')
    variants = {}
    for name, out in outs.items():
        variants[name] = (y, out)
    for name in ('pool+0K', 'alloc0', 'alloc1'):
        variants[f'{name} (input clone)'] = (y2, outs[name])
    times = {k: [] for k in variants}
    for _ in range(int(os.environ.get('KOUT_ROUNDS', 4))):
        for name, (yy, out) in variants.items():
            fn = (lambda yy=yy, out=out: kern.combine_reduce(MODE_FUSED, yy, out, T, table=table, row_weights=ex_w,
                                                              wtable=table, wsrc=ex_w, out_weights=ow, stream=s))
            times[name].append(timeit(fn, s, iters=30))
    ref = None
    res = {}
    for name, (yy, out) in variants.items():
        kern.combine_reduce(MODE_FUSED, yy, out, T, table=table, row_weights=ex_w, wtable=table, wsrc=ex_w,
                            out_weights=ow, stream=s)
        torch.cuda.synchronize()
        ref = out.clone() if ref is None else ref
        us = statistics.median(times[name])
        res[name] = dict(us=round(us, 2), frac=round(nbytes / us / 8e6, 4), spread=round(max(times[name]) -
                         min(times[name]), 2), out_addr_mod_64M=(out.data_ptr() - y.data_ptr()) % (64 * MiB),
                         bitwise=bool(torch.equal(out, ref)))
        print(json.dumps(dict(variant=name, **res[name])), flush=True)
    vals = [r['us'] for r in res.values()]
    print(json.dumps(dict(summary=dict(min_us=min(vals), max_us=max(vals), median_us=statistics.median(vals)))),
          flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
