"""The fused combine across MoE shapes beyond config 2 (diagnostic): does the launch shape tuned at
8192 x 7168 x top-8 hold its roofline fraction at other hidden sizes, top-k, expert counts and batches?

For each shape: a real dispatch (uniform routing) makes the expanded layout and the handle; the fused
kernel (weighted + pass-through, the bench's step) is timed back to back with HIP events under the
automatic launch shape and under the launch-config knobs (rows in flight 4 / 8, 1 / 2 vectors per lane,
4- / 8-wave workgroups); the token-major placement of the same rows (the layout reference of bench.py)
runs beside it, and every variant's output is checked bitwise against the automatic shape's.
"""
import json
import os
import statistics
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402

SHAPES = [  # (tokens, hidden, top-k, experts)
    (8192, 7168, 8, 256), (16384, 7168, 8, 256), (2048, 7168, 8, 256), (512, 7168, 8, 256),
    (8192, 4096, 8, 128), (8192, 2048, 8, 128), (8192, 7168, 4, 256), (8192, 5120, 6, 160),
    (8192, 4096, 2, 8), (8192, 1024, 8, 64),
]


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29631')
    dist.init_process_group('gloo', rank=0, world_size=1)
    import socket
    props = torch.cuda.get_device_properties(0)
    print(json.dumps(dict(box=socket.gethostname(), uuid=str(getattr(props, 'uuid', '')), gcn=getattr(props, 'gcnArchName', ''))), flush=True)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED
    s = torch.cuda.current_stream()
    only = os.environ.get('KSHAPES_ONLY')
    for si, (T, H, K, E) in enumerate(SHAPES):
        if only and str(si) not in only.split(','):
            continue
        torch.manual_seed(si)
        w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
        buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
        _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                             topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E,
                                             do_expand=True)
        y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
        buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
        table = handle._combine_plans[('multi', 1)].local_table
        kern, lib = buf.kernels, buf.kernels.lib
        nbytes = T * (K * H * 2 + H * 2 + K * 8)

        def run(yl, wl, tab, out, ow, upb=0):
            return lambda: kern.combine_reduce(MODE_FUSED, yl, out, T, table=tab, row_weights=wl, wtable=tab,
                                               wsrc=wl, out_weights=ow, units_per_block=upb, stream=s)
        ref = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
        ref_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
        run(y, ex_w, table, ref, ref_w)()
        kk = torch.arange(K, device='cuda').view(1, K)
        pos = torch.arange(T, device='cuda').view(T, 1) * K + kk
        yt = torch.empty((T * K, H), dtype=y.dtype, device='cuda')
        wt = torch.empty((T * K,), dtype=ex_w.dtype, device='cuda')
        yt[pos.reshape(-1)] = y[table.long().reshape(-1)]
        wt[pos.reshape(-1)] = ex_w[table.long().reshape(-1)]
        tab_t = pos.to(torch.int32).contiguous()
        # name: (launch config (vpt, lds, policy, rows in flight), units_per_block (= waves), token-major)
        variants = {'auto': ((0, -1, -1, 0), 0, False), 'token-major rows (diagnostic)': ((0, -1, -1, 0), 0, True)}
        for vpt in (1, 2):
            for rows in (2, 4, 8):
                for waves in (4, 8):
                    variants[f'vpt{vpt} rows{rows} waves{waves}'] = ((vpt, 1, 2, rows), waves, False)
        if os.environ.get('KSHAPES_POLICIES') == '1':      # store policies on the 1-KiB-chunk shapes
            for pol, pname in ((0, 'plain'), (1, 'nt'), (3, 'sc1nt')):
                variants[f'vpt1 rows2 waves4 {pname}'] = ((1, 1, pol, 2), 4, False)
        # one output for every variant (the output's placement alone moved the kernel by up to 6 % on one
        # box, tools/koutplace.py), checked against the automatic shape's bits after each variant's timing
        out = torch.empty_like(ref)
        ow = torch.empty_like(ref_w)
        fns = {name: (run(yt, wt, tab_t, out, ow, upb) if tm else run(y, ex_w, table, out, ow, upb))
               for name, (cfg, upb, tm) in variants.items()}
        times, bitwise = {k: [] for k in variants}, {k: True for k in variants}
        iters = max(10, min(200, int(2e10 / max(nbytes, 1))))
        for _ in range(int(os.environ.get('KSHAPES_ROUNDS', 3))):
            for name, (cfg, upb, tm) in variants.items():
                assert lib.deepep_set_launch_config(*cfg) == 0
                times[name].append(timeit(fns[name], s, iters=iters))
                bitwise[name] = bitwise[name] and bool(torch.equal(out, ref) and torch.equal(ow, ref_w))
        res = {}
        for name in variants:
            us = statistics.median(times[name])
            res[name] = dict(us=round(us, 2), frac=round(nbytes / us / 1e6 / 8.0, 4), bitwise=bitwise[name])
        if os.environ.get('KSHAPES_CACHE_STATE') == '1':
            # store policies of the automatic shape under different cache states: back to back into one
            # output, alternating between two outputs, single launches after a 512 MB read / write flush
            flush = torch.empty((512 << 20) // 4, dtype=torch.int32, device='cuda')
            sink = torch.empty((1,), dtype=torch.int64, device='cuda')
            out2, ow2 = torch.empty_like(ref), torch.empty_like(ref_w)
            for pol, pname in ((-1, 'sc1 (auto)'), (3, 'sc1 nt'), (1, 'nt'), (0, 'plain')):
                assert lib.deepep_set_launch_config(0, -1, pol, 0) == 0
                flip = [0]

                def alt():
                    flip[0] ^= 1
                    run(y, ex_w, table, out2 if flip[0] else out, ow2 if flip[0] else ow)()
                row = dict(same_output=round(timeit(run(y, ex_w, table, out, ow), s, iters=iters), 2),
                           alternating_outputs=round(timeit(alt, s, iters=iters), 2))
                for mode, pre in (('read_flush', lambda: torch.sum(flush, dim=0, dtype=torch.int64, out=sink)),
                                  ('write_flush', lambda: flush.fill_(1))):
                    ts = []
                    for _ in range(15):
                        pre()
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(s)
                        run(y, ex_w, table, out, ow)()
                        e1.record(s)
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3)
                    row[mode] = round(statistics.median(ts), 2)
                res[f'cache state, {pname}'] = row
            lib.deepep_set_launch_config(0, -1, -1, 0)
            del flush, out2, ow2
        best = min((k for k in res if k.startswith('vpt')), key=lambda k: res[k]['us'])
        res['best'] = dict(variant=best, vs_auto=round(res[best]['us'] / res['auto']['us'], 4))
        lib.deepep_set_launch_config(0, -1, -1, 0)
        print(json.dumps(dict(tokens=T, hidden=H, topk=K, experts=E, bytes=nbytes, variants=res)), flush=True)
        del y, yt, wt, buf, handle
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
