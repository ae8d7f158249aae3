"""Round-6 experiment: the fused combine with its source rows arriving by LDS-DMA
(global_load_lds_dwordx4, nt or default policy) instead of global_load_dwordx4 nt into registers.

BASELINE config 2 (8192 x 7168 x top-8 over 256 experts, weighted, bench.py's inputs), the same kernel
arithmetic, both layouts in one process: the product's expert-grouped rows and the same rows placed
token-major.  Interleaved rounds (every variant once per round, N launches back to back, HIP events
on the launch stream), median per variant; every variant's output compared bit for bit with the
product's.  One JSON line per (layout, variant) and a summary line.

usage: python tools/kldsdma.py [--rounds 5] [--launches 100]
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, load path, vectors per lane, rows in flight, waves per workgroup); path 0 = registers (product)
VARIANTS = [
    ('product', 0, 0, 0, 0),
    ('vgpr_v1_r2_w4', 0, 1, 2, 4),
    ('ldsnt_v1_r4_w4', 1, 1, 4, 4),
    ('ldsnt_v1_r8_w4', 1, 1, 8, 4),
    ('ldsnt_v2_r4_w4', 1, 2, 4, 4),
    ('ldsnt_v1_r4_w8', 1, 1, 4, 8),
    ('lds_v1_r4_w4', 2, 1, 4, 4),
    ('lds_v1_r8_w4', 2, 1, 8, 4),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--launches', type=int, default=100)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29617')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED
    T, H, K, E = 8192, 7168, 8, 256
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    scores = torch.rand((T, E), device=dev)
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    x = torch.randn((T, H), device=dev).to(torch.bfloat16)
    _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E,
                                         do_expand=True)
    del x
    y = torch.randn((handle.num_expanded_tokens, H), device=dev).to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
    plan = handle._combine_plans[('multi', 1)]
    tab = plan.local_table
    valid = int((tab >= 0).sum().item())
    bytes_launch = valid * H * 2 + T * H * 2 + valid * 8
    # token-major placement of the same rows (bench.py's same_run_token_major_rows)
    pos = torch.arange(T * K, device=dev).view(T, K)
    yt = torch.empty_like(y)
    wt = torch.empty_like(ex_w)
    yt[pos.reshape(-1)] = y[tab.long().reshape(-1)]
    wt[pos.reshape(-1)] = ex_w[tab.long().reshape(-1)]
    tab_t = pos.to(torch.int32)
    layouts = {'expert_grouped': (y, ex_w, tab), 'token_major': (yt, wt, tab_t)}
    kern = buf.kernels
    lib = kern.lib
    stream = torch.cuda.current_stream()
    out = torch.empty((T, H), dtype=torch.bfloat16, device=dev)
    out_w = torch.empty((T, K), dtype=torch.float32, device=dev)

    def launch(layout, v):
        src, wsrc, table = layouts[layout]
        kern.combine_reduce(MODE_FUSED, src, out, T, table=table, row_weights=wsrc, wtable=table, wsrc=wsrc,
                            out_weights=out_w, units_per_block=v[4], stream=stream)

    def configure(v):
        assert lib.deepep_amd_exp_load_path(v[1]) == 0
        assert lib.deepep_set_launch_config(v[2], v[3]) == 0

    ref = {}
    times = {(l, v[0]): [] for l in layouts for v in VARIANTS}
    exact = {}
    try:
        for layout in layouts:
            configure(VARIANTS[0])
            launch(layout, VARIANTS[0])
            torch.cuda.synchronize()
            ref[layout] = (out.clone(), out_w.clone())
            for v in VARIANTS:
                configure(v)
                out.zero_()
                launch(layout, v)
                torch.cuda.synchronize()
                exact[(layout, v[0])] = bool(torch.equal(out, ref[layout][0]) and torch.equal(out_w, ref[layout][1]))
        for r in range(args.rounds):
            for layout in layouts:
                for v in VARIANTS:
                    configure(v)
                    for _ in range(3):
                        launch(layout, v)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(stream)
                    for _ in range(args.launches):
                        launch(layout, v)
                    b.record(stream)
                    torch.cuda.synchronize()
                    times[(layout, v[0])].append(a.elapsed_time(b) * 1e3 / args.launches)
            print(f'round {r} done', file=sys.stderr, flush=True)
    finally:
        lib.deepep_amd_exp_load_path(0)
        lib.deepep_set_launch_config(0, 0)
    summary = {}
    for (layout, name), ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        rec = dict(layout=layout, variant=name, kernel_us_median=round(med, 2), kernel_us_all=[round(t, 2) for t in ts],
                   frac=round(bytes_launch / (med * 1e-6) / 8e12, 4), bitwise_equal_to_product=exact[(layout, name)])
        print(json.dumps(rec), flush=True)
        summary[f'{layout}/{name}'] = (round(med, 2), rec['frac'], rec['bitwise_equal_to_product'])
    print(json.dumps(dict(summary=summary, bytes_per_launch=bytes_launch,
                          build_id=lib.deepep_amd_build_id().decode())), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
