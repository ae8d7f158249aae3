"""Bisect of the fused combine's cost (tuning aid).

The plain-sum gather probe (tools/probe.hip gather_burst) ran 1.5-2.5 % faster than the product
kernel.  What the product adds on top of a plain gather: LDS staging of the slot table per
workgroup, the gating weights (a dependent gather of each slot's weight), the top-k weight
pass-through (one more gather + a 32-byte store per token), the FUSED epilogue (a second
rounding pass).  Each variant below removes one of them; all run on the same buffers in the same
process, interleaved over several rounds, so a difference is a property of the kernel and not of the
box.  Prints one JSON line per (round, variant) and a final summary with medians.
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
    os.environ.setdefault('MASTER_PORT', '29617')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED, MODE_LOCAL
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    scores = torch.rand((T, E), device='cuda')
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'), topk_idx=idx,
                                         topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w)
    table = handle._combine_plans[('multi', 1)].local_table
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    s = torch.cuda.current_stream()
    kern = buf.kernels
    lib = kern.lib
    rows_bytes = T * K * H * 2 + T * H * 2

    def fused(weighted, passthrough, mode=MODE_FUSED):
        return lambda: kern.combine_reduce(mode, y, out, T, table=table, row_weights=ex_w if weighted else None,
                                           wtable=table if passthrough else None, wsrc=ex_w if passthrough else None,
                                           out_weights=out_w if passthrough else None, stream=s)

    def with_config(fn, cfg=None, choice=None):
        def run():
            if cfg is not None:
                lib.deepep_set_launch_config(*cfg)
            if choice is not None:
                lib.deepep_set_kernel_choice(choice)
            try:
                fn()
            finally:
                lib.deepep_set_launch_config(0, -1, -1, 0)
                lib.deepep_set_kernel_choice(-1)
        return run

    variants = {
        'product (weighted, pass-through, LDS slots, FUSED)': fused(True, True),
        'no pass-through': fused(True, False),
        'plain sum + pass-through': fused(False, True),
        'plain sum, no pass-through': fused(False, False),
        'LOCAL (one rounding, no epilogue), weighted, no pass-through': fused(True, False, MODE_LOCAL),
        'LOCAL plain, no pass-through': fused(False, False, MODE_LOCAL),
        'slots in registers (no LDS staging)': with_config(fused(True, True), cfg=(0, 0, -1, 0)),
        '4 rows in flight': with_config(fused(True, True), cfg=(0, -1, -1, 4)),
        '4-wave workgroups': lambda: kern.combine_reduce(MODE_FUSED, y, out, T, table=table, row_weights=ex_w,
                                                         wtable=table, wsrc=ex_w, out_weights=out_w,
                                                         units_per_block=4, stream=s),
        'stores sc1 nt': with_config(fused(True, True), cfg=(0, -1, 3, 0)),
        'stores nt': with_config(fused(True, True), cfg=(0, -1, 1, 0)),
        'stores plain': with_config(fused(True, True), cfg=(0, -1, 0, 0)),
        'persistent grid (choice 5)': with_config(fused(True, True), choice=5),
        'streaming kernel (choice 1)': with_config(fused(True, True), choice=1),
    }
    rounds = int(os.environ.get('KBISECT_ROUNDS', 4))
    res = {k: [] for k in variants}
    for r in range(rounds):
        for name, fn in variants.items():
            us = timeit(fn, s, iters=30)
            res[name].append(us)
            print(json.dumps(dict(round=r, variant=name, us=round(us, 2),
                                  tbps=round(rows_bytes / us / 1e6, 3))), flush=True)
    base = statistics.median(res[next(iter(variants))])
    print(json.dumps(dict(summary={k: dict(median_us=round(statistics.median(v), 2),
                                           vs_product=round(statistics.median(v) / base, 4))
                                   for k, v in res.items()})), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
