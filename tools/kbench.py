"""Kernel-level sweep of the fused combine launch (tuning aid, not the driver's bench).

Times deepep_combine_reduce(FUSED) on BASELINE config 2 for several LDS tile heights,
plain and weighted, against a device-to-device copy of the same bytes as a ceiling.
Prints one JSON line per variant.
"""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, stream, iters=20, warm=3):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters     # us


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29611')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    scores = torch.rand((T, E), device='cuda')
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    x = torch.zeros((T, H), dtype=torch.bfloat16, device='cuda')
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w)
    plan = handle._combine_plans[('multi', 1)]
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    s = torch.cuda.current_stream()
    nbytes = T * K * H * 2 + T * H * 2 + T * K * 8
    copy_dst = torch.empty_like(y)
    us = timeit(lambda: copy_dst.copy_(y), s)
    print(json.dumps(dict(variant='d2d_copy_939MB', us=round(us, 1), gbps=round(2 * y.numel() * 2 / us / 1e3, 1))))
    us = timeit(lambda: copy_dst.fill_(1.0), s)
    print(json.dumps(dict(variant='fill_939MB (write only)', us=round(us, 1), gbps=round(y.numel() * 2 / us / 1e3, 1))))
    del copy_dst
    lib = buf.kernels.lib
    configs = [  # (vec_per_lane, stage_lds, store_policy); 0/-1 = auto
        (0, -1, -1), (2, 1, 2), (2, 0, 2), (1, 1, 2), (1, 0, 2), (2, 1, 0), (2, 1, 1), (2, 0, 0)]
    for weighted in (True, False):
        for cfg in configs:
            assert lib.deepep_set_launch_config(*cfg, 0) == 0
            fn = lambda: buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=plan.local_table,
                                                    row_weights=ex_w if weighted else None,
                                                    wtable=plan.local_table, wsrc=ex_w, out_weights=out_w, stream=s)
            us = timeit(fn, s)
            print(json.dumps(dict(variant=f'fused_{"w" if weighted else "p"}_cfg{cfg}', us=round(us, 1),
                                  gbps=round(nbytes / us / 1e3, 1), frac=round(nbytes / us / 1e3 / 8000, 4))),
                  flush=True)
    lib.deepep_set_launch_config(0, -1, -1, 0)
    # read-only ceiling: sum of all expanded rows (torch reduction kernel)
    us = timeit(lambda: y.sum(dtype=torch.float32), s, iters=10)
    print(json.dumps(dict(variant='torch_sum_939MB', us=round(us, 1), gbps=round(y.numel() * 2 / us / 1e3, 1))))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
