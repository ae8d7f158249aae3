"""Workgroup-shape A/B of the fused combine (tuning aid): 4 waves (units_per_block=4) vs the default 8."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29616')
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
    tab = handle._combine_plans[('multi', 1)].local_table
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    s = torch.cuda.current_stream()
    nbytes = T * K * H * 2 + T * H * 2 + T * K * 8
    ref = None
    for rnd in range(3):
        for waves in (4, 0):
            fn = lambda: buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=tab, row_weights=ex_w, wtable=tab,
                                                    wsrc=ex_w, out_weights=out_w, units_per_block=waves, stream=s)
            fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            eq = bool(torch.equal(out, ref))
            us = timeit(fn, s, iters=30)
            print(json.dumps(dict(round=rnd, waves=waves or 8, us=round(us, 1), frac=round(nbytes / us / 1e3 / 8000, 4),
                                  equal=eq)), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
