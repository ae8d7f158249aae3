"""Does the ORDER in which output tokens are reduced matter?  (tuning aid, BASELINE config 2)

The expanded rows are grouped by expert, so a token's 8 rows sit in 8 different expert regions, and the
tokens reduced at the same moment (consecutive units) read ~all 256 regions at once.  Reordering the
units so that concurrent tokens share experts could make the gather more DRAM-page friendly.  The
phase-A scatter launch (deepep_combine_reduce_scatter: unit u's row stored at any address) reduces the
same tokens in a chosen order and writes each to its own output row; weighted LOCAL = the fused
weighted combine's bits.  Orders: identity, sorted by the lowest expert, by the lane-0 expert, by the
highest expert, random; plus the fused launch itself for reference."""
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
    os.environ.setdefault('MASTER_PORT', '29687')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                         topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    ref, _, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
    table = handle._combine_plans[('multi', 1)].local_table
    kern = buf.kernels
    s = torch.cuda.current_stream()
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    ow = torch.empty((T, K), dtype=torch.float32, device='cuda')
    nbytes = T * (K * H * 2 + H * 2 + K * 8)
    us = timeit(lambda: kern.combine_reduce(MODE_FUSED, y, out, T, table=table, row_weights=ex_w, wtable=table,
                                            wsrc=ex_w, out_weights=ow, stream=s), s)
    print(json.dumps(dict(order='fused (identity)', us=round(us, 1), tbps=round(nbytes / us / 1e6, 3))), flush=True)
    orders = {
        'identity': torch.arange(T, device='cuda'),
        'lowest_expert': torch.argsort(idx.min(dim=1).values * T + torch.arange(T, device='cuda')),
        'lane0_expert': torch.argsort(idx[:, 0] * T + torch.arange(T, device='cuda')),
        'highest_expert': torch.argsort(idx.max(dim=1).values * T + torch.arange(T, device='cuda')),
        'random': torch.randperm(T, device='cuda'),
    }
    for rnd in range(2):
        for name, perm in orders.items():
            tab = table[perm].contiguous()
            rows = (out.data_ptr() + perm.to(torch.int64) * H * 2).contiguous()
            win = (torch.tensor([out.data_ptr()], dtype=torch.int64, device='cuda'), out.numel() * 2)
            us = timeit(lambda: kern.combine_reduce_scatter(y, T, rows, table=tab, row_weights=ex_w, windows=win,
                                                            stream=s), s)
            torch.cuda.synchronize()
            print(json.dumps(dict(order=name, round=rnd, us=round(us, 1), tbps=round(nbytes / us / 1e6, 3),
                                  bitwise=bool(torch.equal(out, ref)))), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
