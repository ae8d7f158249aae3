"""Launch the fused combine kernel a few times on BASELINE config 2 (for rocprofv3 --pmc passes).

usage: rocprofv3 --pmc FETCH_SIZE -d OUT -o pmc --output-format csv -- python3 tools/pmc_run.py [--plain] [--b2b]
--b2b: 20 launches back to back without the flush (the bench's loop), for per-process counter comparisons.
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    weighted = '--plain' not in sys.argv
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29613')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    scores = torch.rand((T, E), device='cuda')
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                         topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w)
    plan = handle._combine_plans[('multi', 1)]
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    # flush the 256 MiB Infinity Cache between launches, as the reference's bench does (testing.py:12-21)
    flush = torch.empty(512 * 1024 * 1024 // 4, dtype=torch.int32, device='cuda')
    b2b = '--b2b' in sys.argv
    for _ in range(20 if b2b else 5):
        if not b2b:
            flush.zero_()
        buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=plan.local_table,
                                   row_weights=ex_w if weighted else None,
                                   wtable=plan.local_table, wsrc=ex_w, out_weights=out_w)
    torch.cuda.synchronize()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
