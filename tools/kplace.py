"""Does the physical placement of the expanded rows change the fused combine's time?  The same data
copied into several fresh allocations (different physical pages), each timed back to back on the
same table, interleaved over rounds (diagnostic for the per-process spread)."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from probe import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29675')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                         topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E, do_expand=True)
    y0 = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    buf.combine(y0, handle, topk_weights=ex_w)
    table = handle._combine_plans[('multi', 1)].local_table
    lib = buf.kernels.lib
    assert lib.deepep_set_kernel_choice(0) == 0
    copies = [y0] + [y0.clone() for _ in range(3)]
    outs = [torch.empty((T, H), dtype=torch.bfloat16, device='cuda') for _ in range(2)]
    ow = torch.empty((T, K), dtype=torch.float32, device='cuda')
    s = torch.cuda.current_stream()
    res = {}
    iters, warm = int(os.environ.get('KPLACE_ITERS', 30)), int(os.environ.get('KPLACE_WARM', 3))
    for rnd in range(int(os.environ.get('KPLACE_ROUNDS', 3))):
        for i, y in enumerate(copies):
            for j, out in enumerate(outs):
                def f():
                    buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=table, row_weights=ex_w, wtable=table,
                                               wsrc=ex_w, out_weights=ow, stream=s)
                res[f'r{rnd} rows{i} out{j}'] = round(timeit(f, iters, warm), 1)
    lib.deepep_set_kernel_choice(-1)
    print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
