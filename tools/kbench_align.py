"""Sensitivity of the fused combine kernel to the base address of its input / output buffers
(tuning aid): the same batch placed at several byte offsets inside a larger allocation."""
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
    os.environ.setdefault('MASTER_PORT', '29612')
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
    del x
    N = handle.num_expanded_tokens
    buf.combine(torch.zeros((N, H), dtype=torch.bfloat16, device='cuda'), handle, topk_weights=ex_w)
    plan = handle._combine_plans[('multi', 1)]
    s = torch.cuda.current_stream()
    nbytes = T * K * H * 2 + T * H * 2 + T * K * 8
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    big = torch.empty((N * H + (4 << 20),), dtype=torch.bfloat16, device='cuda')
    obig = torch.empty((T * H + (4 << 20),), dtype=torch.bfloat16, device='cuda')
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    print(json.dumps(dict(y_base_mod_2M=big.data_ptr() % (2 << 20), out_base_mod_2M=obig.data_ptr() % (2 << 20))))
    for yoff, ooff in [(0, 0), (128, 0), (2048, 0), (4096, 0), (8192, 0), (65536, 0), (1 << 20, 0), (0, 4096),
                       (0, 65536), (7168, 7168), (0, 0)]:
        y = big[yoff // 2: yoff // 2 + N * H].view(N, H)
        y.normal_()
        out = obig[ooff // 2: ooff // 2 + T * H].view(T, H)
        fn = lambda: buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=plan.local_table, row_weights=ex_w,
                                                wtable=plan.local_table, wsrc=ex_w, out_weights=out_w, stream=s)
        us = timeit(fn, s, iters=30)
        print(json.dumps(dict(y_off=yoff, out_off=ooff, us=round(us, 1), frac=round(nbytes / us / 1e3 / 8000, 4))),
              flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
