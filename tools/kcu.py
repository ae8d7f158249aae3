"""Combine time under a CU budget (ElasticBuffer.combine(num_sms=n): kernels on a
hipExtStreamCreateWithCUMask stream), BASELINE config 2 at EP = 1: shows the budget is honoured
(time ~ 1 / CUs until HBM saturates) and what the combine costs when it leaves CUs to compute."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29681')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                         topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    nbytes = T * (K * H * 2 + H * 2 + K * 8)
    s = torch.cuda.current_stream()
    for n in (0, 256, 224, 192, 160, 128, 96, 64, 32, 16):
        def step():
            return buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True, num_sms=n)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(20):
            step()
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 20
        print(json.dumps(dict(num_sms=n, us_per_call=round(us, 1), gbps=round(nbytes / us / 1e3, 1))), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
