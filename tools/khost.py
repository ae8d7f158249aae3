"""Host time of one ElasticBuffer.combine / dispatch call at BASELINE config 2 on the GPU (tuning aid):
the wall time per call over back-to-back calls, the host part alone (until the call returns), and a
cProfile of the host path.  A call whose host part approaches its GPU time would make a loop of calls
host-bound."""
import cProfile
import json
import os
import pstats
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29643')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    x = torch.randn((T, H), device='cuda').to(torch.bfloat16)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    ex_x, _, ex_w, h, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn(ex_x.shape, device='cuda').to(torch.bfloat16)
    calls = {
        'combine (weighted)': lambda: buf.combine(y, h, topk_weights=ex_w, apply_topk_weights=True),
        'dispatch fresh': lambda: buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True),
        'dispatch cached': lambda: buf.dispatch(x, topk_weights=w, do_expand=True, handle=h),
    }
    n = 100
    for name, fn in calls.items():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        host = 0.0
        t0 = time.perf_counter()
        for _ in range(n):
            t1 = time.perf_counter()
            fn()
            host += time.perf_counter() - t1
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / n
        print(json.dumps(dict(call=name, us=round(el * 1e6, 1), host_us=round(host / n * 1e6, 1))), flush=True)
    # The bench's timed region (barrier + sync, K steps, sync + barrier + sync) at several K: the
    # intercept is the region's fixed cost, which the driver's 20-step run spreads over its steps.
    step = calls['combine (weighted)']
    for K in (0, 1, 2, 5, 20, 100):
        rows = []
        for _ in range(7):
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            t_first = None
            for i in range(K):
                step()
                if i == 0:
                    t_first = time.perf_counter() - t0
            torch.cuda.synchronize()
            t_sync = time.perf_counter() - t0
            dist.barrier()
            t_bar = time.perf_counter() - t0
            torch.cuda.synchronize()
            rows.append((time.perf_counter() - t0, t_sync, t_bar, t_first or 0.0))
        med = sorted(rows)[3]
        print(json.dumps(dict(region_steps=K, region_us=round(med[0] * 1e6, 1), until_sync_us=round(med[1] * 1e6, 1),
                              until_barrier_us=round(med[2] * 1e6, 1), first_call_host_us=round(med[3] * 1e6, 1))),
              flush=True)
    for name, fn in calls.items():
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(n):
            fn()
        pr.disable()
        torch.cuda.synchronize()
        print(f'--- cProfile: {name}, {n} calls')
        pstats.Stats(pr).sort_stats('tottime').print_stats(18)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
