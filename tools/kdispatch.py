"""Fresh vs sync-free vs cached dispatch wall time at BASELINE config 2 (tuning aid).

One JSON line per mode: the wall time of ElasticBuffer.dispatch(do_expand=True) over 50 calls, and of
its host part alone (the time until the call returns, the GPU left to drain).  Run under
`rocprofv3 --kernel-trace` to see the launches and the gaps between them (tools/summarize_prof.py
timeline)."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29641')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    scores = torch.rand((T, E), device='cuda')
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    x = torch.randn((T, H), device='cuda').to(torch.bfloat16)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, _, h, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    modes = {
        'fresh (do_cpu_sync=True)': lambda: buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True),
        'fresh sync-free (do_cpu_sync=False)': lambda: buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E,
                                                                   do_expand=True, do_cpu_sync=False),
        'cached handle': lambda: buf.dispatch(x, topk_weights=w, do_expand=True, handle=h),
    }
    n = 50
    nbytes = T * H * 2 + h.num_expanded_tokens * H * 2
    for rnd in range(2):
        for name, fn in modes.items():
            for _ in range(3):
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
            print(json.dumps(dict(round=rnd, mode=name, us=round(el * 1e6, 1), host_us=round(host / n * 1e6, 1),
                                  gbps=round(nbytes / el / 1e9, 1))), flush=True)
    if os.environ.get('KDISPATCH_CPROFILE'):
        import cProfile
        import pstats
        for name, fn in modes.items():
            pr = cProfile.Profile()
            pr.enable()
            for _ in range(n):
                fn()
            pr.disable()
            torch.cuda.synchronize()
            print(f'--- cProfile: {name}, {n} calls')
            pstats.Stats(pr).sort_stats('tottime').print_stats(25)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
