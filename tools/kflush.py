"""Why a cache flush before each launch (the reference's bench_kineto protocol,
deep_ep/utils/testing.py:12-21) slows the fused combine: each launch timed alone with HIP events
after (a) nothing, (b) a 512 MB write flush (zero_, the protocol), (c) a 512 MB read flush (a
reduction over the same buffer: evicts without leaving dirty lines), (d) the write flush followed
by an idle spin (torch.cuda._sleep) so its dirty lines can drain before the launch."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29673')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'), topk_idx=idx,
                                         topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w)
    plan = handle._combine_plans[('multi', 1)]
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    s = torch.cuda.current_stream()
    flush = torch.empty((512 << 20) // 4, dtype=torch.int32, device='cuda')
    sink = torch.empty((), dtype=torch.int64, device='cuda')

    def launch():
        buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=plan.local_table, row_weights=ex_w,
                                   wtable=plan.local_table, wsrc=ex_w, out_weights=out_w, stream=s)

    def series(before, n=60):  # noqa: E306
        evs = []
        for _ in range(n):
            before()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            launch()
            b.record(s)
            evs.append((a, b))
        torch.cuda.synchronize()
        v = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
        return dict(median=round(v[len(v) // 2], 1), p10=round(v[len(v) // 10], 1), p90=round(v[9 * len(v) // 10], 1))

    lib = buf.kernels.lib
    for _ in range(10):
        launch()
    # output store policy under the write flush (0 plain, 1 nt, 2 sc1 = the default)
    by_store = {}
    for pol in (0, 1, 2):
        assert lib.deepep_set_launch_config(0, -1, pol, 0) == 0
        for _ in range(5):
            launch()
        by_store[pol] = {'none': series(lambda: None, 30), 'write_flush': series(lambda: flush.zero_(), 30)}
    assert lib.deepep_set_launch_config(0, -1, -1, 0) == 0
    print(json.dumps({'store_policy': by_store}))
    res = {
        'none': series(lambda: None),
        'write_flush': series(lambda: flush.zero_()),
        'read_flush': series(lambda: torch.sum(flush, dim=0, dtype=torch.int64, out=sink)),
        'write_flush_then_idle_200us': series(lambda: (flush.zero_(), torch.cuda._sleep(200000))),
        'idle_200us': series(lambda: torch.cuda._sleep(200000)),
    }
    print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
