"""Per-launch timing distribution of the fused combine (diagnostic for box-to-box variance):
500 launches timed one by one with HIP events, an idle pause, 500 more; the d2d-copy and
read-only references interleaved."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(v, q):
    v = sorted(v)
    return round(v[min(len(v) - 1, int(q * len(v)))], 1)


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29671')
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
    nbytes = T * K * H * 2 + T * H * 2 + T * K * 8

    def launch():
        buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=plan.local_table, row_weights=ex_w,
                                   wtable=plan.local_table, wsrc=ex_w, out_weights=out_w, stream=s)

    def series(fn, n):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for a, b in evs:
            a.record(s)
            fn()
            b.record(s)
        torch.cuda.synchronize()
        return [a.elapsed_time(b) * 1e3 for a, b in evs]

    # same kernel, same bytes, token-major rows (table[t][k] = t*K + k): no scatter
    ident = (torch.arange(T, device='cuda').view(T, 1) * K + torch.arange(K, device='cuda').view(1, K)).to(torch.int32)
    ident = ident.contiguous()

    def launch_ident():
        buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=ident, row_weights=ex_w,
                                   wtable=ident, wsrc=ex_w, out_weights=out_w, stream=s)
    ti = series(launch_ident, 200)
    print(json.dumps(dict(what='fused_weighted_token_major_rows', p50=pct(ti, .5),
                          frac_p50=round(nbytes / pct(ti, .5) / 1e3 / 8000, 4))), flush=True)
    dst = torch.empty_like(y)
    for phase in range(2):
        ts = series(launch, 500)
        print(json.dumps(dict(phase=phase, what='fused_weighted', first10=[round(t, 1) for t in ts[:10]],
                              p10=pct(ts, .1), p50=pct(ts, .5), p90=pct(ts, .9), mean=round(sum(ts) / len(ts), 1),
                              frac_p50=round(nbytes / pct(ts, .5) / 1e3 / 8000, 4))), flush=True)
        cs = series(lambda: dst.copy_(y), 20)
        print(json.dumps(dict(phase=phase, what='d2d_copy', p50=pct(cs, .5),
                              gbps_p50=round(2 * y.numel() * 2 / pct(cs, .5) / 1e3, 1))), flush=True)
        rs = series(lambda: y.sum(dtype=torch.float32), 10)
        print(json.dumps(dict(phase=phase, what='torch_sum_read_only', p50=pct(rs, .5),
                              gbps_p50=round(y.numel() * 2 / pct(rs, .5) / 1e3, 1))), flush=True)
        time.sleep(2.0)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
