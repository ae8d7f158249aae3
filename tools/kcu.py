"""Combine time under a CU budget (ElasticBuffer.combine(num_sms=n): kernels on a
hipExtStreamCreateWithCUMask stream), BASELINE config 2 at EP = 1: what the combine costs when it
leaves CUs to overlapping compute.

Per budget: `api` = combine(num_sms=n) from the default stream (two cross-stream hops per call),
`api_on_budget_stream` = the same call issued from the budget stream itself (no hops), `kernel` = the
fused launch alone on the budget stream (the default: item kernel on its full grid, 4 rows in flight
per lane on a budget), `kernel_stream` = the streaming kernel forced (deepep_set_kernel_choice(3),
persistent grid), `kernel_persistent` = the item kernel on a persistent grid sized to the budget
(choice 5, round 2's budget default), `kernel_r8` = the full grid with 8 rows in flight per lane."""
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
    from deepep_amd.kernels import MODE_FUSED
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                         topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    ref, _, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
    plan = handle._combine_plans[('multi', 1)]
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    nbytes = T * (K * H * 2 + H * 2 + K * 8)
    lib = buf.kernels.lib

    def timed(fn, s, n=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(n):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    # the reference's bandwidth-model CU counts (get_theoretical_num_sms, elastic.py:728-834) that a
    # DEEPEP_COMBINE_CUS=handle combine is confined to at EP = 2, 4, 8 (this shape's routing)
    model = {}
    saved = (buf.num_ranks, buf.num_nvlink_ranks)
    for r in (2, 4, 8):
        buf.num_ranks = buf.num_nvlink_ranks = r
        model[buf.get_theoretical_num_sms(E, K)] = f'model_ep{r}'
    buf.num_ranks, buf.num_nvlink_ranks = saved
    print(json.dumps(dict(model_num_sms={v: k for k, v in model.items()})), flush=True)
    for n in [0, 224, 192, 160, 128, 96, 64, 32, 24, 16, 8] + sorted(model, reverse=True):
        row = dict(num_sms=n, tag=model.get(n, ''))
        s0 = torch.cuda.current_stream()
        row['api_us'] = round(timed(lambda: buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True,
                                                        num_sms=n), s0), 1)
        bs = buf.get_cu_budget_stream(n) if n else s0
        with torch.cuda.stream(bs):
            res = {}

            def api():
                res['o'] = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True, num_sms=n)[0]
            row['api_on_budget_stream_us'] = round(timed(api, bs), 1)

            def kern():
                buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=plan.local_table, row_weights=ex_w,
                                           wtable=plan.local_table, wsrc=ex_w, out_weights=out_w, stream=bs)
            row['kernel_us'] = round(timed(kern, bs), 1)
            torch.cuda.synchronize()
            row['bitwise'] = bool(torch.equal(out, ref) and torch.equal(res['o'], ref))
            lib.deepep_set_kernel_choice(3)
            row['kernel_stream_us'] = round(timed(kern, bs), 1)
            lib.deepep_set_kernel_choice(5)                    # the item kernel on a persistent grid
            row['kernel_persistent_us'] = round(timed(kern, bs), 1)
            lib.deepep_set_kernel_choice(-1)
            lib.deepep_set_launch_config(0, -1, -1, 8)         # full grid, 8 rows in flight per lane
            row['kernel_r8_us'] = round(timed(kern, bs), 1)
            lib.deepep_set_launch_config(0, -1, -1, 0)
            torch.cuda.synchronize()
            row['bitwise'] = row['bitwise'] and bool(torch.equal(out, ref))
        for k in ('api_us', 'api_on_budget_stream_us', 'kernel_us', 'kernel_stream_us', 'kernel_persistent_us',
                  'kernel_r8_us'):
            row[k.replace('_us', '_tbps')] = round(nbytes / row[k] / 1e6, 2)
        print(json.dumps(row), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
