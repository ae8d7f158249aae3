"""Launch shape of the fused combine under a CU budget: the item kernel on its
full grid (deepep_set_kernel_choice(6)) with every workgroup shape (4 / 8 waves), rows in flight per
lane (2 / 4 / 8) and vectors per lane (1 / 2), against the persistent default, BASELINE config 2 at
EP = 1, on budget streams of several sizes.  Each variant is checked bitwise against the default."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29682')
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

    variants = [('default', -1, 0, 0, 0)]
    for upb in (8, 4):
        for rows in (2, 4, 8):
            for vpt in (2, 1):
                variants.append((f'grid_w{upb}_r{rows}_v{vpt}', 6, upb, rows, vpt))
    for n in (0, 224, 160, 128, 64, 32):
        bs = buf.get_cu_budget_stream(n) if n else torch.cuda.current_stream()
        row = dict(num_sms=n)
        ok = True
        with torch.cuda.stream(bs):
            for name, choice, upb, rows, vpt in variants:
                lib.deepep_set_kernel_choice(choice)
                lib.deepep_set_launch_config(vpt, -1, -1, rows)

                def kern():
                    buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=plan.local_table, row_weights=ex_w,
                                               wtable=plan.local_table, wsrc=ex_w, out_weights=out_w,
                                               units_per_block=upb, stream=bs)
                out.zero_()
                us = timed(kern, bs)
                torch.cuda.synchronize()
                ok = ok and bool(torch.equal(out, ref))
                row[name] = round(us, 1)
            lib.deepep_set_kernel_choice(-1)
            lib.deepep_set_launch_config(0, -1, -1, 0)
        best = min((k for k in row if k not in ('num_sms',)), key=lambda k: row[k])
        row['bitwise'] = ok
        row['best'] = best
        row['best_tbps'] = round(nbytes / row[best] / 1e6, 2)
        print(json.dumps(row), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
