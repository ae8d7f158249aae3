"""Launch each HBM-bound kernel of the path three times, a 512 MB flush before every launch, for
rocprofv3 --pmc passes (one counter set per run):
  fused    EP = 1 combine, BASELINE config 2 (weighted)
  local    EP = 8 phase A, one rank's share of config 3 (round 4's kphase tool, in git history)
  epilogue EP = 8 phase B, same rank
  copy     EP = 1 dispatch copy (expanded), config 2
Writes the algorithmic bytes per launch of each to gpurun_out/pmc_phases_meta.json.
usage: rocprofv3 --pmc FETCH_SIZE -d OUT -o pmc --output-format csv -- python3 tools/pmc_phases.py"""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29617')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from tests.plan_ref import epilogue_tables
    from deepep_amd.kernels import MODE_EPILOGUE, MODE_FUSED, MODE_LOCAL, RowLayout
    T, H, K, E, R = 8192, 7168, 8, 256, 8
    flush = torch.empty((512 << 20) // 4, dtype=torch.int32, device='cuda')
    meta_out = {}
    g = torch.Generator(device='cuda').manual_seed(0)
    # ---- EP = 1 fused combine + dispatch copy
    w, idx = torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
    ex_x, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn(ex_x.shape, device='cuda', generator=g).to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
    plan = handle._combine_plans[('multi', 1)]
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    kern = buf.kernels
    for _ in range(3):
        flush.zero_()
        kern.combine_reduce(MODE_FUSED, y, out, T, table=plan.local_table, row_weights=ex_w, wtable=plan.local_table,
                            wsrc=ex_w, out_weights=out_w)
    meta_out['fused'] = T * (K * H * 2 + H * 2 + K * 8)
    meta = handle.recv_src_metadata
    layout = RowLayout.make(0, 0, K)
    packed = torch.zeros((T, layout.row_bytes), dtype=torch.uint8, device='cuda')
    xb = x.view(torch.uint8).view(T, H * 2)
    recv_x = torch.empty_like(ex_x)
    recv_w = torch.zeros((ex_x.shape[0],), dtype=torch.float32, device='cuda')
    inv, block_offsets = handle._copy_tables           # the product's blocked destination-major copy
    for _ in range(3):
        flush.zero_()
        kern.dispatch_copy(packed, layout, T, meta, True, recv_x.view(torch.uint8), None, recv_w, x_direct=xb,
                           num_max_tokens=T, inv=inv, block_offsets=block_offsets,
                           expert_end=handle.psum_num_recv_tokens_per_expert)
    meta_out['copy'] = T * H * 2 + ex_x.shape[0] * H * 2
    # ---- EP = 8, rank 0's phases (as round 4's kphase tool)
    epr = E // R
    idx8 = torch.stack([torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1)[1] for _ in range(R)])
    local = (idx8 >= 0) & (idx8 < epr)
    recv_mask = local.any(dim=2)
    lanes = local[recv_mask]
    n_recv, n_exp = lanes.shape[0], int(lanes.sum())
    experts = idx8[recv_mask]
    ii, kk = lanes.nonzero(as_tuple=True)
    order = torch.argsort(experts[ii, kk] * n_recv + ii)
    pos = torch.empty_like(order)
    pos[order] = torch.arange(order.numel(), device='cuda')
    table_a = torch.full((n_recv, K), -1, dtype=torch.int32, device='cuda')
    table_a[ii, kk] = pos.to(torch.int32)
    y8 = torch.randn((n_exp, H), device='cuda', generator=g).to(torch.bfloat16)
    w8 = torch.rand((n_exp,), device='cuda', generator=g)
    packed8 = torch.empty((n_recv, H + 64), dtype=torch.bfloat16, device='cuda')   # the library's packed rows
    pw = packed8[:, H:].view(torch.float32)[:, :K]
    for _ in range(3):
        flush.zero_()
        kern.combine_reduce(MODE_LOCAL, y8, packed8[:, :H], n_recv, table=table_a, row_weights=w8, wtable=table_a,
                            wsrc=w8, out_weights=pw, weights_pad=32)
    meta_out['local'] = n_exp * H * 2 + n_recv * (H * 2 + K * 4)
    table_b, _, back = epilogue_tables(idx8[0], E, R)
    recv = torch.randn((sum(back), H + 64), device='cuda', generator=g).to(torch.bfloat16)
    for _ in range(3):
        flush.zero_()
        kern.combine_reduce(MODE_EPILOGUE, recv[:, :H], out, T, table=table_b)
    meta_out['epilogue'] = int((table_b >= 0).sum()) * H * 2 + T * H * 2
    torch.cuda.synchronize()
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    json.dump(meta_out, open(os.path.join(ROOT, 'gpurun_out', 'pmc_phases_meta.json'), 'w'))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
