"""Calibration of the memory-side request counters on the dispatch copy's access pattern (for
rocprofv3 --pmc passes, one counter set per run).  Each launch runs three times behind a 512 MB
flush; the algorithmic bytes of every kind go to gpurun_out/pmc_copycal_meta.json.

  torch_copy      dst.copy_(src), 939.5 MB read + 939.5 MB written, in order (the known reference)
  torch_scatter   recv_x[rows] = x[tok]: the expanded rows of config 2 written by torch's index kernel
  copy_expanded   deepep_dispatch_copy, expanded: x (117 MB) read once, each row stored to its ~8 slots
  copy_rows       deepep_dispatch_copy, not expanded: x read once, one row stored per token
  fused           the combine (known to count exactly: 2 x FETCH_SIZE and WRITE_SIZE = its bytes)
Kernels are told apart by name in the counter CSV (see tools/summarize_prof.py copycal)."""
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
    os.environ.setdefault('MASTER_PORT', '29619')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED, RowLayout
    T, H, K, E = 8192, 7168, 8, 256
    flush = torch.empty((512 << 20) // 4, dtype=torch.int32, device='cuda')
    g = torch.Generator(device='cuda').manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
    ex_x, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    n_exp = ex_x.shape[0]
    meta = handle.recv_src_metadata
    kern = buf.kernels
    out = {}
    # torch copy of the expanded rows' size (in order)
    src = torch.randn((n_exp, H), device='cuda', generator=g).to(torch.bfloat16)
    dst = torch.empty_like(src)
    for _ in range(3):
        flush.zero_()
        dst.copy_(src)
    out['torch_copy'] = dict(read=n_exp * H * 2, write=n_exp * H * 2)
    # torch scatter of the same expanded rows
    slots = meta[:, 2:].long()
    ok = slots >= 0
    rows = slots[ok]
    tok = (meta[:, 0].long() % T).view(-1, 1).expand(-1, K)[ok]
    for _ in range(3):
        flush.zero_()
        dst.index_copy_(0, rows, x.index_select(0, tok))
    out['torch_scatter'] = dict(read=T * H * 2, write=int(rows.numel()) * H * 2,
                                note='index_select materialises the gathered rows first (read + write of them too)')
    # the dispatch copy, expanded and not
    layout = RowLayout.make(0, 0, K)
    packed = torch.zeros((T, layout.row_bytes), dtype=torch.uint8, device='cuda')
    xb = x.view(torch.uint8).view(T, H * 2)
    recv_x = torch.empty_like(ex_x)
    recv_w = torch.zeros((n_exp,), dtype=torch.float32, device='cuda')
    for _ in range(3):
        flush.zero_()
        kern.dispatch_copy(packed, layout, T, meta, True, recv_x.view(torch.uint8), None, recv_w, x_direct=xb,
                           num_max_tokens=T)
    out['copy_expanded'] = dict(read=T * H * 2, write=n_exp * H * 2)
    recv_rows = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    recv_w2 = torch.zeros((T, K), dtype=torch.float32, device='cuda')
    for _ in range(3):
        flush.zero_()
        kern.dispatch_copy(packed, layout, T, meta, False, recv_rows.view(torch.uint8), None, recv_w2, x_direct=xb,
                           num_max_tokens=T)
    out['copy_rows'] = dict(read=T * H * 2, write=T * H * 2)
    # the fused combine
    y = torch.randn(ex_x.shape, device='cuda', generator=g).to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
    plan = handle._combine_plans[('multi', 1)]
    o = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    ow = torch.empty((T, K), dtype=torch.float32, device='cuda')
    for _ in range(3):
        flush.zero_()
        kern.combine_reduce(MODE_FUSED, y, o, T, table=plan.local_table, row_weights=ex_w, wtable=plan.local_table,
                            wsrc=ex_w, out_weights=ow)
    out['fused'] = dict(read=n_exp * H * 2, write=T * H * 2)
    torch.cuda.synchronize()
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, 'gpurun_out', 'pmc_copycal_meta.json'), 'w'))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
