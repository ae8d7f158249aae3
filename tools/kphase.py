"""EP = 8 phase kernels on one GPU (tuning aid): one rank's share of BASELINE config 3 (8 ranks x
8192 tokens, hidden 7168, top-8 over 256 experts), uniform routing.  Phase A = the LOCAL reduce of
the ~43.4K tokens rank 0 receives (1.51 local rows each on average) into packed [partial | weights]
rows; phase B = the EPILOGUE of rank 0's own 8192 tokens over the ~5.3 partial rows each (rank
layout, ascending master lane).  Prints kernel times and GB/s of the bytes each phase moves."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    from deepep_amd.kernels import HipKernels, MODE_EPILOGUE, MODE_LOCAL
    from tests.plan_ref import epilogue_tables
    kern = HipKernels()
    R, T, H, K, E = 8, 8192, 7168, 8, 256
    epr = E // R
    g = torch.Generator(device='cuda').manual_seed(0)
    idx = torch.stack([torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1)[1] for _ in range(R)])
    # ---- phase A on rank 0: received tokens of every source rank, local lanes -> expanded rows
    local = (idx >= 0) & (idx < epr)                                   # [R, T, K] lanes on rank 0
    recv_mask = local.any(dim=2)                                       # [R, T]
    lanes = local[recv_mask]                                           # [N_recv, K]
    n_recv = lanes.shape[0]
    n_exp = int(lanes.sum())
    table_a = torch.full((n_recv, K), -1, dtype=torch.int32, device='cuda')
    # expanded rows grouped by local expert, ascending received token inside an expert (the dispatch
    # layout, dispatch_copy_epilogue.cuh:112-123)
    experts = idx[recv_mask]                                          # [N_recv, K] global experts
    ii, kk = lanes.nonzero(as_tuple=True)
    ee = experts[ii, kk]
    order = torch.argsort(ee * n_recv + ii)                           # by (expert, token)
    pos = torch.empty_like(order)
    pos[order] = torch.arange(order.numel(), device='cuda')
    table_a[ii, kk] = pos.to(torch.int32)
    y = torch.randn((n_exp, H), device='cuda', generator=g).to(torch.bfloat16)
    w = torch.rand((n_exp,), device='cuda', generator=g)
    packed = torch.empty((n_recv, H + 64), dtype=torch.bfloat16, device='cuda')   # the library's packed rows
    pw = packed[:, H:].view(torch.float32)[:, :K]
    s = torch.cuda.current_stream()
    bytes_a = n_exp * H * 2 + n_recv * (H * 2 + K * 4)
    for rif in (8, 4, 2):
        assert kern.lib.deepep_set_launch_config(0, -1, -1, rif) == 0
        for weighted, upb in ((True, 8), (True, 4), (False, 4)):
            us = timeit(lambda: kern.combine_reduce(MODE_LOCAL, y, packed[:, :H], n_recv, table=table_a,
                                                    row_weights=w if weighted else None, wtable=table_a, wsrc=w,
                                                    out_weights=pw, weights_pad=32, units_per_block=upb, stream=s), s)
            print(json.dumps(dict(phase='A', weighted=weighted, rows_in_flight=rif, upb=upb, units=n_recv,
                                  rows=n_exp, us=round(us, 1), gbps=round(bytes_a / us / 1e3, 1))), flush=True)
    kern.lib.deepep_set_launch_config(0, -1, -1, 0)
    # the library's kernels on the automatic shape, forced (0 item, 1 streaming, 2 streaming 1 vector/lane)
    for rnd in range(2):
        for choice in (0, 1, 2, 3, 4, 5):
            assert kern.lib.deepep_set_kernel_choice(choice) == 0
            us = timeit(lambda: kern.combine_reduce(MODE_LOCAL, y, packed[:, :H], n_recv, table=table_a, row_weights=w,
                                                    wtable=table_a, wsrc=w, out_weights=pw, weights_pad=32, stream=s), s)
            print(json.dumps(dict(phase='A', kernel=('item', 'stream', 'stream_vpt1', 'stream_persistent', 'item_xcd', 'item_persistent')[choice], round=rnd, us=round(us, 1),
                                  gbps=round(bytes_a / us / 1e3, 1))), flush=True)
    kern.lib.deepep_set_kernel_choice(-1)
    # packed-row stride: 2H + 32 B (the weights' tail; rows only 32-byte aligned, so every 2 KiB chunk
    # store straddles partial 128-byte lines) vs 2H + 128 B (128-byte aligned rows) vs 2H (no tail)
    for rnd in range(2):
        for tail, pad in ((16, 0), (64, 0), (64, 32), (0, 0), (64, -1)):
            pk = torch.empty((n_recv, H + tail), dtype=torch.bfloat16, device='cuda')
            pkw = pk[:, H:].view(torch.float32)[:, :K] if tail and pad >= 0 else None     # -1: tail left unwritten
            pad = max(pad, 0)
            for choice in (0, 5):
                assert kern.lib.deepep_set_kernel_choice(choice) == 0
                us = timeit(lambda: kern.combine_reduce(MODE_LOCAL, y, pk[:, :H], n_recv, table=table_a, row_weights=w,
                                                        wtable=table_a if pkw is not None else None,
                                                        wsrc=w if pkw is not None else None,
                                                        out_weights=pkw, weights_pad=pad, stream=s), s)
                print(json.dumps(dict(phase='A_stride', row_bytes=(H + tail) * 2, weights_pad=pad,
                                      weights_written=pkw is not None,
                                      kernel=('item', 'item_persistent')[choice // 5],
                                      round=rnd, us=round(us, 1), gbps=round(bytes_a / us / 1e3, 1))), flush=True)
            del pk
    kern.lib.deepep_set_kernel_choice(-1)
    # output store policy of phase A (40 % of its bytes are the partial rows): plain / nt / sc1
    for rnd in range(2):
        for pol in (0, 1, 2, 3):
            assert kern.lib.deepep_set_launch_config(0, -1, pol, 0) == 0
            us = timeit(lambda: kern.combine_reduce(MODE_LOCAL, y, packed[:, :H], n_recv, table=table_a, row_weights=w,
                                                    wtable=table_a, wsrc=w, out_weights=pw, weights_pad=32, stream=s), s)
            print(json.dumps(dict(phase='A_store', policy=('plain', 'nt', 'sc1', 'sc1 nt')[pol], round=rnd,
                                  us=round(us, 1), gbps=round(bytes_a / us / 1e3, 1))), flush=True)
    kern.lib.deepep_set_launch_config(0, -1, -1, 0)
    # same bytes, rows in a random order (no expert grouping): the scatter's cost
    perm = torch.randperm(n_exp, device='cuda', generator=g).to(torch.int32)
    table_r = torch.full((n_recv, K), -1, dtype=torch.int32, device='cuda')
    table_r[lanes] = perm
    us = timeit(lambda: kern.combine_reduce(MODE_LOCAL, y, packed[:, :H], n_recv, table=table_r, row_weights=w,
                                            wtable=table_r, wsrc=w, out_weights=pw, stream=s), s)
    print(json.dumps(dict(phase='A_random_rows', us=round(us, 1), gbps=round(bytes_a / us / 1e3, 1))), flush=True)
    # a plain copy of the same bytes (read n_exp rows in order, write n_recv rows) for reference
    src_c = y[:n_recv]
    us = timeit(lambda: packed[:, :H].copy_(src_c), s)
    print(json.dumps(dict(phase='torch_copy_n_recv_rows', us=round(us, 1),
                          gbps=round(2 * n_recv * H * 2 / us / 1e3, 1))), flush=True)
    # ---- phase B on rank 0: its own tokens over the partial rows it receives (rank layout)
    table_b, row_of_lane, back = epilogue_tables(idx[0], E, R)
    n_back = sum(back)
    recv = torch.randn((n_back, H + 64), device='cuda', generator=g).to(torch.bfloat16)
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    valid_b = int((table_b >= 0).sum())
    bytes_b = valid_b * H * 2 + T * H * 2
    for rif in (8, 4, 2):
        assert kern.lib.deepep_set_launch_config(0, -1, -1, rif) == 0
        for upb in (8, 4):
            us = timeit(lambda: kern.combine_reduce(MODE_EPILOGUE, recv[:, :H], out, T, table=table_b,
                                                    units_per_block=upb, stream=s), s)
            print(json.dumps(dict(phase='B', rows_in_flight=rif, upb=upb, units=T, rows=valid_b, us=round(us, 1),
                                  gbps=round(bytes_b / us / 1e3, 1))), flush=True)
    kern.lib.deepep_set_launch_config(0, -1, -1, 0)
    for rnd in range(2):
        for choice in (0, 1, 2, 3, 4, 5):
            assert kern.lib.deepep_set_kernel_choice(choice) == 0
            us = timeit(lambda: kern.combine_reduce(MODE_EPILOGUE, recv[:, :H], out, T, table=table_b, stream=s), s)
            print(json.dumps(dict(phase='B', kernel=('item', 'stream', 'stream_vpt1', 'stream_persistent', 'item_xcd', 'item_persistent')[choice], round=rnd, us=round(us, 1),
                                  gbps=round(bytes_b / us / 1e3, 1))), flush=True)
    kern.lib.deepep_set_kernel_choice(-1)
    # EP = 1 fused kernel, config 2 (8 rows per token, 65536 random expanded rows)
    tab1 = torch.randperm(T * K, device='cuda', generator=g).to(torch.int32).view(T, K).contiguous()
    y1 = torch.randn((T * K, H), device='cuda', generator=g).to(torch.bfloat16)
    w1 = torch.rand((T * K,), device='cuda', generator=g)
    ow = torch.empty((T, K), device='cuda')
    for rif in (8, 4, 2):
        assert kern.lib.deepep_set_launch_config(0, -1, -1, rif) == 0
        for upb in (8, 4):
            us = timeit(lambda: kern.combine_reduce(2, y1, out, T, table=tab1, row_weights=w1, wtable=tab1, wsrc=w1,
                                                    out_weights=ow, units_per_block=upb, stream=s), s)
            print(json.dumps(dict(phase='fused_ep1', rows_in_flight=rif, upb=upb, us=round(us, 1),
                                  gbps=round(T * (K * H * 2 + H * 2 + K * 8) / us / 1e3, 1))), flush=True)
    kern.lib.deepep_set_launch_config(0, -1, -1, 0)
    # reference points: EP = 1 fused-kernel bytes over the same time budget
    alg = T * (K * H * 2 + H * 2 + K * 8)
    print(json.dumps(dict(algorithmic_bytes_per_rank=alg, note='reduce_only GB/s per rank = alg / (A + B)')))


if __name__ == '__main__':
    main()
