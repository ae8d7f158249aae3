"""The EP = 8 phase kernels exactly as the library launches them, nothing else (for a clean rocprofv3
--kernel-trace --stats summary): one rank's share of BASELINE config 3 (tools/kphase.py's shapes),
phase A = the LOCAL reduce into the line-aligned packed rows [partial | 128-byte weight line], phase B
= the EPILOGUE over the partial rows with the weight pass-through, 50 launches each."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def setup():
    """The phase A / phase B launches of one rank's share of config 3: (launch_a, launch_b, bytes_a, bytes_b)."""
    from deepep_amd.handle import packed_row_layout
    from deepep_amd.kernels import HipKernels, MODE_EPILOGUE, MODE_LOCAL
    from tests.plan_ref import epilogue_tables
    kern = HipKernels()
    R, T, H, K, E = 8, 8192, 7168, 8, 256
    epr = E // R
    g = torch.Generator(device='cuda').manual_seed(0)
    idx = torch.stack([torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1)[1] for _ in range(R)])
    local = (idx >= 0) & (idx < epr)
    recv_mask = local.any(dim=2)
    lanes = local[recv_mask]
    n_recv, n_exp = lanes.shape[0], int(lanes.sum())
    experts = idx[recv_mask]
    ii, kk = lanes.nonzero(as_tuple=True)
    order = torch.argsort(experts[ii, kk] * n_recv + ii)
    pos = torch.empty_like(order)
    pos[order] = torch.arange(order.numel(), device='cuda')
    table_a = torch.full((n_recv, K), -1, dtype=torch.int32, device='cuda')
    table_a[ii, kk] = pos.to(torch.int32)
    y = torch.randn((n_exp, H), device='cuda', generator=g).to(torch.bfloat16)
    w = torch.rand((n_exp,), device='cuda', generator=g)
    row_bytes, w_off, w_pad = packed_row_layout(H, K)
    packed = torch.empty((n_recv, row_bytes // 2), dtype=torch.bfloat16, device='cuda')
    pw = packed.view(torch.float32)[:, w_off // 4:w_off // 4 + K]
    table_b, row_of_lane, back = epilogue_tables(idx[0], E, R)
    recv = torch.randn((sum(back), row_bytes // 2), device='cuda', generator=g).to(torch.bfloat16)
    wtable_b = torch.where(row_of_lane >= 0, row_of_lane * (row_bytes // 4) + w_off // 4 + torch.arange(K, device='cuda'),
                           torch.full_like(row_of_lane, -1)).to(torch.int32).contiguous()
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    bytes_a = n_exp * H * 2 + n_recv * (H * 2 + K * 4)
    bytes_b = int((table_b >= 0).sum()) * H * 2 + T * H * 2 + T * K * 4

    def launch_a(stream):
        kern.combine_reduce(MODE_LOCAL, y, packed[:, :H], n_recv, table=table_a, row_weights=w, wtable=table_a, wsrc=w,
                            out_weights=pw, weights_pad=w_pad, stream=stream)

    def launch_b(stream):
        kern.combine_reduce(MODE_EPILOGUE, recv[:, :H], out, T, table=table_b, wtable=wtable_b,
                            wsrc=recv.view(torch.float32).view(-1), out_weights=out_w, stream=stream)
    return launch_a, launch_b, bytes_a, bytes_b, dict(units_a=n_recv, rows_a=n_exp)


def main():
    torch.cuda.set_device(0)
    launch_a, launch_b, bytes_a, bytes_b, info = setup()
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for _ in range(3):
        launch_a(s)
    ev[0].record(s)
    for _ in range(50):
        launch_a(s)
    ev[1].record(s)
    for _ in range(3):
        launch_b(s)
    ev[2].record(s)
    for _ in range(50):
        launch_b(s)
    ev[3].record(s)
    torch.cuda.synchronize()
    a_us = ev[0].elapsed_time(ev[1]) * 1e3 / 50
    b_us = ev[2].elapsed_time(ev[3]) * 1e3 / 50
    print(json.dumps(dict(phase_a_us=round(a_us, 1), phase_a_bytes=bytes_a, phase_a_gbps=round(bytes_a / a_us / 1e3, 1),
                          phase_b_us=round(b_us, 1), phase_b_bytes=bytes_b, phase_b_gbps=round(bytes_b / b_us / 1e3, 1),
                          **info)), flush=True)


if __name__ == '__main__':
    main()
