"""Phase A under its three store policies, for rocprofv3 --pmc passes (one counter set per run): rank 0's
share of the EP = R combine (R from argv, default 4; bench.py's shape: 8192 tokens x 7168 x top-8 over 256
experts, uniform routing, weighted), launched with sc1 everywhere, sc1 nt everywhere and per unit (sc1 at
>= 3 reduced rows, else sc1 nt; the default), 5 times each behind a 512 MB flush.  The three launches have
different kernel names (the store policy is a template argument: 16, 18, 1003), so one trace separates them.
Writes gpurun_out/pmc_policy_meta.json (units, rows, algorithmic bytes).
usage: rocprofv3 --pmc FETCH_SIZE -d OUT -o pmc --output-format csv -- python3 tools/pmc_policy.py 4"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    torch.cuda.set_device(0)
    from deepep_amd.kernels import HipKernels, MODE_LOCAL
    kern = HipKernels()
    T, H, K, E = 8192, 7168, 8, 256
    epr = E // R
    g = torch.Generator(device='cuda').manual_seed(0)
    idx = torch.stack([torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1)[1] for _ in range(R)])
    local = (idx >= 0) & (idx < epr)
    lanes = local[local.any(dim=2)]
    n_recv, n_exp = lanes.shape[0], int(lanes.sum())
    table = torch.full((n_recv, K), -1, dtype=torch.int32, device='cuda')
    experts = idx[local.any(dim=2)]
    ii, kk = lanes.nonzero(as_tuple=True)
    order = torch.argsort(experts[ii, kk] * n_recv + ii)
    pos = torch.empty_like(order)
    pos[order] = torch.arange(order.numel(), device='cuda')
    table[ii, kk] = pos.to(torch.int32)
    y = torch.randn((n_exp, H), device='cuda', generator=g).to(torch.bfloat16)
    w = torch.rand((n_exp,), device='cuda', generator=g)
    packed = torch.zeros((n_recv, H + 64), dtype=torch.bfloat16, device='cuda')
    pw = packed.view(torch.float32)[:, H // 2:H // 2 + K]
    flush = torch.empty((512 << 20) // 4, dtype=torch.int32, device='cuda')
    s = torch.cuda.current_stream()
    for pol in (2, 3, 4):                       # launch-config store policy: sc1, sc1 nt, per unit
        assert kern.lib.deepep_set_launch_config(0, -1, pol, 0) == 0
        for _ in range(5):
            flush.fill_(1)
            kern.combine_reduce(MODE_LOCAL, y, packed[:, :H], n_recv, table=table, row_weights=w, wtable=table,
                                wsrc=w, out_weights=pw, weights_pad=32, stream=s)
    kern.lib.deepep_set_launch_config(0, -1, -1, 0)
    torch.cuda.synchronize()
    valid_per_unit = (table >= 0).sum(dim=1)
    os.makedirs('gpurun_out', exist_ok=True)
    json.dump(dict(ranks=R, units=n_recv, rows=n_exp, bytes=n_exp * H * 2 + n_recv * (H * 2 + K * 4),
                   units_ge3=int((valid_per_unit >= 3).sum())), open('gpurun_out/pmc_policy_meta.json', 'w'))


if __name__ == '__main__':
    main()
