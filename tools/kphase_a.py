"""Phase A of EP = 8 (one rank's share of BASELINE config 3) under the launch shapes and store
policies the verdict asked about (tuning aid): sc1 vs sc1 nt stores into the RCCL send buffer, 4- vs
8-wave workgroups (LDS slots), 4 vs 8 rows in flight.  Interleaved rounds, medians; every variant's
packed rows are checked bit for bit against the default's.  Prints one JSON line per variant and a
summary line."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    from deepep_amd.kernels import HipKernels, MODE_LOCAL
    kern = HipKernels()
    R, T, H, K, E = 8, 8192, 7168, 8, 256
    epr = E // R
    g = torch.Generator(device='cuda').manual_seed(0)
    idx = torch.stack([torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1)[1] for _ in range(R)])
    local = (idx >= 0) & (idx < epr)
    recv_mask = local.any(dim=2)
    lanes = local[recv_mask]
    n_recv = lanes.shape[0]
    n_exp = int(lanes.sum())
    table_a = torch.full((n_recv, K), -1, dtype=torch.int32, device='cuda')
    experts = idx[recv_mask]
    ii, kk = lanes.nonzero(as_tuple=True)
    ee = experts[ii, kk]
    order = torch.argsort(ee * n_recv + ii)
    pos = torch.empty_like(order)
    pos[order] = torch.arange(order.numel(), device='cuda')
    table_a[ii, kk] = pos.to(torch.int32)
    y = torch.randn((n_exp, H), device='cuda', generator=g).to(torch.bfloat16)
    w = torch.rand((n_exp,), device='cuda', generator=g)
    row_elems = H + 64                                  # the library's packed row: 14336 + 128 B
    s = torch.cuda.current_stream()
    bytes_a = n_exp * H * 2 + n_recv * (H * 2 + K * 4)
    variants = []
    for pol in (2, 3):                                  # launch-config store policy: 2 sc1, 3 sc1 nt
        for upb in (4, 8):
            for rif in (4, 8):
                variants.append((pol, upb, rif))
    ref = None
    outs = {}
    times = {v: [] for v in variants}
    rounds = int(os.environ.get('KPHASE_A_ROUNDS', 5))
    for weighted in (True, False):
        ref = None
        for rnd in range(rounds):
            for v in variants:
                pol, upb, rif = v
                assert kern.lib.deepep_set_launch_config(0, -1, pol, rif) == 0
                packed = torch.zeros((n_recv, row_elems), dtype=torch.bfloat16, device='cuda')
                pw = packed.view(torch.float32)[:, H // 2:H // 2 + K]

                def launch():
                    kern.combine_reduce(MODE_LOCAL, y, packed[:, :H], n_recv, table=table_a,
                                        row_weights=w if weighted else None, wtable=table_a, wsrc=w,
                                        out_weights=pw, weights_pad=32, units_per_block=upb, stream=s)
                us = timeit(launch, s)
                times[v].append(us)
                if rnd == 0:
                    if ref is None:
                        ref = packed.clone()
                    outs[v] = torch.equal(packed.view(torch.int16), ref.view(torch.int16))
                del packed
        kern.lib.deepep_set_launch_config(0, -1, -1, 0)
        res = []
        for v in variants:
            med = statistics.median(times[v])
            res.append((med, v))
            print(json.dumps(dict(phase='A', weighted=weighted, store=('sc1', 'sc1 nt')[v[0] - 2], waves=v[1],
                                  rows_in_flight=v[2], us_median=round(med, 1), us_all=[round(t, 1) for t in times[v]],
                                  gbps=round(bytes_a / med / 1e3, 1), frac=round(bytes_a / med / 1e3 / 8000, 4),
                                  bitwise_equal=outs[v])), flush=True)
            times[v] = []
        best = min(res)
        print(json.dumps(dict(phase='A_best', weighted=weighted, us=round(best[0], 1),
                              store=('sc1', 'sc1 nt')[best[1][0] - 2], waves=best[1][1], rows_in_flight=best[1][2],
                              units=n_recv, rows=n_exp, bytes=bytes_a)), flush=True)


if __name__ == '__main__':
    main()
