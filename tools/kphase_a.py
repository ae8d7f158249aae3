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
    R, T, H, K, E = int(os.environ.get('KPHASE_A_R', 8)), 8192, 7168, 8, 256
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
    # (vpt, store policy, waves, rows in flight); (0, -1, 0, 0) = the automatic shape (sc1 nt, 4 waves,
    # 4 rows, 2 vectors per lane)
    variants = [(0, -1, 0, 0)]
    if os.environ.get('KPHASE_A_FULL') == '1':
        for vpt in (1, 2):
            for upb in (4, 8):
                for rif in (2, 4, 8):
                    variants.append((vpt, 3, upb, rif))
    # store policies at the automatic shape (2 vectors, 4 waves, 4 rows): sc1, sc1 nt, per unit (sc1 when
    # the unit reduces >= 3 rows, else sc1 nt; the default).  Round 4 also tried thresholds 2 / 4 and every
    # 2nd / 4th unit streamed (profiles/r04g_kphasea_*).
    for pol in (2, 3, 4):
        variants.append((2, pol, 4, 4))
    rounds = int(os.environ.get('KPHASE_A_ROUNDS', 5))
    # one send buffer for every variant (the output's placement alone moves a kernel, tools/koutplace.py)
    packed = torch.zeros((n_recv, row_elems), dtype=torch.bfloat16, device='cuda')
    pw = packed.view(torch.float32)[:, H // 2:H // 2 + K]
    for weighted in (True, False):
        def launch(upb):
            kern.combine_reduce(MODE_LOCAL, y, packed[:, :H], n_recv, table=table_a,
                                row_weights=w if weighted else None, wtable=table_a, wsrc=w,
                                out_weights=pw, weights_pad=32, units_per_block=upb, stream=s)
        kern.lib.deepep_set_launch_config(0, -1, -1, 0)
        launch(0)
        ref = packed.clone()
        times = {v: [] for v in variants}
        same = {v: True for v in variants}
        for rnd in range(rounds):
            for v in variants:
                vpt, pol, upb, rif = v
                assert kern.lib.deepep_set_launch_config(vpt, -1, pol, rif) == 0
                times[v].append(timeit(lambda: launch(upb), s))
                same[v] = same[v] and torch.equal(packed.view(torch.int16), ref.view(torch.int16))
        kern.lib.deepep_set_launch_config(0, -1, -1, 0)
        res = []
        for v in variants:
            med = statistics.median(times[v])
            res.append((med, v))
            print(json.dumps(dict(phase='A', ranks=R, weighted=weighted, vpt=v[0], store={-1: 'auto', 2: 'sc1', 3: 'sc1 nt', 4: 'per unit >= 3'}[v[1]],
                                  waves=v[2], rows_in_flight=v[3], us_median=round(med, 1),
                                  us_all=[round(t, 1) for t in times[v]], gbps=round(bytes_a / med / 1e3, 1),
                                  frac=round(bytes_a / med / 1e3 / 8000, 4), bitwise_equal=same[v])), flush=True)
        if os.environ.get('KPHASE_A_FLUSH') == '1':
            # the cache state before a launch: back to back into the same rows (the loop above), back to back
            # alternating between two send buffers, and single launches after a 512 MB read / write flush
            flush = torch.empty((512 << 20) // 4, dtype=torch.int32, device='cuda')
            sink = torch.empty((1,), dtype=torch.int64, device='cuda')
            packed2 = torch.zeros_like(packed)
            pw2 = packed2.view(torch.float32)[:, H // 2:H // 2 + K]

            def launch_into(pk, pkw):
                kern.combine_reduce(MODE_LOCAL, y, pk[:, :H], n_recv, table=table_a,
                                    row_weights=w if weighted else None, wtable=table_a, wsrc=w,
                                    out_weights=pkw, weights_pad=32, stream=s)
            for pol in (2, 3, 4):
                assert kern.lib.deepep_set_launch_config(0, -1, pol, 0) == 0
                flip = [0]

                def alt():
                    flip[0] ^= 1
                    launch_into(packed2 if flip[0] else packed, pw2 if flip[0] else pw)
                row = dict(alternating_buffers=round(timeit(alt, s, iters=30), 1))
                for mode, pre in (('read_flush', lambda: torch.sum(flush, dim=0, dtype=torch.int64, out=sink)),
                                  ('write_flush', lambda: flush.fill_(1))):
                    ts = []
                    for _ in range(20):
                        pre()
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(s)
                        launch_into(packed, pw)
                        e1.record(s)
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3)
                    row[mode] = round(statistics.median(ts), 1)
                print(json.dumps(dict(phase='A_cache_state', ranks=R, weighted=weighted,
                                      store={2: 'sc1', 3: 'sc1 nt', 4: 'per unit >= 3'}[pol], **row)), flush=True)
            kern.lib.deepep_set_launch_config(0, -1, -1, 0)
            del flush, packed2
        best = min(res)
        print(json.dumps(dict(phase='A_best', ranks=R, weighted=weighted, us=round(best[0], 1), variant=best[1],
                              auto_us=round(statistics.median(times[variants[0]]), 1), units=n_recv, rows=n_exp,
                              bytes=bytes_a)), flush=True)

if __name__ == '__main__':
    main()
