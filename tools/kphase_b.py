"""Phase B (the EPILOGUE over one partial row per expert rank) at EP = 2, 4 and 8 (tuning aid): rank 0's
8192 tokens of BASELINE config 3's shape (hidden 7168, top-8 over 256 experts, uniform routing) over the
min(R, K) partial rows per token of the rank layout.  The automatic launch shape beside explicit rows in
flight (2 / 4 / 8) x workgroup waves (4 / 8), interleaved rounds, medians; one output, checked bitwise
against the automatic shape's after every timing."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    from deepep_amd.kernels import HipKernels, MODE_EPILOGUE
    from tests.plan_ref import epilogue_tables
    kern = HipKernels()
    T, H, K, E = 8192, 7168, 8, 256
    s = torch.cuda.current_stream()
    for R in (1, 2, 4, 8):
        g = torch.Generator(device='cuda').manual_seed(R)
        wts = None
        if R == 1:
            # the single reduction's reduce (one weighted EPILOGUE over a token's K unreduced rows in the
            # [K, T] receive window), the bench's single_reduction_phase_b
            table_b = (torch.arange(K, device='cuda').view(1, K) * T +
                       torch.arange(T, device='cuda').view(T, 1)).to(torch.int32).contiguous()
            recv = torch.randn((K * T, H + 64), device='cuda', generator=g).to(torch.bfloat16)
            wts = torch.rand((K * T,), device='cuda', generator=g)
        else:
            idx = torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1)[1]
            table_b, _, back = epilogue_tables(idx, E, R)
            n_back = sum(back)
            recv = torch.randn((n_back, H + 64), device='cuda', generator=g).to(torch.bfloat16)
        out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
        valid = int((table_b >= 0).sum())
        nbytes = valid * H * 2 + T * H * 2 + valid * 4
        variants = {'auto': ((0, -1, -1, 0), 0)}
        if os.environ.get('KPHASE_B_SHAPES') == '1':
            for vpt in (1, 2):
                for rows in (2, 4, 8):
                    for waves in (4, 8):
                        variants[f'vpt{vpt} rows{rows} waves{waves}'] = ((vpt, -1, -1, rows), waves)
        # store policies at the automatic shape: sc1 nt, per unit (sc1 when the token reduces >= 3 partial
        # rows, else sc1 nt); round 4 also tried thresholds 2 / 4 and every 2nd / 4th token streamed
        # (profiles/r04g_kphaseb.jsonl): none beat sc1
        for pol, name in ((3, 'sc1nt'), (4, 'per unit >= 3')):
            variants[name] = ((0, -1, pol, 0), 0)
        kern.combine_reduce(MODE_EPILOGUE, recv[:, :H], out, T, table=table_b, row_weights=wts, stream=s)
        ref = out.clone()
        times, bitwise = {k: [] for k in variants}, {k: True for k in variants}
        for _ in range(int(os.environ.get('KPHASE_B_ROUNDS', 4))):
            for name, (cfg, upb) in variants.items():
                assert kern.lib.deepep_set_launch_config(*cfg) == 0
                times[name].append(timeit(lambda: kern.combine_reduce(MODE_EPILOGUE, recv[:, :H], out, T, table=table_b,
                                                                      row_weights=wts, units_per_block=upb, stream=s), s, iters=30))
                bitwise[name] = bitwise[name] and bool(torch.equal(out, ref))
        kern.lib.deepep_set_launch_config(0, -1, -1, 0)
        res = {k: dict(us=round(statistics.median(v), 2), frac=round(nbytes / statistics.median(v) / 8e6, 4),
                       bitwise=bitwise[k]) for k, v in times.items()}
        print(json.dumps(dict(phase='B', ranks=R, width=table_b.shape[1], rows_per_token=round(valid / T, 3),
                              bytes=nbytes, variants=res)), flush=True)
        del recv, out, ref


if __name__ == '__main__':
    main()
