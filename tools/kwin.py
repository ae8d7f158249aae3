"""Phase B's receive-window row order (diagnostic, BASELINE config 3 at EP = 8, one rank's share).

Phase B (EPILOGUE) reduces, per owned token, the partial rows the expert ranks stored into this rank's
window.  The window is `[slot][T_max]` today (row s * T_max + t, combine.cuh:96-106's receive layout):
8 sweeps whose spacing (T_max rows of 14,464 B = 113 MiB) may alias.  tools/klayout.py showed the DRAM
rewards few sequential sweeps; this probe times the same phase-B launch over the same partials placed
  slot        -- row s * T_max + t (the product);
  slot_skewed -- row s * (T_max + 37) + t;
  token       -- row t * S + s (a token's partials adjacent, tokens in order: one sweep);
with the routing of config 3 (uniform top-8 over 256 experts, 8 ranks: ~5.3 of the 8 slots valid per
token), plain and with the weight pass-through.  Outputs are checked bit for bit against the product's.
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    from deepep_amd import _lib  # noqa: F401  (loads the library)
    from deepep_amd.handle import packed_row_layout
    from deepep_amd.kernels import HipKernels, MODE_EPILOGUE
    T, H, K, E, R = 8192, 7168, 8, 256, 8
    S = min(R, K)
    torch.manual_seed(0)
    idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)[1]
    present = torch.zeros((T, R), dtype=torch.bool, device='cuda')
    present.scatter_(1, idx // (E // R), True)
    row_bytes, w_off, _ = packed_row_layout(H, K)
    re = row_bytes // 2                                        # row pitch in bf16 elements
    tt = torch.arange(T, device='cuda').view(T, 1)
    ss = torch.arange(S, device='cuda').view(1, S)
    pad = 37
    layouts = {'slot': ss * T + tt, 'slot_skewed': ss * (T + pad) + tt, 'token': tt * S + ss}
    # the partials (bf16) and their weight lines, generated once in slot order and placed per layout
    base = torch.randn((S * T, re), device='cuda').to(torch.bfloat16)
    base.view(torch.float32).view(S * T, row_bytes // 4)[:, w_off // 4:w_off // 4 + K] = torch.rand((S * T, K), device='cuda')
    kern = HipKernels()
    s = torch.cuda.current_stream()
    data = {}
    for name, pos in layouts.items():
        n_rows = int(pos.max().item()) + 1
        win = torch.zeros((n_rows, re), dtype=torch.bfloat16, device='cuda')
        win[pos.reshape(-1)] = base[layouts['slot'].reshape(-1)]
        tab = torch.where(present, pos, torch.full_like(pos, -1)).to(torch.int32).contiguous()
        # weight index of (t, k): the float offset of lane k's weight in the row of k's rank
        wrow = torch.gather(tab.long(), 1, idx // (E // R))
        kk = torch.arange(K, device='cuda').view(1, K)
        wtab = torch.where(wrow >= 0, wrow * (row_bytes // 4) + w_off // 4 + kk, torch.full_like(wrow, -1))
        data[name] = (win, tab, wtab.to(torch.int32).contiguous())
    outs, variants = {}, {}
    for passthrough in (False, True):
        for name in layouts:
            win, tab, wtab = data[name]
            out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
            ow = torch.empty((T, K), dtype=torch.float32, device='cuda')
            key = f'{name} {"pass-through" if passthrough else "plain"}'
            outs[key] = (out, ow, passthrough)
            variants[key] = (lambda win=win, tab=tab, wtab=wtab, out=out, ow=ow, pt=passthrough:
                             kern.combine_reduce(MODE_EPILOGUE, win[:, :H], out, T, table=tab,
                                                 wtable=wtab if pt else None, wsrc=win.view(torch.float32).view(-1) if pt else None,
                                                 out_weights=ow if pt else None, stream=s))
    valid = int(present.sum().item())
    nbytes = valid * H * 2 + T * H * 2 + T * K * 8
    res = {k: [] for k in variants}
    for r in range(int(os.environ.get('KWIN_ROUNDS', 4))):
        for key, fn in variants.items():
            us = timeit(fn, s, iters=30)
            res[key].append(us)
            print(json.dumps(dict(round=r, variant=key, us=round(us, 2), tbps=round(nbytes / us / 1e6, 3))), flush=True)
    torch.cuda.synchronize()
    summary = {}
    for key, v in res.items():
        out, ow, pt = outs[key]
        ref = outs[f'slot {"pass-through" if pt else "plain"}']
        summary[key] = dict(median_us=round(statistics.median(v), 2),
                            vs_product=round(statistics.median(v) / statistics.median(res[f'slot {"pass-through" if pt else "plain"}']), 4),
                            bitwise=bool(torch.equal(out, ref[0]) and (not pt or torch.equal(ow, ref[1]))))
    print(json.dumps(dict(valid_partials_per_token=round(valid / T, 2), alg_bytes=nbytes, summary=summary)), flush=True)


if __name__ == '__main__':
    main()
