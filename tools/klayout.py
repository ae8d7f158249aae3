"""Does the LAYOUT of the expanded rows set the fused combine's rate?  (diagnostic, BASELINE config 2)

The same 65,536 rows and the same per-token sums, with the rows placed four ways in HBM:
  expert  -- the dispatch's expanded layout (rows grouped by expert, ascending token inside an expert):
             the tokens reduced at one moment read ~all 256 expert regions at once (the product case);
  slot    -- [K, T]: row k * T + t (the single-reduction receive window's layout: 8 regions);
  token   -- [T, K]: row t * K + k (a token's 8 rows adjacent: one region);
  random  -- a random permutation of the rows;
  pairs / quads -- a token's rows in runs of 2 / 4 adjacent rows, the runs at random places
             (KLAYOUT_RUNS=1; how long a contiguous run has to be before the rate moves);
  token_shuffled -- a token's rows adjacent, tokens in random order; slot_skewed -- [K, T] with each slot's
             region shifted by 37 rows (KLAYOUT_RUNS=1).
Each with the product's weighted reduction + weight pass-through and as a plain sum without it (the
weights are gathered through the slot, so they follow the rows).  Every output is checked bitwise
against the product's.  Interleaved over rounds, one JSON line per (round, variant) + medians.
"""
import json
import os
import statistics
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29619')
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
    buf.combine(y, handle, topk_weights=ex_w)
    table = handle._combine_plans[('multi', 1)].local_table.long()
    assert bool((table >= 0).all()), 'uniform top-8 routing: every slot valid'
    n = T * K
    kk = torch.arange(K, device='cuda').view(1, K)
    tt = torch.arange(T, device='cuda').view(T, 1)
    layouts = {'expert': table, 'slot': (kk * T + tt).expand(T, K), 'token': (tt * K + kk).expand(T, K),
               'random': torch.randperm(n, device='cuda')[(tt * K + kk).expand(T, K)]}
    if os.environ.get('KLAYOUT_RUNS') == '1':
        for name, g in (('pairs', 2), ('quads', 4)):
            # runs of g adjacent rows: run j of token t at a random run slot, row k % g inside it
            run = torch.randperm(n // g, device='cuda').view(T, K // g)
            layouts[name] = run[:, kk.view(-1) // g] * g + kk % g
        # a token's 8 rows adjacent but the tokens in random order (contiguity without one global sweep)
        layouts['token_shuffled'] = (torch.randperm(T, device='cuda').view(T, 1) * K + kk).expand(T, K)
        # [K, T] with each slot's region shifted by a non-power-of-two number of rows (8 sweeps, no aliasing)
        pad = 37
        layouts['slot_skewed'] = (kk * (T + pad) + tt).expand(T, K)
    data = {}
    for name, pos in layouts.items():
        if name == 'expert':
            data[name] = (y, ex_w, table.to(torch.int32).contiguous())
            continue
        rows = int(pos.max().item()) + 1
        yl = torch.empty((rows, H), dtype=y.dtype, device='cuda')
        wl = torch.empty((rows,), dtype=ex_w.dtype, device='cuda')
        yl[pos.reshape(-1)] = y[table.reshape(-1)]
        wl[pos.reshape(-1)] = ex_w[table.reshape(-1)]
        data[name] = (yl, wl, pos.to(torch.int32).contiguous())
    kern = buf.kernels
    s = torch.cuda.current_stream()
    outs = {}
    nbytes = T * (K * H * 2 + H * 2 + K * 8)

    def launch(name, weighted, out, ow):
        yl, wl, tab = data[name]
        return lambda: kern.combine_reduce(MODE_FUSED, yl, out, T, table=tab, row_weights=wl if weighted else None,
                                           wtable=tab if weighted else None, wsrc=wl if weighted else None,
                                           out_weights=ow if weighted else None, stream=s)
    variants = {}
    for weighted in (True, False):
        for name in layouts:
            key = f'{name} {"weighted + pass-through" if weighted else "plain"}'
            out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
            ow = torch.empty((T, K), dtype=torch.float32, device='cuda')
            outs[key] = (out, ow, weighted)
            variants[key] = launch(name, weighted, out, ow)
    res = {k: [] for k in variants}
    for r in range(int(os.environ.get('KLAYOUT_ROUNDS', 4))):
        for key, fn in variants.items():
            us = timeit(fn, s, iters=30)
            res[key].append(us)
            print(json.dumps(dict(round=r, variant=key, us=round(us, 2), tbps=round(nbytes / us / 1e6, 3))),
                  flush=True)
    torch.cuda.synchronize()
    bitwise = {}
    for key, (out, ow, weighted) in outs.items():
        ref = outs[f'expert {"weighted + pass-through" if weighted else "plain"}']
        bitwise[key] = bool(torch.equal(out, ref[0]) and (not weighted or torch.equal(ow, ref[1])))
    base = statistics.median(res[next(iter(variants))])
    print(json.dumps(dict(summary={k: dict(median_us=round(statistics.median(v), 2),
                                           vs_product=round(statistics.median(v) / base, 4), bitwise=bitwise[k])
                                   for k, v in res.items()})), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
