"""Can a window-ordered sweep ahead of the fused combine beat the expert layout's 256 streams?  (diagnostic)

DESIGN.md section 4: the fused combine reads config 2's expanded rows (grouped by expert, ascending token
inside an expert) at 0.75-0.76 of peak, the same rows placed token-major at 0.80-0.81: the DRAM rewards one
sequential sweep, and the expert layout is 256 concurrent sweeps.  The tokens of a window [t0, t1) read, in
every expert segment, one contiguous run of rows.  So the window's rows can be read in ADDRESS order (one
sweep over 256 runs) shortly before the combine gathers them, and the gather then finds them in the
256 MiB Infinity Cache.  This probe tests that with the product kernel unchanged:

  product         one fused launch over all tokens (the bench's kernel)
  win W           the same kernel launched per window of W tokens, no prefetch (launch-split cost)
  pf W g p        per window: prefetch of window w + 1 (tools/probe_prefetch.hip, grid g, load policy p) on a
                  second stream, overlapped with the combine of window w; the combine of w + 1 waits for its
                  prefetch, the prefetch of w + 2 for the combine of w (at most two windows in the cache)
  serial W        per window: prefetch(w) then combine(w) on one stream, each timed with events (the
                  combine's rate from the cache, the sweep's rate from HBM)

Every combine output is checked bitwise against the product's.  Medians of interleaved rounds.
"""
import ctypes
import json
import os
import statistics
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29623')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED
    lib = ctypes.CDLL(os.path.join(ROOT, 'tools', 'libprobe_prefetch.so'))
    P, I, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    lib.probe_prefetch.argtypes = [I, P, L, P, I, I, I, P, P]
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                         topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
    table = handle._combine_plans[('multi', 1)].local_table
    kern = buf.kernels
    s = torch.cuda.current_stream()
    sp = torch.cuda.Stream()
    sink = torch.zeros((256,), dtype=torch.int32, device='cuda')
    nbytes = T * (K * H * 2 + H * 2 + K * 8)

    def combine(out, ow, lo, hi, stream):
        kern.combine_reduce(MODE_FUSED, y, out[lo:hi], hi - lo, table=table[lo:hi], row_weights=ex_w,
                            wtable=table[lo:hi], wsrc=ex_w, out_weights=ow[lo:hi], stream=stream)

    ref = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    ref_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    combine(ref, ref_w, 0, T, s)

    def windows(W):
        return [(lo, min(T, lo + W)) for lo in range(0, T, W)]

    pf_rows = {}

    def rows_of(W):
        if W not in pf_rows:
            lst = []
            for lo, hi in windows(W):
                r = table[lo:hi].reshape(-1)
                lst.append(torch.sort(r[r >= 0])[0].to(torch.int32).contiguous())
            pf_rows[W] = lst
        return pf_rows[W]

    def prefetch(W, i, grid, policy, stream):
        r = rows_of(W)[i]
        assert lib.probe_prefetch(policy, y.data_ptr(), H, r.data_ptr(), r.numel(), H, grid, sink.data_ptr(),
                                  stream.cuda_stream) == 0

    variants, outs = {}, {}

    def add(name, fn_of):
        out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
        ow = torch.empty((T, K), dtype=torch.float32, device='cuda')
        outs[name] = (out, ow)
        variants[name] = fn_of(out, ow)

    add('product', lambda out, ow: (lambda: combine(out, ow, 0, T, s)))
    for W in (512, 1024):
        add(f'win {W}', lambda out, ow, W=W: (lambda: [combine(out, ow, lo, hi, s) for lo, hi in windows(W)]))

    def pipelined(out, ow, W, grid, policy):
        def fn():
            wins = windows(W)
            sp.wait_stream(s)
            with torch.cuda.stream(sp):
                prefetch(W, 0, grid, policy, sp)
            pe = [torch.cuda.Event()]
            pe[0].record(sp)
            ce = []
            for i, (lo, hi) in enumerate(wins):
                s.wait_event(pe[i])
                combine(out, ow, lo, hi, s)
                ev = torch.cuda.Event()
                ev.record(s)
                ce.append(ev)
                if i + 1 < len(wins):
                    if i >= 1:
                        sp.wait_event(ce[i - 1])
                    prefetch(W, i + 1, grid, policy, sp)
                    ev = torch.cuda.Event()
                    ev.record(sp)
                    pe.append(ev)
            s.wait_stream(sp)
        return fn

    for W in (512, 1024):
        for grid in (64, 256):
            add(f'pf {W} g{grid} plain', lambda out, ow, W=W, g=grid: pipelined(out, ow, W, g, 0))
    add('pf 1024 g128 plain', lambda out, ow: pipelined(out, ow, 1024, 128, 0))
    add('pf 1024 g256 nt', lambda out, ow: pipelined(out, ow, 1024, 256, 1))

    res = {k: [] for k in variants}
    for r in range(int(os.environ.get('KPREFETCH_ROUNDS', 4))):
        for key, fn in variants.items():
            us = timeit(fn, s, iters=20)
            res[key].append(us)
            print(json.dumps(dict(round=r, variant=key, us=round(us, 2), tbps=round(nbytes / us / 1e6, 3))),
                  flush=True)

    # serial: the combine's rate from the cache and the sweep's rate from HBM, per window
    for W in (512, 1024):
        for policy in (0, 1):
            out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
            ow = torch.empty((T, K), dtype=torch.float32, device='cuda')
            t_pf, t_c, t_cold = [], [], []
            for rep in range(3):
                for i, (lo, hi) in enumerate(windows(W)):
                    e = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
                    e[0].record(s)
                    combine(out, ow, lo, hi, s)                  # cold (rows not in the cache)
                    e[1].record(s)
                    prefetch(W, i, 512, policy, s)
                    e[2].record(s)
                    combine(out, ow, lo, hi, s)                  # after the sweep
                    e[3].record(s)
                    torch.cuda.synchronize()
                    t_cold.append(e[0].elapsed_time(e[1]) * 1e3)
                    t_pf.append(e[1].elapsed_time(e[2]) * 1e3)
                    t_c.append(e[2].elapsed_time(e[3]) * 1e3)
            wb = W * (K * H * 2 + H * 2 + K * 8)
            pb = W * K * H * 2
            print(json.dumps(dict(serial=W, policy=policy, combine_cold_us=round(statistics.median(t_cold), 2),
                                  combine_after_sweep_us=round(statistics.median(t_c), 2),
                                  sweep_us=round(statistics.median(t_pf), 2),
                                  combine_cold_tbps=round(wb / statistics.median(t_cold) / 1e6, 3),
                                  combine_after_sweep_tbps=round(wb / statistics.median(t_c) / 1e6, 3),
                                  sweep_tbps=round(pb / statistics.median(t_pf) / 1e6, 3))), flush=True)
            outs[f'serial {W} p{policy}'] = (out, ow)

    torch.cuda.synchronize()
    bitwise = {k: bool(torch.equal(o, ref) and torch.equal(ow, ref_w)) for k, (o, ow) in outs.items()}
    base = statistics.median(res['product'])
    print(json.dumps(dict(summary={k: dict(median_us=round(statistics.median(v), 2),
                                           vs_product=round(statistics.median(v) / base, 4), bitwise=bitwise[k])
                                   for k, v in res.items()}, bitwise=bitwise)), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
