"""Generate the committed golden fixtures under tests/golden/ from the reference's
own pure-torch oracle (deep_ep/utils/refs.py, deep_ep/utils/math.py and
deep_ep/utils/gate.py in /root/reference).

This script is the ONLY place that touches /root/reference, and it runs only in
the development container (the GPU box has no /root/reference).  It loads the
three reference files as standalone modules (no `import deep_ep`, which needs
the CUDA extension), with a stub for `deep_ep.utils.envs.get_global_seed`, and
with `sys.dont_write_bytecode` set so nothing is written into the read-only
reference tree.  The fixtures it writes are data only: inputs and the outputs
the reference oracle produced for them.

Usage:  python tests/golden/gen_golden.py [--out tests/golden]

Fixtures (all bf16 tensors stored as uint16 bit patterns):
  f1_ep1_t128_h1024_k2.npz   BASELINE config 1 (EP=1, 128 tokens, hidden 1024, top-2, E=8)
  f2_ep8_t64_h256_k8.npz     simulated EP=8 (64 tokens/rank, hidden 256, top-8, E=64),
                             including refs.dispatch outputs from an 8-process gloo run
  f4_ep4_t96_h256_k2.npz     EP=4 with top-2 (R > K: per-top-k receive slots), with refs.dispatch outputs
  f3_ep8_skew_t128_h64_k8.npz   EP=8 skewed routing (gate.get_random_unbalanced_scores, ratio 4)
"""
import argparse
import importlib.util
import math
import os
import sys
import types

sys.dont_write_bytecode = True

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REF_UTILS = '/root/reference/deep_ep/utils'
GLOBAL_SEED = 0


def _load_reference_modules():
    """Load refs.py / math.py / gate.py as `_ref_deep_ep.utils.*` without executing
    the package __init__ (which imports the CUDA extension)."""
    pkg = types.ModuleType('_ref_deep_ep')
    pkg.__path__ = []
    utils = types.ModuleType('_ref_deep_ep.utils')
    utils.__path__ = []
    envs = types.ModuleType('_ref_deep_ep.utils.envs')
    envs.get_global_seed = lambda: GLOBAL_SEED
    sys.modules.update({'_ref_deep_ep': pkg, '_ref_deep_ep.utils': utils, '_ref_deep_ep.utils.envs': envs})
    loaded = {}
    for name in ('math', 'refs', 'gate'):
        spec = importlib.util.spec_from_file_location(f'_ref_deep_ep.utils.{name}', f'{REF_UTILS}/{name}.py')
        mod = importlib.util.module_from_spec(spec)
        sys.modules[spec.name] = mod
        spec.loader.exec_module(mod)
        loaded[name] = mod
    return loaded


class _CpuTorch:
    """Proxy for `torch` inside gate.py: drops `device=` so the CUDA-only helpers run on CPU."""

    def __getattr__(self, item):
        attr = getattr(torch, item)
        if callable(attr) and not isinstance(attr, type):
            def wrapped(*args, **kwargs):
                kwargs.pop('device', None)
                return attr(*args, **kwargs)
            return wrapped
        return attr


def bf16_bits(t: torch.Tensor) -> np.ndarray:
    assert t.dtype == torch.bfloat16
    return t.contiguous().view(torch.int16).numpy().view(np.uint16).copy()


def _init_single_process_group():
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29561')
        dist.init_process_group('gloo', rank=0, world_size=1)


def _routing(num_tokens, num_experts, num_topk, masked_ratio, gen):
    scores = torch.rand((num_tokens, num_experts), generator=gen)
    topk_weights, topk_idx = torch.topk(scores, num_topk, dim=-1, largest=True, sorted=False)
    topk_idx = topk_idx.to(torch.int64)
    if masked_ratio > 0:
        mask = torch.rand(topk_idx.shape, generator=gen) < masked_ratio
        topk_idx.masked_fill_(mask, -1)
        topk_weights.masked_fill_(topk_idx < 0, 0)
    return topk_idx, topk_weights


def _combine_outputs(refs, y, topk_idx, num_ranks, num_experts, biases):
    """refs.combine for bias in {0,1,2} and both reduction recipes (test_ep.py:109-124)."""
    out = {}
    for nb in (0, 1, 2):
        bias = None if nb == 0 else (biases[0] if nb == 1 else (biases[0], biases[1]))
        multi = refs.combine(y, topk_idx, 1, num_ranks, num_experts, bias, True, False)
        single = refs.combine(y, topk_idx, 1, num_ranks, num_experts, bias, False, False)
        out[f'combined_multi_b{nb}'] = bf16_bits(multi)
        out[f'combined_single_b{nb}'] = bf16_bits(single)
    return out


def gen_f1(mods, out_dir):
    """BASELINE config 1: EP=1 loopback, 128 tokens, hidden=1024, top-2, E=8."""
    refs = mods['refs']
    T, H, K, E = 128, 1024, 2, 8
    gen = torch.Generator().manual_seed(1)
    topk_idx, topk_weights = _routing(T, E, K, 0.1, gen)
    y = refs.generate_pre_combine_data(torch.arange(T), T, K, H)   # [T, K, H] bf16
    y[topk_idx == -1] = 0                                           # test_ep.py:117
    biases = [torch.randn((T, H), generator=gen).to(torch.bfloat16) for _ in range(2)]
    fx = dict(topk_idx=topk_idx.numpy().copy(), topk_weights=topk_weights.numpy().copy(), y=bf16_bits(y),
              bias0=bf16_bits(biases[0]), bias1=bf16_bits(biases[1]),
              meta=np.array([T, H, K, E, 1], dtype=np.int64))
    fx.update(_combine_outputs(refs, y, topk_idx, 1, E, biases))
    # Weighted variant: float64 reference of sum_k w_k * y_k (checked with calc_diff, as
    # tests/legacy/test_low_latency.py:178-181 does for the weighted combine).
    w = topk_weights.masked_fill(topk_idx < 0, 0).double()
    fx['weighted_f64'] = (y.double() * w.unsqueeze(-1)).sum(1).numpy()  # kept in float64
    # refs.ordered_accumulate over the slots (non-expanded caller-side pre-reduce, test_ep.py:193)
    fx['ordered_accumulate'] = bf16_bits(refs.ordered_accumulate(y))
    np.savez_compressed(f'{out_dir}/f1_ep1_t128_h1024_k2.npz', **fx)


def _dispatch_worker(rank, world, port, T, H, K, E, x_all, idx_all, w_all, queue):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    mods = _load_reference_modules()
    recv = mods['refs'].dispatch(x_all[rank], idx_all[rank], w_all[rank], T, E)
    recv_x, recv_topk_idx, recv_topk_weights, recv_src_token_idx, num_recv = recv
    queue.put((rank, bf16_bits(recv_x), recv_topk_idx.numpy(), recv_topk_weights.numpy(),
               recv_src_token_idx.numpy(), num_recv.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def gen_multirank(mods, out_dir, name, R, T, H, K, E, skew_ratio, masked_ratio, seed, with_dispatch):
    refs, gate = mods['refs'], mods['gate']
    gen = torch.Generator().manual_seed(seed)
    fx = {'meta': np.array([T, H, K, E, R], dtype=np.int64)}
    idx_all, w_all, x_all = [], [], []
    dist.get_world_size = lambda *a, **k: R      # generate_pre_combine_data's max_seed uses the world size
    for r in range(R):
        if skew_ratio > 1:
            torch.manual_seed(seed * 100 + r)
            gate.torch = _CpuTorch()
            scores = gate.get_unbalanced_scores(T, E, R, K, skew_ratio, False)
            topk_weights, topk_idx = torch.topk(scores, K, dim=-1, largest=True, sorted=False)
            topk_idx = topk_idx.to(torch.int64)
            if masked_ratio > 0:
                mask = torch.rand(topk_idx.shape, generator=gen) < masked_ratio
                topk_idx.masked_fill_(mask, -1)
                topk_weights.masked_fill_(topk_idx < 0, 0)
        else:
            topk_idx, topk_weights = _routing(T, E, K, masked_ratio, gen)
        y = refs.generate_pre_combine_data(r * T + torch.arange(T), T, K, H)
        y[topk_idx == -1] = 0
        biases = [torch.randn((T, H), generator=gen).to(torch.bfloat16) for _ in range(2)]
        x = torch.randn((T, H), generator=gen).to(torch.bfloat16)
        fx[f'r{r}_topk_idx'] = topk_idx.numpy().copy()
        fx[f'r{r}_topk_weights'] = topk_weights.numpy().copy()
        fx[f'r{r}_y'] = bf16_bits(y)
        fx[f'r{r}_bias0'] = bf16_bits(biases[0])
        fx[f'r{r}_bias1'] = bf16_bits(biases[1])
        fx[f'r{r}_x'] = bf16_bits(x)
        for key, val in _combine_outputs(refs, y, topk_idx, R, E, biases).items():
            fx[f'r{r}_{key}'] = val
        idx_all.append(topk_idx.clone())  # torch.multiprocessing moves storages to shm
        w_all.append(topk_weights.clone())
        x_all.append(x.clone())
    dist.get_world_size = torch.distributed.distributed_c10d.get_world_size

    if with_dispatch:
        ctx = mp.get_context('spawn')
        queue = ctx.Queue()
        procs = [ctx.Process(target=_dispatch_worker,
                             args=(r, R, 29600 + seed, T, H, K, E, x_all, idx_all, w_all, queue))
                 for r in range(R)]
        for p in procs:
            p.start()
        results = [queue.get(timeout=300) for _ in range(R)]
        for p in procs:
            p.join(timeout=60)
        for rank, rx, ridx, rw, rsrc, nrecv in results:
            fx[f'r{rank}_dispatch_recv_x'] = rx
            fx[f'r{rank}_dispatch_recv_topk_idx'] = ridx
            fx[f'r{rank}_dispatch_recv_topk_weights'] = rw
            fx[f'r{rank}_dispatch_recv_src_token_idx'] = rsrc
            fx[f'r{rank}_dispatch_num_recv_tokens_per_rank'] = nrecv
    np.savez_compressed(f'{out_dir}/{name}.npz', **fx)


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument('--out', default=os.path.dirname(os.path.abspath(__file__)))
    args = parser.parse_args()
    torch.manual_seed(GLOBAL_SEED)
    mods = _load_reference_modules()
    _init_single_process_group()
    gen_f1(mods, args.out)
    gen_multirank(mods, args.out, 'f2_ep8_t64_h256_k8', R=8, T=64, H=256, K=8, E=64,
                  skew_ratio=1.0, masked_ratio=0.1, seed=2, with_dispatch=True)
    gen_multirank(mods, args.out, 'f3_ep8_skew_t128_h64_k8', R=8, T=128, H=64, K=8, E=64,
                  skew_ratio=4.0, masked_ratio=0.0, seed=3, with_dispatch=False)
    gen_multirank(mods, args.out, 'f4_ep4_t96_h256_k2', R=4, T=96, H=256, K=2, E=16,
                  skew_ratio=1.0, masked_ratio=0.15, seed=4, with_dispatch=True)
    dist.destroy_process_group()
    print('golden fixtures written to', args.out)


if __name__ == '__main__':
    main()
