"""A/B timing of combine kernel builds in one process (tuning aid): the in-tree library against
earlier builds placed in tools/_ab/ (libold.so: ABI v1 signature, libmid.so: ABI v2)."""
import ctypes
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.kbench import timeit  # noqa: E402

P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29613')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_FUSED
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    scores = torch.rand((T, E), device='cuda')
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    x = torch.zeros((T, H), dtype=torch.bfloat16, device='cuda')
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    buf.combine(y, handle, topk_weights=ex_w)
    tab = handle._combine_plans[('multi', 1)].local_table
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')
    s = torch.cuda.current_stream()
    nbytes = T * K * H * 2 + T * H * 2 + T * K * 8
    variants = {'current': lambda: buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=tab, row_weights=ex_w,
                                                              wtable=tab, wsrc=ex_w, out_weights=out_w, stream=s)}
    for name, v2 in (('old', False), ('mid', True)):
        path = os.path.join(ROOT, 'tools', '_ab', f'lib{name}.so')
        if not os.path.exists(path):
            continue
        lib = ctypes.CDLL(path)
        f = lib.deepep_combine_reduce
        f.restype = I
        f.argtypes = ([I, I, P, I64, I64, P, I64, I, P, P, P, P, I64, I, I, P, I64, P, P, I] + ([I64] if v2 else []) +
                      [I, P, P])
        args = [MODE_FUSED, 1, y.data_ptr(), y.shape[0], H, tab.data_ptr(), K, K, ex_w.data_ptr(), None, None,
                out.data_ptr(), H, T, H, tab.data_ptr(), K, ex_w.data_ptr(), out_w.data_ptr(), K]
        args += ([K] if v2 else []) + [0, None, s.cuda_stream]
        variants[name] = (lambda f=f, args=args: f(*args))
    for rnd in range(3):
        for name, fn in variants.items():
            us = timeit(fn, s, iters=30)
            print(json.dumps(dict(round=rnd, build=name, us=round(us, 1), frac=round(nbytes / us / 1e3 / 8000, 4))),
                  flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
