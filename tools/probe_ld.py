"""Load / store cache-policy sweep of the combine's gather (tools/probe_ld.hip), config 2."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    lib = ctypes.CDLL(os.path.join(ROOT, 'tools', 'libprobe_ld.so'))
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.probe_ld.argtypes = [I, P, P, P, I, I, P]
    T, H, K = 8192, 7168, 8
    g = torch.Generator(device='cuda').manual_seed(0)
    y = torch.randn((T * K, H), device='cuda', generator=g).to(torch.bfloat16)
    table = torch.randperm(T * K, device='cuda', generator=g).to(torch.int32).view(T, K).contiguous()
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    ref = (y.float()[table.long()].sum(1)).to(torch.bfloat16)
    s = torch.cuda.current_stream()
    nbytes = T * (K * H * 2 + H * 2)
    names = ['global nt', 'buf plain', 'buf nt', 'buf sc0', 'buf sc1', 'buf sc0sc1', 'buf sc1nt', 'buf sc0nt',
             'buf sc0sc1nt', 'nt / plain st', 'nt / sc0sc1 st', 'nt / sc1nt st']
    for rnd in range(2):
        for v, name in enumerate(names):
            fn = lambda: lib.probe_ld(v, y.data_ptr(), table.data_ptr(), out.data_ptr(), T, H, s.cuda_stream)
            assert fn() == 0
            torch.cuda.synchronize()
            ok = bool(torch.allclose(out.float(), ref.float(), atol=0.1, rtol=0.02)) if rnd == 0 else None
            us = timeit(fn, s, iters=30)
            print(json.dumps(dict(round=rnd, variant=name, us=round(us, 1), gbps=round(nbytes / us / 1e3, 1),
                                  ok=ok)), flush=True)


if __name__ == '__main__':
    main()
