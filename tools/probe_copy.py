"""Dispatch-copy probes (tools/probe_copy.hip): source-major scatter vs destination-major gather of
the expanded rows at BASELINE config 2 (diagnostic)."""
import ctypes
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29631')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    lib = ctypes.CDLL(os.path.join(ROOT, 'tools', 'libprobe_copy.so'))
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.probe_copy.argtypes = [I, P, P, P, I, I, I, I, P, P]
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    scores = torch.rand((T, E), device='cuda')
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    x = torch.randn((T, H), device='cuda').to(torch.bfloat16)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    ref, _, _, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    N = ref.shape[0]
    meta = handle.recv_src_metadata
    dst = meta[:, 2:].contiguous()                                   # [T, K] (T == N_recv here)
    tok = (meta[:, 0] % T).long()
    inv = torch.full((N,), -1, dtype=torch.int32, device='cuda')
    ii, kk = (dst >= 0).nonzero(as_tuple=True)
    inv[dst[ii, kk].long()] = tok[ii].to(torch.int32)
    out = torch.empty_like(ref)
    s = torch.cuda.current_stream()
    xb = H * 2
    nbytes = T * xb + N * xb
    for v in (0, 300, 301, 302, 303, 304, 104, 105, 111, 0, 300, 201):
        out.zero_()
        fn = lambda: lib.probe_copy(v, x.data_ptr(), dst.data_ptr(), inv.data_ptr(), T, K, N, xb, out.data_ptr(),
                                    s.cuda_stream)
        assert fn() == 0
        torch.cuda.synchronize()
        ok = bool(torch.equal(out, ref)) if v < 200 else None
        us = timeit(fn, s, iters=20)
        print(json.dumps(dict(variant=v, us=round(us, 1), gbps=round(nbytes / us / 1e3, 1), equal=ok)), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
