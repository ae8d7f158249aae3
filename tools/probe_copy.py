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
    # blocked destination-major (probe_blocked_copy): per kTok-token block and expert, the block's rows
    lib.probe_blocked_copy.argtypes = [I, P, P, P, P, I, I, I, P, P]
    valid = idx >= 0
    count_e = torch.bincount(idx[valid], minlength=E)[:E]
    start_e = torch.cumsum(count_e, 0) - count_e
    for tok_blk in [int(v) for v in os.environ.get('PCOPY_BLOCKS', '256,128').split(',') if v]:
        nbk = (T + tok_blk - 1) // tok_blk
        blk_of = (torch.arange(T, device='cuda') // tok_blk).view(T, 1).expand(T, K)
        cnt = torch.zeros((nbk, E), dtype=torch.int64, device='cuda')
        cnt.index_put_((blk_of[valid], idx[valid]), torch.ones_like(idx[valid]), accumulate=True)
        off = (start_e.view(1, E) + torch.cumsum(cnt, 0) - cnt).to(torch.int32).contiguous()
        cnt32 = cnt.to(torch.int32).contiguous()
        for v in [int(v) for v in os.environ.get('PCOPY_BLOCKED', '3,5,6,7,8,9,10,0,3').split(',')]:
            out.zero_()
            fn = lambda: lib.probe_blocked_copy(v, x.data_ptr(), inv.data_ptr(), off.data_ptr(), cnt32.data_ptr(),
                                                nbk, E, xb, out.data_ptr(), s.cuda_stream)
            assert fn() == 0
            torch.cuda.synchronize()
            ok = bool(torch.equal(out, ref))
            us = timeit(fn, s, iters=20)
            print(json.dumps(dict(variant=f'blocked tok{tok_blk} v{v}', us=round(us, 1), gbps=round(nbytes / us / 1e3, 1),
                                  equal=ok)), flush=True)
    for v in [int(v) for v in os.environ.get('PCOPY_VARIANTS', '0,300,104,0,200,201').split(',') if v]:
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
