"""Combine overlapped with compute (the verdict's "not tested against a compute-overlap workload"):
BASELINE config 2's gating-weighted combine on one stream, a BF16 GEMM (hipBLASLt via torch.matmul,
8192 x 7168 x 7168, ~0.84 TFLOP) on another, issued together, for CU splits between them:

  chip      both streams unrestricted (this build's default: the combine takes what it gets)
  n CUs     the combine on its CU-budget stream (the first n CUs, ElasticBuffer.get_cu_budget_stream:
            what DEEPEP_COMBINE_CUS=handle or an explicit num_sms gives), the GEMM on the complement mask

Per split: the GEMM alone, the combine alone, both issued together (wall time per iteration, 20
iterations), and the overlap gain = (gemm + combine) / both.  One JSON line per split."""
import ctypes
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cu_mask_stream(first: int, last: int, n_cus: int):
    """A stream restricted to CU mask bits [first, last) (bit b = CU b / 8 of XCD b % 8)."""
    hip = ctypes.CDLL('libamdhip64.so')
    words = (n_cus + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for b in range(first, last):
        mask[b // 32] |= 1 << (b % 32)
    raw = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(raw), ctypes.c_uint32(words), mask)
    assert rc == 0, f'hipExtStreamCreateWithCUMask: {rc}'
    return torch.cuda.ExternalStream(raw.value)


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29683')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    T, H, K, E = 8192, 7168, 8, 256
    n_cus = torch.cuda.get_device_properties(0).multi_processor_count
    torch.manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    _, _, ex_w, handle, _ = buf.dispatch(torch.zeros((T, H), dtype=torch.bfloat16, device='cuda'),
                                         topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda').to(torch.bfloat16)
    ref, _, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
    a = torch.randn((8192, 7168), device='cuda').to(torch.bfloat16)
    b = torch.randn((7168, 7168), device='cuda').to(torch.bfloat16)
    c = torch.empty((8192, 7168), device='cuda', dtype=torch.bfloat16)
    flops = 2 * 8192 * 7168 * 7168
    iters = 20
    out = {}

    def wall(fns):
        for _ in range(3):
            for fn in fns:
                fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            for fn in fns:
                fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters * 1e6

    for n in (0, 16, 32, 64, 128, 192):
        sc = buf.get_cu_budget_stream(n) if n else torch.cuda.Stream()
        sg = cu_mask_stream(n, n_cus, n_cus) if n else torch.cuda.Stream()

        def gemm():
            with torch.cuda.stream(sg):
                torch.matmul(a, b, out=c)

        def comb():
            with torch.cuda.stream(sc):
                out['x'] = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True, num_sms=n or 0)[0]
        t_g = wall([gemm])
        t_c = wall([comb])
        t_b = wall([gemm, comb])
        same = bool(torch.equal(out['x'], ref))
        print(json.dumps(dict(combine_cus=n or 'chip', gemm_cus=(n_cus - n) if n else 'chip', gemm_us=round(t_g, 1),
                              gemm_tflops=round(flops / t_g / 1e6, 1), combine_us=round(t_c, 1),
                              both_us=round(t_b, 1), serial_us=round(t_g + t_c, 1),
                              overlap_gain=round((t_g + t_c) / t_b, 3), combine_bitwise_equal=same)), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
