"""Token-streaming waves vs the product kernel (diagnostic; tools/probe_tok.hip): same data, same
process, plain sum, config 2 (8192 x 7168 x top-8, expanded rows grouped by expert)."""
import ctypes
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
from probe import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    lib = ctypes.CDLL(os.path.join(ROOT, 'tools', 'libprobe_tok.so'))
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.probe_token_stream.argtypes = [I, I, P, P, P, I, I, I, P]
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29614')
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
    table = handle._combine_plans[('multi', 1)].local_table if ('multi', 1) in handle._combine_plans else None
    buf.combine(y, handle)
    table = handle._combine_plans[('multi', 1)].local_table
    assert int((table < 0).sum()) == 0
    ref = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    s = torch.cuda.current_stream()
    nbytes = T * K * H * 2 + T * H * 2 + T * K * 4

    def product():
        buf.kernels.combine_reduce(MODE_FUSED, y, ref, T, table=table, stream=s)
    out_w = torch.empty((T, K), dtype=torch.float32, device='cuda')

    def lib_kernel(upb, weighted):
        def f():
            buf.kernels.combine_reduce(MODE_FUSED, y, out, T, table=table, row_weights=ex_w if weighted else None,
                                       wtable=table, wsrc=ex_w, out_weights=out_w, units_per_block=upb, stream=s)
        return f
    res = {'product_us': round(timeit(product, 50, 5), 1)}
    # A/B in one process: item kernel (units_per_block 8) vs streaming kernel (automatic), weighted
    # as in bench.py and plain, interleaved rounds
    for rnd in range(3):
        for weighted in (True, False):
            for choice, name in ((0, 'item'), (1, 'stream'), (2, 'stream_vpt1'), (3, 'stream_persistent'),
                                 (4, 'item_xcd')):
                assert buf.kernels.lib.deepep_set_kernel_choice(choice) == 0
                res[f'ab r{rnd} {"w" if weighted else "p"} {name}'] = round(timeit(lib_kernel(0, weighted), 50, 5), 1)
    buf.kernels.lib.deepep_set_kernel_choice(-1)
    for rnd in range(2):
        for vpt in (1, 2):
            for aux in (16, 2):
                for grid in (512, 1024, 2048):
                    def probe():
                        rc = lib.probe_token_stream(vpt, aux, y.data_ptr(), table.data_ptr(), out.data_ptr(), T, H,
                                                    grid, s.cuda_stream)
                        assert rc == 0, rc
                    us = timeit(probe, 50, 5)
                    same = bool(torch.equal(out, ref))
                    res[f'r{rnd} vpt{vpt} aux{aux} grid{grid}'] = (round(us, 1), round(nbytes / us / 1e3, 1), same)
        res[f'product_us_r{rnd}'] = round(timeit(product, 50, 5), 1)
    print(json.dumps(res))
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
