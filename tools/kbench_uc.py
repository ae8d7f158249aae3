"""Cost of the xGMI transport's uncached window on one GPU (tuning aid): phase B (EPILOGUE over
min(R, K) = 8 partial rows per token) reading from an uncached window vs ordinary device memory,
and phase A stores (reduce_scatter) into each."""
import ctypes
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29615')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import _lib
    from deepep_amd.kernels import HipKernels, MODE_EPILOGUE
    from deepep_amd.symmetric import _DeviceArray
    kern = HipKernels()
    lib = kern.lib
    T, H, K, S = 8192, 7168, 8, 8                  # S receive slots (rank layout at EP = 8)
    from deepep_amd.handle import packed_row_layout
    row_bytes = packed_row_layout(H, K)[0]         # the window's packed rows: bf16 partial + weight line
    nbytes = S * T * row_bytes
    p = ctypes.c_void_p()
    _lib.check(lib.deepep_sym_alloc(nbytes, ctypes.byref(p)), 'alloc')
    uc = torch.as_tensor(_DeviceArray(p.value, nbytes), device='cuda')
    cc = torch.empty((nbytes,), dtype=torch.uint8, device='cuda')
    g = torch.Generator(device='cuda').manual_seed(0)
    # 5.3 of 8 slots valid per token on average (EP = 8 uniform routing)
    valid = torch.rand((T, S), device='cuda', generator=g) < 5.3 / 8
    rows = (torch.arange(S, device='cuda').view(1, S) * T + torch.arange(T, device='cuda').view(T, 1))
    table = torch.where(valid, rows, torch.full_like(rows, -1)).to(torch.int32).contiguous()
    out = torch.empty((T, H), dtype=torch.bfloat16, device='cuda')
    s = torch.cuda.current_stream()
    n_valid = int(valid.sum())
    for name, buf in (('cached', cc), ('uncached', uc)):
        src = buf.view(torch.bfloat16).view(S * T, row_bytes // 2)
        src[:, :H].normal_()
        us = timeit(lambda: kern.combine_reduce(MODE_EPILOGUE, src[:, :H], out, T, table=table, stream=s), s, iters=30)
        gb = (n_valid * H * 2 + T * H * 2) / us / 1e3
        print(json.dumps(dict(phase='B_epilogue', memory=name, us=round(us, 1), gbps=round(gb, 1))), flush=True)
    # phase A stores: T units, each a copy of one source row, written to row (t % S) * T + t
    x = torch.randn((T, H), device='cuda').to(torch.bfloat16)
    for name, buf in (('cached', cc), ('uncached', uc)):
        t = torch.arange(T, device='cuda')
        addr = (buf.data_ptr() + ((t % S) * T + t) * row_bytes).to(torch.int64).contiguous()
        win = (torch.tensor([buf.data_ptr()], dtype=torch.int64, device='cuda'), nbytes)
        us = timeit(lambda: kern.combine_reduce_scatter(x, T, addr, windows=win, stream=s), s, iters=30)
        print(json.dumps(dict(phase='A_scatter_copy', memory=name, us=round(us, 1),
                              gbps=round(2 * T * H * 2 / us / 1e3, 1))), flush=True)
    del uc
    torch.cuda.synchronize()
    lib.deepep_sym_free(p)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
