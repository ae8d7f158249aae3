"""Store policy of the dispatch's expanded copy (tuning aid, BASELINE config 2): the blocked
destination-major copy writes 939 MB over 256 expert segments; phase A of the combine ran 3-8 % faster
with its stores split between sc1 and sc1 nt than with either alone, so the copy's
policies are compared the same way: a cached dispatch (the copy plus a few small launches) timed back to
back under every deepep_set_dispatch_copy_policy value, interleaved rounds, medians; outputs checked
bitwise against the default's."""
import json
import os
import statistics
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kbench import timeit  # noqa: E402

NAMES = ['sc1 nt (default)', 'sc1', 'nt', 'plain', 'sc1 on odd rows', 'sc1 on odd experts', 'sc1 on every 4th row']


def main():
    torch.cuda.set_device(0)
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29651')
    dist.init_process_group('gloo', rank=0, world_size=1)
    from deepep_amd import ElasticBuffer
    T, H, K, E = 8192, 7168, 8, 256
    torch.manual_seed(0)
    w, idx = torch.topk(torch.rand((T, E), device='cuda'), K, dim=-1, sorted=False)
    x = torch.randn((T, H), device='cuda').to(torch.bfloat16)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    ref_x, _, ref_w, h, _ = buf.dispatch(x, topk_idx=idx.to(torch.int64), topk_weights=w, num_experts=E,
                                         do_expand=True)
    lib = buf.kernels.lib
    s = torch.cuda.current_stream()
    nbytes = T * H * 2 + ref_x.shape[0] * H * 2
    times = {p: [] for p in range(len(NAMES))}
    same = {p: True for p in range(len(NAMES))}
    for _ in range(int(os.environ.get('KCOPY_ROUNDS', 5))):
        for p in range(len(NAMES)):
            assert lib.deepep_set_dispatch_copy_policy(p) == 0
            times[p].append(timeit(lambda: buf.dispatch(x, topk_weights=w, do_expand=True, handle=h), s, iters=30))
            out_x, _, out_w, _, _ = buf.dispatch(x, topk_weights=w, do_expand=True, handle=h)
            same[p] = same[p] and bool(torch.equal(out_x, ref_x) and torch.equal(out_w, ref_w))
    lib.deepep_set_dispatch_copy_policy(0)
    for p in range(len(NAMES)):
        med = statistics.median(times[p])
        print(json.dumps(dict(policy=NAMES[p], cached_dispatch_us=round(med, 2), gbps=round(nbytes / med / 1e3, 1),
                              bitwise=same[p])), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
