"""The EP = N combine of bench.py, for rocprofv3 --pmc passes (one counter set per run): N ranks
simulated by threads on the one GPU (tests/sim.py: the exchange with NCCL stream semantics), each
with bench.py's inputs (seed = rank, uniform routing, 8192 x 7168 x top-8, 256 experts, gating-weighted,
expanded layout), the real library path (HIP dispatch, device-built plan), ONE chunk per rank so each
rank's phase A is one launch over its whole share.  A 512 MB flush precedes every combine.
Writes gpurun_out/pmc_ep{N}[_nobypass]_meta.json: the algorithmic bytes of every rank's phase-A and phase-B
launch (the definitions bench.py uses for its N > 1 roofline), in launch order, and every rank's rows of
itself (the all-to-all diagonal the local bypass removes) with the packed row size -- `summarize_prof.py
step` sums every kernel of the whole step (phase A + the exchange's copies + phase B) from the same passes.
usage: rocprofv3 --pmc FETCH_SIZE -d OUT -o pmc --output-format csv -- python3 tools/pmc_ep.py N [reps]
       (DEEPEP_LOCAL_BYPASS=0 in the environment: the all-to-all carries the diagonal, for the A/B)"""
import json
import os
import sys
import threading

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    os.environ['DEEPEP_COMBINE_CHUNKS'] = '1'
    os.environ['DEEPEP_TRANSPORT'] = 'rccl'
    from deepep_amd import ElasticBuffer
    from tests.sim import FakeGroup, ThreadComm
    T, H, K, E = 8192, 7168, 8, 256
    torch.cuda.init()
    torch.cuda.get_device_properties(0)
    comm = ThreadComm(world)
    flush = torch.empty((512 << 20) // 4, dtype=torch.int32, device='cuda')
    lock = threading.Lock()
    meta = {'a_bytes': [None] * world, 'b_bytes': [None] * world, 'own_rows': [None] * world,
            'sent_rows': [None] * world}
    errors = []

    def rank_fn(rank):
        try:
            torch.cuda.set_device(0)
            with lock:                                   # bench.py's inputs: torch.manual_seed(0 + rank)
                torch.manual_seed(rank)
                scores = torch.rand((T, E), device='cuda')
                x = torch.randn((T, H), device='cuda').to(torch.bfloat16)
            w, idx = torch.topk(scores, K, dim=-1, sorted=False)
            idx = idx.to(torch.int64)
            buf = ElasticBuffer(FakeGroup(rank, world, comm), num_max_tokens_per_rank=T, hidden=H, num_topk=K)
            comm.install(buf, rank)
            ex_x, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
            y = torch.randn(ex_x.shape, device='cuda').to(torch.bfloat16)
            del ex_x
            n_recv = sum(handle._recv_counts)
            n_rows = int((handle.recv_src_metadata[:n_recv, 2:] >= 0).sum().item())
            valid = int((idx >= 0).sum().item())
            # bench.py: phase A reads the valid expanded rows and writes one partial row + K weights per
            # received token; phase B: the token's output (the combine's algorithmic bytes per rank)
            meta['a_bytes'][rank] = n_rows * H * 2 + n_recv * (H * 2 + K * 4)
            meta['b_bytes'][rank] = valid * H * 2 + T * H * 2 + valid * 4 + valid * 4
            for _ in range(reps):
                comm.bar.wait()
                if rank == 0:
                    flush.zero_()
                    torch.cuda.synchronize()
                comm.bar.wait()
                buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
                torch.cuda.synchronize()
            plan = next(p for k, p in handle._combine_plans.items() if k[0] == 'multi')
            meta['own_rows'][rank] = sum(ch.send_counts[rank] for ch in plan.chunks)
            meta['sent_rows'][rank] = sum(sum(ch.send_counts) for ch in plan.chunks)
        except Exception:
            import traceback
            errors.append(traceback.format_exc())
            comm.bar.abort()

    threads = [threading.Thread(target=rank_fn, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        print(errors[0], file=sys.stderr)
        sys.exit(1)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    from deepep_amd.handle import packed_row_layout
    bypass = os.environ.get('DEEPEP_LOCAL_BYPASS', '1') != '0'
    meta.update(world=world, reps=reps, tokens=T, hidden=H, topk=K, experts=E, local_bypass=bypass,
                packed_row_bytes=packed_row_layout(H, K, True)[0])
    tag = '' if bypass else '_nobypass'
    with open(os.path.join(ROOT, 'gpurun_out', f'pmc_ep{world}{tag}_meta.json'), 'w') as f:
        json.dump(meta, f)
    print(json.dumps(meta))


if __name__ == '__main__':
    main()
