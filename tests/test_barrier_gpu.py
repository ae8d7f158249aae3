"""ElasticBuffer.barrier on the GPU (elastic.py:497-508, buffer.hpp:181-208): a device barrier ordered on the
comm stream that the host does not wait for (unless with_cpu_sync), and that holds every rank's stream until
the last rank's stream arrives.

  rccl   one rank over a real RCCL group: the barrier is queued behind the caller's work and returns to the
         host at once; with_cpu_sync makes the host wait
  xgmi   2 processes sharing the GPU over HIP-IPC windows: rank 0's stream is held by a long device sleep
         before its barrier; rank 1's barrier returns to the host at once, but its stream passes the barrier
         only after rank 0's sleep (the windows' device barrier, deepep_sym_barrier)
"""
import os
import socket
import sys
import time
import traceback

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SLEEP_S = 0.3
MIN_S = 0.05                   # the device sleep must be long enough to time on the host


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _sleep_cycles(seconds: float) -> int:
    """torch.cuda._sleep cycles for about `seconds` on this device (measured)."""
    n = 1_000_000
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(n)                                   # warm-up
    e0.record()
    torch.cuda._sleep(n)
    e1.record()
    torch.cuda.synchronize()
    return max(1, int(n * seconds * 1e3 / max(e0.elapsed_time(e1), 1e-3)))


def _timed_barrier(buf, cycles, **kw):
    """(host seconds until barrier() returned, seconds until the device passed it), with `cycles` of device
    sleep queued before it on the current stream (0: none)."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if cycles:
        torch.cuda._sleep(cycles)
    buf.barrier(**kw)
    t_call = time.perf_counter() - t0
    torch.cuda.synchronize()
    return t_call, time.perf_counter() - t0


def _rccl_worker(port, queue):
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
        from deepep_amd import ElasticBuffer
        buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=16, hidden=64, num_topk=2)
        buf.barrier()                                      # the communicator's first use
        torch.cuda.synchronize()
        cycles = _sleep_cycles(SLEEP_S)
        res = {name: _timed_barrier(buf, cycles, **kw) for name, kw in
               (('comm_stream', {}), ('current_stream', dict(use_comm_stream=False)),
                ('cpu_sync', dict(with_cpu_sync=True)))}
        queue.put(res)
        dist.destroy_process_group()
    except Exception:
        queue.put(traceback.format_exc())


def test_rccl_barrier_is_stream_ordered():
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), queue))
    p.start()
    try:
        res = queue.get(timeout=150)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert isinstance(res, dict), res
    # relative to each run's own device time (the sleep counts shader clocks, which vary with the clock)
    for name in ('comm_stream', 'current_stream'):
        t_call, t_done = res[name]
        assert t_done > MIN_S and t_call < 0.5 * t_done, (name, res)           # queued, not waited for
    t_call, t_done = res['cpu_sync']
    assert t_done > MIN_S and t_call > 0.9 * t_done, res                        # with_cpu_sync: the host waits


def _xgmi_worker(rank, world, port, queue):
    sys.path.insert(0, ROOT)
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        os.environ['DEEPEP_TRANSPORT'] = 'xgmi'
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from deepep_amd import ElasticBuffer
        T, H, K, E = 32, 256, 2, 4 * world
        g = torch.Generator(device='cuda').manual_seed(rank)
        buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                            explicitly_destroy=True, num_gpu_timeout_secs=30)
        x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
        idx = torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1)[1]
        ex_x, _, _, handle, _ = buf.dispatch(x, topk_idx=idx, num_experts=E, do_expand=True)
        buf.combine(ex_x, handle)                          # the window exists from here on
        assert buf._sym is not None
        cycles = _sleep_cycles(SLEEP_S)
        res = {}
        for name, kw in (('comm_stream', {}), ('current_stream', dict(use_comm_stream=False))):
            torch.cuda.synchronize()
            dist.barrier()                                 # both ranks start together
            res[name] = _timed_barrier(buf, cycles if rank == 0 else 0, **kw)
        # the windows still serve a combine after the barriers (epochs agree on every rank)
        out, _, _ = buf.combine(ex_x, handle)
        ref, _, _ = buf.combine(ex_x, handle)
        torch.cuda.synchronize()
        res['combine_after'] = bool(torch.equal(out, ref))
        buf._sym.check()
        buf.destroy()
        queue.put((rank, res))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        queue.put((rank, traceback.format_exc()))


def test_xgmi_barrier_holds_the_stream_not_the_host():
    world = 2
    ctx = mp.get_context('spawn')
    queue = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xgmi_worker, args=(r, world, port, queue)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, res = queue.get(timeout=150)
            results[rank] = res
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(isinstance(v, dict) for v in results.values()) and len(results) == world, results
    for name in ('comm_stream', 'current_stream'):
        c0, d0 = results[0][name]
        c1, d1 = results[1][name]
        assert d0 > MIN_S, (name, results)                                     # rank 0's stream slept
        assert c0 < 0.5 * d0 and c1 < 0.5 * d0, (name, results)               # neither host waited
        assert d1 > 0.5 * d0, (name, results)                                  # rank 1's stream waited for rank 0
    assert all(results[r]['combine_after'] for r in range(world)), results
