"""ElasticBuffer.barrier on the GPU (elastic.py:497-508, buffer.hpp:181-208): a device barrier ordered on the
comm stream that the host does not wait for (unless with_cpu_sync), and that holds every rank's stream until
the last rank's stream arrives.

  rccl   one rank over a real RCCL group: the barrier is queued behind the caller's work and returns to the
         host at once; with_cpu_sync makes the host wait
  xgmi   2 processes sharing the GPU over HIP-IPC windows: rank 0's stream is held by a long device spin
         before its barrier; rank 1's barrier returns to the host at once, but its stream passes the barrier
         only after rank 0's spin (the windows' device barrier, deepep_sym_barrier)

Ordering is proven on the device: kernels of tests/probe/libstamp.so store the GPU's constant 100 MHz clock
(wall_clock64, one counter for every process on the GPU) when a stream reaches them -- at the end of the
pre-barrier spin and right after the barrier -- so "rank 1 passed the barrier after rank 0's work ended" is a
comparison of two device timestamps, not of host wall-clock ratios.  The spin is in that clock too, so its
length does not depend on the shader clock.  The host-returned-early checks stay host-timed.
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
SPIN_S = 0.3                   # the pre-barrier device spin (wall-clock time)
STAMP_LIB = os.path.join(ROOT, 'tests', 'probe', 'libstamp.so')


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


class _Clock:
    """Device clock probes: stamp(i, stream) stores the GPU clock into slot i when `stream` reaches it;
    spin(seconds, i, stream) holds the stream for that long in wall-clock time, then stamps slot i."""

    def __init__(self, n: int = 16):
        import ctypes
        self.lib = ctypes.CDLL(STAMP_LIB)
        self.lib.stamp_clock.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self.lib.spin_ticks.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        self.hz = self.lib.clock_rate_khz() * 1000
        assert self.hz > 0
        self.slots = torch.zeros(n, dtype=torch.int64, device='cuda')

    def _ptr(self, i):
        return self.slots.data_ptr() + 8 * i

    def stamp(self, i, stream=None):
        stream = stream or torch.cuda.current_stream()
        assert self.lib.stamp_clock(self._ptr(i), stream.cuda_stream) == 0

    def spin(self, seconds, i, stream=None):
        stream = stream or torch.cuda.current_stream()
        assert self.lib.spin_ticks(int(seconds * self.hz), self._ptr(i), stream.cuda_stream) == 0

    def seconds(self):
        """All slots as seconds of the device clock."""
        return [v / self.hz for v in self.slots.cpu().tolist()]


def _timed_barrier(buf, clock, spin: bool, base: int, **kw):
    """Slots base+0: end of the pre-barrier spin (or a stamp with no spin), base+1: the current stream right
    after the barrier, base+2: the comm stream right after it.  Returns (host seconds until barrier()
    returned, host seconds until the device had passed it)."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if spin:
        clock.spin(SPIN_S, base)
    else:
        clock.stamp(base)
    buf.barrier(**kw)
    t_call = time.perf_counter() - t0
    clock.stamp(base + 1)
    if kw.get('use_comm_stream', True):
        clock.stamp(base + 2, buf.comm_stream)
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
        clock = _Clock()
        res = {name: _timed_barrier(buf, clock, True, 3 * i, **kw) for i, (name, kw) in
               enumerate((('comm_stream', {}), ('current_stream', dict(use_comm_stream=False)),
                          ('cpu_sync', dict(with_cpu_sync=True))))}
        res['stamps'] = clock.seconds()
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
    st = res['stamps']
    for i, name in enumerate(('comm_stream', 'current_stream', 'cpu_sync')):
        spin_end, after_cur, after_comm = st[3 * i:3 * i + 3]
        # device order: the stream passed the barrier after the caller's pre-barrier work had ended
        assert after_cur >= spin_end, (name, st)
        if name != 'current_stream':
            assert after_comm >= spin_end, (name, st)      # the comm stream waited for the caller's stream
        t_call, t_done = res[name]
        assert t_done > 0.9 * SPIN_S, (name, res)
        if name == 'cpu_sync':
            assert t_call > 0.9 * SPIN_S, res              # with_cpu_sync: the host waits
        else:
            assert t_call < 0.5 * SPIN_S, (name, res)      # queued, not waited for


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
        clock = _Clock()
        res = {}
        for i, (name, kw) in enumerate((('comm_stream', {}), ('current_stream', dict(use_comm_stream=False)))):
            torch.cuda.synchronize()
            dist.barrier()                                 # both ranks start together
            res[name] = _timed_barrier(buf, clock, rank == 0, 3 * i, **kw)
        res['stamps'] = clock.seconds()
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
    s0, s1 = results[0]['stamps'], results[1]['stamps']
    for i, name in enumerate(('comm_stream', 'current_stream')):
        spin_end0, after0 = s0[3 * i], s0[3 * i + 1]
        before1, after1 = s1[3 * i], s1[3 * i + 1]
        # device order (one clock for both processes): rank 1's stream passed the barrier only after rank 0's
        # pre-barrier spin had ended, although rank 1 reached the barrier while rank 0 was still spinning
        assert after1 >= spin_end0, (name, s0, s1)
        assert after0 >= spin_end0, (name, s0, s1)
        assert before1 < spin_end0, (name, s0, s1)
        assert after1 - before1 > 0.5 * SPIN_S, (name, s0, s1)
        if name == 'comm_stream':
            assert s1[3 * i + 2] >= spin_end0, (name, s0, s1)          # rank 1's comm stream too
        c0, d0 = results[0][name]
        c1, _ = results[1][name]
        assert d0 > 0.9 * SPIN_S, (name, results)
        assert c0 < 0.5 * SPIN_S and c1 < 0.5 * SPIN_S, (name, results)   # neither host waited
    assert all(results[r]['combine_after'] for r in range(world)), results
