"""Several EP ranks on one GPU, one host thread each -- TEST INFRASTRUCTURE ONLY.

`ThreadComm` stands in for the RCCL process group of ElasticBuffer's exchanges with the stream
semantics of ProcessGroupNCCL (torch/csrc/distributed/c10d/ProcessGroupNCCL.cpp), not a host-blocking
copy:

* the collective is queued on a per-rank side stream (NCCL's internal stream) behind an event recorded
  on the caller's current stream -- so it starts only after the work the caller queued before it
  (phase A of the chunk);
* it completes as a whole: a rank's completion event comes after every rank's receive copies, so a
  sender's input buffer is never reused while a peer still reads it;
* `Work.wait()` makes the CALLER's current stream wait for that event and returns at once (no host
  synchronisation) -- exactly what `dist.all_to_all_single(..., async_op=True).wait()` does with NCCL;
* the blocking form (`a2a`) is the same collective followed by `wait()`, as a blocking NCCL call is
  stream-ordered too.
`delay_cycles` makes every collective sleep on its side stream first (torch.cuda._sleep), so a consumer
that forgets to wait for it reads the receive buffer before the data lands -- the schedule tests use
it to prove that the ordering they rely on is really enforced.
"""
import threading
from typing import List, Optional

import torch


class Work:
    """The handle of an emulated NCCL collective."""

    def __init__(self, event: torch.cuda.Event):
        self.event = event

    def wait(self) -> bool:
        torch.cuda.current_stream().wait_event(self.event)
        return True

    def is_completed(self) -> bool:
        return self.event.query()


class ThreadComm:
    """all_to_all_single among threads that each drive one simulated rank on the same GPU."""

    def __init__(self, n: int, delay_cycles: int = 0):
        self.n = n
        self.bar = threading.Barrier(n)
        self.slots: List[Optional[tuple]] = [None] * n
        self.done: List[Optional[torch.cuda.Event]] = [None] * n
        self.side: List[Optional[torch.cuda.Stream]] = [None] * n
        self.delay_cycles = delay_cycles
        self.calls = [0] * n

    def a2a_async(self, rank: int, out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None) -> Work:
        if self.side[rank] is None:
            self.side[rank] = torch.cuda.Stream()
        side = self.side[rank]
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream())           # the caller's earlier work (phase A)
        splits = in_splits if in_splits is not None else [inp.shape[0] // self.n] * self.n
        self.slots[rank] = (inp, splits, ready)
        self.bar.wait()                                      # every rank reached the collective
        with torch.cuda.stream(side):
            for s in range(self.n):
                side.wait_event(self.slots[s][2])
            if self.delay_cycles:
                torch.cuda._sleep(self.delay_cycles)
            pos = 0
            for s in range(self.n):
                sinp, ssplits, _ = self.slots[s]
                start, cnt = sum(ssplits[:rank]), ssplits[rank]
                out[pos:pos + cnt].copy_(sinp[start:start + cnt])
                sinp.record_stream(side)
                pos += cnt
            assert pos == out.shape[0], (pos, out.shape)
            out.record_stream(side)
            mine = torch.cuda.Event()
            mine.record(side)
        self.done[rank] = mine
        self.bar.wait()                                      # every rank queued its receive copies
        with torch.cuda.stream(side):
            for s in range(self.n):
                side.wait_event(self.done[s])
            final = torch.cuda.Event()
            final.record(side)
        self.calls[rank] += 1
        self.bar.wait()                                      # slots may be reused by the next collective
        return Work(final)

    def a2a(self, rank: int, out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None) -> None:
        self.a2a_async(rank, out, inp, out_splits, in_splits).wait()

    def install(self, buf, rank: int) -> None:
        """Route `buf`'s exchanges through this communicator."""
        buf._a2a = lambda out, inp, os_=None, is_=None: self.a2a(rank, out, inp, os_, is_)
        buf._a2a_async = lambda out, inp, os_, is_: self.a2a_async(rank, out, inp, os_, is_)


class FakeGroup:
    """The process-group surface ElasticBuffer uses (rank, size, barrier)."""

    def __init__(self, rank: int, n: int, comm: ThreadComm):
        self._rank, self._n, self.comm = rank, n, comm

    def rank(self) -> int:
        return self._rank

    def size(self) -> int:
        return self._n

    def barrier(self) -> None:
        self.comm.bar.wait()


def run_threads(world: int, target, args=(), timeout: float = 300) -> dict:
    """Run target(rank, *args, results) on `world` threads; returns results {rank: failures}."""
    torch.cuda.init()                                   # CUDA initialised here, not lazily by racing threads
    torch.cuda.get_device_properties(0)
    results = {}
    threads = [threading.Thread(target=target, args=(r, *args, results)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=timeout)
    return results
