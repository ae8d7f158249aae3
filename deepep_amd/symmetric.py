"""Symmetric receive buffer over xGMI and its device barrier.

Replaces the reference's NCCLSymmetricMemoryContext (csrc/elastic/nccl.cu:62-153,
csrc/elastic/buffer.hpp:181-208: one window per rank, every peer's window addressable
from kernels) and gpu_barrier (deep_ep/include/deep_ep/common/comm.cuh:88-129).

Every rank allocates one uncached device window (deepep_sym_alloc), exports it with
HIP IPC, and opens every peer's window (deepep_sym_import); kernels then store into a
peer's HBM over xGMI.  Layout of a window:

    [0, 32 KiB)              int64 flags[64 slots][64 ranks]: barrier epochs written by the peers
                             (slot 0: the full barrier; slots 1..63: split barriers of pipelined phases),
                             then int64 counters[3][64 slots]: this rank's device-side epoch counts
    [NOTIFY_OFFSET, HEADER_BYTES)  the notify area: slot s holds rank s's dispatch counts for this rank
    [HEADER_BYTES, ...)      data: the dispatch's received rows / the combine receive rows
"""
import ctypes
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

from . import _lib

HEADER_BYTES = 1 << 20          # DEEPEP_SYM_HEADER_BYTES
NOTIFY_OFFSET = 64 * 1024       # DEEPEP_SYM_NOTIFY_OFFSET


class _DeviceArray:
    """Wrap a raw device allocation as a torch tensor without copying (__cuda_array_interface__)."""

    def __init__(self, address: int, nbytes: int):
        self.__cuda_array_interface__ = {'shape': (nbytes,), 'typestr': '|u1', 'data': (address, False),
                                         'version': 3, 'strides': None}


class SymmetricBuffer:
    """One window per rank, mapped into every peer; `barrier(stream)` is a device-side group barrier.

    exchange: optional hook `exchange(local_base) -> [base of every rank]` for ranks that share a
    process (the single-GPU thread simulation); by default IPC handles are all-gathered over `group`.
    """

    def __init__(self, group, rank: int, num_ranks: int, data_bytes: int, device: torch.device,
                 exchange: Optional[Callable[[int], List[int]]] = None, timeout_s: float = 100.0):
        self.lib = _lib.load()
        self.rank, self.num_ranks = rank, num_ranks
        self.device = device
        self.data_bytes = int(data_bytes)
        self.timeout_us = int(timeout_s * 1e6)
        p = ctypes.c_void_p()
        _lib.check(self.lib.deepep_sym_alloc(HEADER_BYTES + self.data_bytes, ctypes.byref(p)), 'sym_alloc')
        self.base = int(p.value)
        self._imported: List[int] = []
        if exchange is not None:
            bases = [int(b) for b in exchange(self.base)]
        else:
            bases = self._ipc_exchange(group)
        if len(bases) != num_ranks or bases[rank] != self.base:
            raise RuntimeError('deepep_amd: window exchange returned inconsistent bases')
        self.bases = bases
        self.bases_dev = torch.tensor(bases, dtype=torch.int64, device=device)     # flags live at offset 0
        self.data_bases_dev = self.bases_dev + HEADER_BYTES
        self.data = torch.as_tensor(_DeviceArray(self.base + HEADER_BYTES, self.data_bytes), device=device)
        # error record (_lib.ERROR_RECORD_INTS ints): [0] the flag bits every window kernel reads / sets,
        # [1..] the first bad-address fault; error_flag is a view of [0] whose pointer is the record's
        self.error_record = torch.zeros((_lib.ERROR_RECORD_INTS,), dtype=torch.int32, device=device)
        self.error_flag = self.error_record[:1]
        self.epoch = 0
        self._slot_epoch = [0] * 64                 # split-barrier counters (slot 0 = the full barrier)

    def _ipc_exchange(self, group) -> List[int]:
        handle = ctypes.create_string_buffer(64)
        _lib.check(self.lib.deepep_sym_export(ctypes.c_void_p(self.base), handle), 'sym_export')
        handles: List[Optional[bytes]] = [None] * self.num_ranks
        dist.all_gather_object(handles, handle.raw, group=group)
        bases = []
        for s, h in enumerate(handles):
            if s == self.rank:
                bases.append(self.base)
                continue
            p = ctypes.c_void_p()
            _lib.check(self.lib.deepep_sym_import(ctypes.create_string_buffer(h, 64), ctypes.byref(p)), 'sym_import')
            self._imported.append(int(p.value))
            bases.append(int(p.value))
        return bases

    # Epochs are counted on the device (epoch argument 0): every launch -- including each replay of a
    # captured HIP graph -- takes the next one from this rank's counter in its window header.  The
    # host-side counts below are for tracing only.
    def barrier(self, stream) -> None:
        """Device-side group barrier on `stream` (all ranks must call it the same number of times)."""
        self.epoch += 1
        handle = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
        _lib.check(self.lib.deepep_sym_barrier(self.bases_dev.data_ptr(), self.rank, self.num_ranks, 0,
                                               self.timeout_us, self.error_flag.data_ptr(), handle), 'sym_barrier')

    def signal(self, slot: int, stream) -> None:
        """Publish this rank's arrival at split barrier `slot` (1..63) after `stream`'s earlier work."""
        self._slot_epoch[slot] += 1
        handle = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
        _lib.check(self.lib.deepep_sym_signal(self.bases_dev.data_ptr(), self.rank, self.num_ranks, slot, 0, handle),
                   'sym_signal')

    def wait(self, slot: int, stream) -> None:
        """Make `stream` wait until every rank has signalled `slot` as often as this rank waited on it."""
        handle = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
        _lib.check(self.lib.deepep_sym_wait(self.bases_dev.data_ptr(), self.rank, self.num_ranks, slot, 0,
                                            self.timeout_us, self.error_flag.data_ptr(), handle), 'sym_wait')

    def publish(self, stream) -> None:
        """Queue a copy of the error flag to pinned host memory behind `stream`'s work (no host
        sync); poll() reads it once it has landed.  Not for use inside a HIP-graph capture."""
        with torch.cuda.stream(stream):
            if getattr(self, '_flag_host', None) is None:
                self._flag_host = torch.zeros((_lib.ERROR_RECORD_INTS,), dtype=torch.int32, pin_memory=True)
            self._flag_host.copy_(self.error_record, non_blocking=True)
            self._flag_event = torch.cuda.Event()
            self._flag_event.record(stream)

    def poll(self) -> None:
        """Raise if an earlier call's published flag shows a barrier timeout (no host sync: a copy
        that has not landed yet is checked at a later call) -- the reference traps instead."""
        ev = getattr(self, '_flag_event', None)
        if ev is not None and ev.query():
            self._flag_event = None
            rec = self._flag_host.tolist()
            if rec[0]:
                why = ('a peer did not arrive within num_gpu_timeout_secs' if rec[0] & _lib.FLAG_TIMEOUT else
                       'a window address or plan entry was rejected (nothing was stored through it)')
                raise RuntimeError(f'deepep_amd: symmetric buffer {_lib.describe_error_record(rec)}: {why}; '
                                   f'the last results are invalid')

    def put_notify(self, records: torch.Tensor, stream) -> None:
        """Store records[d] (int32 [num_ranks, n], n * 4 a multiple of 16 bytes) into slot `rank` of rank d's
        notify area (the dispatch notify's transport); a barrier must follow before it is read."""
        # explicit checks (not asserts, which python -O strips): the put's extent must stay inside the notify area
        if not (records.dtype == torch.int32 and records.is_contiguous() and records.shape[0] == self.num_ranks):
            raise RuntimeError('deepep_amd: notify records must be contiguous int32 [num_ranks, n]')
        n = records.shape[1]
        if (n * 4) % 16 != 0 or self.num_ranks * n * 4 > HEADER_BYTES - NOTIFY_OFFSET:
            raise RuntimeError(f'deepep_amd: notify record of {n} ints x {self.num_ranks} ranks does not fit the '
                               f'{HEADER_BYTES - NOTIFY_OFFSET}-byte notify area in 16-byte units')
        handle = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
        # dest_extent = the header: the C-ABI bound then covers the region this put may write (the notify
        # area), not the whole window whose data region holds received rows
        _lib.check(self.lib.deepep_sym_put(records.data_ptr(), n * 4, self.bases_dev.data_ptr(), self.num_ranks,
                                           NOTIFY_OFFSET + self.rank * n * 4, HEADER_BYTES,
                                           self.error_flag.data_ptr(), handle),
                   'sym_put')

    def notify_area(self, n: int) -> torch.Tensor:
        """This rank's notify area as int32 [num_ranks, n]: row s = what rank s put here."""
        return torch.as_tensor(_DeviceArray(self.base + NOTIFY_OFFSET, self.num_ranks * n * 4),
                               device=self.device).view(torch.int32).view(self.num_ranks, n)

    def check(self) -> None:
        """Raise if a barrier timed out or a window address was rejected (host sync)."""
        rec = self.error_record.tolist()
        if rec[0]:
            raise RuntimeError(f'deepep_amd: symmetric buffer {_lib.describe_error_record(rec)}')

    def reset_error(self) -> None:
        """Clear the flag and the fault record (stream-ordered on the current stream)."""
        self.error_record.zero_()
        self._flag_event = None

    def destroy(self) -> None:
        if self.base is None:
            return
        torch.cuda.synchronize(self.device)
        self.data = None
        for p in self._imported:
            _lib.check(self.lib.deepep_sym_close(ctypes.c_void_p(p)), 'sym_close')
        self._imported = []
        _lib.check(self.lib.deepep_sym_free(ctypes.c_void_p(self.base)), 'sym_free')
        self.base = None
