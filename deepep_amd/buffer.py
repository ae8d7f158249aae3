"""ElasticBuffer: the drop-in Python surface for DeepEP's combine path on MI355X.

Mirrors deep_ep.ElasticBuffer (deep_ep/buffers/elastic.py:195-1107 in /root/reference):
same constructor and method signatures, same argument meaning, same stream
semantics (csrc/elastic/buffer.hpp:526-584) and the same error behaviour
(RuntimeError on a violated host assertion).  What differs is underneath:

* combine (the hot path) runs hand-written gfx950 kernels from libdeepep_amd.so:
  EP = 1   one fused launch (local reduce + epilogue, no receive buffer);
  EP > 1   phase A (local reduce per received token) -> one RCCL all_to_all_single
           of the bf16 partials over xGMI -> phase B (epilogue reduce + bias).
* dispatch (the handle producer) is seven HIP kernels (csrc/dispatch.hip) around one
  exchange of counts (one host sync) and one RCCL all_to_all_single of packed token
  rows; it produces the reference's handle layout (recv_src_metadata etc.) with the
  deterministic receive order the combine plan relies on (handle.py).

Single node only: num_scaleout_ranks == 1 (hybrid RDMA mode, Engram, PP and AGRS
are out of scope for this build).
"""
import math
import os
from typing import List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist

from .event import EventHandle, EventOverlap
from .exchange import ExchangeMixin
from .handle import BlockCounts, CombinePlan, EPHandle, build_ep_plan, chunk_geometry
from ._lib import DISPATCH_BLOCK_ROWS
from .kernels import MODE_EPILOGUE, MODE_FUSED, MODE_LOCAL, RowLayout
from .utils import align, ceil_div, check_torch_deterministic, value_or

topk_idx_t = torch.int32 if int(os.environ.get('EP_NUM_TOPK_IDX_BITS', 64)) == 32 else torch.int64

BUFFER_ALIGNMENT = 2 * 1024 * 1024          # symmetric::kNumAlignmentBytes (symmetric.hpp:16)
# CU-budget streams (deepep_stream_create_cu_budget), keyed by (device, CUs); they live for the whole
# process, so tensors whose allocator records them stay valid after their buffer is destroyed
_BUDGET_STREAMS = {}
_TOKEN_ALIGN = 32                           # ptx::kNumTMAAlignBytes (ptx.cuh:16)


def _assert(cond: bool, msg: str = '') -> None:
    """EP_HOST_ASSERT: the reference raises EPException, surfaced to Python as RuntimeError."""
    if not cond:
        raise RuntimeError(f'Assertion failed: {msg}')


def _token_bytes(hidden_bytes: int, sf_bytes: int, num_topk: int, with_metadata: bool) -> int:
    """TokenLayout::get_num_bytes<false> (layout.cuh:179-209)."""
    meta = num_topk * 8 + ((1 + num_topk) * 4 if with_metadata else 0)
    return (align(hidden_bytes, _TOKEN_ALIGN) + align(sf_bytes, _TOKEN_ALIGN) + align(meta, _TOKEN_ALIGN))


def calculate_buffer_size(num_ranks: int, num_max_tokens_per_rank: int, hidden: int, num_topk: int,
                          use_fp8_dispatch: bool, allow_multiple_reduction: bool) -> int:
    """ElasticBuffer::calculate_buffer_size for one node (buffer.hpp:589-686)."""
    _assert(num_max_tokens_per_rank > 0 and hidden > 0, 'num_max_tokens_per_rank > 0 and hidden > 0')
    num_topk = 32 if num_topk == 0 else num_topk
    elem = 1 if use_fp8_dispatch else 2
    num_sf_packs = ceil_div(hidden, 32) if use_fp8_dispatch else 0
    dispatch_bytes = num_ranks * num_max_tokens_per_rank * _token_bytes(hidden * elem, num_sf_packs * 4, num_topk, True)
    slots = min(num_ranks, num_topk) if allow_multiple_reduction else num_topk
    combine_bytes = slots * num_max_tokens_per_rank * _token_bytes(hidden * 2, 0, num_topk, False)
    return align(max(dispatch_bytes, combine_bytes), BUFFER_ALIGNMENT)


def notify_layout(notify: List[int], num_ranks: int, rank: int, experts_per_rank: int, all_gathered: bool,
                  num_blocks: int = 0):
    """Host view of the dispatch notify (dispatch.cuh:79-258; buffer.hpp:1017-1064's CPU wait).
    Each record is [tokens | tokens per local expert | tokens per 64-token block | (token, lane) pairs
    per block] (1 + experts_per_rank + 2 * num_blocks ints) from a source to a destination; the block
    counts size the pipeline chunks of the EP > 1 combine (handle.BlockCounts).  `notify` holds the
    records this rank received, one per source (all_gathered False), or every rank's records to every
    destination, [source][destination] (all_gathered True: the xGMI push needs them).  Returns (tokens
    this rank sends per destination -- only when all_gathered, else None -- tokens received per
    source, rows received per local expert, when all_gathered the row offset of this rank's rows
    inside every destination's receive window (the rows the lower source ranks send there come
    first), and the block counts received from every source, [source][2 * num_blocks])."""
    R, r, w = num_ranks, rank, 1 + experts_per_rank + 2 * num_blocks
    if all_gathered:
        grid = [[notify[(s * R + d) * w:(s * R + d + 1) * w] for d in range(R)] for s in range(R)]
        rows = [grid[s][r] for s in range(R)]
        sends = [grid[r][d][0] for d in range(R)]
        offsets = [sum(grid[s][d][0] for s in range(r)) for d in range(R)]
    else:
        rows = [notify[i * w:(i + 1) * w] for i in range(R)]
        sends, offsets = None, None
    recv = [row[0] for row in rows]
    experts = [sum(row[1 + e] for row in rows) for e in range(experts_per_rank)]
    blocks = [list(row[1 + experts_per_rank:]) for row in rows]
    return sends, recv, experts, offsets, blocks


class ElasticBuffer(ExchangeMixin):
    """The elastic EP buffer (single node): dispatch produces an EPHandle, combine reduces.
    The EP > 1 exchanges of the combine (RCCL all-to-all, xGMI windows) live in ExchangeMixin
    (exchange.py)."""

    def __init__(self,
                 group: dist.ProcessGroup,
                 num_bytes: Optional[int] = None,
                 num_cpu_bytes: int = 0,
                 num_max_tokens_per_rank: int = 0,
                 hidden: int = 0,
                 num_topk: int = 0,
                 use_fp8_dispatch: bool = False,
                 deterministic: bool = False,
                 allow_hybrid_mode: bool = True,
                 allow_multiple_reduction: bool = True,
                 prefer_overlap_with_compute: bool = True,
                 sl_idx: int = 3,
                 num_allocated_qps: int = 0,
                 num_cpu_timeout_secs: int = 300, num_gpu_timeout_secs: int = 100,
                 explicitly_destroy: bool = False):
        self.group = group
        self.rank_idx = group.rank()
        self.num_ranks = group.size()
        self.allow_hybrid_mode = allow_hybrid_mode
        self.allow_multiple_reduction = allow_multiple_reduction
        self.prefer_overlap_with_compute = prefer_overlap_with_compute
        self.deterministic = deterministic
        _assert(num_cpu_bytes == 0, 'CPU buffer segments (Engram storage) are not supported by this build')
        if num_bytes is None:
            num_bytes = calculate_buffer_size(self.num_ranks, num_max_tokens_per_rank, hidden, num_topk,
                                              use_fp8_dispatch, allow_multiple_reduction)
        _assert(num_bytes % BUFFER_ALIGNMENT == 0, 'num_bytes must be aligned to 2 MB')
        if os.environ.get('EP_BUFFER_DEBUG', 0):
            print(f'Initializing EP elastic buffer with {num_bytes} bytes at rank EP {self.rank_idx}/{self.num_ranks}')
        self.num_bytes = num_bytes
        self.num_max_tokens_per_rank = num_max_tokens_per_rank
        if num_allocated_qps == 0:
            num_allocated_qps = 17 if not allow_hybrid_mode else 65
        self.num_allocated_qps = num_allocated_qps
        self.num_cpu_timeout_secs = num_cpu_timeout_secs
        self.num_gpu_timeout_secs = num_gpu_timeout_secs
        self.explicitly_destroy = explicitly_destroy
        # One node: every peer is reachable over xGMI (the NVLink domain of the reference)
        self.num_scaleout_ranks, self.num_scaleup_ranks = 1, self.num_ranks
        self.scaleout_rank_idx, self.scaleup_rank_idx = 0, self.rank_idx
        self.num_rdma_ranks, self.num_nvlink_ranks = 1, self.num_ranks
        self.use_cuda = torch.cuda.is_available()
        self.device = torch.device('cuda', torch.cuda.current_device()) if self.use_cuda else torch.device('cpu')
        self.comm_stream = torch.cuda.Stream(device=self.device) if self.use_cuda else None
        self._kernels = None
        self.runtime = self           # non-None while alive (the reference keeps its C++ runtime here)
        self._phase_events = None     # optional list: bench instrumentation of the EP > 1 phases
        self._phase_unpipelined = False   # bench: instrumented calls run one chunk (phases not overlapped)
        # EP > 1 combine transport: 'rccl' (all-to-all of packed partial rows, the default) or 'xgmi'
        # (phase A stores straight into the owners' symmetric windows, deepep_amd/symmetric.py)
        self.transport = os.environ.get('DEEPEP_TRANSPORT', 'rccl')
        _assert(self.transport in ('rccl', 'xgmi'), 'DEEPEP_TRANSPORT must be rccl or xgmi')
        # RCCL combine: this rank's own partials are written in place instead of travelling through the
        # all-to-all's diagonal (DEEPEP_LOCAL_BYPASS=0 turns it off, to measure what it saves)
        self.local_bypass = os.environ.get('DEEPEP_LOCAL_BYPASS', '1') != '0'
        # xGMI combine: CUs for phase A while phase B of earlier chunks runs (0 = the whole chip)
        self.phase_a_cus = int(os.environ.get('DEEPEP_PHASE_A_CUS', 0))
        # CU footprint of a combine called with num_sms=0: 'chip' (default) takes the whole GPU -- the
        # combine is HBM-bound on MI355X, so confining it only slows it; 'handle' is the reference's
        # default: prefer_overlap_with_compute confines the combine to handle.num_sms (its bandwidth
        # model, elastic.py:1086 -> combine_impl's grid, combine.hpp:135) and leaves the rest of the
        # CUs to overlapping compute.  DEEPEP_COMBINE_CUS=handle selects it for every buffer.
        self.combine_cu_mode = os.environ.get('DEEPEP_COMBINE_CUS', 'chip')
        _assert(self.combine_cu_mode in ('chip', 'handle'), 'DEEPEP_COMBINE_CUS must be chip or handle')
        self._sym = None
        self._sym_gen = None
        self._old_sym_gens = set()
        self._capturing = False
        self._sym_exchange = None     # test hook: ranks sharing one process exchange window bases directly
        self._group_barrier()
        # The xGMI transport's symmetric window is allocated here, as the reference allocates its
        # symmetric buffer at construction (buffer.hpp:181-208): a first dispatch / combine then needs
        # no collective set-up (a window too small for a later call is re-allocated there).
        if self.transport == 'xgmi' and self.num_ranks > 1 and self.use_cuda and \
                int(os.environ.get('DEEPEP_EAGER_WINDOW', 1)) and not hasattr(group, 'comm'):
            self._window(self._window_bytes(hidden, num_topk, num_max_tokens_per_rank), slots=1, rows_per_slot=1)

    class _HostCopy:
        """An int32 device vector on its way to pinned host memory (D2H on `stream`, not waited for)."""

        def __init__(self, src: torch.Tensor, pinned: torch.Tensor, stream):
            self.buf = pinned[:src.numel()]
            self.buf.copy_(src, non_blocking=True)
            self.event = torch.cuda.Event()
            self.event.record(stream)

        def wait(self) -> List[int]:
            self.event.synchronize()
            return self.buf.tolist()

    def _host_copy(self, src: torch.Tensor, stream) -> '_HostCopy':
        """Start the D2H of `src` (int32) into this buffer's pinned staging vector; .wait() returns the
        values.  One copy in flight per buffer: a dispatch waits for its own before it returns."""
        n = src.numel()
        prev = getattr(self, '_host_copy_last', None)
        if prev is not None:
            prev.event.synchronize()      # a copy a failed call left in flight must not land on this one's
        if getattr(self, '_pinned', None) is None or self._pinned.numel() < n:
            self._pinned = torch.empty((max(n, 4096),), dtype=torch.int32, pin_memory=True)
        self._host_copy_last = ElasticBuffer._HostCopy(src, self._pinned, stream)
        return self._host_copy_last

    def _group_barrier(self) -> None:
        """torch.cuda.synchronize(); group barrier; synchronize (elastic.py:365-367)."""
        if self.use_cuda:
            torch.cuda.synchronize()
        if isinstance(self.group, dist.ProcessGroup):
            dist.barrier(group=self.group)
        else:
            self.group.barrier()
        if self.use_cuda:
            torch.cuda.synchronize()

    def _window_bytes(self, hidden: int, num_topk: int, num_max_tokens: int) -> int:
        """Bytes the xGMI window needs for calls of the declared shape (this build's line-aligned
        packed rows: handle.packed_row_layout, kernels.RowLayout), so a first dispatch or combine of
        that shape never re-allocates it (a collective with a host sync); 0 when the shape is not
        declared (num_bytes then sizes the window)."""
        if hidden <= 0 or num_max_tokens <= 0:
            return 0
        from .handle import packed_row_layout
        K = num_topk or 32
        R = self.num_ranks
        slots, single = (min(R, K), False) if self.allow_multiple_reduction else (K, True)
        combine = slots * num_max_tokens * packed_row_layout(hidden, K, True, single)[0]
        dispatch = R * num_max_tokens * max(RowLayout.make(hidden * 2, 0, K).row_bytes,
                                            RowLayout.make(hidden, ceil_div(hidden, 128) * 4, K).row_bytes)
        return max(combine, dispatch)

    # ------------------------------------------------------------------ infrastructure
    @property
    def kernels(self):
        if self._kernels is None:
            from .kernels import HipKernels
            self._kernels = HipKernels()
        return self._kernels

    def destroy(self) -> None:
        assert self.explicitly_destroy
        if self.runtime is not None:
            if self.use_cuda:
                torch.cuda.synchronize()
            if self._sym is not None:
                self._group_barrier()             # no peer still stores into this rank's window
                self._sym.destroy()
                self._sym = None
            # the CU-budget streams are process-wide and never destroyed: tensors returned by an async
            # combine may still record events on them after this buffer is gone
            self.runtime = None

    @staticmethod
    def get_buffer_size_hint(group: dist.ProcessGroup, num_max_tokens_per_rank: int, hidden: int,
                             num_topk: int = 0, use_fp8_dispatch: bool = False,
                             allow_hybrid_mode: bool = True, allow_multiple_reduction: bool = True) -> int:
        return calculate_buffer_size(group.size(), num_max_tokens_per_rank, hidden, num_topk,
                                     use_fp8_dispatch, allow_multiple_reduction)

    @staticmethod
    def get_elastic_buffer_alignment() -> int:
        return BUFFER_ALIGNMENT

    def barrier(self, use_comm_stream: bool = True, with_cpu_sync: bool = False, sequential: bool = True) -> None:
        """A GPU-level barrier across all ranks (elastic.py:497-508, buffer.hpp:181-208), ordered on the comm
        stream -- which first waits for the current stream, and which the current stream then waits for -- or
        on the current stream.  The host blocks only with `with_cpu_sync` (a device synchronize before and
        after).  The device barrier is the xGMI windows' (deepep_sym_barrier: device-counted epochs, the
        window's timeout and error record) once this buffer has a window, else a one-element RCCL all-reduce
        on that stream; a host-side group (gloo) gets a host barrier.  `sequential` (scale-out vs scale-up
        order) has no meaning on one node's single fabric."""
        self._note_capture()
        if with_cpu_sync and self.use_cuda:
            torch.cuda.synchronize()
        rccl = isinstance(self.group, dist.ProcessGroup) and dist.get_backend(self.group) == 'nccl'
        if self.use_cuda and (self._sym is not None or rccl):
            compute = torch.cuda.current_stream()
            stream = self.comm_stream if use_comm_stream else compute
            if stream != compute:
                stream.wait_stream(compute)
            if self._sym is not None:
                if not self._capturing:
                    self._sym.poll()                  # an earlier barrier timed out: raise now
                self._sym.barrier(stream)
                if not self._capturing:
                    self._sym.publish(stream)
            else:
                with torch.cuda.stream(stream):
                    dist.all_reduce(torch.zeros(1, dtype=torch.int32, device=self.device), group=self.group)
            if stream != compute:
                compute.wait_stream(stream)
        elif isinstance(self.group, dist.ProcessGroup):
            dist.barrier(group=self.group)
        else:
            self.group.barrier()
        if with_cpu_sync and self.use_cuda:
            torch.cuda.synchronize()

    @staticmethod
    def capture() -> EventHandle:
        return EventHandle()

    def get_comm_stream(self) -> torch.cuda.Stream:
        return self.comm_stream

    def get_physical_domain_size(self) -> Tuple[int, int]:
        return self.num_rdma_ranks, self.num_nvlink_ranks

    def get_logical_domain_size(self) -> Tuple[int, int]:
        return self.num_scaleout_ranks, self.num_scaleup_ranks

    def get_theoretical_num_sms(self, num_experts: int, num_topk: int, num_scaleout_topk: int = 0,
                                rdma_gbs: float = 0, nvlink_gbs: float = 0,
                                sm_read_gbs: float = 200, sm_write_gbs: float = 50) -> int:
        """Bandwidth model of elastic.py:728-834 for one node, with xGMI in place of NVLink.

        On MI355X the combine kernels size their own grids from the CU count and occupancy;
        the value is kept in the handle for API compatibility (and is what `num_sms` means
        to callers that pass it through)."""
        assert num_scaleout_topk == 0
        key = (num_experts, num_topk, rdma_gbs, nvlink_gbs, sm_read_gbs, sm_write_gbs, self.prefer_overlap_with_compute,
               os.environ.get('EP_XGMI_GBS'))
        memo = self.__dict__.setdefault('_num_sms_memo', {})       # every dispatch asks (host time)
        if key in memo:
            return memo[key]
        nvlink_gbs = nvlink_gbs or float(os.environ.get('EP_XGMI_GBS', 7 * 64))
        num_device_sms = torch.cuda.get_device_properties(self.device).multi_processor_count if self.use_cuda else 256

        def expected_topk(groups: int) -> float:
            return groups * (1 - math.comb(num_experts - num_experts // groups, num_topk) / math.comb(num_experts, num_topk))

        num_sms = num_device_sms
        if self.num_ranks > 1:
            e_topk = expected_topk(self.num_ranks)
            sm_read = 1 / e_topk
            sm_write = self.num_nvlink_ranks / self.num_ranks
            traffic = self.num_nvlink_ranks / self.num_ranks * (1 - 1 / self.num_nvlink_ranks)
            num_sms = max(nvlink_gbs / traffic * sm_read / sm_read_gbs, nvlink_gbs / traffic * sm_write / sm_write_gbs)
        num_sms = align(max(4, math.ceil(num_sms * 1.25)), 2)
        num_sms = num_sms if self.prefer_overlap_with_compute else max(num_sms, 64)
        memo[key] = min(num_sms, num_device_sms)
        return memo[key]

    def get_theoretical_num_qps(self, num_sms: int) -> int:
        num_qps = min(num_sms, 8 + 1)
        if self.allow_hybrid_mode:
            num_qps = num_sms * 16 + 1
        return min(num_qps, self.num_allocated_qps)

    # ------------------------------------------------------------------ streams (buffer.hpp:526-584)
    def _sync_mode(self, previous_event, previous_event_before_epilogue, async_with_compute_stream,
                   allocate_on_comm_stream) -> bool:
        """A call that neither overlaps with compute nor waits on events: its kernels run directly on
        the caller's stream.  The reference runs them on its comm stream and then makes the compute
        stream wait (buffer.hpp:526-584); the observable ordering is the same, minus two cross-stream
        hops (~25 us per call measured on MI355X)."""
        return (not async_with_compute_stream and previous_event is None and
                previous_event_before_epilogue is None and not allocate_on_comm_stream)

    def _note_capture(self) -> None:
        """Whether this call is being captured into a HIP graph (read on the caller's stream,
        before any stream switch): the host-side error-flag polling of the xGMI windows is skipped
        then (graph replays still count their barrier epochs on the device)."""
        self._capturing = self.use_cuda and torch.cuda.is_current_stream_capturing()

    def _prologue(self, previous_event: Optional[EventHandle], allocate_on_comm_stream: bool):
        if not self.use_cuda:
            return None
        compute_stream = torch.cuda.current_stream()
        if allocate_on_comm_stream:
            torch.cuda.set_stream(self.comm_stream)
        if previous_event is not None:
            _assert(allocate_on_comm_stream, 'previous_event requires allocate_on_comm_stream')
            previous_event.stream_wait(self.comm_stream)
        else:
            self.comm_stream.wait_stream(compute_stream)
        return compute_stream

    def _before_epilogue(self, previous_event_before_epilogue: Optional[EventHandle]) -> None:
        if previous_event_before_epilogue is not None and self.use_cuda:
            previous_event_before_epilogue.stream_wait(self.comm_stream)

    def _epilogue(self, tensors: Sequence[Optional[torch.Tensor]], compute_stream,
                  allocate_on_comm_stream: bool, async_with_compute_stream: bool) -> Optional[EventHandle]:
        if not self.use_cuda:
            return None
        event = None
        if async_with_compute_stream:
            event = EventHandle(self.comm_stream)
            if int(os.environ.get('EP_AVOID_RECORD_STREAM', 0)):
                event.tensors_to_record = list(tensors)
            else:
                for t in tensors:
                    if t is not None and t.is_cuda:
                        t.record_stream(compute_stream)
                        t.record_stream(self.comm_stream)
        else:
            compute_stream.wait_stream(self.comm_stream)
        if allocate_on_comm_stream:
            torch.cuda.set_stream(compute_stream)
        return event

    def _mark(self, stream) -> None:
        """Record a timing event on the kernel stream when phase instrumentation is on."""
        if self._phase_events is not None and self.use_cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream)
            self._phase_events.append(ev)

    @staticmethod
    def _null_ctx():
        import contextlib
        return contextlib.nullcontext()

    def _stream_ctx(self):
        if self.use_cuda:
            return torch.cuda.stream(self.comm_stream)
        import contextlib
        return contextlib.nullcontext()

    def _a2a(self, out: torch.Tensor, inp: torch.Tensor, out_splits: Optional[List[int]] = None,
             in_splits: Optional[List[int]] = None) -> None:
        """all_to_all_single over the buffer's group (RCCL over xGMI on GPU, gloo on CPU).
        A one-rank group is a plain copy.  Tests on a single device replace this method."""
        if self.num_ranks == 1:
            out.copy_(inp)
            return
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def _all_to_all(self, out: torch.Tensor, inp: torch.Tensor, out_splits: List[int], in_splits: List[int]) -> None:
        """Row all-to-all of byte views: one message per peer, any row dtype."""
        o = out.view(torch.uint8).view(out.shape[0], out.shape[1] * out.element_size())
        i = inp.view(torch.uint8).view(inp.shape[0], inp.shape[1] * inp.element_size())
        self._a2a(o, i, out_splits, in_splits)

    # ------------------------------------------------------------------ dispatch (handle producer)
    def dispatch(self,
                 x: Union[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]],
                 topk_idx: Optional[torch.Tensor] = None,
                 topk_weights: Optional[torch.Tensor] = None,
                 cumulative_local_expert_recv_stats: Optional[torch.Tensor] = None,
                 num_experts: Optional[int] = None,
                 num_max_tokens_per_rank: Optional[int] = None,
                 expert_alignment: Optional[int] = None,
                 num_sms: int = 0, num_qps: int = 0,
                 previous_event: Optional[EventHandle] = None,
                 previous_event_before_epilogue: Optional[EventHandle] = None,
                 async_with_compute_stream: bool = False,
                 allocate_on_comm_stream: bool = False,
                 handle: Optional[EPHandle] = None,
                 do_handle_copy: bool = True,
                 do_cpu_sync: Optional[bool] = None,
                 do_expand: bool = False,
                 do_zero_padding: bool = False,
                 use_tma_aligned_col_major_sf: bool = False):
        """Dispatch tokens to the ranks owning their experts (elastic.py:855-1033 contract).

        A fresh handle costs one host sync (the notify counts, as the reference's do_cpu_sync=True).
        With do_cpu_sync=False the outputs are padded to the worst case as the reference's
        (buffer.hpp:1065-1070) and the call issues kernels only, at every EP size (launches sized for
        the worst case, bounded on the device by the received count; RCCL: a worst-case-padded
        all-to-all, xGMI: the notify through the windows; graph-capturable).  A cached handle
        (`handle=...`) needs no sync.
        The notify also carries per-64-token-block counts, so the handle's combines never sync."""
        check_torch_deterministic()
        args = (x, topk_idx, topk_weights, cumulative_local_expert_recv_stats, num_experts, num_max_tokens_per_rank,
                expert_alignment, num_sms, num_qps, previous_event, previous_event_before_epilogue,
                async_with_compute_stream, allocate_on_comm_stream, handle, do_handle_copy, do_cpu_sync, do_expand,
                do_zero_padding, use_tma_aligned_col_major_sf)
        # An explicit num_sms below the CU count: the dispatch's kernels run on a stream restricted to that many
        # CUs (the reference sizes its dispatch grids with num_sms), the rest stay free for compute -- as the
        # combine (combine() below); that stream plays the comm stream, so the call takes the async-capable path.
        budget = self._cu_budget_stream(num_sms)
        if budget is not None and self.use_cuda and torch.cuda.current_stream() == budget:
            budget = None
        if budget is None:
            return self._dispatch(*args)
        capturing = torch.cuda.is_current_stream_capturing()
        saved, self.comm_stream = self.comm_stream, budget
        if not capturing:
            budget.wait_stream(saved)
        try:
            return self._dispatch(*args, force_comm_stream=True)
        finally:
            self.comm_stream = saved
            if not capturing:
                saved.wait_stream(budget)

    def _dispatch(self, x, topk_idx, topk_weights, cumulative_local_expert_recv_stats, num_experts,
                  num_max_tokens_per_rank, expert_alignment, num_sms, num_qps, previous_event,
                  previous_event_before_epilogue, async_with_compute_stream, allocate_on_comm_stream, handle,
                  do_handle_copy, do_cpu_sync, do_expand, do_zero_padding, use_tma_aligned_col_major_sf,
                  force_comm_stream: bool = False):
        num_topk = (handle.topk_idx if topk_idx is None else topk_idx).shape[1]
        num_sms = self.get_theoretical_num_sms(num_experts or handle.num_experts, num_topk) if num_sms == 0 else num_sms
        num_qps = self.get_theoretical_num_qps(num_sms) if num_qps == 0 else num_qps
        _assert(num_qps <= self.num_allocated_qps, 'Allocated QPs are not enough')
        x, sf = x if isinstance(x, tuple) else (x, None)
        if handle is not None:
            _assert(topk_idx is None, 'topk_idx must be None with a cached handle')
            _assert(do_cpu_sync is None or not do_cpu_sync, 'Cannot do CPU sync with cached handle')
            topk_idx = handle.topk_idx
            num_max_tokens_per_rank = value_or(num_max_tokens_per_rank, handle.num_max_tokens_per_rank)
            num_experts = value_or(num_experts, handle.num_experts)
            expert_alignment = value_or(expert_alignment, handle.expert_alignment)
            do_cpu_sync = False
            _assert((num_experts, expert_alignment, num_max_tokens_per_rank) ==
                    (handle.num_experts, handle.expert_alignment, handle.num_max_tokens_per_rank),
                    'cached handle context mismatch')
            do_expand = handle.do_expand if do_expand is None else do_expand
        num_max_tokens_per_rank = value_or(num_max_tokens_per_rank, self.num_max_tokens_per_rank)
        expert_alignment = value_or(expert_alignment, 1)
        do_cpu_sync = value_or(do_cpu_sync, True)

        T, H = x.shape
        R, r = self.num_ranks, self.rank_idx
        _assert(num_experts is not None and num_experts % R == 0, 'num_experts must be divisible by the rank count')
        _assert(topk_idx.dim() == 2 and topk_idx.shape[0] == T and topk_idx.dtype == topk_idx_t,
                'topk_idx must be [num_tokens, num_topk] of deep_ep.topk_idx_t')
        _assert(T <= num_max_tokens_per_rank, 'num_tokens exceeds num_max_tokens_per_rank')
        _assert(not do_zero_padding or do_expand, 'do_zero_padding requires do_expand')
        if topk_weights is not None:
            _assert(topk_weights.shape == topk_idx.shape and topk_weights.dtype == torch.float32,
                    'topk_weights must be float32 [num_tokens, num_topk]')
        K = num_topk
        epr = num_experts // R
        self._note_capture()
        # a call that neither overlaps nor waits on events runs on the caller's stream (as the combine:
        # the same ordering without the two cross-stream hops)
        sync_mode = self._sync_mode(previous_event, previous_event_before_epilogue, async_with_compute_stream,
                                    allocate_on_comm_stream) and not force_comm_stream
        compute_stream = None if sync_mode else self._prologue(previous_event, allocate_on_comm_stream)
        kern = self.kernels
        with (self._null_ctx() if sync_mode else self._stream_ctx()):
            dev = x.device
            stream = torch.cuda.current_stream() if self.use_cuda else None
            if sync_mode and self.use_cuda and R > 1 and self.transport == 'xgmi' and not self._capturing:
                # the window is shared by every call: order this call after the earlier calls' work on
                # the comm / phase-B / CU-budget streams that still reads it
                for other in [self.comm_stream, getattr(self, '_stream_b', None)] + \
                        [v[1] for k, v in _BUDGET_STREAMS.items() if k[0] == self.device.index]:
                    if other is not None and other != stream:
                        stream.wait_stream(other)
            idx64 = topk_idx if topk_idx.dtype == torch.int64 else topk_idx.to(torch.int64)
            idx64 = idx64.contiguous()
            w = topk_weights.contiguous() if topk_weights is not None else None
            # A cached handle already holds the routing (slots, counts, metadata, expert layout): the
            # dispatch is then pack -> exchange -> copy, with no host sync (graph-capturable at EP = 1
            # and, over xGMI, at EP > 1),
            # as the reference's cached mode skips its notify phase (elastic.py:855-1033).
            # A handle from a dispatch without a CPU sync knows no counts on the host: its cached
            # dispatches reuse its worst-case-sized tables (and, over RCCL, the padded exchange).
            cached = handle if handle is not None and (handle._send_counts is not None or
                                                       getattr(handle, '_sync_free', False)) else None
            if handle is not None:
                _assert(do_expand == handle.do_expand, 'do_expand must match the cached handle')
            worst_handle = cached is not None and getattr(cached, '_sync_free', False)
            # dispatch(do_cpu_sync=False) issues kernels only, at every EP size (the reference's no-sync
            # mode, buffer.hpp:1065-1070): every receive-side launch is sized for the worst case
            # (R * T_max rows) and bounded on the device by the received count; over RCCL the rows travel in
            # a worst-case-padded all-to-all (equal splits, no host sizes), over xGMI the notify and the rows
            # go through the symmetric windows.
            sync_free = cached is None and not do_cpu_sync
            # EP > 1 over xGMI: the pack kernel stores every row straight into its destination's
            # symmetric window (dispatch.cuh:373-392's push), no RCCL exchange for the rows
            use_xgmi = R > 1 and self.transport == 'xgmi' and self.use_cuda
            peer_offsets = None
            host_notify = None                # one rank, host-synced: the counts' D2H, read after the copy launch
            counts = cached._counts if cached is not None else None
            x_bytes = x.contiguous().view(torch.uint8).view(T, H * x.element_size())
            sf_bytes = sf.contiguous().view(torch.uint8).view(T, sf.shape[1] * sf.element_size()) if sf is not None else None
            # One rank: nothing is exchanged, so the packed rows carry only the routing metadata and
            # the copy reads x (and the scale factors) once, straight from the caller's tensors.
            direct = R == 1
            layout = (RowLayout.make(0, 0, K) if direct else
                      RowLayout.make(x_bytes.shape[1], sf_bytes.shape[1] if sf is not None else 0, K))
            sym = self._window(layout.row_bytes, slots=R, rows_per_slot=num_max_tokens_per_rank) if use_xgmi else None
            if cached is not None:
                dst_slot = cached.dst_buffer_slot_idx
                send_counts_l, recv_counts_l = cached._send_counts, cached._recv_counts
                send_offsets = cached._send_offsets
                peer_offsets = getattr(cached, '_peer_offsets', None)
                if use_xgmi and peer_offsets is not None:
                    sym.barrier(stream)                           # peers finished reading their windows
                use_xgmi = use_xgmi and peer_offsets is not None      # a handle made by the RCCL path
                # a sync-free handle's receive rows are laid out by its transport (padded per source over
                # RCCL, packed by the window notify over xGMI): it is reused on that transport only
                _assert(not (worst_handle and R > 1) or use_xgmi == (peer_offsets is not None) and
                        (use_xgmi or cached._row_map is not None),
                        'a handle from dispatch(do_cpu_sync=False) is cached only on the transport that made it')
            else:
                # --- send side: destination slots (deterministic ranks), one packed row per (token, dest),
                # and the notify (dispatch.cuh:79-258): every destination d gets [tokens | tokens per local
                # expert | per-64-token-block tokens | per-block (token, lane) pairs] from this rank -- the
                # block counts size every pipeline chunk of the EP > 1 combine (handle.BlockCounts), so its
                # plan never needs a host sync of its own.  One exchange sizes every receive-side
                # allocation (and, unless sync-free, ONE host sync brings the counts to the host).
                nb = chunk_geometry(num_max_tokens_per_rank, 1)[0] if R > 1 else 0
                w_n = 1 + epr + 2 * nb
                dst_slot = torch.empty((T, R), dtype=torch.int32, device=dev)
                send_offsets = torch.empty((R,), dtype=torch.int32, device=dev)
                notify = torch.empty((R, w_n), dtype=torch.int32, device=dev)
                kern.dispatch_notify(idx64, num_experts, R, nb, dst_slot, notify, send_offsets, stream=stream)
                if R == 1:
                    recv_notify = notify
                elif use_xgmi:
                    # Through the windows: rank r puts [tokens it sends to every rank | its record for d] into
                    # slot r of rank d's notify area; after the barrier rank r holds every source's record for
                    # it and the token matrix its rows' offsets in the peers' windows come from -- the
                    # reference's notify over NVLink, with no host collective (graph-capturable).
                    rec_w = align(R + w_n, 4)
                    rec = torch.zeros((R, rec_w), dtype=torch.int32, device=dev)
                    rec[:, :R] = notify[:, 0].view(1, R)
                    rec[:, R:R + w_n] = notify
                    sym.barrier(stream)                           # peers finished reading their windows
                    sym.put_notify(rec, stream)
                    sym.barrier(stream)                           # every rank's record landed
                    area = sym.notify_area(rec_w)                 # [source, record]
                    recv_notify = area[:, R:R + w_n].clone()
                    # my rows' first row in every destination's window: what the lower source ranks send there
                    peer_offsets = (area[:r, :R].sum(dim=0, dtype=torch.int32) if r > 0 else
                                    torch.zeros((R,), dtype=torch.int32, device=dev))
                else:
                    recv_notify = torch.empty_like(notify)
                    self._a2a(recv_notify, notify)
                if sync_free:
                    # no CPU sync: the sizes stay on the device; launches are sized for the worst case (one
                    # rank: T rows sent, T_max received -- the worst-case rows every launch and table of
                    # this call is sized for, which a cached dispatch over this handle reuses)
                    send_counts_l, recv_counts_l = ([T], [num_max_tokens_per_rank]) if R == 1 else (None, None)
                    expert_counts_l = own_tok = own_pairs = recv_blk = None
                elif R == 1 and self.use_cuda:
                    # one rank: the counts only size the outputs, so they travel to pinned host memory
                    # while the receive-side kernels (sized for all T tokens, as sync-free) run; the host
                    # waits for them just before it allocates the outputs
                    host_notify = self._host_copy(notify.view(-1), stream)
                    send_counts_l = recv_counts_l = [T]
                else:
                    flat = notify.view(-1) if R == 1 else torch.cat([notify.view(-1), recv_notify.reshape(-1)])
                    host = [int(v) for v in flat.tolist()]                # host sync
                    own, rec_host = host[:R * w_n], (host if R == 1 else host[R * w_n:])
                    send_counts_l = own[0::w_n]
                    own_tok = [own[d * w_n + 1 + epr:d * w_n + 1 + epr + nb] for d in range(R)]
                    own_pairs = [own[d * w_n + 1 + epr + nb:(d + 1) * w_n] for d in range(R)]
                    _, recv_counts_l, expert_counts_l, _, recv_blk = notify_layout(
                        rec_host, R, r, epr, all_gathered=False, num_blocks=nb)
                counts = None
                if R > 1:
                    own_b = notify[:, 1 + epr:].reshape(R, 2, nb).transpose(0, 1)
                    rb = recv_notify[:, 1 + epr:].reshape(R, 2, nb).transpose(0, 1)
                    dev_counts = torch.cat([own_b, rb]).contiguous()
                    if sync_free:
                        counts = BlockCounts(nb, None, None, None, None, dev_counts)
                    else:
                        counts = BlockCounts(nb, own_tok, own_pairs, [b[:nb] for b in recv_blk],
                                             [b[nb:] for b in recv_blk], dev_counts)
                recv_counts_t = recv_notify[:, 0]                 # rows per source (a strided view)
            # received rows: known on the host, or the worst case (R * T_max) without a CPU sync (one
            # rank, counts still on their way to the host: all T tokens)
            N = num_max_tokens_per_rank * R if sync_free or worst_handle else sum(recv_counts_l)
            # worst-case-padded RCCL exchange (a sync-free call, or a cached call over its handle)
            padded = (sync_free or worst_handle) and R > 1 and not use_xgmi
            pad_rows = num_max_tokens_per_rank if padded else 0
            row_map = None
            own_first = False
            if use_xgmi:
                kern.dispatch_pack(x_bytes, sf_bytes, idx64, w, r * num_max_tokens_per_rank, dst_slot,
                                   peer_offsets, None, layout, dest_bases=sym.data_bases_dev,
                                   dest_rows=sym.data_bytes // layout.row_bytes, error_flag=sym.error_flag,
                                   stream=stream)
                sym.barrier(stream)                               # every row landed
                if not self._capturing:
                    sym.publish(stream)
                recv_packed = sym.data[:N * layout.row_bytes].view(N, layout.row_bytes)
            elif padded:
                # worst-case-padded all-to-all: T_max rows per destination (rank d's rows at d * T_max); with the
                # local bypass this rank's own T_max rows are packed behind the others' and stay out of the
                # collective: [send rows | own rows | received rows], slots in send / receive order (no host
                # sync: the splits are T_max)
                T_max = num_max_tokens_per_rank
                own_first = cached._bypass if cached is not None else self.local_bypass
                ar = torch.arange(R, dtype=torch.int32, device=dev)
                if own_first:
                    pad_offsets = torch.where(ar == r, R - 1, torch.where(ar > r, ar - 1, ar)) * T_max
                    rows_all = torch.empty(((2 * R - 1) * T_max, layout.row_bytes), dtype=torch.uint8, device=dev)
                    kern.dispatch_pack(x_bytes, sf_bytes, idx64, w, r * T_max, dst_slot, pad_offsets, rows_all, layout,
                                       stream=stream)
                    splits = [0 if d == r else T_max for d in range(R)]
                    self._a2a(rows_all[R * T_max:], rows_all[:(R - 1) * T_max], splits, splits)
                    recv_packed = rows_all[(R - 1) * T_max:]
                else:
                    packed = torch.empty((R * T_max, layout.row_bytes), dtype=torch.uint8, device=dev)
                    kern.dispatch_pack(x_bytes, sf_bytes, idx64, w, r * T_max, dst_slot, ar * T_max, packed, layout,
                                       stream=stream)
                    recv_packed = torch.empty_like(packed)
                    self._a2a(recv_packed, packed)
                row_map = torch.empty((N,), dtype=torch.int32, device=dev)
            elif R > 1 and (cached._bypass if cached is not None else self.local_bypass):
                # Local bypass (the combine's, exchange.py): one allocation [send rows | own rows | received
                # rows]; the pack writes the other destinations' rows in rank order and this rank's own rows
                # right behind them, the all-to-all moves the send rows with a zero split for this rank, and
                # the receive side reads [own rows | received rows] through a row map (own_first) -- the own
                # rows are never copied by the collective.
                own = send_counts_l[r]
                n_send = sum(send_counts_l)
                if cached is None:
                    off, acc = [0] * R, 0
                    for d in [d for d in range(R) if d != r] + [r]:
                        off[d], acc = acc, acc + send_counts_l[d]
                    send_offsets = torch.tensor(off, dtype=torch.int32, device=dev)
                    row_map = torch.empty((N,), dtype=torch.int32, device=dev)
                rows_all = torch.empty((n_send + N - own, layout.row_bytes), dtype=torch.uint8, device=dev)
                kern.dispatch_pack(x_bytes, sf_bytes, idx64, w, r * num_max_tokens_per_rank, dst_slot, send_offsets,
                                   rows_all, layout, stream=stream)
                self._a2a(rows_all[n_send:], rows_all[:n_send - own],
                          [0 if d == r else c for d, c in enumerate(recv_counts_l)],
                          [0 if d == r else c for d, c in enumerate(send_counts_l)])
                recv_packed = rows_all[n_send - own:]
                own_first = True
            else:
                n_send = T if sync_free else sum(send_counts_l)
                packed = torch.empty((n_send, layout.row_bytes), dtype=torch.uint8, device=dev)
                kern.dispatch_pack(x_bytes[:, :0] if direct else x_bytes, None if direct else sf_bytes, idx64, w,
                                   r * num_max_tokens_per_rank, dst_slot, send_offsets, packed, layout, stream=stream)
                if R == 1:
                    recv_packed = packed
                else:
                    recv_packed = torch.empty((N, layout.row_bytes), dtype=torch.uint8, device=dev)
                    self._a2a(recv_packed, packed, recv_counts_l, send_counts_l)
            # --- receive side (dispatch_copy_epilogue_impl): metadata, expert layout, copies
            inv = block_offsets = None                      # the expanded copy's tables (dispatch_copy)
            if cached is not None:
                psum_rank = cached.psum_num_recv_tokens_per_scaleup_rank
                psum_expert = cached.psum_num_recv_tokens_per_expert
                meta = cached.recv_src_metadata[:N]
                inv, block_offsets = getattr(cached, '_copy_tables', (None, None))
                copy_meta, copy_rows = getattr(cached, '_copy_meta', None) or (meta, N)
                row_map = getattr(cached, '_row_map', None)
                out_idx = None if do_expand else cached._recv_topk_idx[:N].clone()
                aligned_l = cached.num_recv_tokens_per_expert_list
                expert_counts = cached.num_unaligned_recv_tokens_per_expert
                if cumulative_local_expert_recv_stats is not None:
                    cumulative_local_expert_recv_stats += expert_counts.to(cumulative_local_expert_recv_stats.dtype)
                self._before_epilogue(previous_event_before_epilogue)
            else:
                psum_rank = torch.empty((R,), dtype=torch.int32, device=dev)
                meta = torch.empty((N, K + 2), dtype=torch.int32, device=dev)
                out_idx = None if do_expand else torch.empty((N, K), dtype=torch.int64, device=dev)
                nblocks = (N + DISPATCH_BLOCK_ROWS - 1) // DISPATCH_BLOCK_ROWS
                block_counts = torch.empty((nblocks, epr), dtype=torch.int32, device=dev)
                expert_counts = torch.empty((epr,), dtype=torch.int32, device=dev)
                psum_expert = torch.empty((epr,), dtype=torch.int32, device=dev)
                # worst-case expanded rows (the count is known after the notify): the inverse map of the
                # slots for the blocked destination-major copy
                inv = torch.empty((N * min(K, epr) + (expert_alignment - 1) * epr,), dtype=torch.int32,
                                  device=dev) if do_expand else None
                block_offsets = block_counts if do_expand else None
                # count -> scan -> slots (expanded; else metadata slot columns -1), back to back
                kern.dispatch_receive(recv_packed, layout, N, r, epr, recv_counts_t, psum_rank, meta, out_idx,
                                      block_counts, expert_alignment, do_expand, expert_counts, psum_expert, inv=inv,
                                      pad_rows=pad_rows, row_map=row_map, own_first=own_first, stream=stream)
                # known since the notify; [] without a CPU sync (as the reference's handle)
                aligned_l = [] if sync_free or host_notify is not None else \
                    [align(c, expert_alignment) for c in expert_counts_l]
                if cumulative_local_expert_recv_stats is not None:
                    cumulative_local_expert_recv_stats += expert_counts.to(cumulative_local_expert_recv_stats.dtype)
                self._before_epilogue(previous_event_before_epilogue)
                copy_meta, copy_rows = meta, N
            num_unaligned = expert_counts
            # one rank, host-synced (host_notify): every launch, the copy included, is sized as without a
            # CPU sync (all T tokens) while the counts travel to the host; the outputs are then the exact
            # leading rows of those allocations
            deferred = host_notify is not None
            worst_tokens = num_max_tokens_per_rank * R if sync_free else T
            if do_expand and cached is not None:
                num_expanded = cached.num_expanded_tokens
                alloc = torch.zeros if do_zero_padding else torch.empty
                n_rows = num_expanded
            elif do_expand and (sync_free or deferred):
                # worst case of buffer.hpp:1067-1069: every token in min(K, local experts) experts
                num_expanded = align(worst_tokens * min(K, epr) + (expert_alignment - 1) * epr, expert_alignment)
                alloc = torch.zeros if do_zero_padding else torch.empty
                n_rows = num_expanded
            elif do_expand:
                num_expanded = sum(aligned_l)
                alloc = torch.zeros if do_zero_padding else torch.empty
                n_rows = num_expanded
            else:
                num_expanded = N
                # without a CPU sync the rows past the received ones are zeros (never written by the copy)
                alloc = torch.zeros if sync_free or worst_handle else torch.empty
                n_rows = N
            out_x = alloc((n_rows, H), dtype=x.dtype, device=dev)
            out_sf = alloc((n_rows, sf.shape[1]), dtype=sf.dtype, device=dev) if sf is not None else None
            out_w = None
            if topk_weights is not None:
                # expanded: the copy writes the weight of every expanded row; rows it never writes (expert
                # alignment padding, the worst-case tail of a sync-free call) hold 0
                exact = expert_alignment == 1 and (bool(cached.num_recv_tokens_per_expert_list)
                                                   if cached is not None else not sync_free)
                out_w = ((torch.empty if exact else torch.zeros)((n_rows,), dtype=torch.float32, device=dev)
                         if do_expand else alloc((N, K), dtype=torch.float32, device=dev))
            kern.dispatch_copy(recv_packed, layout, copy_rows if do_expand else N, copy_meta if do_expand else meta,
                               do_expand,
                               out_x.view(torch.uint8), out_sf.view(torch.uint8) if out_sf is not None else None,
                               out_w, x_direct=x_bytes if direct else None,
                               sf_direct=sf_bytes if direct else None, num_max_tokens=num_max_tokens_per_rank,
                               error_flag=sym.error_flag if use_xgmi else None,
                               inv=inv if do_expand else None, block_offsets=block_offsets if do_expand else None,
                               expert_end=psum_expert if do_expand else None, row_map=row_map, stream=stream)
            if deferred:
                # the counts reached the host while the kernels ran: the handle and the outputs take the
                # received rows / the exact expanded rows (leading views of the allocations above)
                host = host_notify.wait()
                send_counts_l = recv_counts_l = [host[0]]
                expert_counts_l = host[1:1 + epr]
                aligned_l = [align(c, expert_alignment) for c in expert_counts_l]
                N = host[0]
                n_rows = sum(aligned_l) if do_expand else N
                num_expanded = n_rows if do_expand else N
                meta = meta[:N]
                out_idx = out_idx[:N] if out_idx is not None else None
                out_x = out_x[:n_rows]
                out_sf = out_sf[:n_rows] if out_sf is not None else None
                out_w = out_w[:n_rows] if out_w is not None else None
            if out_sf is not None and use_tma_aligned_col_major_sf:
                # the reference's TMA-aligned column-major scale factors for the next GEMM (buffer.hpp:1090-1096):
                # packs of consecutive rows adjacent, each pack column starting on 16 bytes
                n_sf, packs = out_sf.shape
                col_major = torch.empty_strided((n_sf, packs), (1, align(max(n_sf, 1), max(1, 16 // out_sf.element_size()))),
                                                dtype=out_sf.dtype, device=dev)
                col_major.copy_(out_sf)
                out_sf = col_major
            recv_idx64 = out_idx
            if out_idx is not None and topk_idx.dtype != torch.int64:
                out_idx = out_idx.to(topk_idx.dtype)
            # without a CPU sync N is already the worst case (buffer.hpp:1065-1070): metadata rows past the
            # received ones are -1 (dispatch_count), non-expanded outputs there are zeros / -1
            num_recv = N
            # the handle's own routing copy (do_handle_copy); a cached call keeps its handle, so nothing to copy
            cloned_idx = topk_idx.clone() if do_handle_copy and cached is None else topk_idx
        event = None if sync_mode else self._epilogue([x, sf, topk_idx, topk_weights, out_x, out_sf, out_idx, out_w,
                                                       meta], compute_stream, allocate_on_comm_stream,
                                                      async_with_compute_stream)
        is_cached = handle is not None
        if not is_cached:
            handle = EPHandle(do_expand, num_experts, expert_alignment, num_max_tokens_per_rank, num_sms,
                              cloned_idx, num_recv, num_expanded, aligned_l, psum_rank, psum_expert,
                              num_unaligned, meta, dst_slot, None, None)
            handle._recv_counts = recv_counts_l
            handle._send_counts = send_counts_l
            handle._send_offsets = send_offsets
            handle._peer_offsets = peer_offsets
            handle._recv_topk_idx = recv_idx64
            handle._counts = counts
            handle._copy_tables = (inv, block_offsets)      # reused by cached dispatches
            handle._copy_meta = (copy_meta, copy_rows) if copy_rows != N else None
            handle._row_map = row_map
            handle._bypass = own_first
            handle._sync_free = sync_free
        out_x = (out_x, out_sf) if out_sf is not None else out_x
        return out_x, out_idx, out_w, handle, EventOverlap(event)

    # ------------------------------------------------------------------ combine (the hot path)
    @staticmethod
    def _unpack_bias(bias) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
        bias_0, bias_1 = None, None
        if isinstance(bias, torch.Tensor):
            bias_0 = bias
        elif isinstance(bias, tuple):
            assert len(bias) == 2
            bias_0, bias_1 = bias
        return bias_0, bias_1

    def _num_chunks(self, handle: EPHandle) -> int:
        """Pipeline depth of the EP > 1 combine: DEEPEP_COMBINE_CHUNKS, else 4 for batches of at
        least 1024 tokens per rank (1 on the CPU, or when the bench asks for unpipelined phases)."""
        if self.num_ranks == 1 or (self._phase_events is not None and self._phase_unpipelined):
            return 1
        env = os.environ.get('DEEPEP_COMBINE_CHUNKS')
        if env:
            return max(1, int(env))
        return 4 if self.use_cuda and handle.num_max_tokens_per_rank >= 1024 else 1

    def _plan(self, handle: EPHandle, single_reduction: bool, num_chunks: int, hidden: int,
              window=None) -> CombinePlan:
        """The handle's combine plan for this buffer's configuration, built on the first use by kernels
        on the current stream (no host sync: handle.build_ep_plan) and cached on the handle.  A plan
        built while a HIP graph is being captured belongs to that graph (its kernels run at replay),
        so it is not cached for eager calls."""
        R = self.num_ranks
        if R == 1:
            key = ('single' if single_reduction else 'multi', 1)
        elif window is None:
            key = ('single' if single_reduction else 'multi', R, num_chunks, hidden, self.local_bypass)
        else:
            for k in [k for k in handle._combine_plans if k[0] == 'xgmi' and k[-1] in self._old_sym_gens]:
                del handle._combine_plans[k]          # plans that address an earlier (freed) window
            key = ('xgmi', single_reduction, R, num_chunks, hidden, self._sym_gen)
        plan = handle._combine_plans.get(key)
        stream = torch.cuda.current_stream() if self.use_cuda else None
        if plan is not None:
            plan.poll()                               # a plan entry its kernels rejected: raise
            if self.use_cuda and not self._capturing and plan.ready is not None and plan.ready[0] != stream:
                # built on another stream: order this use after it (once per call, cheap)
                stream.wait_event(plan.ready[1])
            return plan
        T, K = handle.topk_idx.shape
        if R == 1:
            meta = handle.recv_src_metadata
            n_recv = handle.num_recv_tokens if handle._recv_counts is None else sum(handle._recv_counts)
            plan = CombinePlan(num_ranks=1, num_tokens=T, num_topk=K, expanded=handle.do_expand)
            width = K if handle.do_expand else 1
            plan.local_table = torch.empty((T, width), dtype=torch.int32, device=meta.device)
            if not handle.do_expand:
                plan.local_wtable = torch.empty((T, K), dtype=torch.int32, device=meta.device)
            self.kernels.build_local_plan(meta, n_recv, K, handle.num_max_tokens_per_rank, handle.do_expand,
                                          plan.local_table, T, handle.topk_idx, plan.local_wtable, stream=stream)
        else:
            _assert(handle._counts is not None, 'the EP > 1 combine needs a handle made by this build\'s dispatch')
            plan = build_ep_plan(self.kernels, handle, num_ranks=R, rank=self.rank_idx, single=single_reduction,
                                 num_chunks=num_chunks, hidden=hidden, window=window, stream=stream,
                                 local_bypass=self.local_bypass)
        if not self._capturing:
            if self.use_cuda:
                ev = torch.cuda.Event()
                ev.record(stream)
                plan.ready = (stream, ev)
                plan.publish(stream)
            handle._combine_plans[key] = plan
        return plan

    def combine(self,
                x: torch.Tensor,
                handle: EPHandle,
                topk_weights: Optional[torch.Tensor] = None,
                bias: Union[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]] = None,
                num_sms: int = 0, num_qps: int = 0,
                previous_event: Optional[EventHandle] = None,
                previous_event_before_epilogue: Optional[EventHandle] = None,
                async_with_compute_stream: bool = False,
                allocate_on_comm_stream: bool = False,
                *,
                apply_topk_weights: bool = False) \
            -> Tuple[torch.Tensor, Optional[torch.Tensor], EventOverlap]:
        """Combine (reduce) tokens back to their source ranks (elastic.py:1046-1107 contract).

        `apply_topk_weights` (extension, default False = reference semantics): scale every
        expanded row by its top-k weight inside the reduction (the gating-weighted sum of the
        legacy low_latency_combine, csrc/kernels/legacy/internode_ll.cu:1072-1135).  Requires
        the expanded layout and `topk_weights`.  The weights are still passed through."""
        check_torch_deterministic()
        explicit_sms = num_sms
        if num_sms == 0 and self.combine_cu_mode == 'handle' and self.prefer_overlap_with_compute:
            explicit_sms = handle.num_sms          # the reference's SM-confined default (elastic.py:1086)
        num_sms = handle.num_sms if num_sms == 0 else num_sms
        num_qps = self.get_theoretical_num_qps(num_sms) if num_qps == 0 else num_qps
        _assert(num_qps <= self.num_allocated_qps, 'Allocated QPs are not enough')
        bias_0, bias_1 = self._unpack_bias(bias)
        budget = self._cu_budget_stream(explicit_sms)
        if budget is not None and self.use_cuda and torch.cuda.current_stream() == budget:
            budget = None     # the caller already runs on the budget stream: no stream hops needed
        if budget is None:
            return self._combine(x, topk_weights, bias_0, bias_1, handle, num_sms, previous_event,
                                 previous_event_before_epilogue, async_with_compute_stream,
                                 allocate_on_comm_stream, apply_topk_weights)
        # An explicit num_sms below the CU count: the combine's kernels run on a stream restricted to
        # that many CUs (the reference's combine_impl grid, combine.hpp:135), the rest stay free for
        # compute.  That stream plays the comm stream, so the call takes the async-capable path.
        # The budget stream is ordered with the regular comm stream both ways: the symmetric window
        # (xGMI transport) is shared by every call, and an earlier async dispatch / a later call on
        # the comm stream must not overlap this combine's use of it.
        capturing = torch.cuda.is_current_stream_capturing()
        saved, self.comm_stream = self.comm_stream, budget
        if not capturing:
            budget.wait_stream(saved)
        try:
            return self._combine(x, topk_weights, bias_0, bias_1, handle, num_sms, previous_event,
                                 previous_event_before_epilogue, async_with_compute_stream,
                                 allocate_on_comm_stream, apply_topk_weights, force_comm_stream=True)
        finally:
            self.comm_stream = saved
            if not capturing:
                saved.wait_stream(budget)

    def get_cu_budget_stream(self, num_sms: int) -> Optional[torch.cuda.Stream]:
        """The stream restricted to `num_sms` CUs (rounded up to whole CUs per XCD) that an explicit
        `combine(..., num_sms=num_sms)` runs on; None for the whole chip.  A caller that issues the
        combine from this stream (torch.cuda.stream(...)) skips the two cross-stream hops."""
        return self._cu_budget_stream(num_sms)

    def _cu_budget_stream(self, num_sms: int):
        """The CU-budget stream for an explicit num_sms (None when 0 or at least the CU count).
        The handle's default num_sms is the reference's NVLink/SM bandwidth model
        (get_theoretical_num_sms); on MI355X the combine is HBM-bound and takes the whole chip
        unless the caller asks for less."""
        if num_sms <= 0 or not self.use_cuda:
            return None
        if num_sms >= torch.cuda.get_device_properties(self.device).multi_processor_count:
            return None
        key = (self.device.index, (num_sms + 7) // 8 * 8)     # budgets are whole CUs per XCD
        if key not in _BUDGET_STREAMS:
            import ctypes
            from . import _lib
            raw = ctypes.c_void_p()
            _lib.check(self.kernels.lib.deepep_stream_create_cu_budget(key[1], ctypes.byref(raw)), 'cu_budget stream')
            _BUDGET_STREAMS[key] = (raw.value, torch.cuda.ExternalStream(raw.value, device=self.device))
        return _BUDGET_STREAMS[key][1]

    def _combine(self, x, topk_weights, bias_0, bias_1, handle, num_sms, previous_event,
                 previous_event_before_epilogue, async_with_compute_stream, allocate_on_comm_stream,
                 apply_topk_weights, force_comm_stream=False):
        # ---- checks of ElasticBuffer::combine (buffer.hpp:1197-1247)
        _assert(self.runtime is not None, 'buffer destroyed')
        _assert(num_sms > 0, 'num_sms > 0')
        _assert(x.dim() == 2 and x.is_contiguous() and x.dtype == torch.bfloat16, 'x must be contiguous bf16 [N, hidden]')
        num_tokens, hidden = x.shape
        _assert((hidden * x.element_size()) % 16 == 0, 'hidden * sizeof(bf16) must be a multiple of 16')
        topk_idx = handle.topk_idx
        _assert(topk_idx.dim() == 2 and topk_idx.is_contiguous() and topk_idx.dtype == topk_idx_t, 'topk_idx layout')
        T, K = topk_idx.shape
        psum = handle.psum_num_recv_tokens_per_scaleup_rank
        _assert(psum.dim() == 1 and psum.shape[0] == self.num_scaleup_ranks and psum.dtype == torch.int32,
                'psum_num_recv_tokens_per_scaleup_rank must be int32 [num_scaleup_ranks]')
        _assert(T <= handle.num_max_tokens_per_rank, 'num_combined_tokens <= num_max_tokens_per_rank')
        meta = handle.recv_src_metadata
        _assert(meta.dim() == 2 and meta.shape[1] == K + 2 and meta.dtype == torch.int32 and meta.is_contiguous(),
                'recv_src_metadata must be contiguous int32 [num_recv_tokens, num_topk + 2]')
        expanded = handle.do_expand
        if not expanded:
            _assert(meta.shape[0] == num_tokens, 'non-expanded x must have one row per received token')
        if topk_weights is not None:
            if expanded:
                _assert(topk_weights.dim() == 1 and topk_weights.shape[0] == num_tokens, 'expanded weights are [N]')
            else:
                _assert(topk_weights.dim() == 2 and tuple(topk_weights.shape) == (num_tokens, K), 'weights are [N, K]')
            _assert(topk_weights.is_contiguous() and topk_weights.dtype == torch.float32, 'weights must be float32')
        for b in (bias_0, bias_1):
            if b is not None:
                _assert(b.dim() == 2 and b.is_contiguous() and b.dtype == x.dtype and tuple(b.shape) == (T, hidden),
                        'bias must be contiguous bf16 [num_combined_tokens, hidden]')
        single_reduction = expanded and not self.allow_multiple_reduction
        if single_reduction:
            # the reference's expanded send carries no weights (combine.cuh:67-69) -- unless they are
            # the gating weights this build applies (the legacy low-latency semantics)
            _assert(topk_weights is None or apply_topk_weights,
                    'expanded combine without multiple reduction cannot carry top-k weights')
        if apply_topk_weights:
            _assert(expanded and topk_weights is not None,
                    'apply_topk_weights needs the expanded layout and topk_weights')

        kern = self.kernels
        R = self.num_ranks
        self._note_capture()
        sync_mode = self._sync_mode(previous_event, previous_event_before_epilogue, async_with_compute_stream,
                                    allocate_on_comm_stream) and not force_comm_stream
        if sync_mode:
            compute_stream = None
            stream = torch.cuda.current_stream() if self.use_cuda else None
        else:
            compute_stream = self._prologue(previous_event, allocate_on_comm_stream)
            stream = self.comm_stream
        with (self._null_ctx() if sync_mode else self._stream_ctx()):
            use_xgmi = R > 1 and self.transport == 'xgmi' and self.use_cuda
            if use_xgmi and sync_mode and not self._capturing:
                # the window is shared by every call: this call's first barrier must come after the
                # earlier calls' work on the comm / phase-B / CU-budget streams that still reads it
                # (a graph replays in stream order with what the capture depended on)
                for other in [self.comm_stream, getattr(self, '_stream_b', None)] + \
                        [v[1] for k, v in _BUDGET_STREAMS.items() if k[0] == self.device.index]:
                    if other is not None and other != stream:
                        stream.wait_stream(other)
            num_chunks = self._num_chunks(handle)
            plan = None if use_xgmi else self._plan(handle, single_reduction, num_chunks, hidden)
            combined_x = torch.empty((T, hidden), dtype=x.dtype, device=x.device)
            combined_w = torch.empty((T, K), dtype=torch.float32, device=x.device) if topk_weights is not None else None
            row_w = topk_weights if apply_topk_weights else None
            wsrc = topk_weights.view(-1) if topk_weights is not None else None
            if R == 1:
                self._before_epilogue(previous_event_before_epilogue)
                if single_reduction:
                    kern.combine_reduce(MODE_EPILOGUE, x, combined_x, T, table=plan.local_table, row_weights=row_w,
                                        bias0=bias_0, bias1=bias_1, wtable=plan.local_table, wsrc=wsrc,
                                        out_weights=combined_w, stream=stream)
                else:
                    wtable = plan.local_table if expanded else plan.local_wtable
                    kern.combine_reduce(MODE_FUSED, x, combined_x, T, table=plan.local_table, row_weights=row_w,
                                        bias0=bias_0, bias1=bias_1, wtable=wtable, wsrc=wsrc,
                                        out_weights=combined_w, stream=stream)
            elif single_reduction and use_xgmi:
                self._combine_xgmi_single(handle, x, row_w, wsrc, K, hidden, bias_0, bias_1, topk_weights,
                                          combined_x, combined_w, previous_event_before_epilogue, stream)
            elif single_reduction:
                self._combine_single_chunks(plan, x, row_w, wsrc, hidden, bias_0, bias_1, combined_x, combined_w,
                                            previous_event_before_epilogue, stream)
            elif use_xgmi:
                self._combine_xgmi(handle, x, expanded, row_w, wsrc, K, hidden, bias_0, bias_1, topk_weights,
                                   combined_x, combined_w, previous_event_before_epilogue, stream)
            else:
                self._combine_chunks(plan, x, expanded, row_w, wsrc, K, hidden, bias_0, bias_1, topk_weights,
                                     combined_x, combined_w, previous_event_before_epilogue, stream)
        event = None
        if not sync_mode:
            event = self._epilogue([x, topk_weights, bias_0, bias_1, meta, topk_idx, combined_x, combined_w, psum],
                                   compute_stream, allocate_on_comm_stream, async_with_compute_stream)
        return combined_x, combined_w, EventOverlap(event)
