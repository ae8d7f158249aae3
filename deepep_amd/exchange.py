"""The EP > 1 exchanges of ElasticBuffer.combine (a mixin of deepep_amd.buffer.ElasticBuffer).

  RCCL transport   phase A (local reduce) -> all_to_all_single of packed [partial | weights] rows ->
                   phase B (epilogue), pipelined in source-token chunks; and the single reduction
                   (rows unreduced, one reduce at the source rank), pipelined the same way
  xGMI transport   phase A stores straight into the owners' symmetric windows (HIP IPC), device
                   barriers / split barriers, phase B over the local window; multiple and single
                   reduction

The per-token arithmetic is the reference's (combine.cuh, combine_reduce_epilogue.cuh in
/root/reference); the exchange design is DESIGN.md section 5.
"""
import itertools
from typing import List, Optional

import torch
import torch.distributed as dist

from .handle import packed_row_layout
from .kernels import MODE_EPILOGUE, MODE_LOCAL

_WINDOW_IDS = itertools.count(1)            # symmetric windows created by this process


def _require_weight_index(plan) -> None:
    """The weight pass-through reads each lane's weight through int32 float indices into the packed
    receive rows (handle.build_ep_plan leaves wtable_b None when they would overflow int32): raise
    instead of reading the wrong floats (not an assert, so `python -O` keeps the check)."""
    if any(ch.wtable_b is None for ch in plan.chunks):
        raise RuntimeError('Assertion failed: the receive rows are too large for int32 weight indices '
                           '(num_max_tokens_per_rank * hidden too large for the weight pass-through)')


def _splits(plan, ch, me: int):
    """(send, receive) all-to-all splits of a chunk: with the local bypass the diagonal is 0 (this
    rank's own rows never enter the collective)."""
    if not plan.local_bypass:
        return list(ch.send_counts), list(ch.back_counts)
    return ([0 if r == me else n for r, n in enumerate(ch.send_counts)],
            [0 if r == me else n for r, n in enumerate(ch.back_counts)])


class ExchangeMixin:
    """EP > 1 exchange paths; uses the host attributes of ElasticBuffer (group, ranks, streams,
    kernels, _mark, _before_epilogue, _all_to_all)."""

    def _a2a_async(self, out: torch.Tensor, inp: torch.Tensor, out_splits: List[int], in_splits: List[int]):
        """Row all-to-all that returns a waitable (RCCL runs it on its own stream; `wait()` makes the
        current stream wait).  Tests on a single device replace this method."""
        o = out.view(torch.uint8).view(out.shape[0], out.shape[1] * out.element_size())
        i = inp.view(torch.uint8).view(inp.shape[0], inp.shape[1] * inp.element_size())
        return dist.all_to_all_single(o, i, out_splits, in_splits, group=self.group, async_op=True)

    def _combine_chunks(self, plan, x, expanded, row_w, wsrc, K, hidden, bias_0, bias_1, topk_weights,
                        combined_x, combined_w, previous_event_before_epilogue, stream) -> None:
        """EP > 1 combine, chunked: phase A (local reduce per received token) -> all-to-all of
        packed rows [bf16 partial | fp32 top-k weights] -> phase B (epilogue + bias).  With more
        than one chunk, phase A of chunk c+1 runs while RCCL moves chunk c and phase B of chunk
        c runs on a second stream while RCCL moves chunk c+1.

        Local bypass: a chunk's rows live in one allocation [send rows | own rows | received rows].
        Phase A writes the units of the other ranks (the send rows, rank order) and then this rank's
        own units right behind them; the all-to-all moves the send rows with a zero split for this
        rank into the received rows; phase B reads [own rows | received rows] -- the own partials
        where phase A wrote them, with no copy (the reference stores them into its own receive slot,
        combine.cuh:96-101).  The plan lays the tables out for it (DEEPEP_PLAN_LOCAL_BYPASS)."""
        kern = self.kernels
        me = self.rank_idx
        # packed rows [bf16 partial | fp32 weights], whole 128-byte lines (handle.packed_row_layout)
        with_w = topk_weights is not None
        row_bytes, w_off, w_pad = packed_row_layout(hidden, K, with_w)
        row_elems = row_bytes // 2
        pipelined = len(plan.chunks) > 1 and self.use_cuda
        if with_w:
            _require_weight_index(plan)
        if pipelined:
            if getattr(self, '_stream_b', None) is None:
                self._stream_b = torch.cuda.Stream(device=self.device)
            stream_b = self._stream_b
            stream_b.wait_stream(stream)                  # bias / outputs were produced before this call
        # Optional CU budget for phase A (DEEPEP_PHASE_A_CUS, as in _combine_xgmi): the CUs it leaves
        # free go to RCCL's kernels and to phase B of the earlier chunks.  Phase A and the exchange
        # it feeds are then issued from the budget stream (RCCL orders after the current stream).
        sa = self._cu_budget_stream(self.phase_a_cus) if pipelined and self.phase_a_cus else None
        sa = stream if sa is None else sa
        if sa is not stream:
            sa.wait_stream(stream)
        in_flight = []
        for ch in plan.chunks:
            with (torch.cuda.stream(sa) if sa is not stream else self._null_ctx()):
                n_units, n_back, own = sum(ch.send_counts), sum(ch.back_counts), ch.own
                n_send = n_units - own                    # rows that travel
                rows = torch.empty((n_units + n_back - own, row_elems), dtype=x.dtype, device=x.device)
                partial_w = rows.view(torch.float32)[:n_units, w_off // 4:w_off // 4 + K] if with_w else None
                self._mark(sa)
                kern.combine_reduce(MODE_LOCAL, x, rows[:n_units, :hidden], n_units, table=ch.table_a,
                                    row_weights=row_w, wtable=ch.wtable_a, wsrc=wsrc, out_weights=partial_w,
                                    weights_pad=w_pad, stream=sa)
                self._mark(sa)
                send_splits, back_splits = _splits(plan, ch, me)
                send, recv = rows[:n_send], rows[n_units:]
                if pipelined:
                    work = self._a2a_async(recv, send, back_splits, send_splits)
                else:
                    self._all_to_all(recv, send, back_splits, send_splits)
                    work = None
            in_flight.append((ch, rows[n_send:], rows, work))
        if sa is not stream:
            stream.wait_stream(sa)
        self._before_epilogue(previous_event_before_epilogue)
        if pipelined and previous_event_before_epilogue is not None:
            previous_event_before_epilogue.stream_wait(stream_b)
        for ch, src_b, rows, work in in_flight:
            ctx = torch.cuda.stream(stream_b) if pipelined else self._null_ctx()
            with ctx:
                sb = stream_b if pipelined else stream
                if work is not None:
                    work.wait()
                wtable_b = ch.wtable_b if with_w else None
                recv_wsrc = src_b.view(torch.float32).view(-1) if with_w else None
                lo, hi = ch.lo, ch.hi
                self._mark(sb)
                kern.combine_reduce(MODE_EPILOGUE, src_b[:, :hidden], combined_x[lo:hi], hi - lo, table=ch.table_b,
                                    bias0=bias_0[lo:hi] if bias_0 is not None else None,
                                    bias1=bias_1[lo:hi] if bias_1 is not None else None,
                                    wtable=wtable_b, wsrc=recv_wsrc,
                                    out_weights=combined_w[lo:hi] if combined_w is not None else None, stream=sb)
                self._mark(sb)
        if pipelined:
            stream.wait_stream(stream_b)
            for _, _, rows, _ in in_flight:               # used on stream_b / the RCCL stream
                rows.record_stream(stream_b)

    def _combine_single_chunks(self, plan, x, row_w, wsrc, hidden, bias_0, bias_1, combined_x, combined_w,
                               previous_event_before_epilogue, stream) -> None:
        """Single-reduction combine over RCCL, chunked like _combine_chunks (and with its local bypass:
        this rank's own rows are written in place): the pack of chunk c+1 runs while RCCL moves
        chunk c, and the one reduction of chunk c (weighted: the legacy fma chain) runs on a second
        stream while RCCL moves chunk c+1."""
        kern = self.kernels
        me = self.rank_idx
        w_elems = 1 if row_w is not None else 0          # one gating weight per unreduced row
        row_bytes, w_off, w_pad = packed_row_layout(hidden, 1, bool(w_elems), single=True)
        row_elems = row_bytes // 2
        pipelined = self.use_cuda
        if pipelined:
            if getattr(self, '_stream_b', None) is None:
                self._stream_b = torch.cuda.Stream(device=self.device)
            stream_b = self._stream_b
            stream_b.wait_stream(stream)
        in_flight = []
        for ch in plan.chunks:
            n_units, n_back, own = sum(ch.send_counts), sum(ch.back_counts), ch.own
            n_send = n_units - own
            rows = torch.empty((n_units + n_back - own, row_elems), dtype=x.dtype, device=x.device)
            send_w = rows.view(torch.float32)[:n_units, w_off // 4:w_off // 4 + 1] if w_elems else None
            self._mark(stream)
            kern.combine_reduce(MODE_LOCAL, x, rows[:n_units, :hidden], n_units, table=ch.table_a,
                                wtable=ch.table_a if w_elems else None, wsrc=wsrc if w_elems else None,
                                out_weights=send_w, weights_pad=w_pad, stream=stream)
            self._mark(stream)
            send_splits, back_splits = _splits(plan, ch, me)
            send, recv = rows[:n_send], rows[n_units:]
            if pipelined:
                work = self._a2a_async(recv, send, back_splits, send_splits)
            else:
                self._all_to_all(recv, send, back_splits, send_splits)
                work = None
            in_flight.append((ch, rows[n_send:], rows, work))
        self._before_epilogue(previous_event_before_epilogue)
        if pipelined and previous_event_before_epilogue is not None:
            previous_event_before_epilogue.stream_wait(stream_b)
        for ch, src_b, rows, work in in_flight:
            with (torch.cuda.stream(stream_b) if pipelined else self._null_ctx()):
                sb = stream_b if pipelined else stream
                if work is not None:
                    work.wait()
                recv_w = src_b.view(torch.float32)[:, w_off // 4].contiguous() if w_elems else None
                lo, hi = ch.lo, ch.hi
                self._mark(sb)
                kern.combine_reduce(MODE_EPILOGUE, src_b[:, :hidden], combined_x[lo:hi], hi - lo, table=ch.table_b,
                                    row_weights=recv_w, bias0=bias_0[lo:hi] if bias_0 is not None else None,
                                    bias1=bias_1[lo:hi] if bias_1 is not None else None,
                                    wtable=ch.table_b if w_elems else None, wsrc=recv_w,
                                    out_weights=combined_w[lo:hi] if combined_w is not None else None, stream=sb)
                self._mark(sb)
        if pipelined:
            stream.wait_stream(stream_b)
            for _, _, rows, _ in in_flight:
                rows.record_stream(stream_b)

    # ------------------------------------------------------------------ EP > 1 over xGMI windows
    def _window(self, row_bytes: int, slots: Optional[int] = None, rows_per_slot: Optional[int] = None):
        """The symmetric window: `num_bytes` (the reference's symmetric buffer size, buffer.hpp:589-686,
        which holds every combine layout of the declared shape: min(R, K) or K receive slots x T_max
        rows) or more if a call needs it; allocated on first use (collective: every rank reaches the
        same combine)."""
        slots = self._window_slots if slots is None else slots
        need = slots * (rows_per_slot or self.num_max_tokens_per_rank) * row_bytes
        if self._sym is not None and self._sym.data_bytes >= need:
            if not self._capturing:
                self._sym.poll()                  # an earlier call's barrier timed out: raise now
            return self._sym
        from .symmetric import SymmetricBuffer
        old = self._sym
        if old is not None:
            self._group_barrier()                 # no rank still uses the old window
        # the new window is allocated (and exported) before the old one is freed: exporting an
        # allocation that reuses a freed, previously exported address fails (hipIpcGetMemHandle)
        self._sym = SymmetricBuffer(self.group, self.rank_idx, self.num_ranks, max(need, self.num_bytes),
                                    self.device, exchange=self._sym_exchange, timeout_s=self.num_gpu_timeout_secs)
        if old is not None:
            old.destroy()
        # plans cache peer row addresses: they are valid for this window only (a process-unique id,
        # since one handle may serve several buffers)
        if self._sym_gen is not None:
            self._old_sym_gens.add(self._sym_gen)
        self._sym_gen = next(_WINDOW_IDS)
        return self._sym

    def _combine_xgmi(self, handle, x, expanded, row_w, wsrc, K, hidden, bias_0, bias_1, topk_weights,
                      combined_x, combined_w, previous_event_before_epilogue, stream) -> None:
        """EP > 1 combine over the symmetric windows (the reference's NVLink design on xGMI):
        barrier (peers done reading their windows) -> phase A storing every partial and its top-k
        weights straight into the owner's window row slot * T_max + t (combine.cuh:96-106, 215-226)
        -> all partials landed (comm.cuh:88-129) -> phase B over the local window.  Split into
        source-token chunks like the RCCL path: phase A of chunk c is followed by a signal on split
        barrier c, and phase B of chunk c runs on a second stream behind the wait for every rank's
        signal c, so it overlaps phase A of the later chunks."""
        T_max = handle.num_max_tokens_per_rank
        self._window_slots = min(self.num_ranks, K)       # rank layout when R <= K (combine_utils.cuh:8-13)
        row_bytes, w_off, w_pad = packed_row_layout(hidden, K)     # the weight tail is always reserved
        sym = self._window(row_bytes, rows_per_slot=T_max)
        num_chunks = min(self._num_chunks(handle), 63)
        plan = self._plan(handle, False, num_chunks, hidden, window=sym)
        kern = self.kernels
        if topk_weights is not None:
            _require_weight_index(plan)
        windows = (sym.data_bases_dev, sym.data_bytes)
        n_rows = self._window_slots * T_max
        rows = sym.data[:n_rows * row_bytes].view(torch.bfloat16).view(n_rows, row_bytes // 2)
        recv_wsrc = sym.data[:n_rows * row_bytes].view(torch.float32) if topk_weights is not None else None
        pipelined = len(plan.chunks) > 1
        err = sym.error_flag                              # a timed-out barrier poisons the launches below
        sym.barrier(stream)                               # peers finished reading their windows
        if pipelined:
            if getattr(self, '_stream_b', None) is None:
                self._stream_b = torch.cuda.Stream(device=self.device)
            stream_b = self._stream_b
            stream_b.wait_stream(stream)
        # Optional CU budget for phase A (DEEPEP_PHASE_A_CUS): its stores wait on the xGMI links, so
        # its waves can hold CUs long after their loads; fewer CUs for it leave the rest to phase B
        # of the earlier chunks.  Results are identical; only the overlap changes.
        sa = self._cu_budget_stream(self.phase_a_cus) if pipelined and self.phase_a_cus else None
        sa = stream if sa is None else sa
        if sa is not stream:
            sa.wait_stream(stream)
        for c, ch in enumerate(plan.chunks):
            self._mark(sa)
            kern.combine_reduce_scatter(x, ch.out_rows.shape[0], ch.out_rows, table=ch.table_a, row_weights=row_w,
                                        wtable=ch.wtable_a, wsrc=wsrc,
                                        num_weights=K if topk_weights is not None else 0,
                                        weights_offset=w_off, weights_pad=w_pad, error_flag=err, windows=windows,
                                        stream=sa)
            self._mark(sa)
            sym.signal(1 + c, sa)
        if sa is not stream:
            stream.wait_stream(sa)
        self._before_epilogue(previous_event_before_epilogue)
        sb = stream_b if pipelined else stream
        if pipelined and previous_event_before_epilogue is not None:
            previous_event_before_epilogue.stream_wait(stream_b)
        for c, ch in enumerate(plan.chunks):
            sym.wait(1 + c, sb)
            wtable_b = ch.wtable_b if topk_weights is not None else None
            lo, hi = ch.lo, ch.hi
            self._mark(sb)
            kern.combine_reduce(MODE_EPILOGUE, rows[:, :hidden], combined_x[lo:hi], hi - lo, table=ch.table_b,
                                bias0=bias_0[lo:hi] if bias_0 is not None else None,
                                bias1=bias_1[lo:hi] if bias_1 is not None else None,
                                wtable=wtable_b, wsrc=recv_wsrc,
                                out_weights=combined_w[lo:hi] if combined_w is not None else None,
                                error_flag=err, stream=sb)
            self._mark(sb)
        if pipelined:
            stream.wait_stream(stream_b)
        if not self._capturing:
            sym.publish(stream)

    def _combine_xgmi_single(self, handle, x, row_w, wsrc, K, hidden, bias_0, bias_1, topk_weights,
                             combined_x, combined_w, previous_event_before_epilogue, stream) -> None:
        """Single-reduction combine over the symmetric windows (kDoExpandedSend, combine.cuh:177-213):
        every valid expanded row of (token t, lane k) is copied unreduced -- with its gating weight in
        a 16-byte tail when weights are given -- straight into the source rank's window row
        k * T_max + t (per-top-k slot layout, buffer.hpp:616-633), then one EPILOGUE reduce per token
        over its K rows (weighted: the legacy low-latency fma chain).  Chunked by source token like
        _combine_xgmi, phase B of chunk c behind the split barrier of chunk c."""
        T_max = handle.num_max_tokens_per_rank
        with_w = topk_weights is not None
        self._window_slots = K
        # the weight tail is always reserved: one window size per buffer
        row_bytes, w_off, w_pad = packed_row_layout(hidden, 1, True, single=True)
        sym = self._window(row_bytes, rows_per_slot=T_max)
        num_chunks = min(self._num_chunks(handle), 63)
        plan = self._plan(handle, True, num_chunks, hidden, window=sym)
        kern = self.kernels
        n_rows = K * T_max
        win = sym.data[:n_rows * row_bytes]
        rows = win.view(torch.bfloat16).view(n_rows, row_bytes // 2)
        win_w = win.view(torch.float32).view(K, T_max, row_bytes // 4)[:, :, w_off // 4] if with_w else None
        recv_w = torch.empty((K, T_max), dtype=torch.float32, device=x.device) if with_w else None
        pipelined = len(plan.chunks) > 1
        err = sym.error_flag                              # a timed-out barrier poisons the launches below
        sym.barrier(stream)                               # peers finished reading their windows
        if pipelined:
            if getattr(self, '_stream_b', None) is None:
                self._stream_b = torch.cuda.Stream(device=self.device)
            stream_b = self._stream_b
            stream_b.wait_stream(stream)
        for c, ch in enumerate(plan.chunks):
            self._mark(stream)
            kern.combine_reduce_scatter(x, ch.out_rows.shape[0], ch.out_rows, table=ch.table_a,
                                        wtable=ch.table_a if with_w else None, wsrc=wsrc if with_w else None,
                                        num_weights=1 if with_w else 0, weights_offset=w_off, weights_pad=w_pad,
                                        error_flag=err, windows=(sym.data_bases_dev, sym.data_bytes),
                                        stream=stream)
            self._mark(stream)
            sym.signal(1 + c, stream)
        self._before_epilogue(previous_event_before_epilogue)
        sb = stream_b if pipelined else stream
        if pipelined and previous_event_before_epilogue is not None:
            previous_event_before_epilogue.stream_wait(stream_b)
        for c, ch in enumerate(plan.chunks):
            sym.wait(1 + c, sb)
            lo, hi = ch.lo, ch.hi
            rw = None
            if with_w:
                with torch.cuda.stream(sb):
                    recv_w[:, lo:hi].copy_(win_w[:, lo:hi])      # the chunk's weights out of the row tails
                rw = recv_w.view(-1)
            self._mark(sb)
            kern.combine_reduce(MODE_EPILOGUE, rows[:, :hidden], combined_x[lo:hi], hi - lo, table=ch.table_b,
                                row_weights=rw if row_w is not None else None,
                                bias0=bias_0[lo:hi] if bias_0 is not None else None,
                                bias1=bias_1[lo:hi] if bias_1 is not None else None,
                                wtable=ch.table_b if with_w else None, wsrc=rw,
                                out_weights=combined_w[lo:hi] if combined_w is not None else None,
                                error_flag=err, stream=sb)
            self._mark(sb)
        if pipelined:
            stream.wait_stream(stream_b)
            if recv_w is not None:
                recv_w.record_stream(stream_b)
        if not self._capturing:
            sym.publish(stream)
