"""CPU oracle for the combine reduction -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
package, and only as the checker.  The product package (deepep_amd/) never imports
it and has no CPU fallback.

Arithmetic lives in combine_ref.c (a C restatement of the reference kernels,
file:line citations there); this module wraps it with numpy and restates the
data movement the reference performs between the two kernels:

* `simulate_dispatch` restates refs.dispatch's receive order
  (deep_ep/utils/refs.py:10-123: tokens grouped by source rank, ascending source
  token inside a rank) and the expanded layout of dispatch_copy_epilogue_impl
  (deep_ep/include/deep_ep/impls/dispatch_copy_epilogue.cuh:117-121, 188-207:
  expanded rows grouped by local expert; recv_src_metadata = {src_global_idx,
  src_rank*K + master_topk, slot_0..slot_{K-1}}).
* `combine_ep` runs phase A on every expert rank, scatters each partial into the
  owner's receive slot (combine.cuh:95-106: slot = rank under the rank layout,
  else the master top-k lane), then phase B on every source rank.

bf16 tensors are numpy uint16 arrays holding the bit patterns.
"""
import ctypes
import os
import subprocess
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# DEEPEP_ORACLE_LIB=asan: the AddressSanitizer + UBSan build of the same source (`make asan`; the
# process must have the ASan runtime preloaded -- tests/test_oracle_asan.py does that)
_SANITIZED = os.environ.get('DEEPEP_ORACLE_LIB', '') == 'asan'
_LIB_PATH = os.path.join(_HERE, '_build', 'liboracle_asan.so' if _SANITIZED else 'liboracle.so')
_lib = None


def build() -> str:
    subprocess.run(['make', '-s', '-C', _HERE] + (['asan'] if _SANITIZED else []), check=True)
    return _LIB_PATH


def loaded_library() -> str:
    """Path of the checker library this process uses."""
    return _LIB_PATH


def _get_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
                os.path.join(_HERE, 'combine_ref.c')):
            build()
        lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        I, I64 = ctypes.c_int, ctypes.c_int64
        lib.oracle_combine_phase_a.argtypes = [P, I64, I, P, I, I, I, P, I, P, P]
        lib.oracle_combine_phase_b.argtypes = [P, P, I, I, P, I, I, I, I, I, I, P, P, I, P, P]
        lib.oracle_combine_weighted_ll.argtypes = [P, P, P, I, I, I, P]
        lib.oracle_combine_rows.argtypes = [I, I, P, I64, I64, P, I64, I, P, P, P, P, I64, I, I, P, I64, P, P, I, I64]
        for f in (lib.oracle_combine_phase_a, lib.oracle_combine_phase_b, lib.oracle_combine_weighted_ll,
                  lib.oracle_combine_rows):
            f.restype = ctypes.c_int
        _lib = lib
    return _lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype):
    return None if a is None else np.ascontiguousarray(a, dtype=dtype)


# ---------------------------------------------------------------- bf16 helpers

def f32_to_bf16(a: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even (NaN quieted), vectorised; same as combine_ref.c."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7fffffff) > 0x7f800000
    r = ((u + 0x7fff + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_to_f32(a: np.ndarray) -> np.ndarray:
    return (np.ascontiguousarray(a, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def calc_diff(x: np.ndarray, y: np.ndarray) -> float:
    """deep_ep/utils/math.py:5-9 (1 - cosine-like similarity of x+1 and y+1)."""
    x = x.astype(np.float64) + 1
    y = y.astype(np.float64) + 1
    denom = (x * x + y * y).sum()
    return float(1 - 2 * (x * y).sum() / denom)


# ---------------------------------------------------------------- kernels

def phase_a(x: np.ndarray, src_metadata: np.ndarray, num_topk: int, expanded: bool,
            topk_weights: Optional[np.ndarray] = None, weighted: bool = False,
            ) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """combine_impl's local part for every received token (see combine_ref.c)."""
    x = _c(x, np.uint16)
    meta = _c(src_metadata, np.int32)
    n, hidden = meta.shape[0], x.shape[1]
    out = np.zeros((n, hidden), dtype=np.uint16)
    w = _c(topk_weights, np.float32)
    out_w = np.zeros((n, num_topk), dtype=np.float32) if w is not None else None
    rc = _get_lib().oracle_combine_phase_a(_ptr(x), x.shape[0], hidden, _ptr(meta), n, num_topk,
                                           int(expanded), _ptr(w), int(weighted), _ptr(out), _ptr(out_w))
    if rc != 0:
        raise ValueError('oracle phase A: invalid slot index')
    return out, out_w


def phase_b(recv: np.ndarray, recv_w: Optional[np.ndarray], topk_idx: np.ndarray,
            num_experts: int, num_ranks: int, rank_layout: bool, dedup: bool = True,
            bias0: Optional[np.ndarray] = None, bias1: Optional[np.ndarray] = None,
            ) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """combine_reduce_epilogue_impl over a [slots, T_max, H] receive buffer."""
    recv = _c(recv, np.uint16)
    num_slots, t_max, hidden = recv.shape
    idx = _c(topk_idx, np.int64)
    t, k = idx.shape
    out = np.zeros((t, hidden), dtype=np.uint16)
    rw = _c(recv_w, np.float32)
    out_w = np.zeros((t, k), dtype=np.float32) if rw is not None else None
    rc = _get_lib().oracle_combine_phase_b(_ptr(recv), _ptr(rw), num_slots, t_max, _ptr(idx), t, k,
                                           num_experts, num_ranks, int(rank_layout), int(dedup),
                                           _ptr(_c(bias0, np.uint16)), _ptr(_c(bias1, np.uint16)), hidden,
                                           _ptr(out), _ptr(out_w))
    if rc != 0:
        raise ValueError('oracle phase B: invalid arguments')
    return out, out_w


def weighted_ll(y: np.ndarray, topk_idx: np.ndarray, w: np.ndarray) -> np.ndarray:
    """Legacy low-latency weighted combine (y: [T, K, H])."""
    y = _c(y, np.uint16)
    t, k, hidden = y.shape
    out = np.zeros((t, hidden), dtype=np.uint16)
    rc = _get_lib().oracle_combine_weighted_ll(_ptr(y), _ptr(_c(topk_idx, np.int64)), _ptr(_c(w, np.float32)),
                                               t, k, hidden, _ptr(out))
    if rc != 0:
        raise ValueError('oracle weighted: invalid arguments')
    return out


def rows_lib():
    """The C library, for callers that drive oracle_combine_rows with raw host pointers."""
    return _get_lib()


def use_rank_layout(allow_multiple_reduction: bool, num_ranks: int, num_topk: int) -> bool:
    """combine_utils.cuh:8-13."""
    return allow_multiple_reduction and num_ranks <= num_topk


# ---------------------------------------------------------------- data movement

def simulate_dispatch(topk_idx_per_rank: Sequence[np.ndarray], num_experts: int, num_max_tokens: int,
                      expert_alignment: int = 1) -> List[Dict[str, np.ndarray]]:
    """Per expert rank: the received tokens in refs.dispatch order and the expanded layout.

    Returns for every rank r a dict with
      src_global_idx [N_r]   (src_rank * num_max_tokens + src_token), ascending
      src_metadata   [N_r, K+2] int32 in the dispatch_copy_epilogue layout
      expanded_src   [N_exp_r, 2] int64: (src_global_idx, k) feeding each expanded row (-1 for padding)
      num_expanded   int
    """
    R = len(topk_idx_per_rank)
    K = topk_idx_per_rank[0].shape[1]
    epr = num_experts // R
    out = []
    for r in range(R):
        lo, hi = r * epr, (r + 1) * epr
        rows = []                       # (src_rank, src_tok)
        for s in range(R):
            idx = topk_idx_per_rank[s]
            in_r = (idx >= lo) & (idx < hi)
            for t in np.nonzero(in_r.any(axis=1))[0]:
                rows.append((s, int(t)))
        n = len(rows)
        meta = np.full((n, K + 2), -1, dtype=np.int32)
        # Expanded rows grouped by local expert, each expert's group aligned
        per_expert: List[List[Tuple[int, int]]] = [[] for _ in range(epr)]
        for i, (s, t) in enumerate(rows):
            idx = topk_idx_per_rank[s][t]
            for k in range(K):
                if lo <= idx[k] < hi:
                    per_expert[idx[k] - lo].append((i, k))
        cursor = 0
        exp_src = []
        for e in range(epr):
            for (i, k) in per_expert[e]:
                meta[i, 2 + k] = cursor
                s, t = rows[i]
                exp_src.append((s * num_max_tokens + t, k))
                cursor += 1
            pad = (-len(per_expert[e])) % expert_alignment
            exp_src.extend([(-1, -1)] * pad)
            cursor += pad
        for i, (s, t) in enumerate(rows):
            idx = topk_idx_per_rank[s][t]
            in_r = (idx >= lo) & (idx < hi)
            master = int(np.nonzero(in_r)[0].max())
            meta[i, 0] = s * num_max_tokens + t
            meta[i, 1] = s * K + master
        out.append(dict(src_global_idx=meta[:, 0].copy(), src_metadata=meta,
                        expanded_src=np.array(exp_src, dtype=np.int64).reshape(-1, 2),
                        num_expanded=cursor))
    return out


def combine_ep(recv_x_per_rank: Sequence[np.ndarray], src_metadata_per_rank: Sequence[np.ndarray],
               topk_idx_per_rank: Sequence[np.ndarray], num_experts: int, num_max_tokens: int,
               expanded: bool, allow_multiple_reduction: bool = True,
               topk_weights_per_rank: Optional[Sequence[np.ndarray]] = None,
               bias_per_rank: Optional[Sequence[Tuple[Optional[np.ndarray], Optional[np.ndarray]]]] = None,
               weighted: bool = False,
               ) -> List[Tuple[np.ndarray, Optional[np.ndarray]]]:
    """The reference combine across R ranks: phase A -> receive-slot scatter -> phase B.
    weighted: phase A scales each row by its top-k weight (legacy fma chain, this build's
    apply_topk_weights with multiple reduction)."""
    R = len(recv_x_per_rank)
    K = topk_idx_per_rank[0].shape[1]
    hidden = recv_x_per_rank[0].shape[1]
    rank_layout = use_rank_layout(allow_multiple_reduction, R, K)
    expanded_send = expanded and not allow_multiple_reduction      # kDoExpandedSend, combine.cuh:42
    num_slots = min(R, K) if rank_layout else K                    # get_num_tokens_in_layout
    recv = [np.zeros((num_slots, num_max_tokens, hidden), dtype=np.uint16) for _ in range(R)]
    with_w = topk_weights_per_rank is not None and not expanded_send
    recv_w = [np.zeros((num_slots, num_max_tokens, K), dtype=np.float32) for _ in range(R)] if with_w else None
    for r in range(R):
        meta = np.asarray(src_metadata_per_rank[r], dtype=np.int32)
        x = np.asarray(recv_x_per_rank[r], dtype=np.uint16)
        src_tok = meta[:, 0] % num_max_tokens
        src_rank = meta[:, 1] // K
        src_topk = meta[:, 1] % K
        if expanded_send:
            for i in range(meta.shape[0]):
                for k in range(K):
                    slot = meta[i, 2 + k]
                    if slot >= 0:
                        recv[src_rank[i]][k, src_tok[i]] = x[slot]
            continue
        w = topk_weights_per_rank[r] if topk_weights_per_rank is not None else None
        partial, pw = phase_a(x, meta, K, expanded, w, weighted=weighted)
        for i in range(meta.shape[0]):
            slot = r if rank_layout else src_topk[i]
            recv[src_rank[i]][slot, src_tok[i]] = partial[i]
            if with_w:
                recv_w[src_rank[i]][slot, src_tok[i]] = pw[i]
    results = []
    for s in range(R):
        idx = np.asarray(topk_idx_per_rank[s], dtype=np.int64)
        b0, b1 = (None, None) if bias_per_rank is None else bias_per_rank[s]
        dedup = not expanded_send
        out, out_w = phase_b(recv[s], recv_w[s] if with_w else None, idx, num_experts, R,
                             rank_layout, dedup, b0, b1)
        results.append((out, out_w))
    return results


def _split_rows(n: int, parts: int):
    step = max(1, -(-n // max(1, parts)))
    return [(lo, min(n, lo + step)) for lo in range(0, n, step)]


def combine_ep_one(rank: int, recv_x_per_rank: Sequence[np.ndarray], src_metadata_per_rank: Sequence[np.ndarray],
                   topk_idx: np.ndarray, num_experts: int, num_max_tokens: int, expanded: bool,
                   allow_multiple_reduction: bool = True,
                   topk_weights_per_rank: Optional[Sequence[np.ndarray]] = None,
                   bias: Tuple[Optional[np.ndarray], Optional[np.ndarray]] = (None, None),
                   weighted: bool = False, threads: int = 1) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """combine_ep for ONE source rank: only the received rows whose source is `rank` are reduced (phase A
    on every expert rank), only `rank`'s receive buffer is filled and reduced (phase B).  The same
    arithmetic as combine_ep (same C kernels); phase A and phase B are split over `threads` host threads
    (the ctypes calls release the GIL), so a full-size rank (8192 tokens x 7168 x top-8) is checked in
    seconds.  topk_idx: this rank's [T, K] routing."""
    from concurrent.futures import ThreadPoolExecutor
    R = len(recv_x_per_rank)
    K = topk_idx.shape[1]
    hidden = recv_x_per_rank[0].shape[1]
    rank_layout = use_rank_layout(allow_multiple_reduction, R, K)
    assert not (expanded and not allow_multiple_reduction), 'the single reduction is checked by combine_ep'
    num_slots = min(R, K) if rank_layout else K
    recv = np.zeros((num_slots, num_max_tokens, hidden), dtype=np.uint16)
    with_w = topk_weights_per_rank is not None
    recv_w = np.zeros((num_slots, num_max_tokens, K), dtype=np.float32) if with_w else None
    with ThreadPoolExecutor(max_workers=max(1, threads)) as pool:
        for r in range(R):
            meta = np.asarray(src_metadata_per_rank[r], dtype=np.int32)
            mine = np.nonzero(meta[:, 1] // K == rank)[0] if meta.shape[0] else np.zeros(0, np.int64)
            if mine.size == 0:
                continue
            m = np.ascontiguousarray(meta[mine])
            x = np.asarray(recv_x_per_rank[r], dtype=np.uint16)
            w = topk_weights_per_rank[r] if with_w else None
            if expanded:                  # slots index the whole expanded x / weight arrays
                parts = list(pool.map(lambda lh: phase_a(x, m[lh[0]:lh[1]], K, True, w, weighted=weighted),
                                      _split_rows(m.shape[0], threads)))
            else:                         # received row i is x row i: select and slice the rows with the metadata
                xs = np.ascontiguousarray(x[mine])
                ws = np.ascontiguousarray(np.asarray(w, np.float32).reshape(-1, K)[mine]) if w is not None else None
                parts = list(pool.map(lambda lh: phase_a(xs[lh[0]:lh[1]], m[lh[0]:lh[1]], K, False,
                                                         ws[lh[0]:lh[1]] if ws is not None else None),
                                      _split_rows(m.shape[0], threads)))
            partial = np.concatenate([p[0] for p in parts])
            tok = m[:, 0] % num_max_tokens
            slot = np.full(m.shape[0], r) if rank_layout else m[:, 1] % K
            recv[slot, tok] = partial
            if with_w:
                recv_w[slot, tok] = np.concatenate([p[1] for p in parts])
    idx = np.asarray(topk_idx, dtype=np.int64)
    T = idx.shape[0]
    b0, b1 = bias
    out = np.zeros((T, hidden), dtype=np.uint16)
    out_w = np.zeros((T, K), dtype=np.float32) if with_w else None

    def part_b(lh):
        lo, hi = lh
        o, ow = phase_b(recv[:, lo:hi], recv_w[:, lo:hi] if with_w else None, idx[lo:hi], num_experts, R, rank_layout,
                        True, None if b0 is None else b0[lo:hi], None if b1 is None else b1[lo:hi])
        out[lo:hi] = o
        if with_w:
            out_w[lo:hi] = ow
    with ThreadPoolExecutor(max_workers=max(1, threads)) as pool:
        list(pool.map(part_b, _split_rows(T, threads)))
    return out, out_w
