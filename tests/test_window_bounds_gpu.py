"""Memory safety of the window paths (the xGMI transport) on the GPU: every address the product
computes for a store into a symmetric window is checked against the windows' extents, and a bad one
is never stored through -- it sets a flag bit and leaves a fault record (include/deepep_amd.h,
DEEPEP_ERROR_RECORD_INTS) that the host turns into a RuntimeError.

Each case feeds deliberately inconsistent inputs -- an out-of-window row address, counts that
disagree with the metadata, a window too small for its rows, destination offsets past the buffer --
and checks that (1) nothing outside the windows changed (canary regions around them stay zero),
(2) the flag and the record name the fault, (3) the consistent units are still exact.  The "windows"
here are regions of one local allocation, so a store that escaped the check would land in a canary
(detected), not in unmapped memory.  Reference behaviour: the NVLink push only ever addresses rows
of the registered window (deep_ep/common/handle.cuh:64-92, impls/combine.cuh:95-106 in
/root/reference); the reference has no recovery path -- EP_DEVICE_ASSERT traps.
"""
import numpy as np
import pytest
import torch

import oracle
from tests.oracle_kernels import OracleKernels

pytestmark = pytest.mark.gpu

MODE_LOCAL = 0
FLAG_BAD_SLOT, FLAG_BAD_ADDRESS = 1, 4
FAULT_SCATTER_ROW, FAULT_PLAN_ROW, FAULT_PLAN_UNIT, FAULT_PACK_ROW = 1, 2, 3, 4


@pytest.fixture(scope='module')
def kern():
    from deepep_amd.kernels import HipKernels
    assert torch.cuda.is_available()
    return HipKernels()


def _bf16(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16).cuda()


def _addr(rec) -> int:
    return (int(rec[5]) & 0xffffffff) << 32 | (int(rec[4]) & 0xffffffff)


@pytest.mark.parametrize('cfg', [(0, 0), (1, 2), (2, 8)])
def test_scatter_never_stores_outside_its_windows(kern, cfg):
    """Units whose row address is in a canary region, straddles a window's end, is misaligned or is
    null are skipped; every other unit lands exactly; the first bad unit is recorded."""
    rng = np.random.default_rng(7)
    H, K, units = 1024, 8, 12
    row_bytes = 2 * H + 128                          # bf16 row + a whole weight line
    W = 6 * row_bytes                                # one window holds 6 rows
    src = oracle.f32_to_bf16(rng.standard_normal((units * K, H)).astype(np.float32))
    table = rng.integers(0, units * K, size=(units, K)).astype(np.int32)
    wsrc = torch.rand(units * K, device='cuda')
    buf = torch.zeros((5 * W,), dtype=torch.uint8, device='cuda')   # [win0 | canary | win1 | canary | canary]
    base = buf.data_ptr()
    wins = torch.tensor([base, base + 2 * W], dtype=torch.int64, device='cuda')
    good = [base + 0 * row_bytes, base + 2 * W + 1 * row_bytes, base + 3 * row_bytes, base + 2 * W + 5 * row_bytes,
            base + 5 * row_bytes, base + 2 * W]
    bad = {6: base + W,                              # inside the first canary
           7: base + W - row_bytes + 16,             # starts inside window 0, ends past it
           8: base + 8,                              # not 16-byte aligned
           9: base + 4 * W + 4096,                   # far past both windows (the last canary)
           10: 0}                                    # a unit plan_expert rejected
    addr = good + [bad[u] for u in range(6, 11)] + [base + 2 * W + 3 * row_bytes]
    err = torch.zeros((8,), dtype=torch.int32, device='cuda')
    assert kern.lib.deepep_set_launch_config(*cfg) == 0
    try:
        kern.combine_reduce_scatter(_bf16(src), units, torch.tensor(addr, dtype=torch.int64, device='cuda'),
                                    table=torch.from_numpy(table).cuda(), wtable=torch.from_numpy(table).cuda(),
                                    wsrc=wsrc, num_weights=K, weights_offset=2 * H, weights_pad=32,
                                    error_flag=err, windows=(wins, W))
        torch.cuda.synchronize()
    finally:
        kern.lib.deepep_set_launch_config(0, 0)
    host = buf.cpu()
    assert int(host[W:2 * W].count_nonzero()) == 0, 'a store escaped into canary 1'
    assert int(host[3 * W:].count_nonzero()) == 0, 'a store escaped into canary 2'
    out = torch.empty((units, H), dtype=torch.bfloat16)
    out_w = torch.empty((units, K))
    OracleKernels().combine_reduce(MODE_LOCAL, _bf16(src).cpu(), out, units, table=torch.from_numpy(table),
                                   wtable=torch.from_numpy(table), wsrc=wsrc.cpu(), out_weights=out_w)
    for u in list(range(6)) + [11]:
        off = addr[u] - base
        row = host[off:off + row_bytes]
        assert torch.equal(row[:2 * H].view(torch.bfloat16), out[u]), u
        assert torch.equal(row[2 * H:2 * H + 4 * K].view(torch.float32), out_w[u]), u
    rec = err.tolist()
    assert rec[0] == FLAG_BAD_SLOT | FLAG_BAD_ADDRESS, rec
    assert rec[1] == FAULT_SCATTER_ROW and rec[2] in (6, 7, 8, 9) and _addr(rec) == bad[rec[2]], rec
    # the unaligned row of unit 8 must not have been stored either (window 0 bytes 8.. belong to unit 0)
    assert torch.equal(host[:2 * H].view(torch.bfloat16), out[0])


def test_plan_expert_rejects_inconsistent_counts_and_small_windows(kern):
    """Counts that claim more received rows than the metadata holds, single-reduction pair counts
    below the metadata's valid lanes, and a window too small for a row: the affected units keep the
    caller's fill (-1 slots, 0 rows) and the fault is recorded; consistent units are unchanged."""
    from deepep_amd.handle import PLAN_EXPANDED, PLAN_INTERLEAVE, PLAN_RANK_LAYOUT, PLAN_SINGLE
    R, K, T_max, rank, row_bytes = 2, 2, 64, 0, 1024
    meta = torch.tensor([[0, 0 * K + 1, 0, 1],             # rank 0 token 0: both lanes local
                         [1, 0 * K + 0, 2, -1],            # rank 0 token 1
                         [64 + 3, 1 * K + 1, -1, 3],       # rank 1 token 3
                         [64 + 60, 1 * K + 0, 4, -1]],     # rank 1 token 60 (window row 60)
                        dtype=torch.int32, device='cuda')
    bases = torch.tensor([1 << 40, 2 << 40], dtype=torch.int64, device='cuda')
    flags = PLAN_EXPANDED | PLAN_RANK_LAYOUT | PLAN_INTERLEAVE

    def run(recv_tok, recv_pairs, fl, total, width, window_bytes):
        table = torch.full((total, width), -1, dtype=torch.int32, device='cuda')
        rows = torch.zeros((total,), dtype=torch.int64, device='cuda')
        err = torch.zeros((8,), dtype=torch.int32, device='cuda')
        kern.plan_expert(meta, K, R, rank, T_max, recv_tok, recv_pairs, 1, 1, fl, table, None, bases, row_bytes,
                         rows, window_bytes=window_bytes, error_flag=err)
        torch.cuda.synchronize()
        return table.cpu(), rows.cpu(), err.tolist()

    ok = torch.tensor([[2], [2]], dtype=torch.int32, device='cuda')
    pairs = torch.tensor([[3], [3]], dtype=torch.int32, device='cuda')
    full = K * T_max * row_bytes
    table, rows, rec = run(ok, pairs, flags, 4, K, full)
    assert rec[0] == 0 and (rows != 0).all() and (table != -1).any(dim=1).all(), (rec, rows, table)
    # (1) rank 1 claims 3 rows: row 4 does not exist -> its unit is left as filled, the others are exact
    t3, r3, rec = run(torch.tensor([[2], [3]], dtype=torch.int32, device='cuda'), pairs, flags, 5, K, full)
    assert rec[0] == FLAG_BAD_SLOT and rec[1] == FAULT_PLAN_UNIT and rec[2] == 4 and rec[3] == 1, rec
    assert int((r3 == 0).sum()) == 1 and int((t3 == -1).all(dim=1).sum()) == 1
    assert sorted(r3[r3 != 0].tolist()) == sorted(rows.tolist())
    # (2) single reduction with pair counts below the valid lanes: the excess units are not written
    t4, r4, rec = run(ok, torch.tensor([[2], [2]], dtype=torch.int32, device='cuda'),
                      PLAN_EXPANDED | PLAN_SINGLE | PLAN_INTERLEAVE, 4, 1, full)
    assert rec[0] == FLAG_BAD_SLOT and rec[1] == FAULT_PLAN_UNIT, rec
    assert int((r4 != 0).sum()) == int((t4 != -1).sum()) <= 4
    # (3) a window that holds only 32 rows: token 60's row (and only it) becomes 0
    t5, r5, rec = run(ok, pairs, flags, 4, K, 32 * row_bytes)
    assert rec[0] == FLAG_BAD_SLOT and rec[1] == FAULT_PLAN_ROW and rec[3] == 1, rec
    assert _addr(rec) == (2 << 40) + (rank * T_max + 60) * row_bytes
    assert int((r5 == 0).sum()) == 1 and set(r5[r5 != 0].tolist()) <= set(rows.tolist())
    assert torch.equal(t5, table)


@pytest.mark.parametrize('peer', [False, True])
def test_dispatch_pack_never_stores_past_its_destination(kern, peer):
    """Destination offsets that overrun the destination buffer (dest_rows): those rows are not
    stored (the bytes past dest_rows stay zero) and the fault is recorded; rows inside are exact."""
    from deepep_amd.kernels import RowLayout
    T, R, K, E, H = 40, 2, 4, 8, 256
    g = torch.Generator().manual_seed(3)
    idx = torch.stack([torch.randperm(E, generator=g)[:K] for _ in range(T)]).cuda()
    w = torch.rand((T, K), generator=g).cuda()
    x = torch.randn((T, H), generator=g).to(torch.bfloat16).cuda()
    dst = torch.empty((T, R), dtype=torch.int32, device='cuda')
    cnt = torch.empty((R,), dtype=torch.int32, device='cuda')
    kern.dispatch_route(idx, E, R, dst, cnt)
    cl = cnt.tolist()
    layout = RowLayout.make(2 * H, 0, K)
    xb = x.view(torch.uint8).view(T, -1)

    lead = 8                                             # canary rows in front of the destination buffer

    def pack(offs, dest_rows, rows_alloc):
        big = torch.zeros((lead + rows_alloc, layout.row_bytes), dtype=torch.uint8, device='cuda')
        packed = big[lead:]
        err = torch.zeros((8,), dtype=torch.int32, device='cuda')
        o = torch.tensor(offs, dtype=torch.int32, device='cuda')
        if peer:          # every destination "window" is the same local buffer, dest_rows rows long
            kern.dispatch_pack(xb, None, idx, w, 0, dst, o, None, layout,
                               dest_bases=torch.tensor([packed.data_ptr()] * R, dtype=torch.int64, device='cuda'),
                               dest_rows=dest_rows, error_flag=err)
        else:
            kern.dispatch_pack(xb, None, idx, w, 0, dst, o, packed, layout, dest_rows=dest_rows, error_flag=err)
        torch.cuda.synchronize()
        big = big.cpu()
        assert int(big[:lead].count_nonzero()) == 0, 'a row was stored in front of the destination buffer'
        return big[lead:], err.tolist()

    n = sum(cl)
    ref, rec = pack([0, cl[0]], n, n)
    assert rec[0] == 0
    cut = n - 5
    got, rec = pack([0, cl[0]], cut, n)
    assert int(got[cut:].count_nonzero()) == 0, 'rows past dest_rows were stored'
    assert torch.equal(got[:cut], ref[:cut])
    assert rec[0] == FLAG_BAD_ADDRESS and rec[1] == FAULT_PACK_ROW and rec[3] == 1, rec
    # a negative offset is rejected the same way: nothing lands in front of the buffer
    got, rec = pack([0, -3], n, n)
    assert rec[0] == FLAG_BAD_ADDRESS and rec[1] == FAULT_PACK_ROW and rec[3] == 1, rec


def test_sym_put_never_stores_past_the_window(kern):
    """deepep_sym_put (the window notify's put) checks its extent at the C-ABI: a put whose
    [dest_offset, dest_offset + bytes) reaches past the destination window's extent is rejected before
    any launch -- nothing is stored, the canaries after the window stay zero -- and an in-bounds put
    lands exactly where it was asked to."""
    R, window, tail = 2, 4096, 1024
    big = torch.zeros((R, window + tail), dtype=torch.uint8, device='cuda')       # window + canary tail per rank
    bases = torch.tensor([big[d].data_ptr() for d in range(R)], dtype=torch.int64, device='cuda')
    src = torch.arange(R * 64, dtype=torch.int32, device='cuda').view(R, 64) + 1       # 256 bytes per rank
    stream = torch.cuda.current_stream().cuda_stream
    lib = kern.lib
    # past the end: offset + bytes = window + 16
    rc = lib.deepep_sym_put(src.data_ptr(), 256, bases.data_ptr(), R, window - 240, window, None, stream)
    assert rc == -1                                   # DEEPEP_ERR_INVALID_ARG
    assert b'outside' in lib.deepep_amd_last_error()
    torch.cuda.synchronize()
    assert int(big.count_nonzero()) == 0, 'a rejected put stored something'
    # exactly at the end: accepted, stored in every destination, the tail untouched
    rc = lib.deepep_sym_put(src.data_ptr(), 256, bases.data_ptr(), R, window - 256, window, None, stream)
    assert rc == 0, lib.deepep_amd_last_error()
    torch.cuda.synchronize()
    for d in range(R):
        assert torch.equal(big[d, window - 256:window].view(torch.int32), src[d])
        assert int(big[d, window:].count_nonzero()) == 0
        assert int(big[d, :window - 256].count_nonzero()) == 0


def test_padded_plan_never_overwrites_another_source(kern):
    """A dispatch without a CPU sync pads the single reduction's plan per source to min(K, experts per
    rank) lanes per token (buffer.hpp:1067-1069's bound).  A token routed twice to one expert breaks that
    bound: its excess units must be rejected and recorded -- never written into the next source's
    positions -- and the source side must not point past its destination's padded rows."""
    from deepep_amd import _lib
    from tests import plan_ref
    R, K, E, T = 2, 4, 4, 64                               # 2 experts per rank < K
    idx0 = np.tile(np.array([[0, 0, 1, 1]], dtype=np.int64), (T, 1))     # 4 lanes on rank 0: duplicates
    idx1 = np.tile(np.array([[0, 1, 2, 3]], dtype=np.int64), (T, 1))     # 2 lanes on rank 0
    disp = oracle.simulate_dispatch([idx0, idx1], E, T)
    meta = torch.from_numpy(disp[0]['src_metadata']).cuda()
    recv_tok = torch.tensor([[T], [T]], dtype=torch.int32, device='cuda')
    recv_pairs = torch.tensor([[4 * T], [2 * T]], dtype=torch.int32, device='cuda')
    padded = T * min(K, E // R)                            # 128 positions per source
    for bypass in (False, True):
        flags = _lib.PLAN_EXPANDED | _lib.PLAN_SINGLE | (_lib.PLAN_LOCAL_BYPASS if bypass else 0)
        table = torch.full((R * padded, 1), -1, dtype=torch.int32, device='cuda')
        err = torch.zeros((8,), dtype=torch.int32, device='cuda')
        kern.plan_expert(meta, K, R, 0, T, recv_tok, recv_pairs, 1, 1, flags, table, None, None, 0, None,
                         error_flag=err, padded_stride=padded)
        torch.cuda.synchronize()
        rec = err.tolist()
        assert rec[0] == FLAG_BAD_SLOT and rec[1] == FAULT_PLAN_UNIT and rec[3] == 0, rec
        ref = torch.full((R * padded, 1), -1, dtype=torch.int32)
        plan_ref.plan_expert(meta.cpu(), K, R, 0, T, recv_tok.cpu(), recv_pairs.cpu(), 1, 1, flags, ref, None, None,
                             0, None, padded=padded)
        assert torch.equal(table.cpu(), ref), bypass
        # source 1's 128 units are all there, in its own positions (send order: 1 first with the bypass)
        own1 = slice(0, padded) if bypass else slice(padded, 2 * padded)
        assert bool((table.cpu()[own1] >= 0).all()), bypass
        rows1 = meta.cpu()[meta.cpu()[:, 1] // K == 1][:, 2:]
        assert sorted(table.cpu()[own1].view(-1).tolist()) == sorted(rows1[rows1 >= 0].tolist())
    # the source side of rank 0's tokens: destination 0's rows stop at its padded rows (-1 past them)
    dst = torch.empty((T, R), dtype=torch.int32, device='cuda')
    kern.dispatch_route(torch.from_numpy(idx0).cuda(), E, R, dst, torch.empty((R,), dtype=torch.int32, device='cuda'))
    tok, pairs = plan_ref.route_block_counts(torch.from_numpy(idx0), E, R, 1)
    for bypass in (False, True):
        flags = _lib.PLAN_SINGLE | (_lib.PLAN_LOCAL_BYPASS if bypass else 0)
        tb = torch.full((T, K), -7, dtype=torch.int32, device='cuda')
        kern.plan_source(torch.from_numpy(idx0).cuda(), E, R, 0, T, dst, tok.cuda(), pairs.cuda(), 1, 1, flags, 0, 0,
                         tb, None, padded_stride=padded)
        ref = torch.full((T, K), -7, dtype=torch.int32)
        plan_ref.plan_source(torch.from_numpy(idx0), E, R, 0, T, dst.cpu(), tok, pairs, 1, 1, flags, 0, 0, ref, None,
                             padded=padded)
        got = tb.cpu()
        assert torch.equal(got, ref), bypass
        assert int((got >= 0).sum()) == padded and int(got.max()) < (1 if bypass else 0) * padded + padded


def test_rccl_plan_fault_raises_at_the_next_call():
    """Over the RCCL transport the plan kernels' fault record (here: duplicate experts in a sync-free
    dispatch's handle, more lanes per rank than its padding) is published behind the plan build and
    raises RuntimeError at the handle's next combine -- no silently wrong repeats."""
    from deepep_amd import ElasticBuffer
    from tests.sim import FakeGroup, ThreadComm, run_threads
    R, K, E, T, H = 2, 4, 4, 64, 256
    comm = ThreadComm(R)

    def rank_fn(rank, results):
        try:
            torch.cuda.set_device(0)
            buf = ElasticBuffer(FakeGroup(rank, R, comm), num_max_tokens_per_rank=T, hidden=H, num_topk=K,
                                allow_multiple_reduction=False)
            comm.install(buf, rank)
            row = [0, 0, 1, 1] if rank == 0 else [0, 1, 2, 3]
            idx = torch.tensor([row] * T, dtype=torch.int64, device='cuda')
            w = torch.rand((T, K), device='cuda')
            x = torch.randn((T, H), device='cuda').to(torch.bfloat16)
            ex_x, _, _, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True,
                                                 do_cpu_sync=False)
            buf.combine(ex_x, handle)
            torch.cuda.synchronize()
            comm.bar.wait()
            try:
                buf.combine(ex_x, handle)
                results[rank] = 'no error' if rank == 1 else 'rank 0 (expert side of the duplicates) did not raise'
            except RuntimeError as e:
                results[rank] = 'raised' if 'combine plan' in str(e) else f'wrong error: {e}'
                comm.bar.abort()                  # the peer waits in the call's exchange: release it
        except Exception:
            import traceback
            results[rank] = traceback.format_exc()
            comm.bar.abort()

    results = run_threads(R, rank_fn, (), timeout=120)
    # rank 0 receives rank 0's duplicate lanes: its expert-side plan rejects them
    assert results.get(0) == 'raised', results
