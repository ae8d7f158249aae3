"""GPU parity tests: the HIP kernels (through the C-ABI) against the oracle, bitwise.

* kernel level: every reduction mode, weighted/unweighted (weighted EPILOGUE = the single-reduction
  gating-weighted combine), bias 0/1/2, slot-table widths
  1..32, ragged hidden sizes (tail lanes), empty tables, -0/inf edge values;
* ElasticBuffer level on one GPU: the golden fixtures of the reference oracle at EP = 1
  (BASELINE config 1) and, with 4 or 8 ranks simulated by threads on the one device
  (the all-to-all replaced by device copies), at EP = 4 and EP = 8 (incl. skewed routing);
* BASELINE config 2 at full size (8192 tokens x 7168 x top-8): full output bitwise vs the
  oracle, plain and gating-weighted.
Tolerance: bitwise for everything (bf16 outputs and the fp32 weight pass-through).
"""
import os
import threading

import numpy as np
import pytest
import torch

import oracle
from tests.helpers import (WEIGHTED_TOLERANCE, exact_weighted, load, ordered_accumulate, ranks_of,
                           weighted_multi_expected)
from tests.oracle_kernels import OracleKernels

pytestmark = pytest.mark.gpu

MODE_LOCAL, MODE_EPILOGUE, MODE_FUSED = 0, 1, 2


def _u16(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _bf16(a: np.ndarray, device='cuda') -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16).to(device)


@pytest.fixture(scope='module')
def kern():
    from deepep_amd.kernels import HipKernels
    assert torch.cuda.is_available()
    return HipKernels()


def _random_rows(rng, n, h, special=False):
    a = rng.standard_normal((n, h)).astype(np.float32) * rng.choice([1e-3, 1.0, 300.0], size=(n, 1)).astype(np.float32)
    u = oracle.f32_to_bf16(a)
    if special:
        m = rng.random((n, h))
        u[m < 0.05] = 0x8000        # -0
        u[(m >= 0.05) & (m < 0.10)] = 0x0000
        u[(m >= 0.10) & (m < 0.11)] = 0x7f80   # +inf
        u[(m >= 0.11) & (m < 0.12)] = 0x0001   # denormal
    return u


def _run(kern, mode, weighted, units, width, hidden, nb, seed, identity=False, special=False, upb=0, wt=True):
    rng = np.random.default_rng(seed)
    nsrc = units * max(width, 1) + 3
    src = _random_rows(rng, nsrc, hidden, special)
    if identity:
        table = None
    else:
        table = rng.integers(0, nsrc, size=(units, width)).astype(np.int32)
        table[rng.random((units, width)) < 0.3] = -1
        if units > 2:
            table[0] = -1                         # a row with no valid source
            table[1, 1:] = -1                     # exactly one
    row_w = rng.random(nsrc).astype(np.float32) if weighted else None
    b = [_random_rows(rng, units, hidden, special) for _ in range(2)]
    bias0 = b[0] if nb >= 1 else None
    bias1 = b[1] if nb >= 2 else None
    K = 4
    wtable = rng.integers(-1, units * K, size=(units, K)).astype(np.int32) if wt else None
    wsrc = rng.random(units * K).astype(np.float32)
    # GPU through the C-ABI
    g = dict(src=_bf16(src), out=torch.empty((units, hidden), dtype=torch.bfloat16, device='cuda'),
             table=None if table is None else torch.from_numpy(table).cuda(),
             row_weights=None if row_w is None else torch.from_numpy(row_w).cuda(),
             bias0=None if bias0 is None else _bf16(bias0), bias1=None if bias1 is None else _bf16(bias1),
             wtable=None if wtable is None else torch.from_numpy(wtable).cuda(),
             wsrc=torch.from_numpy(wsrc).cuda(), out_weights=torch.empty((units, K), device='cuda'))
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    kern.combine_reduce(mode, g['src'], g['out'], units, table=g['table'], row_weights=g['row_weights'],
                        bias0=g['bias0'], bias1=g['bias1'], wtable=g['wtable'], wsrc=g['wsrc'],
                        out_weights=g['out_weights'], units_per_block=upb, error_flag=err)
    torch.cuda.synchronize()
    # oracle on the host
    c = {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in g.items()}
    c['out'] = torch.empty((units, hidden), dtype=torch.bfloat16)
    c['out_weights'] = torch.empty((units, K))
    OracleKernels().combine_reduce(mode, c['src'], c['out'], units, table=c['table'], row_weights=c['row_weights'],
                                   bias0=c['bias0'], bias1=c['bias1'], wtable=c['wtable'], wsrc=c['wsrc'],
                                   out_weights=c['out_weights'])
    assert int(err.item()) == 0
    got, exp = _u16(g['out']), _u16(c['out'])
    if not np.array_equal(got, exp):
        bad = np.argwhere(got != exp)[:5]
        raise AssertionError(f'mismatch at {bad.tolist()}: got {[hex(got[tuple(i)]) for i in bad]} '
                             f'expected {[hex(exp[tuple(i)]) for i in bad]}')
    assert torch.equal(g['out_weights'].cpu(), c['out_weights'])


@pytest.mark.parametrize('mode', [MODE_LOCAL, MODE_EPILOGUE, MODE_FUSED])
@pytest.mark.parametrize('width', [1, 2, 3, 8, 17, 32])
@pytest.mark.parametrize('hidden', [64, 520, 2056, 7168])
def test_kernel_modes_widths(kern, mode, width, hidden):
    nbs = [0] if mode == MODE_LOCAL else [0, 1, 2]
    for nb in nbs:
        _run(kern, mode, False, 37, width, hidden, nb, seed=width * 100 + nb)
        _run(kern, mode, True, 37, width, hidden, nb, seed=width * 100 + nb + 7)


@pytest.mark.parametrize('mode', [MODE_LOCAL, MODE_EPILOGUE, MODE_FUSED])
def test_kernel_identity_table_and_special_values(kern, mode):
    for nb in ([0] if mode == MODE_LOCAL else [0, 1, 2]):
        _run(kern, mode, False, 19, 1, 1024, nb, seed=5 + nb, identity=True, special=True)
        _run(kern, mode, False, 19, 8, 1024, nb, seed=9 + nb, special=True)


@pytest.mark.parametrize('upb', [1, 3, 4, 16])
def test_kernel_units_per_block(kern, upb):
    _run(kern, MODE_FUSED, False, 53, 8, 7168, 1, seed=upb, upb=upb)
    _run(kern, MODE_LOCAL, True, 53, 8, 7168, 0, seed=upb + 1, upb=upb, wt=False)


@pytest.mark.parametrize('cfg', [(1, 0), (2, 0), (0, 2), (0, 4), (0, 8), (1, 2), (1, 8), (2, 2), (2, 4)])
@pytest.mark.parametrize('upb', [0, 4, 8])
def test_kernel_launch_configs_identical(kern, cfg, upb):
    """Every deepep_set_launch_config variant (vectors per lane, rows in flight) and workgroup shape
    gives the same bits (deepep_set_launch_config, the diagnostic launch-shape knob)."""
    assert kern.lib.deepep_set_launch_config(*cfg) == 0
    try:
        for mode in (MODE_LOCAL, MODE_EPILOGUE, MODE_FUSED):
            _run(kern, mode, False, 29, 8, 2056, 0 if mode == MODE_LOCAL else 2, seed=sum(cfg) + 2 + mode, upb=upb)
            _run(kern, mode, True, 29, 8, 7168, 0 if mode == MODE_LOCAL else 1, seed=sum(cfg) + 2 + 3 * mode,
                 upb=upb)
            _run(kern, mode, True, 29, 17, 520, 0 if mode == MODE_LOCAL else 2, seed=sum(cfg) + 10 + 5 * mode,
                 upb=upb)                                                       # > 8 valid rows
    finally:
        kern.lib.deepep_set_launch_config(0, 0)


@pytest.mark.parametrize('weighted,hidden', [(False, 7168), (True, 520), (False, 64)])
def test_kernel_reduce_scatter_rows(kern, weighted, hidden):
    """deepep_combine_reduce_scatter (phase A of the xGMI transport) = the LOCAL reduce with each
    unit's row and weights stored at an arbitrary 16-byte aligned address."""
    rng = np.random.default_rng(hidden + weighted)
    units, width, K = 41, 8, 8
    nsrc = units * width
    src = _random_rows(rng, nsrc, hidden)
    table = rng.integers(0, nsrc, size=(units, width)).astype(np.int32)
    table[rng.random((units, width)) < 0.3] = -1
    table[0] = -1
    row_w = rng.random(nsrc).astype(np.float32)
    row_bytes = hidden * 2 + 48                    # weights at hidden * 2 + 16
    perm = rng.permutation(units)
    win = torch.zeros((units * row_bytes,), dtype=torch.uint8, device='cuda')
    addr = torch.tensor([win.data_ptr() + int(p) * row_bytes for p in perm], dtype=torch.int64, device='cuda')
    g_src, g_tab = _bf16(src), torch.from_numpy(table).cuda()
    g_w = torch.from_numpy(row_w).cuda()
    kern.combine_reduce_scatter(g_src, units, addr, table=g_tab, row_weights=g_w if weighted else None,
                                wtable=g_tab, wsrc=g_w, num_weights=K, weights_offset=hidden * 2 + 16,
                                windows=(torch.tensor([win.data_ptr()], device='cuda'), win.numel()))
    torch.cuda.synchronize()
    out = torch.empty((units, hidden), dtype=torch.bfloat16)
    out_w = torch.empty((units, K))
    OracleKernels().combine_reduce(MODE_LOCAL, g_src.cpu(), out, units, table=g_tab.cpu(),
                                   row_weights=g_w.cpu() if weighted else None, wtable=g_tab.cpu(), wsrc=g_w.cpu(),
                                   out_weights=out_w)
    rows = win.cpu().view(units, row_bytes)[torch.from_numpy(perm)]
    got = rows[:, :hidden * 2].contiguous().view(torch.bfloat16)
    got_w = rows[:, hidden * 2 + 16:hidden * 2 + 16 + 4 * K].contiguous().view(torch.float32)
    assert np.array_equal(_u16(got), _u16(out))
    assert torch.equal(got_w, out_w)


def test_kernel_poisoned_by_timed_out_barrier(kern):
    """Bit 2 of the error flag (a symmetric-window barrier timed out): the reduce writes NaN rows and the
    scatter (phase A into peers' windows) stores nothing; bit 1 (bad slot) alone changes nothing."""
    rng = np.random.default_rng(3)
    src = _bf16(_random_rows(rng, 64, 1024))
    table = torch.randint(0, 64, (16, 8), dtype=torch.int32, device='cuda')
    for flag, cfg in ((2, (0, 0)), (3, (1, 2)), (2, (2, 8))):
        assert kern.lib.deepep_set_launch_config(*cfg) == 0
        try:
            err = torch.zeros((8,), dtype=torch.int32, device='cuda')
            err[0] = flag
            out = torch.zeros((16, 1024), dtype=torch.bfloat16, device='cuda')
            kern.combine_reduce(MODE_FUSED, src, out, 16, table=table, error_flag=err)
            win = torch.zeros((16 * 2048,), dtype=torch.uint8, device='cuda')
            addr = torch.arange(16, device='cuda', dtype=torch.int64) * 2048 + win.data_ptr()
            kern.combine_reduce_scatter(src, 16, addr, table=table, error_flag=err,
                                        windows=(torch.tensor([win.data_ptr()], device='cuda'), win.numel()))
            torch.cuda.synchronize()
            assert bool(torch.isnan(out.float()).all()), flag
            assert int(win.count_nonzero()) == 0, flag
        finally:
            kern.lib.deepep_set_launch_config(0, 0)
    err = torch.ones((1,), dtype=torch.int32, device='cuda')
    out = torch.zeros((16, 1024), dtype=torch.bfloat16, device='cuda')
    kern.combine_reduce(MODE_FUSED, src, out, 16, table=table, error_flag=err)
    ref = torch.zeros_like(out)
    kern.combine_reduce(MODE_FUSED, src, ref, 16, table=table)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize('cfg', [(0, 0), (1, 2), (2, 8)])
def test_kernel_weights_pad_fills_the_tail_line(kern, cfg):
    """weights_pad: each unit's weight row is written as weights_pad floats (the weights, then zeros) --
    a packed row's whole 128-byte tail line -- and nothing past it."""
    rng = np.random.default_rng(sum(cfg))
    units, K, H = 23, 8, 1024
    src = _bf16(_random_rows(rng, units * K, H))
    table = torch.from_numpy(rng.integers(0, units * K, size=(units, K)).astype(np.int32)).cuda()
    wsrc = torch.rand(units * K, device='cuda')
    packed = torch.full((units, H + 128), 7.0, dtype=torch.bfloat16, device='cuda')
    ow = packed.view(torch.float32)[:, H // 2:H // 2 + K]
    assert kern.lib.deepep_set_launch_config(*cfg) == 0
    try:
        kern.combine_reduce(MODE_LOCAL, src, packed[:, :H], units, table=table, wtable=table, wsrc=wsrc,
                            out_weights=ow, weights_pad=32)
        torch.cuda.synchronize()
    finally:
        kern.lib.deepep_set_launch_config(0, 0)
    tail = packed.view(torch.float32)[:, H // 2:]
    assert torch.equal(tail[:, :K], wsrc[table.long()])
    assert bool((tail[:, K:32] == 0).all())
    assert bool((packed[:, H + 64:] == 7.0).all())                 # past the 32 floats: untouched
    win = torch.full((units, H + 128), 7.0, dtype=torch.bfloat16, device='cuda')
    addr = torch.arange(units, device='cuda', dtype=torch.int64) * (2 * H + 256) + win.data_ptr()
    kern.combine_reduce_scatter(src, units, addr, table=table, wtable=table, wsrc=wsrc, num_weights=K,
                                weights_offset=2 * H, weights_pad=32,
                                windows=(torch.tensor([win.data_ptr()], device='cuda'), win.numel() * 2))
    torch.cuda.synchronize()
    assert torch.equal(win[:, :H], packed[:, :H])
    assert torch.equal(win.view(torch.float32)[:, H // 2:], tail)


def test_kernel_empty_and_errors(kern):
    src = torch.zeros((4, 64), dtype=torch.bfloat16, device='cuda')
    out = torch.empty((0, 64), dtype=torch.bfloat16, device='cuda')
    kern.combine_reduce(MODE_FUSED, src, out, 0)                    # no units: no launch, no error
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    out = torch.empty((1, 64), dtype=torch.bfloat16, device='cuda')
    table = torch.tensor([[0, 99]], dtype=torch.int32, device='cuda')   # 99 >= num_src_rows
    kern.combine_reduce(MODE_EPILOGUE, src, out, 1, table=table, error_flag=err)
    torch.cuda.synchronize()
    assert err.item() == 1
    with pytest.raises(RuntimeError):
        kern.combine_reduce(MODE_LOCAL, src, out, 1, table=table, bias0=out)    # bias in phase A
    with pytest.raises(RuntimeError):
        kern.combine_reduce(MODE_EPILOGUE, src[:, :60], out[:, :60], 1)          # hidden % 8 != 0


# ----------------------------------------------------------------------------- ElasticBuffer level

# the simulated ranks' exchange has ProcessGroupNCCL's stream semantics (tests/sim.py)
from tests.sim import FakeGroup as _FakeGroup, ThreadComm as _ThreadComm  # noqa: E402


def _buffer_case(rank, world, fixture, comm, results):
    try:
        torch.cuda.set_device(0)
        from deepep_amd import ElasticBuffer
        fx = load(fixture)
        T, H, K, E, R = (int(v) for v in fx['meta'])
        ranks = ranks_of(fx)
        me = ranks[rank]
        grp = _FakeGroup(rank, world, comm) if world > 1 else None
        if grp is None:
            import torch.distributed as dist
            if not dist.is_initialized():
                os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
                os.environ.setdefault('MASTER_PORT', '29541')
                dist.init_process_group('gloo', rank=0, world_size=1)
            grp = dist.group.WORLD
        buf = ElasticBuffer(grp, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
        if world > 1:
            comm.install(buf, rank)
        idx = torch.from_numpy(me['topk_idx'].copy()).cuda()
        w = torch.from_numpy(me['topk_weights'].copy()).cuda()
        x = _bf16(me['x']) if 'x' in me else torch.randn((T, H), device='cuda').to(torch.bfloat16)
        failures = []

        def y_of(g):
            s, t = divmod(int(g), T)
            return ranks[s]['y'][t]

        recv_x, recv_idx, recv_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E)
        n = handle.num_recv_tokens
        src = handle.recv_src_metadata[:n, 0].cpu().numpy()
        if 'dispatch_recv_src_token_idx' in me:          # the HIP dispatch vs refs.dispatch (refs.py:10-123)
            if not np.array_equal(src, me['dispatch_recv_src_token_idx']):
                failures.append('dispatch order != refs.dispatch')
            if not np.array_equal(recv_idx.cpu().numpy(), me['dispatch_recv_topk_idx']):
                failures.append('recv_topk_idx != refs.dispatch')
            if not np.array_equal(_u16(recv_x), me['dispatch_recv_x']):
                failures.append('recv_x != refs.dispatch')
            if not np.array_equal(recv_w.cpu().numpy(), me['dispatch_recv_topk_weights']):
                failures.append('recv_topk_weights != refs.dispatch')
        local = np.stack([y_of(g) for g in src]) if n else np.zeros((0, K, H), np.uint16)
        local = np.where((recv_idx.cpu().numpy() == -1)[..., None], np.uint16(0), local)
        x_red = _bf16(ordered_accumulate(local)) if n else torch.empty((0, H), dtype=torch.bfloat16, device='cuda')
        ex_x, _, ex_w, ex_handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
        meta = ex_handle.recv_src_metadata.cpu().numpy()
        x_exp = np.full((ex_x.shape[0], H), 0x7fc1, dtype=np.uint16)
        for i in range(meta.shape[0]):
            y = y_of(meta[i, 0])
            for k in range(K):
                if meta[i, 2 + k] >= 0:
                    x_exp[meta[i, 2 + k]] = y[k]
        x_exp = _bf16(x_exp)
        biases = [_bf16(me['bias0']), _bf16(me['bias1'])]
        for nb in (0, 1, 2):
            bias = None if nb == 0 else (biases[0] if nb == 1 else tuple(biases))
            for xin, h, ww, tag in ((x_red, handle, recv_w, 'non-expanded'), (x_exp, ex_handle, ex_w, 'expanded')):
                out, out_w, _ = buf.combine(xin, h, topk_weights=ww, bias=bias)
                torch.cuda.synchronize()
                if not np.array_equal(_u16(out), me[f'combined_multi_b{nb}']):
                    failures.append(f'{tag} b{nb}')
                if not torch.equal(out_w.cpu(), torch.from_numpy(me['topk_weights'])):
                    failures.append(f'{tag} weights b{nb}')
            # gating-weighted with multiple reduction (the N > 1 bench recipe): bitwise vs the oracle's
            # restatement, and within the reference's weighted tolerance (calc_diff < 1e-5,
            # test_low_latency.py:178-181) of the exact float64 sum
            out, out_w, _ = buf.combine(x_exp, ex_handle, topk_weights=ex_w, bias=bias, apply_topk_weights=True)
            torch.cuda.synchronize()
            bias_u16 = (None, None) if nb == 0 else (me['bias0'], me['bias1'] if nb == 2 else None)
            if not np.array_equal(_u16(out), weighted_multi_expected(fx, rank, bias_u16)):
                failures.append(f'weighted multi-reduction b{nb}')
            if not torch.equal(out_w.cpu(), torch.from_numpy(me['topk_weights'])):
                failures.append(f'weighted multi-reduction weights b{nb}')
            if nb == 0:
                d = oracle.calc_diff(oracle.bf16_to_f32(_u16(out)), exact_weighted(me))
                if not d < WEIGHTED_TOLERANCE:
                    failures.append(f'weighted multi-reduction calc_diff {d} >= {WEIGHTED_TOLERANCE}')
        # allow_multiple_reduction=False: every expanded row travels unreduced, one reduction at the
        # source rank -- plain (refs.combine single-level fixtures) and gating-weighted (legacy
        # low-latency fma chain, bias in front)
        from tests.test_buffer_cpu import _weighted_single
        sbuf = ElasticBuffer(grp, num_max_tokens_per_rank=T, hidden=H, num_topk=K, allow_multiple_reduction=False)
        if world > 1:
            comm.install(sbuf, rank)
        for nb in (0, 1, 2):
            bias = None if nb == 0 else (biases[0] if nb == 1 else tuple(biases))
            out, out_w, _ = sbuf.combine(x_exp, ex_handle, bias=bias)
            torch.cuda.synchronize()
            if not np.array_equal(_u16(out), me[f'combined_single_b{nb}']) or out_w is not None:
                failures.append(f'single-reduction b{nb}')
            out, out_w, _ = sbuf.combine(x_exp, ex_handle, topk_weights=ex_w, bias=bias, apply_topk_weights=True)
            torch.cuda.synchronize()
            cpu_bias = None if bias is None else (bias.cpu() if nb == 1 else tuple(b.cpu() for b in bias))
            exp = _weighted_single(me['y'], torch.from_numpy(me['topk_idx']), torch.from_numpy(me['topk_weights']),
                                   cpu_bias)
            if not torch.equal(out.cpu(), exp):
                failures.append(f'single-reduction weighted b{nb}')
            if not torch.equal(out_w.cpu(), torch.from_numpy(me['topk_weights'])):
                failures.append(f'single-reduction weighted pass-through b{nb}')
        results[rank] = failures
    except Exception:
        import traceback
        results[rank] = [traceback.format_exc()]
        comm.bar.abort() if comm is not None else None


@pytest.mark.parametrize('fixture,world,chunks,phase_a_cus', [
    ('f1_ep1_t128_h1024_k2.npz', 1, 0, 0),
    ('f4_ep4_t96_h256_k2.npz', 4, 0, 0),
    ('f2_ep8_t64_h256_k8.npz', 8, 0, 0),
    ('f3_ep8_skew_t128_h64_k8.npz', 8, 0, 0),
    ('f4_ep4_t96_h256_k2.npz', 4, 3, 0),        # pipelined: phase B of each chunk on the second stream
    ('f3_ep8_skew_t128_h64_k8.npz', 8, 5, 0),
    ('f2_ep8_t64_h256_k8.npz', 8, 4, 64),       # pipelined, phase A on a 64-CU budget stream
])
def test_elastic_buffer_golden_on_gpu(fixture, world, chunks, phase_a_cus, monkeypatch):
    if chunks:
        monkeypatch.setenv('DEEPEP_COMBINE_CHUNKS', str(chunks))
    monkeypatch.setenv('DEEPEP_PHASE_A_CUS', str(phase_a_cus))
    comm = _ThreadComm(world) if world > 1 else None
    results = {}
    threads = [threading.Thread(target=_buffer_case, args=(r, world, fixture, comm, results)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert len(results) == world, results
    bad = {r: f for r, f in results.items() if f}
    assert not bad, bad


@pytest.mark.parametrize('weighted,T,skew', [(False, 8192, 1.0), (True, 8192, 1.0), (False, 16384, 4.0)])
def test_config2_full_size_bitwise(weighted, T, skew):
    """BASELINE config 2: EP=1, 8192 tokens, hidden 7168, top-8, E=256; full output vs the oracle.
    (16384, skew 4): config 5's per-rank batch and routing skew (get_unbalanced_scores) on one GPU."""
    import torch.distributed as dist
    from deepep_amd import ElasticBuffer
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29542')
        dist.init_process_group('gloo', rank=0, world_size=1)
    H, K, E = 7168, 8, 256
    g = torch.Generator(device='cuda').manual_seed(11)
    if skew != 1.0:
        from workloads import get_unbalanced_scores
        torch.manual_seed(11)
        scores = get_unbalanced_scores(T, E, 8, K, skew, device='cuda')
    else:
        scores = torch.rand((T, E), device='cuda', generator=g)
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    x = torch.zeros((T, H), dtype=torch.bfloat16, device='cuda')
    _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda', generator=g).to(torch.bfloat16)
    meta = handle.recv_src_metadata.cpu().numpy()
    part, _ = oracle.phase_a(_u16(y), meta, K, True, ex_w.cpu().numpy(), weighted=weighted)
    recv = np.zeros((1, T, H), np.uint16)
    recv[0, meta[:, 0] % T] = part
    ref, _ = oracle.phase_b(recv, None, idx.cpu().numpy(), E, 1, True, True)
    lib = buf.kernels.lib
    try:
        # the automatic shape (last) and the other launch shapes (vectors per lane, rows in flight)
        for cfg in ((1, 2), (1, 8), (2, 4), (2, 8), (0, 0)):
            assert lib.deepep_set_launch_config(*cfg) == 0
            out, out_w, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=weighted)
            torch.cuda.synchronize()
            assert np.array_equal(_u16(out), ref), f'launch config {cfg}'
            assert torch.equal(out_w, w)
    finally:
        lib.deepep_set_launch_config(0, 0)
    if weighted:
        # and within the reference's weighted tolerance of the exact sum (test_low_latency.py:178-181)
        yd = y.double()
        exact = torch.zeros((T, H), dtype=torch.float64, device='cuda')
        slots = handle.recv_src_metadata[:, 2:].long()
        tok = (handle.recv_src_metadata[:, 0] % T).long()
        for k in range(K):
            exact[tok] += yd[slots[:, k]] * ex_w.double()[slots[:, k]].unsqueeze(1)
        assert oracle.calc_diff(oracle.bf16_to_f32(_u16(out)), exact.cpu().numpy()) < 1e-5


def _ep1_setup(T, H, K, E, seed=3):
    import torch.distributed as dist
    from deepep_amd import ElasticBuffer
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29543')
        dist.init_process_group('gloo', rank=0, world_size=1)
    g = torch.Generator(device='cuda').manual_seed(seed)
    scores = torch.rand((T, E), device='cuda', generator=g)
    w, idx = torch.topk(scores, K, dim=-1, sorted=False)
    idx = idx.to(torch.int64)
    idx[torch.rand(idx.shape, device='cuda', generator=g) < 0.1] = -1
    w = w.masked_fill(idx < 0, 0)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    return buf, idx, w, g


def test_hip_graph_capture_replays_combine():
    """The sync-mode combine is capturable into a HIP graph (torch.cuda.graph) and replays bitwise."""
    T, H, K, E = 512, 7168, 8, 64
    buf, idx, w, g = _ep1_setup(T, H, K, E)
    x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
    ex_x, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn(ex_x.shape, device='cuda', generator=g).to(torch.bfloat16)
    bias = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            buf.combine(y, handle, topk_weights=ex_w, bias=bias, apply_topk_weights=True)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out, out_w, _ = buf.combine(y, handle, topk_weights=ex_w, bias=bias, apply_topk_weights=True)
    y.copy_(torch.randn(y.shape, device='cuda', generator=g).to(torch.bfloat16))
    graph.replay()
    ref, ref_w, _ = buf.combine(y, handle, topk_weights=ex_w, bias=bias, apply_topk_weights=True)
    torch.cuda.synchronize()
    assert torch.equal(out, ref) and torch.equal(out_w, ref_w)


def test_hip_graph_cached_dispatch_and_combine():
    """With a cached handle the dispatch has no host sync, so a whole EP = 1 layer's token traffic
    -- cached expanded dispatch + combine -- captures into one HIP graph and replays bitwise."""
    T, H, K, E = 640, 2048, 8, 64
    buf, idx, w, g = _ep1_setup(T, H, K, E, seed=5)
    x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
    _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)

    def layer():
        ex_x, _, ex_w2, _, _ = buf.dispatch(x, topk_weights=w, do_expand=True, handle=handle)
        return buf.combine(ex_x, handle, topk_weights=ex_w2, apply_topk_weights=True)[:2]

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            layer()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out, out_w = layer()
    x.copy_(torch.randn(x.shape, device='cuda', generator=g).to(torch.bfloat16))
    graph.replay()
    ref, ref_w = layer()
    torch.cuda.synchronize()
    assert torch.equal(out, ref) and torch.equal(out_w, ref_w)
    # the weighted sum of a token's own expanded copies: x scaled by the sum of its valid weights
    exact = x.double() * (w.double() * (idx >= 0)).sum(dim=1, keepdim=True)
    assert oracle.calc_diff(oracle.bf16_to_f32(_u16(out)), exact.cpu().numpy()) < 1e-5


def test_fp8_dispatch_then_bf16_combine():
    """BASELINE config 4 at EP=1: FP8 (e4m3, per-128 scales) dispatch, BF16 combine."""
    from workloads import per_token_cast_back, per_token_cast_to_fp8
    T, H, K, E = 256, 7168, 8, 64
    buf, idx, w, g = _ep1_setup(T, H, K, E, seed=4)
    x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
    xq = per_token_cast_to_fp8(x)
    (ex_q, ex_sf), _, ex_w, handle, _ = buf.dispatch(xq, topk_idx=idx, topk_weights=w, num_experts=E,
                                                     do_expand=True)
    meta = handle.recv_src_metadata
    tok = (meta[:, 0] % T).long()
    for k in range(K):
        rows = meta[:, 2 + k]
        ok = rows >= 0
        assert torch.equal(ex_q[rows[ok].long()].view(torch.uint8), xq[0][tok[ok]].view(torch.uint8))
        assert torch.equal(ex_sf[rows[ok].long()], xq[1][tok[ok]])
    # the reference's TMA-aligned column-major scale factors (its expanded test dispatches with them,
    # tests/elastic/test_ep.py:157, 174): the same values, packs of consecutive rows adjacent, fresh and cached
    for h in (None, handle):
        args = dict(topk_weights=w, do_expand=True, use_tma_aligned_col_major_sf=True)
        args.update(handle=h) if h is not None else args.update(topk_idx=idx, num_experts=E)
        (cq, csf), _, _, _, _ = buf.dispatch(xq, **args)
        n = csf.shape[0]
        assert csf.stride() == (1, (n + 3) // 4 * 4), csf.stride()
        assert torch.equal(csf, ex_sf) and torch.equal(cq.view(torch.uint8), ex_q.view(torch.uint8))
    y = per_token_cast_back(ex_q, ex_sf)                     # "expert output" = dequantised input
    out, out_w, _ = buf.combine(y, handle, topk_weights=ex_w)
    torch.cuda.synchronize()
    part, _ = oracle.phase_a(_u16(y), meta.cpu().numpy(), K, True)
    recv = np.zeros((1, T, H), np.uint16)
    recv[0, meta[:, 0].cpu().numpy() % T] = part
    ref, _ = oracle.phase_b(recv, None, idx.cpu().numpy(), E, 1, True, True)
    assert np.array_equal(_u16(out), ref)
    assert torch.equal(out_w, w)
