"""The host checks of ElasticBuffer::combine (csrc/elastic/buffer.hpp:1197-1247 in the reference): each one
raises RuntimeError ("Assertion failed: ...", the reference's EPException surfaced by pybind) before any
kernel runs, and a valid call after a rejected one still gives the right bits.  CPU, one gloo rank, the
oracle's row kernels injected (as tests/test_buffer_cpu.py)."""
import os

import pytest
import torch
import torch.distributed as dist

T, H, K, E = 16, 64, 4, 8


@pytest.fixture(scope='module')
def setup():
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    created = not dist.is_initialized()
    if created:
        import socket
        with socket.socket() as s:
            s.bind(('127.0.0.1', 0))
            port = s.getsockname()[1]
        dist.init_process_group('gloo', rank=0, world_size=1, init_method=f'tcp://127.0.0.1:{port}')
    from deepep_amd import ElasticBuffer
    from tests.oracle_kernels import OracleKernels
    g = torch.Generator().manual_seed(3)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K, explicitly_destroy=True)
    buf._kernels = OracleKernels()
    idx = torch.topk(torch.rand((T, E), generator=g), K, dim=-1)[1].to(torch.int64)
    w = torch.rand((T, K), generator=g)
    x = torch.randn((T, H), generator=g).to(torch.bfloat16)
    ex_x, _, ex_w, ex_h, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    rx, _, rw, h, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E)
    yield dict(buf=buf, ex_x=ex_x, ex_w=ex_w, ex_h=ex_h, rx=rx, rw=rw, h=h)
    buf.destroy()
    if created:
        dist.destroy_process_group()


def _raises(fn, text):
    with pytest.raises(RuntimeError, match='Assertion failed: .*' + text):
        fn()


def test_each_check_raises_runtime_error(setup):
    b, ex_x, ex_w, ex_h, rx, rw, h = (setup[k] for k in ('buf', 'ex_x', 'ex_w', 'ex_h', 'rx', 'rw', 'h'))
    _raises(lambda: b.combine(ex_x.float(), ex_h), 'contiguous bf16')                       # dtype
    _raises(lambda: b.combine(ex_x.t(), ex_h), 'contiguous bf16')                           # layout
    _raises(lambda: b.combine(ex_x[:, :12].contiguous(), ex_h), 'multiple of 16')           # hidden * 2 % 16
    _raises(lambda: b.combine(rx[:-1].contiguous(), h, topk_weights=rw[:-1]), 'one row per received token')
    _raises(lambda: b.combine(ex_x, ex_h, topk_weights=ex_w[:-1].contiguous()), r'expanded weights are \[N\]')
    _raises(lambda: b.combine(rx, h, topk_weights=rw[:, :K - 1].contiguous()), r'weights are \[N, K\]')
    _raises(lambda: b.combine(ex_x, ex_h, topk_weights=ex_w.double()), 'float32')
    _raises(lambda: b.combine(ex_x, ex_h, bias=torch.zeros((T + 1, H), dtype=torch.bfloat16)), 'bias must be')
    _raises(lambda: b.combine(ex_x, ex_h, bias=(torch.zeros((T, H), dtype=torch.bfloat16),
                                                torch.zeros((T, H), dtype=torch.float32))), 'bias must be')
    _raises(lambda: b.combine(rx, h, topk_weights=rw, apply_topk_weights=True), 'apply_topk_weights needs')
    _raises(lambda: b.combine(ex_x, ex_h, apply_topk_weights=True), 'apply_topk_weights needs')
    _raises(lambda: b.combine(ex_x, ex_h, num_qps=b.num_allocated_qps + 1), 'QPs')


def test_a_valid_call_after_rejected_ones(setup):
    b, ex_x, ex_w, ex_h, rx, rw, h = (setup[k] for k in ('buf', 'ex_x', 'ex_w', 'ex_h', 'rx', 'rw', 'h'))
    with pytest.raises(RuntimeError):
        b.combine(ex_x.float(), ex_h)
    out_e, w_e, _ = b.combine(ex_x, ex_h, topk_weights=ex_w)
    out_r, w_r, _ = b.combine(rx, h, topk_weights=rw)
    assert out_e.shape == (T, H) and torch.equal(w_e, w_r)
    assert torch.isfinite(out_e.float()).all()
