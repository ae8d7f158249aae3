"""The reference's pressure test (tests/elastic/test_ep.py:548-557, `--do-pressure-test`: loop over seeds,
optionally recreating the buffer), on one GPU: 12 seeds, each with a NEW ElasticBuffer (explicitly destroyed
afterwards), a fresh dispatch and the gating-weighted and plain combines bitwise against the oracle; then the
same seeds through ONE buffer.  Nothing may leak: after every destroyed buffer and its tensors are gone, the
allocator's allocated bytes return to where the first iteration left them."""
import gc
import os

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

T, H, K, E = 512, 2048, 8, 64


@pytest.fixture(scope='module')
def group():
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29561')
        dist.init_process_group('gloo', rank=0, world_size=1)
    return dist.group.WORLD


def _u16(t):
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _one_seed(buf, seed):
    g = torch.Generator(device='cuda').manual_seed(seed)
    idx = torch.topk(torch.rand((T, E), device='cuda', generator=g), K, dim=-1, sorted=False)[1].to(torch.int64)
    idx[torch.rand((T, K), device='cuda', generator=g) < 0.05] = -1
    w = torch.rand((T, K), device='cuda', generator=g)
    x = torch.randn((T, H), device='cuda', generator=g).to(torch.bfloat16)
    _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=idx, topk_weights=w, num_experts=E, do_expand=True)
    y = torch.randn((handle.num_expanded_tokens, H), device='cuda', generator=g).to(torch.bfloat16)
    out_w, _, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=True)
    out_p, pass_w, _ = buf.combine(y, handle, topk_weights=ex_w)
    torch.cuda.synchronize()
    meta, yy, ew = handle.recv_src_metadata.cpu().numpy(), _u16(y), ex_w.cpu().numpy()
    i = idx.cpu().numpy()
    bad = []
    for weighted, out in ((True, out_w), (False, out_p)):
        part, _ = oracle.phase_a(yy, meta, K, True, ew, weighted=weighted)
        recv = np.zeros((1, T, H), np.uint16)
        recv[0, meta[:, 0] % T] = part
        exp, _ = oracle.phase_b(recv, None, i, E, 1, True, True)
        if not np.array_equal(_u16(out), exp):
            bad.append(f'seed {seed} weighted={weighted}')
    if not torch.equal(pass_w, torch.where(idx >= 0, w, torch.zeros_like(w))):
        bad.append(f'seed {seed} weight pass-through')
    return bad


def test_pressure_recreating_the_buffer(group):
    from deepep_amd import ElasticBuffer
    bad, base = [], None
    for seed in range(12):
        buf = ElasticBuffer(group, num_max_tokens_per_rank=T, hidden=H, num_topk=K, explicitly_destroy=True)
        bad += _one_seed(buf, seed)
        buf.destroy()
        del buf
        gc.collect()
        torch.cuda.synchronize()
        # the first iteration may leave process-wide state (the library's error records, cached streams): the
        # allocated bytes after it are the baseline every later iteration must come back to
        if base is None:
            base = torch.cuda.memory_allocated()
        assert torch.cuda.memory_allocated() == base, (seed, torch.cuda.memory_allocated() - base)
    assert not bad, bad


def test_pressure_one_buffer(group):
    from deepep_amd import ElasticBuffer
    buf = ElasticBuffer(group, num_max_tokens_per_rank=T, hidden=H, num_topk=K, explicitly_destroy=True)
    bad = []
    for seed in range(100, 112):
        bad += _one_seed(buf, seed)
    buf.destroy()
    assert not bad, bad
