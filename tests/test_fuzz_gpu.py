"""Randomised EP = 1 parity sweep on the GPU: ElasticBuffer dispatch + combine over seeded random
shapes (ragged hidden sizes, top-k 1..16, expert counts, masked slots, empty batches), every
combine flavour (expanded / non-expanded, multiple / single reduction, plain / gating-weighted,
bias 0/1/2) against the oracle, bitwise.  Mirrors the reference's mode matrix
(tests/elastic/test_ep.py:22-31) on shapes its fixed configs do not reach."""
import os

import numpy as np
import pytest
import torch

import oracle
from tests.test_buffer_cpu import _weighted_single

pytestmark = pytest.mark.gpu

HIDDENS = [8, 64, 520, 1024, 2056, 4104, 7168]
TOPKS = [1, 2, 3, 4, 6, 8, 12, 16]


def _u16(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().contiguous().view(torch.int16).numpy().view(np.uint16)


def _bf16(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.bfloat16).cuda()


def _case(seed: int):
    rng = np.random.default_rng(seed)
    T = int(rng.choice([0, 1, 7, 64, 129, 300]))
    H = int(rng.choice(HIDDENS))
    K = int(rng.choice(TOPKS))
    E = int(K * rng.integers(1, 9))
    masked = float(rng.choice([0.0, 0.1, 0.4]))
    return rng, T, H, K, E, masked


@pytest.fixture(scope='module')
def group():
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29547')
        dist.init_process_group('gloo', rank=0, world_size=1)
    return dist.group.WORLD


@pytest.mark.parametrize('seed', range(24))
def test_random_shapes_ep1(group, seed):
    from deepep_amd import ElasticBuffer
    rng, T, H, K, E, masked = _case(seed)
    idx = np.array([rng.permutation(E)[:K] for _ in range(T)], dtype=np.int64).reshape(T, K)
    idx[rng.random((T, K)) < masked] = -1
    w = (rng.random((T, K)).astype(np.float32) * (idx >= 0)).astype(np.float32)
    biases = [oracle.f32_to_bf16(rng.standard_normal((T, H)).astype(np.float32)) for _ in range(2)]
    T_max = max(T, 1)
    x = torch.zeros((T, H), dtype=torch.bfloat16, device='cuda')
    g_idx, g_w = torch.from_numpy(idx).cuda(), torch.from_numpy(w).cuda()
    failures = []
    for amr in (True, False):
        buf = ElasticBuffer(group, num_max_tokens_per_rank=T_max, hidden=H, num_topk=K, allow_multiple_reduction=amr)
        _, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=g_idx, topk_weights=g_w, num_experts=E,
                                             num_max_tokens_per_rank=T_max, do_expand=True)
        meta = handle.recv_src_metadata.cpu().numpy()
        n_exp = handle.num_expanded_tokens
        y = oracle.f32_to_bf16((rng.standard_normal((n_exp, H)) * rng.choice([1e-2, 1.0, 50.0])).astype(np.float32))
        # the token-major view of the same rows: y3[t, k] = y[slot of (t, k)]
        y3 = np.zeros((T, K, H), np.uint16)
        for i in range(meta.shape[0]):
            for k in range(K):
                if meta[i, 2 + k] >= 0:
                    y3[meta[i, 0] % T_max, k] = y[meta[i, 2 + k]]
        for nb in (0, 1, 2):
            b = [biases[0] if nb >= 1 else None, biases[1] if nb >= 2 else None]
            g_bias = None if nb == 0 else (_bf16(b[0]) if nb == 1 else (_bf16(b[0]), _bf16(b[1])))
            for weighted in (False, True):
                out, out_w, _ = buf.combine(_bf16(y), handle, topk_weights=ex_w if (weighted or amr) else None,
                                            bias=g_bias, apply_topk_weights=weighted)
                torch.cuda.synchronize()
                if amr:
                    part, _ = oracle.phase_a(y, meta, K, True, ex_w.cpu().numpy(), weighted=weighted)
                    recv = np.zeros((1, T_max, H), np.uint16)
                    recv[0, meta[:, 0] % T_max] = part
                    exp, _ = oracle.phase_b(recv, None, idx, E, 1, True, True, b[0], b[1])
                elif weighted:
                    cb = None if nb == 0 else (torch.from_numpy(b[0].view(np.int16)).view(torch.bfloat16) if nb == 1
                                               else tuple(torch.from_numpy(v.view(np.int16)).view(torch.bfloat16)
                                                          for v in b))
                    exp = _u16(_weighted_single(y3, torch.from_numpy(idx), torch.from_numpy(w), cb))
                else:
                    exp = oracle.combine_ep([y], [meta], [idx], E, T_max, expanded=True,
                                            allow_multiple_reduction=False, bias_per_rank=[tuple(b)])[0][0][:T]
                if not np.array_equal(_u16(out), exp):
                    failures.append(f'amr={amr} nb={nb} weighted={weighted}')
                if out_w is not None and not np.array_equal(out_w.cpu().numpy(), w):
                    failures.append(f'weights amr={amr} nb={nb} weighted={weighted}')
        if amr:
            # non-expanded: the caller pre-reduced its local experts; the combine copies/epilogues
            _, _, recv_w, nh, _ = buf.dispatch(x, topk_idx=g_idx, topk_weights=g_w, num_experts=E,
                                               num_max_tokens_per_rank=T_max)
            n = nh.num_recv_tokens
            x_red = oracle.f32_to_bf16(rng.standard_normal((n, H)).astype(np.float32))
            out, out_w, _ = buf.combine(_bf16(x_red), nh, topk_weights=recv_w, bias=_bf16(biases[0]) if T else None)
            torch.cuda.synchronize()
            recv = np.zeros((1, T_max, H), np.uint16)
            recv[0, nh.recv_src_metadata.cpu().numpy()[:n, 0] % T_max] = x_red
            exp, _ = oracle.phase_b(recv, None, idx, E, 1, True, True, biases[0] if T else None)
            if not np.array_equal(_u16(out), exp):
                failures.append('non-expanded')
            if not np.array_equal(out_w.cpu().numpy(), w):
                failures.append('non-expanded weights')
    assert not failures, (seed, T, H, K, E, masked, failures)
