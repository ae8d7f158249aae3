"""Synthetic inputs of the BASELINE configurations -- used by bench.py and the tests, not by the
product package (deepep_amd/).

Restatements of the reference's input utilities (paths in /root/reference):
  per_token_cast_to_fp8 / per_token_cast_back   deep_ep/utils/math.py:30-57  (config 4's FP8 dispatch)
  get_unbalanced_scores                         deep_ep/utils/gate.py:140-180 (config 5's skewed routing)
  calc_diff                                     deep_ep/utils/math.py:5-9
"""


def _align(x: int, y: int) -> int:
    return (x + y - 1) // y * y



def calc_diff(x, y) -> float:
    """1 - similarity of x+1 and y+1 (deep_ep/utils/math.py:5-9)."""
    x, y = x.double() + 1, y.double() + 1
    denominator = (x * x + y * y).sum()
    return (1 - 2 * (x * y).sum() / denominator).item()


def per_token_cast_to_fp8(x):
    """Per-token, per-128-column e4m3 cast with fp32 scales (deep_ep/utils/math.py:30-39)."""
    import torch
    assert x.dim() == 2
    m, n = x.shape
    aligned_n = _align(n, 128)
    x_padded = torch.nn.functional.pad(x, (0, aligned_n - n), mode='constant', value=0)
    view = x_padded.view(m, -1, 128)
    amax = view.abs().float().amax(dim=2).view(m, -1).clamp(1e-4)
    q = (view * (448.0 / amax.unsqueeze(2))).to(torch.float8_e4m3fn).view(m, aligned_n)[:, :n].contiguous()
    return q, (amax / 448.0).view(m, -1)


def per_token_cast_back(x_fp8, x_scales):
    """Inverse of per_token_cast_to_fp8 (deep_ep/utils/math.py:42-57)."""
    import torch
    m, n = x_fp8.shape
    aligned_n = _align(n, 128)
    padded = torch.nn.functional.pad(x_fp8, (0, aligned_n - n), mode='constant', value=0)
    x32 = padded.to(torch.float32).view(m, -1, 128)
    return (x32 * x_scales.view(m, -1, 1)).view(m, aligned_n).to(torch.bfloat16)[:, :n].contiguous()


def _scores_by_factor(num_tokens, num_experts, num_ranks, factor, device):
    import torch
    epr = num_experts // num_ranks
    scores = torch.empty((num_tokens, num_experts), dtype=torch.float32, device=device)
    scores[:, :epr].uniform_(to=factor)
    scores[:, epr:].uniform_(to=1)
    return scores


def get_unbalanced_scores(num_tokens: int, num_experts: int, num_ranks: int, num_topk: int, ratio: float,
                          device='cuda'):
    """Routing scores where rank 0's experts receive `ratio` x the tokens of the other ranks
    (get_random_unbalanced_scores + map_unbalanced_ratio_to_factor, deep_ep/utils/gate.py:143-180)."""
    import torch
    factor = 1.0
    if ratio != 1.0:
        lo, hi = 1.0, 100.0
        epr = num_experts // num_ranks
        for _ in range(20):
            mid = (lo + hi) / 2
            s = _scores_by_factor(num_tokens, num_experts, num_ranks, mid, device)
            _, idx = torch.topk(s, num_topk, dim=-1, largest=True, sorted=False)
            counts = torch.nn.functional.one_hot(idx // epr, num_ranks).any(dim=1).to(torch.float).sum(dim=0)
            if counts[0].item() > counts[1:].mean().item() * ratio:
                hi = mid
            else:
                lo = mid
        factor = lo
    return _scores_by_factor(num_tokens, num_experts, num_ranks, factor, device)
