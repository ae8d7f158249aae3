"""Small integer helpers (deep_ep/utils/math.py:17-27, deep_ep/utils/semantic.py in the reference)."""


def ceil_div(x: int, y: int) -> int:
    return (x + y - 1) // y


def align(x: int, y: int) -> int:
    return ceil_div(x, y) * y


def value_or(value, default):
    return default if value is None else value


def check_torch_deterministic() -> None:
    """deep_ep/utils/envs.py:183-189: deterministic algorithms together with fill_uninitialized_memory make
    torch.empty launch a fill kernel that may overlap the communication streams; the reference refuses the
    combination in dispatch and combine (elastic.py:924, :1083) with a plain `assert`, so this build raises
    the same exception type, AssertionError -- explicitly, so that `python -O` does not strip it."""
    import torch
    if torch.are_deterministic_algorithms_enabled() and torch.utils.deterministic.fill_uninitialized_memory:
        raise AssertionError('deterministic algorithms with fill_uninitialized_memory would launch fill kernels '
                             'that overlap the communication streams; disable one of them')
