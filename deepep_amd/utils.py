"""Small integer helpers (deep_ep/utils/math.py:17-27, deep_ep/utils/semantic.py in the reference)."""


def ceil_div(x: int, y: int) -> int:
    return (x + y - 1) // y


def align(x: int, y: int) -> int:
    return ceil_div(x, y) * y


def value_or(value, default):
    return default if value is None else value
