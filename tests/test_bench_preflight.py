"""bench.py's xGMI preflight (xgmi_preflight.py run as a child before the bench touches the GPU):
a child that cannot run reports ok=False with its error instead of raising or hanging, and the
line's xGMI legs are then skipped.  CPU: the child finds no GPU and fails on purpose."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(torch.cuda.is_available(), reason='the child must fail: CPU-only check')
def test_preflight_failure_is_reported(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv('RANK', '0')
    monkeypatch.setenv('WORLD_SIZE', '1')
    monkeypatch.setenv('MASTER_PORT', '29871')
    monkeypatch.setenv('TORCHELASTIC_USE_AGENT_STORE', 'True')     # must not reach the child
    res = bench._xgmi_preflight()
    assert res['ok'] is False
    assert res['exit_status'] == 1
    assert res['error']
    assert res['rank'] == 0 and res['world'] == 1
