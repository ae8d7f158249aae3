"""The C-ABI from plain C: tests/abi_c/combine_abi (built by __graft_entry__.build()) allocates
with hipMalloc, builds the slot plan from handle metadata, runs the fused combine (plain, bias,
gating-weighted, weight pass-through) and compares every bit with the oracle; no Python or torch
in the process."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, 'tests', 'abi_c', 'combine_abi')


@pytest.mark.gpu
def test_c_consumer_bitwise():
    if not os.path.exists(BIN):                 # normally built by __graft_entry__.build(); gcc, < 1 s
        import __graft_entry__ as g
        subprocess.run(g.C_CONSUMER_CMD, check=True, timeout=60)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith('PASS')
