"""The N > 1 bench's safety net (bench.py `_Line`): a secondary leg that hangs on a real node must not cost
the line.  At the hard deadline the watchdog prints the line built so far -- with `incomplete` naming the
leg that was running and `skipped_legs` -- and ends the rank with status 0; the line is printed once even if
the run then finishes normally.  A leg that raises still prints the line (then the error propagates).
CPU only (no GPU is touched)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r'''
import sys, time
sys.path.insert(0, {root!r})
import bench
bench.HARD_DEADLINE_S = {deadline}
line = bench._Line(0)
line.fields = {{'metric': 'm', 'value': 1.0, 'launch': {{'world_size_seen': 2}}}}
line.skipped.append('dispatch_sync_free (soft budget 300 s spent)')
line.leg = 'xgmi'
line.start_watchdog()
time.sleep({sleep})
line.emit()
print('normal end', flush=True)
'''


def _run(deadline: float, sleep: float):
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, '-c', _SCRIPT.format(root=ROOT, deadline=deadline, sleep=sleep)],
                       capture_output=True, text=True, timeout=120)
    return r, time.perf_counter() - t0


def test_watchdog_emits_the_partial_line_and_exits_zero():
    r, el = _run(deadline=3.0, sleep=60)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1 and 'normal end' not in r.stdout, r.stdout
    d = json.loads(lines[0])
    assert d['value'] == 1.0 and 'xgmi' in d['incomplete'] and d['skipped_legs'], d
    assert d['launch']['world_size_seen'] == 2 and 'wall_s' in d['launch']
    assert el < 60, el                                       # ended at the deadline, not after the hang


def test_line_is_printed_once_when_the_run_finishes_first():
    r, _ = _run(deadline=30.0, sleep=0.1)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1 and 'incomplete' not in json.loads(lines[0]) and 'normal end' in r.stdout


_RAISE = r'''
import sys
sys.path.insert(0, {root!r})
import bench

def fake_main():
    line = bench._Line(0)
    bench._LINE[0] = line
    line.fields = {{'metric': 'm', 'value': 2.0, 'launch': {{}}}}
    line.leg = 'dispatch'
    raise RuntimeError('boom')

bench.main = fake_main
bench._entry()
'''


def test_a_leg_that_raises_still_prints_the_line():
    r = subprocess.run([sys.executable, '-c', _RAISE.format(root=ROOT)], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and 'RuntimeError: boom' in r.stderr, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d['value'] == 2.0 and 'dispatch' in d['incomplete'] and 'boom' in d['incomplete'], d
