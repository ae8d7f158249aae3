"""The N > 1 headline survives an RCCL failure: before touching the GPU every rank runs
rccl_preflight.py and xgmi_preflight.py as children, the ranks agree on the verdicts over a TCP store
(MASTER_PORT + 3) and bench.py picks the headline transport -- RCCL when every rank's RCCL preflight passed,
else the xGMI windows when every xGMI preflight passed, else the all-to-all through host memory over gloo --
naming it in config.transport with the preflight errors in the line.  CPU only: `--preflight-check` runs
exactly that selection and prints its fields; with no GPU both preflights fail, as they would on a broken node.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, 'bench.py')
sys.path.insert(0, ROOT)


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_PORT') and not k.startswith('TORCHELASTIC_')}
    env.update(MASTER_ADDR='127.0.0.1', HIP_VISIBLE_DEVICES='')
    env.update(kw)
    return env


def _check(n: int, **env):
    r = subprocess.run([sys.executable, BENCH, '--gpus', str(n), '--preflight-check'], env=_env(**env), cwd='/tmp',
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_choose_headline_every_case():
    import bench
    assert bench._choose_headline('nccl', True, True)['label'] == 'rccl'
    assert bench._choose_headline('nccl', True, False) == dict(
        backend='nccl', transport='rccl', label='rccl', reason='rccl_preflight passed on every rank')
    h = bench._choose_headline('nccl', False, True)
    assert (h['backend'], h['transport'], h['label']) == ('gloo', 'xgmi', 'xgmi') and 'rccl_preflight failed' in h['reason']
    h = bench._choose_headline('nccl', False, False)
    assert (h['backend'], h['transport'], h['label']) == ('gloo', 'rccl', 'gloo-host-exchange')
    h = bench._choose_headline('gloo', None, True)
    assert h['label'] == 'gloo-host-exchange' and 'rehearsal' in h['reason']


def test_rccl_failure_falls_back_and_reports():
    """Default backend (RCCL): the RCCL children fail (here: no GPU), so does xGMI -> the marked gloo line,
    with each preflight's error in it."""
    d = _check(2, DEEPEP_BENCH_BACKEND='nccl')
    assert d['headline_transport']['backend'] == 'gloo'
    assert d['config']['transport'] == 'gloo-host-exchange'
    rp = d['rccl_preflight']
    assert rp['ok'] is False and rp['all_ranks_ok'] is False and rp['error'] and rp['exit_status'] == 1
    xp = d['xgmi_preflight']
    assert xp['ok'] is False and xp['all_ranks_ok'] is False and xp['error']


def test_injected_rccl_failure_is_named():
    d = _check(2, DEEPEP_BENCH_BACKEND='nccl', DEEPEP_BENCH_FAIL_RCCL_PREFLIGHT='1', DEEPEP_BENCH_XGMI='0')
    assert 'failure injected' in d['rccl_preflight']['error']
    assert d['xgmi_preflight'] is None                      # DEEPEP_BENCH_XGMI=0: not run
    assert d['config']['transport'] == 'gloo-host-exchange'


def test_gloo_rehearsal_runs_no_rccl_preflight():
    d = _check(2, DEEPEP_BENCH_BACKEND='gloo', DEEPEP_BENCH_XGMI='0')
    assert d['rccl_preflight'] == {'ok': False, 'skipped': 'DEEPEP_BENCH_BACKEND=gloo', 'all_ranks_ok': False,
                                   'agreement': 'store'}
    assert d['config']['transport'] == 'gloo-host-exchange'


def test_torchrun_agreement_uses_the_agent_store():
    """Under torchrun (the driver's N > 1 form) the ranks agree through the launcher's own store."""
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                        '--master-addr', '127.0.0.1', '--master-port', '29741', BENCH, '--gpus', '2',
                        '--preflight-check'], env=_env(DEEPEP_BENCH_BACKEND='nccl', DEEPEP_BENCH_XGMI='0',
                                                       DEEPEP_BENCH_FAIL_RCCL_PREFLIGHT='1'),
                       cwd='/tmp', capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{')][-1])
    assert d['rccl_preflight']['agreement'] == 'store' and d['rccl_preflight']['all_ranks_ok'] is False
    assert d['config']['transport'] == 'gloo-host-exchange'


def test_failed_agreement_falls_back_to_the_default(monkeypatch):
    import bench

    def broken(*a, **k):
        raise RuntimeError('store unreachable')
    monkeypatch.setattr(bench, '_agree', broken)
    got = bench._agree_or_default({'rccl': False, 'xgmi': True}, 0, 2)
    assert got['rccl'] is True and got['xgmi'] is False and 'store unreachable' in got['agreement']


_AGREE = r'''
import os, sys, json
sys.path.insert(0, {root!r})
import bench
rank = int(sys.argv[1])
os.environ['MASTER_ADDR'] = '127.0.0.1'
os.environ['MASTER_PORT'] = sys.argv[2]
flags = {{'rccl': rank != 1, 'xgmi': True}}          # rank 1's RCCL preflight failed
print(json.dumps(bench._agree(flags, rank, 3)), flush=True)
'''


def test_agreement_is_the_and_over_ranks():
    import bench
    port = bench._free_port_pair()
    procs = [subprocess.Popen([sys.executable, '-c', _AGREE.format(root=ROOT), str(r), str(port)],
                              stdout=subprocess.PIPE, text=True) for r in range(3)]
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    for o in outs:
        assert json.loads(o.strip().splitlines()[-1]) == {'rccl': False, 'xgmi': True}


def test_headline_hang_still_leaves_a_line():
    """N > 1: the watchdog starts before the headline; a line built from the preflights alone has value null."""
    import bench
    line = bench._Line(0)
    line.fields = {'metric': 'm', 'value': None, 'launch': {}}
    line.leg = 'headline'
    import io
    import contextlib
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        line.emit(incomplete='hard deadline hit during leg "headline"')
    d = json.loads(buf.getvalue())
    assert d['value'] is None and 'headline' in d['incomplete']


def test_a_hanging_preflight_child_is_killed_and_reported(tmp_path, monkeypatch):
    """A preflight child that never finishes (a hung collective) is killed at the limit: ok=False with
    the reason, no exception, and the bench goes on."""
    import bench
    script = tmp_path / 'hang.py'
    script.write_text('import time\ntime.sleep(600)\n')
    monkeypatch.setattr(bench, 'ROOT', str(tmp_path))
    c = bench._start_child('hang.py', 1)
    res = bench._finish_child(c, limit=2.0)
    assert res['ok'] is False and 'timed out' in res['error']
    assert c['proc'].poll() is not None                   # the child is gone


def test_a_crashing_preflight_child_reports_its_last_stderr_line(tmp_path, monkeypatch):
    import bench
    script = tmp_path / 'crash.py'
    script.write_text('import sys\nprint("diagnostic", file=sys.stderr)\nraise SystemExit(7)\n')
    monkeypatch.setattr(bench, 'ROOT', str(tmp_path))
    res = bench._finish_child(bench._start_child('crash.py', 2), limit=60.0)
    assert res == {'exit_status': 7, 'ok': False, 'error': 'diagnostic'}
