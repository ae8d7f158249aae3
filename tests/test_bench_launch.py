"""bench.py launches and verifies its own ranks: `python bench.py --gpus N` (the driver's command form)
starts N rank processes itself, as the reference's harness spawns its ranks
(/root/reference tests/elastic/test_ep.py:568,609), and every rank checks the world it joined.  CPU
only: gloo, `--launch-check` (the world is formed and verified exactly as in a measured run, nothing
is measured)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, 'bench.py')


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_PORT') and not k.startswith('TORCHELASTIC_')}
    env.update(DEEPEP_BENCH_BACKEND='gloo', MASTER_ADDR='127.0.0.1')
    env.update(kw)
    return env


def _run(args, env, timeout=180):
    return subprocess.run([sys.executable, BENCH, *args], env=env, cwd='/tmp', capture_output=True, text=True,
                          timeout=timeout)


def _line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize('n', [2, 4])
def test_plain_command_launches_n_ranks(n):
    """`python bench.py --gpus N` with no launcher: N distinct rank processes form one world of N."""
    res = _run(['--gpus', str(n), '--launch-check'], _env())
    assert res.returncode == 0, res.stderr[-2000:]
    line = _line(res.stdout)
    assert line['n_gpus'] == n and line['world_size_seen'] == n
    assert line['distinct_rank_processes'] == n
    assert line['launcher'] == 'bench.py'


def test_torchrun_form_still_works():
    res = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                          '--master-addr', '127.0.0.1', '--master-port', '29731', BENCH, '--gpus', '2',
                          '--launch-check'], env=_env(), cwd='/tmp', capture_output=True, text=True, timeout=180)
    assert res.returncode == 0, res.stderr[-2000:]
    line = _line(res.stdout)
    assert line['n_gpus'] == 2 and line['launcher'] == 'external'


def test_world_mismatch_under_a_launcher_fails():
    """torchrun starts 2 ranks but the command says --gpus 4: every rank refuses, exit != 0."""
    res = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                          '--master-addr', '127.0.0.1', '--master-port', '29733', BENCH, '--gpus', '4',
                          '--launch-check'], env=_env(), cwd='/tmp', capture_output=True, text=True, timeout=180)
    assert res.returncode != 0
    assert 'launcher started 2 ranks' in res.stderr
    assert not [ln for ln in res.stdout.splitlines() if ln.startswith('{')]


def test_one_process_world_with_gpus_gt_1_fails():
    """A rank that was told it is a world of one (RANK=0, WORLD_SIZE=1) but --gpus 2: refused."""
    res = _run(['--gpus', '2', '--launch-check'], _env(RANK='0', WORLD_SIZE='1', MASTER_PORT='29735'))
    assert res.returncode != 0
    assert 'world of one' in res.stderr


def test_rccl_needs_n_visible_gpus():
    """Over RCCL every rank needs its own GPU: with none visible the ranks refuse and the launcher
    returns their non-zero status."""
    res = _run(['--gpus', '2', '--launch-check'], _env(DEEPEP_BENCH_BACKEND='nccl', HIP_VISIBLE_DEVICES=''))
    assert res.returncode != 0
    assert 'visible GPUs' in res.stderr


def test_bad_gpu_count_fails():
    res = _run(['--gpus', '0', '--launch-check'], _env())
    assert res.returncode != 0
