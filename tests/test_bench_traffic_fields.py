"""bench.py's N > 1 line states the step's HBM bytes per rank by transport (phases.hbm_bytes_per_rank), from the
same-build PMC passes folded by tools/summarize_prof.py stepfold -- and reports nothing for another build's
counters.  CPU only."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_stepfold_and_bench_field(tmp_path, monkeypatch):
    import bench
    step = {'build_id': 'abcd', 'step_bytes': 8e9,
            'kernels': {'phase_a': {'read_bytes_per_step': 3e9, 'write_bytes_per_step': 2e9},
                        'phase_b': {'read_bytes_per_step': 1e9, 'write_bytes_per_step': 0.5e9},
                        'exchange': {'read_bytes_per_step': 0.75e9, 'write_bytes_per_step': 0.75e9}},
            'meta': {'world': 2, 'tokens': 8192, 'hidden': 7168, 'topk': 8, 'local_bypass': True,
                     'b_bytes': [1e9, 1e9]}}
    sj, tj = tmp_path / 'step.json', tmp_path / 'traffic.json'
    sj.write_text(json.dumps(step))
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'summarize_prof.py'), 'stepfold', str(tj), str(sj)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    entry = json.loads(tj.read_text())['step_ep2_t8192_h7168_k8']
    h = entry['hbm_bytes_per_rank']
    assert h['rccl'] == 4e9 and h['xgmi'] == 3.25e9 and h['algorithmic'] == 1e9
    monkeypatch.setattr(bench, '_pmc_entry', lambda w: entry if w == 'step_ep2_t8192_h7168_k8' else {})
    got = bench._hbm_bytes_per_rank(2, 8192, 7168, 8, 'abcd')
    assert got['rccl'] == 4e9 and got['xgmi'] == 3.25e9 and got['build_id'] == 'abcd'
    stale = bench._hbm_bytes_per_rank(2, 8192, 7168, 8, 'other')
    assert stale['rccl'] is None and 'stale' in stale['note']
    assert bench._hbm_bytes_per_rank(4, 8192, 7168, 8, 'abcd')['rccl'] is None
