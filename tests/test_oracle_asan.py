"""The host-side sanitizer pass ("build with -fsanitize=address for the host
path"; the reference has none): the checker oracle/combine_ref.c built with AddressSanitizer and
UndefinedBehaviorSanitizer (`make -C oracle asan`, every UB report fatal) runs the oracle's own CPU
suites -- the golden vectors of refs.py (tests/test_oracle_golden.py) and the one-rank restatement
(tests/test_oracle_one_rank.py) -- in a child python with the ASan runtime preloaded.  An
out-of-bounds index in the checker would abort that child.  A canary library with a deliberate heap
overflow, built with the same flags, shows that the preloaded runtime does catch a bad access in a
ctypes-loaded library under this setup."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SANFLAGS = ['-O1', '-g', '-std=c11', '-fPIC', '-fno-omit-frame-pointer', '-fsanitize=address,undefined',
            '-fno-sanitize-recover=undefined']


def _asan_runtime() -> str:
    path = subprocess.run(['gcc', '-print-file-name=libasan.so'], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(path) or not os.path.exists(path):
        pytest.skip('gcc has no ASan runtime here')
    return path


def _env() -> dict:
    env = dict(os.environ)
    # the ASan runtime must come first in the initial library list; whatever else the environment
    # preloads stays after it
    env['LD_PRELOAD'] = ':'.join(p for p in (_asan_runtime(), os.environ.get('LD_PRELOAD', '')) if p)
    env['ASAN_OPTIONS'] = 'detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=86'
    env['UBSAN_OPTIONS'] = 'halt_on_error=1:print_stacktrace=1'
    env['DEEPEP_ORACLE_LIB'] = 'asan'
    env['PYTHONPATH'] = ROOT
    return env


def test_asan_runtime_catches_an_overflow_in_a_loaded_library(tmp_path):
    so = tmp_path / 'libcanary.so'
    subprocess.run(['gcc', *SANFLAGS, '-shared', '-o', str(so), os.path.join(ROOT, 'tests', 'asan', 'canary.c')],
                   check=True)
    code = f'import ctypes; print(ctypes.CDLL({str(so)!r}).canary_overflow(16))'
    res = subprocess.run([sys.executable, '-c', code], env=_env(), capture_output=True, text=True, timeout=120)
    assert res.returncode == 86, (res.returncode, res.stderr[-2000:])
    assert 'heap-buffer-overflow' in res.stderr


def test_sanitized_oracle_passes_golden_and_one_rank_suites():
    subprocess.run(['make', '-s', '-C', os.path.join(ROOT, 'oracle'), 'asan'], check=True)
    code = (
        'import sys, pytest\n'
        f'rc = pytest.main(["-q", "-x", "-p", "no:cacheprovider", {os.path.join(ROOT, "tests", "test_oracle_golden.py")!r},'
        f' {os.path.join(ROOT, "tests", "test_oracle_one_rank.py")!r}])\n'
        'import oracle\n'
        'maps = open("/proc/self/maps").read()\n'
        'print("LOADED", oracle.loaded_library(), "liboracle_asan.so" in maps, "libasan" in maps)\n'
        'sys.exit(int(rc))\n')
    res = subprocess.run([sys.executable, '-c', code], env=_env(), capture_output=True, text=True, timeout=900,
                         cwd=ROOT)
    assert res.returncode == 0, (res.returncode, res.stdout[-3000:], res.stderr[-3000:])
    loaded = [ln for ln in res.stdout.splitlines() if ln.startswith('LOADED')]
    assert loaded and loaded[-1].endswith('liboracle_asan.so True True'), res.stdout[-2000:]
    assert 'passed' in res.stdout and 'failed' not in res.stdout
