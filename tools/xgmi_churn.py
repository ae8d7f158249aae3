"""Back-to-back runs of the config-3 xGMI test body (tests/test_xgmi_gpu.py::_full_worker): 8 fresh
processes per run, started as soon as the previous 8 have exited.  Checks whether the test's rare
failures need the process churn of the preceding multi-process tests.  Env: XCHURN_RUNS (default 5),
XCHURN_GAP (seconds to wait between runs, default 0)."""
import json
import os
import sys
import time

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from tests.test_xgmi_gpu import _free_port, _full_worker
    runs = int(os.environ.get('XCHURN_RUNS', 5))
    gap = float(os.environ.get('XCHURN_GAP', 0))
    ctx = mp.get_context('spawn')
    for i in range(runs):
        queue = ctx.Queue()
        port = _free_port()
        t0 = time.time()
        procs = [ctx.Process(target=_full_worker, args=(r, 8, port, queue)) for r in range(8)]
        for p in procs:
            p.start()
        results = {}
        try:
            for _ in range(8):
                rank, failures = queue.get(timeout=150)
                results[rank] = failures
                if failures:
                    break
        except Exception as e:  # noqa: BLE001
            results['timeout'] = [repr(e)]
        finally:
            for p in procs:
                p.join(timeout=30)
                if p.is_alive():
                    p.kill()
        bad = {r: [f[-600:] for f in fl] for r, fl in results.items() if fl}
        print(json.dumps(dict(run=i, seconds=round(time.time() - t0, 1), reported=len(results), bad=bad)), flush=True)
        if gap:
            time.sleep(gap)


if __name__ == '__main__':
    main()
