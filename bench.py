"""Benchmark of the combine reduction (BASELINE.json metric: "combine GB/s (device-resident
BF16 top-k weighted reduce) at 1/2/4/8 MI355X").

One step = one ElasticBuffer.combine over one synthetic batch already resident in HBM:
8192 tokens/rank x hidden 7168 x top-8 over 256 experts (BASELINE configs 2 and 3),
expanded layout, gating-weighted (apply_topk_weights=True), weights passed through.
At N = 1 the combine is one fused HIP launch; at N > 1 it is phase A -> exchange over xGMI ->
phase B: `value` is the default RCCL all-to-all transport (pipelined), and the other legs timed on
the same batch (phase A on a CU budget; direct stores into the peers' symmetric windows; the single
reduction) stay beside it in the line, checked bit for bit.

Algorithmic bytes per token: K*H*2 (rows read) + H*2 (row written)
+ K*4 (slot index) + K*4 (fp32 weight), with K = the token's valid top-k slots.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1: `python bench.py --gpus N` starts its own N rank processes (one per GPU, as the reference's
harness spawns its ranks, tests/elastic/test_ep.py:568,609) and relays rank 0's line; under
torch.distributed.run (RANK set) it runs as one of the launched ranks.  Either way every rank checks
that the world it joined has N ranks (and, over RCCL, that N GPUs are visible) and fails otherwise.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def _fail(msg: str, code: int = 3):
    print(f'[bench] {msg}', file=sys.stderr, flush=True)
    sys.exit(code)


# Ports above the ranks' MASTER_PORT P: the xGMI preflight children's gloo world, the RCCL preflight
# children's world, and the store on which the ranks agree on the preflights' verdicts.
PORT_XGMI_PREFLIGHT, PORT_RCCL_PREFLIGHT, PORT_AGREE = 1, 2, 3


def _free_port_pair() -> int:
    """A port P with P .. P + 3 free on 127.0.0.1 (P: the ranks' rendezvous; P + 1 / + 2 / + 3: see
    PORT_XGMI_PREFLIGHT, PORT_RCCL_PREFLIGHT, PORT_AGREE)."""
    import contextlib
    import socket
    for _ in range(64):
        with socket.socket() as a:
            a.bind(('127.0.0.1', 0))
            port = a.getsockname()[1]
            if port + PORT_AGREE > 65535:
                continue
            try:
                with contextlib.ExitStack() as stack:
                    for off in range(1, PORT_AGREE + 1):
                        b = stack.enter_context(socket.socket())
                        b.bind(('127.0.0.1', port + off))
            except OSError:
                continue
            return port
    raise RuntimeError('no free port range on 127.0.0.1')


def _launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes of this script (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT set, rendezvous on 127.0.0.1), relay rank 0's JSON line to
    stdout (everything else to stderr), and return non-zero when any rank fails.  This process never
    touches the GPU and never execs: the ranks are ordinary children.  When one rank fails the others
    get 30 s to finish before they are killed (a peer stuck in a collective would otherwise hang)."""
    import signal
    import subprocess
    import threading
    port = _free_port_pair()
    base = {k: v for k, v in os.environ.items() if not k.startswith('TORCHELASTIC_')}
    base.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                DEEPEP_BENCH_LAUNCHER='bench.py')
    cmd = [sys.executable, '-u', os.path.abspath(__file__), *sys.argv[1:]]
    procs, lines = [], []
    print(f'[bench] launching {n} ranks (rendezvous 127.0.0.1:{port})', file=sys.stderr, flush=True)
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(cmd, env=env, cwd=ROOT, text=True,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))

    def relay():                       # rank 0's stdout: JSON lines kept, the rest to stderr
        for ln in procs[0].stdout:
            if ln.startswith('{'):
                lines.append(ln.rstrip('\n'))
            else:
                sys.stderr.write(ln)
                sys.stderr.flush()
    reader = threading.Thread(target=relay, daemon=True)
    reader.start()

    def kill_all(*_):
        for p in procs:
            if p.poll() is None:
                p.kill()
    old_term = signal.signal(signal.SIGTERM, lambda *a: (kill_all(), sys.exit(143)))
    failed_at = None
    try:
        while any(p.poll() is None for p in procs):
            time.sleep(0.5)
            bad = [p for p in procs if p.poll() not in (None, 0)]
            if bad and failed_at is None:
                failed_at = time.perf_counter()
                print(f'[bench] rank {procs.index(bad[0])} exited with {bad[0].returncode}; waiting 30 s for the '
                      f'others', file=sys.stderr, flush=True)
            if failed_at is not None and time.perf_counter() - failed_at > 30:
                kill_all()
    finally:
        kill_all()
        signal.signal(signal.SIGTERM, old_term)
    reader.join(timeout=10)
    rcs = [p.wait() for p in procs]
    for ln in lines:
        print(ln, flush=True)
    if any(rcs):
        print(f'[bench] rank exit codes {rcs}', file=sys.stderr, flush=True)
        return next(rc for rc in rcs if rc) if all(rc >= 0 for rc in rcs if rc) else 1
    if not lines:
        print('[bench] rank 0 printed no result line', file=sys.stderr, flush=True)
        return 1
    return 0


def _init_dist(n_gpus: int, use_gpu: bool = True, backend: str = None):
    """Join the ranks' process group and check it: the world must have exactly --gpus ranks, and over
    RCCL every rank needs its own GPU.  A mismatch exits non-zero (never a silent one-rank line).
    `backend` (default DEEPEP_BENCH_BACKEND, else nccl): gloo after a failed RCCL preflight."""
    backend = backend or os.environ.get('DEEPEP_BENCH_BACKEND', 'nccl')
    if 'RANK' in os.environ and int(os.environ.get('WORLD_SIZE', '1')) > 1:
        local_rank = int(os.environ.get('LOCAL_RANK', 0))
        world_env = int(os.environ['WORLD_SIZE'])
        if world_env != n_gpus:
            _fail(f'--gpus {n_gpus} but the launcher started {world_env} ranks')
        # DEEPEP_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices)
        if use_gpu:
            n_dev = torch.cuda.device_count()
            if backend == 'nccl' and n_dev < n_gpus:
                _fail(f'--gpus {n_gpus} over RCCL needs {n_gpus} visible GPUs, this node shows {n_dev}')
            dev = local_rank % n_dev
            torch.cuda.set_device(dev)
        if backend == 'nccl' and use_gpu:
            dist.init_process_group('nccl', device_id=torch.device('cuda', dev))
        else:
            dist.init_process_group('gloo')
    else:
        if n_gpus != 1:
            _fail(f'--gpus {n_gpus} needs {n_gpus} rank processes (run `python bench.py --gpus {n_gpus}` or '
                  f'torch.distributed.run --nproc-per-node {n_gpus}); this process is a world of one')
        if use_gpu:
            torch.cuda.set_device(0)
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', str(29500 + os.getpid() % 1000))
        dist.init_process_group('gloo', rank=0, world_size=1)
    rank, world = dist.get_rank(), dist.get_world_size()
    if world != n_gpus:
        _fail(f'rank {rank}: the process group has {world} ranks, --gpus says {n_gpus}')
    return rank, world


def _launch_check(args) -> None:
    """--launch-check: form the world exactly as the bench does (without touching a GPU when the
    backend is gloo), verify it, and print the line's launch fields -- what the CPU tests run."""
    rank, world = _init_dist(args.gpus, use_gpu=os.environ.get('DEEPEP_BENCH_BACKEND', 'nccl') == 'nccl')
    seen = torch.zeros((world,), dtype=torch.int64)
    seen[rank] = os.getpid()
    dist.all_reduce(seen)
    if rank == 0:
        print(json.dumps({'launch_check': True, 'n_gpus': world, 'world_size_seen': world,
                          'launcher': os.environ.get('DEEPEP_BENCH_LAUNCHER', 'external'),
                          'distinct_rank_processes': len(set(seen.tolist())),
                          'backend': dist.get_backend()}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


_XGMI = {'enabled': os.environ.get('DEEPEP_BENCH_XGMI', '1') != '0', 'preflight': None}
_RCCL = {'preflight': None}
PREFLIGHT_LIMIT_S = 150.0


def _start_child(script: str, port_offset: int):
    """Start a preflight script as a child (before this process touches the GPU) on MASTER_PORT +
    port_offset, its output in temporary files."""
    import subprocess
    import tempfile
    # the children's own store: torchrun's agent store (TORCHELASTIC_USE_AGENT_STORE) serves the parents
    env = {k: v for k, v in os.environ.items() if not k.startswith('TORCHELASTIC_')}
    env['MASTER_PORT'] = str(int(os.environ.get('MASTER_PORT', '29500')) + port_offset)
    env['MASTER_ADDR'] = os.environ.get('MASTER_ADDR', '127.0.0.1')
    out, err = tempfile.TemporaryFile('w+'), tempfile.TemporaryFile('w+')
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, script)], env=env, cwd=ROOT, stdout=out, stderr=err,
                         text=True)
    return dict(script=script, proc=p, out=out, err=err, t0=time.perf_counter())


def _finish_child(c, limit: float = PREFLIGHT_LIMIT_S) -> dict:
    """Wait for a preflight child (killed at `limit` s after its start) and read its JSON verdict; a child
    that fails, hangs or prints nothing is ok=False with an error, never an exception."""
    import subprocess
    p, rc = c['proc'], None
    while rc is None and time.perf_counter() - c['t0'] < limit:
        try:
            rc = p.wait(timeout=max(0.1, min(30.0, limit - (time.perf_counter() - c['t0']))))
        except subprocess.TimeoutExpired:
            print(f'[bench] {c["script"]} running ({time.perf_counter() - c["t0"]:.0f} s)', file=sys.stderr, flush=True)
    if rc is None:
        p.kill()
        p.wait()
        c['out'].close()
        c['err'].close()
        return dict(ok=False, error=f'preflight timed out ({limit:.0f} s)', seconds=round(time.perf_counter() - c['t0'], 1))
    c['out'].seek(0)
    c['err'].seek(0)
    stdout, stderr = c['out'].read(), c['err'].read()
    c['out'].close()
    c['err'].close()
    lines = [ln for ln in stdout.splitlines() if ln.startswith('{')]
    try:
        res = json.loads(lines[-1]) if lines else {}
    except ValueError:
        res = {}
    res['exit_status'] = rc
    res['ok'] = bool(res.get('ok')) and rc == 0
    if not res['ok'] and not res.get('error'):
        res['error'] = (stderr.strip().splitlines() or ['no output'])[-1][:300]
    return res


def _xgmi_preflight() -> dict:
    """xgmi_preflight.py as a child: a small xGMI dispatch + combine checked bit for bit against the
    default transport, in a gloo world of the children on MASTER_PORT + 1.  A GPU fault there ends the
    child, not the bench."""
    return _finish_child(_start_child('xgmi_preflight.py', PORT_XGMI_PREFLIGHT))


def _rccl_preflight() -> dict:
    """rccl_preflight.py as a child: a small RCCL dispatch + combine (pipelined all-to-alls) checked bit for
    bit against the same calls over gloo, in an RCCL world of the children on MASTER_PORT + 2."""
    return _finish_child(_start_child('rccl_preflight.py', PORT_RCCL_PREFLIGHT))


def _run_preflights(rccl: bool, xgmi: bool):
    """Both preflights at once (each child on its own port), before this process touches the GPU."""
    kids = {}
    if rccl:
        kids['rccl'] = _start_child('rccl_preflight.py', PORT_RCCL_PREFLIGHT)
    if xgmi:
        kids['xgmi'] = _start_child('xgmi_preflight.py', PORT_XGMI_PREFLIGHT)
    return {k: _finish_child(c) for k, c in kids.items()}


def _agree(flags: dict, rank: int, world: int, timeout_s: float = 120.0) -> dict:
    """Every rank's preflight verdicts, ANDed over the ranks through a TCP store (no process group exists
    yet: which backend the ranks' group uses depends on the result).  Under torchrun the launcher's agent
    store on MASTER_PORT serves it (keys under a prefix, as the env:// rendezvous uses it); when bench.py
    starts its own ranks, rank 0 hosts a store on MASTER_PORT + 3 (checked free at launch)."""
    from datetime import timedelta
    host, port = os.environ.get('MASTER_ADDR', '127.0.0.1'), int(os.environ.get('MASTER_PORT', '29500'))
    agent = os.environ.get('TORCHELASTIC_USE_AGENT_STORE', '').lower() == 'true'
    base = dist.TCPStore(host, port if agent else port + PORT_AGREE, world, rank == 0 and not agent,
                         timeout=timedelta(seconds=timeout_s))
    store = dist.PrefixStore(f'deepep_bench_preflight_{os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")}/', base)
    store.set(f'preflight/{rank}', json.dumps(flags))
    keys = [f'preflight/{r}' for r in range(world)]
    store.wait(keys)
    every = [json.loads(store.get(k)) for k in keys]
    out = {name: all(bool(f.get(name)) for f in every) for name in flags}
    # rank 0 may host the store: it leaves only after every rank has read the verdicts
    store.set(f'preflight_read/{rank}', '1')
    if rank == 0:
        store.wait([f'preflight_read/{r}' for r in range(world)])
    return out


def _agree_or_default(flags: dict, rank: int, world: int) -> dict:
    """_agree, or -- when the store itself fails, on every rank alike (rank 0 could not host it, or the
    others timed out reaching it) -- the pre-preflight default (RCCL headline, no xGMI legs), named in
    the line."""
    try:
        return dict(_agree(flags, rank, world), agreement='store')
    except Exception as e:          # noqa: BLE001 -- reported in the line
        print(f'[bench] rank {rank}: preflight agreement failed ({type(e).__name__}: {e}); default transport',
              file=sys.stderr, flush=True)
        return dict(rccl=True, xgmi=False, agreement=f'failed ({type(e).__name__}: {str(e)[:200]}): default')


def _choose_headline(backend_env: str, rccl_ok, xgmi_ok: bool) -> dict:
    """The N > 1 headline's transport from the agreed preflight verdicts:
      RCCL ok                 -> nccl group, RCCL all-to-all (the north star's transport)
      RCCL failed, xGMI ok    -> gloo group (control only), xGMI window stores
      both failed             -> gloo group, the all-to-all through host memory (marked)
    DEEPEP_BENCH_BACKEND=gloo (rehearsal on shared GPUs) keeps the gloo exchange and runs no RCCL preflight."""
    if backend_env == 'gloo':
        return dict(backend='gloo', transport='rccl', label='gloo-host-exchange',
                    reason='DEEPEP_BENCH_BACKEND=gloo rehearsal: the all-to-all goes through host memory')
    if rccl_ok:
        return dict(backend='nccl', transport='rccl', label='rccl', reason='rccl_preflight passed on every rank')
    if xgmi_ok:
        return dict(backend='gloo', transport='xgmi', label='xgmi',
                    reason='rccl_preflight failed on at least one rank; xgmi_preflight passed on every rank')
    return dict(backend='gloo', transport='rccl', label='gloo-host-exchange',
                reason='rccl_preflight and xgmi_preflight failed: the all-to-all goes through host memory over gloo')


def _xgmi_enabled() -> bool:
    return _XGMI['enabled']


_T_START = time.perf_counter()
# N > 1: the secondary legs (phase-A budget, xGMI, single reduction, dispatch, sync-free) start only while the
# run is inside a soft time budget, checked at every leg boundary with the MAX over ranks (every rank skips
# the same legs); and a watchdog ends the run at a hard deadline with the line built so far (the headline
# `value` first), so that a leg that hangs on a node never costs the whole line.  The driver's run of
# `python bench.py --gpus 8` must fit its time limit.
SOFT_BUDGET_S = float(os.environ.get('DEEPEP_BENCH_SOFT_S', 300))
HARD_DEADLINE_S = float(os.environ.get('DEEPEP_BENCH_HARD_S', 480))


_LINE = [None]          # rank 0's line once the headline is measured (emitted if a later leg raises)


class _Line:
    """Rank 0's result line, filled leg by leg; `emit()` prints it once (normally at the end, or from the
    watchdog at the hard deadline with `incomplete` naming the leg that was running)."""

    def __init__(self, rank: int):
        self.rank, self.fields, self.leg, self.skipped = rank, None, 'setup', []
        self._printed = False
        self._lock = __import__('threading').Lock()

    def emit(self, incomplete: str = None) -> None:
        with self._lock:
            if self._printed or self.rank != 0 or self.fields is None:
                return
            self._printed = True
            line = dict(self.fields)
            line['launch'] = dict(line.get('launch') or {}, wall_s=round(time.perf_counter() - _T_START, 1))
            if self.skipped:
                line['skipped_legs'] = list(self.skipped)
            if incomplete:
                line['incomplete'] = incomplete
            print(json.dumps(line), flush=True)

    def start_watchdog(self) -> None:
        import threading

        def fire():
            self.emit(incomplete=f'hard deadline {HARD_DEADLINE_S:.0f} s hit during leg "{self.leg}"; the '
                                 f'fields present were measured before it')
            print(f'[bench] rank {self.rank}: hard deadline during leg {self.leg}, exiting', file=sys.stderr,
                  flush=True)
            os._exit(0)
        t = threading.Timer(max(1.0, HARD_DEADLINE_S - (time.perf_counter() - _T_START)), fire)
        t.daemon = True
        t.start()


def _within_budget(dev, world: int) -> bool:
    """True while the slowest rank is inside the soft budget (a collective every rank reaches)."""
    el = torch.tensor([time.perf_counter() - _T_START], dtype=torch.float64, device=dev if world > 1 else 'cpu')
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return float(el.item()) < SOFT_BUDGET_S


def _memory(dev, world: int) -> dict:
    """Peak device memory (allocator) and host RSS of the worst rank."""
    import resource
    v = torch.tensor([torch.cuda.max_memory_allocated(dev) / 2 ** 30, torch.cuda.max_memory_reserved(dev) / 2 ** 30,
                      resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2 ** 20], dtype=torch.float64,
                     device=dev if world > 1 else 'cpu')
    if world > 1:
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
    return dict(device_max_allocated_gib=round(float(v[0]), 2), device_max_reserved_gib=round(float(v[1]), 2),
                host_max_rss_gib=round(float(v[2]), 2), note='max over ranks')


def _cpu_threads() -> int:
    """Host threads for the CPU baseline: the GPU box's CPU share per GPU (16; os.cpu_count() there
    reports the whole machine's CPUs, many times as many -- both are in the line)."""
    return max(1, min(16, int(os.environ.get('OMP_NUM_THREADS', '16')), os.cpu_count() or 1))


def _cpu_model() -> str:
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def _cpu_baseline(y: torch.Tensor, table: torch.Tensor, w: torch.Tensor, weighted: bool, min_seconds: float):
    """The CPU oracle (oracle/combine_ref.c, the C restatement of the reference arithmetic; kind
    "port") timed on the host cores over the SAME batch: the expanded rows, slot table and weights
    copied to host memory (not cache-resident: ~0.94 GB), tokens split over threads, full passes
    repeated for >= min_seconds."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    import oracle
    lib = oracle.rows_lib()
    yh, th, wh = y.cpu(), table.cpu().contiguous(), w.cpu().contiguous()
    T, K = th.shape
    H = yh.shape[1]
    out = torch.empty((T, H), dtype=torch.bfloat16)
    out_w = torch.empty((T, K), dtype=torch.float32)
    n_thr = _cpu_threads()
    bounds = [(T * i // n_thr, T * (i + 1) // n_thr) for i in range(n_thr)]

    def part(lo_hi):
        lo, hi = lo_hi
        rc = lib.oracle_combine_rows(
            2, int(weighted), ctypes.c_void_p(yh.data_ptr()), yh.shape[0], H,
            ctypes.c_void_p(th.data_ptr() + lo * K * 4), K, K, ctypes.c_void_p(wh.data_ptr()) if weighted else None,
            None, None, ctypes.c_void_p(out.data_ptr() + lo * H * 2), H, hi - lo, H,
            ctypes.c_void_p(th.data_ptr() + lo * K * 4), K, ctypes.c_void_p(wh.data_ptr()),
            ctypes.c_void_p(out_w.data_ptr() + lo * K * 4), K, K)
        assert rc == 0

    valid = int((th >= 0).sum())
    bytes_per = valid * H * 2 + T * H * 2 + valid * 4 + valid * 4
    reps, t0 = 0, time.perf_counter()
    with ThreadPoolExecutor(n_thr) as ex:
        while True:
            list(ex.map(part, bounds))
            reps += 1
            el = time.perf_counter() - t0
            if el >= min_seconds:
                break
    return dict(value=round(bytes_per * reps / el / 1e9, 3), unit='GB/s', cores=n_thr, kind='port',
                cpu_model=_cpu_model(), os_cpu_count=os.cpu_count(),
                sample=f'{reps} full pass(es) of the bench batch ({T} tokens x top-{K} x hidden {H}, host copy) '
                       f'through oracle_combine_rows (C restatement, fused {"weighted" if weighted else "plain"}), '
                       f'{n_thr} threads, {el:.1f} s')


def _cpu_torch(tokens: int, hidden: int, topk: int, min_seconds: float):
    """BASELINE.md section 3's PyTorch-CPU weighted sum, [T, K, H] rows, same batch size."""
    g = torch.Generator().manual_seed(0)
    y = torch.randn((tokens, topk, hidden), generator=g).to(torch.bfloat16)
    w = torch.rand((tokens, topk), generator=g)
    reps, t0 = 0, time.perf_counter()
    while True:
        acc = torch.zeros((tokens, hidden), dtype=torch.float32)
        for k in range(topk):
            acc.addcmul_(y[:, k].float(), w[:, k:k + 1])
        out = acc.to(torch.bfloat16)
        reps += 1
        el = time.perf_counter() - t0
        if el >= min_seconds:
            break
    bytes_per = tokens * (topk * hidden * 2 + hidden * 2 + topk * 4 + topk * 4)
    del out, y
    return dict(value=round(bytes_per * reps / el / 1e9, 3), unit='GB/s', threads=torch.get_num_threads(),
                sample=f'{reps} x ({tokens} tokens x top-{topk} x hidden {hidden}) torch.addcmul_ fp32 loop, {el:.1f} s')


def _bench_xgmi(buf, y, handle, ex_w, weighted, total_bytes, steps, warmup, dev):
    """EP > 1 combine over the xGMI symmetric windows (DEEPEP_TRANSPORT=xgmi), timed like the main
    loop and checked bit for bit against the default (RCCL) transport on the same batch.  Failures
    (IPC, barrier timeout, mismatch) are reported, never raised: the main measurement stands."""
    from deepep_amd import ElasticBuffer

    def agree(ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    ref, _, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=weighted)
    torch.cuda.synchronize()
    err = None
    xb = None
    try:
        xb = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=buf.num_max_tokens_per_rank,
                           hidden=y.shape[1], num_topk=handle.topk_idx.shape[1], explicitly_destroy=True,
                           num_gpu_timeout_secs=5)
        xb.transport = 'xgmi'
        out, _, _ = xb.combine(y, handle, topk_weights=ex_w, apply_topk_weights=weighted)
        torch.cuda.synchronize()
        xb._sym.check()
        equal = bool(torch.equal(out, ref))
    except Exception as e:          # noqa: BLE001 -- reported in the JSON line
        err, equal = f'{type(e).__name__}: {e}'[:300], False
    if not agree(err is None):
        return dict(error=err or 'failed on another rank')
    equal_all = agree(equal)

    def step():
        return xb.combine(y, handle, topk_weights=ex_w, apply_topk_weights=weighted)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    # a device barrier that timed out in warm-up would make every timed step wait the timeout
    if not agree(int(xb._sym.error_flag.item()) == 0):
        xb.destroy()
        return dict(error='device barrier timeout during warm-up', bitwise_equal_to_rccl=equal_all)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    timed_out = not agree(int(xb._sym.error_flag.item()) == 0)
    # the same loop with phase A held to 128 CUs (DEEPEP_PHASE_A_CUS): does freeing CUs for phase B
    # of the earlier chunks help the overlap on this node?
    budget = None
    if not timed_out and xb._num_chunks(handle) > 1:
        xb.phase_a_cus = 128
        out_b, _, _ = step()
        same_b = agree(bool(torch.equal(out_b, ref)))
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        el_b = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(el_b, op=dist.ReduceOp.MAX)
        el_b = float(el_b.item())
        budget = dict(phase_a_cus=128, value=round(total_bytes * steps / el_b / 1e9, 2),
                      ms_per_step=round(el_b * 1e3 / steps, 4), bitwise_equal_to_rccl=same_b,
                      barrier_timeout=not agree(int(xb._sym.error_flag.item()) == 0))
        xb.phase_a_cus = 0
    xb.destroy()
    return dict(value=round(total_bytes * steps / el / 1e9, 2), unit='GB/s', ms_per_step=round(el * 1e3 / steps, 4),
                bitwise_equal_to_rccl=equal_all, barrier_timeout=timed_out, phase_a_budget=budget,
                note='same batch and bytes as `value`, DEEPEP_TRANSPORT=xgmi: phase A stores into the peers\' '
                     'symmetric windows over xGMI, device barriers, phase B from the local window')


def _bench_xgmi_dispatch(buf, x, topk_idx, topk_w, E, disp_bytes, time_dispatch, dev):
    """The dispatch with every packed row stored straight into its destination's symmetric window
    (DEEPEP_TRANSPORT=xgmi), checked bit for bit against the RCCL dispatch of the same batch.
    Failures are reported, never raised."""
    from deepep_amd import ElasticBuffer

    def agree(ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    ref = buf.dispatch(x, topk_idx=topk_idx, topk_weights=topk_w, num_experts=E, do_expand=True)
    torch.cuda.synchronize()
    err, equal, xb = None, False, None
    try:
        xb = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=buf.num_max_tokens_per_rank,
                           hidden=_hidden_of(x), num_topk=topk_idx.shape[1], explicitly_destroy=True,
                           num_gpu_timeout_secs=5)
        xb.transport = 'xgmi'
        got = xb.dispatch(x, topk_idx=topk_idx, topk_weights=topk_w, num_experts=E, do_expand=True)
        torch.cuda.synchronize()
        xb._sym.check()
        rx, gx = (ref[0][0], got[0][0]) if isinstance(ref[0], tuple) else (ref[0], got[0])
        equal = (torch.equal(rx.view(torch.uint8), gx.view(torch.uint8)) and torch.equal(ref[2], got[2]) and
                 torch.equal(ref[3].recv_src_metadata, got[3].recv_src_metadata))
    except Exception as e:          # noqa: BLE001 -- reported in the JSON line
        err = f'{type(e).__name__}: {e}'[:300]
    if not agree(err is None):
        if xb is not None:
            xb.destroy()
        return dict(error=err or 'failed on another rank')
    equal_all = agree(equal)
    t_d, t_c = time_dispatch(xb)
    timed_out = not agree(int(xb._sym.error_flag.item()) == 0)
    xb.destroy()
    return dict(ms=round(t_d * 1e3, 3), cached_ms=round(t_c * 1e3, 3), cached_gbps=round(disp_bytes / t_c / 1e9, 1),
                bitwise_equal_to_rccl=equal_all, barrier_timeout=timed_out,
                note='rows pushed straight into the destinations\' symmetric windows (system-scope stores), '
                     'device barriers, receive-side kernels on the local window; per-rank wall time')


def _bench_sync_free(buf, x, topk_idx, topk_w, E, weighted, dev, n_iter: int = 8):
    """What dispatch(do_cpu_sync=False) costs over RCCL (buffer.hpp:1065-1070's no-sync mode): a fresh
    dispatch plus the handle's FIRST combine (plan built on the device), per iteration, against the same
    pair with the host-synced dispatch; and the bytes each exchange moves.  Without a CPU sync the host
    knows no split sizes, so the dispatch all-to-all moves T_max rows to every rank and the combine plan
    is worst-case padded (R x chunk tokens per chunk) -- the padding travels too.  The combine input is
    the dispatch's own expanded output (its shape is the handle's).  Max over ranks.  Failures are
    reported, never raised."""
    from deepep_amd.handle import packed_row_layout
    from deepep_amd.kernels import RowLayout
    R, T_max = buf.num_ranks, buf.num_max_tokens_per_rank
    xr, sf = (x if isinstance(x, tuple) else (x, None))
    K = topk_idx.shape[1]
    disp_row = RowLayout.make(xr.shape[1] * xr.element_size(), sf.shape[1] * sf.element_size() if sf is not None
                              else 0, K).row_bytes
    comb_row = packed_row_layout(xr.shape[1], K, True)[0]

    def vmax(v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def run(do_cpu_sync: bool):
        h = None
        for i in range(n_iter + 1):
            if i == 1:
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
            ex_x, _, ex_w, h, _ = buf.dispatch(x, topk_idx=topk_idx, topk_weights=topk_w, num_experts=E,
                                               do_expand=True, do_cpu_sync=do_cpu_sync)
            if not isinstance(ex_x, tuple):                  # FP8 rows are not a combine input
                buf.combine(ex_x, h, topk_weights=ex_w, apply_topk_weights=weighted)
            del ex_x, ex_w
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / n_iter
        plan = next((p for k, p in h._combine_plans.items() if k[0] == 'multi'), None)
        # rows the all-to-all moves (the local bypass keeps a rank's own rows out of it)
        comb_rows = sum(sum(ch.send_counts) - ch.own for ch in plan.chunks) if plan is not None else None
        return vmax(el * 1e3), comb_rows

    try:
        ms_sync, rows_sync = run(True)
        ms_free, rows_free = run(False)
        h_sync = buf.dispatch(x, topk_idx=topk_idx, topk_weights=topk_w, num_experts=E, do_expand=True)[3]
        n_sent = int(sum(c for d, c in enumerate(h_sync._send_counts) if not (h_sync._bypass and d == buf.rank_idx)))
        # the padded exchange moves T_max rows to every rank but itself (the local bypass keeps its own block)
        moved = torch.tensor([n_sent * disp_row, (R - (1 if buf.local_bypass else 0)) * T_max * disp_row,
                              (rows_sync or 0) * comb_row,
                              (rows_free or 0) * comb_row], dtype=torch.float64, device=dev)
        dist.all_reduce(moved)
        moved = [float(v) for v in moved.tolist()]
        return dict(ms=round(ms_free, 3), synced_ms=round(ms_sync, 3),
                    dispatch_exchange_bytes=moved[1], synced_dispatch_exchange_bytes=moved[0],
                    combine_exchange_bytes=moved[3], synced_combine_exchange_bytes=moved[2],
                    padding_factor_dispatch=round(moved[1] / max(moved[0], 1), 3),
                    padding_factor_combine=round(moved[3] / max(moved[2], 1), 3),
                    fp8_input=sf is not None,
                    note='fresh dispatch(do_expand=True, do_cpu_sync=False) + the handle\'s first combine (plan '
                         'built on the device), per iteration, RCCL transport, max over ranks; synced_* = the same '
                         'pair with the host-synced dispatch; *_exchange_bytes = all ranks\' all-to-all bytes '
                         '(worst-case padded without a CPU sync; the local bypass keeps a rank\'s own rows / '
                         'padded block out of both); fp8 input: dispatch only')
    except Exception as e:          # noqa: BLE001 -- reported in the JSON line
        return dict(error=f'{type(e).__name__}: {e}'[:300])


def _hidden_of(x) -> int:
    return (x[0] if isinstance(x, tuple) else x).shape[1]


def _calc_diff(a: torch.Tensor, b: torch.Tensor) -> float:
    """deep_ep/utils/math.py:5-9."""
    a, b = a.double() + 1, b.double() + 1
    return float(1 - 2 * (a * b).sum() / (a * a + b * b).sum())


def _bench_single(y, handle, ex_w, weighted, total_bytes, steps, warmup, dev, ref_multi):
    """EP > 1 combine with allow_multiple_reduction=False on the same batch: every expanded row
    travels unreduced (weighted: with its gating weight) and the source rank reduces once -- the
    legacy low-latency semantics, and the north star's "all-to-all feeding each rank's local reduce".
    Timed like the main loop on both transports; per-phase times on RCCL (phase A = pack copy, B =
    the one reduce).  Failures are reported, never raised."""
    from deepep_amd import ElasticBuffer
    T_max, H, K = handle.num_max_tokens_per_rank, y.shape[1], handle.topk_idx.shape[1]

    def agree(ok: bool) -> bool:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def vmax(v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    res, outs = {}, {}
    # over a gloo group (a failed RCCL preflight) the 'rccl' recipe would move its rows through host memory:
    # then only the xGMI recipe runs, when it can
    rccl_ok = dist.get_backend() == 'nccl' or not _xgmi_enabled()
    transports = (['rccl'] if rccl_ok else []) + (['xgmi'] if _xgmi_enabled() else [])
    for transport in transports:
        sb, err = None, None
        try:
            sb = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T_max, hidden=H, num_topk=K,
                               allow_multiple_reduction=False, explicitly_destroy=True, num_gpu_timeout_secs=5)
            sb.transport = transport

            def step():
                return sb.combine(y, handle, topk_weights=ex_w if weighted else None, apply_topk_weights=weighted)
            outs[transport] = step()[0]
            torch.cuda.synchronize()
            if sb._sym is not None:
                sb._sym.check()
        except Exception as e:      # noqa: BLE001 -- reported in the JSON line
            err = f'{type(e).__name__}: {e}'[:300]
        if not agree(err is None):
            res[transport] = dict(error=err or 'failed on another rank')
            outs.pop(transport, None)
            continue
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        if sb._sym is not None and not agree(int(sb._sym.error_flag.item()) == 0):
            res[transport] = dict(error='device barrier timeout during warm-up')
            outs.pop(transport, None)
            sb.destroy()
            continue
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        el = vmax(time.perf_counter() - t0)
        entry = dict(value=round(total_bytes * steps / el / 1e9, 2), ms_per_step=round(el * 1e3 / steps, 4))
        if transport == 'rccl':
            sb._phase_events, sb._phase_unpipelined = [], True          # one chunk: the exchange separable
            n_ph = max(5, steps // 2)
            for _ in range(n_ph):
                step()
            torch.cuda.synchronize()
            ev, sb._phase_events, sb._phase_unpipelined = sb._phase_events, None, False
            t_a = vmax(sum(ev[4 * i].elapsed_time(ev[4 * i + 1]) for i in range(n_ph)) / n_ph)
            t_x = vmax(sum(ev[4 * i + 1].elapsed_time(ev[4 * i + 2]) for i in range(n_ph)) / n_ph)
            t_b = vmax(sum(ev[4 * i + 2].elapsed_time(ev[4 * i + 3]) for i in range(n_ph)) / n_ph)
            # the device-resident work of this recipe is the send-side pass (every valid expanded row copied
            # unreduced into the send buffer) AND the one reduce: both count
            entry.update(phase_a_ms=round(t_a, 4), exchange_ms=round(t_x, 4), phase_b_ms=round(t_b, 4),
                         reduce_only_gbps=round(total_bytes / ((t_a + t_b) * 1e-3) / 1e9, 1))
        else:
            entry['barrier_timeout'] = not agree(int(sb._sym.error_flag.item()) == 0)
        res[transport] = entry
        sb.destroy()
    if 'rccl' in outs and 'xgmi' in outs and 'value' in res.get('xgmi', {}):
        res['xgmi']['bitwise_equal_to_rccl'] = agree(bool(torch.equal(outs['rccl'], outs['xgmi'])))
    if outs:
        d = vmax(_calc_diff(outs.get('rccl', outs.get('xgmi')), ref_multi))
        res['calc_diff_vs_multi_reduction'] = d
    res['note'] = ('allow_multiple_reduction=False, same batch and bytes: rows unreduced to the source rank '
                   '(weighted: legacy low-latency fma chain), one reduce there; reduce_only = algorithmic bytes '
                   'of all ranks / (phase A: the send-side pass over every expanded row + phase B: the reduce), '
                   'unpipelined, max over ranks')
    return res


def _pmc_entry(workload: str) -> dict:
    try:
        with open(os.path.join(ROOT, 'profiles', 'pmc_traffic.json')) as f:
            return json.load(f).get(workload) or {}
    except (OSError, ValueError):
        return {}


def _pmc_traffic(workload: str, build_id: str):
    """HBM bytes per launch of the dominant kernel from the rocprofv3 PMC passes in
    profiles/pmc_traffic.json (tools/gpu_session.sh `pmc` step -> tools/summarize_prof.py), accepted
    only when they were collected with THIS library build (same build id: sources, header, flags);
    otherwise None and the reason.  Returns (bytes or None, build id of the counters, note)."""
    path = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    try:
        with open(path) as f:
            entry = json.load(f).get(workload)
    except (OSError, ValueError):
        entry = None
    if entry is None or 'hbm_bytes_per_launch' not in entry:
        return None, None, f'no PMC pass for {workload} in profiles/pmc_traffic.json'
    if entry.get('build_id') != build_id:
        return None, entry.get('build_id'), (f'PMC pass collected with build {entry.get("build_id")}, this is '
                                             f'{build_id}: stale, not reported')
    return float(entry['hbm_bytes_per_launch']), build_id, ('2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), '
                                                             'MI355X_MICROARCH.md gfx950 corrections, same build')


def _hbm_bytes_per_rank(world: int, T: int, H: int, K: int, build_id: str) -> dict:
    """The whole EP = N step's HBM bytes per rank by transport (rccl / xgmi / algorithmic) from the same-build
    PMC passes (tools/pmc_ep.py -> summarize_prof.py stepfold -> profiles/pmc_traffic.json); another build's
    counters are not reported."""
    e = _pmc_entry(f'step_ep{world}_t{T}_h{H}_k{K}')
    if not e:
        return dict(rccl=None, xgmi=None, algorithmic=None, note=f'no step PMC pass for EP = {world}')
    if e.get('build_id') != build_id:
        return dict(rccl=None, xgmi=None, algorithmic=None,
                    note=f'step PMC pass of build {e.get("build_id")}, this is {build_id}: stale, not reported')
    return dict(e['hbm_bytes_per_rank'], build_id=build_id, source=e.get('source'),
                note='HBM bytes of one whole combine step per rank (2 x FETCH_SIZE + WRITE_SIZE): rccl = phase A + '
                     'the exchange\'s copies + phase B; xgmi = phase A + phase B of the same passes (phase A stores '
                     'into the owners\' windows, no exchange pass); algorithmic = `value`\'s bytes per rank')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=1000)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--tokens', type=int, default=8192)
    ap.add_argument('--hidden', type=int, default=7168)
    ap.add_argument('--topk', type=int, default=8)
    ap.add_argument('--experts', type=int, default=256)
    ap.add_argument('--plain', action='store_true', help='reference (unweighted) combine instead of weighted')
    ap.add_argument('--fp8-dispatch', action='store_true', help='BASELINE config 4: FP8 e4m3 dispatch, BF16 combine')
    ap.add_argument('--skew', type=float, default=1.0, help='BASELINE config 5: rank-0 overload ratio (e.g. 4)')
    ap.add_argument('--cpu-seconds', type=float, default=10.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-loopback', action='store_true')
    ap.add_argument('--no-flushed', action='store_true',
                    help='skip the per-launch flushed timing (keeps a rocprof kernel average to back-to-back launches)')
    ap.add_argument('--no-layout-ref', action='store_true',
                    help='skip the token-major layout reference (keeps a rocprof kernel average to the product input)')
    ap.add_argument('--launch-check', action='store_true',
                    help='form and verify the N-rank world, print its launch fields, measure nothing')
    ap.add_argument('--preflight-check', action='store_true',
                    help='N > 1: run the RCCL / xGMI preflights, agree on them, print the chosen headline '
                         'transport and the preflight fields, measure nothing')
    args = ap.parse_args()
    if args.gpus < 1:
        _fail('--gpus must be >= 1')
    if args.gpus > 1 and 'RANK' not in os.environ:
        sys.exit(_launch_ranks(args.gpus))
    if args.launch_check:
        _launch_check(args)
        return

    multi = 'RANK' in os.environ and int(os.environ.get('WORLD_SIZE', '1')) > 1
    backend_env = os.environ.get('DEEPEP_BENCH_BACKEND', 'nccl')
    headline = dict(backend=None, transport='rccl', label='local', reason='one rank')
    if multi:
        # Before this process touches the GPU: the RCCL and xGMI preflights as children (a fault or hang
        # there ends a child, not the bench), their verdicts agreed over a store, and the headline's
        # transport chosen from them -- so an RCCL failure on a new node never costs the line.
        if args.gpus != int(os.environ['WORLD_SIZE']):
            _fail(f'--gpus {args.gpus} but the launcher started {os.environ["WORLD_SIZE"]} ranks')
        pf = _run_preflights(rccl=backend_env == 'nccl', xgmi=_XGMI['enabled'])
        _RCCL['preflight'] = pf.get('rccl') or dict(ok=False, skipped=f'DEEPEP_BENCH_BACKEND={backend_env}')
        _XGMI['preflight'] = pf.get('xgmi')
        agreed = _agree_or_default({'rccl': bool(_RCCL['preflight'].get('ok')),
                                    'xgmi': bool(_XGMI['preflight'] and _XGMI['preflight'].get('ok'))},
                                   int(os.environ['RANK']), int(os.environ['WORLD_SIZE']))
        _RCCL['preflight']['all_ranks_ok'] = agreed['rccl']
        _RCCL['preflight']['agreement'] = agreed['agreement']
        if _XGMI['preflight'] is not None:
            _XGMI['preflight']['all_ranks_ok'] = agreed['xgmi']
        _XGMI['enabled'] = _XGMI['enabled'] and agreed['xgmi']    # the xGMI legs run only when every rank passed
        headline = _choose_headline(backend_env, agreed['rccl'], agreed['xgmi'])
    if args.preflight_check:
        if not multi:
            _fail('--preflight-check needs N > 1 ranks')
        rank, world = _init_dist(args.gpus, use_gpu=headline['backend'] == 'nccl', backend=headline['backend'])
        if rank == 0:
            print(json.dumps({'preflight_check': True, 'n_gpus': world, 'headline_transport': headline,
                              'config': {'transport': headline['label']}, 'rccl_preflight': _RCCL['preflight'],
                              'xgmi_preflight': _XGMI['preflight']}), flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return
    rank, world = _init_dist(args.gpus, backend=headline['backend'])
    line = _Line(rank)
    if world > 1:
        # N > 1: the watchdog runs from here, so even a headline that hangs on a node leaves a line (value
        # null, `incomplete` naming the leg) with the preflight fields that explain it
        line.fields = {'metric': 'combine GB/s (device-resident BF16 top-k weighted reduce) at 1/2/4/8 MI355X',
                       'value': None, 'unit': 'GB/s', 'n_gpus': world, 'higher_is_better': True,
                       'config': {'parallelism': f'ep{world}', 'transport': headline['label']},
                       'headline_transport': headline, 'rccl_preflight': _RCCL['preflight'],
                       'xgmi_preflight': _XGMI['preflight']}
        _LINE[0] = line
        line.start_watchdog()
    from deepep_amd import ElasticBuffer
    from deepep_amd.kernels import MODE_EPILOGUE, MODE_FUSED
    T, H, K, E = args.tokens, args.hidden, args.topk, args.experts
    weighted = not args.plain
    dev = torch.device('cuda', torch.cuda.current_device())
    torch.manual_seed(0 + rank)
    if args.skew != 1.0:
        from workloads import get_unbalanced_scores
        scores = get_unbalanced_scores(T, E, world, K, args.skew, device=dev)
    else:
        scores = torch.rand((T, E), device=dev)
    topk_w, topk_idx = torch.topk(scores, K, dim=-1, sorted=False)
    topk_idx = topk_idx.to(torch.int64)
    x = torch.randn((T, H), device=dev).to(torch.bfloat16)
    buf = ElasticBuffer(dist.group.WORLD, num_max_tokens_per_rank=T, hidden=H, num_topk=K)
    if world > 1:
        buf.transport = headline['transport']
    if args.fp8_dispatch:
        from workloads import per_token_cast_to_fp8
        x = per_token_cast_to_fp8(x)
    ex_x, _, ex_w, handle, _ = buf.dispatch(x, topk_idx=topk_idx, topk_weights=topk_w, num_experts=E, do_expand=True)
    ex_shape = (ex_x[0] if isinstance(ex_x, tuple) else ex_x).shape
    y = torch.randn(ex_shape, device=dev).to(torch.bfloat16)            # expert outputs, expanded layout
    del ex_x, x
    valid = int((topk_idx >= 0).sum().item())
    bytes_rank = valid * H * 2 + T * H * 2 + valid * 4 + valid * 4

    def step():
        return buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=weighted)

    line.leg = 'headline'
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    stream = torch.cuda.current_stream()        # sync-mode combine runs on the caller's stream
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    comm_ms = ev0.elapsed_time(ev1) / args.steps
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        t = t.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    total_bytes = torch.tensor([float(bytes_rank)], dtype=torch.float64, device=dev if world > 1 else 'cpu')
    if world > 1:
        dist.all_reduce(total_bytes)
    total_bytes = float(total_bytes.item())
    value = total_bytes * args.steps / elapsed / 1e9
    ms_per_step = elapsed * 1e3 / args.steps

    _LINE[0] = line
    res = dict(roofline=None, cpu_baseline=None, cpu_torch=None, loopback=None, phases=None, su_bandwidth=None,
               rccl=None, xgmi=None, single_reduction=None, fastest_leg=None, dispatch=None)

    def publish():
        line.fields = {
            'metric': 'combine GB/s (device-resident BF16 top-k weighted reduce) at 1/2/4/8 MI355X',
            'value': round(value, 2), 'unit': 'GB/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 4), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'bf16', 'data': 'synthetic',
            'config': {'workload': f'EP={world} combine, {T} tokens/rank x hidden {H} x top-{K}, '
                                   f'{E} experts, {"skewed x%g" % args.skew if args.skew != 1.0 else "uniform"} routing, '
                                   f'{"FP8 dispatch, " if args.fp8_dispatch else ""}expanded layout, '
                                   f'{"gating-weighted" if weighted else "plain (reference semantics)"}',
                       'tokens_per_rank': T, 'hidden': H, 'topk': K, 'experts': E, 'accumulate': 'fp32',
                       'parallelism': f'ep{world}', 'transport': headline['label'] if world > 1 else None},
            **res, 'headline_transport': headline if world > 1 else None,
            'rccl_preflight': _RCCL['preflight'], 'xgmi_preflight': _XGMI['preflight'],
            'launch': {'world_size_seen': world, 'launcher': os.environ.get('DEEPEP_BENCH_LAUNCHER', 'external')
                       if world > 1 else 'single process', 'backend': dist.get_backend(),
                       'devices_visible': torch.cuda.device_count(), 'soft_budget_s': SOFT_BUDGET_S,
                       'hard_deadline_s': HARD_DEADLINE_S},
        }
    publish()

    def leg(name: str, secondary: bool = True) -> bool:
        """Enter leg `name`; a secondary leg runs only inside the soft budget (every rank agrees)."""
        line.leg = name
        if secondary and world > 1 and not _within_budget(dev, world):
            line.skipped.append(f'{name} (soft budget {SOFT_BUDGET_S:.0f} s spent)')
            return False
        return True

    # Dominant kernel, timed alone on the comm stream (launches back to back, same arguments)
    roofline = None
    if world == 1:
        plan = handle._combine_plans[('multi', 1)]
        out = torch.empty((T, H), dtype=torch.bfloat16, device=dev)
        out_w = torch.empty((T, K), dtype=torch.float32, device=dev)
        kern = buf.kernels

        def launch():
            kern.combine_reduce(MODE_FUSED, y, out, T, table=plan.local_table, row_weights=ex_w if weighted else None,
                                wtable=plan.local_table, wsrc=ex_w, out_weights=out_w, stream=stream)
        for _ in range(5):
            launch()
        k0, k1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k0.record(stream)
        for _ in range(args.steps):
            launch()
        k1.record(stream)
        torch.cuda.synchronize()
        kern_us = k0.elapsed_time(k1) * 1e3 / args.steps
        # the reference's protocol (deep_ep/utils/testing.py:12-21, bench_kineto): a 256 MB+ cache flush
        # before every launch, each launch timed alone (here: 512 MB written, HIP events around the kernel)
        # The write flush leaves up to the caches' size of dirty lines that this launch then writes
        # back (round-4 probe, CHANGELOG.md: +11 us on one box, and no change after a 200 us idle); a read flush
        # (a reduction over the same 512 MB) evicts as much without dirtying, so it isolates the kernel.
        flush = torch.empty((512 << 20) // 4, dtype=torch.int32, device=dev)
        sink = torch.empty((), dtype=torch.int64, device=dev)

        def flushed_median(before):
            evs = []
            for _ in range(0 if args.no_flushed else min(args.steps, 50)):
                before()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                launch()
                b.record(stream)
                evs.append((a, b))
            torch.cuda.synchronize()
            v = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
            return v[len(v) // 2] if v else None
        kern_us_flushed = flushed_median(flush.zero_)
        kern_us_read_flushed = flushed_median(lambda: torch.sum(flush, dim=0, dtype=torch.int64, out=sink))
        del flush, sink
        achieved = bytes_rank / (kern_us * 1e-6) / 1e9
        # same-run memory reference: a device-to-device copy of the expanded rows (boxes differ by up
        # to ~20 % in copy bandwidth; this contextualises `achieved`)
        dst = torch.empty_like(y)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dst.copy_(y)
        c0.record(stream)
        for _ in range(5):
            dst.copy_(y)
        c1.record(stream)
        torch.cuda.synchronize()
        copy_gbps = 2 * y.numel() * 2 * 5 / (c0.elapsed_time(c1) * 1e-3) / 1e9
        del dst
        # same-run layout reference (round-4 probe, CHANGELOG.md): the same kernel over the same rows with each token's
        # K rows adjacent ([T, K] placement) instead of grouped by expert -- what the kernel reaches when
        # the rows a workgroup reads at once are one contiguous run; output checked bit for bit
        token_major = None
        tab = plan.local_table.long()
        if not args.no_layout_ref and bool((tab >= 0).all().item()):
            pos = torch.arange(T * K, device=dev).view(T, K)
            yt = torch.empty_like(y)
            wt = torch.empty_like(ex_w)
            yt[pos.reshape(-1)] = y[tab.reshape(-1)]
            wt[pos.reshape(-1)] = ex_w[tab.reshape(-1)]
            tab_t = pos.to(torch.int32)
            ref_o, ref_w = out.clone(), out_w.clone()

            def launch_t():
                kern.combine_reduce(MODE_FUSED, yt, out, T, table=tab_t, row_weights=wt if weighted else None,
                                    wtable=tab_t, wsrc=wt, out_weights=out_w, stream=stream)
            for _ in range(5):
                launch_t()
            c0.record(stream)
            for _ in range(args.steps):
                launch_t()
            c1.record(stream)
            torch.cuda.synchronize()
            t_us = c0.elapsed_time(c1) * 1e3 / args.steps
            token_major = dict(kernel_us=round(t_us, 2), frac=round(bytes_rank / (t_us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
                               bitwise_equal=bool(torch.equal(out, ref_o) and torch.equal(out_w, ref_w)),
                               note='diagnostic only: the same kernel and bytes over the same rows placed token-major '
                                    '(a token\'s K rows adjacent); the product input is expert-grouped')
            del yt, wt, tab_t, ref_o, ref_w
        del tab
        # The reduce phase of the EP > 1 single-reduction combine (allow_multiple_reduction=False): after
        # the exchange a rank's receive window holds its tokens' K unreduced rows at k * T_max + t (rows
        # of 2H + 16 bytes, weight in the tail); one weighted EPILOGUE launch reduces them.  Same
        # algorithmic bytes per token; what every rank runs at N GPUs once the rows have landed.
        row_e = H + 8
        win = torch.randn((K * T, row_e), device=dev).to(torch.bfloat16)
        win_w = torch.rand((K * T,), device=dev)
        kk = torch.arange(K, device=dev).view(1, K)
        tt = torch.arange(T, device=dev).view(T, 1)
        tab_b = torch.where(topk_idx >= 0, kk * T + tt, torch.full_like(topk_idx, -1)).to(torch.int32).contiguous()

        def launch_b():
            kern.combine_reduce(MODE_EPILOGUE, win[:, :H], out, T, table=tab_b, row_weights=win_w if weighted else None,
                                wtable=tab_b, wsrc=win_w, out_weights=out_w, stream=stream)
        for _ in range(5):
            launch_b()
        k0.record(stream)
        for _ in range(args.steps):
            launch_b()
        k1.record(stream)
        torch.cuda.synchronize()
        b_us = k0.elapsed_time(k1) * 1e3 / args.steps
        single_b = dict(kernel_us=round(b_us, 2), gbps=round(bytes_rank / (b_us * 1e-6) / 1e9, 1),
                        frac=round(bytes_rank / (b_us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
                        note='reduce phase of the EP > 1 single-reduction combine (one weighted EPILOGUE launch over '
                             'the K unreduced rows per token in a [K, T] receive window), same algorithmic bytes')
        del win, win_w
        workload = f'combine_fused_{"weighted" if weighted else "plain"}_t{T}_h{H}_k{K}'
        build_id = kern.lib.deepep_amd_build_id().decode()
        traffic, traffic_build, traffic_note = _pmc_traffic(workload, build_id)
        roofline = dict(bound='hbm', achieved=round(achieved, 1), peak=HBM_PEAK_GBPS, unit='GB/s',
                        frac=round(achieved / HBM_PEAK_GBPS, 4), traffic=traffic, traffic_build_id=traffic_build,
                        traffic_note=traffic_note, build_id=build_id,
                        kernel='combine_rows_kernel<FUSED>',
                        kernel_us=round(kern_us, 2),
                        kernel_us_flushed_median=None if kern_us_flushed is None else round(kern_us_flushed, 2),
                        kernel_us_read_flushed_median=(None if kern_us_read_flushed is None
                                                       else round(kern_us_read_flushed, 2)),
                        bytes_per_launch=bytes_rank, in_region_us_per_step=round(comm_ms * 1e3, 2),
                        same_run_d2d_copy_gbps=round(copy_gbps, 1), same_run_token_major_rows=token_major,
                        single_reduction_phase_b=single_b)
        res['roofline'] = roofline
        publish()

    phases = su_line = None
    if world > 1 and leg('phases', secondary=False):
        n_ph = max(5, args.steps // 2)

        def phase_events(unpipelined: bool):
            buf._phase_events, buf._phase_unpipelined = [], unpipelined
            for _ in range(n_ph):
                step()
            torch.cuda.synchronize()
            ev, buf._phase_events, buf._phase_unpipelined = buf._phase_events, None, False
            return ev
        # Phase kernels timed INSIDE the pipelined step (`value`'s schedule): per call, the events around
        # every chunk's phase-A launch (on the phase-A stream), then around every chunk's phase B
        n_chunks = buf._num_chunks(handle)
        ev = phase_events(False)
        per = 4 * n_chunks
        t_a_pipe = sum(ev[per * i + 2 * c].elapsed_time(ev[per * i + 2 * c + 1])
                       for i in range(n_ph) for c in range(n_chunks)) / n_ph
        t_b_pipe = sum(ev[per * i + 2 * n_chunks + 2 * c].elapsed_time(ev[per * i + 2 * n_chunks + 2 * c + 1])
                       for i in range(n_ph) for c in range(n_chunks)) / n_ph
        # ... and the same step unpipelined (one chunk), which separates the exchange
        ev = phase_events(True)
        t_a = sum(ev[4 * i].elapsed_time(ev[4 * i + 1]) for i in range(n_ph)) / n_ph
        t_x = sum(ev[4 * i + 1].elapsed_time(ev[4 * i + 2]) for i in range(n_ph)) / n_ph
        t_b = sum(ev[4 * i + 2].elapsed_time(ev[4 * i + 3]) for i in range(n_ph)) / n_ph
        sent_rows = sum(c for r_, c in enumerate(handle._recv_counts) if r_ != rank)
        x_bytes = sent_rows * (H * 2 + K * 4)
        # The dominant GPU kernel at N > 1 is phase A (LOCAL reduce): its algorithmic bytes on this rank
        # (the valid expanded rows read + one partial row with its K weights written per received
        # token) over its measured time; the worst rank is reported.
        n_recv = sum(handle._recv_counts)
        n_rows = int((handle.recv_src_metadata[:n_recv, 2:] >= 0).sum().item())
        a_bytes = n_rows * H * 2 + n_recv * (H * 2 + K * 4)
        # worst rank of the phase-A rate inside the pipelined step (all chunks' launches) and unpipelined
        a_rate = torch.tensor([a_bytes / (t_a_pipe * 1e-3) / 1e9, a_bytes / (t_a * 1e-3) / 1e9], dtype=torch.float64,
                              device=dev)
        dist.all_reduce(a_rate, op=dist.ReduceOp.MIN)
        a_rate, a_rate_unpiped = float(a_rate[0]), float(a_rate[1])
        build_id = buf.kernels.lib.deepep_amd_build_id().decode()
        # measured HBM bytes of the same phase-A launch (tools/pmc_ep.py: bench.py's inputs at EP = N, ranks
        # simulated on one GPU, the same kernels), accepted only from this build
        traffic, traffic_build, traffic_note = _pmc_traffic(f'phase_a_ep{world}_t{T}_h{H}_k{K}', build_id)
        pmc_algo = _pmc_entry(f'phase_a_ep{world}_t{T}_h{H}_k{K}').get('algorithmic_bytes_per_launch')
        roofline = dict(bound='hbm', achieved=round(a_rate, 1), peak=HBM_PEAK_GBPS, unit='GB/s',
                        frac=round(a_rate / HBM_PEAK_GBPS, 4), traffic=traffic, traffic_build_id=traffic_build,
                        traffic_note=traffic_note, traffic_algorithmic_bytes_per_launch=pmc_algo, build_id=build_id,
                        kernel='combine_rows_kernel<LOCAL> (phase A)', bytes_per_launch=a_bytes,
                        kernel_us=round(t_a_pipe * 1e3, 2), pipeline_chunks=n_chunks,
                        achieved_unpipelined=round(a_rate_unpiped, 1), kernel_us_unpipelined=round(t_a * 1e3, 2),
                        note='worst rank; phase A = the sum of its per-chunk launches inside the pipelined step, '
                             'timed with HIP events on the phase-A stream (achieved_unpipelined: the same step '
                             'with one chunk); traffic: mean PMC bytes of one rank\'s phase-A launch of this '
                             'workload (traffic_algorithmic_bytes_per_launch its algorithmic bytes); the '
                             'end-to-end step is bound by the xGMI exchange (see phases, DESIGN.md section 5)')
        vals = torch.tensor([t_a + t_b, t_x, t_a, t_b], dtype=torch.float64, device=dev)
        dist.all_reduce(vals, op=dist.ReduceOp.MAX)
        xb = torch.tensor([float(x_bytes)], dtype=torch.float64, device=dev)
        dist.all_reduce(xb)
        # The reference's "SU" combine bandwidth (tests/elastic/test_ep.py:287-346, the BASELINE.md
        # figure): num_scaleup_recv_tokens x (H * 2 + K * 4) bytes / combine time, per rank, local
        # tokens included (ignore_local_traffic off); the bottleneck (slowest) rank is reported.
        su_bytes = n_recv * (H * 2 + K * 4)
        su = torch.tensor([su_bytes / (ms_per_step * 1e-3) / 1e9, su_bytes / ((t_a + t_x) * 1e-3) / 1e9],
                          dtype=torch.float64, device=dev)
        dist.all_reduce(su, op=dist.ReduceOp.MIN)
        su_line = dict(gbps_per_rank=round(float(su[0]), 1), gbps_per_rank_phase_a_exchange=round(float(su[1]), 1),
                       bytes_rank0=su_bytes,
                       note='reference definition: received tokens x (2H + 4K) / t; gbps_per_rank uses the whole '
                            'pipelined combine step (the headline transport, the main loop), gbps_per_rank_phase_a_exchange '
                            'the unpipelined phase A + exchange (the analogue of combine_impl, which the reference '
                            'times); min over ranks')
        pipe = torch.tensor([t_a_pipe, t_b_pipe], dtype=torch.float64, device=dev)
        dist.all_reduce(pipe, op=dist.ReduceOp.MAX)
        phases = dict(phase_a_ms=round(float(vals[2]), 4), exchange_ms=round(float(vals[1]), 4),
                      phase_b_ms=round(float(vals[3]), 4),
                      pipelined_phase_a_ms=round(float(pipe[0]), 4), pipelined_phase_b_ms=round(float(pipe[1]), 4),
                      reduce_only_gbps=round(total_bytes / (float(vals[0]) * 1e-3) / 1e9, 1),
                      exchange_gbps_per_rank=round(float(xb.item()) / world / (float(vals[1]) * 1e-3) / 1e9, 1),
                      pipeline_chunks=buf._num_chunks(handle), transport=buf.transport,
                      local_bypass=buf.local_bypass, hbm_bytes_per_rank=_hbm_bytes_per_rank(world, T, H, K, build_id),
                      note='phase_*_ms / exchange_ms: the step unpipelined (1 chunk); pipelined_phase_*_ms: the sum of the '
                           'per-chunk launches inside the pipelined step (`value`); max over ranks; reduce_only = algorithmic bytes of all ranks / (phase A + phase B); '
                           'exchange = off-rank partial rows + weights / exchange time, per rank (local_bypass: the '
                           'own-rank partials are written in place, the all-to-all has a zero diagonal)')
        res.update(roofline=roofline, phases=phases, su_bandwidth=su_line)
        publish()

    # N > 1: the same loop with phase A held to 128 CUs (DEEPEP_PHASE_A_CUS) -- do RCCL's kernels and
    # phase B of the earlier chunks gain more from the freed CUs than phase A loses?
    rccl_budget = None
    if world > 1 and buf._num_chunks(handle) > 1 and leg('rccl_phase_a_budget'):
        ref_out, _, _ = step()
        buf.phase_a_cus = 128
        same_b = bool(torch.equal(step()[0], ref_out))
        del ref_out
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0b = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        el_b = torch.tensor([time.perf_counter() - t0b], dtype=torch.float64, device=dev)
        dist.all_reduce(el_b, op=dist.ReduceOp.MAX)
        same = torch.tensor([1 if same_b else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(same, op=dist.ReduceOp.MIN)
        el_b = float(el_b.item())
        rccl_budget = dict(phase_a_cus=128, value=round(total_bytes * args.steps / el_b / 1e9, 2),
                           ms_per_step=round(el_b * 1e3 / args.steps, 4), bitwise_equal=bool(same.item()))
        buf.phase_a_cus = 0
    if world > 1 and headline['label'] == 'rccl':
        res['rccl'] = dict(value=round(value, 2), ms_per_step=round(ms_per_step, 4), phase_a_budget=rccl_budget)
        publish()
    elif world > 1:
        res['rccl'] = dict(skipped=headline['reason'], headline=dict(transport=headline['label'], value=round(value, 2),
                                                                   ms_per_step=round(ms_per_step, 4),
                                                                   phase_a_budget=rccl_budget))
        publish()

    xgmi = None
    if world > 1 and not _xgmi_enabled() and _XGMI['preflight'] is not None:
        xgmi = dict(skipped='xgmi_preflight failed on at least one rank (see xgmi_preflight)')
    if world > 1 and headline['transport'] == 'xgmi':
        xgmi = dict(skipped='the xGMI transport is the headline (`value`); xgmi_preflight checked it bit for bit '
                            'against the gloo exchange')
        res['xgmi'] = xgmi
    elif world > 1 and _xgmi_enabled() and leg('xgmi'):
        xgmi = _bench_xgmi(buf, y, handle, ex_w, weighted, total_bytes, args.steps, args.warmup, dev)
        res['xgmi'] = xgmi
        publish()
    single = None
    if world > 1 and os.environ.get('DEEPEP_BENCH_SINGLE', '1') != '0' and leg('single_reduction'):
        ref_multi, _, _ = buf.combine(y, handle, topk_weights=ex_w, apply_topk_weights=weighted)
        single = _bench_single(y, handle, ex_w, weighted, total_bytes, args.steps, args.warmup, dev, ref_multi)
        del ref_multi
        res['single_reduction'] = single
        publish()

    # Handle producer: dispatch of the same batch, expanded layout.  Includes its
    # host syncs (received-token counts), as the reference's dispatch with do_cpu_sync=True.
    torch.cuda.synchronize()
    dist.barrier()
    n_disp = 50
    run_dispatch = leg('dispatch')
    x_disp = torch.randn((T, H), device=dev).to(torch.bfloat16)
    if args.fp8_dispatch:
        from workloads import per_token_cast_to_fp8
        x_disp = per_token_cast_to_fp8(x_disp)

    def time_dispatch(b):
        _, _, _, h, _ = b.dispatch(x_disp, topk_idx=topk_idx, topk_weights=topk_w, num_experts=E, do_expand=True)
        torch.cuda.synchronize()
        t_d = time.perf_counter()
        for _ in range(n_disp):
            b.dispatch(x_disp, topk_idx=topk_idx, topk_weights=topk_w, num_experts=E, do_expand=True)
        torch.cuda.synchronize()
        t_d = (time.perf_counter() - t_d) / n_disp
        # cached handle: no routing kernels, no host sync (pack -> exchange -> copy)
        t_c = time.perf_counter()
        for _ in range(n_disp):
            b.dispatch(x_disp, topk_weights=topk_w, do_expand=True, handle=h)
        torch.cuda.synchronize()
        return t_d, (time.perf_counter() - t_c) / n_disp

    dispatch = None
    if run_dispatch:
        t_d, t_c = time_dispatch(buf)
        elem = 1 if args.fp8_dispatch else 2
        disp_bytes = T * H * elem + handle.num_expanded_tokens * H * elem     # read x once, write every expanded row
        dispatch = dict(ms=round(t_d * 1e3, 3), gbps=round(disp_bytes / t_d / 1e9, 1),
                        cached_ms=round(t_c * 1e3, 3), cached_gbps=round(disp_bytes / t_c / 1e9, 1),
                        transport=buf.transport if world > 1 else 'local',
                        note='ElasticBuffer.dispatch(do_expand=True) wall time incl. host count syncs; cached = '
                             'dispatch(handle=...) (no sync); bytes = x read once + expanded rows written')
        res['dispatch'] = dispatch
        publish()
        if world > 1 and _xgmi_enabled() and headline['transport'] != 'xgmi' and leg('dispatch_xgmi'):
            dispatch['xgmi'] = _bench_xgmi_dispatch(buf, x_disp, topk_idx, topk_w, E, disp_bytes, time_dispatch, dev)
            publish()
        if world > 1 and os.environ.get('DEEPEP_BENCH_SYNC_FREE', '1') != '0' and headline['transport'] == 'rccl' \
                and leg('dispatch_sync_free'):
            dispatch['sync_free'] = _bench_sync_free(buf, x_disp, topk_idx, topk_w, E, weighted, dev)
            publish()
    del x_disp

    loopback = None
    if world == 1 and not args.no_loopback:
        # Host-staged loopback (north_star): pinned host rows -> H2D -> combine -> D2H, batches back to
        # back.  The D2H of batch i runs on its own stream, so it overlaps the H2D of batch i + 1 (PCIe
        # is full duplex); the serial chain is timed as well.
        host_y = torch.empty(y.shape, dtype=y.dtype, pin_memory=True).copy_(y)
        host_out = torch.empty((T, H), dtype=torch.bfloat16, pin_memory=True)
        dev_y = torch.empty_like(y)
        d2h = torch.cuda.Stream(device=dev)
        n_lb = 4

        def loop(overlap: bool) -> float:
            torch.cuda.synchronize()
            t_lb = time.perf_counter()
            for _ in range(n_lb):
                dev_y.copy_(host_y, non_blocking=True)
                o, _, _ = buf.combine(dev_y, handle, topk_weights=ex_w, apply_topk_weights=weighted)
                if overlap:
                    d2h.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(d2h):
                        host_out.copy_(o, non_blocking=True)
                    o.record_stream(d2h)
                else:
                    host_out.copy_(o, non_blocking=True)
            torch.cuda.synchronize()
            return (time.perf_counter() - t_lb) / n_lb
        el_serial = loop(False)
        el_lb = loop(True)
        loopback = dict(gbps=round(bytes_rank / el_lb / 1e9, 2), ms_per_batch=round(el_lb * 1e3, 2),
                        serial_gbps=round(bytes_rank / el_serial / 1e9, 2), serial_ms_per_batch=round(el_serial * 1e3, 2),
                        note='algorithmic bytes / (H2D of the expanded rows + combine + D2H of the output) per batch, '
                             'batches back to back with the D2H overlapping the next H2D; serial = one chain')
        del host_y, host_out, dev_y

    # EP > 1: `value` is the default configuration -- the RCCL all-to-all transport the north star names,
    # phase A on the whole chip.  The other legs (phase A on a CU budget, the xGMI window transport, the
    # single reduction) are complete implementations of the same combine timed with the same protocol on
    # the same batch; they stay beside it in the line, and `fastest_leg` names the fastest one whose
    # output matched the default bit for bit (information, never the headline).
    line.leg = 'summary'
    if world > 1:
        legs = [(headline['label'], value)]
        if rccl_budget is not None and rccl_budget['bitwise_equal']:
            legs.append((f'rccl, DEEPEP_PHASE_A_CUS={rccl_budget["phase_a_cus"]}', rccl_budget['value']))
        if xgmi is not None and 'value' in xgmi and xgmi['bitwise_equal_to_rccl'] and not xgmi['barrier_timeout']:
            legs.append(('xgmi', xgmi['value']))
            xb_ = xgmi.get('phase_a_budget')
            if xb_ and xb_['bitwise_equal_to_rccl'] and not xb_['barrier_timeout']:
                legs.append((f'xgmi, DEEPEP_PHASE_A_CUS={xb_["phase_a_cus"]}', xb_['value']))
        best = max(legs, key=lambda kv: kv[1])
        res['fastest_leg'] = dict(leg=best[0], value=round(best[1], 2), vs_value=round(best[1] / value, 3))

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line.leg = 'cpu_baseline'
        plan = handle._combine_plans[('multi', 1)]
        res['cpu_baseline'] = _cpu_baseline(y, plan.local_table, ex_w, weighted, args.cpu_seconds)
        res['cpu_torch'] = _cpu_torch(T, H, K, args.cpu_seconds)
    res['loopback'] = loopback
    memory = _memory(dev, world)
    publish()
    line.fields['launch']['memory'] = memory
    line.emit()
    dist.barrier()
    dist.destroy_process_group()


def _entry() -> None:
    """main(); an exception after the headline was measured still prints rank 0's line (with `incomplete`
    naming the leg), then propagates."""
    try:
        main()
    except Exception as e:                  # noqa: BLE001 -- the measured fields still reach the driver
        if _LINE[0] is not None:
            _LINE[0].emit(incomplete=f'leg "{_LINE[0].leg}" raised {type(e).__name__}: {e}; the fields '
                                     f'present were measured before it')
        raise


if __name__ == '__main__':
    _entry()
