"""Summaries of rocprofv3 output for profiles/ (kernel stats and PMC traffic).

  python tools/summarize_prof.py stats  <kernel_stats.csv> <out.md>
  python tools/summarize_prof.py timed  <kernel_trace.csv> <kernel-name substring> <out.md> [labels,...]
  python tools/summarize_prof.py pmc    <out.json> <workload> <bytes_per_launch> <counter_csv>...
The PMC summary applies the gfx950 corrections of MI355X_MICROARCH.md (HBM section):
FETCH_SIZE (KiB) counts half the bytes of a wide coalesced read stream -> x2; WRITE_SIZE (KiB)
is exact for 16-B-per-lane stores.  TCC_EA0_RDREQ/WRREQ x 64 B are recorded alongside.
"""
import csv
import json
import sys
from collections import defaultdict


def stats(path, out):
    rows = list(csv.DictReader(open(path)))
    lines = ['| kernel | calls | avg us | min us | max us | share % |', '|---|---|---|---|---|---|']
    for r in rows[:12]:
        name = r['Name'].replace('(anonymous namespace)::', '')
        short = name.split('(')[0][:90]
        lines.append(f"| `{short}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | "
                     f"{float(r['MaxNs']) / 1e3:.2f} | {float(r['Percentage']):.1f} |")
    open(out, 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines))


def timed(path, needle, out, labels=''):
    """Per-loop averages of one kernel from a --kernel-trace run of the default `python bench.py`: the
    maximal runs of >= 50 back-to-back dispatches of the kernel (in dispatch order), each averaged
    without its first 5 launches (warmup).  bench.py's loops of the fused kernel come in a fixed order
    (the timed combine steps of `value`, the kernel-alone loop of `roofline.kernel_us`, the token-major
    layout reference), so run i is loop i; the whole-process --stats average mixes them with the
    flushed single launches."""
    rows = [r for r in csv.DictReader(open(path))]
    rows.sort(key=lambda r: int(r['Dispatch_Id']))
    runs, cur = [], []
    for r in rows:
        if needle in r['Kernel_Name']:
            cur.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
        else:
            if len(cur) >= 50:
                runs.append(cur)
            cur = []
    if len(cur) >= 50:
        runs.append(cur)
    names = [v for v in labels.split(',') if v] if labels else []
    lines = [f'Kernel `{needle}`: loops of >= 50 back-to-back launches (first 5 of each dropped)', '',
             '| loop | launches | avg us | min us | max us |', '|---|---|---|---|---|']
    for i, run in enumerate(runs):
        body = run[5:] if len(run) > 10 else run
        name = names[i] if i < len(names) else f'loop {i + 1}'
        lines.append(f'| {name} | {len(body)} | {sum(body) / len(body):.2f} | {min(body):.2f} | {max(body):.2f} |')
    open(out, 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines))


def _build_id():
    """The build id of the in-tree library the counters were collected with (bench.py accepts the
    traffic only for the same build)."""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from deepep_amd import _lib
    return _lib.binary_build_id(_lib.LIB_PATH)


def pmc(out, workload, algo_bytes, *paths):
    per = defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if 'combine_rows_kernel' not in r.get('Kernel_Name', ''):
                continue
            per[r['Counter_Name']].append(float(r['Counter_Value']))
    avg = {k: sum(v) / len(v) for k, v in per.items()}
    entry = {'counters_avg_per_launch': avg, 'algorithmic_bytes_per_launch': int(algo_bytes),
             'build_id': _build_id()}
    read = 2 * avg['FETCH_SIZE'] * 1024 if 'FETCH_SIZE' in avg else None
    write = avg['WRITE_SIZE'] * 1024 if 'WRITE_SIZE' in avg else None
    if read is not None and write is not None:
        entry['hbm_read_bytes_per_launch'] = read
        entry['hbm_write_bytes_per_launch'] = write
        entry['hbm_bytes_per_launch'] = read + write
        entry['traffic_over_algorithmic'] = (read + write) / int(algo_bytes)
    try:
        data = json.load(open(out))
    except (OSError, ValueError):
        data = {}
    data[workload] = entry
    json.dump(data, open(out, 'w'), indent=1, sort_keys=True)
    print(json.dumps({workload: entry}, indent=1))


def pmc_phases(out, meta_json, *paths):
    """Per-kernel HBM bytes of tools/pmc_phases.py's launches (kinds told apart by kernel name:
    combine_rows_kernel<2,...> fused, <0,...> local, <1,...> epilogue, copy_kernel), 2 x FETCH_SIZE +
    WRITE_SIZE (KiB) as in pmc(), against the algorithmic bytes the run recorded."""
    algo = json.load(open(meta_json))

    def kind(name):
        # the dispatch copy is `copy_kernel(...)`; torch's dtype conversions (`..._copy_kernel_cuda`) also
        # contain the substring, and counting them as the copy gave round 1's "anomaly"
        name = name[5:] if name.startswith('void ') else name
        if name.startswith('copy_kernel(') or name.startswith('copy_expanded_kernel<'):
            return 'copy'
        if 'combine_rows_kernel<2' in name:
            return 'fused'
        if 'combine_rows_kernel<0' in name:
            return 'local'
        if 'combine_rows_kernel<1' in name:
            return 'epilogue'
        return None
    per = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = kind(r.get('Kernel_Name', '').replace('(anonymous namespace)::', '').lstrip())
            if k is not None:
                per[k][r['Counter_Name']].append(float(r['Counter_Value']))
    res = {}
    for k, counters in per.items():
        avg = {c: sum(v) / len(v) for c, v in counters.items()}
        e = {'counters_avg_per_launch': avg, 'algorithmic_bytes_per_launch': algo[k], 'build_id': _build_id(),
             'launches': len(next(iter(counters.values())))}
        if 'TCC_EA0_RDREQ_sum' in avg and 'TCC_EA0_WRREQ_64B_sum' in avg:
            e['ea_read_bytes_per_launch (RDREQ x 128 B)'] = avg['TCC_EA0_RDREQ_sum'] * 128
            e['ea_write_bytes_per_launch (WRREQ_64B x 64 B)'] = avg['TCC_EA0_WRREQ_64B_sum'] * 64
        if 'FETCH_SIZE' in avg and 'WRITE_SIZE' in avg:
            e['hbm_read_bytes_per_launch'] = 2 * avg['FETCH_SIZE'] * 1024
            e['hbm_write_bytes_per_launch'] = avg['WRITE_SIZE'] * 1024
            e['traffic_over_algorithmic'] = (e['hbm_read_bytes_per_launch'] + e['hbm_write_bytes_per_launch']) / algo[k]
        res[k] = e
    json.dump(res, open(out, 'w'), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


def pmc_ep(out, meta_json, *paths):
    """Phase A (combine_rows_kernel<0,...>) HBM bytes of tools/pmc_ep.py's EP = N run (every rank's
    launches; the kernels are serialised under --pmc), 2 x FETCH_SIZE + WRITE_SIZE (KiB) as in pmc(),
    against the mean algorithmic bytes per launch bench.py's N > 1 roofline uses; folded into `out`
    (profiles/pmc_traffic.json) as phase_a_ep{N}_t{T}_h{H}_k{K}, with this build's id."""
    meta = json.load(open(meta_json))
    per = defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r.get('Kernel_Name', '').replace('(anonymous namespace)::', '').lstrip()
            if 'combine_rows_kernel<0' in name:
                per[r['Counter_Name']].append(float(r['Counter_Value']))
    avg = {c: sum(v) / len(v) for c, v in per.items()}
    algo = sum(meta['a_bytes']) / len(meta['a_bytes'])
    key = f"phase_a_ep{meta['world']}_t{meta['tokens']}_h{meta['hidden']}_k{meta['topk']}"
    entry = {'counters_avg_per_launch': avg, 'algorithmic_bytes_per_launch': algo, 'build_id': _build_id(),
             'launches': {c: len(v) for c, v in per.items()}, 'source': 'tools/pmc_ep.py (ranks simulated on one GPU)'}
    if 'FETCH_SIZE' in avg and 'WRITE_SIZE' in avg:
        entry['hbm_read_bytes_per_launch'] = 2 * avg['FETCH_SIZE'] * 1024
        entry['hbm_write_bytes_per_launch'] = avg['WRITE_SIZE'] * 1024
        entry['hbm_bytes_per_launch'] = entry['hbm_read_bytes_per_launch'] + entry['hbm_write_bytes_per_launch']
        entry['traffic_over_algorithmic'] = entry['hbm_bytes_per_launch'] / algo
    try:
        data = json.load(open(out))
    except (OSError, ValueError):
        data = {}
    data[key] = entry
    json.dump(data, open(out, 'w'), indent=1, sort_keys=True)
    print(json.dumps({key: entry}, indent=1))


def step(out, meta_json, *paths):
    """The whole EP = N combine step of tools/pmc_ep.py (every rank, ranks simulated on one GPU): HBM bytes
    of every kernel after the first 512 MB flush fill (the set-up -- inputs, dispatch -- runs before it) but
    the flushes, grouped as phase A (combine_rows_kernel<0), phase B (<1) and the exchange (the simulated
    all-to-all's copies), per step (the passes' totals / reps), 2 x FETCH_SIZE +
    WRITE_SIZE (KiB).  `diagonal_bytes` = what the own-rank rows cost when they travel (read + write of every
    rank's rows of itself); with the local bypass they do not."""
    meta = json.load(open(meta_json))
    tot = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(int)

    def kind(name):
        if 'combine_rows_kernel<0' in name:
            return 'phase_a'
        if 'combine_rows_kernel<1' in name:
            return 'phase_b'
        if 'fill' in name.lower():
            return None                      # the flush before every step
        return 'exchange'
    for p in paths:
        rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r['Dispatch_Id']))
        # the set-up (inputs, dispatch) runs before the first flush; every combine step follows a flush
        first = next((i for i, r in enumerate(rows) if kind(r.get('Kernel_Name', '')) is None), len(rows))
        for r in rows[first:]:
            k = kind(r.get('Kernel_Name', '').replace('(anonymous namespace)::', ''))
            if k is None:
                continue
            tot[k][r['Counter_Name']] += float(r['Counter_Value'])
            if r['Counter_Name'] == 'WRITE_SIZE':
                launches[k] += 1
    reps = meta['reps']
    res = {}
    for k, cs in tot.items():
        e = {}
        if 'FETCH_SIZE' in cs:
            e['read_bytes_per_step'] = 2 * cs['FETCH_SIZE'] * 1024 / reps
        if 'WRITE_SIZE' in cs:
            e['write_bytes_per_step'] = cs['WRITE_SIZE'] * 1024 / reps
        e['launches'] = launches.get(k, 0)
        res[k] = e
    total = sum(e.get('read_bytes_per_step', 0) + e.get('write_bytes_per_step', 0) for e in res.values())
    diag = 2 * sum(meta['own_rows']) * meta['packed_row_bytes']
    summary = dict(meta=meta, kernels=res, step_bytes=total, diagonal_bytes=diag,
                   exchanged_rows=sum(meta['sent_rows']) - (sum(meta['own_rows']) if meta['local_bypass'] else 0),
                   build_id=_build_id())
    json.dump(summary, open(out, 'w'), indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1))


def bykernel(out, *paths):
    """HBM bytes per launch of every combine_rows_kernel instantiation in PMC passes (2 x FETCH_SIZE +
    WRITE_SIZE, KiB), keyed by the kernel's template arguments: variants of one run told apart."""
    per = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r.get('Kernel_Name', '').replace('(anonymous namespace)::', '')
            if 'combine_rows_kernel<' not in name:
                continue
            key = name[name.index('combine_rows_kernel<'):].split('(')[0]
            per[key][r['Counter_Name']].append(float(r['Counter_Value']))
    res = {}
    for k, cs in per.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {'counters_avg_per_launch': avg, 'launches': {c: len(v) for c, v in cs.items()}}
        if 'FETCH_SIZE' in avg:
            e['hbm_read_bytes_per_launch'] = 2 * avg['FETCH_SIZE'] * 1024
        if 'WRITE_SIZE' in avg:
            e['hbm_write_bytes_per_launch'] = avg['WRITE_SIZE'] * 1024
        res[k] = e
    json.dump(dict(kernels=res, build_id=_build_id()), open(out, 'w'), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


def step_fold(out, step_json):
    """Fold a `step` summary into `out` (profiles/pmc_traffic.json) as step_ep{N}_t{T}_h{H}_k{K}: the HBM bytes
    per rank of one whole EP = N combine step by transport, with the build id -- what bench.py's N > 1 line
    reports as phases.hbm_bytes_per_rank (its own build only).
      rccl         every kernel of the step: phase A + the exchange's copies (on a real node RCCL's own read of
                   the send rows and write of the received rows) + phase B
      xgmi         phase A + phase B of the same passes: over the windows phase A stores each partial straight
                   into its owner's window row and phase B reads it there, so the exchange adds no HBM pass
                   (derived from the same counters, not a separate run)
      algorithmic  the combine's algorithmic bytes per rank (bench.py's `value` numerator)"""
    st = json.load(open(step_json))
    m = st['meta']
    n = m['world']
    k = st['kernels']

    def both(name):
        e = k.get(name, {})
        return e.get('read_bytes_per_step', 0.0) + e.get('write_bytes_per_step', 0.0)
    key = f"step_ep{n}_t{m['tokens']}_h{m['hidden']}_k{m['topk']}"
    entry = dict(build_id=st['build_id'], local_bypass=m['local_bypass'],
                 source='tools/pmc_ep.py + summarize_prof.py step (ranks simulated on one GPU, one chunk per rank)',
                 hbm_bytes_per_rank=dict(rccl=st['step_bytes'] / n, xgmi=(both('phase_a') + both('phase_b')) / n,
                                         algorithmic=sum(m['b_bytes']) / n),
                 kernels_bytes_per_step_all_ranks={name: both(name) for name in k})
    entry['hbm_bytes_per_rank']['rccl_over_xgmi'] = entry['hbm_bytes_per_rank']['rccl'] / entry['hbm_bytes_per_rank']['xgmi']
    try:
        data = json.load(open(out))
    except (OSError, ValueError):
        data = {}
    data[key] = entry
    json.dump(data, open(out, 'w'), indent=1, sort_keys=True)
    print(json.dumps({key: entry}, indent=1))


if __name__ == '__main__':
    if sys.argv[1] == 'step':
        step(sys.argv[2], sys.argv[3], *sys.argv[4:])
    elif sys.argv[1] == 'bykernel':
        bykernel(sys.argv[2], *sys.argv[3:])
    elif sys.argv[1] == 'stepfold':
        step_fold(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == 'ep':
        pmc_ep(sys.argv[2], sys.argv[3], *sys.argv[4:])
    elif sys.argv[1] == 'phases':
        pmc_phases(sys.argv[2], sys.argv[3], *sys.argv[4:])
    elif sys.argv[1] == 'stats':
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == 'timed':
        timed(sys.argv[2], sys.argv[3], sys.argv[4], *(sys.argv[5:6]))
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4], *sys.argv[5:])
