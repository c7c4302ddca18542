#!/usr/bin/env python3
"""Collect one scripts/profile_set.sh run into profiles/: the bench lines, the
rocprofv3 kernel-stats summaries per config, PMC HBM traffic (FETCH_SIZE x2 +
WRITE_SIZE, scripts/pmc_summary.py), SQ counters per launch and the spawn-ahead
counters.

    python scripts/collect_set.py gpurun_out/r05 --tag r05
"""
import argparse
import csv
import json
import os
import re
import shutil
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import per_kernel  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def last_json(path):
    lines = [x for x in open(path) if x.startswith('{"metric"')]
    return json.loads(lines[-1]) if lines else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('run')
    ap.add_argument('--tag', required=True)
    a = ap.parse_args()
    prof = os.path.join(ROOT, 'profiles')
    lines = {'note': f'scripts/profile_set.sh on one MI355X ({a.run}); bench_<cfg>: --steps 2000 --warmup 200; '
                     'driverwin: the driver\'s --steps 20 --warmup 5 with the CPU baseline'}
    for name in sorted(os.listdir(a.run)):
        m = re.match(r'(bench_\w+|driverwin)\.log$', name)
        if m:
            lines[m.group(1)] = last_json(os.path.join(a.run, name))
    with open(os.path.join(prof, f'{a.tag}_bench_lines.json'), 'w') as fh:
        json.dump(lines, fh, indent=1)
        fh.write('\n')
    stats = {}
    for name in sorted(os.listdir(a.run)):
        m = re.match(r'prof_(\w+)$', name)
        if not m:
            continue
        src = os.path.join(a.run, name, 'run_kernel_stats.csv')
        if os.path.exists(src):
            dst = os.path.join(prof, f'{a.tag}_{m.group(1)}_kernel_stats.csv')
            shutil.copy(src, dst)
            for r in csv.DictReader(open(src)):
                k = re.search(r'snake::(k_\w+)', r['Name'])
                if k:
                    stats.setdefault(m.group(1), {})[k.group(1)] = {
                        'calls': int(r['Calls']), 'avg_us': round(float(r['AverageNs']) / 1e3, 2),
                        'min_us': round(float(r['MinNs']) / 1e3, 2), 'max_us': round(float(r['MaxNs']) / 1e3, 2)}
    traffic, sq = {'note': 'per launch; FETCH_SIZE x2 (gfx950 16-B streaming-read correction) + WRITE_SIZE, KB x 1024'}, \
        {'note': 'rocprofv3 --pmc SQ_* pass, per-launch averages (bench.py --steps 40 --warmup 60 --timing-stride 0)'}
    for name in sorted(os.listdir(a.run)):
        m = re.match(r'pmcF_(\w+)$', name)
        if m and os.path.isdir(os.path.join(a.run, f'pmcW_{m.group(1)}')):
            c = m.group(1)
            fe = per_kernel(os.path.join(a.run, name), 'FETCH_SIZE')
            wr = per_kernel(os.path.join(a.run, f'pmcW_{c}'), 'WRITE_SIZE')
            for k in sorted(set(fe) | set(wr)):
                rd = 2048 * statistics.mean(fe[k]) if k in fe else None
                wb = 1024 * statistics.mean(wr[k]) if k in wr else None
                traffic[f'{k}_{c}'] = {'dispatches': len(fe.get(k, [])), 'read_bytes_per_launch': round(rd) if rd else None,
                                       'write_bytes_per_launch': round(wb) if wb else None,
                                       'hbm_bytes_per_launch': round(rd + wb) if rd and wb else None}
        m = re.match(r'pmcSQ_(\w+)$', name)
        if m:
            f = os.path.join(a.run, name, 'pmc_counter_collection.csv')
            acc = {}
            for r in csv.DictReader(open(f)):
                k = re.search(r'snake::(k_\w+)', r['Kernel_Name'])
                if k:
                    acc.setdefault(k.group(1), {}).setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
            for k, d in acc.items():
                sq[f'{k}_{m.group(1)}'] = {n: round(statistics.mean(v)) for n, v in sorted(d.items())}
                sq[f'{k}_{m.group(1)}']['dispatches'] = max(len(v) for v in d.values())
    for fn, obj in ((f'{a.tag}_kernel_stats.json', stats), (f'{a.tag}_pmc_traffic.json', traffic), (f'{a.tag}_pmc_sq.json', sq)):
        with open(os.path.join(prof, fn), 'w') as fh:
            json.dump(obj, fh, indent=1)
            fh.write('\n')
    cnt = os.path.join(a.run, 'counters.log')
    if os.path.exists(cnt):   # (scripts/spawn_counters.py's lines only)
        with open(os.path.join(prof, f'{a.tag}_spawn_counters.txt'), 'w') as fh:
            fh.writelines(x for x in open(cnt) if x.startswith('cfg'))
    # the bench line's dominant-kernel average against rocprof's
    for c, ln in lines.items():
        if isinstance(ln, dict) and c.startswith('bench_'):
            cfg = c[len('bench_'):]
            rk = ln['roofline']['kernel']
            rp = stats.get(cfg, {}).get(rk) or stats.get(cfg, {}).get(rk + '_lean')
            print(f"{cfg}: {ln['ms_per_step']} ms/step, {ln['value'] / 1e6:.1f} M env-steps/s, {rk} bench "
                  f"{ln['roofline']['kernel_ms'] * 1e3:.1f} us vs rocprof {rp['avg_us'] if rp else None} us, "
                  f"frac {ln['roofline']['frac']}")
    for k, v in traffic.items():
        if k != 'note':
            print(k, v)


if __name__ == '__main__':
    main()
