#!/usr/bin/env python3
"""Per-step timeline of the step kernels from a rocprofv3 --kernel-trace CSV:
median duration of each kernel and median gap from each kernel's end to the
next kernel's start (same step order), over the last --last launches.

    python scripts/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv
"""
import argparse
import collections
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--last', type=int, default=300)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.csv)) if 'snake::' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    rows = rows[-a.last:]
    ev = [(r['Kernel_Name'].split('snake::')[1].split('(')[0].split('<')[0],
           int(r['Start_Timestamp']) / 1e3, int(r['End_Timestamp']) / 1e3) for r in rows]
    dur, gap = collections.defaultdict(list), collections.defaultdict(list)
    for i, (n, s, e) in enumerate(ev):
        dur[n].append(e - s)
        if i + 1 < len(ev):
            gap[f'{n}->{ev[i + 1][0]}'].append(ev[i + 1][1] - e)
    starts = [s for n, s, e in ev if n == 'k_logic']
    per_step = statistics.median([b - a for a, b in zip(starts, starts[1:])]) if len(starts) > 1 else None
    print(json.dumps({'step_us': round(per_step, 2) if per_step is not None else None,
                      'dur_us': {k: round(statistics.median(v), 1) for k, v in dur.items()},
                      'gap_us': {k: round(statistics.median(v), 1) for k, v in gap.items()}}))


if __name__ == '__main__':
    main()
