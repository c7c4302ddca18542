#!/usr/bin/env python3
"""HBM traffic per kernel launch from rocprofv3 PMC passes (gpu_check.sh `pmc`).

    python scripts/pmc_summary.py gpurun_out/pmcF gpurun_out/pmcW [--key SUFFIX] [--out profiles/pmc_traffic.json]

FETCH_SIZE and WRITE_SIZE are kilobytes per dispatch, each from its own pass
(they do not fit one TCC pass). Per /opt/skills/guides/MI355X_MICROARCH.md (HBM):
on gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads, so
it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores. The step kernels'
bulk traffic is exactly those two patterns (stage_to_lds / 16-B obs stores).
"""
import argparse
import csv
import json
import os
import re
import statistics


def per_kernel(path, counter):
    out = {}
    f = os.path.join(path, 'pmc_counter_collection.csv')
    for r in csv.DictReader(open(f)):
        if r['Counter_Name'] != counter:
            continue
        m = re.search(r'snake::(k_\w+)', r['Kernel_Name'])
        if not m:
            continue
        out.setdefault(m.group(1), []).append(float(r['Counter_Value']))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch_dir')
    ap.add_argument('write_dir')
    ap.add_argument('--key', default='20x20_S4_vr5_fs1_N65536')
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    fe, wr = per_kernel(a.fetch_dir, 'FETCH_SIZE'), per_kernel(a.write_dir, 'WRITE_SIZE')
    res = {}
    for k in sorted(set(fe) | set(wr)):
        rd = 2.0 * 1024 * statistics.mean(fe[k]) if k in fe else None
        wb = 1024 * statistics.mean(wr[k]) if k in wr else None
        res[f'{k}_{a.key}'] = {
            'kernel': k, 'dispatches': max(len(fe.get(k, [])), len(wr.get(k, []))),
            'read_bytes_per_launch': round(rd) if rd is not None else None,
            'write_bytes_per_launch': round(wb) if wb is not None else None,
            'hbm_bytes_per_launch': round(rd + wb) if rd is not None and wb is not None else None,
            'note': 'FETCH_SIZE x2 (gfx950 16-B streaming-read correction) + WRITE_SIZE, KB x 1024',
        }
    text = json.dumps(res, indent=1)
    print(text)
    if a.out:
        old = json.load(open(a.out)) if os.path.exists(a.out) else {}
        old.update(res)
        with open(a.out, 'w') as fh:
            json.dump(old, fh, indent=1)
            fh.write('\n')


if __name__ == '__main__':
    main()
