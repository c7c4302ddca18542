#!/usr/bin/env python3
"""Interleaved A/B of bench.py runs on one box: each spec is
    name=[VAR=value,VAR=value;]bench args
run `--rounds` times in turn (so box drift hits every variant alike), each in
its own process under a time limit; prints one summary line per run and the
per-variant medians, and writes every JSON line to <out>/ab.jsonl.

    python scripts/ab.py --out gpurun_out/ab 'old=--config cfg3 --spawn-ahead 3' 'new=--config cfg3'
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse(spec):
    name, rest = spec.split('=', 1)
    env = {}
    if ';' in rest:
        ev, rest = rest.split(';', 1)
        for kv in ev.split(','):
            k, v = kv.split('=', 1)
            env[k] = v
    return name, env, rest.split()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--timeout', type=int, default=240)
    ap.add_argument('specs', nargs='+')
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    specs = [parse(s) for s in a.specs]
    res = {n: [] for n, _, _ in specs}
    with open(os.path.join(a.out, 'ab.jsonl'), 'a') as fp:
        for r in range(a.rounds):
            for name, env, args in specs:
                cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--no-cpu-baseline'] + args
                p = subprocess.run(cmd, env=dict(os.environ, **env), capture_output=True, text=True,
                                   timeout=a.timeout, cwd=ROOT)
                if p.returncode != 0:
                    print(f'{name}: rc {p.returncode}\n{p.stderr[-2000:]}', flush=True)
                    sys.exit(3)
                d = json.loads(p.stdout.strip().splitlines()[-1])
                d['ab_name'], d['ab_round'] = name, r
                fp.write(json.dumps(d) + '\n')
                fp.flush()
                sa = d.get('spawn_ahead') or {}
                res[name].append(d['ms_per_step'])
                k = d['kernels']
                print(f"{name:14s} r{r} {d['ms_per_step']:.4f} ms  logic {k['k_logic'] * 1e3:5.1f} post "
                      f"{k['k_post'] * 1e3:5.1f} us  jobs {sa.get('jobs_per_step')} hits {sa.get('hits_per_step')} "
                      f"void {sa.get('ready_voided_per_step')} part {sa.get('resets_from_partial_per_step')} "
                      f"miss {sa.get('resets_without_record_per_step')} hit {sa.get('hit_rate')}", flush=True)
    for name in res:
        print(f'median {name:14s} {statistics.median(res[name]):.4f} ms  {res[name]}', flush=True)


if __name__ == '__main__':
    main()
