#!/usr/bin/env python3
"""In-process A/B timing of libsnake_amd.so builds (cdna_hip_programming.md
rule 24: interleaved rounds in one process, report median and min).

    python scripts/ab_probe.py marl-snake_amd/build/var/libsnake_v2.so ... [--N 65536]

Per library: one env batch in the bench configuration; every round times
`--steps` auto-reset steps (the bench workload) and 8 steps right after a
reset with autoreset off (no resets run: the pure step).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]

import torch  # noqa: E402

from marlenv import SnakeVecEnv  # noqa: E402


HOST = {}


def timed(fn, reps, key=None):
    """Device ms per call; the host's enqueue ms per call goes to HOST[key] (when
    it approaches the device time the loop is host-bound)."""
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    b.record(s)
    torch.cuda.synchronize()
    if key is not None:
        HOST.setdefault(key, []).append((t1 - t0) * 1e3 / reps)
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('libs', nargs='+')
    ap.add_argument('--N', type=int, default=65536)
    ap.add_argument('--rounds', type=int, default=8)
    ap.add_argument('--steps', type=int, default=40)
    ap.add_argument('--cfg', default='cfg3')
    a = ap.parse_args()
    cfgs = {'cfg3': (4, dict(height=20, width=20, snake_length=3, vision_range=5)),
            'cfg2': (4, dict(height=20, width=20, snake_length=3)),
            'cfg5': (8, dict(height=40, width=40, snake_length=3, vision_range=5, frame_stack=4))}
    S, kw = cfgs[a.cfg]
    N = a.N
    g = torch.Generator(device='cuda').manual_seed(12345)
    acts = torch.randint(0, 3, (256, N, S), generator=g, device='cuda', dtype=torch.int8)
    envs = {}
    for p in a.libs:
        v = SnakeVecEnv(N, num_snakes=S, seed=0, lib_path=os.path.abspath(p), **kw)
        v.reset()
        for t in range(200):
            v.step(acts[t % 256])
        f = SnakeVecEnv(N, num_snakes=S, seed=0, autoreset=False, lib_path=os.path.abspath(p), **kw)
        envs[p] = (v, f)
    res = {p: {'auto': [], 'fresh': []} for p in a.libs}
    ctr = [0]

    def nxt():
        ctr[0] += 1
        return acts[ctr[0] % 256]
    for r in range(a.rounds):
        for p in a.libs:
            v, f = envs[p]
            res[p]['auto'].append(timed(lambda: v.step(nxt()), a.steps, key=p))
            f.reset()
            res[p]['fresh'].append(timed(lambda: f.step(nxt()), 8))
    out = {'N': N, 'cfg': a.cfg}
    for p in a.libs:
        out[os.path.basename(p)] = {k: {'median_ms': round(statistics.median(x), 4), 'min_ms': round(min(x), 4)}
                                    for k, x in res[p].items()}
        out[os.path.basename(p)]['auto']['host_enqueue_ms'] = round(statistics.median(HOST[p]), 4)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
