#!/usr/bin/env python3
"""Per-step device time of the first steps after a full reset (the regime the
driver's short bench, --steps 20 --warmup 5, measures): ms per step, resets,
spawn-ahead hits/jobs, per kernel.

    python scripts/early_steps.py [--steps 40] [--N 65536] [--lib path] [--spawn-ahead k]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]

import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402


KERNELS = ('k_logic', 'k_post')
COUNTS = ('resets_timed', 'spawn_hits', 'spawn_jobs', 'spawn_void', 'reset_partial')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=40)
    ap.add_argument('--N', type=int, default=65536)
    ap.add_argument('--lib', default=None)
    ap.add_argument('--spawn-ahead', type=int, default=0)
    a = ap.parse_args()
    lib = os.path.abspath(a.lib) if a.lib else None
    L = _native.lib(lib)
    v = SnakeVecEnv(a.N, num_snakes=4, seed=0, lib_path=lib, height=20, width=20, snake_length=3, vision_range=5,
                    spawn_ahead=a.spawn_ahead)
    g = torch.Generator(device='cuda').manual_seed(12345)
    acts = torch.randint(0, 3, (a.steps, a.N, 4), generator=g, device='cuda', dtype=torch.int8)
    v.reset()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    rows = []
    for t in range(a.steps):
        for k in KERNELS + COUNTS:
            _native.timing_read(k, L)
        _native.timing_enable(True, L)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        v.step(acts[t])
        e1.record(s)
        _native.timing_enable(False, L)
        torch.cuda.synchronize()
        row = {'t': t, 'ms': round(e0.elapsed_time(e1), 4)}
        for k in KERNELS:
            row[k] = round(_native.timing_read(k, L)[0], 4)
        for k in COUNTS:
            row[k] = _native.timing_read(k, L)[1]
        rows.append(row)
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
