#!/usr/bin/env python3
"""Phase timeline of k_logic's block 0 (diagnostic build with -DSNAKE_STAMPS,
scripts/build_variants.sh stamps:-DSNAKE_STAMPS): s_memtime stamps at the phase
boundaries (LSTAMP 40..49) of one wave under the full step's load, per step,
medians over the steps (cycles from the wave's start).

    python scripts/logic_stamps.py marl-snake_amd/build/var/libsnake_stamps.so [--cfg cfg3] [--steps 200]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402

NAMES = {40: 'start', 41: 'rules', 42: 'second_round_issued', 43: 'grid_update', 44: 'dying_walk',
         45: 'respawn', 48: 'outputs', 49: 'stats', 46: 'queues', 47: 'records_stored'}
CFGS = {'cfg3': (65536, dict(height=20, width=20, vision_range=5)),
        'cfg2': (4096, dict(height=20, width=20))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('lib')
    ap.add_argument('--cfg', default='cfg3')
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--skip', type=int, default=100)
    a = ap.parse_args()
    L = _native.lib(os.path.abspath(a.lib))
    L.snake_debug_stamps.argtypes = [ctypes.c_void_p]
    N, kw = CFGS[a.cfg]
    v = SnakeVecEnv(N, num_snakes=4, seed=0, lib_path=os.path.abspath(a.lib), **kw)
    v.reset()
    g = torch.Generator(device='cuda').manual_seed(7)
    acts = torch.randint(0, 3, (a.skip + a.steps, N, 4), generator=g, device='cuda', dtype=torch.int8)
    buf = np.zeros(72, np.uint64)
    rows = []
    for t in range(a.skip + a.steps):
        v.step(acts[t])
        torch.cuda.synchronize()
        if t < a.skip:
            continue
        L.snake_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p))
        t0 = int(buf[40])
        rows.append({n: int(buf[i]) - t0 for i, n in NAMES.items() if buf[i]})
    med = {n: statistics.median(r[n] for r in rows if n in r) for n in NAMES.values() if any(n in r for r in rows)}
    order = sorted(med, key=med.get)
    print(json.dumps({'cfg': a.cfg, 'steps': len(rows), 'median_cycles_from_start': {n: med[n] for n in order}}))


if __name__ == '__main__':
    main()
