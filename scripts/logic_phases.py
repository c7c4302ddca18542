#!/usr/bin/env python3
"""Which phase makes k_logic's slow waves slow (diagnostic build with
-DSNAKE_STAMPS): every wave's s_memrealtime at each phase boundary (LSTAMP),
per step after --skip steps; phase durations of the slowest decile of waves
against the median wave, and the start-time spread.

    python scripts/logic_phases.py marl-snake_amd/build/var/libsnake_stamps.so [--cfg cfg3]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402

CFGS = {'cfg3': (65536, 4, dict(height=20, width=20, vision_range=5)),
        'cfg4': (32768, 4, dict(height=20, width=20, vision_range=5)),
        'cfg2': (4096, 4, dict(height=20, width=20)),
        'cfg5': (8192, 8, dict(height=40, width=40, vision_range=5, frame_stack=4))}
# LSTAMP indices in program order and the phase that ends at each
ORDER = [40, 51, 52, 41, 42, 43, 44, 45, 48, 49, 46, 47]
PHASES = ['stage_grid', 'load_stats', 'rules', 'second_round', 'grid_update', 'dying_walk', 'respawn',
          'outputs', 'queues', 'stats', 'commit_records']
KWT = 8192


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('lib')
    ap.add_argument('--cfg', default='cfg3')
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--skip', type=int, default=200)
    a = ap.parse_args()
    lib = os.path.abspath(a.lib)
    L = _native.lib(lib)
    L.snake_debug_wphase.argtypes = [ctypes.c_void_p]
    N, S, kw = CFGS[a.cfg]
    v = SnakeVecEnv(N, num_snakes=S, seed=0, lib_path=lib, **kw)
    v.reset()
    g = torch.Generator(device='cuda').manual_seed(12345)
    acts = torch.randint(0, 3, (a.skip + a.steps, N, S), generator=g, device='cuda', dtype=torch.int8)
    buf = np.zeros(16 * KWT, np.uint64)
    slow, med, starts, spans, totals = [], [], [], [], []
    for t in range(a.skip + a.steps):
        v.step(acts[t])
        torch.cuda.synchronize()
        if t < a.skip:
            continue
        L.snake_debug_wphase(buf.ctypes.data_as(ctypes.c_void_p))
        w = buf.reshape(KWT, 16).astype(np.int64)
        cols = np.stack([w[:, i - 40] for i in ORDER], 1)
        used = (cols > 0).all(1)
        cols = cols[used] * 10                        # ns
        t0 = cols[:, 0].min()
        dur = np.diff(cols, axis=1)                   # (waves, phases)
        tot = cols[:, -1] - cols[:, 0]
        order = np.argsort(tot)
        k = max(1, len(tot) // 10)
        slow.append(dur[order[-k:]].mean(0))
        med.append(np.median(dur, 0))
        starts.append(np.percentile(cols[:, 0] - t0, [50, 90, 100]))
        spans.append(cols[:, -1].max() - t0)
        totals.append(np.percentile(tot, [10, 50, 90, 100]))
    slow, med = np.mean(slow, 0), np.mean(med, 0)
    out = dict(cfg=a.cfg, steps=a.steps,
               span_ns=float(np.median(spans)),
               wave_start_ns_p50_p90_max=[float(x) for x in np.median(starts, 0)],
               wave_dur_ns_p10_p50_p90_max=[float(x) for x in np.median(totals, 0)],
               phases_ns={p: dict(median_wave=round(float(m)), slowest_decile=round(float(s)))
                          for p, m, s in zip(PHASES, med, slow)})
    print(json.dumps(out))


if __name__ == '__main__':
    main()
