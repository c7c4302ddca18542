#!/usr/bin/env python3
"""Per-step time distribution (HIP events around every step on the env's
stream) and the DRAWING-wait counters for one config under several spawn-ahead
settings: what sets the tail of the step.

    python scripts/step_tail.py --cfg cfg5 --spawn-ahead 0 4 5 --draw-wait 200000 0
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402
from spawn_counters import CFGS  # noqa: E402

KEYS = ('resets_timed', 'spawn_hits', 'spawn_jobs', 'draw_wait', 'draw_timeout')


def run(cfg, thr, wait, steps, skip):
    N, S, kw = CFGS[cfg]
    _native.debug_set('draw_wait_ticks', wait)
    v = SnakeVecEnv(N, num_snakes=S, seed=0, spawn_ahead=thr, **kw)
    v.reset()
    g = torch.Generator(device='cuda').manual_seed(12345)
    acts = torch.randint(0, 3, (skip + steps, N, S), generator=g, device='cuda', dtype=torch.int8)
    for t in range(skip):
        v.step(acts[t])
    for k in KEYS:
        _native.timing_read(k)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    torch.cuda.synchronize()
    _native.timing_enable(True)
    ev[0].record()
    for t in range(steps):
        v.step(acts[skip + t])
        ev[t + 1].record()
    torch.cuda.synchronize()
    _native.timing_enable(False)
    dt = np.array([ev[t].elapsed_time(ev[t + 1]) * 1e3 for t in range(steps)])   # us
    cnt = {k: round(_native.timing_read(k)[1] / steps, 3) for k in KEYS}
    kp = _native.timing_read('k_post')
    v.close()
    _native.debug_set('draw_wait_ticks', 200000)
    return {'cfg': cfg, 'spawn_ahead': thr, 'draw_wait_ticks': wait, 'steps': steps,
            'step_us': {'mean': round(float(dt.mean()), 2), 'p50': round(float(np.percentile(dt, 50)), 2),
                        'p99': round(float(np.percentile(dt, 99)), 2), 'max': round(float(dt.max()), 2),
                        'n_over_2x_mean': int((dt > 2 * dt.mean()).sum())},
            'k_post_avg_us': round(kp[0] * 1e3 / max(kp[1], 1), 2), 'counters_per_step': cnt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cfg', default='cfg5')
    ap.add_argument('--spawn-ahead', type=int, nargs='+', default=[0])
    ap.add_argument('--draw-wait', type=int, nargs='+', default=[200000])
    ap.add_argument('--steps', type=int, default=1000)
    ap.add_argument('--skip', type=int, default=200)
    a = ap.parse_args()
    for thr in a.spawn_ahead:
        for w in a.draw_wait:
            print(json.dumps(run(a.cfg, thr, w, a.steps, a.skip)), flush=True)


if __name__ == '__main__':
    main()
