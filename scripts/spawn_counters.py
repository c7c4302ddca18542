#!/usr/bin/env python3
"""Device-side spawn-ahead counters per step (the library's timing/diag mode):
resets, resets served by a ready record / a partial one, spawn-ahead jobs
run, ready records voided by a later fruit draw, k_logic respawns that
waited on a slow draw, steps whose background queue set was still busy
(gate_shut) and resets that waited for a record being drawn (draw_wait).

    python scripts/spawn_counters.py [--cfg cfg3 cfg5] [--steps 100 --skip 200]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]
import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402

CFGS = {'cfg3': (65536, 4, dict(height=20, width=20, vision_range=5)),
        'cfg4': (32768, 4, dict(height=20, width=20, vision_range=5)),
        'cfg2': (4096, 4, dict(height=20, width=20)),
        'cfg3s8': (8192, 4, dict(height=20, width=20, vision_range=5)),
        'cfg5': (8192, 8, dict(height=40, width=40, vision_range=5, frame_stack=4))}
KEYS = ('resets_timed', 'spawn_hits', 'reset_partial', 'spawn_jobs', 'spawn_void', 'respawn_slow', 'respawn_slow2', 'gate_shut', 'draw_wait', 'draw_timeout')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cfg', nargs='+', default=['cfg3', 'cfg5'])
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--skip', type=int, default=200)
    a = ap.parse_args()
    for cfg in a.cfg:
        N, S, kw = CFGS[cfg]
        v = SnakeVecEnv(N, num_snakes=S, seed=0, **kw)
        v.reset()
        g = torch.Generator(device='cuda').manual_seed(12345)
        for t in range(a.skip + a.steps):
            act = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
            if t == a.skip:
                for k in KEYS:
                    _native.timing_read(k)   # (reading clears)
                _native.timing_enable(True)
            v.step(act)
        _native.timing_enable(False)
        torch.cuda.synchronize()
        print(cfg, {k: round(_native.timing_read(k)[1] / a.steps, 3) for k in KEYS})
        v.close()


if __name__ == '__main__':
    main()
