#!/usr/bin/env python3
"""Kernel-level timing probes (GPU): where does a step's time go?

Prints one JSON line per experiment: average device time per launch (HIP events
on the launch stream) of
  step_auto   -- SnakeVecEnv.step with all-done auto-reset (the bench workload)
  step_fresh  -- the first steps after a reset with autoreset off (no resets run)
  reset_all   -- snake_reset of every env (a whole batch of resets)
for a few batch sizes / configs.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]

import torch  # noqa: E402

from marlenv import SnakeVecEnv  # noqa: E402


def timed(fn, reps):
    s = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    return dict(mean_ms=round(sum(ts) / len(ts), 4), median_ms=round(ts[len(ts) // 2], 4),
                min_ms=round(ts[0], 4), max_ms=round(ts[-1], 4))


def probe(N, S, kw, reps, tag):
    g = torch.Generator(device='cuda').manual_seed(1)
    acts = torch.randint(0, 3, (max(reps, 64) + 200, N, S), generator=g, device='cuda', dtype=torch.int8)
    v = SnakeVecEnv(N, num_snakes=S, seed=0, **kw)
    out = {'tag': tag, 'N': N, 'S': S, **{k: v_ for k, v_ in kw.items() if k != 'reward_dict'}}
    out['reset_all'] = timed(lambda: v.reset(), 5)
    it = iter(range(10 ** 9))
    for t in range(200):
        v.step(acts[t])
    out['step_auto'] = timed(lambda: v.step(acts[200 + next(it) % reps]), reps)
    vf = SnakeVecEnv(N, num_snakes=S, seed=0, autoreset=False, **kw)
    vf.reset()
    it2 = iter(range(10 ** 9))
    out['step_fresh'] = timed(lambda: vf.step(acts[next(it2)]), 8)
    print(json.dumps(out), flush=True)
    del v, vf
    torch.cuda.empty_cache()


def probe_reset_latency(N=65536):
    """snake_reset over a mask of m envs out of N: latency of m concurrent resets."""
    kw = dict(height=20, width=20, snake_length=3, vision_range=5)
    v = SnakeVecEnv(N, num_snakes=4, seed=0, **kw)
    v.reset()
    out = {'tag': 'reset_mask', 'N': N}
    for m in (1, 16, 256, 1024, 4096, N):
        mask = torch.zeros(N, dtype=torch.bool, device='cuda')
        mask[torch.randperm(N, device='cuda')[:m]] = True
        out[f'm{m}'] = timed(lambda: v.reset(mask), 10)
    print(json.dumps(out), flush=True)
    small = SnakeVecEnv(64, num_snakes=4, seed=0, **kw)
    small.reset()
    g = torch.Generator(device='cuda').manual_seed(1)
    acts = torch.randint(0, 3, (400, 64, 4), generator=g, device='cuda', dtype=torch.int8)
    it = iter(range(10 ** 9))
    print(json.dumps({'tag': 'step_auto_N64', **timed(lambda: small.step(acts[next(it) % 400]), 300)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--quick', action='store_true')
    ap.add_argument('--reset-latency', action='store_true')
    a = ap.parse_args()
    if a.reset_latency:
        probe_reset_latency()
        return
    cfg3 = dict(height=20, width=20, snake_length=3, vision_range=5)
    for N in ((65536,) if a.quick else (4096, 16384, 65536, 262144)):
        probe(N, 4, cfg3, a.reps, 'cfg3')
    if not a.quick:
        probe(4096, 4, dict(height=20, width=20, snake_length=3), a.reps, 'cfg2_full')
        probe(8192, 8, dict(height=40, width=40, snake_length=3, vision_range=5, frame_stack=4), a.reps, 'cfg5_shard')


if __name__ == '__main__':
    main()
