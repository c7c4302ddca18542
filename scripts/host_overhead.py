#!/usr/bin/env python3
"""Host cost of SnakeVecEnv.step: the time one call takes to
enqueue its work (no synchronisation inside the measured calls), split into
its parts, at cfg2 and cfg3 sizes. Prints one JSON line.

    python scripts/host_overhead.py [--steps 300]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'marl-snake_amd'))


def per_call(fn, n):
    """median and mean wall time of n back-to-back calls, in microseconds."""
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 2), round(sum(ts) / len(ts) * 1e6, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=300)
    args = ap.parse_args()
    import torch
    from marlenv import SnakeVecEnv
    out = {}
    for name, N, kw in (('cfg2', 4096, dict(height=20, width=20)),
                        ('cfg3s8', 8192, dict(height=20, width=20, vision_range=5)),
                        ('cfg3', 65536, dict(height=20, width=20, vision_range=5))):
        v = SnakeVecEnv(N, num_snakes=4, seed=0, **kw)
        v.reset()
        g = torch.Generator(device='cuda').manual_seed(1)
        acts = torch.randint(0, 3, (args.steps + 64, N, 4), generator=g, device='cuda', dtype=torch.int8)
        for t in range(64):
            v.step(acts[t])
        torch.cuda.synchronize()
        it = iter(range(64, 64 + args.steps))
        r = {'step_enqueue_us': per_call(lambda: v.step(acts[next(it)]), args.steps)}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(args.steps):
            v.step(acts[t])
        torch.cuda.synchronize()
        r['step_wall_us'] = round((time.perf_counter() - t0) / args.steps * 1e6, 2)
        # the parts: one output slab; the C-ABI call alone on fixed outputs
        r['slab_alloc_us'] = per_call(lambda: torch.empty(v._slab_bytes, dtype=torch.uint8, device='cuda'),
                                      args.steps)
        slab, so = v._new_out()
        a = acts[0]
        L, cfg, st = v._L, ctypes.byref(v.cfg), ctypes.byref(v._state)
        stream = torch._C._cuda_getCurrentRawStream(0)
        torch.cuda.synchronize()
        r['capi_step_us'] = per_call(lambda: L.snake_step(cfg, st, N, a.data_ptr(), ctypes.byref(so), stream),
                                     args.steps)
        torch.cuda.synchronize()
        r['info_read_us'] = per_call(lambda: v.step(acts[1])[3]['rank'], 50)
        torch.cuda.synchronize()
        out[name] = r
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
