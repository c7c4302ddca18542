#!/usr/bin/env python3
"""hipGraph replay of SnakeVecEnv.step vs eager stepping: the
whole step (k_logic, the fork, k_autoreset beside k_encode, the join) captured
once through torch.cuda.graph and replayed on fixed action/output buffers, at
cfg2 and cfg3 sizes. Prints one JSON line of ms/step per mode.

    python scripts/graph_probe.py [--steps 400]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'marl-snake_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=400)
    args = ap.parse_args()
    import torch
    from marlenv import SnakeVecEnv
    out = {}
    for name, N, kw in (('cfg2', 4096, dict(height=20, width=20)),
                        ('cfg3', 65536, dict(height=20, width=20, vision_range=5))):
        v = SnakeVecEnv(N, num_snakes=4, seed=0, spawn_background=-1, **kw)
        v.reset()
        g = torch.Generator(device='cuda').manual_seed(1)
        acts = torch.randint(0, 3, (args.steps, N, 4), generator=g, device='cuda', dtype=torch.int8)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        r = {}
        with torch.cuda.stream(s):
            for t in range(50):                      # warm up (and the side stream of `s`)
                v.step(acts[t])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for t in range(args.steps):
                v.step(acts[t])
            torch.cuda.synchronize()
            r['eager_ms'] = round((time.perf_counter() - t0) / args.steps * 1e3, 4)
            static_a = acts[0].clone()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=s):
                o, rew, done, info = v.step(static_a)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for t in range(args.steps):
                static_a.copy_(acts[t])
                graph.replay()
            torch.cuda.synchronize()
            r['graph_ms'] = round((time.perf_counter() - t0) / args.steps * 1e3, 4)
        out[name] = r
        del v
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
