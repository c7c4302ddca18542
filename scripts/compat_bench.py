#!/usr/bin/env python3
"""Time the num_envs=1 compat path every reference caller uses
(make_snake(num_envs=1, ...) then env.reset()/env.step(), train_dqn.py:187-188,287;
test_env.py:3-25): host list actions in, numpy obs / list rewards out, numpy's
global RNG synced every call. Config = train_dqn.py's Config (20x20, 4 snakes,
snake_length 5, full-map observation).

    python scripts/compat_bench.py [--steps 3000] [--root DIR]

--root points at another checkout's repo root (A/B against an older tree).
"""
import argparse
import json
import os
import sys
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=3000)
    ap.add_argument('--root', default=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    ap.add_argument('--vision-range', type=int, default=0)
    a = ap.parse_args()
    sys.path[:0] = [os.path.join(a.root, 'marl-snake_amd'), a.root]
    import numpy as np
    from marlenv.wrappers import make_snake

    np.random.seed(0)
    env, _, _, props = make_snake(num_envs=1, num_snakes=4, height=20, width=20, snake_length=5,
                                  vision_range=a.vision_range or None)
    S = props['num_snakes']
    rs = np.random.RandomState(1)
    obs = env.reset()
    for _ in range(50):                                  # warm up (first launches, allocator)
        _, _, done, _ = env.step([int(x) for x in rs.randint(0, 3, S)])
        if all(done):
            env.reset()
    step_t, reset_t, n_reset = 0.0, 0.0, 0
    for _ in range(a.steps):
        acts = [int(x) for x in rs.randint(0, 3, S)]
        t0 = time.perf_counter()
        obs, rew, done, info = env.step(acts)
        step_t += time.perf_counter() - t0
        if all(done):
            t0 = time.perf_counter()
            obs = env.reset()
            reset_t += time.perf_counter() - t0
            n_reset += 1
    print(json.dumps({'root': a.root, 'obs_shape': list(np.asarray(obs).shape), 'steps': a.steps,
                      'step_ms': round(step_t / a.steps * 1e3, 4),
                      'reset_ms': round(reset_t / max(n_reset, 1) * 1e3, 4), 'resets': n_reset,
                      'env_steps_per_s': round(a.steps / (step_t + reset_t), 1)}), flush=True)


if __name__ == '__main__':
    main()
