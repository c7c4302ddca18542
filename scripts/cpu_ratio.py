#!/usr/bin/env python3
"""Speed ratio of the C restatement (oracle/snake_oracle.c) to the REAL reference
SnakeEnv, measured in THIS container (the reference cannot travel to the GPU box).

    python3 -B scripts/cpu_ratio.py [seconds]

Both run the same workload on one core: 20x20, 4 snakes, snake_length 3,
vision_range 5 (BASELINE config 3) and the full-map config 2, uniform random
actions, reset whenever all dones are True (the vector-env auto-reset), 16 envs
stepped round-robin. Writes profiles/cpu_ratio.json, which bench.py's
cpu_baseline leg reads to state the reference-equivalent rate next to the
measured C rate.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests', 'golden', 'gen', 'gymstub'), '/root/reference/marlenv']


def ref_rollout(kw, seconds, n_env=16, S=4):
    """The reference SnakeEnv (numpy's global RNG seeded per env at creation)."""
    from marlenv.envs.snake_env import SnakeEnv      # the reference (read-only import)
    envs = []
    for i in range(n_env):
        np.random.seed(i)
        envs.append(SnakeEnv(num_snakes=S, **kw))
    for e in envs:
        e.reset()
    rs = np.random.RandomState(12345)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        a = rs.randint(0, 3, size=(n_env, S))
        for i, e in enumerate(envs):
            _, _, d, _ = e.step([int(x) for x in a[i]])
            if all(d):
                e.reset()
        steps += n_env
    return steps / (time.perf_counter() - t0)


def ref_single(kw, seconds, S=4):
    """One reference env the way train_dqn.py drives it (reset when all done):
    ms per step() and per reset()."""
    from marlenv.envs.snake_env import SnakeEnv
    np.random.seed(0)
    e = SnakeEnv(num_snakes=S, **kw)
    e.reset()
    rs = np.random.RandomState(1)
    st = rt = 0.0
    n = nr = 0
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        a = [int(x) for x in rs.randint(0, 3, S)]
        t0 = time.perf_counter()
        _, _, d, _ = e.step(a)
        st += time.perf_counter() - t0
        n += 1
        if all(d):
            t0 = time.perf_counter()
            e.reset()
            rt += time.perf_counter() - t0
            nr += 1
    return {'step_ms': round(st / n * 1e3, 4), 'reset_ms': round(rt / max(nr, 1) * 1e3, 4), 'steps': n,
            'resets': nr}


def port_rollout(kw, seconds, n_env=16, S=4):
    """oracle/snake_oracle.c's so_rollout (no Python in the loop)."""
    from oracle.snake_oracle import rollout
    steps, n, t0 = 64, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        n += rollout(n_env, 0, steps, num_snakes=S, **kw)
        steps = min(steps * 2, 4096)
    return n / (time.perf_counter() - t0)


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    out = {}
    for name, kw in (('cfg3_20x20_s4_vr5', dict(height=20, width=20, snake_length=3, vision_range=5)),
                     ('cfg2_20x20_s4_full', dict(height=20, width=20, snake_length=3))):
        ref = ref_rollout(kw, seconds)
        port = port_rollout(kw, seconds)
        out[name] = {'reference_env_steps_per_s_1core': round(ref, 1),
                     'port_env_steps_per_s_1core': round(port, 1),
                     'port_over_reference': round(port / ref, 2)}
        print(name, out[name], flush=True)
    # the num_envs=1 path of train_dqn.py's Config (20x20, 4 snakes, length 5, full map)
    out['compat_train_dqn_reference'] = ref_single(dict(height=20, width=20, snake_length=5), seconds)
    print('compat', out['compat_train_dqn_reference'], flush=True)
    out['note'] = ('one core each, 16 envs round-robin, random actions, all-done resets included; '
                   'reference = /root/reference SnakeEnv under the offline gym stub '
                   '(tests/golden/gen/gymstub), port = oracle/snake_oracle.c so_rollout (C loop, xorshift actions)')
    with open(os.path.join(ROOT, 'profiles', 'cpu_ratio.json'), 'w') as fp:
        json.dump(out, fp, indent=1)


if __name__ == '__main__':
    main()
