#!/usr/bin/env python3
"""Golden-fixture generator: runs the REAL reference SnakeEnv in this container.

Run (container only -- /root/reference does not exist on the GPU box):

    python3 -B tests/golden/gen/make_golden.py

It imports ``marlenv.envs.snake_env.SnakeEnv`` from
/root/reference/marlenv (read-only; -B keeps bytecode out of it) through the
offline gym stub next to this file, drives it with recorded action sequences
and writes small fixtures (inputs + outputs only, no reference source) to
tests/golden/:

* rng.npz          -- numpy legacy RandomState (MT19937) vectors: raw 32-bit
                      stream, randint(0,n,size=k), permutation(n); the three
                      RNG entry points the env uses (snake_env.py:581,
                      grid_util.py:130 via np.random.seed).
* candidates.npz   -- dfs_sweep_empty(make_grid(H,W), L) tables / digests
                      (grid_util.py:14-20, 73-115).
* traj_<name>.npz  -- seeded trajectories: per-step rewards, dones, grids,
                      obs digests, episode info at all-done, reset grids.
* crafted.json     -- hand-built states injected into env.grid/env.snakes,
                      then stepped: head-on, tail entry, fruit-eater tail rule,
                      double decrement, self-kill, win, truncation, dead crop,
                      human observer.

The parity contract these pin: env i of a batch ==
a standalone SnakeEnv after np.random.seed(seed_i), actions supplied
externally, reset() called right after a step whose dones are all True.
"""
import base64
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(HERE, 'gymstub'), '/root/reference/marlenv']

from marlenv.envs.snake_env import SnakeEnv  # noqa: E402
from marlenv.envs.coop_snake_env import CoopSnakeEnv  # noqa: E402
from marlenv.core.snake import Snake  # noqa: E402
from marlenv.core import grid_util  # noqa: E402


def digest(arr):
    """8-byte blake2b of the C-contiguous bytes, as a python int."""
    a = np.ascontiguousarray(arr)
    return int.from_bytes(hashlib.blake2b(a.tobytes(), digest_size=8).digest(), 'little')


# ---------------------------------------------------------------- RNG vectors
def make_rng():
    seeds = [0, 1, 7, 12345, 2**32 - 1]
    raw = np.stack([np.random.RandomState(s)._bit_generator.random_raw(1500).astype(np.uint32)
                    for s in seeds])
    ri_cases = [(0, 1, 5), (0, 2, 9), (1, 397, 4), (7, 1000, 7), (12345, 65536, 3),
                (12345, 65537, 3), (2**32 - 1, 3, 30), (1, 2**31 + 5, 4)]
    ri_out, ri_next = [], []
    for s, n, k in ri_cases:
        np.random.seed(s)
        ri_out.append(np.random.randint(0, n, size=k).astype(np.int64))
        # randint(0, 2**32) is one raw draw: pins how many draws the case consumed
        ri_next.append(int(np.random.randint(0, 2**32, dtype=np.uint64)))
    perm_cases = [(0, 2), (1, 5), (7, 64), (12345, 100), (0, 3464), (3, 16424), (9, 26184)]
    perm_head, perm_digest, perm_next = [], [], []
    for s, n in perm_cases:
        np.random.seed(s)
        p = np.random.permutation(n).astype(np.int64)
        perm_head.append(np.pad(p[:16], (0, 16 - min(16, n)), constant_values=-1))
        perm_digest.append(digest(p))
        perm_next.append(int(np.random.randint(0, 2**32, dtype=np.uint64)))
    np.savez_compressed(
        os.path.join(OUT, 'rng.npz'),
        seeds=np.array(seeds, np.uint64), raw=raw,
        ri_cases=np.array(ri_cases, np.uint64), ri_out=np.concatenate(ri_out),
        ri_next=np.array(ri_next, np.uint64),
        perm_cases=np.array(perm_cases, np.uint64), perm_head=np.stack(perm_head),
        perm_digest=np.array(perm_digest, np.uint64), perm_next=np.array(perm_next, np.uint64))


# ---------------------------------------------------------- candidate tables
def cand_array(H, W, L):
    grid = grid_util.make_grid(H, W, empty_value=0, wall_value=1)
    cands = grid_util.dfs_sweep_empty(grid, L)
    return np.array(cands, dtype=np.int16).reshape(len(cands), L, 2)


def make_candidates():
    out = {}
    for H, W, L in [(6, 6, 2), (10, 10, 3), (20, 20, 3), (8, 8, 2), (12, 12, 3)]:
        out[f'full_{H}x{W}_L{L}'] = cand_array(H, W, L)
    meta = []
    for H, W, L in [(40, 40, 3), (20, 20, 5), (12, 12, 4), (20, 20, 3), (10, 10, 3)]:
        a = cand_array(H, W, L)
        meta.append((H, W, L, a.shape[0], digest(a)))
    out['digest_meta'] = np.array(meta, dtype=np.uint64)
    np.savez_compressed(os.path.join(OUT, 'candidates.npz'), **out)


# --------------------------------------------------------------- trajectories
def greedy_actions(env, rs, eps):
    """Fruit-seeking, death-avoiding policy (only to grow long snakes)."""
    acts = []
    fr = np.argwhere(env.grid == 2)
    n_act = len(env.action_dict)
    for sn in env.snakes:
        if not sn.alive or rs.rand() < eps or len(fr) == 0:
            acts.append(int(rs.randint(n_act)))
            continue
        best, best_a = None, 0
        for a in range(n_act):
            if env.observer == 'human':
                d = env._next_direction_global(sn.direction, a)
            else:
                d = env._next_direction(sn.direction, a)
            nh = sn.head_coord + d
            v = env.grid[nh] % 10
            safe = v in (0, 2, 5)
            dist = np.abs(fr - np.array(nh)).sum(1).min()
            key = (0 if safe else 1, dist, rs.rand())
            if best is None or key < best:
                best, best_a = key, a
        acts.append(best_a)
    return acts


def run_traj(name, T, seed, policy='random', eps=0.1, full_obs_every=0, coop=False, **kw):
    np.random.seed(seed)
    env = (CoopSnakeEnv if coop else SnakeEnv)(**kw)
    S = env.num_snakes
    n_act = len(env.action_dict)
    rs = np.random.RandomState(seed + 100003)
    obs0 = env.reset()
    H, W = env.grid_shape
    rec = dict(actions=[], rews=[], dones=[], grids=[], obs_digest=[], alive_snakes=[],
               heads=[], alive=[], reset_at=[], ep_len=[])
    resets = dict(grid=[env.grid.astype(np.int8).copy()], obs_digest=[digest(obs0)])
    infos = dict(step=[], rank=[], scores=[], steps=[], fruits=[], kills=[])
    full_obs_steps, full_obs = [], []
    for t in range(T):
        if policy == 'random':
            acts = [int(a) for a in rs.randint(0, n_act, size=S)]
        else:
            acts = greedy_actions(env, rs, eps)
        obs, rews, dones, info = env.step(list(acts))
        rec['actions'].append(acts)
        rec['rews'].append([float(r) for r in rews])
        rec['dones'].append(list(dones))
        rec['grids'].append(env.grid.astype(np.int8).copy())
        rec['obs_digest'].append(digest(obs))
        rec['alive_snakes'].append(env.alive_snakes)
        rec['heads'].append([sn.head_coord for sn in env.snakes])
        rec['alive'].append([sn.alive for sn in env.snakes])
        rec['ep_len'].append(env.episode_length)
        if full_obs_every and t % full_obs_every == 0:
            full_obs_steps.append(t)
            full_obs.append(obs.copy())
        if info:
            infos['step'].append(t)
            infos['rank'].append([int(x) for x in info['rank']])
            infos['scores'].append(np.asarray(info['episode_scores'], np.float64))
            infos['steps'].append(np.asarray(info['episode_steps'], np.float64))
            infos['fruits'].append(np.asarray(info['episode_fruits'], np.float64))
            infos['kills'].append(np.asarray(info['episode_kills'], np.float64))
        if all(dones):
            rec['reset_at'].append(True)
            o = env.reset()
            resets['grid'].append(env.grid.astype(np.int8).copy())
            resets['obs_digest'].append(digest(o))
        else:
            rec['reset_at'].append(False)
    cfg = dict(height=kw.get('height', 20), width=kw.get('width', 20), num_snakes=S,
               snake_length=env.snake_length, vision_range=env.vision_range,
               frame_stack=env.frame_stack, observer=env.observer,
               reward_dict=env.reward_dict, num_fruits=env.num_fruits,
               max_episode_steps=float(env.max_episode_steps))
    if coop:
        cfg['coop'] = True
    f = lambda k, dt: np.array(rec[k], dtype=dt)  # noqa: E731
    np.savez_compressed(
        os.path.join(OUT, f'traj_{name}.npz'),
        config=np.array(json.dumps(cfg)), seed=np.uint64(seed), policy=np.array(policy),
        obs0=obs0, obs0_digest=np.uint64(digest(obs0)),
        actions=f('actions', np.int8), rews=f('rews', np.float64), dones=f('dones', bool),
        grids=f('grids', np.int8), obs_digest=f('obs_digest', np.uint64),
        alive_snakes=f('alive_snakes', np.int64), heads=f('heads', np.int16),
        alive=f('alive', bool), reset_at=f('reset_at', bool), ep_len=f('ep_len', np.int64),
        reset_grid=np.stack(resets['grid']), reset_obs_digest=np.array(resets['obs_digest'], np.uint64),
        info_step=np.array(infos['step'], np.int64),
        info_rank=np.array(infos['rank'], np.int64).reshape(-1, S),
        info_scores=np.array(infos['scores']).reshape(-1, S),
        info_steps=np.array(infos['steps']).reshape(-1, S),
        info_fruits=np.array(infos['fruits']).reshape(-1, S),
        info_kills=np.array(infos['kills']).reshape(-1, S),
        full_obs_steps=np.array(full_obs_steps, np.int64),
        full_obs=(np.stack(full_obs) if full_obs else np.zeros((0,), np.uint8)))
    n_resets = len(resets['grid']) - 1
    print(f'{name}: T={T} resets={n_resets} infos={len(infos["step"])} '
          f'max_len={max(len(s.coords) for s in env.snakes)}')


CUSTOM_REW = {'fruit': 1.0, 'kill': 2.0, 'lose': 3.0, 'win': 4.0, 'time': 0.1}  # test_snake.py:14-20
KILL_REW = {'fruit': 1.0, 'kill': 1.0, 'lose': -1.0, 'win': 5.0, 'time': -0.01}
SMALL_REW = {'fruit': 10.0, 'kill': 1.5, 'lose': -0.5, 'win': 2.0, 'time': -0.001}


def make_coop_trajs():
    # SnakeCoop-v1 (coop_snake_env.py:14-22): any done ends the episode, every
    # done is then True; the statistics are masked with the per-snake dones
    # before the override (snake_env.py:385-389), ranks come from any-done
    run_traj('coop_vr5_s4', 500, 12, coop=True, height=20, width=20, num_snakes=4,
             vision_range=5, full_obs_every=83)
    run_traj('coop_trunc_s3', 300, 13, coop=True, height=10, width=10, num_snakes=3,
             max_episode_steps=9, policy='greedy', eps=0.1, reward_dict=KILL_REW,
             full_obs_every=47)
    run_traj('coop_greedy_s2', 800, 14, coop=True, height=12, width=12, num_snakes=2,
             snake_length=2, policy='greedy', eps=0.05, frame_stack=2, vision_range=3,
             reward_dict=SMALL_REW, full_obs_every=157)


def make_trajs():
    run_traj('full20_s4', 400, 0, height=20, width=20, num_snakes=4, full_obs_every=97)
    run_traj('vr5_s4', 400, 1, height=20, width=20, num_snakes=4, vision_range=5, full_obs_every=61)
    run_traj('vr5_s8_40_fs4', 700, 2, height=40, width=40, num_snakes=8, vision_range=5,
             frame_stack=4, full_obs_every=233)
    run_traj('single_custom', 300, 3, height=20, width=20, num_snakes=1, num_fruits=4,
             reward_dict=CUSTOM_REW, full_obs_every=101)
    run_traj('human_s4', 400, 4, height=12, width=12, num_snakes=4, vision_range=3, frame_stack=2,
             observer='human', full_obs_every=50)
    run_traj('small_s2', 400, 5, height=8, width=8, num_snakes=2, snake_length=2, vision_range=2,
             frame_stack=3, reward_dict=SMALL_REW, full_obs_every=40)
    run_traj('trunc', 150, 6, height=10, width=10, num_snakes=3, max_episode_steps=8,
             policy='greedy', eps=0.0, full_obs_every=30)
    run_traj('l5_vr5', 200, 7, height=20, width=20, num_snakes=4, snake_length=5, vision_range=5,
             full_obs_every=50)
    run_traj('many_fruit', 300, 8, height=8, width=8, num_snakes=3, snake_length=2, num_fruits=20,
             policy='greedy', eps=0.2, full_obs_every=25)
    run_traj('kill_rew', 600, 9, height=20, width=20, num_snakes=4, reward_dict=KILL_REW,
             full_obs_every=150)
    run_traj('greedy_20_s2', 1500, 10, height=20, width=20, num_snakes=2, policy='greedy',
             eps=0.05, full_obs_every=300)
    run_traj('greedy_12_s1', 1200, 11, height=12, width=12, num_snakes=1, policy='greedy',
             eps=0.0, vision_range=4, full_obs_every=300)


# ---------------------------------------------------------- crafted scenarios
def inject(env, H, W, fruits, snakes, alive_snakes=None, episode_length=0):
    """Build grid + Snake objects exactly as reset() paints them (snake_env.py:131-159)."""
    grid = grid_util.make_grid(H, W, empty_value=0, wall_value=1)
    objs = []
    for idx, (coords, alive) in enumerate(snakes):
        sn = Snake(idx, [tuple(c) for c in coords])
        sn.alive = alive
        objs.append(sn)
        if alive:
            for c in sn.coords:
                grid[c] = 4 + 10 * idx
            grid[sn.head_coord] = 3 + 10 * idx
            grid[sn.tail_coord] = 5 + 10 * idx
    for f in fruits:
        grid[tuple(f)] = 2
    env.grid = grid
    env.snakes = objs
    env.alive_snakes = sum(a for _, a in snakes) if alive_snakes is None else alive_snakes
    env.frame_buffer = []
    env._init_obs()
    env._reset_epi_stats()
    env.episode_length = episode_length
    return grid.copy()


def crafted_case(name, H, W, fruits, snakes, actions, seed=0, alive_snakes=None,
                 episode_length=0, **kw):
    np.random.seed(seed)
    env = SnakeEnv(height=H, width=W, num_snakes=len(snakes), **kw)
    g0 = inject(env, H, W, fruits, snakes, alive_snakes, episode_length)
    steps = []
    for acts in actions:
        obs, rews, dones, info = env.step(list(acts))
        steps.append(dict(
            actions=list(acts), rews=[float(r) for r in rews], dones=[bool(d) for d in dones],
            grid=env.grid.astype(int).tolist(), alive_snakes=int(env.alive_snakes),
            heads=[list(map(int, s.head_coord)) for s in env.snakes],
            tails=[list(map(int, s.tail_coord)) for s in env.snakes],
            alive=[bool(s.alive) for s in env.snakes],
            lens=[len(s.coords) for s in env.snakes],
            obs_shape=list(obs.shape),
            obs_b64=base64.b64encode(np.ascontiguousarray(obs).tobytes()).decode(),
            info=({'rank': [int(x) for x in info['rank']],
                   'episode_scores': [float(x) for x in info['episode_scores']],
                   'episode_steps': [float(x) for x in info['episode_steps']],
                   'episode_fruits': [float(x) for x in info['episode_fruits']],
                   'episode_kills': [float(x) for x in info['episode_kills']]} if info else {})))
    cfg = dict(height=H, width=W, num_snakes=len(snakes), snake_length=env.snake_length,
               vision_range=env.vision_range, frame_stack=env.frame_stack,
               observer=env.observer, reward_dict=env.reward_dict, num_fruits=env.num_fruits,
               max_episode_steps=float(env.max_episode_steps))
    return dict(name=name, config=cfg, seed=seed, init_grid=g0.astype(int).tolist(),
                snakes=[dict(coords=[list(c) for c in co], alive=a) for co, a in snakes],
                alive_snakes=env_alive0(snakes, alive_snakes), episode_length=episode_length,
                steps=steps)


def env_alive0(snakes, alive_snakes):
    return sum(a for _, a in snakes) if alive_snakes is None else alive_snakes


def make_crafted():
    R = {'fruit': 10.0, 'kill': 3.0, 'lose': -0.5, 'win': 7.0, 'time': -0.001}
    cases = []
    # 1. head-on into a FRUIT cell: both die, fruit_taken += 1 so one extra fruit spawns
    #    (snake_env.py:529-536). Snake 0 moving RIGHT, snake 1 moving LEFT.
    cases.append(crafted_case('headon_fruit', 8, 8, [(3, 4)],
                              [([(3, 3), (3, 2)], True), ([(3, 5), (3, 6)], True)],
                              [[0, 0]], seed=11, reward_dict=R))
    # 2. head-on into an empty cell (3 snakes, third unaffected -> alive_snakes==1 -> win)
    cases.append(crafted_case('headon_empty_win', 9, 9, [(6, 6)],
                              [([(2, 3), (2, 2)], True), ([(2, 5), (2, 6)], True),
                               ([(6, 2), (6, 1)], True)],
                              [[0, 0, 0], [0, 0, 0]], seed=12, reward_dict=R))
    # 3. tail entry is safe: snake 1's head enters snake 0's tail twice while snake 0 moves on
    cases.append(crafted_case('tail_entry', 8, 8, [(6, 6)],
                              [([(2, 4), (2, 3), (2, 2)], True), ([(3, 2), (4, 2)], True)],
                              [[0, 0], [0, 2]], seed=13, reward_dict=R))
    #    same with snake indices swapped (update order matters for the tail clear)
    cases.append(crafted_case('tail_entry_swapped', 8, 8, [(6, 6)],
                              [([(3, 2), (4, 2)], True), ([(2, 4), (2, 3), (2, 2)], True)],
                              [[0, 0], [2, 0]], seed=13, reward_dict=R))
    # 4. fruit-eater tail rule (snake_env.py:338-345): snake 0 eats, snake 1 enters its tail
    cases.append(crafted_case('eater_tail', 8, 8, [(2, 5)],
                              [([(2, 4), (2, 3), (2, 2)], True), ([(3, 2), (4, 2)], True)],
                              [[0, 0]], seed=14, reward_dict=R))
    # 5. double decrement: two snakes head-on at the eater's tail -> alive_snakes -= 2 twice
    cases.append(crafted_case('double_decrement', 9, 9, [(3, 6)],
                              [([(3, 5), (3, 4), (3, 3)], True), ([(2, 3), (1, 3)], True),
                               ([(4, 3), (5, 3)], True), ([(7, 7), (7, 6)], True)],
                              [[0, 0, 0, 0], [0, 0, 0, 0]], seed=15, reward_dict=R))
    # 6. self-kill: head turns into own body; kill credited to itself (snake_env.py:537-538)
    cases.append(crafted_case('self_kill', 8, 8, [(6, 6)],
                              [([(2, 2), (2, 3), (3, 3), (3, 2), (4, 2)], True), ([(6, 2), (6, 1)], True)],
                              [[1, 0], [0, 0]], seed=16, reward_dict=R))
    # 7. body kill credited to the body owner, owner dies (into the wall) in the same step
    cases.append(crafted_case('kill_credit_owner_dies', 8, 8, [(6, 6)],
                              [([(1, 1), (1, 2), (1, 3)], True), ([(2, 2), (3, 2)], True),
                               ([(5, 5), (5, 4)], True)],
                              [[0, 0, 0], [0, 0, 0]], seed=17, reward_dict=R))
    # 8. dead-snake obs crop centred at (0, 0) (argmax of an all-zero head channel)
    cases.append(crafted_case('dead_crop', 10, 10, [(5, 5), (7, 2)],
                              [([(2, 2), (2, 3)], False), ([(6, 6), (6, 7), (6, 8)], True)],
                              [[0, 0], [1, 2], [2, 0]], seed=18, vision_range=3, frame_stack=2,
                              reward_dict=R))
    # 9. truncation at max_episode_steps: all dones True, snakes stay alive (:391-394)
    cases.append(crafted_case('truncation', 9, 9, [(1, 7)],
                              [([(4, 2), (4, 1)], True), ([(6, 6), (6, 7)], True)],
                              [[0, 0], [1, 2], [0, 0]], seed=19, episode_length=3,
                              max_episode_steps=5, reward_dict=R))
    # 10. human observer: perpendicular absolute turns only (:610-632)
    cases.append(crafted_case('human', 9, 9, [(1, 1)],
                              [([(4, 4), (4, 3)], True), ([(6, 2), (7, 2)], True)],
                              [[3, 1], [4, 2], [1, 4], [0, 3]], seed=20, observer='human',
                              vision_range=2, reward_dict=R))
    # 11. a dying snake's tail already re-owned by a lower-index snake is not erased (:561-563)
    cases.append(crafted_case('dead_tail_owned', 8, 8, [(6, 6)],
                              [([(2, 1), (3, 1)], True), ([(1, 3), (1, 2), (1, 1)], True),
                               ([(4, 4), (4, 5)], True)],
                              [[0, 1, 0], [0, 0, 0]], seed=21, reward_dict=R))
    #     ... and by a higher-index snake: the dying snake erases it first, then it is re-painted
    cases.append(crafted_case('dead_tail_owned_rev', 8, 8, [(6, 6)],
                              [([(1, 3), (1, 2), (1, 1)], True), ([(2, 1), (3, 1)], True),
                               ([(4, 4), (4, 5)], True)],
                              [[1, 0, 0], [0, 0, 0]], seed=21, reward_dict=R))
    # 12. single empty cell left: randint(0,1) consumes no draw; then no empty cell at all
    snake0 = [(3, 3), (3, 2), (3, 1), (2, 1), (2, 2), (2, 3), (2, 4), (1, 4), (1, 3), (1, 2)]
    cases.append(crafted_case('last_cells', 6, 6, [(3, 4), (4, 1), (4, 2), (4, 3), (4, 4)],
                              [(snake0, True), ([(2, 2), (2, 3)], False)],
                              [[0, 0], [2, 0], [2, 0], [1, 0]], seed=22, reward_dict=R))
    # 13. head-on into a wall-adjacent fruit + duplicate fruit draws on a tiny board
    cases.append(crafted_case('two_eaters', 7, 7, [(1, 3), (5, 3)],
                              [([(1, 2), (1, 1)], True), ([(5, 4), (5, 5)], True)],
                              [[0, 0], [1, 1], [0, 0]], seed=23, reward_dict=R))
    with open(os.path.join(OUT, 'crafted.json'), 'w') as fp:
        json.dump(cases, fp, indent=0)
    for c in cases:
        print('crafted', c['name'], [s['rews'] for s in c['steps']], [s['alive_snakes'] for s in c['steps']])


if __name__ == '__main__':
    which = sys.argv[1:] or ['rng', 'cand', 'traj', 'crafted']
    if 'rng' in which:
        make_rng()
    if 'cand' in which:
        make_candidates()
    if 'crafted' in which:
        make_crafted()
    if 'traj' in which:
        make_trajs()
    if 'traj' in which or 'coop' in which:
        make_coop_trajs()
