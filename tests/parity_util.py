"""Shared helpers for the GPU parity tests: drive a SnakeVecEnv and the CPU
oracle (oracle/snake_oracle.c) with the same seeds and actions."""
import numpy as np


def oracle_batch(oracle, n, seed, num_snakes, **kw):
    envs = [oracle.OracleEnv(seed=seed + i, num_snakes=num_snakes, **kw) for i in range(n)]
    return envs, np.stack([e.reset() for e in envs])


def compare_step(refs, idx, actions, obs, rew, done, info, grids=None, where=''):
    """Step oracle envs `idx` with `actions` (auto-reset on all-done) and compare."""
    ep_done = info['episode_done']
    for row, i in enumerate(idx):
        r = refs[i]
        ro, rr, rd, rinfo = r.step(actions[row])
        assert rr.tobytes() == rew[row].tobytes(), f'{where} env {i}: rew {rew[row]} != {rr}'
        assert (rd == done[row]).all(), f'{where} env {i}: done {done[row]} != {rd}'
        assert bool(ep_done[row]) == bool(rinfo), f'{where} env {i}: episode_done'
        if rinfo:
            assert list(info['rank'][row]) == [int(x) for x in rinfo['rank']], f'{where} env {i}: rank'
            for k in ('episode_scores', 'episode_steps', 'episode_fruits', 'episode_kills'):
                assert info[k][row].tobytes() == rinfo[k].tobytes(), f'{where} env {i}: {k}'
        if all(rd):
            ro = r.reset()
        if grids is not None:
            assert (grids[row] == r.grid).all(), f'{where} env {i}: grid'
        assert (ro == obs[row]).all(), f'{where} env {i}: obs'
