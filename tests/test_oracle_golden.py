"""Pin the CPU oracle (oracle/snake_oracle.c) against fixtures produced by the REAL
reference (tests/golden/gen/make_golden.py). No GPU needed."""
import numpy as np
import pytest

import golden_io as G


def test_mt_raw_stream(oracle):
    z = G.load('rng.npz')
    for i, s in enumerate(z['seeds']):
        np.testing.assert_array_equal(oracle.rng_raw(int(s), z['raw'].shape[1]), z['raw'][i])


def test_randint_masked(oracle):
    z = G.load('rng.npz')
    off = 0
    for (s, n, k), nxt in zip(z['ri_cases'], z['ri_next']):
        out, got_next = oracle.rng_randint(int(s), int(n), int(k))
        np.testing.assert_array_equal(out, z['ri_out'][off:off + int(k)])
        assert got_next == int(nxt), (s, n, k)
        off += int(k)


def test_permutation(oracle):
    z = G.load('rng.npz')
    for (s, n), head, dg, nxt in zip(z['perm_cases'], z['perm_head'], z['perm_digest'], z['perm_next']):
        p, got_next = oracle.rng_permutation(int(s), int(n))
        m = min(16, int(n))
        np.testing.assert_array_equal(p[:m], head[:m])
        assert G.digest(p.astype(np.int64)) == int(dg)
        assert got_next == int(nxt)


def test_candidates(oracle):
    z = G.load('candidates.npz')
    for k in z.files:
        if not k.startswith('full_'):
            continue
        H, W = map(int, k.split('_')[1].split('x'))
        L = int(k.split('_L')[1])
        np.testing.assert_array_equal(oracle.candidates(H, W, L), z[k])
    for H, W, L, C, dg in z['digest_meta']:
        a = oracle.candidates(int(H), int(W), int(L))
        assert a.shape[0] == int(C)
        assert G.digest(a) == int(dg), (H, W, L)


def replay_traj(oracle, t, steps=None):
    cfg = t['config']
    env = oracle.OracleEnv(seed=t['seed'], **G.env_kwargs(cfg))
    obs = env.reset()
    assert G.digest(obs) == int(t['obs0_digest'])
    np.testing.assert_array_equal(obs, t['obs0'])
    np.testing.assert_array_equal(env.grid, t['reset_grid'][0])
    T = len(t['actions']) if steps is None else steps
    n_reset = 0
    n_info = 0
    full_at = {int(s): i for i, s in enumerate(t['full_obs_steps'])}
    for i in range(T):
        obs, rews, dones, info = env.step(t['actions'][i])
        np.testing.assert_array_equal(env.grid, t['grids'][i], err_msg=f'grid step {i}')
        assert rews.tobytes() == t['rews'][i].tobytes(), (i, rews, t['rews'][i])
        np.testing.assert_array_equal(dones, t['dones'][i])
        assert env.alive_snakes == int(t['alive_snakes'][i]), i
        assert env.episode_length == int(t['ep_len'][i])
        assert G.digest(obs) == int(t['obs_digest'][i]), f'obs step {i}'
        if i in full_at:
            np.testing.assert_array_equal(obs, t['full_obs'][full_at[i]])
        sn = env.snakes()
        np.testing.assert_array_equal(sn[:, 5].astype(bool), t['alive'][i])
        np.testing.assert_array_equal(sn[:, 0:2], t['heads'][i])
        if info:
            assert int(t['info_step'][n_info]) == i
            np.testing.assert_array_equal(info['rank'], t['info_rank'][n_info])
            for k, kk in [('episode_scores', 'info_scores'), ('episode_steps', 'info_steps'),
                          ('episode_fruits', 'info_fruits'), ('episode_kills', 'info_kills')]:
                assert info[k].tobytes() == t[kk][n_info].tobytes(), (i, k)
            n_info += 1
        if t['reset_at'][i]:
            assert all(dones)
            n_reset += 1
            o = env.reset()
            np.testing.assert_array_equal(env.grid, t['reset_grid'][n_reset])
            assert G.digest(o) == int(t['reset_obs_digest'][n_reset])
    return n_reset


@pytest.mark.parametrize('name', G.traj_names())
def test_trajectory(oracle, name):
    t = G.load_traj(name)
    replay_traj(oracle, t)


def test_crafted(oracle):
    for case in G.load_crafted():
        cfg = case['config']
        env = oracle.OracleEnv(seed=case['seed'], **G.env_kwargs(cfg))
        snakes = [(s['coords'], s['alive']) for s in case['snakes']]
        env.inject(case['init_grid'], snakes, case['alive_snakes'], case['episode_length'])
        for i, st in enumerate(case['steps']):
            obs, rews, dones, info = env.step(st['actions'])
            where = f"{case['name']} step {i}"
            np.testing.assert_array_equal(env.grid, np.array(st['grid']), err_msg=where)
            assert rews.tolist() == st['rews'], where
            assert [float(x) for x in rews] == st['rews'] and \
                np.array(st['rews']).tobytes() == rews.tobytes(), where
            assert dones.tolist() == st['dones'], where
            assert env.alive_snakes == st['alive_snakes'], where
            np.testing.assert_array_equal(obs, st['obs'], err_msg=where)
            sn = env.snakes()
            assert sn[:, 0:2].tolist() == st['heads'], where
            assert sn[:, 2:4].tolist() == st['tails'], where
            assert sn[:, 5].astype(bool).tolist() == st['alive'], where
            assert sn[:, 6].tolist() == st['lens'], where
            if st['info']:
                assert info['rank'] == st['info']['rank'], where
                assert info['episode_scores'].tolist() == st['info']['episode_scores'], where
            else:
                assert not info, where


def test_invalid_action_is_keyerror(oracle):
    env = oracle.OracleEnv(seed=0, num_snakes=2)
    env.reset()
    with pytest.raises(KeyError):
        env.step([0, 3])


def test_rgb_from_grid_golden():
    """oracle.rgb_from_grid == the reference's rgb_from_grid (grid_util.py:164-175)
    on the fixture grids, owners 0..15 included (0.7**cycle darkening)."""
    from oracle.snake_oracle import rgb_from_grid
    z = G.load('render.npz')
    for g, want in zip(z['grids'], z['rgb']):
        np.testing.assert_array_equal(rgb_from_grid(g), want)
