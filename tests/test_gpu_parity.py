"""Parity of the HIP path (through the C-ABI) with the reference: the golden
fixtures generated from the real reference SnakeEnv, and the CPU oracle
(oracle/snake_oracle.c, itself pinned to the fixtures) on seeded batches.
Bar: bit-exact grids, dones, observations, info; float64 rewards compared by
their bytes (identical, tolerance 0)."""
import numpy as np
import pytest

import golden_io as G
from parity_util import compare_step, oracle_batch

torch = pytest.importorskip('torch')
pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip('needs a HIP device')
    from marlenv import _native
    _native.lib()


def _np(x):
    return {k: v.cpu().numpy() for k, v in x.items()} if isinstance(x, dict) else x.cpu().numpy()


# ------------------------------------------------------------- golden fixtures
@pytest.mark.parametrize('name', G.traj_names())
def test_compat_env_replays_golden(name):
    """make_snake(num_envs=1)-style SnakeEnv following numpy's global RNG, exactly
    as the reference does: np.random.seed(seed); env.reset(); env.step(...)."""
    from marlenv.envs.coop_snake_env import CoopSnakeEnv
    from marlenv.envs.snake_env import SnakeEnv
    t = G.load_traj(name)
    np.random.seed(t['seed'])
    kw = G.env_kwargs(t['config'])
    env = (CoopSnakeEnv if kw.pop('coop', False) else SnakeEnv)(**kw)
    obs = env.reset()
    np.testing.assert_array_equal(obs, t['obs0'])
    n_reset = n_info = 0
    full_at = {int(s): i for i, s in enumerate(t['full_obs_steps'])}
    for i in range(len(t['actions'])):
        obs, rews, dones, info = env.step([int(a) for a in t['actions'][i]])
        assert isinstance(obs, np.ndarray) and obs.dtype == np.uint8
        assert isinstance(rews, list) and isinstance(dones, list)
        np.testing.assert_array_equal(env.grid, t['grids'][i], err_msg=f'{name} grid step {i}')
        assert np.array(rews).tobytes() == t['rews'][i].tobytes(), (name, i, rews)
        assert dones == t['dones'][i].tolist(), (name, i)
        assert G.digest(obs) == int(t['obs_digest'][i]), (name, i)
        if i in full_at:
            np.testing.assert_array_equal(obs, t['full_obs'][full_at[i]])
        assert env.alive_snakes == int(t['alive_snakes'][i])
        if info:
            assert int(t['info_step'][n_info]) == i
            assert [int(x) for x in info['rank']] == t['info_rank'][n_info].tolist()
            assert info['episode_scores'].tobytes() == t['info_scores'][n_info].tobytes()
            assert info['episode_kills'].tobytes() == t['info_kills'][n_info].tobytes()
            n_info += 1
        else:
            assert n_info >= len(t['info_step']) or int(t['info_step'][n_info]) != i
        if t['reset_at'][i]:
            n_reset += 1
            o = env.reset()
            np.testing.assert_array_equal(env.grid, t['reset_grid'][n_reset])
            assert G.digest(o) == int(t['reset_obs_digest'][n_reset])
    assert n_info == len(t['info_step'])


@pytest.mark.parametrize('name', G.traj_names())
def test_vec_env_autoreset_replays_golden(name):
    """The batched env (N=1, per-env seed) with in-kernel auto-reset: the obs of
    an all-done step is the reset observation (wrappers.py:139-145)."""
    from marlenv import SnakeVecEnv
    t = G.load_traj(name)
    kw = G.env_kwargs(t['config'])
    S = kw.pop('num_snakes')
    v = SnakeVecEnv(1, num_snakes=S, seed=t['seed'], **kw)
    assert G.digest(_np(v.reset())[0]) == int(t['obs0_digest'])
    n_reset = 0
    for i in range(len(t['actions'])):
        obs, rew, done, info = v.step(torch.from_numpy(t['actions'][i][None].astype(np.int64)))
        obs, rew, done = _np(obs)[0], _np(rew)[0], _np(done)[0]
        assert rew.tobytes() == t['rews'][i].tobytes(), (name, i)
        assert done.tolist() == t['dones'][i].tolist(), (name, i)
        assert bool(info['episode_done'][0]) == bool(t['reset_at'][i])
        if t['reset_at'][i]:
            n_reset += 1
            assert G.digest(obs) == int(t['reset_obs_digest'][n_reset]), (name, i)
            np.testing.assert_array_equal(_np(v.grids())[0], t['reset_grid'][n_reset])
        else:
            assert G.digest(obs) == int(t['obs_digest'][i]), (name, i)
            np.testing.assert_array_equal(_np(v.grids())[0], t['grids'][i])


def test_crafted_scenarios():
    from marlenv import SnakeVecEnv
    for case in G.load_crafted():
        kw = G.env_kwargs(case['config'])
        S = kw.pop('num_snakes')
        v = SnakeVecEnv(1, num_snakes=S, seed=case['seed'], autoreset=False, **kw)
        v.inject(0, np.array(case['init_grid']), [(s['coords'], s['alive']) for s in case['snakes']],
                 case['alive_snakes'], case['episode_length'])
        for i, st in enumerate(case['steps']):
            where = f"{case['name']} step {i}"
            obs, rew, done, info = v.step(torch.tensor([st['actions']]))
            np.testing.assert_array_equal(_np(v.grids())[0], np.array(st['grid']), err_msg=where)
            assert _np(rew)[0].tobytes() == np.array(st['rews']).tobytes(), (where, _np(rew)[0], st['rews'])
            assert _np(done)[0].tolist() == st['dones'], where
            assert int(v.alive_counters()[0]) == st['alive_snakes'], where
            np.testing.assert_array_equal(_np(obs)[0], st['obs'], err_msg=where)
            tab = _np(v.snake_table())[0]
            assert tab[:, 5].astype(bool).tolist() == st['alive'], where
            live = [k for k in range(S) if st['alive'][k]]
            assert tab[live, 0:2].tolist() == [st['heads'][k] for k in live], where
            assert tab[live, 2:4].tolist() == [st['tails'][k] for k in live], where
            assert tab[live, 6].tolist() == [st['lens'][k] for k in live], where
            assert bool(info['episode_done'][0]) == bool(st['info']), where
            if st['info']:
                assert _np(info['rank'])[0].tolist() == st['info']['rank'], where
                assert _np(info['episode_scores'])[0].tolist() == st['info']['episode_scores'], where


# -------------------------------------------------------- batches vs the oracle
BATCH_CASES = {
    'cfg2_full20_s4': (dict(height=20, width=20, snake_length=3), 4, 96, 300),
    'cfg3_vr5_s4': (dict(height=20, width=20, snake_length=3, vision_range=5), 4, 128, 300),
    'cfg5_40_s8_vr5_fs4': (dict(height=40, width=40, snake_length=3, vision_range=5, frame_stack=4), 8, 24, 400),
    'human_12_vr3_fs2': (dict(height=12, width=12, vision_range=3, frame_stack=2, observer='human'), 4, 64, 300),
    'small_8_many_fruit': (dict(height=8, width=8, snake_length=2, num_fruits=20, vision_range=2), 3, 64, 300),
    'l5_vr5': (dict(height=20, width=20, snake_length=5, vision_range=5), 4, 16, 150),
    'kill_win_rewards': (dict(height=14, width=14, reward_dict={'fruit': 1.0, 'kill': 1.0, 'lose': -1.0,
                                                               'win': 5.0, 'time': -0.01}), 4, 64, 300),
    'single_s1': (dict(height=10, width=10, vision_range=4, num_fruits=4), 1, 64, 300),
    'trunc_s2': (dict(height=12, width=12, max_episode_steps=7), 2, 64, 100),
    # SnakeCoop-v1 (coop_snake_env.py:14-22): any-done episodes, truncation with coop
    'coop_vr5_s4': (dict(height=20, width=20, vision_range=5, coop=True), 4, 96, 300),
    'coop_trunc_s3_fs2': (dict(height=10, width=10, vision_range=2, frame_stack=2, coop=True,
                               max_episode_steps=6), 3, 64, 150),
    's16': (dict(height=24, width=24, snake_length=2, vision_range=3), 16, 16, 200),
    # spawn-ahead for every env (include/snake_env.h): nearly every reset starts
    # from a ready record, partial records carry retries across steps
    'spawn_all_vr5': (dict(height=20, width=20, snake_length=3, vision_range=5, spawn_ahead=4), 4, 96, 300),
    'spawn_off_vr5': (dict(height=20, width=20, snake_length=3, vision_range=5, spawn_ahead=-1), 4, 32, 150),
    'spawn_all_40_s8': (dict(height=40, width=40, snake_length=3, vision_range=5, spawn_ahead=8), 8, 16, 250),
    # 20 168 spawn poses: the reset workers' global link tables (no LDS draw record)
    'big_44_s4_global_links': (dict(height=44, width=44, snake_length=3, vision_range=4, spawn_ahead=4), 4, 16, 200),
    # 100x100: k_logic's eight frames per wave take 80 KB of LDS, one wave per workgroup
    'big_100_l2': (dict(height=100, width=100, snake_length=2, vision_range=3), 4, 16, 120),
    # the fused one-launch step (k_step: one frame, <= 4 snakes, table encode,
    # in-step spawn-ahead -- spawn_background=-1 keeps these small batches off
    # the background kernel): vision crop, full map, coop, human observer,
    # truncation, two snakes, eight lanes per env (N <= 8192)
    'fused_vr5_s4': (dict(height=20, width=20, snake_length=3, vision_range=5, spawn_background=-1), 4, 128, 300),
    'fused_full20_s4': (dict(height=20, width=20, snake_length=3, spawn_background=-1), 4, 96, 300),
    'fused_coop_vr5_s4': (dict(height=20, width=20, vision_range=5, coop=True, spawn_background=-1), 4, 96, 300),
    'fused_human_12_vr3': (dict(height=12, width=12, vision_range=3, observer='human', spawn_background=-1), 4, 64, 300),
    'fused_trunc_12_s2': (dict(height=12, width=12, max_episode_steps=7, spawn_background=-1), 2, 64, 100),
    'fused_s2_vr4': (dict(height=12, width=12, vision_range=4, num_fruits=6, spawn_background=-1), 2, 64, 300),
}


@pytest.fixture
def fused_on():
    """The fused one-launch step (k_step) switched on for the test
    (snake_debug_set "fused"; off by default until it wins)."""
    from marlenv import _native
    _native.debug_set('fused', 1)
    yield
    _native.debug_set('fused', 0)


@pytest.mark.parametrize('case', sorted(BATCH_CASES))
def test_batch_matches_oracle(oracle, case, request):
    from marlenv import SnakeVecEnv
    if case.startswith('fused_'):
        request.getfixturevalue('fused_on')
    kw, S, N, T = BATCH_CASES[case]
    seed = 1000 + 17 * len(case)
    v = SnakeVecEnv(N, num_snakes=S, seed=seed, **kw)
    obs0 = _np(v.reset())
    okw = {k: x for k, x in kw.items() if k not in ('spawn_ahead', 'spawn_background')}   # GPU scheduling knobs only
    refs, robs = oracle_batch(oracle, N, seed, S, **okw)
    np.testing.assert_array_equal(obs0, robs)
    rs = np.random.RandomState(seed)
    n_act = 5 if kw.get('observer') == 'human' else 3
    for t in range(T):
        a = rs.randint(0, n_act, size=(N, S))
        obs, rew, done, info = v.step(torch.from_numpy(a))
        compare_step(refs, range(N), a, _np(obs), _np(rew), _np(done), _np(info),
                     grids=_np(v.grids()), where=f'{case} step {t}')


@pytest.mark.parametrize('N,kw,fused', [
    (256, dict(height=20, width=20, vision_range=5, spawn_background=-1), True),
    (256, dict(height=20, width=20, spawn_background=-1), True),
    (256, dict(height=20, width=20, vision_range=5), False),            # (small batch: background spawn kernel)
    (128, dict(height=40, width=40, vision_range=5, frame_stack=4), False),
])
def test_fused_step_is_used(N, kw, fused, fused_on):
    """The one-launch step (k_step) runs exactly where snake_plan enables it."""
    from marlenv import SnakeVecEnv, _native
    v = SnakeVecEnv(N, num_snakes=4 if kw['height'] == 20 else 8, seed=1, **kw)
    v.reset()
    S = v.num_snakes
    for k in ('k_step', 'k_logic', 'k_post'):
        _native.timing_read(k)
    _native.timing_enable(True)
    try:
        v.step(torch.zeros((N, S), dtype=torch.int8, device='cuda'))
    finally:
        _native.timing_enable(False)
    n_step, n_logic = _native.timing_read('k_step')[1], _native.timing_read('k_logic')[1]
    assert (n_step, n_logic) == ((1, 0) if fused else (0, 1))
    assert _native.timing_read('fused_timeout')[1] == 0
    v.close()


def test_coop_any_done(oracle):
    """SnakeCoop-v1 (coop_snake_env.py:14-22): episode ends when any snake dies."""
    from marlenv import SnakeVecEnv
    N, S = 64, 4
    v = SnakeVecEnv(N, num_snakes=S, seed=5, coop=True, autoreset=False, height=12, width=12)
    v.reset()
    rs = np.random.RandomState(3)
    seen = 0
    for t in range(40):
        a = rs.randint(0, 3, size=(N, S))
        _, _, done, info = v.step(torch.from_numpy(a))
        d, ed = _np(done), _np(info['episode_done'])
        assert (ed == d.any(1)).all()
        assert (d[ed] == True).all()  # noqa: E712
        seen += int(ed.sum())
        if ed.any():
            v.reset(torch.from_numpy(ed))
    assert seen > 0


def test_shards_equal_full_batch():
    """Envs are keyed by global index: two shards == one batch (multi-GPU sharding)."""
    from marlenv import SnakeVecEnv
    N, S = 256, 4
    kw = dict(height=20, width=20, vision_range=5)
    full = SnakeVecEnv(N, num_snakes=S, seed=9, **kw)
    parts = [SnakeVecEnv(N // 2, num_snakes=S, seed=9, env_offset=o, **kw) for o in (0, N // 2)]
    o_full = full.reset()
    o_parts = torch.cat([p.reset() for p in parts])
    assert torch.equal(o_full, o_parts)
    g = torch.Generator(device='cuda').manual_seed(1)
    for t in range(150):
        a = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        of, rf, df, _ = full.step(a)
        outs = [p.step(a[i * (N // 2):(i + 1) * (N // 2)]) for i, p in enumerate(parts)]
        assert torch.equal(of, torch.cat([x[0] for x in outs]))
        assert torch.equal(rf, torch.cat([x[1] for x in outs]))
        assert torch.equal(df, torch.cat([x[2] for x in outs]))


FULL_SIZE_CASES = {
    # BASELINE config 3: the u16 draw record, 4-lane k_logic
    'cfg3_65536': (65536, 4, 400, dict(height=20, width=20, snake_length=3, vision_range=5)),
    # config 4's per-GPU shard (262 144 / 8): the u32 LDS link table, 4-lane
    # k_logic, 16 envs per k_logic wave -- the instantiation the 8-GPU headline runs
    'cfg4_32768': (32768, 4, 400, dict(height=20, width=20, snake_length=3, vision_range=5)),
    # 50x50 (26 000+ spawn poses): global link tables, in-step spawn-ahead, and
    # k_logic with one wave per workgroup (four would need 162 KB of LDS)
    'big50_16384': (16384, 4, 200, dict(height=50, width=50, snake_length=3, vision_range=4)),
    # config 3's per-GPU shard under strong scaling at 8 GPUs (65 536 / 8): the
    # last rank's envs (offset 57 344); batches of up to 8 192 envs default to
    # the background spawn kernel (two library streams, 512 reset / spawn
    # workers, threshold 4): this is that default at its boundary
    'cfg3s8_8192': (8192, 4, 400, dict(height=20, width=20, snake_length=3, vision_range=5), 57344),
}


@pytest.mark.parametrize('case', sorted(FULL_SIZE_CASES))
def test_full_size_sampled_parity(oracle, case):
    """Full-size batches: a sample of envs replayed through the oracle
    bit-exactly, plus whole-batch invariants. 400 steps reach the steady regime
    the bench times (past 200 steps almost every reset starts from a spawn-ahead
    record)."""
    from marlenv import SnakeVecEnv
    N, S, T, kw = FULL_SIZE_CASES[case][:4]
    off = FULL_SIZE_CASES[case][4] if len(FULL_SIZE_CASES[case]) > 4 else 0
    vr = kw['vision_range']
    v = SnakeVecEnv(N, num_snakes=S, seed=0, env_offset=off, **kw)
    obs = v.reset()
    idx = np.unique(np.concatenate([np.arange(8), np.linspace(0, N - 1, 40).astype(int),
                                    np.random.RandomState(0).randint(0, N, 16)]))
    refs = {int(i): oracle.OracleEnv(seed=off + int(i), num_snakes=S, **kw) for i in idx}
    o0 = obs[torch.from_numpy(idx).cuda()].cpu().numpy()
    for row, i in enumerate(idx):
        assert (refs[int(i)].reset() == o0[row]).all()
    g = torch.Generator(device='cuda').manual_seed(12345)
    n_ep = 0
    sel = torch.from_numpy(idx).cuda()
    for t in range(T):
        a = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        obs, rew, done, info = v.step(a)
        n_ep += int(info['episode_done'].sum())
        sub = {k: x[sel].cpu().numpy() for k, x in info.items()}
        compare_step([refs[int(i)] for i in idx], range(len(idx)), a[sel].cpu().numpy(),
                     obs[sel].cpu().numpy(), rew[sel].cpu().numpy(), done[sel].cpu().numpy(), sub,
                     where=f'{case} step {t}')
        # invariants over every env (every 10th step): one own-head cell at the
        # crop centre of each alive snake; no own-head channel for dead snakes
        if t % 10:
            continue
        tab = v.snake_table()
        alive = tab[..., 5].bool()
        centre = obs[:, :, vr, vr, 5]
        heads = obs[..., 5].sum(dim=(2, 3))
        assert torch.equal(centre.bool() | ~alive, torch.ones_like(alive))
        assert torch.equal(heads[alive], torch.ones_like(heads[alive]))
        assert int(heads[~alive].sum()) == 0
        assert not bool(info['error'].any())
    assert n_ep > 0.005 * N * T / 60
    if case == 'cfg3s8_8192':   # (a spawn record buffer per queue set: the background kernel's default here)
        assert v.layout.spawn == 4 * N * 672 * 4
    v.close()


@pytest.mark.parametrize('S,kw,spawn', [
    # dict: the background spawn kernel on / off (on by default for boards of
    # more than 8192 poses and for batches of up to 8192 envs like this one)
    (4, dict(height=20, width=20, vision_range=5),
     (0, -1, 1, 4, dict(spawn_ahead=0, spawn_background=-1), dict(spawn_ahead=3, spawn_background=-1))),
    (4, dict(height=12, width=12, coop=True), (0, -1)),             # coop: every env queued
    # 40x40, two frames: four-wave lean encodes (k_post_lean). By default the
    # attempts run in the background kernel; spawn_background=-1 runs them in
    # the step, on the k_post_lean workers' global link tables
    (8, dict(height=40, width=40, vision_range=5, frame_stack=2),
     (0, -1, 8, dict(spawn_ahead=0, spawn_background=-1), dict(spawn_ahead=8, spawn_background=-1))),
    # 20 168 spawn poses: the draw record does not fit LDS, the k_post workers'
    # global link tables
    (4, dict(height=44, width=44, vision_range=4), (0, -1, 4)),
])
def test_spawn_ahead_is_invisible(S, kw, spawn):
    """The spawn-ahead records only move reset draws off the critical path: every
    threshold gives bit-identical rollouts, and the default one actually serves
    resets from ready records."""
    from marlenv import SnakeVecEnv, _native
    N, T = 1024, 160

    def make(sp):
        if isinstance(sp, dict):
            return SnakeVecEnv(N, num_snakes=S, seed=77, **sp, **kw)
        return SnakeVecEnv(N, num_snakes=S, seed=77, spawn_ahead=sp, **kw)
    envs = [make(sp) for sp in spawn]
    outs = [v.reset() for v in envs]
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    g = torch.Generator(device='cuda').manual_seed(4)
    for k in ('resets', 'spawn_hits', 'spawn_jobs'):
        _native.timing_read(k)
    hits = jobs = 0
    for t in range(T):
        a = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        res = []
        for j, v in enumerate(envs):
            if j == 0:
                _native.timing_enable(True)
            res.append(v.step(a))
            if j == 0:
                _native.timing_enable(False)
                hits += _native.timing_read('spawn_hits')[1]
                jobs += _native.timing_read('spawn_jobs')[1]
        o0, r0, d0, i0 = res[0]
        for o, r, d, i in res[1:]:
            assert torch.equal(o0, o) and torch.equal(r0, r) and torch.equal(d0, d), f'step {t}'
            assert torch.equal(i0['episode_done'], i['episode_done'])
        for v in envs[1:]:
            assert torch.equal(envs[0].grids(), v.grids())
    assert jobs > 0 and hits > 0


@pytest.mark.parametrize('S,kw', [(4, dict(height=20, width=20, vision_range=5)),
                                  (8, dict(height=40, width=40, vision_range=5, frame_stack=2))])
def test_reset_draws_spawn_ahead(S, kw):
    """With spawn-ahead on, an explicit reset also draws the next reset's spawn
    poses (a READY or PARTIAL record for every env), and the next resets built
    on those records equal the ones drawn without them."""
    from marlenv import SnakeVecEnv
    N = 512
    a = SnakeVecEnv(N, num_snakes=S, seed=5, **kw)
    b = SnakeVecEnv(N, num_snakes=S, seed=5, spawn_ahead=-1, **kw)
    assert torch.equal(a.reset(), b.reset())
    sa, sb = a.env_rec.view(N, 8)[:, 4].cpu(), b.env_rec.view(N, 8)[:, 4].cpu()
    assert bool((sa != 0).all()) and bool((sb == 0).all())
    assert float(((sa & 3) == 2).float().mean()) > 0.9    # READY for almost every env (bits 0-1)
    for _ in range(2):                                     # resets from the records
        assert torch.equal(a.reset(), b.reset())
        assert torch.equal(a.grids(), b.grids())
        assert torch.equal(a.mt_state()[0], b.mt_state()[0])
        assert torch.equal(a.mt_state()[1], b.mt_state()[1])


def test_set_mt_state_voids_spawn_records():
    """Rewriting an env's MT state (compat env's global-RNG sync) must void its
    spawn-ahead record: the next reset draws from the new state."""
    from marlenv import SnakeVecEnv
    N, S = 64, 4
    kw = dict(height=10, width=10, num_snakes=S, seed=3, spawn_ahead=4)
    a, b = SnakeVecEnv(N, **kw), SnakeVecEnv(N, **dict(kw, spawn_ahead=-1))
    a.reset(), b.reset()
    g = torch.Generator(device='cuda').manual_seed(0)
    for t in range(30):   # builds ready records in `a`
        act = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        a.step(act), b.step(act)
    key = torch.from_numpy(np.random.RandomState(11).randint(0, 2 ** 31, 624).astype(np.int32))
    for v in (a, b):
        for i in range(N):
            v.set_mt_state(i, key, 624)
    assert torch.equal(a.reset(), b.reset())


def test_invalid_actions():
    from marlenv import SnakeVecEnv
    from marlenv.envs.snake_env import SnakeEnv
    env = SnakeEnv(num_snakes=2)
    env.reset()
    g = env.grid
    with pytest.raises(KeyError):
        env.step([0, 3])
    np.testing.assert_array_equal(env.grid, g)   # env untouched
    env.step([0, 0])
    v = SnakeVecEnv(4, num_snakes=2, seed=1)
    v.reset()
    g0 = _np(v.grids())
    _, rew, done, info = v.step(torch.tensor([[0, 0], [0, 7], [1, 2], [-1, 0]]))
    assert _np(info['error']).tolist() == [0, 1, 0, 1]
    # rejected envs: untouched, reward 0 and done False (defined outputs, not garbage)
    rew, done = _np(rew), _np(done)
    assert rew[[1, 3]].tobytes() == np.zeros((2, 2)).tobytes() and not done[[1, 3]].any()
    np.testing.assert_array_equal(_np(v.grids())[[1, 3]], g0[[1, 3]])
    ed = _np(info['episode_done'])
    assert not ed[[1, 3]].any()
    # the episode summary is zero wherever the episode did not end
    for k in ('rank', 'episode_scores', 'episode_steps', 'episode_fruits', 'episode_kills'):
        assert not _np(info[k])[~ed].any(), k
    vs = SnakeVecEnv(2, num_snakes=2, seed=1, strict=True)
    vs.reset()
    with pytest.raises(KeyError):
        vs.step(torch.tensor([[0, 0], [0, 5]]))


def test_make_snake_surface():
    from marlenv import make_snake
    env, a, b, props = make_snake(num_envs=1, num_snakes=4, height=20, width=20, vision_range=5)
    assert a is None and b is None
    assert props == {'action_info': {'action_n': 3}, 'num_envs': 1, 'num_snakes': 4}
    assert env.observation_space.shape == (4, 11, 11, 8)
    assert env.action_space.n == 3
    obs = env.reset()
    assert obs.shape == (4, 11, 11, 8) and obs.dtype == np.uint8
    acts = [env.action_space.sample() for _ in range(4)]
    obs2, rews, dones, info = env.step(acts)
    assert len(rews) == 4 and all(isinstance(r, float) for r in rews)
    assert obs2 is not obs
    single, _, _, p1 = make_snake(num_envs=1, num_snakes=1)
    o = single.reset()
    assert o.shape == (20, 20, 8)
    o, r, d, i = single.step(0)
    assert isinstance(r, float) and isinstance(d, bool) and i == {}
    venv, _, _, pv = make_snake(num_envs=64, num_snakes=4, vision_range=5)
    assert pv['num_envs'] == 64
    ob = venv.reset()
    assert tuple(ob.shape) == (64, 4, 11, 11, 8) and ob.is_cuda


@pytest.mark.parametrize('S,kw', [(4, dict(height=20, width=20, vision_range=5)),
                                  (16, dict(height=24, width=24, snake_length=2, vision_range=3)),
                                  (3, dict(height=9, width=7, snake_length=2))])
def test_render_rgb_matches_oracle(S, kw):
    """k_render (snake_render_rgb) == rgb_from_grid (grid_util.py:164-175) of the
    current grids, checked by the oracle's cell-by-cell restatement, along a
    random rollout (owners up to 15: every darkening cycle). N*H*W % 4 != 0 for
    the 9x7 case exercises the byte-wise tail."""
    from marlenv import SnakeVecEnv
    from oracle.snake_oracle import rgb_from_grid
    N = 37
    v = SnakeVecEnv(N, num_snakes=S, seed=77, **kw)
    v.reset()
    rs = np.random.RandomState(4)
    for t in range(25):
        if t % 8 == 0:
            rgb, grids = _np(v.render_rgb()), _np(v.grids())
            assert rgb.shape == (N, kw['height'], kw['width'], 3) and rgb.dtype == np.uint8
            for i in range(N):
                np.testing.assert_array_equal(rgb[i], rgb_from_grid(grids[i]), err_msg=f'S{S} t{t} env {i}')
        v.step(torch.from_numpy(rs.randint(0, 3, size=(N, S))))


def test_compat_render_modes(tmp_path):
    """SnakeEnv.render: 'rgb_array' frame, 'gif' frames + save_gif (snake_env.py:267-296, 419-437)."""
    from marlenv.envs.snake_env import SnakeEnv
    from oracle.snake_oracle import rgb_from_grid
    np.random.seed(3)
    env = SnakeEnv(num_snakes=4)
    env.reset()
    for _ in range(3):
        env.step([0, 1, 2, 0])
        np.testing.assert_array_equal(env.render('rgb_array'), rgb_from_grid(env.grid))
        env.render('gif')
    assert len(env.frame_buffer) == 3 and env.frame_buffer[0].size == (300, 300)
    fp = env.save_gif(str(tmp_path / 'play.gif'))
    assert (tmp_path / 'play.gif').stat().st_size > 0 and fp.endswith('play.gif')


def test_info_zero_where_episode_continues():
    """rank / episode_* are the episode summary where episode_done, zeros elsewhere."""
    from marlenv import SnakeVecEnv
    N, S = 512, 4
    v = SnakeVecEnv(N, num_snakes=S, seed=2, height=10, width=10)
    v.reset()
    g = torch.Generator(device='cuda').manual_seed(5)
    ended = 0
    for t in range(60):
        a = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        _, _, _, info = v.step(a)
        ed = info['episode_done']
        ended += int(ed.sum())
        assert not bool(info['rank'][~ed].any())
        assert bool((info['rank'][ed] >= 1).all())
        for k in ('episode_scores', 'episode_steps', 'episode_fruits', 'episode_kills'):
            assert not bool(info[k][~ed].any()), k
    assert ended > 0


@pytest.mark.parametrize('kw,S', [(dict(height=20, width=20, vision_range=5), 4),
                                  (dict(height=12, width=12, frame_stack=3, vision_range=3, coop=True), 3),
                                  (dict(height=44, width=44, vision_range=4, spawn_ahead=4), 4),
                                  (dict(height=40, width=40, vision_range=5, frame_stack=4,
                                        spawn_background=-1), 8),
                                  (dict(height=20, width=20, vision_range=5, spawn_background=1), 4)])
def test_snapshot_restore_roundtrip(kw, S):
    """state_dict() mid-episode -> K steps -> load_state_dict() -> the same K steps
    reproduce bit-identically, in the same env and in a fresh one (and from a
    CPU copy, the torch.save path)."""
    from marlenv import SnakeVecEnv
    N, K = 256, 40
    v = SnakeVecEnv(N, num_snakes=S, seed=31, **kw)
    v.reset()
    g = torch.Generator(device='cuda').manual_seed(8)
    acts = torch.randint(0, 3, (60 + K, N, S), generator=g, device='cuda', dtype=torch.int8)
    for t in range(60):
        v.step(acts[t])
    snap = v.state_dict()
    snap_cpu = v.state_dict(device='cpu')

    def roll(env):
        outs = []
        for t in range(60, 60 + K):
            o, r, d, i = env.step(acts[t])
            outs.append((o.clone(), r.clone(), d.clone(), i['episode_done'].clone(), env.grids().clone()))
        return outs

    ref = roll(v)
    v.load_state_dict(snap)
    again = roll(v)
    fresh = SnakeVecEnv(N, num_snakes=S, seed=999, **kw)     # other seed: everything comes from the snapshot
    fresh.load_state_dict(snap_cpu)
    other = roll(fresh)
    for t, (a, b, c) in enumerate(zip(ref, again, other)):
        for x, y, z in zip(a, b, c):
            assert torch.equal(x, y) and torch.equal(x, z), f'step {t}'
    bad = SnakeVecEnv(N // 2, num_snakes=S, seed=31, **kw)
    with pytest.raises(ValueError):
        bad.load_state_dict(snap)


def test_snapshot_is_canonical():
    """Snapshots hold the env state, not the spawn-ahead cache: twins stepped
    with the background spawn kernel, the in-step spawn-ahead and none at all
    give equal state_dicts (the background one's records depend on when each
    k_spawn ran), and a snapshot loads into an env of another spawn-ahead mode
    and continues bit-identically."""
    from marlenv import SnakeVecEnv
    N, S = 512, 4
    kw = dict(height=20, width=20, vision_range=5)
    modes = [dict(spawn_background=1), dict(spawn_background=-1), dict(spawn_ahead=-1, spawn_background=-1)]
    envs = [SnakeVecEnv(N, num_snakes=S, seed=3, **m, **kw) for m in modes]
    for v in envs:
        v.reset()
    g = torch.Generator(device='cuda').manual_seed(6)
    acts = torch.randint(0, 3, (90, N, S), generator=g, device='cuda', dtype=torch.int8)
    for t in range(50):
        for v in envs:
            v.step(acts[t])
    sds = [v.state_dict(device='cpu') for v in envs]
    for sd in sds[1:]:
        for k in SnakeVecEnv._STATE_BUFFERS:
            assert torch.equal(sds[0][k], sd[k]), k
    assert int(sds[0]['env_rec'].view(N, 8)[:, 4].abs().sum()) == 0
    other = SnakeVecEnv(N, num_snakes=S, seed=0, **modes[1], **kw)
    other.load_state_dict(sds[0])
    for t in range(50, 90):
        a, b = envs[0].step(acts[t]), other.step(acts[t])
        for x, y in zip(a[:3], b[:3]):
            assert torch.equal(x, y), t
    for v in envs + [other]:
        v.close()


def test_vec_env_on_non_current_device():
    """A SnakeVecEnv on cuda:1 launches on its own device whatever device is current."""
    if torch.cuda.device_count() < 2:
        pytest.skip('needs two GPUs')
    from marlenv import SnakeVecEnv
    torch.cuda.set_device(0)
    a = SnakeVecEnv(64, num_snakes=4, seed=4, device='cuda:1', vision_range=5)
    b = SnakeVecEnv(64, num_snakes=4, seed=4, device='cuda:0', vision_range=5)
    assert torch.equal(a.reset().cpu(), b.reset().cpu())
    g = torch.Generator().manual_seed(0)
    for t in range(50):
        act = torch.randint(0, 3, (64, 4), generator=g, dtype=torch.int8)
        oa, ra, _, _ = a.step(act)
        ob, rb, _, _ = b.step(act)
        assert torch.equal(oa.cpu(), ob.cpu()) and torch.equal(ra.cpu(), rb.cpu())


@pytest.mark.parametrize('S,kw', [(4, dict(height=20, width=20, vision_range=5)),
                                  (2, dict(height=12, width=12, snake_length=4))])
def test_autoreset_every_step_matches_oracle(oracle, S, kw):
    """autoreset='every_step' (gym 0.23.1's worker behind make_snake,
    wrappers.py:212): the step's rewards/dones/info, then a reset of every env,
    whose obs is returned."""
    from marlenv import SnakeVecEnv
    N = 48
    v = SnakeVecEnv(N, num_snakes=S, seed=21, autoreset='every_step', **kw)
    refs, o0 = oracle_batch(oracle, N, 21, S, **kw)
    assert (_np(v.reset()) == o0).all()
    rs = np.random.RandomState(4)
    for t in range(40):
        a = rs.randint(0, 3, size=(N, S))
        obs, rew, done, info = v.step(torch.from_numpy(a))
        obs, rew, done = _np(obs), _np(rew), _np(done)
        ep_done = _np(info['episode_done'])
        for i, r in enumerate(refs):
            _, rr, rd, rinfo = r.step(a[i])
            assert rr.tobytes() == rew[i].tobytes(), (t, i)
            assert (rd == done[i]).all(), (t, i)
            assert bool(ep_done[i]) == bool(rinfo), (t, i)
            assert (r.reset() == obs[i]).all(), (t, i)


def test_single_snake_vector_surface(oracle):
    """make_snake(num_envs > 1, num_snakes=1): the reference wraps each vector
    worker in SingleAgent (wrappers.py:84-105, 204-212), so obs (N, h, w, C),
    actions (N,), rewards (N,) float64, dones (N,) bool -- replayed against the
    oracle env by env (env i seeded i, all-done auto-reset)."""
    from marlenv import make_snake
    N = 24
    kw = dict(height=10, width=10, vision_range=4, num_fruits=4)
    env, _, _, props = make_snake(num_envs=N, num_snakes=1, **kw)
    assert props == {'action_info': {'action_n': 3}, 'num_envs': N, 'num_snakes': 1}
    assert env.observation_space.shape == (N, 9, 9, 8)
    assert env.single_observation_space.shape == (9, 9, 8)
    assert env.action_space.shape == (N,)
    refs, o0 = oracle_batch(oracle, N, 0, 1, **kw)
    obs = env.reset()
    assert tuple(obs.shape) == (N, 9, 9, 8)
    np.testing.assert_array_equal(_np(obs), o0[:, 0])
    rs = np.random.RandomState(6)
    ended = 0
    for t in range(120):
        a = rs.randint(0, 3, size=N)
        obs, rew, done, info = env.step(torch.from_numpy(a))
        assert tuple(obs.shape) == (N, 9, 9, 8) and tuple(rew.shape) == (N,) and tuple(done.shape) == (N,)
        assert rew.dtype == torch.float64 and done.dtype == torch.bool
        assert tuple(info['rank'].shape) == (N,) and tuple(info['episode_scores'].shape) == (N,)
        ended += int(info['episode_done'].sum())
        for i, r in enumerate(refs):
            ro, rr, rd, rinfo = r.step(a[i:i + 1])
            assert rr.tobytes() == _np(rew)[i:i + 1].tobytes(), (t, i)
            assert bool(rd[0]) == bool(_np(done)[i]), (t, i)
            if rd[0]:
                ro = r.reset()
            np.testing.assert_array_equal(_np(obs)[i], ro[0], err_msg=f'step {t} env {i}')
    assert ended > 0


@pytest.mark.parametrize('kw,S', [(dict(height=20, width=20, vision_range=5), 4),
                                  (dict(height=12, width=12, frame_stack=2), 2)])
def test_every_step_invalid_action_keeps_obs(oracle, kw, S):
    """autoreset='every_step' with an invalid action in some envs: those envs are
    left unchanged (the reference raises KeyError before touching them) and their
    returned obs is the observation of the unchanged state, not uninitialised
    memory; every other env is stepped and reset."""
    from marlenv import SnakeVecEnv
    N = 40
    v = SnakeVecEnv(N, num_snakes=S, seed=13, autoreset='every_step', **kw)
    refs, o0 = oracle_batch(oracle, N, 13, S, **kw)
    assert (_np(v.reset()) == o0).all()
    last = o0.copy()
    rs = np.random.RandomState(9)
    for t in range(12):
        a = rs.randint(0, 3, size=(N, S))
        bad = rs.rand(N) < 0.3
        a[bad, 0] = 7
        obs, rew, done, info = v.step(torch.from_numpy(a))
        obs, rew, err = _np(obs), _np(rew), _np(info['error'])
        for i, r in enumerate(refs):
            if bad[i]:
                assert err[i] == 1 and not rew[i].any()
                np.testing.assert_array_equal(obs[i], last[i], err_msg=f'step {t} env {i}')
                continue
            assert err[i] == 0
            _, rr, _, _ = r.step(a[i])
            assert rr.tobytes() == rew[i].tobytes()
            last[i] = r.reset()
            np.testing.assert_array_equal(obs[i], last[i], err_msg=f'step {t} env {i}')


@pytest.mark.parametrize('kw,S', [(dict(height=20, width=20, vision_range=5), 4),
                                  (dict(height=12, width=12), 3)])
def test_fused_invalid_action_keeps_obs(oracle, kw, S, fused_on):
    """The fused step (k_step) with invalid actions in some envs: a rejected env
    is left unchanged and its observation is that of its unchanged state (the
    logic wave hands the encodes its old slot and heads); every other env steps
    (and auto-resets) exactly like the oracle."""
    from marlenv import SnakeVecEnv
    N = 64
    v = SnakeVecEnv(N, num_snakes=S, seed=17, spawn_background=-1, **kw)
    refs, o0 = oracle_batch(oracle, N, 17, S, **kw)
    assert (_np(v.reset()) == o0).all()
    last = o0.copy()
    rs = np.random.RandomState(4)
    for t in range(80):
        a = rs.randint(0, 3, size=(N, S))
        bad = rs.rand(N) < 0.2
        a[bad, 0] = 9
        obs, rew, done, info = v.step(torch.from_numpy(a))
        obs, rew, done, err = _np(obs), _np(rew), _np(done), _np(info['error'])
        for i, r in enumerate(refs):
            try:   # (the reference raises KeyError only for an ALIVE snake's invalid action)
                ro, rr, rd, _ = r.step(a[i])
            except KeyError:
                assert bad[i] and err[i] == 1 and not rew[i].any() and not done[i].any(), (t, i)
                np.testing.assert_array_equal(obs[i], last[i], err_msg=f'step {t} env {i}')
                continue
            if all(rd):
                ro = r.reset()
            assert err[i] == 0 and rr.tobytes() == rew[i].tobytes(), (t, i)
            np.testing.assert_array_equal(obs[i], ro, err_msg=f'step {t} env {i}')
            last[i] = ro


def test_full_size_cfg2_every_env(oracle):
    """BASELINE config 2 at full size (4 096 envs, 20x20, 4 snakes, full-map
    obs): EVERY env against the oracle batch (oracle/snake_oracle.c so_batch,
    host threads) for 400 steps -- obs, rewards (bytes), dones, the episode
    summary, and every grid every 25 steps."""
    from marlenv import SnakeVecEnv
    N, S, T = 4096, 4, 400
    kw = dict(height=20, width=20, snake_length=3)
    v = SnakeVecEnv(N, num_snakes=S, seed=0, **kw)
    ref = oracle.OracleBatch(N, seed=0, num_snakes=S, **kw)
    np.testing.assert_array_equal(_np(v.reset()), ref.reset())
    g = torch.Generator(device='cuda').manual_seed(2024)
    n_ep = 0
    for t in range(T):
        a = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        obs, rew, done, info = v.step(a)
        robs, rrew, rdone, rinfo = ref.step(a.cpu().numpy())
        where = f'cfg2 step {t}'
        assert _np(rew).tobytes() == rrew.tobytes(), where
        np.testing.assert_array_equal(_np(done), rdone, err_msg=where)
        ed = _np(info['episode_done'])
        np.testing.assert_array_equal(ed, rinfo['episode_done'], err_msg=where)
        np.testing.assert_array_equal(_np(info['rank']), rinfo['rank'], err_msg=where)
        for k in ('episode_scores', 'episode_steps', 'episode_fruits', 'episode_kills'):
            assert _np(info[k]).tobytes() == rinfo[k].tobytes(), (where, k)
        if not np.array_equal(_np(obs), robs):
            bad = np.nonzero((_np(obs) != robs).reshape(N, -1).any(1))[0]
            raise AssertionError(f'{where}: obs differ in envs {bad[:8].tolist()}')
        if t % 25 == 0:
            np.testing.assert_array_equal(_np(v.grids()), ref.grids(), err_msg=where)
        n_ep += int(ed.sum())
    assert n_ep > 0.005 * N * T / 60


def test_full_size_cfg5_sampled(oracle):
    """BASELINE config 5's per-GPU shard at full size (8 192 envs, 40x40, 8
    snakes, vision_range 5, frame_stack 4): sampled envs against the oracle for
    500 steps (several worker rounds, the 40x40 draw records, spawn-ahead under
    load), plus whole-batch crop invariants."""
    from marlenv import SnakeVecEnv
    N, S, T = 8192, 8, 500
    kw = dict(height=40, width=40, snake_length=3, vision_range=5, frame_stack=4)
    v = SnakeVecEnv(N, num_snakes=S, seed=0, **kw)
    obs = v.reset()
    idx = np.unique(np.concatenate([np.arange(4), np.linspace(0, N - 1, 24).astype(int),
                                    np.random.RandomState(1).randint(0, N, 12)]))
    refs = {int(i): oracle.OracleEnv(seed=int(i), num_snakes=S, **kw) for i in idx}
    sel = torch.from_numpy(idx).cuda()
    o0 = obs[sel].cpu().numpy()
    for row, i in enumerate(idx):
        assert (refs[int(i)].reset() == o0[row]).all()
    g = torch.Generator(device='cuda').manual_seed(55)
    n_ep = 0
    for t in range(T):
        a = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        obs, rew, done, info = v.step(a)
        n_ep += int(info['episode_done'].sum())
        sub = {k: x[sel].cpu().numpy() for k, x in info.items()}
        compare_step([refs[int(i)] for i in idx], range(len(idx)), a[sel].cpu().numpy(),
                     obs[sel].cpu().numpy(), rew[sel].cpu().numpy(), done[sel].cpu().numpy(), sub,
                     where=f'cfg5 step {t}')
        if t % 25:
            continue
        # newest frame (channels 24-31): one own-head cell at the crop centre of
        # every alive snake, none for a dead one
        tab = v.snake_table()
        alive = tab[..., 5].bool()
        heads = obs[..., 24 + 5].sum(dim=(2, 3))
        assert torch.equal(obs[:, :, 5, 5, 24 + 5].bool() | ~alive, torch.ones_like(alive))
        assert torch.equal(heads[alive], torch.ones_like(heads[alive]))
        assert int(heads[~alive].sum()) == 0
        assert not bool(info['error'].any())
    assert n_ep > 0


def test_background_state_lifetime():
    """snake_release / SnakeVecEnv.close() on a background spawn-ahead board
    (40x40, 8 snakes: k_spawn on the library's per-state stream): closing twice
    is harmless, and an env created afterwards -- its state buffers likely at
    the freed addresses, which key the library's background context -- rolls
    out bit-identically to a twin that lived beside it throughout, with its
    spawn-ahead records still served (a stale context's launch count would
    leave the device-side queue gate shut: identical results, no hits)."""
    from marlenv import SnakeVecEnv, _native
    N, S = 512, 8
    kw = dict(height=40, width=40, vision_range=5, frame_stack=2)
    twin = SnakeVecEnv(N, num_snakes=S, seed=5, **kw)
    a = SnakeVecEnv(N, num_snakes=S, seed=9, **kw)
    a.reset()
    g = torch.Generator(device='cuda').manual_seed(3)
    for _ in range(30):
        a.step(torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8))
    freed = {a.env_rec.data_ptr(), a.mt.data_ptr(), a.grid.data_ptr()}
    a.close()
    a.close()
    del a
    b = SnakeVecEnv(N, num_snakes=S, seed=5, **kw)
    reused = bool(freed & {b.env_rec.data_ptr(), b.mt.data_ptr(), b.grid.data_ptr()})
    assert torch.equal(b.reset(), twin.reset())
    for k in ('spawn_hits', 'spawn_jobs'):
        _native.timing_read(k)
    hits = 0
    for t in range(120):
        act = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        _native.timing_enable(True)
        ob, rb, db, ib = b.step(act)
        _native.timing_enable(False)
        hits += _native.timing_read('spawn_hits')[1]
        ot, rt, dt, it = twin.step(act)
        assert torch.equal(ob, ot) and torch.equal(rb, rt) and torch.equal(db, dt), f'step {t}'
        assert torch.equal(ib['episode_done'], it['episode_done']), f'step {t}'
    assert torch.equal(b.grids(), twin.grids())
    assert hits > 0, f'no spawn-ahead hits after the re-created state (addresses reused: {reused})'
    b.close()
    twin.close()


@pytest.mark.parametrize('kw', [
    dict(height=40, width=40, vision_range=5, num_fruits=24),   # 40x40: 110 us jobs, overlapping sets
    dict(height=20, width=20, num_fruits=12),                   # small board, short jobs
])
def test_background_overlap_stress(kw):
    """The background protocol under load (round 5: the two queue sets' spawn
    kernels on two streams may overlap): many fruits, so k_logic's fruit draws
    void records while their jobs still run and the env is queued again into
    the other set; threshold 8 queues every env every step. The rollout must
    equal the in-step spawn-ahead run bit for bit, step by step, and the env
    state at the end."""
    from marlenv import SnakeVecEnv, _native
    N, S = 384, 8
    bg = SnakeVecEnv(N, num_snakes=S, seed=21, spawn_ahead=8, spawn_background=1, **kw)
    ref = SnakeVecEnv(N, num_snakes=S, seed=21, spawn_ahead=-1, spawn_background=-1, **kw)
    assert torch.equal(bg.reset(), ref.reset())
    g = torch.Generator(device='cuda').manual_seed(8)
    for k in ('spawn_hits', 'spawn_void'):
        _native.timing_read(k)
    _native.timing_enable(True)
    for t in range(200):
        a = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        ob, rb, db, ib = bg.step(a)
        orf, rr, dr, ir = ref.step(a)
        assert torch.equal(ob, orf) and torch.equal(rb, rr) and torch.equal(db, dr), f'step {t}'
        assert torch.equal(ib['episode_done'], ir['episode_done']), f'step {t}'
    _native.timing_enable(False)
    hits, voids = _native.timing_read('spawn_hits')[1], _native.timing_read('spawn_void')[1]
    bg.sync()
    assert torch.equal(bg.grids(), ref.grids()) and torch.equal(bg.mt, ref.mt)
    assert torch.equal(bg.env_records(), ref.env_records())   # (all eight words, word 4 canonical)
    assert hits > 0 and voids > 0, (hits, voids)
    bg.close()
    ref.close()


@pytest.mark.parametrize('wait', [0, 200000])
def test_draw_wait_fallback(wait):
    """The DRAWING wait of claim_reset_mt and its fallback, with background jobs
    held DRAWING for 300 us each (snake_debug_set "spawn_delay_ticks", fault
    injection) so that resets meet them: with the default wait (2 ms) such a
    reset waits for the job's record; with the wait at 0 ticks it voids the job
    at once and draws from the env's own MT state while the job is still running
    (and later writes its queue set's record buffer). Either way the rollout
    equals the in-step spawn-ahead run bit for bit, and the counters show the
    path was taken ("draw_wait": resets that met a job drawing; "draw_timeout":
    those that gave up waiting)."""
    from marlenv import SnakeVecEnv, _native
    N, S = 384, 8
    kw = dict(height=40, width=40, vision_range=5, num_fruits=24)
    bg = SnakeVecEnv(N, num_snakes=S, seed=23, spawn_ahead=8, spawn_background=1, **kw)
    ref = SnakeVecEnv(N, num_snakes=S, seed=23, spawn_ahead=-1, spawn_background=-1, **kw)
    assert torch.equal(bg.reset(), ref.reset())
    g = torch.Generator(device='cuda').manual_seed(9)
    for k in ('draw_wait', 'draw_timeout'):
        _native.timing_read(k)
    _native.debug_set('draw_wait_ticks', wait)
    _native.debug_set('spawn_delay_ticks', 30000)
    try:
        _native.timing_enable(True)
        for t in range(160):
            a = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
            ob, rb, db, ib = bg.step(a)
            orf, rr, dr, ir = ref.step(a)
            assert torch.equal(ob, orf) and torch.equal(rb, rr) and torch.equal(db, dr), f'step {t}'
        bg.sync()
        torch.cuda.synchronize()
    finally:
        _native.timing_enable(False)
        _native.debug_set('draw_wait_ticks', 200000)
        _native.debug_set('spawn_delay_ticks', 0)
    waits, timeouts = _native.timing_read('draw_wait')[1], _native.timing_read('draw_timeout')[1]
    assert torch.equal(bg.grids(), ref.grids()) and torch.equal(bg.mt, ref.mt)
    assert torch.equal(bg.env_records(), ref.env_records())
    assert waits > 0, (waits, timeouts)
    assert timeouts == (waits if wait == 0 else 0), (waits, timeouts)
    with pytest.raises(Exception):
        _native.debug_set('no_such_knob', 1)
    bg.close()
    ref.close()


def test_info_read_on_another_stream():
    """The episode summary is filled on the stream the step ran on; read from
    another stream it is ordered after that fill: the values equal
    the ones read on the step's own stream."""
    from marlenv import SnakeVecEnv
    N, S = 256, 4
    v = SnakeVecEnv(N, num_snakes=S, seed=2, height=10, width=10)
    w = SnakeVecEnv(N, num_snakes=S, seed=2, height=10, width=10)
    v.reset(), w.reset()
    side = torch.cuda.Stream()
    g = torch.Generator(device='cuda').manual_seed(5)
    seen = 0
    for t in range(60):
        a = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            _, _, _, iv = v.step(a)
        _, _, _, iw = w.step(a)
        # read v's info on the default stream (not the one it was stepped on)
        for k in ('rank', 'episode_scores', 'episode_steps', 'episode_fruits', 'episode_kills'):
            assert torch.equal(iv[k], iw[k]), (t, k)
        seen += int(iw['episode_done'].sum())
    assert seen > 0
