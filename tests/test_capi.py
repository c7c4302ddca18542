"""CPU checks of the product's C-ABI library (no GPU needed): it loads, exports
every symbol include/snake_env.h declares, plans buffers, rejects bad configs
the way SnakeEnv.__init__ does, and its host-side spawn-pose table equals the
reference's dfs_sweep_empty order (golden digests)."""
import ctypes
import os
import re

import numpy as np
import pytest

import golden_io as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def native():
    from marlenv import _native
    if not os.path.exists(_native.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return _native


def header_functions():
    src = open(os.path.join(ROOT, 'include', 'snake_env.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'^\s*(?:const\s+)?\w+\s*\*?\s*(snake_\w+)\s*\(', src, flags=re.M)))


def test_exports_match_header(native):
    names = header_functions()
    assert set(names) == set(native.EXPORTS), names
    L = native.lib()
    for n in names:
        assert hasattr(L, n), n
    assert L.snake_abi_version() == native.SNAKE_ABI_VERSION


def cfg(native, **kw):
    from marlenv.config import build_cfg
    return build_cfg(**kw)[0]


def test_plan_sizes(native):
    c = cfg(native, height=20, width=20, num_snakes=4, vision_range=5)
    lay = native.SnakeLayout()
    assert native.lib().snake_plan(ctypes.byref(c), 65536, ctypes.byref(lay)) == 0
    assert (lay.obs_h, lay.obs_w, lay.obs_c) == (11, 11, 8)
    assert lay.obs == 65536 * 4 * 11 * 11 * 8
    assert lay.n_cand == 3464 and lay.jscratch == 0
    assert lay.grid_stride == 400 and lay.ring_cap == 512
    assert lay.spawn == 65536 * 672 * 4                        # spawn-ahead records
    assert lay.stats == 65536 * 4 * 16                         # snake_epi_stat: one 16-B record per snake
    # two sets (step parity) of three queues + counters (one per 128-B line)
    # two queue sets, then the fused step's counts, flags and hand-off records
    queues = 4 * (3 * 64 * (4096 // 64) * 16 + 227 * 32)   # (four queue sets)
    assert lay.resetq == (queues + 64 * 32 + 2 * 65536 // 4 + 4 * 65536) * 4
    c = cfg(native, height=40, width=40, num_snakes=8, vision_range=5, frame_stack=4)
    assert native.lib().snake_plan(ctypes.byref(c), 8192, ctypes.byref(lay)) == 0
    assert lay.obs_c == 32 and lay.obs == 8192 * 8 * 11 * 11 * 32
    # the u16 draw record fits LDS (the spawn kernel keeps it there), and with
    # background spawn-ahead the one-launch workers (k_post_lean) keep a global
    # link table per worker for resets without a ready record
    assert lay.n_cand == 16424 and lay.jscratch == 2048 * (16424 + 64) * 4
    assert lay.spawn == 4 * 8192 * 672 * 4                        # background spawn-ahead: a record per queue set and env
    c = cfg(native, height=44, width=44, num_snakes=4)
    lay2 = native.SnakeLayout()
    assert native.lib().snake_plan(ctypes.byref(c), 8192, ctypes.byref(lay2)) == 0
    assert lay2.n_cand == 20168 and lay2.jscratch == 2048 * (20168 + 64) * 4   # global link tables
    assert lay.grid == 8192 * 4 * 1600
    # every-step / no auto-reset: the 40x40 four-frame board needs no worker link tables
    for kw in (dict(autoreset=False), dict(autoreset='every_step')):
        c = cfg(native, height=40, width=40, num_snakes=8, vision_range=5, frame_stack=4, **kw)
        assert native.lib().snake_plan(ctypes.byref(c), 64, ctypes.byref(lay)) == 0
        assert lay.jscratch == 0 and lay.spawn == 64 * 672 * 4, kw
    # in-step spawn-ahead on that board (spawn_background=-1): one record per env,
    # the k_post_lean workers' link tables
    c = cfg(native, height=40, width=40, num_snakes=8, vision_range=5, frame_stack=4, spawn_background=-1)
    assert native.lib().snake_plan(ctypes.byref(c), 64, ctypes.byref(lay)) == 0
    assert lay.jscratch == 64 * (16424 + 64) * 4 and lay.spawn == 64 * 672 * 4


@pytest.mark.parametrize('kw,N,bg', [
    (dict(height=20, width=20), 4096, True),                     # cfg2: 50 MiB of obs per step
    (dict(height=20, width=20), 8192, False),                    # 100 MiB
    (dict(height=20, width=20, vision_range=5), 8192, True),     # cfg3's board at 8 192 envs
    (dict(height=20, width=20, vision_range=5), 16384, False),   # more than 8 192 envs
    (dict(height=20, width=20, spawn_background=-1), 4096, False),
    (dict(height=20, width=20, spawn_ahead=-1), 1024, False),    # nothing to draw ahead
])
def test_plan_background_automatic(native, kw, N, bg):
    """spawn_background = 0 (automatic) turns the background spawn kernel on for
    batches of at most 8 192 envs and 64 MiB of observations per step (round 5):
    the layout then holds a spawn-ahead record per queue set (four) and env."""
    c = cfg(native, num_snakes=4, **kw)
    lay = native.SnakeLayout()
    assert native.lib().snake_plan(ctypes.byref(c), N, ctypes.byref(lay)) == 0
    assert lay.spawn == (4 if bg else 1) * N * 672 * 4, (kw, N)


@pytest.mark.parametrize('H,W,L,N', [(50, 50, 3, 16384), (72, 72, 3, 4096), (100, 100, 2, 65536)])
def test_plan_large_boards(native, H, W, L, N):
    """Boards whose k_logic frames do not fit four waves per workgroup (ADVICE r4:
    4 x 41 KB at 50x50 and 16 envs per wave) still plan: snake_plan runs the
    launch-side checks too (build_kcfg), which pick one wave per workgroup or
    fewer envs per wave instead of a launch that fails."""
    c = cfg(native, height=H, width=W, snake_length=L, num_snakes=4, vision_range=3)
    lay = native.SnakeLayout()
    assert native.lib().snake_plan(ctypes.byref(c), N, ctypes.byref(lay)) == 0, \
        native.lib().snake_last_error().decode()


@pytest.mark.parametrize('kw,msg', [
    (dict(num_snakes=0), 'num_snakes'), (dict(num_snakes=17), 'num_snakes'),
    (dict(snake_length=1), 'snake_length'), (dict(height=2), 'height'),
    (dict(num_fruits=0), 'num_fruits'), (dict(frame_stack=0), 'frame_stack'),
    (dict(height=5, width=5, num_snakes=4, snake_length=3), 'too small'),
    # 61 interior cells for 60 snake cells: ~1e-5 of the spawn draws are disjoint
    (dict(height=3, width=63, num_snakes=4, snake_length=15), 'too crowded'),
])
def test_plan_rejects(native, kw, msg):
    c = cfg(native, **kw)
    lay = native.SnakeLayout()
    rc = native.lib().snake_plan(ctypes.byref(c), 16, ctypes.byref(lay))
    assert rc == -1
    assert msg in native.lib().snake_last_error().decode()
    with pytest.raises(ValueError):
        native.check(rc)


def test_reward_dict_keys_are_checked(native):
    from marlenv.config import build_cfg
    with pytest.raises(KeyError):                   # snake_env.py:77-80
        build_cfg(reward_dict={'fruit': 1.0})
    c, meta = build_cfg(num_snakes=4)
    assert meta['num_fruits'] == 3                  # int(round(0.8 * 4))
    assert build_cfg(num_snakes=1)[1]['num_fruits'] == 1


def table(native, H, W, L):
    c = cfg(native, height=H, width=W, snake_length=L, num_snakes=1)
    n = native.lib().snake_build_candidates(ctypes.byref(c), None, 0)
    out = np.zeros(n * L, np.int16)
    assert native.lib().snake_build_candidates(ctypes.byref(c), out.ctypes.data_as(ctypes.c_void_p), out.size) == n
    cells = out.reshape(n, L).astype(np.int64)
    return np.stack([cells // W, cells % W], -1).astype(np.int16)


def test_spawn_table_matches_reference(native):
    z = G.load('candidates.npz')
    for k in z.files:
        if k.startswith('full_'):
            H, W = map(int, k.split('_')[1].split('x'))
            L = int(k.split('_L')[1])
            np.testing.assert_array_equal(table(native, H, W, L), z[k])
    for H, W, L, C, dg in z['digest_meta']:
        t = table(native, int(H), int(W), int(L))
        assert t.shape[0] == int(C) and G.digest(t) == int(dg)
