"""Host-side logic that needs no GPU: env-id registry, wrappers' spaces,
sharding arithmetic used by bench.py, and the library refusing to run
without a HIP device (no CPU fallback)."""
import numpy as np
import pytest


def test_graph_env_is_out_of_scope():
    from marlenv import make_snake
    with pytest.raises(NotImplementedError):
        make_snake(num_envs=1, env_id='SnakeGraph-v1')
    with pytest.raises(KeyError):
        make_snake(num_envs=1, env_id='Nope-v0')


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from marlenv import SnakeVecEnv
    with pytest.raises(RuntimeError, match='no CPU fallback'):
        SnakeVecEnv(4, num_snakes=4)


def test_spaces():
    from marlenv import spaces
    d = spaces.Discrete(3, seed=0)
    xs = {d.sample() for _ in range(200)}
    assert xs == {0, 1, 2}
    st = np.random.get_state()
    d.sample()
    assert (np.random.get_state()[1] == st[1]).all()   # never touches the global RNG
    b = spaces.Box(0, 255, (4, 11, 11, 8), np.uint8)
    assert b.shape == (4, 11, 11, 8) and b.contains(np.zeros(b.shape, np.uint8))


def test_shard_ranges():
    from bench import shard_range
    N = 262144
    for G in (1, 2, 4, 8):
        spans = [shard_range(N, G, r) for r in range(G)]
        assert spans[0][0] == 0 and spans[-1][1] == N
        for (a, b), (c, d) in zip(spans, spans[1:]):
            assert b == c
        assert sum(b - a for a, b in spans) == N


def test_reference_import_paths_resolve():
    """train_dqn.py:22 / train_ga.py:25 / test_env.py:1 import through the
    distribution dir: `from marlenv.marlenv.wrappers import make_snake, RenderGUI`."""
    from marlenv.marlenv.wrappers import RenderGUI, make_snake
    import marlenv
    import marlenv.marlenv.envs.snake_env as se
    assert make_snake is marlenv.make_snake
    assert se.SnakeEnv is marlenv.SnakeEnv
    assert issubclass(RenderGUI, marlenv.wrappers.Wrapper)


def test_render_palette_matches_reference():
    """The palette the product hands snake_render_rgb == the reference's colour
    of every (code, owner) (tests/golden/render.npz, from grid_util.rgb_from_grid)."""
    from marlenv.core.render import palette, upscale
    import golden_io as G
    z = G.load('render.npz')
    np.testing.assert_array_equal(palette(), z['palette'])
    big = upscale(z['rgb'][0])
    assert big.shape == (300, 300, 3) and (big[::15, ::15] == z['rgb'][0]).all()


def test_autoreset_codes():
    from marlenv.config import autoreset_code, build_cfg
    assert autoreset_code(True) == 1 and autoreset_code(False) == 0
    assert autoreset_code('every_step') == 2
    with pytest.raises(ValueError):
        autoreset_code('sometimes')
    cfg, _ = build_cfg(autoreset='every_step')
    assert cfg.autoreset == 2


def test_dqn_rejects_mismatched_state_dict():
    """The DQN kernels hard-code the reference's layer widths (train_dqn.py:104-151):
    a state dict with other conv/fc widths or bias lengths must raise before any
    weight is packed (no GPU needed to reach the check)."""
    torch = pytest.importorskip('torch')
    from marlenv import _native
    try:
        _native.lib()
    except _native.NativeError:
        pytest.skip('libsnake_amd.so not built')
    from marlenv.dqn import DQNForward
    H = W = 11
    C, A = 8, 3

    def sd(**over):
        d = {'conv1.weight': (32, C, 3, 3), 'conv1.bias': (32,), 'conv2.weight': (64, 32, 3, 3),
             'conv2.bias': (64,), 'conv3.weight': (64, 64, 3, 3), 'conv3.bias': (64,),
             'fc1.weight': (256, 64 * H * W), 'fc1.bias': (256,), 'fc2.weight': (128, 256), 'fc2.bias': (128,),
             'fc3.weight': (A, 128), 'fc3.bias': (A,)}
        d.update(over)
        return {k: torch.zeros(v) for k, v in d.items()}

    for over in ({'conv2.weight': (48, 32, 3, 3)}, {'fc2.weight': (128, 128)}, {'conv3.bias': (63,)},
                 {'fc1.weight': (256, 64 * H * W + 1)}, {'fc3.bias': (A + 1,)}):
        for precision in ('bf16', 'fp32'):
            with pytest.raises(ValueError):
                DQNForward(sd(**over), H, W, C, A, device='cpu', precision=precision)
    bad = sd()
    del bad['fc2.bias']
    with pytest.raises(ValueError):
        DQNForward(bad, H, W, C, A, device='cpu')
