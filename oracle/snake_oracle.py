"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE -- see snake_oracle.h).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, as the parity checker / the timed CPU baseline. The product
(marl-snake_amd/) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, 'libsnake_oracle.so')

DEFAULT_REWARD = {'fruit': 10.0, 'kill': 0.0, 'lose': -0.5, 'win': 0.0, 'time': -0.001}


class SoCfg(ctypes.Structure):
    _fields_ = [('height', ctypes.c_int32), ('width', ctypes.c_int32),
                ('num_snakes', ctypes.c_int32), ('snake_length', ctypes.c_int32),
                ('vision_range', ctypes.c_int32), ('frame_stack', ctypes.c_int32),
                ('observer', ctypes.c_int32), ('num_fruits', ctypes.c_int32),
                ('rew_fruit', ctypes.c_double), ('rew_kill', ctypes.c_double),
                ('rew_lose', ctypes.c_double), ('rew_win', ctypes.c_double),
                ('rew_time', ctypes.c_double), ('max_episode_steps', ctypes.c_double),
                ('coop', ctypes.c_int32)]


class SoInfo(ctypes.Structure):
    _fields_ = [('rank', ctypes.c_int64 * 16), ('scores', ctypes.c_double * 16),
                ('steps', ctypes.c_double * 16), ('fruits', ctypes.c_double * 16),
                ('kills', ctypes.c_double * 16)]


def build():
    subprocess.run(['make', '-s', '-C', _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.so_create.restype = P
        L.so_create.argtypes = [ctypes.POINTER(SoCfg), ctypes.c_uint32]
        L.so_destroy.argtypes = [P]
        L.so_obs_size.restype = ctypes.c_int64
        L.so_obs_size.argtypes = [P]
        L.so_reset.argtypes = [P, P]
        L.so_step.argtypes = [P, P, P, P, P, ctypes.POINTER(SoInfo)]
        L.so_get_grid.argtypes = [P, P]
        L.so_alive_snakes.restype = ctypes.c_int64
        L.so_alive_snakes.argtypes = [P]
        L.so_episode_length.restype = ctypes.c_int64
        L.so_episode_length.argtypes = [P]
        L.so_get_snakes.argtypes = [P, P]
        L.so_inject.argtypes = [P, P, P, P, P, ctypes.c_int64, ctypes.c_int64]
        L.so_rng_raw.argtypes = [ctypes.c_uint32, ctypes.c_int64, P]
        L.so_rng_randint.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64, P,
                                     ctypes.POINTER(ctypes.c_uint32)]
        L.so_rng_permutation.argtypes = [ctypes.c_uint32, ctypes.c_int64, P,
                                         ctypes.POINTER(ctypes.c_uint32)]
        L.so_rollout.restype = ctypes.c_int64
        L.so_rollout.argtypes = [ctypes.POINTER(SoCfg), ctypes.c_int32, ctypes.c_uint32, ctypes.c_int64,
                                 ctypes.c_uint32]
        L.so_candidates.restype = ctypes.c_int64
        L.so_candidates.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, P]
        L.so_batch_create.restype = P
        L.so_batch_create.argtypes = [ctypes.POINTER(SoCfg), ctypes.c_int64, ctypes.c_uint32]
        L.so_batch_destroy.argtypes = [P]
        L.so_batch_reset.argtypes = [P, P, ctypes.c_int]
        L.so_batch_step.argtypes = [P, P, P, P, P, P, P, P, P, ctypes.c_int]
        L.so_batch_grids.argtypes = [P, P]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def make_cfg(height=20, width=20, num_snakes=4, snake_length=3, vision_range=None,
             frame_stack=1, observer='snake', reward_dict=None, num_fruits=None,
             max_episode_steps=1e4, coop=False):
    r = dict(DEFAULT_REWARD if reward_dict is None else reward_dict)
    if num_fruits is None:
        num_fruits = int(round(num_snakes * 0.8))
    return SoCfg(height, width, num_snakes, snake_length, int(vision_range or 0), frame_stack,
                 1 if observer == 'human' else 0, num_fruits, float(r['fruit']), float(r['kill']),
                 float(r['lose']), float(r['win']), float(r['time']), float(max_episode_steps),
                1 if coop else 0)


class OracleEnv:
    """One reference SnakeEnv, restated in C: env == SnakeEnv after np.random.seed(seed)."""

    def __init__(self, seed=0, **cfg):
        self.cfg_kw = cfg
        self.cfg = make_cfg(**cfg)
        self.S = self.cfg.num_snakes
        self.H, self.W = self.cfg.height, self.cfg.width
        vr = self.cfg.vision_range
        self.oh = self.ow = 2 * vr + 1 if vr else None
        if not vr:
            self.oh, self.ow = self.H, self.W
        self.C = 8 * self.cfg.frame_stack
        self._h = lib().so_create(ctypes.byref(self.cfg), ctypes.c_uint32(seed & 0xffffffff))
        if not self._h:
            raise ValueError('invalid oracle config')
        self.obs_shape = (self.S, self.oh, self.ow, self.C)

    def __del__(self):
        h = getattr(self, '_h', None)
        if h:
            lib().so_destroy(h)
            self._h = None

    def reset(self):
        obs = np.zeros(self.obs_shape, np.uint8)
        lib().so_reset(self._h, _ptr(obs))
        return obs

    def step(self, actions):
        a = np.ascontiguousarray(np.asarray(actions, dtype=np.int32).reshape(self.S))
        obs = np.zeros(self.obs_shape, np.uint8)
        rews = np.zeros(self.S, np.float64)
        dones = np.zeros(self.S, np.uint8)
        info = SoInfo()
        rc = lib().so_step(self._h, _ptr(a), _ptr(obs), _ptr(rews), _ptr(dones), ctypes.byref(info))
        if rc < 0:
            raise KeyError('invalid action')
        out_info = {}
        if rc == 1:
            S = self.S
            out_info = {'rank': list(info.rank[:S]),
                        'episode_scores': np.array(info.scores[:S]),
                        'episode_steps': np.array(info.steps[:S]),
                        'episode_fruits': np.array(info.fruits[:S]),
                        'episode_kills': np.array(info.kills[:S])}
        return obs, rews, dones.astype(bool), out_info

    @property
    def grid(self):
        g = np.zeros((self.H, self.W), np.uint8)
        lib().so_get_grid(self._h, _ptr(g))
        return g

    @property
    def alive_snakes(self):
        return int(lib().so_alive_snakes(self._h))

    @property
    def episode_length(self):
        return int(lib().so_episode_length(self._h))

    def snakes(self):
        out = np.zeros((self.S, 7), np.int32)
        lib().so_get_snakes(self._h, _ptr(out))
        return out

    def inject(self, grid, snakes, alive_snakes, episode_length=0):
        """snakes: list of (coords[(r,c),...], alive)."""
        g = np.ascontiguousarray(np.asarray(grid, np.int32))
        coords = np.ascontiguousarray(np.concatenate([np.asarray(c, np.int32).reshape(-1, 2)
                                                      for c, _ in snakes]))
        off = np.ascontiguousarray(np.cumsum([0] + [len(c) for c, _ in snakes]).astype(np.int32))
        alive = np.ascontiguousarray(np.array([bool(a) for _, a in snakes], np.uint8))
        rc = lib().so_inject(self._h, _ptr(g), _ptr(coords), _ptr(off), _ptr(alive),
                             int(alive_snakes), int(episode_length))
        if rc != 0:
            raise ValueError('inject failed')


class OracleBatch:
    """n oracle envs (env i == SnakeEnv after np.random.seed(seed + i)) stepped
    together on `threads` host threads with the vector env's auto-reset; outputs
    shaped like SnakeVecEnv.step's (so_batch_step)."""

    def __init__(self, n, seed=0, threads=None, **cfg):
        self.cfg = make_cfg(**cfg)
        self.n, self.S = int(n), self.cfg.num_snakes
        self.H, self.W = self.cfg.height, self.cfg.width
        vr = self.cfg.vision_range
        oh = ow = 2 * vr + 1 if vr else None
        if not vr:
            oh, ow = self.H, self.W
        self.obs_shape = (self.n, self.S, oh, ow, 8 * self.cfg.frame_stack)
        self.threads = int(threads or min(16, len(os.sched_getaffinity(0))))
        self._h = lib().so_batch_create(ctypes.byref(self.cfg), self.n, ctypes.c_uint32(seed & 0xffffffff))
        if not self._h:
            raise ValueError('invalid oracle config')

    def __del__(self):
        h = getattr(self, '_h', None)
        if h:
            lib().so_batch_destroy(h)
            self._h = None

    def reset(self):
        obs = np.zeros(self.obs_shape, np.uint8)
        lib().so_batch_reset(self._h, _ptr(obs), self.threads)
        return obs

    def step(self, actions):
        a = np.ascontiguousarray(np.asarray(actions).astype(np.int8).reshape(self.n, self.S))
        n, S = self.n, self.S
        obs = np.zeros(self.obs_shape, np.uint8)
        rew = np.zeros((n, S), np.float64)
        done = np.zeros((n, S), np.uint8)
        ep_done = np.zeros(n, np.uint8)
        rank = np.zeros((n, S), np.int32)
        ep_stats = np.zeros((n, 4, S), np.float64)
        err = np.zeros(n, np.int32)
        lib().so_batch_step(self._h, _ptr(a), _ptr(obs), _ptr(rew), _ptr(done), _ptr(ep_done), _ptr(rank),
                            _ptr(ep_stats), _ptr(err), self.threads)
        info = {'episode_done': ep_done.astype(bool), 'rank': rank, 'episode_scores': ep_stats[:, 0],
                'episode_steps': ep_stats[:, 1], 'episode_fruits': ep_stats[:, 2],
                'episode_kills': ep_stats[:, 3], 'error': err}
        return obs, rew, done.astype(bool), info

    def grids(self):
        g = np.zeros((self.n, self.H, self.W), np.uint8)
        lib().so_batch_grids(self._h, _ptr(g))
        return g


def rollout(n_env, seed, steps, act_seed=12345, **cfg):
    """so_rollout: n_env C envs x `steps` random-action steps with all-done resets;
    returns the env-steps run (the CPU baseline's unit of work)."""
    c = make_cfg(**cfg)
    n = lib().so_rollout(ctypes.byref(c), int(n_env), int(seed) & 0xffffffff, int(steps), int(act_seed))
    if n < 0:
        raise ValueError('so_rollout failed')
    return int(n)


def rng_raw(seed, n):
    out = np.zeros(n, np.uint32)
    lib().so_rng_raw(seed, n, _ptr(out))
    return out


def rng_randint(seed, n, k):
    out = np.zeros(k, np.int64)
    nxt = ctypes.c_uint32()
    lib().so_rng_randint(seed, n, k, _ptr(out), ctypes.byref(nxt))
    return out, nxt.value


def rng_permutation(seed, n):
    out = np.zeros(n, np.int64)
    nxt = ctypes.c_uint32()
    lib().so_rng_permutation(seed, n, _ptr(out), ctypes.byref(nxt))
    return out, nxt.value


def candidates(H, W, L):
    n = lib().so_candidates(H, W, L, None)
    out = np.zeros((n, L, 2), np.int16)
    lib().so_candidates(H, W, L, _ptr(out))
    return out


# ------------------------------------------------------------------ rendering
# CellColors (marlenv/marlenv/core/snake.py:14-30), restated for the checker.
_WHEEL = [(104, 255, 0), (255, 191, 0), (255, 0, 92), (0, 111, 255)]
_HEAD_WHEEL = [tuple(min(255, int(x * 2.0)) for x in rgb) for rgb in _WHEEL]
CELL_COLORS = {0: [(0, 0, 0)], 1: [(32, 32, 32)], 2: [(223, 7, 22)],
               3: _HEAD_WHEEL, 4: _WHEEL, 5: _WHEEL}


def rgb_from_grid(grid):
    """rgb_from_grid(grid, Cell, CellColors) (grid_util.py:164-175): per cell,
    colour list of code v % 10, entry (v // 10) % len, times 0.7 ** cycle with
    cycle = (v // 10) // len, truncated to uint8. Cell-by-cell, as the reference."""
    grid = np.asarray(grid)
    rgb = np.zeros((*grid.shape, 3), dtype=np.uint8)
    for r in range(grid.shape[0]):
        for c in range(grid.shape[1]):
            v = int(grid[r, c])
            colors = CELL_COLORS[v % 10]
            cell_id = v // 10
            color = np.array(colors[cell_id % len(colors)])
            rgb[r, c] = (color * 0.7**(cell_id // len(colors))).astype(np.uint8)
    return rgb
