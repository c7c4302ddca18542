"""SnakeEnv: the reference's single-env class, backed by the HIP kernels.

Drop-in for marlenv/marlenv/envs/snake_env.py:SnakeEnv (reset :131-159,
step :301-414): same constructor kwargs, same attributes callers read
(num_snakes, grid_shape, vision_range, frame_stack, obs_ch, action_dict,
observation_space, action_space, reward_dict, num_fruits, max_episode_steps),
same return types -- a fresh uint8 ndarray of shape (S, h, w, 8*fs), a list of
float rewards, a list of bool dones and an info dict ({} or the episode
summary: rank, episode_scores/steps/fruits/kills).

Randomness: the reference draws from numpy's GLOBAL legacy RandomState
(np.random.permutation / np.random.randint). This class follows it exactly:
before each reset()/step() the global MT19937 state is loaded into the env's
device-side generator, and after the call the advanced state is written back
with np.random.set_state. So ``np.random.seed(s)`` before make_snake() /
reset() reproduces the reference trajectory bit for bit, and user code that
interleaves its own np.random calls sees the same stream it would with the
reference. (rng='own' keeps a private per-env stream seeded with ``seed``.)

Transfers: one pinned host->device copy and one device->host copy per call
(_setup_io); code that writes this env's device state directly (the vector
env's set_mt_state/inject on env._vec) calls env._fetch() afterwards so the
host mirror of the key and env record is current.

Deviation: on an invalid action the reference raises KeyError after having
already turned the lower-index snakes; here KeyError is raised with the env
untouched.
"""
import datetime
import os
import warnings

import numpy as np

from .. import spaces
from ..config import ACTION_ANGLE_DICT, DEFAULT_ACTION_DICT, DEFAULT_REWARD_DICT, MAX_EPISODE_STEPS
from ..vec_env import SnakeVecEnv, _torch

FEATURE_CHANNEL = 8     # envs/constants.py:2
RGB_CHANNEL = 3         # envs/constants.py:1


def _mt_twist(key):
    """mt19937_gen on a uint32[624] key (numpy's generator), in three slices:
    new[i] mixes old[i], old[i+1] and old[i+397] for i < 227, new[i-227] after,
    and the last word wraps to new[0]."""
    k = key.astype(np.uint32).copy()

    def mix(cur, nxt, x):
        y = (cur & np.uint32(0x80000000)) | (nxt & np.uint32(0x7fffffff))
        return x ^ (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), np.uint32(0x9908b0df), np.uint32(0))
    k[0:227] = mix(k[0:227], k[1:228], k[397:624])
    k[227:454] = mix(k[227:454], k[228:455], k[0:227])
    k[454:623] = mix(k[454:623], k[455:624], k[227:396])
    k[623] = mix(k[623:624], k[0:1], k[396:397])[0]
    return k


class SnakeEnv:
    default_action_dict = DEFAULT_ACTION_DICT
    action_angle_dict = ACTION_ANGLE_DICT
    default_reward_dict = DEFAULT_REWARD_DICT
    reward_keys = DEFAULT_REWARD_DICT.keys()
    max_episode_steps = MAX_EPISODE_STEPS
    _coop = False

    def __init__(self, height=20, width=20, num_snakes=4, snake_length=3, vision_range=None,
                 frame_stack=1, observer='snake', *args, device=None, rng='global', seed=0,
                 **kwargs):
        self._vec = SnakeVecEnv(1, num_snakes=num_snakes, height=height, width=width,
                                snake_length=snake_length, vision_range=vision_range,
                                frame_stack=frame_stack, observer=observer, coop=self._coop,
                                autoreset=False, device=device, seed=seed, **kwargs)
        m = self._vec.meta
        self.reward_dict = m['reward_dict']
        self.max_episode_steps = m['max_episode_steps']
        self.num_snakes = num_snakes
        self.num_fruits = m['num_fruits']
        self.grid_shape = (height, width)
        self.frame_buffer = []
        self.snake_length = snake_length
        self.vision_range = vision_range
        self.observer = observer
        self.low = 0
        self.image_obs = False
        self.high = 1
        self.action_dict = (SnakeEnv.default_action_dict if observer == 'human'
                            else SnakeEnv.action_angle_dict)
        self.action_space = spaces.Discrete(len(self.action_dict) * self.num_snakes)
        self.frame_stack = frame_stack
        self.obs_ch = FEATURE_CHANNEL * self.frame_stack
        self.observation_space = spaces.Box(self.low, self.high, self._vec.obs_shape, np.uint8)
        if rng not in ('global', 'own'):
            raise ValueError("rng must be 'global' or 'own'")
        self._rng = rng
        self.np_random = None
        self._setup_io()

    # ------------------------------------------------------- packed transfers
    def _setup_io(self):
        """One device buffer holds everything a step moves between host and
        device: [MT key | env record | actions | obs | rew | done | ep_done |
        rank | ep_stats | err]. The env's key and env-record state tensors are
        re-pointed into it, so a step is ONE pinned host->device copy (the
        global numpy MT19937 state, the env record, the actions), the launches,
        and ONE device->host copy (outputs + the advanced key) -- instead of a
        624-word push, scalar writes, a gather and three read-backs."""
        torch = _torch()
        v, S = self._vec, self.num_snakes
        dev = v.device
        obs_bytes = int(np.prod(v.obs_shape))
        sizes = [('env', 32), ('mt', 624 * 4), ('act', S), ('obs', obs_bytes), ('rew', 8 * S), ('done', S),
                 ('ep_done', 1), ('rank', 4 * S), ('ep_stats', 32 * S), ('err', 4)]
        off, o = {}, 0
        for name, n in sizes:
            off[name] = (o, n)
            o = (o + n + 15) // 16 * 16
        # bytes [12, obs) go host -> device: env words 3.. (MT position, spawn
        # status, failure flag), the key, the actions; words 0-2 (alive, episode
        # length, ring slot) are only ever written on the device
        self._io_in = off['obs'][0]
        self._io_bytes = o
        buf = torch.zeros(o, dtype=torch.uint8, device=dev)
        buf[off['mt'][0]:off['mt'][0] + 2496].copy_(v.mt.view(torch.uint8)[:2496])
        buf[off['env'][0]:off['env'][0] + 32].copy_(v.env_rec.view(torch.uint8)[:32])
        view = lambda name, dt: buf[off[name][0]:off[name][0] + off[name][1]].view(dt)  # noqa: E731
        v.mt = view('mt', torch.int32)
        v.env_rec = view('env', torch.int32)
        st = v._state
        st.mt = v.mt.data_ptr()
        st.env = v.env_rec.data_ptr()
        self._dev = buf
        self._act_dev = view('act', torch.int8)
        self._obs_dev = view('obs', torch.uint8).view((1,) + v.obs_shape)
        from .._native import SnakeOut
        self._so = SnakeOut(*(buf.data_ptr() + off[k][0] for k in ('obs', 'rew', 'done', 'ep_done', 'rank',
                                                                    'ep_stats', 'err')))
        self._hin = torch.empty(self._io_in, dtype=torch.uint8, pin_memory=True)
        self._hout = torch.empty(o, dtype=torch.uint8, pin_memory=True)
        hin, hout = self._hin.numpy(), self._hout.numpy()
        self._in_key = hin[off['mt'][0]:off['mt'][0] + 2496].view(np.uint32)
        self._in_env = hin[off['env'][0]:off['env'][0] + 32].view(np.int32)
        self._in_act = hin[off['act'][0]:off['act'][0] + S].view(np.int8)
        hv = lambda name, dt: hout[off[name][0]:off[name][0] + off[name][1]].view(dt)  # noqa: E731
        self._out = {k: hv(k, dt) for k, dt in (('mt', np.uint32), ('env', np.int32), ('obs', np.uint8),
                                                 ('rew', np.float64), ('done', np.uint8), ('ep_done', np.uint8),
                                                 ('rank', np.int32), ('ep_stats', np.float64), ('err', np.int32))}
        self._fetch()                                   # host mirror of the key and env record

    def _fetch(self, upto=None):
        torch = _torch()
        n = self._io_bytes if upto is None else upto
        self._hout[:n].copy_(self._dev[:n], non_blocking=True)
        torch.cuda.current_stream(self._vec.device).synchronize()

    def _stage_in(self, acts=None):
        """Host side of the push: the key (numpy's global MT19937, or the env's
        own), the env record as last fetched (MT position from numpy's state, the
        spawn-ahead record voided as set_mt_state does), the actions."""
        out = self._out
        self._in_env[:] = out['env']
        if self._rng == 'global':
            st = np.random.get_state(legacy=True)
            self._in_key[:] = np.asarray(st[1], dtype=np.uint32)
            self._in_env[3] = int(st[2])
            self._in_env[4] = 0
        else:
            self._in_key[:] = out['mt']
        if acts is not None:
            self._in_act[:] = acts
        self._dev[12:self._io_in].copy_(self._hin[12:], non_blocking=True)

    def _publish_rng(self):
        if self._rng != 'global':
            return
        key, pos = self._out['mt'].copy(), int(self._out['env'][3])
        if pos > 624:          # the device left the key's twist pending (include/snake_env.h)
            key, pos = _mt_twist(key), pos - 624
        st = np.random.get_state(legacy=True)
        np.random.set_state((st[0], key, pos, st[3], st[4]))

    # -------------------------------------------------------------- the API
    def reset(self):
        import ctypes
        torch = _torch()
        v = self._vec
        self._stage_in()
        with torch.cuda.device(v.device):
            from .._native import check
            check(v._L.snake_reset(ctypes.byref(v.cfg), ctypes.byref(v._state), 1, None,
                                   ctypes.byref(self._so), v._stream()))
        v._reset_done = True
        self._fetch()
        self._publish_rng()
        if int(self._out['env'][5]):
            raise RuntimeError('reset gave up after 2^16 spawn permutations without disjoint snakes')
        self.frame_buffer = []
        return self._out['obs'].reshape(v.obs_shape).copy()

    def seed(self, seed=42):
        # snake_env.py:161-163 only seeds an unused self.np_random
        self.np_random = np.random.RandomState(seed)
        return [seed]

    def step(self, actions):
        import ctypes
        if isinstance(actions, int):
            actions = [actions]
        assert len(actions) == self.num_snakes
        acts = []
        for a in actions:
            if isinstance(a, np.ndarray):
                a = a.item()
            if isinstance(a, float) and not a.is_integer():
                a = -1 if self.observer == 'snake' else 99  # KeyError / ignored, as the dict lookup
            acts.append(int(a))
        if self.observer == 'human':
            acts = [a if 0 <= a <= 4 else 0 for a in acts]  # non-matching actions keep the heading
        v = self._vec
        if not v._reset_done:
            raise RuntimeError('call reset() before step()')
        acts = np.clip(np.asarray(acts, np.int64), -128, 127).astype(np.int8)
        self._stage_in(acts)
        from .._native import check
        check(v._L.snake_step(ctypes.byref(v.cfg), ctypes.byref(v._state), 1,
                              ctypes.c_void_p(self._act_dev.data_ptr()), ctypes.byref(self._so), v._stream()))
        self._fetch()
        out = self._out
        if int(out['err'][0]) == 1:
            # the env was left untouched on the device; numpy's stream was not advanced
            raise KeyError('invalid action for an alive snake (action_angle_dict lookup)')
        self._publish_rng()
        S = self.num_snakes
        info_out = {}
        if out['ep_done'][0]:
            es = out['ep_stats'].reshape(4, S)
            info_out = {'rank': [np.int64(r) for r in out['rank']],
                        'episode_scores': es[0].copy(), 'episode_steps': es[1].copy(),
                        'episode_fruits': es[2].copy(), 'episode_kills': es[3].copy()}
        return (out['obs'].reshape(v.obs_shape).copy(), [float(r) for r in out['rew']],
                [bool(d) for d in out['done']], info_out)

    def _done_fn(self, dones):
        return all(dones)

    # ----------------------------------------------------------- inspection
    @property
    def grid(self):
        """Current grid as an int64 ndarray (the reference's self.grid)."""
        return self._vec.grids()[0].cpu().numpy().astype(np.int64)

    @property
    def alive_snakes(self):
        return int(self._vec.alive_counters()[0].item())

    @property
    def episode_length(self):
        return int(self._vec.episode_lengths()[0].item())

    def render(self, mode='ascii'):
        """SnakeEnv.render (snake_env.py:267-296): 'ascii' prints the grid,
        'rgb_array' returns rgb_from_grid of it (H, W, 3) uint8, 'gif' appends
        image_from_grid's PIL frame to frame_buffer (save_gif writes them),
        'human' does nothing. The RGB frame comes from the device (k_render)."""
        if mode == 'ascii':
            sym = {0: '.', 1: '#', 2: 'o', 3: 'H', 4: 'b', 5: 't'}
            print('\n'.join(''.join(sym[v % 10] for v in row) for row in self.grid))
        elif mode == 'rgb_array':
            return self._vec.render_rgb()[0].cpu().numpy()
        elif mode == 'gif':
            from PIL import Image
            from ..core.render import upscale
            rgb = self._vec.render_rgb()[0].cpu().numpy()
            self.frame_buffer.append(Image.fromarray(upscale(rgb), 'RGB'))
        elif mode == 'human':
            pass

    def save_gif(self, fp=None):
        """SnakeEnv.save_gif (snake_env.py:419-437)."""
        if fp is None:
            save_dir = os.path.join(os.getcwd(), 'tmp')
            fp = os.path.join(save_dir, '{}.gif'.format(datetime.datetime.now().strftime('%Y%m%d%H%M%S')))
            os.makedirs(save_dir, exist_ok=True)
        if not self.frame_buffer:
            warnings.warn("You must call render('gif') first. No images to save.")
        else:
            print('Saving image to {}'.format(fp))
            self.frame_buffer[0].save(fp, save_all=True, append_images=self.frame_buffer[1:],
                                      format='GIF', loop=0)
        return fp

    def close(self):
        pass
