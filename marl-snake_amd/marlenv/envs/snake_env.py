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
        torch = _torch()
        self._pin = torch.empty(0)

    # ------------------------------------------------------------- RNG sync
    def _push_rng(self):
        if self._rng != 'global':
            return
        torch = _torch()
        st = np.random.get_state(legacy=True)
        key = np.ascontiguousarray(np.asarray(st[1], dtype=np.uint32)).view(np.int32)
        self._vec.set_mt_state(0, torch.from_numpy(key), int(st[2]))

    def _pull_rng(self):
        if self._rng != 'global':
            return
        mt, pos = self._vec.mt_state()
        key = mt[0].cpu().numpy().view(np.uint32).copy()
        p = int(pos[0].item())
        st = np.random.get_state(legacy=True)
        np.random.set_state((st[0], key, p, st[3], st[4]))

    # -------------------------------------------------------------- the API
    def reset(self):
        self._push_rng()
        obs = self._vec.reset()
        out = obs[0].cpu().numpy()
        self._pull_rng()
        if int(self._vec.spawn_failures()[0]):
            raise RuntimeError('reset gave up after 2^16 spawn permutations without disjoint snakes')
        self.frame_buffer = []
        return np.array(out, dtype=np.uint8)

    def seed(self, seed=42):
        # snake_env.py:161-163 only seeds an unused self.np_random
        self.np_random = np.random.RandomState(seed)
        return [seed]

    def step(self, actions):
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
        self._push_rng()
        obs, rew, done, info = self._vec.step(np.array(acts, np.int64).reshape(1, -1))
        torch = _torch()
        packed = [obs[0].reshape(-1), rew[0].view(torch.uint8), done[0].view(torch.uint8),
                  info['episode_done'].view(torch.uint8), info['rank'][0].view(torch.uint8),
                  info['episode_scores'][0].contiguous().view(torch.uint8),
                  info['episode_steps'][0].contiguous().view(torch.uint8),
                  info['episode_fruits'][0].contiguous().view(torch.uint8),
                  info['episode_kills'][0].contiguous().view(torch.uint8),
                  info['error'].view(torch.uint8)]
        host = torch.cat(packed).cpu().numpy()
        self._pull_rng()
        S = self.num_snakes
        o = 0
        n = obs[0].numel()
        obs_np = host[o:o + n].reshape(self._vec.obs_shape).copy(); o += n
        rews = host[o:o + 8 * S].view(np.float64); o += 8 * S
        dones = host[o:o + S].astype(bool); o += S
        ep_done = bool(host[o]); o += 1
        rank = host[o:o + 4 * S].view(np.int32); o += 4 * S
        stats = []
        for _ in range(4):
            stats.append(host[o:o + 8 * S].view(np.float64).copy()); o += 8 * S
        err = int(host[o:o + 4].view(np.int32)[0])
        if err:
            raise KeyError('invalid action for an alive snake (action_angle_dict lookup)')
        info_out = {}
        if ep_done:
            info_out = {'rank': [np.int64(r) for r in rank],
                        'episode_scores': stats[0], 'episode_steps': stats[1],
                        'episode_fruits': stats[2], 'episode_kills': stats[3]}
        return obs_np, [float(r) for r in rews], [bool(d) for d in dones], info_out

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
