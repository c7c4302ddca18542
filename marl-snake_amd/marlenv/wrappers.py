"""make_snake and the agent wrappers (reference marlenv/marlenv/wrappers.py).

make_snake(num_envs=1, ...) returns the single-env compat SnakeEnv wrapped in
SingleMultiAgent (or SingleAgent when num_snakes == 1), as wrappers.py:203-223.
make_snake(num_envs>1, ...) returns a SnakeVecEnv: all envs stepped by one HIP
launch with all-done auto-reset (the reference forks one gym AsyncVectorEnv
worker per env, wrappers.py:211-212); its outputs are torch tensors on the GPU.
With num_snakes == 1 it is wrapped in SingleAgentVec (the snake axis dropped, as
SingleAgent does inside each reference worker).
AsyncVectorMultiEnv (the process pool) is replaced by SnakeVecEnv. RenderGUI is
kept as a pass-through wrapper so callers that import or wrap with it run
unchanged; drawing an OpenCV window / video is out of scope (render() raises).
"""
import numpy as np

from . import spaces
from .envs import REGISTRY, UNSUPPORTED
from .vec_env import SnakeVecEnv


class Wrapper:
    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):
        if name.startswith('__'):
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return getattr(self.env, 'unwrapped', self.env)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)

    def step(self, action):
        return self.env.step(action)

    def close(self):
        return self.env.close()


class RenderGUI(Wrapper):                         # wrappers.py:20-82
    def __init__(self, env, window_name='Snake AI', save_video=False, video_path='output.mp4', fps=20):
        super().__init__(env)
        self.window_name, self.save_video, self.video_path, self.fps = window_name, save_video, video_path, fps

    def render(self, *args, **kwargs):
        raise NotImplementedError('RenderGUI windows/videos (OpenCV) are not part of the MI355X build; '
                                  'env.render() gives an ASCII grid')


class SingleAgent(Wrapper):                       # wrappers.py:84-105
    def __init__(self, env):
        super().__init__(env)
        assert env.num_snakes == 1, 'Number of player must be one'
        self.action_space = spaces.Discrete(len(self.env.action_dict))
        if getattr(self.env, 'vision_range', None):
            h = w = self.env.vision_range * 2 + 1
            shape = (h, w, self.env.obs_ch)
        else:
            shape = (*self.env.grid_shape, self.env.obs_ch)
        self.observation_space = spaces.Box(0, 255, shape, np.uint8)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)[0]

    def step(self, action, **kwargs):
        obs, rews, dones, infos = self.env.step([action], **kwargs)
        return obs[0], rews[0], dones[0], {}


class SingleAgentVec(Wrapper):
    """num_envs > 1 with one snake: the reference wraps every AsyncVectorEnv worker
    in SingleAgent (wrappers.py:84-105, 204-212), so the batch surface drops the
    snake axis -- obs (N, h, w, C), actions (N,), rewards (N,) float64, dones (N,)
    bool. A view of the SnakeVecEnv outputs (same tensors, no copy); info keeps
    SnakeVecEnv's tensors with the snake axis dropped."""

    def __init__(self, env):
        super().__init__(env)
        assert env.num_snakes == 1, 'Number of player must be one'
        N, shape = env.num_envs, tuple(env.obs_shape[1:])
        self.single_action_space = spaces.Discrete(env.action_n)
        self.single_observation_space = spaces.Box(0, 255, shape, np.uint8)
        self.observation_space = spaces.Box(0, 255, (N,) + shape, np.uint8)
        self.action_space = spaces.Box(0, env.action_n - 1, (N,), np.int64)

    def reset(self, **kwargs):
        return self.env.reset(**kwargs)[:, 0]

    def step(self, actions):
        obs, rew, done, info = self.env.step(actions)   # (N,) actions == (N, 1)
        info = {k: (v[:, 0] if v.dim() == 2 else v) for k, v in info.items()}
        return obs[:, 0], rew[:, 0], done[:, 0], info


class SingleMultiAgent(Wrapper):                  # wrappers.py:107-124
    def __init__(self, env):
        super().__init__(env)
        self.action_space = spaces.Discrete(len(self.env.action_dict))
        vision_range = getattr(self.env, 'vision_range', None)
        obs_ch = getattr(self.env, 'obs_ch', 3)
        if vision_range:
            h = w = vision_range * 2 + 1
            shape = (self.env.num_snakes, h, w, obs_ch)
        else:
            shape = (self.env.num_snakes, *self.env.grid_shape, obs_ch)
        self.observation_space = spaces.Box(0, 255, shape, np.uint8)


def make_snake(num_envs=1, num_snakes=4, env_id='Snake-v1', **kwargs):
    """wrappers.py:203-223. Returns (env, None, None, properties)."""
    if env_id in UNSUPPORTED:
        raise NotImplementedError(f'{env_id} is not provided by the MI355X build (see DESIGN.md)')
    if env_id not in REGISTRY:
        raise KeyError(f'unknown env id {env_id!r}')
    observer = kwargs.get('observer', 'snake')
    action_n = 5 if observer == 'human' else 3
    if num_envs > 1:
        env = SnakeVecEnv(num_envs, num_snakes=num_snakes, coop=(env_id == 'SnakeCoop-v1'), **kwargs)
        if num_snakes == 1:          # SingleAgent inside every vector worker (wrappers.py:204)
            env = SingleAgentVec(env)
    else:
        env_wrapper = SingleMultiAgent if num_snakes > 1 else SingleAgent
        env = env_wrapper(REGISTRY[env_id](num_snakes=num_snakes, **kwargs))
    properties = {
        'action_info': {'action_n': action_n},
        'num_envs': num_envs,
        'num_snakes': num_snakes,
    }
    return env, None, None, properties
