"""Offline stand-in for the `gym` package, used ONLY by make_golden.py.

gym (pinned gym==0.24.1 in the reference's requirements.txt:1) is not
installed in this image. SnakeEnv (reference marlenv/envs/snake_env.py) only
touches gym.Env (base class), gym.spaces.Discrete/Box (shape bookkeeping),
gym.utils.seeding.np_random (the unused self.np_random) and
gym.envs.registration.register. None of these is on the step/reset
arithmetic, so this stub does not change any number the fixtures record.
"""
from . import spaces, utils  # noqa: F401


class Env:
    pass


class Wrapper(Env):
    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):
        return getattr(self.env, name)
