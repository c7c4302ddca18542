"""CoopSnakeEnv (reference marlenv/marlenv/envs/coop_snake_env.py:4-22): the
episode ends when ANY snake is done and then every done is True."""
from .snake_env import SnakeEnv


class CoopSnakeEnv(SnakeEnv):
    _coop = True

    def _done_fn(self, dones):
        return any(dones)
