"""Env ids (reference marlenv/marlenv/envs/__init__.py:3-16)."""
from .coop_snake_env import CoopSnakeEnv
from .snake_env import SnakeEnv

REGISTRY = {
    'Snake-v1': SnakeEnv,
    'SnakeCoop-v1': CoopSnakeEnv,
}
# 'SnakeGraph-v1' (graph_snake_env.py: ray-cast feature obs) is out of scope.
UNSUPPORTED = {'SnakeGraph-v1'}


def make(env_id, **kwargs):
    if env_id in UNSUPPORTED:
        raise NotImplementedError(f'{env_id} is not provided by the MI355X build (see DESIGN.md)')
    if env_id not in REGISTRY:
        raise KeyError(f'unknown env id {env_id!r}')
    return REGISTRY[env_id](**kwargs)
