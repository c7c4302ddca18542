"""marlenv (MI355X build): the batched multi-snake grid environment of
tranthai189765/MARL-Snake, stepped by hand-written HIP kernels on CDNA4.

    from marlenv.wrappers import make_snake
    env, _, _, props = make_snake(num_envs=1, num_snakes=4)        # reference API
    venv, _, _, _ = make_snake(num_envs=65536, num_snakes=4, vision_range=5)  # GPU batch
"""
from .envs import CoopSnakeEnv, SnakeEnv  # noqa: F401
from .vec_env import SnakeVecEnv  # noqa: F401
from .dqn import DQNForward  # noqa: F401
from .wrappers import RenderGUI, SingleAgent, SingleAgentVec, SingleMultiAgent, make_snake  # noqa: F401

__version__ = '0.1.0'


def _alias_nested_path():
    """The reference's callers import `marlenv.marlenv.wrappers` (train_dqn.py:22,
    train_ga.py:25, test_env.py:1: a distribution dir around the package). With
    this package's parent on sys.path, map that nested path onto this package."""
    import importlib
    import sys
    me = sys.modules[__name__]
    sys.modules.setdefault(__name__ + '.marlenv', me)
    for sub in ('wrappers', 'envs', 'envs.snake_env', 'envs.coop_snake_env', 'envs.constants',
                'core', 'core.snake', 'vec_env', 'spaces', 'config'):
        sys.modules.setdefault(f'{__name__}.marlenv.{sub}', importlib.import_module(f'{__name__}.{sub}'))


_alias_nested_path()
