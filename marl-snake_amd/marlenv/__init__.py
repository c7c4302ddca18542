"""marlenv (MI355X build): the batched multi-snake grid environment of
tranthai189765/MARL-Snake, stepped by hand-written HIP kernels on CDNA4.

    from marlenv.wrappers import make_snake
    env, _, _, props = make_snake(num_envs=1, num_snakes=4)        # reference API
    venv, _, _, _ = make_snake(num_envs=65536, num_snakes=4, vision_range=5)  # GPU batch
"""
from .envs import CoopSnakeEnv, SnakeEnv  # noqa: F401
from .vec_env import SnakeVecEnv  # noqa: F401
from .wrappers import SingleAgent, SingleMultiAgent, make_snake  # noqa: F401

__version__ = '0.1.0'
