"""SnakeEnv keyword handling, shared by the compat env and the vector env.

Restates SnakeEnv.__init__'s argument semantics (snake_env.py:58-129):
reward_dict keys must equal the default keys (KeyError otherwise, :76-82),
max_episode_steps defaults to 1e4 (:56, :83-84), num_fruits to
int(round(0.8 * num_snakes)) (:87-88), unknown kwargs are accepted and ignored
(as the reference's **kwargs does, e.g. README's reward_func=).
"""
import math

from ._native import SnakeCfg

DEFAULT_REWARD_DICT = {'fruit': 10.0, 'kill': 0.0, 'lose': -0.5, 'win': 0.0, 'time': -0.001}
REWARD_KEYS = DEFAULT_REWARD_DICT.keys()
MAX_EPISODE_STEPS = 1e4

# action dicts (snake_env.py:32-44)
DEFAULT_ACTION_DICT = {'noop': 0, 'left': 1, 'right': 2, 'down': 3, 'up': 4}
ACTION_ANGLE_DICT = {0: 0.0, 1: math.pi / 2.0, 2: -math.pi / 2.0}


def autoreset_code(autoreset):
    """True -> 1 (reset when all dones are True, wrappers.py:141-143), False -> 0,
    'every_step' -> 2: gym 0.23.1's worker as make_snake's AsyncVectorEnv runs it
    (`if done: reset` on the list of dones, always truthy: a reset after every
    step)."""
    if autoreset == 'every_step':
        return 2
    if isinstance(autoreset, str):
        raise ValueError(f"autoreset must be True, False or 'every_step' (got {autoreset!r})")
    return 1 if autoreset else 0


def build_cfg(height=20, width=20, num_snakes=4, snake_length=3, vision_range=None,
              frame_stack=1, observer='snake', coop=False, autoreset=True, **kwargs):
    reward_dict = kwargs.pop('reward_dict', DEFAULT_REWARD_DICT)
    if reward_dict.keys() != REWARD_KEYS:
        raise KeyError(f'reward dict keys must correspond to {REWARD_KEYS}')
    max_episode_steps = kwargs.pop('max_episode_steps', MAX_EPISODE_STEPS)
    # spawn-ahead threshold of the GPU step (include/snake_env.h; 0 default, -1 off)
    spawn_ahead = int(kwargs.pop('spawn_ahead', 0))
    # spawn-ahead attempts in a background kernel (0 automatic, 1 on, -1 off)
    spawn_background = int(kwargs.pop('spawn_background', 0))
    num_fruits = kwargs.pop('num_fruits', int(round(num_snakes * 0.8)))
    if observer not in ('snake', 'human'):
        raise ValueError(f"observer must be 'snake' or 'human' (got {observer!r})")
    cfg = SnakeCfg(
        int(height), int(width), int(num_snakes), int(snake_length), int(vision_range or 0),
        int(frame_stack), 1 if observer == 'human' else 0, int(num_fruits),
        float(reward_dict['fruit']), float(reward_dict['kill']), float(reward_dict['lose']),
        float(reward_dict['win']), float(reward_dict['time']), float(max_episode_steps),
        1 if coop else 0, autoreset_code(autoreset), spawn_ahead, spawn_background)
    meta = dict(height=int(height), width=int(width), num_snakes=int(num_snakes),
                snake_length=int(snake_length), vision_range=vision_range,
                frame_stack=int(frame_stack), observer=observer, reward_dict=reward_dict,
                num_fruits=int(num_fruits), max_episode_steps=max_episode_steps, coop=bool(coop))
    return cfg, meta
