"""Helpers to read the committed golden fixtures (tests/golden/*.npz, crafted.json)."""
import base64
import glob
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def digest(arr):
    """Same 8-byte blake2b digest as tests/golden/gen/make_golden.py:digest."""
    a = np.ascontiguousarray(arr)
    return int.from_bytes(hashlib.blake2b(a.tobytes(), digest_size=8).digest(), 'little')


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def traj_names():
    return sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLDEN, 'traj_*.npz')))


def load_traj(name):
    z = load(f'traj_{name}.npz')
    d = {k: z[k] for k in z.files}
    d['config'] = json.loads(str(d['config']))
    d['seed'] = int(d['seed'])
    return d


def load_crafted():
    with open(os.path.join(GOLDEN, 'crafted.json')) as fp:
        cases = json.load(fp)
    for c in cases:
        for st in c['steps']:
            st['obs'] = np.frombuffer(base64.b64decode(st['obs_b64']), np.uint8).reshape(st['obs_shape'])
    return cases


def env_kwargs(cfg):
    """Fixture config -> SnakeEnv/make_snake keyword arguments."""
    return dict(height=cfg['height'], width=cfg['width'], num_snakes=cfg['num_snakes'],
                snake_length=cfg['snake_length'], vision_range=cfg['vision_range'],
                frame_stack=cfg['frame_stack'], observer=cfg['observer'],
                reward_dict=cfg['reward_dict'], num_fruits=cfg['num_fruits'],
                max_episode_steps=cfg['max_episode_steps'], **({'coop': True} if cfg.get('coop') else {}))
