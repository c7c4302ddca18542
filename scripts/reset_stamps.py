#!/usr/bin/env python3
"""Phase breakdown of one env reset (diagnostic build with -DSNAKE_STAMPS):
s_memtime stamps of env 0's wave around the permutation draws, the trace, the
fruit draws and the encode, alone on the GPU and inside a full-batch reset."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402

path = os.path.abspath(sys.argv[1])
L = _native.lib(path)
L.snake_debug_stamps.argtypes = [ctypes.c_void_p]
names = {0: 'start', 20: 'paint_done', 21: 'fruits_done', 22: 'stored', 23: 'encoded'}
for a in range(4):
    names[1 + 3 * a] = f'a{a}_begin'
    names[2 + 3 * a] = f'a{a}_drawn'
    names[3 + 3 * a] = f'a{a}_traced'


def run(v, mask):
    buf = np.zeros(72, np.uint64)
    L.snake_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p))   # clear counters
    v.reset(mask)
    torch.cuda.synchronize()
    buf[:] = 0
    L.snake_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p))
    st = {names[i]: int(buf[i]) for i in sorted(names) if buf[i]}
    t0 = st['start']
    return {'cycles': {k: x - t0 for k, x in st.items()}, 'twists': int(buf[64]), 'rounds': int(buf[65]),
            'twist_cycles': int(buf[66]), 'refine_iters': int(buf[67]), 'round_cycles': {
                'select': int(buf[71]), 'setup': int(buf[68]), 'refine': int(buf[69]), 'epilogue': int(buf[70])}}


for N in (1, 65536):
    v = SnakeVecEnv(N, num_snakes=4, seed=0, lib_path=path, height=20, width=20, vision_range=5)
    v.reset()
    for rep in range(3):
        m = torch.zeros(N, dtype=torch.bool, device='cuda')
        m[0] = True
        print(json.dumps({'N': N, 'mask': 'env0', **run(v, m)}))
    print(json.dumps({'N': N, 'mask': 'all', **run(v, None)}))
