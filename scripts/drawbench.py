#!/usr/bin/env python3
"""Isolated permutation-draw latency (diagnostic SNAKE_STAMPS build): one wave
runs one env's permutation(n_cand) draws alone; cycles per call and rounds."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]
import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402

path = os.path.abspath(sys.argv[1])
L = _native.lib(path)
L.snake_debug_drawbench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
hw = int(sys.argv[2]) if len(sys.argv) > 2 else 20   # board size (40: cfg5's 16 424 poses)
v = SnakeVecEnv(64, num_snakes=4, seed=0, lib_path=path, height=hw, width=hw, vision_range=5)
v.reset()
out = torch.zeros(4, dtype=torch.int64, device='cuda')
res, tr = [], []
for e in range(16):
    mt = v.mt.view(64, 624)[e]
    for rep in range(3):
        L.snake_debug_drawbench(mt.data_ptr(), 624, v.layout.n_cand, 4, out.data_ptr())
        res.append(int(out[0]))
        tr.append(int(out[2]))
print(json.dumps({'lib': os.path.basename(path), 'n_cand': v.layout.n_cand, 'cycles_min': min(res), 'cycles_median': sorted(res)[len(res) // 2],
                  'trace_cycles_median': sorted(tr)[len(tr) // 2]}))
