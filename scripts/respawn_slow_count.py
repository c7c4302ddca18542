import sys, os, json
sys.path[:0] = ['/root/repo/marl-snake_amd', '/root/repo']
import torch
from marlenv import SnakeVecEnv, _native
for cfg, (N, S, kw) in {'cfg3': (65536, 4, dict(height=20, width=20, vision_range=5)), 'cfg5': (8192, 8, dict(height=40, width=40, vision_range=5, frame_stack=4))}.items():
    v = SnakeVecEnv(N, num_snakes=S, seed=0, **kw); v.reset()
    g = torch.Generator(device='cuda').manual_seed(12345)
    for t in range(300):
        a = torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8)
        if t == 200:
            for k in ('resets', 'respawn_slow', 'respawn_slow2'): _native.timing_read(k)
            _native.timing_enable(True)
        v.step(a)
    _native.timing_enable(False); torch.cuda.synchronize()
    print(cfg, {k: _native.timing_read(k)[1] / 100 for k in ('resets_timed', 'respawn_slow', 'respawn_slow2')}, 'waves', N * S // 64)
