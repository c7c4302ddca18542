#!/usr/bin/env python3
"""Timeline of the fused step (k_step) by block role (diagnostic build with
-DSNAKE_STAMPS: scripts/build_variants.sh stamps:-DSNAKE_STAMPS): every block's
start and end (s_memrealtime, 10 ns ticks) of the last launch, per role --
rules (logic groups), reset workers, encodes -- as percentiles from the first
block's start, over --steps steps after --skip.

    SNAKE_LIB=marl-snake_amd/build/var/libsnake_stamps.so python scripts/step_roles.py --cfg cfg3
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402

CFGS = {'cfg3': (65536, 4, dict(height=20, width=20, vision_range=5)),
        'cfg4': (32768, 4, dict(height=20, width=20, vision_range=5)),
        'cfg3s8': (8192, 4, dict(height=20, width=20, vision_range=5, spawn_background=-1))}
KWT, KPT = 8192, 40960


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cfg', default='cfg3')
    ap.add_argument('--skip', type=int, default=200)
    ap.add_argument('--steps', type=int, default=10)
    a = ap.parse_args()
    N, S, kw = CFGS[a.cfg]
    L = _native.lib()
    L.snake_debug_stamps.argtypes = [ctypes.c_void_p]
    v = SnakeVecEnv(N, num_snakes=S, seed=0, **kw)
    v.reset()
    E = 64 // (4 if N > 8192 else 8)
    nlg, G = (N + E - 1) // E, min(N, 2048)
    nb = nlg + G + (N + 3) // 4
    g = torch.Generator(device='cuda').manual_seed(12345)
    buf = np.zeros(64 + 2 * KWT + 2 * KPT, np.uint64)
    res = {k: [] for k in ('span', 'rules_end_p50', 'rules_end_max', 'worker_start_p50', 'worker_end_p50',
                           'worker_end_max', 'enc_start_p10', 'enc_start_p50', 'enc_start_max', 'enc_end_max',
                           'enc_dur_p50')}
    for t in range(a.skip + a.steps):
        v.step(torch.randint(0, 3, (N, S), generator=g, device='cuda', dtype=torch.int8))
        if t < a.skip:
            continue
        torch.cuda.synchronize()
        L.snake_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p))
        pt = buf[64 + 2 * KWT:].reshape(KPT, 2)[:nb].astype(np.int64)
        t0 = pt[:, 0].min()
        st, en = (pt[:, 0] - t0) * 10, (pt[:, 1] - t0) * 10   # ns
        r, w, e = slice(0, nlg), slice(nlg, nlg + G), slice(nlg + G, nb)
        res['span'].append(int(en.max()))
        res['rules_end_p50'].append(int(np.median(en[r]))); res['rules_end_max'].append(int(en[r].max()))
        res['worker_start_p50'].append(int(np.median(st[w]))); res['worker_end_p50'].append(int(np.median(en[w])))
        res['worker_end_max'].append(int(en[w].max()))
        res['enc_start_p10'].append(int(np.percentile(st[e], 10))); res['enc_start_p50'].append(int(np.median(st[e])))
        res['enc_start_max'].append(int(st[e].max())); res['enc_end_max'].append(int(en[e].max()))
        res['enc_dur_p50'].append(int(np.median(en[e] - st[e])))
    print(json.dumps({'cfg': a.cfg, 'N': N, 'blocks': nb, 'ns_median_over_steps': {k: int(np.median(x)) for k, x in res.items()}}))


if __name__ == '__main__':
    main()
