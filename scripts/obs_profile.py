#!/usr/bin/env python3
"""Timeline of one step's observation phase (diagnostic SNAKE_STAMPS build): s_memrealtime
(100 MHz) at start/end of the first 128 queued resets, of the first 128
spawn-ahead jobs and of every 512th env's encode block, relative to the
earliest recorded start.

    python scripts/obs_profile.py marl-snake_amd/build/libsnake_stamps.so
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlenv import SnakeVecEnv  # noqa: E402


CFGS = {'cfg3': (65536, 4, dict(height=20, width=20, snake_length=3, vision_range=5)),
        'cfg2': (4096, 4, dict(height=20, width=20, snake_length=3)),
        'cfg5': (8192, 8, dict(height=40, width=40, snake_length=3, vision_range=5, frame_stack=4))}


def spans(r):
    """kernel spans, us from k_logic's first wave: r = obsprof words 1400.. (starts
    stored complemented by the max-atomics, ends plain; 0 = not recorded)"""
    M = (1 << 64) - 1
    t0 = M - r[0] if r[0] else None
    out = {}
    for n, i, inv in (('logic_end', 1, 0), ('autoreset_start', 6, 1), ('autoreset_end', 2, 0),
                      ('encode_start', 4, 1), ('encode_end', 3, 0), ('spawn_end', 5, 0)):
        v = r[i]
        if not v or t0 is None:
            out[n] = None
            continue
        out[n] = round(((M - v) if inv else v) - t0) / 100.0
    return out


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('lib')
    ap.add_argument('--cfg', default='cfg3', choices=sorted(CFGS))
    a = ap.parse_args()
    lib = os.path.abspath(a.lib)
    N, S, kw = CFGS[a.cfg]
    v = SnakeVecEnv(N, num_snakes=S, seed=0, lib_path=lib, **kw)
    L = ctypes.CDLL(lib)
    L.snake_debug_obsprof.argtypes = [ctypes.c_void_p]
    L.snake_debug_stamps.argtypes = [ctypes.c_void_p]
    st = np.zeros(72, dtype=np.uint64)
    buf = np.zeros(1408, dtype=np.uint64)
    g = torch.Generator(device='cuda').manual_seed(7)
    acts = torch.randint(0, 3, (300, N, S), generator=g, device='cuda', dtype=torch.int8)
    v.reset()
    for t in range(250):
        v.step(acts[t])
    torch.cuda.synchronize()
    for t in range(250, 256):
        L.snake_debug_obsprof(buf.ctypes.data_as(ctypes.c_void_p))
        _, _, done, info = v.step(acts[t])
        torch.cuda.synchronize()
        nres = int(info['episode_done'].sum())
        L.snake_debug_stamps(st.ctypes.data_as(ctypes.c_void_p))
        ls = st[40:50].astype(np.int64)
        logic = {n: int(x - ls[0]) for n, x in zip(('start', 'loaded', 'rules', 'grid', 'dying', 'fruit', 'stats', 'end',
                                                    'outputs', 'queued'), ls)}
        L.snake_debug_obsprof(buf.ctypes.data_as(ctypes.c_void_p))
        b = buf.astype(np.int64)
        rs, re_, es, ee = b[:128], b[128:256], b[256:384], b[384:512]
        ss, se = b[512:640], b[640:768]
        ph = b[768:768 + 5 * 128].reshape(128, 5)[:min(nres, 128)]
        sok = (ss > 0) & (se > 0)
        nr = min(nres, 128)
        rs, re_ = rs[:nr], re_[:nr]
        ok = ee > 0
        t0 = min(rs.min() if nr else 1 << 62, es[es > 0].min())
        us = lambda x: (x - t0) / 100.0   # noqa: E731
        pct = lambda x: [round(float(np.percentile(x, p)), 1) for p in (0, 50, 90, 100)]  # noqa: E731
        print(json.dumps({
            'resets': nres, 'k_logic_block0_cycles': logic,
            'reset_start_us': pct(us(rs)) if nr else None,
            'reset_dur_us': pct((re_ - rs) / 100.0) if nr else None,
            'reset_end_us': pct(us(re_)) if nr else None,
            'encode_start_us': pct(us(es[es > 0])),
            'encode_end_us': pct(us(ee[ok])),
            'encode_dur_us': pct((ee[ok] - es[ok]) / 100.0),
            'spawn_start_us': pct(us(ss[sok])) if sok.any() else None,
            'spawn_end_us': pct(us(se[sok])) if sok.any() else None,
            'spawn_dur_us': pct((se[sok] - ss[sok]) / 100.0) if sok.any() else None,
            # per reset: status at start (0 none, 1 partial, 2 ready, 3 in progress) and the
            # phase durations: poses, paint, fruits, grid/key stores, encode
            # kernel spans (us from k_logic block 0's start): k_logic end, k_autoreset end,
            # lean encode start (block 0) / end, k_spawn end
            'spans_us': spans([int(x) for x in buf[1400:1408]]),
            'spans_raw': [int(x) for x in buf[1400:1408]],
            'reset_phases_us': [[int(p[4]) & 3] + [round(float(x), 1) for x in np.diff(
                np.array([r, p[0], p[1], p[2], p[3], en], dtype=np.int64)) / 100.0]
                for r, p, en in zip(rs, ph, re_)][:12],
        }), flush=True)


if __name__ == '__main__':
    main()
