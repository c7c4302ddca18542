#!/usr/bin/env python3
"""k_logic timeline (diagnostic build with -DSNAKE_STAMPS: scripts/build_variants.sh
stamps:-DSNAKE_STAMPS).

Per step, after --skip warm-up steps: block 0's phase stamps (s_memtime, LSTAMP
40..52, cycles from its start) and every wave's start/end (s_memrealtime, 100
MHz): the kernel's span, the spread of wave starts (dispatch), wave durations.
Medians over the steps.

    python scripts/logic_stamps.py marl-snake_amd/build/var/libsnake_stamps.so [--cfg cfg3] [--steps 100]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402

NAMES = {40: 'start', 51: 'grid_staged', 52: 'stats_loaded', 41: 'rules', 42: 'second_round_issued',
         43: 'grid_update', 44: 'dying_walk', 45: 'respawn', 48: 'outputs', 49: 'stats', 46: 'queues',
         47: 'records_stored'}
CFGS = {'cfg3': (65536, 4, dict(height=20, width=20, vision_range=5)),
        'cfg4': (32768, 4, dict(height=20, width=20, vision_range=5)),
        'cfg2': (4096, 4, dict(height=20, width=20)),
        'cfg5': (8192, 8, dict(height=40, width=40, vision_range=5, frame_stack=4))}
KWT = 8192
KPT = 40960


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('lib')
    ap.add_argument('--cfg', default='cfg3')
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--skip', type=int, default=200)
    a = ap.parse_args()
    L = _native.lib(os.path.abspath(a.lib))
    L.snake_debug_stamps.argtypes = [ctypes.c_void_p]
    N, S, kw = CFGS[a.cfg]
    v = SnakeVecEnv(N, num_snakes=S, seed=0, lib_path=os.path.abspath(a.lib), **kw)
    v.reset()
    g = torch.Generator(device='cuda').manual_seed(7)
    acts = torch.randint(0, 3, (a.skip + a.steps, N, S), generator=g, device='cuda', dtype=torch.int8)
    buf = np.zeros(64 + 2 * KWT + 2 * KPT, np.uint64)
    posts = []
    nblk = (N + 64 // v.cfg.num_snakes - 1)   # upper bound; the used blocks have nonzero stamps
    rows, waves = [], []
    for t in range(a.skip + a.steps):
        v.step(acts[t])
        torch.cuda.synchronize()
        if t < a.skip:
            continue
        L.snake_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p))
        t0 = int(buf[40])
        rows.append({n: int(buf[i]) - t0 for i, n in NAMES.items() if buf[i]})
        # k_post: worker blocks [0, reset_slots), then the encode blocks; times
        # relative to the first k_post block's start
        pt = buf[64 + 2 * KWT:].reshape(KPT, 2).astype(np.int64)
        G = min(N, 2048)
        pu = pt[:, 0] > 0
        if pu.any():
            p0 = pt[pu, 0].min()
            wk, en_ = pt[:G][pu[:G]], pt[G:][pu[G:]]
            posts.append(dict(span_ns=int((pt[pu, 1].max() - p0) * 10),
                              workers_end_p50_ns=int((np.median(wk[:, 1]) - p0) * 10),
                              workers_end_p90_ns=int((np.percentile(wk[:, 1], 90) - p0) * 10),
                              workers_end_max_ns=int((wk[:, 1].max() - p0) * 10),
                              enc_start_p50_ns=int((np.median(en_[:, 0]) - p0) * 10) if len(en_) else -1,
                              enc_start_max_ns=int((en_[:, 0].max() - p0) * 10) if len(en_) else -1,
                              enc_end_p50_ns=int((np.median(en_[:, 1]) - p0) * 10) if len(en_) else -1,
                              enc_end_p99_ns=int((np.percentile(en_[:, 1], 99) - p0) * 10) if len(en_) else -1,
                              enc_end_max_ns=int((en_[:, 1].max() - p0) * 10) if len(en_) else -1,
                              enc_blocks_timed=int(len(en_))))
        wt = buf[64:64 + 2 * KWT].reshape(KWT, 2).astype(np.int64)
        used = wt[:, 0] > 0
        wt = wt[used]
        s0 = wt[:, 0].min()
        st, en = (wt[:, 0] - s0) * 10, (wt[:, 1] - s0) * 10   # ns
        dur = en - st
        waves.append(dict(span_ns=int(en.max()), start_p50_ns=int(np.median(st)), start_p90_ns=int(np.percentile(st, 90)),
                          start_max_ns=int(st.max()), dur_p10_ns=int(np.percentile(dur, 10)),
                          dur_p50_ns=int(np.median(dur)), dur_p90_ns=int(np.percentile(dur, 90)),
                          dur_max_ns=int(dur.max()), end_p50_ns=int(np.median(en)), waves=int(used.sum())))
        buf[:] = 0
        L.snake_debug_stamps  # (stamps are overwritten every step)
    med = {n: statistics.median(r[n] for r in rows if n in r) for n in NAMES.values() if any(n in r for r in rows)}
    order = sorted(med, key=med.get)
    wmed = {k: statistics.median(w[k] for w in waves) for k in waves[0]}
    pmed = {k: statistics.median(w[k] for w in posts) for k in posts[0]} if posts else None
    print(json.dumps({'cfg': a.cfg, 'steps': len(rows), 'block0_cycles_from_start': {n: med[n] for n in order},
                      'waves_median_over_steps': wmed, 'k_post_median_over_steps': pmed}))


if __name__ == '__main__':
    main()
