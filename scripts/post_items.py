#!/usr/bin/env python3
"""What sets k_post's end: every reset-worker item (diagnostic build with
-DSNAKE_STAMPS: scripts/build_variants.sh stamps:-DSNAKE_STAMPS) and every
k_post block's start/end, per step after --skip steps.

Item types: 0 reset from a ready record, 1 reset continuing a partial record,
2 reset without a record (a whole attempt inline), 3 queue-1 spawn-ahead job,
4 queue-2 job. Per step: the span (first block start -> last block end), the
encodes' last end, and which item type ends last; per type: items per step,
duration and end percentiles (ns), over the steps.

    python scripts/post_items.py marl-snake_amd/build/var/libsnake_stamps.so --cfg cfg3 [--spawn-ahead 3]
"""
import argparse
import ctypes
import json
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402

CFGS = {'cfg3': (65536, 4, dict(height=20, width=20, vision_range=5)),
        'cfg4': (32768, 4, dict(height=20, width=20, vision_range=5)),
        'cfg2': (4096, 4, dict(height=20, width=20)),
        'cfg3s8': (8192, 4, dict(height=20, width=20, vision_range=5)),
        'cfg5': (8192, 8, dict(height=40, width=40, vision_range=5, frame_stack=4))}
KWT, KPT, KIT = 8192, 40960, 16384
TYPES = ('reset_ready', 'reset_partial', 'reset_none', 'job_q1', 'job_q2')


def pct(x, q):
    return int(np.percentile(x, q)) if len(x) else -1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('lib')
    ap.add_argument('--cfg', default='cfg3')
    ap.add_argument('--steps', type=int, default=100)
    ap.add_argument('--skip', type=int, default=200)
    ap.add_argument('--spawn-ahead', type=int, default=0)
    a = ap.parse_args()
    lib = os.path.abspath(a.lib)
    L = _native.lib(lib)
    L.snake_debug_stamps.argtypes = [ctypes.c_void_p]
    L.snake_debug_items.argtypes = [ctypes.c_void_p, ctypes.c_int]
    N, S, kw = CFGS[a.cfg]
    v = SnakeVecEnv(N, num_snakes=S, seed=0, lib_path=lib, spawn_ahead=a.spawn_ahead, **kw)
    v.reset()
    g = torch.Generator(device='cuda').manual_seed(12345)
    acts = torch.randint(0, 3, (a.skip + a.steps, N, S), generator=g, device='cuda', dtype=torch.int8)
    buf = np.zeros(64 + 2 * KWT + 2 * KPT, np.uint64)
    items = np.zeros(4 * KIT, np.uint64)
    G = v._kcfg_reset_slots() if hasattr(v, '_kcfg_reset_slots') else min(N, 512 if N <= 8192 else 2048)
    G = G // (4 if a.cfg == 'cfg5' else 1)   # worker blocks (k_post_lean: four workers each)
    spans, enc_ends, crit, encs, gaps, lspan = [], [], Counter(), [], [], []
    per = {t: dict(n=[], dur=[], end=[]) for t in range(5)}
    chains = Counter()
    for t in range(a.skip + a.steps):
        v.step(acts[t])
        torch.cuda.synchronize()
        n = L.snake_debug_items(items.ctypes.data_as(ctypes.c_void_p), KIT)
        L.snake_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p))
        if t < a.skip:
            continue
        pt = buf[64 + 2 * KWT:].reshape(KPT, 2).astype(np.int64)
        pu = pt[:, 0] > 0
        p0 = pt[pu, 0].min()
        span = (pt[pu, 1].max() - p0) * 10
        enc = pt[G:][pu[G:]]
        enc_end = (enc[:, 1].max() - p0) * 10 if len(enc) else 0
        it = items[:4 * n].reshape(n, 4).astype(np.int64)
        typ = it[:, 0] >> 32
        st, en = (it[:, 1] - p0) * 10, (it[:, 2] - p0) * 10
        if len(enc):
            ed = (enc[:, 1] - enc[:, 0]) * 10
            es = (enc[:, 0] - p0) * 10
            ee = (enc[:, 1] - p0) * 10
            # encode blocks running at 25 / 50 / 75 % of the span
            conc = [int(((es <= f * span) & (ee > f * span)).sum()) for f in (0.25, 0.5, 0.75)]
            wk = pt[:G][pu[:G]]
            wconc = [int((((wk[:, 0] - p0) * 10 <= f * span) & ((wk[:, 1] - p0) * 10 > f * span)).sum())
                     for f in (0.25, 0.5, 0.75)]
            encs.append(dict(dur_p10=pct(ed, 10), dur_p50=pct(ed, 50), dur_p90=pct(ed, 90), dur_max=int(ed.max()),
                             start_p10=pct(es, 10), start_p50=pct(es, 50), start_p90=pct(es, 90),
                             start_max=int(es.max()), conc25=conc[0], conc50=conc[1], conc75=conc[2],
                             wconc25=wconc[0], wconc50=wconc[1], wconc75=wconc[2]))
        wt = buf[64:64 + 2 * KWT].reshape(KWT, 2).astype(np.int64)
        wu = wt[:, 0] > 0
        if wu.any():
            gaps.append(int((p0 - wt[wu, 1].max()) * 10))     # last k_logic wave end -> first k_post block start
            lspan.append(int((wt[wu, 1].max() - wt[wu, 0].min()) * 10))
        spans.append(int(span))
        enc_ends.append(int(enc_end))
        last_item = int(np.argmax(en)) if n else -1
        crit['encode' if n == 0 or enc_end >= en[last_item] else TYPES[typ[last_item]]] += 1
        for k in range(5):
            m = typ == k
            per[k]['n'].append(int(m.sum()))
            per[k]['dur'] += list((en - st)[m])
            per[k]['end'] += list(en[m])
        wk = it[:, 0] & 0xffffffff
        for w, c in Counter(wk.tolist()).items():
            chains[c] += 1
        buf[:] = 0
    out = dict(cfg=a.cfg, steps=a.steps, skip=a.skip, spawn_ahead=a.spawn_ahead,
               span_ns=dict(p50=pct(spans, 50), p90=pct(spans, 90), max=int(max(spans))),
               k_logic_span_ns=dict(p50=pct(lspan, 50), p90=pct(lspan, 90)),
               logic_end_to_post_start_ns=dict(p10=pct(gaps, 10), p50=pct(gaps, 50), p90=pct(gaps, 90)),
               enc_end_ns=dict(p50=pct(enc_ends, 50), p90=pct(enc_ends, 90)),
               last_to_end=dict(crit),
               encode_blocks={k: int(np.median([x[k] for x in encs])) for k in encs[0]} if encs else None,
               items_per_worker=dict(sorted((int(k), v / a.steps) for k, v in chains.items())),
               types={TYPES[k]: dict(per_step=float(np.mean(p['n'])), dur_p50=pct(p['dur'], 50),
                                     dur_p90=pct(p['dur'], 90), dur_max=int(max(p['dur'])) if p['dur'] else -1,
                                     end_p50=pct(p['end'], 50), end_p90=pct(p['end'], 90),
                                     end_max=int(max(p['end'])) if p['end'] else -1)
                      for k, p in per.items()})
    print(json.dumps(out))


if __name__ == '__main__':
    main()
