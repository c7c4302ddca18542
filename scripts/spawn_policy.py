#!/usr/bin/env python3
"""Offline study of spawn-ahead queuing policies on a recorded trace
(scripts/spawn_trace.py). CPU only.

Model of the protocol (snake_kernels.hip k_logic / do_spawn / do_reset): after
env.reset() every env holds a READY record (k_reset draws it). Per step and env,
after the transition: an episode end resets the env (READY record: hit, PARTIAL:
continues it, NONE: a whole attempt inline) and leaves it with no record; else a
draw from the MT state (fruit respawn) voids the record, and a queued env without
a READY record gets one permutation attempt, which yields disjoint poses with
probability p_ok (READY) or leaves a PARTIAL record to continue.

    python scripts/spawn_policy.py gpurun_out/trace_cfg3.npz
"""
import sys

import numpy as np

NONE, PARTIAL, READY = 0, 1, 2


def simulate(trace, policy, windows, p_ok=1 / 1.105, seed=1, tries=None):
    """tries(prod=..., am=...) -> attempts per job (default 1)"""
    T, N = trace.shape
    rng = np.random.default_rng(seed)
    status = np.full(N, READY, np.int8)
    eplen = np.zeros(N, np.int32)
    since_void = np.full(N, 1 << 20, np.int32)
    voids_ep = np.zeros(N, np.int32)
    acc = {w: dict(jobs=0, resets=0, hits=0, part=0, voids=0, steps=0) for w in windows}
    for t in range(T):
        f = trace[t].astype(np.int32)
        am = f & 7
        drew = ((f >> 3) & 1).astype(bool)
        mind = (f >> 4) & 15
        prod = (f >> 8) & 127
        end = am == 0
        eplen += 1
        hit = end & (status == READY)
        part = end & (status == PARTIAL)
        void = ~end & drew & (status == READY)
        status[end] = NONE
        status[~end & drew] = NONE
        since_void[void] = 0
        since_void[~void] += 1
        voids_ep[void] += 1
        q = ~end & (status != READY) & policy(am=am, mind=mind, prod=prod, eplen=eplen, since_void=since_void,
                                              voids_ep=voids_ep, drew=drew)
        nt = tries(am=am, prod=prod) if tries is not None else 1
        ok = rng.random(N) < 1 - (1 - p_ok) ** nt
        status[q & ok] = READY
        status[q & ~ok] = PARTIAL
        for (a, b), s in acc.items():
            if a <= t < b:
                s['att'] = s.get('att', 0) + float((q * (1 + (nt > 1) * (1 - p_ok))).sum())
                s['jobs'] += int(q.sum()); s['resets'] += int(end.sum()); s['hits'] += int(hit.sum())
                s['part'] += int(part.sum()); s['voids'] += int(void.sum()); s['steps'] += 1
        eplen[end] = 0
        voids_ep[end] = 0
        since_void[end] = 1 << 20
    out = {}
    for w, s in acc.items():
        n = max(s['steps'], 1)
        out[w] = dict(jobs=s['jobs'] / n, resets=s['resets'] / n, voids=s['voids'] / n,
                      hit=s['hits'] / max(s['resets'], 1), miss=(s['resets'] - s['hits'] - s['part']) / n,
                      jps=s['jobs'] / max(s['hits'], 1), att=s.get('att', 0) / n)
    return out


def thr(k):
    return lambda am, **_: am <= k


POLICIES = {
    'thr3 (current)': thr(3),
    'thr2': thr(2),
    'thr1': thr(1),
}


def main():
    d = np.load(sys.argv[1])
    trace = d['trace']
    T = trace.shape[0]
    windows = [(5, 25), (200, T)]
    for name, pol in POLICIES.items():
        r = simulate(trace, pol, windows)
        print(f'{name:40s}', '  '.join(
            f"[{a}-{b}) jobs {v['jobs']:7.1f} resets {v['resets']:6.1f} voids {v['voids']:6.1f} "
            f"hit {v['hit']:.4f} miss {v['miss']:5.2f} jps {v['jps']:.3f}" for (a, b), v in r.items()))


if __name__ == '__main__':
    main()
