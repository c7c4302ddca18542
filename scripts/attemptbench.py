#!/usr/bin/env python3
"""Lone permutation-attempt latency, one wave vs the cooperative four-wave
draws (diagnostic build with -DSNAKE_DRAWBENCH: scripts/build_variants.sh
dbench:-DSNAKE_DRAWBENCH). For 20x20 and 40x40 boards (L = 3) and every record
kind (JL 1 u16 record, 2 u32 link table in LDS, 0 u32 link table in global
memory): the same MT states through both forms, their final stream positions
and arr[0..S) compared (they must be identical), s_memtime cycles of the draws
(incl. the record clear) and of the trace, medians over the states.

    python scripts/attemptbench.py marl-snake_amd/build/var/libsnake_dbench.so
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'marl-snake_amd'), ROOT]
import torch  # noqa: E402

from marlenv import SnakeVecEnv, _native  # noqa: E402


def main():
    path = os.path.abspath(sys.argv[1])
    L = _native.lib(path)
    P = ctypes.c_void_p
    L.snake_debug_attemptbench.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           P, P]
    S, n_states = 4, int(sys.argv[2]) if len(sys.argv) > 2 else 24
    res = {}
    for hw in (20, 40):
        v = SnakeVecEnv(n_states, num_snakes=S, seed=0, lib_path=path, height=hw, width=hw, vision_range=5)
        v.reset()
        n = v.layout.n_cand
        gl = torch.zeros(n + 128, dtype=torch.int32, device='cuda')
        out = torch.zeros(8, dtype=torch.int64, device='cuda')
        keys, pos = v.mt_state()
        for jl in (1, 2, 0):
            rows = {0: [], 1: []}
            for e in range(n_states):
                got = {}
                for coop in (0, 1):
                    for rep in range(2):
                        rc = L.snake_debug_attemptbench(keys[e].data_ptr(), int(pos[e]), n, S, coop, jl,
                                                        gl.data_ptr(), out.data_ptr())
                        assert rc == 0, 'launch failed'
                        o = out.cpu().tolist()
                        if rep:
                            rows[coop].append((o[0], o[1]))
                        got[coop] = (o[2], o[3:3 + S])
                assert got[0] == got[1], (hw, jl, e, got)
            med = {c: (statistics.median(r[0] for r in rows[c]), statistics.median(r[1] for r in rows[c]))
                   for c in (0, 1)}
            res[f'{hw}x{hw}_jl{jl}'] = dict(
                n_cand=n, states=n_states, identical=True,
                one_wave_draw_cycles=med[0][0], one_wave_trace_cycles=med[0][1],
                coop_draw_cycles=med[1][0], coop_trace_cycles=med[1][1],
                attempt_ratio=round((med[1][0] + med[1][1]) / (med[0][0] + med[0][1]), 3))
            print(json.dumps({f'{hw}x{hw}_jl{jl}': res[f'{hw}x{hw}_jl{jl}']}), flush=True)
        del v
    print(json.dumps(res))


if __name__ == '__main__':
    main()
