#!/usr/bin/env python3
"""Render fixtures from the REAL reference rgb_from_grid (container only).

    python3 -B tests/golden/gen/make_render_golden.py

Imports marlenv.core.grid_util.rgb_from_grid / core.snake.{Cell, CellColors}
from /root/reference/marlenv through the offline gym stub and writes
tests/golden/render.npz (inputs + outputs only):

* palette  uint8 (6, 16, 3): rgb_from_grid of a 1x1 grid holding 10*i + code,
           for every code 0..5 and owner i 0..15 (codes 0..2 only occur
           with owner 0 in a grid; the table holds what the function returns);
* grids    uint8 (G, 20, 20): the first grids of two committed trajectories
           (S=4) plus crafted grids with snake owners up to 15 (the 0.7**cycle
           darkening, cycles 0..3);
* rgb      uint8 (G, 20, 20, 3): rgb_from_grid of each grid.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(HERE, 'gymstub'), '/root/reference/marlenv']

from marlenv.core.grid_util import rgb_from_grid  # noqa: E402
from marlenv.core.snake import Cell, CellColors  # noqa: E402


def main():
    pal = np.zeros((6, 16, 3), np.uint8)
    for code in range(6):
        for i in range(16):
            pal[code, i] = rgb_from_grid(np.array([[10 * i + code]]), Cell, CellColors)[0, 0]
    grids = []
    for name in ('vr5_s4', 'full20_s4'):
        z = np.load(os.path.join(OUT, f'traj_{name}.npz'), allow_pickle=False)
        grids.append(z['grids'][0].astype(np.uint8))
    rs = np.random.RandomState(2024)
    for _ in range(3):
        g = np.zeros((20, 20), np.int64)
        g[0, :] = g[-1, :] = g[:, 0] = g[:, -1] = 1
        inner = rs.randint(0, 6, size=(18, 18))
        owner = rs.randint(0, 16, size=(18, 18))
        g[1:-1, 1:-1] = np.where(inner >= 3, 10 * owner + inner, inner)
        grids.append(g.astype(np.uint8))
    grids = np.stack(grids)
    rgb = np.stack([rgb_from_grid(g.astype(np.int64), Cell, CellColors) for g in grids])
    np.savez_compressed(os.path.join(OUT, 'render.npz'), palette=pal, grids=grids, rgb=rgb)
    print('render.npz', grids.shape, rgb.shape)


if __name__ == '__main__':
    main()
