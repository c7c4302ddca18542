"""Colours of the reference renderer and the palette snake_render_rgb looks up.

CELL_COLORS restates CellColors (marlenv/marlenv/core/snake.py:14-30): one list
of RGB triples per cell code, indexed by the owning snake (cell value // 10)
modulo the list length; each further cycle through the list darkens by 0.7
(rgb_from_grid, grid_util.py:164-175). palette() evaluates that expression for
every (code, owner) a grid can hold, with the reference's own numpy arithmetic
(int64 colour * python-float 0.7**cycle, truncated by astype(uint8)), so the
device kernel is a pure table lookup."""
import numpy as np

from .snake import Cell

MAX_OWNERS = 16   # snake_cfg.num_snakes <= 16 (include/snake_env.h)

_COLOR_WHEEL = [(104, 255, 0), (255, 191, 0), (255, 0, 92), (0, 111, 255)]
_HEAD_COLOR_WHEEL = [(min(255, int(r * 2.0)), min(255, int(g * 2.0)), min(255, int(b * 2.0)))
                     for (r, g, b) in _COLOR_WHEEL]

CELL_COLORS = {
    Cell.EMPTY.value: [(0, 0, 0)],
    Cell.WALL.value: [(32, 32, 32)],
    Cell.FRUIT.value: [(223, 7, 22)],
    Cell.HEAD.value: _HEAD_COLOR_WHEEL,
    Cell.BODY.value: _COLOR_WHEEL,
    Cell.TAIL.value: _COLOR_WHEEL,
}


def palette():
    """uint8 (6, MAX_OWNERS, 3): colour of a cell of code c owned by snake i."""
    pal = np.zeros((6, MAX_OWNERS, 3), np.uint8)
    for code, colors in CELL_COLORS.items():
        for cell_id in range(MAX_OWNERS):
            cell_color = np.array(colors[cell_id % len(colors)])
            cycle = cell_id // len(colors)
            pal[code, cell_id] = (cell_color * 0.7**cycle).astype(np.uint8)
    return pal


def upscale(rgb, max_size=300):
    """image_from_grid's nearest-neighbour enlargement (grid_util.py:178-185),
    on an (H, W, 3) uint8 array; returns the enlarged array."""
    scale = max(max_size // max(rgb.shape[:2]), 1)
    return np.repeat(np.repeat(rgb, scale, axis=0), scale, axis=1)
