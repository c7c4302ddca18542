"""Cell / Direction enums of the reference (marlenv/marlenv/core/snake.py:5-49),
kept for callers that decode grids or obs channels."""
from enum import Enum


class Cell(Enum):
    EMPTY = 0
    WALL = 1
    FRUIT = 2
    HEAD = 3
    BODY = 4
    TAIL = 5


class Direction(Enum):
    UP = (-1, 0)
    RIGHT = (0, 1)
    DOWN = (1, 0)
    LEFT = (0, -1)

    def __radd__(self, other):
        dr, dc = self.value
        return other[0] + dr, other[1] + dc

    def __rsub__(self, other):
        dr, dc = self.value
        return other[0] - dr, other[1] - dc


# kernel direction index -> Direction (csrc/snake_kernels.hip dir_dr/dir_dc)
DIRECTION_OF_INDEX = (Direction.UP, Direction.RIGHT, Direction.DOWN, Direction.LEFT)
