"""Rectangle obstacles (dgppo/env/obstacle.py:30-105) as packed 16-float device records.

Record layout (include/dgppo_hip.h, DGPPO_OBST_FIELDS):
    [cx, cy, width, height, theta, cos(theta), sin(theta), type, p0x, p0y, p1x, p1y, p2x, p2y, p3x, p3y]
`Rectangle` exposes the reference's field names as views of that record (no copies); the
rectangles themselves are created on the GPU by the reset kernel (Rectangle.create semantics).
"""
from __future__ import annotations

import torch

OBST_FIELDS = 16


class Rectangle:
    __slots__ = ("packed",)

    def __init__(self, packed: torch.Tensor):
        assert packed.shape[-1] == OBST_FIELDS
        self.packed = packed

    @property
    def type(self):
        return self.packed[..., 7:8]

    @property
    def center(self):
        return self.packed[..., 0:2]

    @property
    def width(self):
        return self.packed[..., 2]

    @property
    def height(self):
        return self.packed[..., 3]

    @property
    def theta(self):
        return self.packed[..., 4]

    @property
    def points(self):
        return self.packed[..., 8:16].unflatten(-1, (4, 2))

    @property
    def n(self) -> int:
        return self.packed.shape[-2]

    def _map_tensors(self, fn):
        return Rectangle(fn(self.packed))

    def __getitem__(self, idx):
        return Rectangle(self.packed[idx])
