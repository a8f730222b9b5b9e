"""Axis helpers with haiku's published semantics (test shim)."""
from typing import Any

AxisOrAxes = Any


def to_axes_or_slice(axis):
    if isinstance(axis, slice):
        return axis
    if isinstance(axis, int):
        return (axis,)
    return tuple(axis)


def to_abs_axes(axis, ndim):
    if isinstance(axis, slice):
        return tuple(range(ndim)[axis])
    return tuple(sorted({a % ndim for a in axis}))
