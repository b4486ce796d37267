"""``solid::dot_product`` (src/dot_product/{mod,execute}.rs) on MI355X.

``DotProduct(coefs, Direction.REVERSE).execute(samples)`` sums
``c[i] * s[i]`` for ``i < min(len(s), len(c))`` from zero, left to right, with
the coefficients stored forward or reversed — bit-identical to the reference
at the coefficient precision.  ``execute_batched_device`` evaluates many sample
vectors in one launch.
"""
from __future__ import annotations

import enum

import numpy as np

from . import _lib as L


class Direction(enum.IntEnum):  # src/dot_product/mod.rs:31-34
    FORWARD = 0
    REVERSE = 1


class DotProduct:
    def __init__(self, coefficients, direction=Direction.FORWARD, sample_dtype=None):
        c = np.asarray(coefficients)
        if c.dtype not in (np.float32, np.float64, np.complex64, np.complex128):
            c = c.astype(np.float64)
        self._c = np.ascontiguousarray(c)
        self.direction = Direction(int(direction))
        if sample_dtype is None:
            sample_dtype = self._c.dtype
        self.dtype = L.dtype_code(self._c.dtype, sample_dtype)
        self.sample_dtype = L.SAMPLE_DTYPE[self.dtype]

    @classmethod
    def new(cls, coefficients, direction, **kw):  # DotProduct::new  mod.rs:57-87
        return cls(coefficients, direction, **kw)

    def coefficents(self) -> np.ndarray:  # sic (mod.rs:102-109): stored order
        return self._c[::-1].copy() if self.direction == Direction.REVERSE else self._c.copy()

    coefficients = coefficents

    def len(self) -> int:
        return len(self._c)

    def __len__(self):
        return len(self._c)

    def is_empty(self) -> bool:
        return len(self._c) == 0

    def execute(self, samples):
        s = np.ascontiguousarray(samples, dtype=self.sample_dtype)
        out = np.zeros(1, dtype=self.sample_dtype)
        L.check(L.lib().sdsp_dot_execute(self.dtype, L.ptr(self._c) if len(self._c) else None, len(self._c),
                                         int(self.direction), L.ptr(s) if s.size else None, s.size, L.ptr(out)))
        return out[0]

    def execute_batched_device(self, d_samples, n: int, stride: int, batch: int, d_out, stream=None):
        L.check(L.lib().sdsp_dot_execute_batched_device(self.dtype, L.ptr(self._c) if len(self._c) else None,
                                                        len(self._c), int(self.direction), L.device_ptr(d_samples),
                                                        n, stride, batch, L.device_ptr(d_out),
                                                        L.stream_handle(stream)))
