"""``solid::filter::auto_correlator::AutoCorrelator`` on MI355X
(src/filter/auto_correlator/mod.rs:26-214).

After every pushed sample the correlator returns
``sum_{j < window} x[n-j] * conj(x[n-j-delay])``, where the terms with
``j + delay >= window`` are zero: the reference's delayed ``Window`` has
``window + delay`` zeroed slots but shifts only the first ``window - 1``, so
``to_vec()`` reads an unfilled tail (src/window/mod.rs:63-71).  The sum runs
newest first from zero in the sample precision — bit-identical to the
reference at ``Complex<f64>``.  ``get_energy`` is the sum of ``|x|^2`` over the
last ``window`` inputs in f64.  The work runs in ``kern_rx.hip``; there is no
CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import _lib as L


class AutoCorrelator:
    def __init__(self, window_size: int, delay: int, dtype=np.complex128, channels: int = 1, device: int = 0):
        self.dtype = np.dtype(dtype)
        if self.dtype not in (np.dtype(np.complex64), np.dtype(np.complex128)):
            raise TypeError("AutoCorrelator samples are Complex<f32> or Complex<f64>")
        self._prec = 1 if self.dtype == np.complex128 else 0
        self.channels = int(channels)
        h = C.c_void_p()
        L.check(L.lib().sdsp_acorr_create(C.byref(h), int(window_size), int(delay), self._prec, int(device)))
        self._h = h
        if self.channels != 1:
            L.check(L.lib().sdsp_acorr_set_channels(self._h, self.channels))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            L.lib().sdsp_acorr_destroy(h)
            self._h = None

    @property
    def window_size(self) -> int:
        return int(L.lib().sdsp_acorr_window_size(self._h))

    @property
    def delay(self) -> int:
        return int(L.lib().sdsp_acorr_delay(self._h))

    def _x(self, samples):
        x = np.ascontiguousarray(samples, dtype=self.dtype)
        if self.channels > 1 and (x.ndim != 2 or x.shape[0] != self.channels):
            raise ValueError(f"expected [{self.channels}, n] samples")
        return x

    def set_tuning(self, key: int, value: int):
        """Kernel-variant knob (L.TUNE_ACORR_KERNEL; performance only, same results)."""
        L.check(L.lib().sdsp_acorr_set_tuning(self._h, int(key), int(value)))

    def reset(self):  # :76-85
        L.check(L.lib().sdsp_acorr_reset(self._h))

    def push(self, sample):  # :99-111
        a = np.array([sample], dtype=self.dtype)
        L.check(L.lib().sdsp_acorr_push(self._h, L.ptr(a)))

    def write(self, samples):  # :128-137
        x = self._x(samples)
        n = x.shape[-1]
        L.check(L.lib().sdsp_acorr_write(self._h, L.ptr(x) if x.size else None, n))

    def execute(self):  # :156-163
        out = np.zeros(self.channels, dtype=self.dtype)
        L.check(L.lib().sdsp_acorr_execute(self._h, L.ptr(out)))
        return out[0] if self.channels == 1 else out

    def execute_block(self, samples) -> np.ndarray:  # :181-191
        x = self._x(samples)
        out = np.zeros_like(x)
        n = x.shape[-1]
        L.check(L.lib().sdsp_acorr_execute_block(self._h, L.ptr(x) if x.size else None, n,
                                                 L.ptr(out) if out.size else None))
        return out

    def execute_block_device(self, d_in, n: int, d_out, stream=None):
        L.check(L.lib().sdsp_acorr_execute_block_device(self._h, L.device_ptr(d_in), n, L.device_ptr(d_out),
                                                        L.stream_handle(stream)))

    def write_device(self, d_in, n: int, stream=None):
        L.check(L.lib().sdsp_acorr_write_device(self._h, L.device_ptr(d_in), n, L.stream_handle(stream)))

    def get_energy(self):  # :212-214
        e = np.zeros(self.channels)
        L.check(L.lib().sdsp_acorr_get_energy(self._h, L.dptr(e)))
        return float(e[0]) if self.channels == 1 else e

    def synchronize(self):
        L.check(L.lib().sdsp_acorr_synchronize(self._h))

    def __str__(self):  # fmt::Display  :217-226
        t = "f64" if self._prec else "f32"
        e = self.get_energy()
        return f"AutoCorrelator<{t}> [Size={self.window_size}] [Delay={self.delay}] [Energy={e}]"
