"""``solid::fft`` on MI355X (src/fft/mod.rs:175-215).

``FFT(nfft, FFTDirection.FORWARD).execute(x)`` is ``FFT::new(nfft, FORWARD,
ESTIMATE).execute(&x)``: unnormalised in both directions, any size 1 .. 2^24.
The device runs a radix-4 Stockham FFT in LDS (powers of two up to 4096), a
four-step FFT (larger powers of two), a direct DFT (other sizes up to 512) or
Bluestein's chirp-z transform (other sizes).
"""
from __future__ import annotations

import ctypes as C
import enum

import numpy as np

from . import _lib as L


class FFTDirection(enum.IntEnum):  # src/fft/mod.rs:14-18
    FORWARD = 0
    REVERSE = 1


class FFTFlags(enum.IntEnum):  # src/fft/mod.rs:49-53 (planning hint; one plan kind on the device)
    ESTIMATE = 0
    MEASURE = 1


class FFT:
    def __init__(self, nfft: int, direction=FFTDirection.FORWARD, flags=FFTFlags.ESTIMATE, precision=np.complex128,
                 device=0):
        self.nfft = int(nfft)
        self.direction = FFTDirection(int(direction))
        self.dtype = np.dtype(precision)
        if self.dtype not in (np.complex64, np.complex128):
            raise TypeError("precision must be complex64 or complex128")
        h = C.c_void_p()
        L.check(L.lib().sdsp_fft_create(C.byref(h), self.nfft, int(self.direction),
                                        1 if self.dtype == np.complex128 else 0, device))
        self._h = h

    @classmethod
    def new(cls, nfft, direction=FFTDirection.FORWARD, flags=FFTFlags.ESTIMATE, **kw):
        return cls(nfft, direction, flags, **kw)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            L.lib().sdsp_fft_destroy(h)
            self._h = None

    METHODS = {0: "direct DFT", 1: "Stockham (LDS)", 2: "Bluestein", 3: "four-step"}

    def set_tuning(self, key: int, value: int):
        """Kernel-variant knobs (L.TUNE_FFT_GROUP, L.TUNE_FFT_WAVE1024; performance only)."""
        L.check(L.lib().sdsp_fft_set_tuning(self._h, int(key), int(value)))

    @property
    def method(self) -> str:
        """Device plan of this size (the reference plans Rader / mixed radix / DFT leaves)."""
        return self.METHODS[int(L.lib().sdsp_fft_method(self._h))]

    def execute(self, x) -> np.ndarray:
        """One transform of nfft samples, or a [batch, nfft] array of them."""
        a = np.ascontiguousarray(x, dtype=self.dtype)
        if a.shape[-1] != self.nfft:
            raise ValueError("input length must equal nfft")
        batch = a.size // self.nfft
        out = np.empty_like(a)
        L.check(L.lib().sdsp_fft_execute(self._h, L.ptr(a), L.ptr(out), batch))
        return out

    def execute_device(self, d_in, d_out, batch: int, stream=None):
        L.check(L.lib().sdsp_fft_execute_device(self._h, L.device_ptr(d_in), L.device_ptr(d_out), batch,
                                                 L.stream_handle(stream)))
