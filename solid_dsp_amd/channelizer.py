"""PFB + FFT channeliser (BASELINE config 5; build-defined composition of the
reference's PolyPhaseFilterBank coefficient layout, src/filter/fir/pfb.rs:24-49,
and FFT FORWARD, src/fft/mod.rs:175-215 — SURVEY Appendix A.6).

    v_p[m] = sum_{i<K} h[p + (K-1-i) M] x[(m-i) M + (M-1-p)]
    X[m]   = FFT_M(v[m])          (forward, unnormalised)
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class Channelizer:
    def __init__(self, taps, channels: int, sample_dtype=np.complex64, device=0, streams=1):
        sdt = np.dtype(sample_dtype)
        self.dtype = L.RC32 if sdt == np.complex64 else L.RC64
        self.coef_dtype = L.COEF_DTYPE[self.dtype]
        self.sample_dtype = L.SAMPLE_DTYPE[self.dtype]
        t = np.ascontiguousarray(taps, dtype=self.coef_dtype)
        h = C.c_void_p()
        L.check(L.lib().sdsp_chan_create(C.byref(h), self.dtype, L.ptr(t) if len(t) else None, len(t), channels,
                                         device))
        self._h = h
        self.M = channels
        self.device = device
        self.streams = 1
        if streams != 1:
            self.set_streams(streams)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            L.lib().sdsp_chan_destroy(h)
            self._h = None

    def set_tuning(self, key: int, value: int):
        """Kernel-variant knobs (L.TUNE_CHAN_STREAMING, L.TUNE_CHAN_FRAMES_PER_BLOCK, L.TUNE_CHAN_XCD_ORDER;
        performance only, same results)."""
        L.check(L.lib().sdsp_chan_set_tuning(self._h, int(key), int(value)))

    def set_streams(self, streams: int):
        L.check(L.lib().sdsp_chan_set_streams(self._h, streams))
        self.streams = streams

    def reset(self):
        L.check(L.lib().sdsp_chan_reset(self._h))

    def execute_block(self, samples) -> np.ndarray:
        """[streams, n] (or [n]) samples -> [streams, n/M, M] (or [n/M, M]) channel outputs."""
        x = np.ascontiguousarray(samples, dtype=self.sample_dtype)
        n = x.shape[-1]
        out = np.zeros(x.shape[:-1] + (n // self.M, self.M), dtype=self.sample_dtype)
        fr = C.c_size_t(0)
        L.check(L.lib().sdsp_chan_execute_block(self._h, L.ptr(x), n, L.ptr(out) if out.size else None,
                                                C.byref(fr)))
        return out

    def execute_block_device(self, d_in, n: int, d_out, stream=None) -> int:
        fr = C.c_size_t(0)
        pin = L.device_ptr(d_in, self.sample_dtype, self.streams * n, self.device, "input")
        pout = L.device_ptr(d_out, self.sample_dtype, self.streams * n, self.device, "output")
        L.check(L.lib().sdsp_chan_execute_block_device(self._h, pin, n, pout, C.byref(fr), L.stream_handle(stream)))
        return fr.value

    def synchronize(self):
        L.check(L.lib().sdsp_chan_synchronize(self._h))
