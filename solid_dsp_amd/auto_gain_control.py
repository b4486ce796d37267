"""``solid::auto_gain_control::AGC`` on MI355X (src/auto_gain_control/mod.rs:97-677).

An ``AGC`` here is a bank of ``channels`` independent gain controllers (1 by
default, the reference's object).  Their state lives on the device; one lane
per channel runs the reference's per-sample recurrence (``execute`` :214-246:
output, energy estimate, ``gain *= exp(-alpha/2 ln E)``, the 1e6 gain cap and
the squelch state machine :631-677) in ``kern_rx.hip``.  Samples are f64 or
complex128 — the two types the reference's trait bounds admit.  The
recurrence's exp/ln/log10 are the device's f64 functions, so outputs match the
reference to libm rounding (tests/test_gpu_rx.py states the tolerance), not bit
for bit.  There is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import enum
import math

import numpy as np

from . import _lib as L


class AGCErrorCode(enum.IntEnum):  # :49-56
    BandwidthOutOfRange = 40
    SignalLevelOutOfRange = 41
    GainBelowThreshold = 42
    ScaleBelowThreshold = 43
    SamplesTooLow = 44


class AGCError(L.SdspError):
    """AGCError(AGCErrorCode, value)  (:58-80)."""


class SquelchMode(enum.IntEnum):  # :84-94
    UNKNOWN = 0
    ENABLED = 1
    RISE = 2
    SIGNALHI = 3
    FALL = 4
    SINGALLO = 5
    TIMEOUT = 6
    DISABLED = 7


def _check(rc: int):
    if rc in AGCErrorCode._value2member_map_:
        raise AGCError(rc, L.lib().sdsp_last_error().decode(errors="replace"))
    L.check(rc)


class AGC:
    def __init__(self, channels: int = 1, device: int = 0):  # AGC::new  :136-149
        h = C.c_void_p()
        L.check(L.lib().sdsp_agc_create(C.byref(h), int(channels), int(device)))
        self._h = h
        self.channels = int(channels)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            L.lib().sdsp_agc_destroy(h)
            self._h = None

    def set_tuning(self, key: int, value: int):
        """Kernel-variant knob (L.TUNE_AGC_KERNEL; performance only, same results)."""
        _check(L.lib().sdsp_agc_set_tuning(self._h, int(key), int(value)))

    # ---- state ---------------------------------------------------------------
    def state(self, channel: int = 0) -> L.AgcState:
        st = L.AgcState()
        L.check(L.lib().sdsp_agc_get_state(self._h, int(channel), C.byref(st)))
        return st

    def set_state(self, st: L.AgcState, channel: int = 0):
        L.check(L.lib().sdsp_agc_set_state(self._h, int(channel), C.byref(st)))

    def _field(self, name):
        if self.channels == 1:
            return getattr(self.state(), name)
        return np.array([getattr(self.state(c), name) for c in range(self.channels)])

    # ---- processing ------------------------------------------------------------
    def _x(self, samples):
        x = np.ascontiguousarray(samples)
        x = x.astype(np.complex128 if np.iscomplexobj(x) else np.float64, copy=False)
        if self.channels > 1 and (x.ndim != 2 or x.shape[0] != self.channels):
            raise ValueError(f"expected [{self.channels}, n] samples")
        return x, (1 if np.iscomplexobj(x) else 0)

    def execute(self, sample):  # :214-246
        y = self.execute_block(np.array([sample]))
        return y[0]

    def execute_block(self, samples) -> np.ndarray:  # :273-285
        x, st = self._x(samples)
        out = np.empty_like(x)
        n = x.shape[-1]
        L.check(L.lib().sdsp_agc_execute_block(self._h, st, L.ptr(x) if x.size else None, n,
                                               L.ptr(out) if out.size else None))
        return out

    def execute_block_device(self, d_in, n: int, d_out, complex_: bool = True, stream=None):
        L.check(L.lib().sdsp_agc_execute_block_device(self._h, 1 if complex_ else 0, L.device_ptr(d_in), n,
                                                      L.device_ptr(d_out), L.stream_handle(stream)))

    def init(self, samples):  # :568-586; returns the linear signal level
        x, st = self._x(samples)
        lv = np.zeros(self.channels)
        _check(L.lib().sdsp_agc_init(self._h, st, L.ptr(x) if x.size else None, x.shape[-1], L.dptr(lv)))
        return float(lv[0]) if self.channels == 1 else lv

    def reset(self):  # :178-188
        L.check(L.lib().sdsp_agc_reset(self._h))

    # ---- lock ------------------------------------------------------------------
    def lock(self):  # :303-305
        L.check(L.lib().sdsp_agc_lock(self._h))

    def unlock(self):  # :322-324
        L.check(L.lib().sdsp_agc_unlock(self._h))

    def is_unlocked(self) -> bool:  # :341-343 — returns the lock flag, as the reference does
        return bool(self.state().lock)

    # ---- getters / setters -----------------------------------------------------------
    def get_bandwidth(self):  # :357-359
        return self._field("bandwidth")

    def set_bandwidth(self, bandwidth: float) -> float:  # :374-386
        _check(L.lib().sdsp_agc_set_bandwidth(self._h, float(bandwidth)))
        return bandwidth

    def get_signal_level(self):  # :400-402
        g = self._field("gain")
        return 1.0 / g

    def set_signal_level(self, level: float) -> float:  # :416-428
        _check(L.lib().sdsp_agc_set_signal_level(self._h, float(level)))
        return level

    def get_rssi(self):  # :442-444
        g = self._field("gain")
        if self.channels == 1:
            return math.log10(g) * -20.0
        return np.log10(g) * -20.0

    def set_rssi(self, rssi: float):  # :458-466
        L.check(L.lib().sdsp_agc_set_rssi(self._h, float(rssi)))

    def get_gain(self):  # :480-482
        return self._field("gain")

    def set_gain(self, gain: float) -> float:  # :497-504
        _check(L.lib().sdsp_agc_set_gain(self._h, float(gain)))
        return gain

    def get_scale(self):  # :518-520
        return self._field("scale")

    def set_scale(self, scale: float) -> float:  # :535-542
        _check(L.lib().sdsp_agc_set_scale(self._h, float(scale)))
        return scale

    # ---- squelch ---------------------------------------------------------------
    def squelch_enable(self):  # :589-591
        L.check(L.lib().sdsp_agc_squelch_enable(self._h))

    def squelch_disable(self):  # :594-596
        L.check(L.lib().sdsp_agc_squelch_disable(self._h))

    def is_squelch_enabled(self) -> bool:  # :598-604
        return self.state().squelch_mode != SquelchMode.DISABLED

    def squelch_get_threshold(self) -> float:
        return self.state().squelch_threshold

    def squelch_set_threshold(self, threshold: float):
        L.check(L.lib().sdsp_agc_squelch_set_threshold(self._h, float(threshold)))

    def squelch_get_timeout(self) -> int:
        return int(self.state().squelch_timeout)

    def squelch_set_timeout(self, timeout: int):
        L.check(L.lib().sdsp_agc_squelch_set_timeout(self._h, int(timeout)))

    def update_squelch_mode(self):  # :631-677 (one step per channel)
        L.check(L.lib().sdsp_agc_update_squelch_mode(self._h))

    def squelch_get_mode(self) -> SquelchMode:
        return SquelchMode(self.state().squelch_mode)

    def synchronize(self):
        L.check(L.lib().sdsp_agc_synchronize(self._h))

    def __str__(self):  # fmt::Display  :686-693
        s = self.state()
        return (f"AGC [Gain={s.gain:.5f}] [Scale={s.scale:.5f}] [Bandwidth={s.bandwidth:.5f}] "
                f"[Alpha={s.alpha:.5f}] [Energy={s.energy_estimate:.5f}]")
