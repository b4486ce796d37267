"""``solid::nco::NCO`` on MI355X (src/nco/mod.rs:27-203).

The phase (``theta``) and frequency (``delta_theta``) are u32 registers held on
the host, updated exactly as the reference does (``constrain``, wrapping adds).
Sample blocks are mixed on the device (``kern_rx.hip``) with the reference's
1024-entry f64 sine table and index rule: ``mix_up_block(x)[i]`` is
``mix_up(x[i])`` at the phase reached after ``i`` steps.  The reference's own
``mix_up_block`` / ``mix_down_block`` (:153-172) index an empty ``Vec`` and
panic for any non-empty input; these are the per-sample loop they spell out.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def constrain(theta: float) -> int:  # :175-187 (the u32 phase of an angle)
    return int(L.lib().sdsp_nco_constrain(float(theta)))


class NCOError(L.SdspError):
    """NCOError(NCOErrorCode::BandwidthOutOfRange)  (src/nco/mod.rs:7-24)."""


class NCO:
    def __init__(self, device: int = 0):
        h = C.c_void_p()
        L.check(L.lib().sdsp_nco_create(C.byref(h), int(device)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            L.lib().sdsp_nco_destroy(h)
            self._h = None

    def reset(self):
        L.check(L.lib().sdsp_nco_reset(self._h))

    def set_frequency(self, delta_theta: float):
        L.check(L.lib().sdsp_nco_set_frequency(self._h, float(delta_theta)))

    def adjust_frequency(self, dt: float):
        L.check(L.lib().sdsp_nco_adjust_frequency(self._h, float(dt)))

    def get_frequency(self) -> float:
        return float(L.lib().sdsp_nco_get_frequency(self._h))

    def set_phase(self, phi: float):
        L.check(L.lib().sdsp_nco_set_phase(self._h, float(phi)))

    def adjust_phase(self, delta_phi: float):
        L.check(L.lib().sdsp_nco_adjust_phase(self._h, float(delta_phi)))

    def get_phase(self) -> float:
        return float(L.lib().sdsp_nco_get_phase(self._h))

    def step(self):
        L.check(L.lib().sdsp_nco_step(self._h))

    def sincos(self):
        sc = np.zeros(2)
        L.check(L.lib().sdsp_nco_sincos(self._h, L.dptr(sc)))
        return float(sc[0]), float(sc[1])

    def sin(self) -> float:
        return self.sincos()[0]

    def cos(self) -> float:
        return self.sincos()[1]

    def complex_exponential(self) -> complex:
        s, c = self.sincos()
        return complex(c, s)

    def set_internal_pll_bandwidth(self, bandwidth: float):
        rc = L.lib().sdsp_nco_set_internal_pll_bandwidth(self._h, float(bandwidth))
        if rc == 30:
            raise NCOError(rc, "NCO Error Bandwidth out Range [0, inf)")
        L.check(rc)

    def pll_step(self, delta_phi: float):
        L.check(L.lib().sdsp_nco_pll_step(self._h, float(delta_phi)))

    def state(self):
        th, dt = C.c_uint32(), C.c_uint32()
        L.check(L.lib().sdsp_nco_get_state(self._h, C.byref(th), C.byref(dt)))
        return th.value, dt.value

    def set_state(self, theta: int, delta_theta: int):
        L.check(L.lib().sdsp_nco_set_state(self._h, int(theta) & 0xFFFFFFFF, int(delta_theta) & 0xFFFFFFFF))

    def _mix(self, x, down):
        x = np.ascontiguousarray(x)
        if x.dtype not in (np.complex64, np.complex128):
            x = x.astype(np.complex128)
        out = np.empty_like(x)
        prec = 1 if x.dtype == np.complex128 else 0
        L.check(L.lib().sdsp_nco_mix_block(self._h, int(down), prec, L.ptr(x) if x.size else None, x.size,
                                           L.ptr(out) if out.size else None))
        return out

    def mix_up_block(self, x) -> np.ndarray:  # :153-161
        return self._mix(x, False)

    def mix_down_block(self, x) -> np.ndarray:  # :164-172
        return self._mix(x, True)

    def mix_up(self, x) -> complex:  # :141-144 (no step)
        th, dt = self.state()
        y = self._mix(np.array([x], dtype=np.complex128), False)[0]
        self.set_state(th, dt)
        return complex(y)

    def mix_down(self, x) -> complex:  # :147-150 (no step)
        th, dt = self.state()
        y = self._mix(np.array([x], dtype=np.complex128), True)[0]
        self.set_state(th, dt)
        return complex(y)

    def mix_block_device(self, d_in, n: int, d_out, down: bool = False, precision: int = 0, stream=None):
        L.check(L.lib().sdsp_nco_mix_block_device(self._h, int(down), int(precision), L.device_ptr(d_in), n,
                                                  L.device_ptr(d_out), L.stream_handle(stream)))

    def __str__(self):
        th, dt = self.state()
        return f"NCO [Theta={th}] [ΔTheta={dt}]"
