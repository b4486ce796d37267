"""``solid::filter::iirdes::pll`` (src/filter/iirdes/pll/mod.rs:24-99)."""
from __future__ import annotations

import numpy as np

from .. import _lib as L


class IirdesError(ValueError):
    CODES = {1: "Bandwidth", 2: "DampingFactor", 3: "Gain"}

    def __init__(self, code):
        self.code = code
        super().__init__(f"Iirdes Error: {self.CODES.get(code, code)}")


class pll:  # noqa: N801 — module path solid::filter::iirdes::pll
    @staticmethod
    def active_lag(bandwidth: float, damping_factor: float, loop_gain: float):
        n, d = np.zeros(3), np.zeros(3)
        rc = L.lib().sdsp_active_lag(bandwidth, damping_factor, loop_gain, L.dptr(n), L.dptr(d))
        if rc:
            raise IirdesError(rc)
        return n, d

    @staticmethod
    def active_proportional_integral(bandwidth: float, damping_factor: float, loop_gain: float):
        n, d = np.zeros(3), np.zeros(3)
        rc = L.lib().sdsp_active_proportional_integral(bandwidth, damping_factor, loop_gain, L.dptr(n), L.dptr(d))
        if rc:
            raise IirdesError(rc)
        return n, d
