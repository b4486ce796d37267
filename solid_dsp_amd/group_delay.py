"""``solid::group_delay`` (src/group_delay/mod.rs:51-129), host f64."""
from __future__ import annotations

import numpy as np

from . import _lib as L


class DelayError(ValueError):
    CODES = {1: "Empty Coefficients", 2: "Frequency Out of Bounds [-0.5, 0.5]",
             3: "Denominator Coefficents Divide Numerator by Zero"}

    def __init__(self, code):
        self.code = code
        super().__init__(f"Delay Error: {self.CODES.get(code, code)}")


def fir_group_delay(coefs, frequency: float) -> float:
    h = np.ascontiguousarray(coefs, dtype=np.float64)
    out = np.zeros(1)
    rc = L.lib().sdsp_fir_group_delay_taps(L.dptr(h), len(h), frequency, L.dptr(out))
    if rc:
        raise DelayError(rc)
    return float(out[0])


def iir_group_delay(numerator, denominator, frequency: float) -> float:
    b = np.ascontiguousarray(numerator, dtype=np.float64)
    a = np.ascontiguousarray(denominator, dtype=np.float64)
    out = np.zeros(1)
    rc = L.lib().sdsp_iir_group_delay_taps(L.dptr(b), len(b), L.dptr(a), len(a), frequency, L.dptr(out))
    if rc:
        raise DelayError(rc)
    return float(out[0])
