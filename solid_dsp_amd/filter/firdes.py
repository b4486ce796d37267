"""``solid::filter::firdes`` (host f64 tap design, src/filter/firdes/mod.rs).

Evaluated by libsdsp.so's host code (design.cpp), exactly as the reference
does it on the host; returns float64 taps.
"""
from __future__ import annotations

import numpy as np

from .. import _lib as L


class FirdesError(ValueError):
    CODES = {1: "Bandwidth", 2: "StopBandLevel", 3: "Mu", 4: "SemiLength"}

    def __init__(self, code):
        self.code = code
        super().__init__(f"Firdes Error: {self.CODES.get(code, code)}")


def kaiser_beta(stop_band_attenuation: float) -> float:  # :243-253
    return float(L.lib().sdsp_kaiser_beta(stop_band_attenuation))


def firdes_kaiser(filter_length: int, cutoff_frequency: float, stop_band_attenuation: float,
                  fractional_sample_offset: float = 0.0) -> np.ndarray:  # :278-305
    h = np.zeros(filter_length)
    rc = L.lib().sdsp_firdes_kaiser(filter_length, cutoff_frequency, stop_band_attenuation,
                                    fractional_sample_offset, L.dptr(h))
    if rc:
        raise FirdesError(rc)
    return h


def firdes_notch(semi_length: int, notch_frequency: float, stop_band_attenuation: float) -> np.ndarray:  # :329-368
    h = np.zeros(2 * semi_length + 1)
    rc = L.lib().sdsp_firdes_notch(semi_length, notch_frequency, stop_band_attenuation, L.dptr(h))
    if rc:
        raise FirdesError(rc)
    return h
