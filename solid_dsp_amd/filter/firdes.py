"""``solid::filter::firdes`` (host f64 tap design, src/filter/firdes/mod.rs).

Evaluated by libsdsp.so's host code (design.cpp), exactly as the reference
does it on the host; returns float64 taps.
"""
from __future__ import annotations

import numpy as np

import ctypes as C
import enum

from .. import _lib as L


class EstimationMethod(enum.IntEnum):  # :46-49
    Kaiser = 0
    Herrmann = 1


def _check(rc):
    if rc:
        raise FirdesError(rc)


class FirdesError(ValueError):
    CODES = {1: "Bandwidth", 2: "StopBandLevel", 3: "Mu", 4: "SemiLength", 5: "FilterSize", 6: "FFTSize"}

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


def estimate_required_filter_length(transition_bandwidth: float, stop_band_attenuation: float,
                                    method: EstimationMethod) -> int:  # :71-94
    out = C.c_size_t(0)
    _check(L.lib().sdsp_firdes_estimate_length(transition_bandwidth, stop_band_attenuation, int(method),
                                               C.byref(out)))
    return out.value


def estimate_required_filter_stop_band_attenuation(transition_bandwidth: float, filter_length: int,
                                                   method: EstimationMethod) -> float:  # :117-145
    out = C.c_double(0.0)
    _check(L.lib().sdsp_firdes_estimate_stop_band_attenuation(transition_bandwidth, filter_length, int(method),
                                                              C.byref(out)))
    return out.value


def estimate_required_filter_transition(stop_band_attenuation: float, filter_length: int,
                                        method: EstimationMethod) -> float:  # :168-196
    out = C.c_double(0.0)
    _check(L.lib().sdsp_firdes_estimate_transition(stop_band_attenuation, filter_length, int(method),
                                                   C.byref(out)))
    return out.value


def estimate_required_filter_length_kaiser(transition_bandwidth: float, stop_band_attenuation: float) -> float:
    out = C.c_double(0.0)  # :199-211
    _check(L.lib().sdsp_firdes_estimate_length_kaiser(transition_bandwidth, stop_band_attenuation, C.byref(out)))
    return out.value


def estimate_required_filter_length_herrmann(transition_bandwidth: float, stop_band_attenuation: float) -> float:
    out = C.c_double(0.0)  # :213-240
    _check(L.lib().sdsp_firdes_estimate_length_herrmann(transition_bandwidth, stop_band_attenuation, C.byref(out)))
    return out.value


def firdes_doppler(filter_length: int, doppler_frequency: float, rice_fading_factor: float,
                   theta: float) -> np.ndarray:  # :389-419
    h = np.zeros(filter_length)
    _check(L.lib().sdsp_firdes_doppler(filter_length, doppler_frequency, rice_fading_factor, theta, L.dptr(h)))
    return h


def _f64(h):
    return np.ascontiguousarray(h, dtype=np.float64)


def filter_autocorrelation(filter, lag: int) -> float:  # :443-456
    h = _f64(filter)
    return float(L.lib().sdsp_filter_autocorrelation(L.dptr(h), h.size, lag))


def filter_crosscorrelation(h, g, lag: int) -> float:  # :487-527
    h, g = _f64(h), _f64(g)
    return float(L.lib().sdsp_filter_crosscorrelation(L.dptr(h), h.size, L.dptr(g), g.size, lag))


def filter_isi(filter, samples_per_symbol: int, filter_delay: int) -> tuple:  # :552-577
    h = _f64(filter)
    rms, mx = C.c_double(0.0), C.c_double(0.0)
    _check(L.lib().sdsp_filter_isi(L.dptr(h), h.size, samples_per_symbol, filter_delay, C.byref(rms), C.byref(mx)))
    return rms.value, mx.value


def filter_energy(filter, cutoff_frequency: float, fft_size: int) -> float:  # :602-640
    h = _f64(filter)
    out = C.c_double(0.0)
    _check(L.lib().sdsp_filter_energy(L.dptr(h) if h.size else None, h.size, cutoff_frequency, fft_size,
                                      C.byref(out)))
    return out.value
