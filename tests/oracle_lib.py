"""ctypes loader for the CPU restatement in ``oracle/`` (test infrastructure only).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg use
this module; the product package ``solid_dsp_amd`` never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "libsdsp_oracle.so")

RR32, RC32, CC32, RR64, RC64, CC64 = range(6)
NORMAL, SECOND_ORDER = 0, 1

_IN_DT = {RR32: np.float32, RC32: np.complex64, CC32: np.complex64,
          RR64: np.float64, RC64: np.complex128, CC64: np.complex128}
_COEF_DT = {RR32: np.float32, RC32: np.float32, CC32: np.complex64,
            RR64: np.float64, RC64: np.float64, CC64: np.complex128}

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return ORACLE_SO


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        build()
    L = C.CDLL(ORACLE_SO)
    vp, sz, ip, dp = C.c_void_p, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_double)
    sig = {
        "orc_msb_index": (sz, [sz]),
        "orc_fir_new": (vp, [C.c_int, vp, sz, vp, ip]),
        "orc_decim_new": (vp, [C.c_int, vp, sz, vp, sz, ip]),
        "orc_pfb_new": (vp, [C.c_int, vp, sz, sz, vp, ip]),
        "orc_interp_new": (vp, [C.c_int, vp, sz, sz, ip]),
        "orc_execute_block": (sz, [vp, vp, sz, vp]),
        "orc_push": (None, [vp, vp]),
        "orc_write": (None, [vp, vp, sz]),
        "orc_reset": (None, [vp]),
        "orc_clone": (vp, [vp]),
        "orc_free": (None, [vp]),
        "orc_sos_state": (C.c_int, [vp, vp, C.c_int]),
        "orc_group_delay": (C.c_double, [vp, C.c_double]),
        "orc_frequency_response": (None, [vp, C.c_double, dp]),
        "orc_pfb_execute": (C.c_int, [vp, C.c_int, sz, vp]),
        "orc_iir_new": (vp, [C.c_int, vp, sz, vp, sz, C.c_int, ip]),
        "orc_iir_decim_new": (vp, [C.c_int, vp, sz, vp, sz, C.c_int, sz, ip]),
        "orc_iir_interp_new": (vp, [C.c_int, vp, sz, vp, sz, C.c_int, sz, ip]),
        "orc_sos_new": (vp, [dp, sz, dp, sz, ip]),
        "orc_sos_execute": (C.c_double, [vp, C.c_double]),
        "orc_sos_group_delay": (C.c_double, [vp, C.c_double]),
        "orc_sos_coefs": (None, [vp, dp, dp]),
        "orc_sos_free": (None, [vp]),
        "orc_dot_execute": (None, [C.c_int, vp, sz, C.c_int, vp, sz, dp]),
        "orc_fir_group_delay": (C.c_double, [dp, sz, C.c_double, ip]),
        "orc_iir_group_delay": (C.c_double, [dp, sz, dp, sz, C.c_double, ip]),
        "orc_sinc": (C.c_double, [C.c_double]),
        "orc_besseli": (C.c_double, [C.c_double, C.c_double]),
        "orc_lngamma": (C.c_double, [C.c_double]),
        "orc_kaiser": (C.c_double, [sz, sz, C.c_double]),
        "orc_kaiser_beta": (C.c_double, [C.c_double]),
        "orc_firdes_kaiser": (C.c_int, [sz, C.c_double, C.c_double, C.c_double, dp]),
        "orc_firdes_notch": (C.c_int, [sz, C.c_double, C.c_double, dp]),
        "orc_estimate_req_filter_len": (C.c_int, [C.c_double, C.c_double, C.c_int, C.POINTER(sz)]),
        "orc_estimate_req_filter_as": (C.c_double, [C.c_double, sz, C.c_int]),
        "orc_estimate_req_filter_df": (C.c_double, [C.c_double, sz, C.c_int]),
        "orc_firdes_doppler": (None, [sz, C.c_double, C.c_double, C.c_double, dp]),
        "orc_filter_autocorrelation": (C.c_double, [dp, sz, C.c_long]),
        "orc_filter_crosscorrelation": (C.c_double, [dp, sz, dp, sz, C.c_long]),
        "orc_filter_isi": (None, [dp, sz, sz, sz, dp, dp]),
        "orc_filter_energy": (C.c_int, [dp, sz, C.c_double, sz, dp]),
        "orc_active_lag": (C.c_int, [C.c_double, C.c_double, C.c_double, dp, dp]),
        "orc_active_pi": (C.c_int, [C.c_double, C.c_double, C.c_double, dp, dp]),
        "orc_synth_f32": (None, [C.c_uint64, C.c_uint64, C.c_uint64, sz, C.POINTER(C.c_float)]),
    }
    optional = {
        "orc_fft_new": (vp, [sz, C.c_int]),
        "orc_fft_execute": (C.c_int, [vp, vp, vp]),
        "orc_fft_free": (None, [vp]),
        "orc_fft_method": (C.c_int, [vp]),
        "orc_channelize": (sz, [vp, sz, sz, vp, sz, vp]),
        # sdsp_oracle_rx.cpp: AutoCorrelator / NCO
        "orc_acorr_new": (vp, [sz, sz, C.c_int]),
        "orc_acorr_free": (None, [vp]),
        "orc_acorr_reset": (None, [vp]),
        "orc_acorr_write": (None, [vp, vp, sz]),
        "orc_acorr_execute_block": (None, [vp, vp, sz, vp]),
        "orc_acorr_execute": (None, [vp, vp]),
        "orc_acorr_get_energy": (C.c_double, [vp]),
        "orc_nco_new": (vp, []),
        "orc_nco_free": (None, [vp]),
        "orc_nco_constrain": (C.c_uint32, [C.c_double]),
        "orc_nco_set_frequency": (None, [vp, C.c_double]),
        "orc_nco_adjust_frequency": (None, [vp, C.c_double]),
        "orc_nco_set_phase": (None, [vp, C.c_double]),
        "orc_nco_adjust_phase": (None, [vp, C.c_double]),
        "orc_nco_reset": (None, [vp]),
        "orc_nco_state": (None, [vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
        "orc_nco_sincos": (None, [vp, dp]),
        "orc_nco_set_pll_bandwidth": (C.c_int, [vp, C.c_double]),
        "orc_nco_pll_step": (None, [vp, C.c_double]),
        "orc_nco_step": (None, [vp]),
        "orc_nco_mix_block": (None, [vp, C.c_int, dp, sz, dp]),
        "orc_agc_new": (vp, []),
        "orc_agc_free": (None, [vp]),
        "orc_agc_reset": (None, [vp]),
        "orc_agc_execute_block": (None, [vp, C.c_int, vp, sz, vp]),
        "orc_agc_init": (C.c_int, [vp, C.c_int, vp, sz, dp]),
        "orc_agc_set_bandwidth": (C.c_int, [vp, C.c_double]),
        "orc_agc_set_rssi": (None, [vp, C.c_double]),
        "orc_agc_set_gain": (None, [vp, C.c_double]),
        "orc_agc_set_scale": (None, [vp, C.c_double]),
        "orc_agc_lock": (None, [vp, C.c_int]),
        "orc_agc_squelch": (None, [vp, C.c_int]),
        "orc_agc_squelch_set_threshold": (None, [vp, C.c_double]),
        "orc_agc_squelch_set_timeout": (None, [vp, C.c_uint64]),
        "orc_agc_get_gain": (C.c_double, [vp]),
        "orc_agc_get_energy": (C.c_double, [vp]),
        "orc_agc_get_rssi": (C.c_double, [vp]),
        "orc_agc_get_mode": (C.c_int, [vp]),
        "orc_agc_get_timer": (C.c_uint64, [vp]),
    }
    for name, (res, args) in list(sig.items()) + list(optional.items()):
        if not hasattr(L, name):
            if name in optional:
                continue
            raise RuntimeError(f"oracle missing symbol {name}")
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _dptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class OracleObj:
    """Generic wrapper over an oracle filter handle."""

    def __init__(self, h, dtype, out_per_in=1, kind="fir", M=1):
        self.h = h
        self.dtype = dtype
        self.out_per_in = out_per_in
        self.kind = kind
        self.M = M

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_free(self.h)
            self.h = None

    @property
    def in_dt(self):
        return _IN_DT[self.dtype]

    def execute_block(self, x):
        x = np.ascontiguousarray(x, dtype=self.in_dt)
        cap = len(x) * self.out_per_in
        out = np.zeros(max(cap, 1), dtype=self.in_dt)
        n = lib().orc_execute_block(self.h, _ptr(x), len(x), _ptr(out))
        return out[:n]

    def push(self, s):
        a = np.array([s], dtype=self.in_dt)
        lib().orc_push(self.h, _ptr(a))

    def write(self, xs):
        a = np.ascontiguousarray(xs, dtype=self.in_dt)
        lib().orc_write(self.h, _ptr(a), len(a))

    def reset(self):
        lib().orc_reset(self.h)

    def group_delay(self, f):
        return lib().orc_group_delay(self.h, f)

    def frequency_response(self, f):
        out = np.zeros(2)
        lib().orc_frequency_response(self.h, f, _dptr(out))
        return complex(out[0], out[1])

    def sos_state(self, state=None):
        """SecondOrder IIR: the (w1, w2) state per section in the device handle's layout;
        with `state`, set it instead"""
        n = 2 * self._sections
        if state is None:
            st = np.zeros(n, dtype=self.in_dt)
            assert lib().orc_sos_state(self.h, _ptr(st), 0) == 0
            return st
        st = np.ascontiguousarray(state, dtype=self.in_dt)
        assert lib().orc_sos_state(self.h, _ptr(st), 1) == 0

    def pfb_execute(self, index):
        out = np.zeros(1, dtype=self.in_dt)
        rc = lib().orc_pfb_execute(self.h, self.dtype, index, _ptr(out))
        if rc:
            raise IndexError(index)
        return out[0]


def _mk(fn, *args):
    err = C.c_int(0)
    h = fn(*args, C.byref(err))
    if not h:
        raise ValueError(f"oracle construction error {err.value}")
    return h


def fir(dtype, taps, scale):
    t = np.ascontiguousarray(taps, dtype=_COEF_DT[dtype])
    s = np.array([scale], dtype=_COEF_DT[dtype])
    return OracleObj(_mk(lib().orc_fir_new, dtype, _ptr(t), len(t), _ptr(s)), dtype)


def decim(dtype, taps, scale, M):
    t = np.ascontiguousarray(taps, dtype=_COEF_DT[dtype])
    s = np.array([scale], dtype=_COEF_DT[dtype])
    return OracleObj(_mk(lib().orc_decim_new, dtype, _ptr(t), len(t), _ptr(s), M), dtype, kind="decim", M=M)


def pfb(dtype, taps, M, scale):
    t = np.ascontiguousarray(taps, dtype=_COEF_DT[dtype])
    s = np.array([scale], dtype=_COEF_DT[dtype])
    return OracleObj(_mk(lib().orc_pfb_new, dtype, _ptr(t), len(t), M, _ptr(s)), dtype, out_per_in=M, kind="pfb", M=M)


def interp(dtype, taps, M):
    t = np.ascontiguousarray(taps, dtype=_COEF_DT[dtype])
    return OracleObj(_mk(lib().orc_interp_new, dtype, _ptr(t), len(t), M), dtype, out_per_in=M, kind="interp", M=M)


def iir(dtype, ff, fb, type_):
    a = np.ascontiguousarray(ff, dtype=_COEF_DT[dtype])
    b = np.ascontiguousarray(fb, dtype=_COEF_DT[dtype])
    o = OracleObj(_mk(lib().orc_iir_new, dtype, _ptr(a), len(a), _ptr(b), len(b), type_), dtype, kind="iir")
    o._sections = len(a) // 3
    return o


def iir_decim(dtype, ff, fb, type_, M):
    a = np.ascontiguousarray(ff, dtype=_COEF_DT[dtype])
    b = np.ascontiguousarray(fb, dtype=_COEF_DT[dtype])
    return OracleObj(_mk(lib().orc_iir_decim_new, dtype, _ptr(a), len(a), _ptr(b), len(b), type_, M), dtype,
                     kind="iir_decim", M=M)


def iir_interp(dtype, ff, fb, type_, M):
    a = np.ascontiguousarray(ff, dtype=_COEF_DT[dtype])
    b = np.ascontiguousarray(fb, dtype=_COEF_DT[dtype])
    return OracleObj(_mk(lib().orc_iir_interp_new, dtype, _ptr(a), len(a), _ptr(b), len(b), type_, M), dtype,
                     out_per_in=M, kind="iir_interp", M=M)


def firdes_kaiser(n, fc, as_, mu):
    h = np.zeros(n)
    rc = lib().orc_firdes_kaiser(n, fc, as_, mu, _dptr(h))
    if rc:
        raise ValueError(rc)
    return h


def firdes_notch(m, f0, as_):
    h = np.zeros(2 * m + 1)
    rc = lib().orc_firdes_notch(m, f0, as_, _dptr(h))
    if rc:
        raise ValueError(rc)
    return h


def active_lag(bw, zeta, k):
    n, d = np.zeros(3), np.zeros(3)
    rc = lib().orc_active_lag(bw, zeta, k, _dptr(n), _dptr(d))
    if rc:
        raise ValueError(rc)
    return n, d


class AutoCorr:
    """Restated AutoCorrelator (oracle/sdsp_oracle_rx.cpp); dtype complex64 or complex128."""

    def __init__(self, window_size, delay, dtype=np.complex128):
        self.dt = np.dtype(dtype)
        self.h = lib().orc_acorr_new(window_size, delay, 1 if self.dt == np.complex128 else 0)
        if not self.h:
            raise ValueError("window_size must be > 0")

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_acorr_free(self.h)
            self.h = None

    def execute_block(self, x):
        x = np.ascontiguousarray(x, dtype=self.dt)
        out = np.zeros_like(x)
        lib().orc_acorr_execute_block(self.h, _ptr(x), len(x), _ptr(out))
        return out

    def write(self, x):
        x = np.ascontiguousarray(x, dtype=self.dt)
        lib().orc_acorr_write(self.h, _ptr(x), len(x))

    def execute(self):
        out = np.zeros(1, dtype=self.dt)
        lib().orc_acorr_execute(self.h, _ptr(out))
        return out[0]

    def get_energy(self):
        return lib().orc_acorr_get_energy(self.h)

    def reset(self):
        lib().orc_acorr_reset(self.h)


class Nco:
    """Restated NCO (oracle/sdsp_oracle_rx.cpp)."""

    def __init__(self):
        self.h = lib().orc_nco_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_nco_free(self.h)
            self.h = None

    def __getattr__(self, name):
        f = getattr(lib(), "orc_nco_" + name)
        return lambda *a: f(self.h, *a)

    def state(self):
        th, dt = C.c_uint32(), C.c_uint32()
        lib().orc_nco_state(self.h, C.byref(th), C.byref(dt))
        return th.value, dt.value

    def sincos(self):
        sc = np.zeros(2)
        lib().orc_nco_sincos(self.h, _dptr(sc))
        return float(sc[0]), float(sc[1])

    def mix_block(self, x, down=False):
        x = np.ascontiguousarray(x, dtype=np.complex128)
        out = np.zeros_like(x)
        lib().orc_nco_mix_block(self.h, int(down), x.ctypes.data_as(C.POINTER(C.c_double)), len(x),
                                out.ctypes.data_as(C.POINTER(C.c_double)))
        return out


class Agc:
    """Restated AGC (oracle/sdsp_oracle_rx.cpp); samples f64 or complex128."""

    def __init__(self):
        self.h = lib().orc_agc_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_agc_free(self.h)
            self.h = None

    def __getattr__(self, name):
        f = getattr(lib(), "orc_agc_" + name)
        return lambda *a: f(self.h, *a)

    def execute_block(self, x):
        x = np.ascontiguousarray(x)
        st = 1 if np.iscomplexobj(x) else 0
        x = x.astype(np.complex128 if st else np.float64)
        out = np.zeros_like(x)
        lib().orc_agc_execute_block(self.h, st, _ptr(x), len(x), _ptr(out))
        return out

    def init(self, x):
        x = np.ascontiguousarray(x)
        st = 1 if np.iscomplexobj(x) else 0
        x = x.astype(np.complex128 if st else np.float64)
        lv = np.zeros(1)
        rc = lib().orc_agc_init(self.h, st, _ptr(x) if len(x) else None, len(x), _dptr(lv))
        return rc, float(lv[0])


def synth(seed, channel, start, count, complex_=False):
    """Build-defined synthetic stream.  count = samples."""
    scal = count * (2 if complex_ else 1)
    out = np.zeros(scal, dtype=np.float32)
    lib().orc_synth_f32(seed, channel, start * (2 if complex_ else 1), scal,
                        out.ctypes.data_as(C.POINTER(C.c_float)))
    return out.view(np.complex64) if complex_ else out
