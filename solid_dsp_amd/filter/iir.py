"""``solid::filter::iir`` on MI355X (src/filter/iir/{mod,sos,decim,interp}.rs).

IIRFilter(ff, fb, IIRFilterType.SecondOrder, sample_dtype=np.float64) is
``IIRFilter::<f64, f64>::new(&ff, &fb, IIRFilterType::SecondOrder)``.
Coefficients are real (the reference's Conj + Real bound holds for f64 only;
f32 coefficients are this engine's extension).  Errors carry the
reference's IIRErrorCode / SecondOrderErrorCode as ``SdspError.code``.
"""
from __future__ import annotations

import ctypes as C
import enum

import numpy as np

from .. import _lib as L


class IIRFilterType(enum.IntEnum):  # mod.rs:62-66
    Normal = 0
    SecondOrder = 1


def _default_sample(coef_dtype):
    return {np.dtype(np.float32): np.float32, np.dtype(np.float64): np.float64}[np.dtype(coef_dtype)]


class _IirBase:
    _mode = 0

    def __init__(self, feed_forward, feed_back, iirtype=IIRFilterType.SecondOrder, factor=1, sample_dtype=None,
                 coef_dtype=None, device=0, channels=1, algo=None):
        ff = np.asarray(feed_forward)
        cdt = np.dtype(coef_dtype) if coef_dtype is not None else (
            ff.dtype if ff.dtype in (np.float32, np.float64) else np.dtype(np.float64))
        ff = np.ascontiguousarray(ff, dtype=cdt)
        fb = np.ascontiguousarray(feed_back, dtype=cdt)
        if sample_dtype is None:
            sample_dtype = _default_sample(cdt)
        self.dtype = L.dtype_code(cdt, sample_dtype)
        self.coef_dtype = L.COEF_DTYPE[self.dtype]
        self.sample_dtype = L.SAMPLE_DTYPE[self.dtype]
        self.iirtype = IIRFilterType(int(iirtype))
        h = C.c_void_p()
        lib = L.lib()
        args = (C.byref(h), self.dtype, L.ptr(ff) if len(ff) else None, len(ff), L.ptr(fb) if len(fb) else None,
                len(fb), int(self.iirtype))
        if self._mode == 0:
            L.check(lib.sdsp_iir_create(*args, device))
        elif self._mode == 1:
            L.check(lib.sdsp_iir_decim_create(*args, factor, device))
        else:
            L.check(lib.sdsp_iir_interp_create(*args, factor, device))
        self._h = h
        self._factor = factor
        self.device = device
        self.channels = 1
        if channels != 1:
            self.set_channels(channels)
        if algo is not None:  # default: the handle's ALGO_EXACT (bit-identical to the reference)
            self.set_algo(algo)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            L.lib().sdsp_iir_destroy(h)
            self._h = None

    def clone(self):
        h = C.c_void_p()
        L.check(L.lib().sdsp_iir_clone(self._h, C.byref(h)))
        obj = type(self).__new__(type(self))
        obj.__dict__.update({k: v for k, v in self.__dict__.items() if k != "_h"})
        obj._h = h
        return obj

    def set_channels(self, channels):
        L.check(L.lib().sdsp_iir_set_channels(self._h, channels))
        self.channels = channels

    def set_algo(self, algo):
        L.check(L.lib().sdsp_iir_set_algo(self._h, algo))

    def set_tuning(self, key: int, value: int):
        """kernel-variant knobs (SDSP_TUNE_*, include/sdsp.h): performance only"""
        L.check(L.lib().sdsp_iir_set_tuning(self._h, int(key), int(value)))

    def scan_info(self, group=0):
        wc, ch = C.c_int(0), C.c_int(0)
        L.check(L.lib().sdsp_iir_scan_info(self._h, group, C.byref(wc), C.byref(ch)))
        return wc.value, ch.value

    def reset(self):
        L.check(L.lib().sdsp_iir_reset(self._h))

    def get_state(self):
        n = int(L.lib().sdsp_iir_state_len(self._h))
        st = np.zeros(n, dtype=self.sample_dtype)
        ph = C.c_size_t(0)
        L.check(L.lib().sdsp_iir_get_state(self._h, L.ptr(st) if n else None, C.byref(ph)))
        return st, ph.value

    def set_state(self, state, phase=0):
        st = np.ascontiguousarray(state, dtype=self.sample_dtype)
        L.check(L.lib().sdsp_iir_set_state(self._h, L.ptr(st) if st.size else None, phase))

    def wscan_mode(self, group: int = 0) -> int:
        """0 serial recurrence, 1 wave scan with warm-up, 2 wave scan with exact carries"""
        return int(L.lib().sdsp_iir_wscan_mode(self._h, group))

    def output_count(self, n):
        return int(L.lib().sdsp_iir_output_count(self._h, n))

    # ---- coefficient accessors (mod.rs:123-127 / 156-157) ------------------
    def numerator_coefs(self) -> np.ndarray:
        nn = int(L.lib().sdsp_iir_num_coefs(self._h, 0))
        nd = int(L.lib().sdsp_iir_num_coefs(self._h, 1))
        num, den = np.zeros(max(nn, 1)), np.zeros(max(nd, 1))
        L.check(L.lib().sdsp_iir_coefficients(self._h, L.dptr(num), L.dptr(den)))
        return num[:nn]

    def denominator_coefs(self) -> np.ndarray:
        nn = int(L.lib().sdsp_iir_num_coefs(self._h, 0))
        nd = int(L.lib().sdsp_iir_num_coefs(self._h, 1))
        num, den = np.zeros(max(nn, 1)), np.zeros(max(nd, 1))
        L.check(L.lib().sdsp_iir_coefficients(self._h, L.dptr(num), L.dptr(den)))
        return den[:nd]

    def iir_type(self):
        return self.iirtype

    def second_order_filters(self):
        """[(numerator_coefs = a[1..]/a0, denominator_coefs = b/a0)] per section (sos.rs:116-150)."""
        if self.iirtype != IIRFilterType.SecondOrder:
            return []
        out = []
        n = len(self.numerator_coefs()) // 3
        for s in range(n):
            a, b = np.zeros(2), np.zeros(3)
            L.check(L.lib().sdsp_sos_section_coefs(self._h, s, L.dptr(a), L.dptr(b)))
            out.append((a, b))
        return out

    # ---- Filter trait ------------------------------------------------------
    def execute(self, sample) -> list:
        x = np.array([sample], dtype=self.sample_dtype)
        y = np.zeros(max(self.output_count(1), 1), dtype=self.sample_dtype)
        n = C.c_size_t(0)
        L.check(L.lib().sdsp_iir_execute(self._h, L.ptr(x), L.ptr(y), C.byref(n)))
        return list(y[: n.value])

    def execute_block(self, samples) -> np.ndarray:
        x = np.ascontiguousarray(samples, dtype=self.sample_dtype)
        n = x.shape[-1] if x.ndim else 0
        nout = self.output_count(n)
        shape = (self.channels, nout) if self.channels > 1 else (nout,)
        y = np.zeros(shape, dtype=self.sample_dtype)
        got = C.c_size_t(0)
        L.check(L.lib().sdsp_iir_execute_block(self._h, L.ptr(x) if n else None, n, L.ptr(y) if y.size else None,
                                                C.byref(got)))
        return y

    def execute_block_device(self, d_in, n, d_out, stream=None) -> int:
        got = C.c_size_t(0)
        pin = L.device_ptr(d_in, self.sample_dtype, self.channels * n, self.device, "input")
        pout = L.device_ptr(d_out, self.sample_dtype, self.channels * self.output_count(n), self.device, "output")
        L.check(L.lib().sdsp_iir_execute_block_device(self._h, pin, n, pout, C.byref(got), L.stream_handle(stream)))
        return got.value

    def synchronize(self):
        L.check(L.lib().sdsp_iir_synchronize(self._h))

    def frequency_response(self, frequency: float) -> complex:
        out = np.zeros(2)
        L.check(L.lib().sdsp_iir_frequency_response(self._h, frequency, L.dptr(out)))
        return complex(out[0], out[1])

    def group_delay(self, frequency: float) -> float:
        out = np.zeros(1)
        L.check(L.lib().sdsp_iir_group_delay(self._h, frequency, L.dptr(out)))
        return float(out[0])


class IIRFilter(_IirBase):
    """IIRFilter<Coef, In>  (src/filter/iir/mod.rs:62-414)."""

    def __init__(self, feed_forward, feed_back, iirtype=IIRFilterType.SecondOrder, **kw):
        super().__init__(feed_forward, feed_back, iirtype, 1, **kw)

    @classmethod
    def new(cls, feed_forward, feed_back, iirtype, **kw):
        return cls(feed_forward, feed_back, iirtype, **kw)


class DecimatingIIRFilter(_IirBase):
    """DecimatingIIRFilter<Coef, In>  (src/filter/iir/decim.rs:5-280)."""

    _mode = 1

    def __init__(self, feed_forward, feed_back, iirtype, decimation, **kw):
        super().__init__(feed_forward, feed_back, iirtype, decimation, **kw)

    @classmethod
    def new(cls, feed_forward, feed_back, iirtype, decimation, **kw):  # decim.rs:11-30
        return cls(feed_forward, feed_back, iirtype, decimation, **kw)

    def get_decimation(self):
        return self._factor


class InterpolatingIIRFilter(_IirBase):
    """InterpolatingIIRFilter<Coef, In>  (src/filter/iir/interp.rs:6-268)."""

    _mode = 2

    def __init__(self, feed_forward, feed_back, iirtype, interpolation, **kw):
        super().__init__(feed_forward, feed_back, iirtype, interpolation, **kw)

    @classmethod
    def new(cls, feed_forward, feed_back, iirtype, interpolation, **kw):  # interp.rs:12-31
        return cls(feed_forward, feed_back, iirtype, interpolation, **kw)

    def get_interpolation(self):
        return self._factor


class SecondOrderFilter:
    """SecondOrderFilter<f64, f64>  (src/filter/iir/sos.rs:34-231)."""

    def __init__(self, feed_forward, feed_back, device=0):
        ff = np.ascontiguousarray(feed_forward, dtype=np.float64)
        fb = np.ascontiguousarray(feed_back, dtype=np.float64)
        h = C.c_void_p()
        L.check(L.lib().sdsp_sos_create(C.byref(h), L.dptr(ff) if len(ff) else None, len(ff),
                                        L.dptr(fb) if len(fb) else None, len(fb), device))
        self._f = IIRFilter.__new__(IIRFilter)
        self._f._h = h
        self._f.dtype = L.RR64
        self._f.coef_dtype = np.dtype(np.float64)
        self._f.sample_dtype = np.dtype(np.float64)
        self._f.iirtype = IIRFilterType.SecondOrder
        self._f.channels = 1
        self._f._factor = 1

    @classmethod
    def new(cls, feed_forward, feed_back, coef_dtype=np.float64, sample_dtype=np.float64, **kw):  # sos.rs:55-75
        """SecondOrderFilter::<f64, f64>::new.  The reference is generic
        (`impl<C: Copy + Num + Sum, T: Copy> SecondOrderFilter<C, T>`, sos.rs:41), so other
        instantiations such as <f32, f32> compile there; this binding offers f64 only, and
        f32 / complex-sample SecondOrderFilter parity is not covered."""
        if np.dtype(coef_dtype) != np.float64 or np.dtype(sample_dtype) != np.float64:
            raise NotImplementedError("this binding implements SecondOrderFilter<f64, f64> only "
                                      "(the reference's generic instantiations are not bound)")
        return cls(feed_forward, feed_back, **kw)

    def execute(self, sample: float) -> float:  # sos.rs:92-114 (Left(input))
        return float(self._f.execute(sample)[0])

    def execute_block(self, samples):
        return self._f.execute_block(samples)

    def numerator_coefs(self):  # a[1..]/a0 (swapped name, sos.rs:72)
        return self._f.second_order_filters()[0][0]

    def denominator_coefs(self):  # b/a0 (sos.rs:73)
        return self._f.second_order_filters()[0][1]

    def frequency_response(self, frequency: float) -> complex:  # sos.rs:171-190
        import cmath
        a, b = self.numerator_coefs(), self.denominator_coefs()
        num = sum(c * cmath.rect(1.0, frequency * 2.0 * np.pi * i) for i, c in enumerate(a))
        den = sum(c * cmath.rect(1.0, frequency * 2.0 * np.pi * i) for i, c in enumerate(b))
        return num / den

    def group_delay(self, frequency: float) -> float:  # sos.rs:208-230
        return self._f.group_delay(frequency) - 2.0
