"""``solid::filter::fir`` on MI355X.

Mirrors the reference's FIR family (src/filter/fir/{mod,decim,pfb,interp}.rs):
same constructors, argument meaning, error codes (``SdspError.code`` =
FIRErrorCode + 1) and streaming semantics.  All sample processing runs in
libsdsp.so's HIP kernels; this module only marshals host/device buffers.

Type parameters become numpy dtypes: ``FIRFilter(coefs, scale,
sample_dtype=np.complex128)`` is ``FIRFilter::<f64, Complex<f64>>``; the
coefficient dtype is the dtype of ``coefs`` (float32/float64/complex64/
complex128).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import _lib as L


def _coef_array(coefs, coef_dtype):
    a = np.asarray(coefs)
    if coef_dtype is None:
        coef_dtype = a.dtype if a.dtype in (np.float32, np.float64, np.complex64, np.complex128) else np.float64
    return np.ascontiguousarray(a, dtype=coef_dtype)


def _default_sample(coef_dtype):
    return {np.dtype(np.float32): np.complex64, np.dtype(np.float64): np.complex128,
            np.dtype(np.complex64): np.complex64, np.dtype(np.complex128): np.complex128}[np.dtype(coef_dtype)]


class _FirBase:
    _decim = False

    def __init__(self, coefs, scale, decimation=1, sample_dtype=None, coef_dtype=None, device=0, channels=1,
                 algo=None, host_step=None):
        c = _coef_array(coefs, coef_dtype)
        if sample_dtype is None:
            sample_dtype = _default_sample(c.dtype)
        self.dtype = L.dtype_code(c.dtype, sample_dtype)
        self.coef_dtype = L.COEF_DTYPE[self.dtype]
        self.sample_dtype = L.SAMPLE_DTYPE[self.dtype]
        s = np.array([scale], dtype=self.coef_dtype)
        h = C.c_void_p()
        lib = L.lib()
        if self._decim:
            L.check(lib.sdsp_decim_create(C.byref(h), self.dtype, L.ptr(c), len(c), L.ptr(s), decimation, device))
        else:
            L.check(lib.sdsp_fir_create(C.byref(h), self.dtype, L.ptr(c), len(c), L.ptr(s), device))
        self._h = h
        self.device = device
        self.channels = 1
        if channels != 1:
            self.set_channels(channels)
        if algo is not None:  # default: the handle's ALGO_EXACT (bit-identical to the reference)
            self.set_algo(algo)
        if host_step is not None:  # default: the handle's host step (sdsp.h SDSP_TUNE_HOST_STEP)
            self.set_host_step(host_step)

    @classmethod
    def _wrap(cls, handle, dtype, channels, device=0):
        obj = cls.__new__(cls)
        obj._h = handle
        obj.dtype = dtype
        obj.coef_dtype = L.COEF_DTYPE[dtype]
        obj.sample_dtype = L.SAMPLE_DTYPE[dtype]
        obj.channels = channels
        obj.device = device
        return obj

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            L.lib().sdsp_fir_destroy(h)
            self._h = None

    # ---- configuration -------------------------------------------------
    def set_channels(self, channels: int):
        L.check(L.lib().sdsp_fir_set_channels(self._h, channels))
        self.channels = channels

    def set_algo(self, algo: int):
        L.check(L.lib().sdsp_fir_set_algo(self._h, algo))

    def set_tuning(self, key: int, value: int):
        """kernel-variant knobs (SDSP_TUNE_*, include/sdsp.h): performance only"""
        L.check(L.lib().sdsp_fir_set_tuning(self._h, int(key), int(value)))

    def set_host_step(self, on: bool, block_macs: int = None):
        """execute(sample), push and host blocks of n * len <= block_macs multiply-adds on the host
        against the handle's delay line (True, the default) or as device launches (False)."""
        L.check(L.lib().sdsp_fir_set_tuning(self._h, L.TUNE_HOST_STEP, 1 if on else 0))
        if block_macs is not None:
            L.check(L.lib().sdsp_fir_set_tuning(self._h, L.TUNE_HOST_BLOCK_MACS, int(block_macs)))

    def set_scale(self, scale):  # fir/mod.rs:103-106
        s = np.array([scale], dtype=self.coef_dtype)
        L.check(L.lib().sdsp_fir_set_scale(self._h, L.ptr(s)))

    def get_scale(self):  # fir/mod.rs:121-124
        s = np.zeros(1, dtype=self.coef_dtype)
        L.check(L.lib().sdsp_fir_get_scale(self._h, L.ptr(s)))
        return s[0]

    def len(self) -> int:  # fir/mod.rs:139-142
        return int(L.lib().sdsp_fir_len(self._h))

    def __len__(self):
        return self.len()

    def is_empty(self) -> bool:
        return self.len() == 0

    def coefficients(self) -> np.ndarray:
        """The stored (reversed) taps, as DotProduct::coefficents (fir/mod.rs:173-176)."""
        out = np.zeros(self.len(), dtype=self.coef_dtype)
        L.check(L.lib().sdsp_fir_coefficients(self._h, L.ptr(out)))
        return out

    def clone(self):
        h = C.c_void_p()
        L.check(L.lib().sdsp_fir_clone(self._h, C.byref(h)))
        return type(self)._wrap(h, self.dtype, self.channels, self.device)

    __copy__ = clone

    def reset(self):
        L.check(L.lib().sdsp_fir_reset(self._h))

    def get_state(self):
        n = int(L.lib().sdsp_fir_state_len(self._h))
        hist = np.zeros(n, dtype=self.sample_dtype)
        phase = C.c_size_t(0)
        L.check(L.lib().sdsp_fir_get_state(self._h, L.ptr(hist), C.byref(phase)))
        return hist, phase.value

    def set_state(self, hist, phase=0):
        hist = np.ascontiguousarray(hist, dtype=self.sample_dtype)
        L.check(L.lib().sdsp_fir_set_state(self._h, L.ptr(hist), phase))

    # ---- Filter trait ----------------------------------------------------
    def output_count(self, n: int) -> int:
        return int(L.lib().sdsp_fir_output_count(self._h, n))

    def execute(self, sample) -> list:
        """Filter::execute — one input, returns a list of 0 or 1 outputs."""
        x = np.array([sample], dtype=self.sample_dtype)
        y = np.zeros(1, dtype=self.sample_dtype)
        n = C.c_size_t(0)
        L.check(L.lib().sdsp_fir_execute(self._h, L.ptr(x), L.ptr(y), C.byref(n)))
        return list(y[: n.value])

    def execute_block(self, samples) -> np.ndarray:
        """Filter::execute_block over host samples (channel-major [channels, n] when channels > 1)."""
        x = np.ascontiguousarray(samples, dtype=self.sample_dtype)
        n = x.shape[-1] if x.ndim else 0
        if self.channels > 1 and (x.ndim != 2 or x.shape[0] != self.channels):
            raise ValueError("multi-channel input must be [channels, n]")
        nout = self.output_count(n)
        y = np.zeros((self.channels, max(nout, 0)), dtype=self.sample_dtype) if self.channels > 1 else \
            np.zeros(nout, dtype=self.sample_dtype)
        got = C.c_size_t(0)
        L.check(L.lib().sdsp_fir_execute_block(self._h, L.ptr(x), n, L.ptr(y) if y.size else None, C.byref(got)))
        return y

    def execute_block_device(self, d_in, n: int, d_out, stream=None) -> int:
        """Device-resident execute_block: d_in/d_out are torch tensors or raw device pointers
        (channel-major, n samples per channel in, output_count(n) per channel out)."""
        got = C.c_size_t(0)
        pin = L.device_ptr(d_in, self.sample_dtype, self.channels * n, self.device, "input")
        pout = L.device_ptr(d_out, self.sample_dtype, self.channels * self.output_count(n), self.device, "output")
        L.check(L.lib().sdsp_fir_execute_block_device(self._h, pin, n, pout, C.byref(got), L.stream_handle(stream)))
        return got.value

    def synchronize(self):
        L.check(L.lib().sdsp_fir_synchronize(self._h))

    def frequency_response(self, frequency: float) -> complex:
        out = np.zeros(2)
        L.check(L.lib().sdsp_fir_frequency_response(self._h, frequency, L.dptr(out)))
        return complex(out[0], out[1])

    def group_delay(self, frequency: float) -> float:
        out = np.zeros(1)
        L.check(L.lib().sdsp_fir_group_delay(self._h, frequency, L.dptr(out)))
        return float(out[0])


class FIRFilter(_FirBase):
    """FIRFilter<Coef, In>  (src/filter/fir/mod.rs:58-304).

    ``FIRFilter(coefs, scale)`` = ``FIRFilter::new(&coefs, scale)`` (:79-88).
    """

    def __init__(self, coefs, scale=1.0, sample_dtype=None, coef_dtype=None, device=0, channels=1,
                 algo=None, host_step=None):
        super().__init__(coefs, scale, 1, sample_dtype, coef_dtype, device, channels, algo, host_step)

    @classmethod
    def new(cls, coefs, scale, **kw):
        return cls(coefs, scale, **kw)


class DecimatingFIRFilter(_FirBase):
    """DecimatingFIRFilter<Coef, In>  (src/filter/fir/decim.rs:5-281)."""

    _decim = True

    def __init__(self, coefs, scale=1.0, decimation=1, sample_dtype=None, coef_dtype=None, device=0,
                 channels=1, algo=None, host_step=None):
        super().__init__(coefs, scale, decimation, sample_dtype, coef_dtype, device, channels, algo, host_step)

    @classmethod
    def new(cls, coefs, scale, decimation, **kw):
        return cls(coefs, scale, decimation, **kw)

    def get_decimation(self) -> int:  # decim.rs:92-95
        return int(L.lib().sdsp_fir_decimation(self._h))

    def push(self, sample):  # decim.rs:115-118
        x = np.array([sample], dtype=self.sample_dtype)
        L.check(L.lib().sdsp_decim_push(self._h, L.ptr(x)))

    def write(self, samples):  # decim.rs:136-139
        x = np.ascontiguousarray(samples, dtype=self.sample_dtype)
        L.check(L.lib().sdsp_decim_write(self._h, L.ptr(x), x.shape[-1]))


class PolyPhaseFilterBank:
    """PolyPhaseFilterBank<Coef, In>  (src/filter/fir/pfb.rs:3-91)."""

    def __init__(self, coefs, filters, scale=1.0, sample_dtype=None, coef_dtype=None, device=0, _interp=None,
                 algo=None, channels=1):
        c = _coef_array(coefs, coef_dtype)
        if sample_dtype is None:
            sample_dtype = _default_sample(c.dtype)
        self.dtype = L.dtype_code(c.dtype, sample_dtype)
        self.coef_dtype = L.COEF_DTYPE[self.dtype]
        self.sample_dtype = L.SAMPLE_DTYPE[self.dtype]
        h = C.c_void_p()
        if _interp is None:
            s = np.array([scale], dtype=self.coef_dtype)
            L.check(L.lib().sdsp_pfb_create(C.byref(h), self.dtype, L.ptr(c), len(c), filters, L.ptr(s), device))
        else:
            L.check(L.lib().sdsp_interp_create(C.byref(h), self.dtype, L.ptr(c), len(c), _interp, device))
        self._h = h
        self.device = device
        self.channels = channels
        if algo is not None:
            L.check(L.lib().sdsp_pfb_set_algo(self._h, algo))
        if channels != 1:
            L.check(L.lib().sdsp_pfb_set_channels(self._h, channels))

    @classmethod
    def new(cls, coefs, filters, scale, **kw):
        return cls(coefs, filters, scale, **kw)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            L.lib().sdsp_pfb_destroy(h)
            self._h = None

    def clone(self):
        h = C.c_void_p()
        L.check(L.lib().sdsp_pfb_clone(self._h, C.byref(h)))
        obj = type(self).__new__(type(self))
        obj.__dict__.update({k: v for k, v in self.__dict__.items() if k != "_h"})
        obj._h = h
        return obj

    def set_scale(self, scale):  # pfb.rs:56-59
        s = np.array([scale], dtype=self.coef_dtype)
        L.check(L.lib().sdsp_pfb_set_scale(self._h, L.ptr(s)))

    def get_scale(self):
        s = np.zeros(1, dtype=self.coef_dtype)
        L.check(L.lib().sdsp_pfb_get_scale(self._h, L.ptr(s)))
        return s[0]

    def len(self) -> int:  # number of filters (pfb.rs:66-69)
        return int(L.lib().sdsp_pfb_len(self._h))

    def __len__(self):
        return self.len()

    def is_empty(self):
        return self.len() == 0

    def subfilter_len(self) -> int:
        return int(L.lib().sdsp_pfb_subfilter_len(self._h))

    def coefficents(self) -> np.ndarray:  # sic, pfb.rs:72-75
        out = np.zeros((self.len(), self.subfilter_len()), dtype=self.coef_dtype)
        L.check(L.lib().sdsp_pfb_coefficients(self._h, L.ptr(out)))
        return out

    coefficients = coefficents

    def reset(self):  # pfb.rs:77-79
        L.check(L.lib().sdsp_pfb_reset(self._h))

    def push(self, sample):  # pfb.rs:81-83
        x = np.array([sample], dtype=self.sample_dtype)
        L.check(L.lib().sdsp_pfb_push(self._h, L.ptr(x)))

    def execute(self, index: int):  # pfb.rs:85-90
        out = np.zeros(1, dtype=self.sample_dtype)
        L.check(L.lib().sdsp_pfb_execute(self._h, index, L.ptr(out)))
        return out[0]

    def execute_block(self, samples) -> np.ndarray:
        """push each sample then emit all M branch outputs (out[n*M + p]); channel-major
        [channels, n] -> [channels, n*M] when channels > 1."""
        x = np.ascontiguousarray(samples, dtype=self.sample_dtype)
        if self.channels > 1 and (x.ndim != 2 or x.shape[0] != self.channels):
            raise ValueError("multi-channel input must be [channels, n]")
        n = x.shape[-1]
        y = np.zeros((self.channels, n * self.len()) if self.channels > 1 else n * self.len(), dtype=self.sample_dtype)
        if n:
            L.check(L.lib().sdsp_pfb_execute_block(self._h, L.ptr(x), n, L.ptr(y)))
        return y

    def execute_block_device(self, d_in, n: int, d_out, stream=None):
        """n inputs per channel ([channels][n] in, [channels][n*M] out), device resident."""
        pin = L.device_ptr(d_in, self.sample_dtype, self.channels * n, self.device, "input")
        pout = L.device_ptr(d_out, self.sample_dtype, self.channels * n * self.len(), self.device, "output")
        L.check(L.lib().sdsp_pfb_execute_block_device(self._h, pin, n, pout, L.stream_handle(stream)))
        return n * self.len()

    def synchronize(self):
        L.check(L.lib().sdsp_pfb_synchronize(self._h))


class InterpolatingFIRFilter(PolyPhaseFilterBank):
    """InterpolatingFIRFilter<Coef, In>  (src/filter/fir/interp.rs:6-138)."""

    def __init__(self, coefs, interpolation, sample_dtype=None, coef_dtype=None, device=0, algo=None, channels=1):
        super().__init__(coefs, interpolation, 1.0, sample_dtype, coef_dtype, device, _interp=interpolation,
                         algo=algo, channels=channels)
        self._interpolation = interpolation

    @classmethod
    def new(cls, coefs, interpolation, **kw):
        return cls(coefs, interpolation, **kw)

    def interpolation(self) -> int:  # interp.rs:84-87
        return self._interpolation

    def coefficents(self) -> np.ndarray:  # flattened branches (interp.rs:77-80)
        return super().coefficents().reshape(-1)

    coefficients = coefficents

    def execute(self, sample) -> list:  # interp.rs:93-100
        return list(self.execute_block(np.array([sample], dtype=self.sample_dtype)))

    def frequency_response(self, frequency: float) -> complex:  # interp.rs:113-124
        out = np.zeros(2)
        L.check(L.lib().sdsp_pfb_frequency_response(self._h, frequency, L.dptr(out)))
        return complex(out[0], out[1])

    def group_delay(self, frequency: float) -> float:  # interp.rs:126-137
        out = np.zeros(1)
        L.check(L.lib().sdsp_pfb_group_delay(self._h, frequency, L.dptr(out)))
        return float(out[0])
