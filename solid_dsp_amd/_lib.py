"""Loader for libsdsp.so, the gfx950 C-ABI library (include/sdsp.h).

The library is built in-tree (``solid_dsp_amd/_build/libsdsp.so``) by
``__graft_entry__.build()`` / ``make -C solid_dsp_amd/csrc``.  There is no
pure-Python or CPU fallback: if the library is missing, or no gfx950 device is
visible when a filter is constructed, the call raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "_build", "libsdsp.so")

# sdsp_dtype (Coef, In)
RR32, RC32, CC32, RR64, RC64, CC64 = range(6)
ALGO_AUTO, ALGO_EXACT, ALGO_FMA, ALGO_FFT = range(4)
# sdsp_tune_key values used by the bindings (include/sdsp.h)
TUNE_DECIM_SEG = 6
TUNE_IIR_WAVE_SCAN, TUNE_CHAN_STREAMING, TUNE_CHAN_FRAMES_PER_BLOCK = 7, 8, 9
TUNE_OLS_KERNEL, TUNE_CHAN_XCD_ORDER = 14, 15
TUNE_HOST_STEP, TUNE_HOST_BLOCK_MACS = 16, 17
TUNE_FFT_GROUP, TUNE_FFT_WAVE1024, TUNE_ACORR_KERNEL, TUNE_AGC_KERNEL = 18, 19, 20, 21

_PAIRS = {
    (np.dtype(np.float32), np.dtype(np.float32)): RR32,
    (np.dtype(np.float32), np.dtype(np.complex64)): RC32,
    (np.dtype(np.complex64), np.dtype(np.complex64)): CC32,
    (np.dtype(np.float64), np.dtype(np.float64)): RR64,
    (np.dtype(np.float64), np.dtype(np.complex128)): RC64,
    (np.dtype(np.complex128), np.dtype(np.complex128)): CC64,
}
COEF_DTYPE = {v: k[0] for k, v in _PAIRS.items()}
SAMPLE_DTYPE = {v: k[1] for k, v in _PAIRS.items()}

STATUS = {
    0: "Ok",
    1: "CoefficientsLengthZero", 2: "DecimationLessThanOne", 3: "InterpolationLessThanOne",
    4: "NotEnoughFilters",
    10: "NumeratorLengthZero", 11: "DenominatorLengthZero", 12: "SecondOrderSectionSizeZero",
    13: "SecondOrderSectionSizeMismatch", 14: "SecondOrderSectionSizeNotMultpleOf3",
    15: "DecimationLessThanOne", 16: "InterpolationLessThanOne",
    20: "CoefficientsNotInRange",
    30: "BandwidthOutOfRange",
    40: "BandwidthOutOfRange", 41: "SignalLevelOutOfRange", 42: "GainBelowThreshold", 43: "ScaleBelowThreshold",
    44: "SamplesTooLow",
    90: "InvalidArgument", 91: "Unsupported",
    100: "DeviceError", 101: "NoDevice", 102: "OutOfMemory",
}


class SdspError(RuntimeError):
    """A non-zero sdsp_status.  ``code`` mirrors the reference error enums."""

    def __init__(self, code: int, msg: str = ""):
        self.code = code
        self.name = STATUS.get(code, f"status {code}")
        super().__init__(f"{self.name} ({code}){': ' + msg if msg else ''}")


def dtype_code(coef_dtype, sample_dtype) -> int:
    key = (np.dtype(coef_dtype), np.dtype(sample_dtype))
    if key not in _PAIRS:
        raise TypeError(f"unsupported (Coef, In) pair {key}")
    return _PAIRS[key]


_lib = None


def _declare(L):
    vp, sz, i, d, dp, szp = C.c_void_p, C.c_size_t, C.c_int, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_size_t)
    vpp = C.POINTER(C.c_void_p)
    sig = {
        "sdsp_last_error": (C.c_char_p, []),
        "sdsp_version": (C.c_char_p, []),
        "sdsp_device_count": (i, []),
        "sdsp_sample_size": (sz, [i]),
        "sdsp_coef_size": (sz, [i]),
        "sdsp_fir_create": (i, [vpp, i, vp, sz, vp, i]),
        "sdsp_decim_create": (i, [vpp, i, vp, sz, vp, sz, i]),
        "sdsp_fir_set_channels": (i, [vp, sz]),
        "sdsp_fir_set_algo": (i, [vp, i]),
        "sdsp_fir_get_algo": (i, [vp]),
        "sdsp_set_default_algo": (i, [i]),
        "sdsp_get_default_algo": (i, []),
        "sdsp_fir_set_tuning": (i, [vp, i, i]),
        "sdsp_fir_destroy": (None, [vp]),
        "sdsp_fir_clone": (i, [vp, vpp]),
        "sdsp_fir_set_scale": (i, [vp, vp]),
        "sdsp_fir_get_scale": (i, [vp, vp]),
        "sdsp_fir_len": (sz, [vp]),
        "sdsp_fir_decimation": (sz, [vp]),
        "sdsp_fir_coefficients": (i, [vp, vp]),
        "sdsp_fir_output_count": (sz, [vp, sz]),
        "sdsp_fir_execute": (i, [vp, vp, vp, szp]),
        "sdsp_fir_execute_block": (i, [vp, vp, sz, vp, szp]),
        "sdsp_fir_execute_block_device": (i, [vp, vp, sz, vp, szp, vp]),
        "sdsp_decim_push": (i, [vp, vp]),
        "sdsp_decim_write": (i, [vp, vp, sz]),
        "sdsp_fir_reset": (i, [vp]),
        "sdsp_fir_state_len": (sz, [vp]),
        "sdsp_fir_get_state": (i, [vp, vp, szp]),
        "sdsp_fir_set_state": (i, [vp, vp, sz]),
        "sdsp_fir_frequency_response": (i, [vp, d, dp]),
        "sdsp_fir_group_delay": (i, [vp, d, dp]),
        "sdsp_fir_synchronize": (i, [vp]),
        "sdsp_pfb_create": (i, [vpp, i, vp, sz, sz, vp, i]),
        "sdsp_interp_create": (i, [vpp, i, vp, sz, sz, i]),
        "sdsp_pfb_destroy": (None, [vp]),
        "sdsp_pfb_clone": (i, [vp, vpp]),
        "sdsp_pfb_len": (sz, [vp]),
        "sdsp_pfb_subfilter_len": (sz, [vp]),
        "sdsp_pfb_set_scale": (i, [vp, vp]),
        "sdsp_pfb_get_scale": (i, [vp, vp]),
        "sdsp_pfb_coefficients": (i, [vp, vp]),
        "sdsp_pfb_push": (i, [vp, vp]),
        "sdsp_pfb_execute": (i, [vp, sz, vp]),
        "sdsp_pfb_reset": (i, [vp]),
        "sdsp_pfb_set_algo": (i, [vp, i]),
        "sdsp_iir_wscan_mode": (i, [vp, i]),
        "sdsp_pfb_set_channels": (i, [vp, sz]),
        "sdsp_pfb_execute_block": (i, [vp, vp, sz, vp]),
        "sdsp_pfb_execute_block_device": (i, [vp, vp, sz, vp, vp]),
        "sdsp_pfb_frequency_response": (i, [vp, d, dp]),
        "sdsp_pfb_group_delay": (i, [vp, d, dp]),
        "sdsp_pfb_synchronize": (i, [vp]),
        "sdsp_synth_f32_device": (i, [vp, C.c_uint64, C.c_uint64, C.c_uint64, sz, vp]),
        "sdsp_bandwidth_copy_device": (i, [vp, vp, sz, vp]),
        "sdsp_firdes_kaiser": (i, [sz, d, d, d, dp]),
        "sdsp_firdes_notch": (i, [sz, d, d, dp]),
        "sdsp_kaiser_beta": (d, [d]),
        "sdsp_firdes_estimate_length": (i, [d, d, i, C.POINTER(sz)]),
        "sdsp_firdes_estimate_length_kaiser": (i, [d, d, dp]),
        "sdsp_firdes_estimate_length_herrmann": (i, [d, d, dp]),
        "sdsp_firdes_estimate_stop_band_attenuation": (i, [d, sz, i, dp]),
        "sdsp_firdes_estimate_transition": (i, [d, sz, i, dp]),
        "sdsp_firdes_doppler": (i, [sz, d, d, d, dp]),
        "sdsp_filter_autocorrelation": (d, [dp, sz, C.c_ssize_t]),
        "sdsp_filter_crosscorrelation": (d, [dp, sz, dp, sz, C.c_ssize_t]),
        "sdsp_filter_isi": (i, [dp, sz, sz, sz, dp, dp]),
        "sdsp_filter_energy": (i, [dp, sz, d, sz, dp]),
        "sdsp_active_lag": (i, [d, d, d, dp, dp]),
        "sdsp_active_proportional_integral": (i, [d, d, d, dp, dp]),
        "sdsp_fir_group_delay_taps": (i, [dp, sz, d, dp]),
        "sdsp_iir_group_delay_taps": (i, [dp, sz, dp, sz, d, dp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)  # AttributeError = the .so does not export what include/sdsp.h declares
        f.restype = res
        f.argtypes = args
    # optional families (declared when the library exports them)
    for name, (res, args) in _optional_sigs().items():
        if hasattr(L, name):
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args


def _optional_sigs():
    vp, sz, i, d, dp, szp = C.c_void_p, C.c_size_t, C.c_int, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_size_t)
    vpp = C.POINTER(C.c_void_p)
    return {
        "sdsp_fir_device_ops": (C.c_ulonglong, [C.c_void_p]),  # round 5 (older builds lack it)
        "sdsp_iir_create": (i, [vpp, i, vp, sz, vp, sz, i, i]),
        "sdsp_iir_decim_create": (i, [vpp, i, vp, sz, vp, sz, i, sz, i]),
        "sdsp_iir_interp_create": (i, [vpp, i, vp, sz, vp, sz, i, sz, i]),
        "sdsp_iir_destroy": (None, [vp]),
        "sdsp_iir_clone": (i, [vp, vpp]),
        "sdsp_iir_set_channels": (i, [vp, sz]),
        "sdsp_iir_set_algo": (i, [vp, i]),
        "sdsp_iir_set_tuning": (i, [vp, i, i]),
        "sdsp_chan_set_tuning": (i, [vp, i, i]),
        "sdsp_fft_set_tuning": (i, [vp, i, i]),
        "sdsp_acorr_set_tuning": (i, [vp, i, i]),
        "sdsp_agc_set_tuning": (i, [vp, i, i]),
        "sdsp_iir_output_count": (sz, [vp, sz]),
        "sdsp_iir_execute_block": (i, [vp, vp, sz, vp, szp]),
        "sdsp_iir_execute_block_device": (i, [vp, vp, sz, vp, szp, vp]),
        "sdsp_iir_reset": (i, [vp]),
        "sdsp_iir_state_len": (sz, [vp]),
        "sdsp_iir_get_state": (i, [vp, vp, szp]),
        "sdsp_iir_set_state": (i, [vp, vp, sz]),
        "sdsp_iir_frequency_response": (i, [vp, d, dp]),
        "sdsp_iir_group_delay": (i, [vp, d, dp]),
        "sdsp_iir_coefficients": (i, [vp, dp, dp]),
        "sdsp_iir_num_coefs": (sz, [vp, i]),
        "sdsp_iir_synchronize": (i, [vp]),
        "sdsp_iir_scan_info": (i, [vp, i, C.POINTER(i), C.POINTER(i)]),
        "sdsp_sos_section_coefs": (i, [vp, i, dp, dp]),
        "sdsp_sos_create": (i, [vpp, C.POINTER(C.c_double), sz, C.POINTER(C.c_double), sz, i]),
        "sdsp_chan_create": (i, [vpp, i, vp, sz, sz, i]),
        "sdsp_chan_destroy": (None, [vp]),
        "sdsp_chan_set_streams": (i, [vp, sz]),
        "sdsp_chan_execute_block_device": (i, [vp, vp, sz, vp, szp, vp]),
        "sdsp_chan_execute_block": (i, [vp, vp, sz, vp, szp]),
        "sdsp_chan_reset": (i, [vp]),
        "sdsp_chan_synchronize": (i, [vp]),
        "sdsp_fft_create": (i, [vpp, sz, i, i, i]),
        "sdsp_fft_destroy": (None, [vp]),
        "sdsp_fft_execute": (i, [vp, vp, vp, sz]),
        "sdsp_fft_execute_device": (i, [vp, vp, vp, sz, vp]),
        "sdsp_dot_execute_batched_device": (i, [i, vp, sz, i, vp, sz, sz, sz, vp, vp]),
        "sdsp_fft_len": (sz, [vp]),
        "sdsp_fft_method": (i, [vp]),
        "sdsp_dot_execute": (i, [i, vp, sz, i, vp, sz, vp]),
        # AutoCorrelator / NCO
        "sdsp_acorr_create": (i, [vpp, sz, sz, i, i]),
        "sdsp_acorr_destroy": (None, [vp]),
        "sdsp_acorr_set_channels": (i, [vp, sz]),
        "sdsp_acorr_window_size": (sz, [vp]),
        "sdsp_acorr_delay": (sz, [vp]),
        "sdsp_acorr_reset": (i, [vp]),
        "sdsp_acorr_push": (i, [vp, vp]),
        "sdsp_acorr_write": (i, [vp, vp, sz]),
        "sdsp_acorr_write_device": (i, [vp, vp, sz, vp]),
        "sdsp_acorr_execute": (i, [vp, vp]),
        "sdsp_acorr_execute_block": (i, [vp, vp, sz, vp]),
        "sdsp_acorr_execute_block_device": (i, [vp, vp, sz, vp, vp]),
        "sdsp_acorr_get_energy": (i, [vp, dp]),
        "sdsp_acorr_synchronize": (i, [vp]),
        "sdsp_nco_create": (i, [vpp, i]),
        "sdsp_nco_destroy": (None, [vp]),
        "sdsp_nco_reset": (i, [vp]),
        "sdsp_nco_constrain": (C.c_uint32, [d]),
        "sdsp_nco_set_frequency": (i, [vp, d]),
        "sdsp_nco_adjust_frequency": (i, [vp, d]),
        "sdsp_nco_get_frequency": (d, [vp]),
        "sdsp_nco_set_phase": (i, [vp, d]),
        "sdsp_nco_adjust_phase": (i, [vp, d]),
        "sdsp_nco_get_phase": (d, [vp]),
        "sdsp_nco_step": (i, [vp]),
        "sdsp_nco_sincos": (i, [vp, dp]),
        "sdsp_nco_set_internal_pll_bandwidth": (i, [vp, d]),
        "sdsp_nco_pll_step": (i, [vp, d]),
        "sdsp_nco_get_state": (i, [vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
        "sdsp_nco_set_state": (i, [vp, C.c_uint32, C.c_uint32]),
        "sdsp_nco_mix_block": (i, [vp, i, i, vp, sz, vp]),
        "sdsp_nco_mix_block_device": (i, [vp, i, i, vp, sz, vp, vp]),
        "sdsp_nco_synchronize": (i, [vp]),
        "sdsp_agc_create": (i, [vpp, sz, i]),
        "sdsp_agc_destroy": (None, [vp]),
        "sdsp_agc_channels": (sz, [vp]),
        "sdsp_agc_reset": (i, [vp]),
        "sdsp_agc_execute_block": (i, [vp, i, vp, sz, vp]),
        "sdsp_agc_execute_block_device": (i, [vp, i, vp, sz, vp, vp]),
        "sdsp_agc_init": (i, [vp, i, vp, sz, dp]),
        "sdsp_agc_lock": (i, [vp]),
        "sdsp_agc_unlock": (i, [vp]),
        "sdsp_agc_set_bandwidth": (i, [vp, d]),
        "sdsp_agc_set_signal_level": (i, [vp, d]),
        "sdsp_agc_set_rssi": (i, [vp, d]),
        "sdsp_agc_set_gain": (i, [vp, d]),
        "sdsp_agc_set_scale": (i, [vp, d]),
        "sdsp_agc_update_squelch_mode": (i, [vp]),
        "sdsp_agc_squelch_enable": (i, [vp]),
        "sdsp_agc_squelch_disable": (i, [vp]),
        "sdsp_agc_squelch_set_threshold": (i, [vp, d]),
        "sdsp_agc_squelch_set_timeout": (i, [vp, C.c_uint64]),
        "sdsp_agc_get_state": (i, [vp, sz, C.POINTER(AgcState)]),
        "sdsp_agc_set_state": (i, [vp, sz, C.POINTER(AgcState)]),
        "sdsp_agc_synchronize": (i, [vp]),
    }


class AgcState(C.Structure):
    """sdsp_agc_state (include/sdsp.h) = the fields of struct AGC (src/auto_gain_control/mod.rs:96-108)."""
    _fields_ = [("gain", C.c_double), ("scale", C.c_double), ("bandwidth", C.c_double), ("alpha", C.c_double),
                ("energy_estimate", C.c_double), ("lock", C.c_int32), ("squelch_mode", C.c_int32),
                ("squelch_threshold", C.c_double), ("squelch_timeout", C.c_uint64), ("squelch_timer", C.c_uint64)]


def lib():
    """The loaded libsdsp.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch wheels bundle their own
        # libamdhip64.so (soname libamdhip64.so.7).  Importing torch first makes
        # libsdsp.so bind to that already-loaded runtime, so torch tensors,
        # torch streams and our kernels share one device context.
        try:
            import torch  # noqa: F401
        except ImportError:  # pragma: no cover - torch is plumbing, not required
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C solid_dsp_amd/csrc` (there is no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


def check(rc: int):
    if rc != 0:
        raise SdspError(rc, lib().sdsp_last_error().decode(errors="replace"))


def ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def dptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def device_ptr(t, dtype=None, count=None, device=None, what="buffer") -> int:
    """Raw device pointer of a torch tensor or int (torch is plumbing only).

    For a torch tensor the call checks what the C ABI cannot: that it lives on
    the handle's GPU (``device``), is contiguous, has the sample dtype the handle
    was built for (``dtype``, a numpy dtype) and holds at least ``count``
    elements.  A raw int pointer is passed through unchecked (the caller vouches
    for it, as a Rust caller of the C ABI does)."""
    if isinstance(t, int):
        return t
    if not getattr(t, "is_cuda", False):
        raise ValueError(f"{what}: expected a device (HIP) tensor")
    if device is not None and t.device.index is not None and t.device.index != device:
        raise ValueError(f"{what}: tensor on device {t.device.index}, handle on device {device}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: tensor must be contiguous")
    if dtype is not None:
        want = _torch_dtype(dtype)
        if t.dtype != want:
            raise ValueError(f"{what}: dtype {t.dtype}, handle expects {want}")
    if count is not None and t.numel() < count:
        raise ValueError(f"{what}: {t.numel()} elements, the call needs {count}")
    return int(t.data_ptr())


def _torch_dtype(np_dtype):
    import torch
    return {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
            np.dtype(np.complex64): torch.complex64, np.dtype(np.complex128): torch.complex128}[np.dtype(np_dtype)]


HIP_STREAM_LEGACY = 1  # hipStreamLegacy: the legacy null stream (torch's default stream)


def stream_handle(stream) -> int | None:
    """None -> the handle's own stream; a torch stream (or raw handle) -> that
    stream, with handle 0 (torch's default stream) mapped to hipStreamLegacy
    because NULL means "the handle's stream" in the C ABI."""
    if stream is None:
        return None
    h = stream if isinstance(stream, int) else int(stream.cuda_stream)
    return h if h != 0 else HIP_STREAM_LEGACY
