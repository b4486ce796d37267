"""solid_dsp_amd — MI355X-native streaming FIR / polyphase / IIR engine.

Drop-in for juliantos/solid-dsp's ``filter::*`` / ``dot_product::*`` hot
path.  The compute runs in hand-written gfx950 HIP kernels inside
``_build/libsdsp.so`` (C ABI: ``include/sdsp.h``); this package is a thin
host mirror of the reference's Rust API (module paths, constructor
arguments, error codes).  There is no CPU execution path.
"""
from ._lib import (SdspError, lib, LIB_PATH, RR32, RC32, CC32, RR64, RC64, CC64,  # noqa: F401
                   ALGO_AUTO, ALGO_EXACT, ALGO_FMA, ALGO_FFT)
from . import filter, group_delay, fft, dot_product, channelizer  # noqa: F401
from .fft import FFT, FFTDirection, FFTFlags  # noqa: F401
from .dot_product import DotProduct, Direction  # noqa: F401
from .channelizer import Channelizer  # noqa: F401
from . import nco  # noqa: F401
from .nco import NCO, NCOError  # noqa: F401
from . import auto_gain_control  # noqa: F401
from .auto_gain_control import AGC, AGCError, AGCErrorCode, SquelchMode  # noqa: F401
from .filter.auto_correlator import AutoCorrelator  # noqa: F401
from .filter import (Filter, FIRFilter, DecimatingFIRFilter, PolyPhaseFilterBank,  # noqa: F401
                     InterpolatingFIRFilter, IIRFilter, IIRFilterType, SecondOrderFilter, DecimatingIIRFilter,
                     InterpolatingIIRFilter)

__version__ = "0.1.0"


def device_count() -> int:
    return int(lib().sdsp_device_count())


def set_default_algo(algo: int) -> None:
    """Starting algorithm of handles created from now on (ALGO_EXACT, ALGO_AUTO or ALGO_FMA;
    sdsp_set_default_algo, include/sdsp.h).  Not part of the reference API; the environment
    variable SDSP_DEFAULT_ALGO sets it for a whole process."""
    from ._lib import check
    check(lib().sdsp_set_default_algo(int(algo)))


def get_default_algo() -> int:
    return int(lib().sdsp_get_default_algo())
