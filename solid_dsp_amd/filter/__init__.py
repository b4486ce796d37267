"""``solid::filter`` — the reference's filter trait and its implementors.

``Filter`` mirrors ``trait Filter<I, O>`` (src/filter/mod.rs:9-22):
``execute(sample) -> list``, ``execute_block(samples) -> ndarray``,
``frequency_response(f) -> complex``, ``group_delay(f) -> float``.
"""
from __future__ import annotations

import abc

from . import fir, firdes, iirdes  # noqa: F401


class Filter(abc.ABC):
    """trait Filter<I, O>  (src/filter/mod.rs:9-22)."""

    @abc.abstractmethod
    def execute(self, sample):
        """Filter::execute(&mut self, sample: I) -> Vec<O>  (mod.rs:13)"""

    @abc.abstractmethod
    def execute_block(self, samples):
        """Filter::execute_block(&mut self, &[I]) -> Vec<O>  (mod.rs:17)"""

    @abc.abstractmethod
    def frequency_response(self, frequency: float) -> complex:
        """Filter::frequency_response(&self, f64) -> Complex<f64>  (mod.rs:19)"""

    @abc.abstractmethod
    def group_delay(self, frequency: float) -> float:
        """Filter::group_delay(&self, f64) -> f64  (mod.rs:21)"""


from .fir import FIRFilter, DecimatingFIRFilter, PolyPhaseFilterBank, InterpolatingFIRFilter  # noqa: E402

for _cls in (FIRFilter, DecimatingFIRFilter, InterpolatingFIRFilter):
    Filter.register(_cls)

from . import iir  # noqa: E402,F401
from .iir import (IIRFilter, IIRFilterType, SecondOrderFilter, DecimatingIIRFilter,  # noqa: E402,F401
                  InterpolatingIIRFilter)

for _cls in (IIRFilter, DecimatingIIRFilter, InterpolatingIIRFilter):
    Filter.register(_cls)

from . import auto_correlator  # noqa: E402,F401
from .auto_correlator import AutoCorrelator  # noqa: E402,F401
