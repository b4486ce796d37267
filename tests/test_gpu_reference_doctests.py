"""The reference's doctests of the hot path (juliantos/solid-dsp src/filter/{fir,iir,firdes}/*.rs,
src/filter/auto_correlator, src/dot_product/*.rs, src/nco, src/auto_gain_control), translated statement by statement by tools/port_doctests.py to the
Python mirror of the C ABI (solid_dsp_amd) and run on the MI355X: every call goes through
libsdsp.so, and each asserted literal is the reference's, compared exactly as Rust's
assert_eq! compares (f64 / Complex<f64> equality).  Generated -- edit the porter, not this file."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sd = pytest.importorskip("solid_dsp_amd")
from solid_dsp_amd import (FIRFilter, DecimatingFIRFilter, InterpolatingFIRFilter, PolyPhaseFilterBank,  # noqa
                           IIRFilter, IIRFilterType, SecondOrderFilter, DecimatingIIRFilter, InterpolatingIIRFilter,
                           DotProduct, Direction, AGC, NCO, AutoCorrelator)
from solid_dsp_amd.filter import firdes, iirdes  # noqa: E402
from solid_dsp_amd.filter.firdes import *  # noqa: E402,F401,F403


def _plain(v):
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, (list, tuple)):
        return [_plain(u) for u in v]
    if isinstance(v, np.generic):
        return v.item()
    return v


def _eq(a, b):
    """assert_eq!: exact equality, element by element for sequences"""
    pa, pb = _plain(a), _plain(b)
    assert pa == pb, (pa, pb)


def _len(x):
    return x.len() if hasattr(x, "len") and callable(x.len) else len(x)


def _round(v):  # f64::round: half away from zero
    return math.floor(v + 0.5) if v >= 0 else -math.floor(-v + 0.5)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_mod_l73(host_step):
    """src/filter/fir/mod.rs:73"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = FIRFilter.new(coefficients, 1.0, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_mod_l96(host_step):
    """src/filter/fir/mod.rs:96"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = FIRFilter.new(coefficients, 1.0, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    filter.set_scale(2.0)
    _eq(filter.get_scale(), 2.0)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_mod_l116(host_step):
    """src/filter/fir/mod.rs:116"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = FIRFilter.new(coefficients, 1.0, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    _eq(filter.get_scale(), 1.0)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_mod_l132(host_step):
    """src/filter/fir/mod.rs:132"""
    coefs = [0.0] * 12
    filter = FIRFilter.new(coefs, 1.0, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    len = _len(filter)
    _eq(len, 12)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_mod_l150(host_step):
    """src/filter/fir/mod.rs:150"""
    coefs = [0.0] * 12
    filter = FIRFilter.new(coefs, 1.0, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    _eq(filter.is_empty(), False)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_mod_l166(host_step):
    """src/filter/fir/mod.rs:166"""
    coefs = [0.0] * 12
    filter = FIRFilter.new(coefs, 1.0, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    ref_coefs = filter.coefficients()
    _eq(coefs, ref_coefs)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_mod_l195(host_step):
    """src/filter/fir/mod.rs:195"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = FIRFilter.new(coefficients, 1.0, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    window = [complex(2.02, 0.0), complex(4.04, 0.0), complex(1.02, 0.0), complex(0.23, 0.0), complex(9.19, 0.0)]
    output = filter.execute(window[0])
    _eq(output[0], complex(10.1, 0.0))


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_mod_l221(host_step):
    """src/filter/fir/mod.rs:221"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = FIRFilter.new(coefficients, 1.0, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    window = [complex(2.02, 0.0), complex(4.04, 0.0), complex(1.02, 0.0), complex(0.23, 0.0), complex(9.19, 0.0)]
    output = filter.execute_block(window)
    _eq(output[4], complex(60.03, 0.0))


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_mod_l247(host_step):
    """src/filter/fir/mod.rs:247"""
    coefs = firdes_notch(25, 0.35, 120.0)
    filter = FIRFilter.new(coefs, 1.0, coef_dtype=np.float64, sample_dtype=np.float64, host_step=host_step)
    response = filter.frequency_response(0.0)
    _eq(_round(response.real), 1.0)
    _eq(response.imag, 0.0)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_mod_l279(host_step):
    """src/filter/fir/mod.rs:279"""
    coefs = firdes.firdes_notch(12, 0.35, 120.0)
    filter = FIRFilter.new(coefs, 1.0, coef_dtype=np.float64, sample_dtype=np.float64, host_step=host_step)
    delay = filter.group_delay(0.0)
    _eq(int(delay + 0.5), 12)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l21(host_step):
    """src/filter/fir/decim.rs:21"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = DecimatingFIRFilter.new(coefficients, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l50(host_step):
    """src/filter/fir/decim.rs:50"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = DecimatingFIRFilter.new(coefficients, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    filter.set_scale(2.0)
    _eq(filter.get_scale(), 2.0)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l70(host_step):
    """src/filter/fir/decim.rs:70"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = DecimatingFIRFilter.new(coefficients, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    _eq(filter.get_scale(), 1.0)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l88(host_step):
    """src/filter/fir/decim.rs:88"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = DecimatingFIRFilter.new(coefficients, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    _eq(filter.get_decimation(), 2)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l106(host_step):
    """src/filter/fir/decim.rs:106"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = DecimatingFIRFilter.new(coefficients, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    filter.push(complex(4.0, 0.0))


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l126(host_step):
    """src/filter/fir/decim.rs:126"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = DecimatingFIRFilter.new(coefficients, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    window = [complex(2.02, 0.0), complex(4.04, 0.0)]
    filter.write(window)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l145(host_step):
    """src/filter/fir/decim.rs:145"""
    coefs = [0.0] * 12
    filter = DecimatingFIRFilter.new(coefs, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    len = _len(filter)
    _eq(len, 12)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l163(host_step):
    """src/filter/fir/decim.rs:163"""
    coefs = [0.0] * 12
    filter = DecimatingFIRFilter.new(coefs, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    _eq(filter.is_empty(), False)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l179(host_step):
    """src/filter/fir/decim.rs:179"""
    coefs = [0.0] * 12
    filter = DecimatingFIRFilter.new(coefs, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    ref_coefs = filter.coefficients()
    _eq(coefs, ref_coefs)


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l208(host_step):
    """src/filter/fir/decim.rs:208"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = DecimatingFIRFilter.new(coefficients, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    window = [complex(2.02, 0.0), complex(4.04, 0.0)]
    first_output = filter.execute(window[0])
    second_output = filter.execute(window[1])
    _eq(first_output, [])
    _eq(second_output, [complex(28.28, 0.0)])


@pytest.mark.parametrize("host_step", [None, False])
def test_filter_fir_decim_l237(host_step):
    """src/filter/fir/decim.rs:237"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = DecimatingFIRFilter.new(coefficients, 1.0, 2, coef_dtype=np.float64, sample_dtype=np.complex128, host_step=host_step)
    window = [complex(2.02, 0.0), complex(4.04, 0.0), complex(1.02, 0.0), complex(0.23, 0.0)]
    output = filter.execute_block(window)
    _eq(output, [complex(28.28, 0.0), complex(21.39, 0.0)])


def test_filter_fir_interp_l21():
    """src/filter/fir/interp.rs:21"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = InterpolatingFIRFilter.new(coefficients, 4, coef_dtype=np.float64, sample_dtype=np.complex128)


def test_filter_fir_pfb_l18():
    """src/filter/fir/pfb.rs:18"""
    coefficients = [1.0, 2.0, 3.0, 4.0, 5.0]
    filter = PolyPhaseFilterBank.new(coefficients, 2, 1.0, coef_dtype=np.float64, sample_dtype=np.complex128)


def test_filter_iir_mod_l84():
    """src/filter/iir/mod.rs:84"""
    filter = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    iir_filter = IIRFilter.new(filter[0], filter[1], IIRFilterType.SecondOrder, coef_dtype=np.float64, sample_dtype=np.complex128)


def test_filter_iir_mod_l170():
    """src/filter/iir/mod.rs:170"""
    filter = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    iir_filter = IIRFilter.new(filter[0], filter[1], IIRFilterType.SecondOrder, coef_dtype=np.float64, sample_dtype=np.float64)
    numerators = iir_filter.numerator_coefs()
    _eq(numerators, filter[0])


def test_filter_iir_mod_l190():
    """src/filter/iir/mod.rs:190"""
    filter = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    iir_filter = IIRFilter.new(filter[0], filter[1], IIRFilterType.SecondOrder, coef_dtype=np.float64, sample_dtype=np.float64)
    denominators = iir_filter.denominator_coefs()
    _eq(denominators, filter[1])


def test_filter_iir_mod_l210():
    """src/filter/iir/mod.rs:210"""
    filter = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    iir_filter = IIRFilter.new(filter[0], filter[1], IIRFilterType.SecondOrder, coef_dtype=np.float64, sample_dtype=np.float64)
    filters = iir_filter.second_order_filters()
    _eq(_len(filters), 1)


def test_filter_iir_mod_l230():
    """src/filter/iir/mod.rs:230"""
    filter = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    iir_filter = IIRFilter.new(filter[0], filter[1], IIRFilterType.SecondOrder, coef_dtype=np.float64, sample_dtype=np.float64)
    _eq(iir_filter.iir_type(), IIRFilterType.SecondOrder)


def test_filter_iir_mod_l257():
    """src/filter/iir/mod.rs:257"""
    filter = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    iir_filter = IIRFilter.new(filter[0], filter[1], IIRFilterType.SecondOrder)
    output = iir_filter.execute(1.0)
    _eq(output[0], 0.05816769596076701)


def test_filter_iir_mod_l297():
    """src/filter/iir/mod.rs:297"""
    filter = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    iir_filter = IIRFilter.new(filter[0], filter[1], IIRFilterType.SecondOrder)
    output = iir_filter.execute_block([1.0, 0.0, 1.0, 0.0, 1.0])
    _eq(output, [0.05816769596076701, 0.119535296293297, 0.18410279587774706, 0.2518701895942824, 0.32283747232307686])


def test_filter_iir_mod_l322():
    """src/filter/iir/mod.rs:322"""
    filter = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    iir_filter = IIRFilter.new(filter[0], filter[1], IIRFilterType.SecondOrder)
    output = iir_filter.execute_block([1.0, 0.0, 1.0, 0.0, 1.0])
    freq_res = iir_filter.frequency_response(0.0)
    _eq(freq_res, complex(0.0, 0.0))


def test_filter_iir_mod_l378():
    """src/filter/iir/mod.rs:378"""
    filter = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    iir_filter = IIRFilter.new(filter[0], filter[1], IIRFilterType.SecondOrder)
    output = iir_filter.execute_block([1.0, 0.0, 1.0, 0.0, 1.0])
    delay = iir_filter.group_delay(0.0)
    _eq(delay, 19.6774211296624)


def test_filter_iir_sos_l48():
    """src/filter/iir/sos.rs:48"""
    ff_coefs, fb_coefs = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    second_order_filter = SecondOrderFilter.new(ff_coefs, fb_coefs, coef_dtype=np.float64, sample_dtype=np.float64)


def test_filter_iir_sos_l81():
    """src/filter/iir/sos.rs:81"""
    ff_coefs, fb_coefs = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    second_order_filter = SecondOrderFilter.new(ff_coefs, fb_coefs, coef_dtype=np.float64, sample_dtype=np.float64)
    output = second_order_filter.execute((1.0))
    _eq(output, 0.05816769596076701)


def test_filter_iir_sos_l120():
    """src/filter/iir/sos.rs:120"""
    ff_coefs, fb_coefs = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    second_order_filter = SecondOrderFilter.new(ff_coefs, fb_coefs, coef_dtype=np.float64, sample_dtype=np.float64)
    numerators = second_order_filter.numerator_coefs()
    _eq(_len(numerators), 2)
    _eq(numerators[1], 0.99999840000128)


def test_filter_iir_sos_l140():
    """src/filter/iir/sos.rs:140"""
    ff_coefs, fb_coefs = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    second_order_filter = SecondOrderFilter.new(ff_coefs, fb_coefs, coef_dtype=np.float64, sample_dtype=np.float64)
    denominators = second_order_filter.denominator_coefs()
    _eq(_len(denominators), 3)
    _eq(denominators[1], 0.003199997440002048)


def test_filter_iir_sos_l160():
    """src/filter/iir/sos.rs:160"""
    ff_coefs, fb_coefs = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    second_order_filter = SecondOrderFilter.new(ff_coefs, fb_coefs, coef_dtype=np.float64, sample_dtype=np.float64)
    freq_res = second_order_filter.frequency_response(0.0)
    assert freq_res != complex(0.0, 0.0)


def test_filter_iir_sos_l197():
    """src/filter/iir/sos.rs:197"""
    ff_coefs, fb_coefs = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    second_order_filter = SecondOrderFilter.new(ff_coefs, fb_coefs, coef_dtype=np.float64, sample_dtype=np.float64)
    delay = second_order_filter.group_delay(0.0)
    _eq(delay, 17.6774211296624)


def test_filter_iir_decim_l21():
    """src/filter/iir/decim.rs:21"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = DecimatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.Normal, 2, coef_dtype=np.float64, sample_dtype=np.complex128)


def test_filter_iir_decim_l53():
    """src/filter/iir/decim.rs:53"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = DecimatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.Normal, 2, coef_dtype=np.float64, sample_dtype=np.complex128)
    _eq(filter.get_decimation(), 2)


def test_filter_iir_decim_l72():
    """src/filter/iir/decim.rs:72"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = DecimatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.Normal, 2, coef_dtype=np.float64, sample_dtype=np.complex128)
    numerators = filter.numerator_coefs()
    orig_ratio = coefficients[0][0] / coefficients[0][1]
    new_ratio = numerators[0] / numerators[1]
    _eq(orig_ratio, new_ratio)


def test_filter_iir_decim_l96():
    """src/filter/iir/decim.rs:96"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = DecimatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.Normal, 2, coef_dtype=np.float64, sample_dtype=np.complex128)
    denominators = filter.denominator_coefs()
    orig_ratio = coefficients[1][0] / coefficients[1][1]
    new_ratio = denominators[1] / denominators[0]
    assert abs(orig_ratio - new_ratio) < 0.00001


def test_filter_iir_decim_l120():
    """src/filter/iir/decim.rs:120"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = DecimatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2, coef_dtype=np.float64, sample_dtype=np.complex128)
    filters = filter.second_order_filters()
    _eq(_len(filters), 1)


def test_filter_iir_decim_l142():
    """src/filter/iir/decim.rs:142"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = DecimatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2, coef_dtype=np.float64, sample_dtype=np.complex128)
    _eq(filter.iir_type(), IIRFilterType.SecondOrder)


def test_filter_iir_decim_l174():
    """src/filter/iir/decim.rs:174"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = DecimatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2)
    output = filter.execute(0.0)
    _eq(output, [])
    output = filter.execute(1.0)
    _eq(output[0], 0.05816769596076701)


def test_filter_iir_decim_l207():
    """src/filter/iir/decim.rs:207"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = DecimatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2)
    output = filter.execute_block([1.0, 0.0, 1.0, 0.0, 1.0])
    _eq(output, [0.119535296293297, 0.2518701895942824])


def test_filter_iir_decim_l239():
    """src/filter/iir/decim.rs:239"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = DecimatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2)
    output = filter.execute_block([1.0, 0.0, 1.0, 0.0, 1.0])
    freq_res = filter.frequency_response(0.0)
    _eq(freq_res, complex(0.0, 0.0))


def test_filter_iir_decim_l262():
    """src/filter/iir/decim.rs:262"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = DecimatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2)
    output = filter.execute_block([1.0, 0.0, 1.0, 0.0, 1.0])
    delay = filter.group_delay(0.0)
    _eq(delay, 19.6774211296624)


def test_filter_iir_interp_l20():
    """src/filter/iir/interp.rs:20"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = InterpolatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.Normal, 2, coef_dtype=np.float64, sample_dtype=np.complex128)


def test_filter_iir_interp_l51():
    """src/filter/iir/interp.rs:51"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = InterpolatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.Normal, 2, coef_dtype=np.float64, sample_dtype=np.complex128)
    _eq(filter.get_interpolation(), 2)


def test_filter_iir_interp_l70():
    """src/filter/iir/interp.rs:70"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = InterpolatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.Normal, 2, coef_dtype=np.float64, sample_dtype=np.complex128)
    numerators = filter.numerator_coefs()
    orig_ratio = coefficients[0][0] / coefficients[0][1]
    new_ratio = numerators[0] / numerators[1]
    _eq(orig_ratio, new_ratio)


def test_filter_iir_interp_l94():
    """src/filter/iir/interp.rs:94"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = InterpolatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.Normal, 2, coef_dtype=np.float64, sample_dtype=np.complex128)
    denominators = filter.denominator_coefs()
    orig_ratio = coefficients[1][0] / coefficients[1][1]
    new_ratio = denominators[1] / denominators[0]
    assert abs(orig_ratio - new_ratio) < 0.00001


def test_filter_iir_interp_l118():
    """src/filter/iir/interp.rs:118"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = InterpolatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2, coef_dtype=np.float64, sample_dtype=np.complex128)
    filters = filter.second_order_filters()
    _eq(_len(filters), 1)


def test_filter_iir_interp_l140():
    """src/filter/iir/interp.rs:140"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = InterpolatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2, coef_dtype=np.float64, sample_dtype=np.complex128)
    _eq(filter.iir_type(), IIRFilterType.SecondOrder)


def test_filter_iir_interp_l170():
    """src/filter/iir/interp.rs:170"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = InterpolatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2)
    output = filter.execute(1.0)
    _eq(output, [0.05816769596076701, 0.119535296293297])


def test_filter_iir_interp_l198():
    """src/filter/iir/interp.rs:198"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    interpolation = 5
    filter = InterpolatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, interpolation)
    input = [1.0, 0.0, 1.0, 0.0, 1.0]
    output = filter.execute_block(input)
    _eq(_len(output), _len(input) * interpolation)


def test_filter_iir_interp_l227():
    """src/filter/iir/interp.rs:227"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = InterpolatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2)
    output = filter.execute_block([1.0, 0.0, 1.0, 0.0, 1.0])
    freq_res = filter.frequency_response(0.0)
    _eq(freq_res, complex(0.0, 0.0))


def test_filter_iir_interp_l250():
    """src/filter/iir/interp.rs:250"""
    coefficients = iirdes.pll.active_lag(0.02, 1.0 / math.sqrt(2.0), 1000.0)
    filter = InterpolatingIIRFilter.new(coefficients[0], coefficients[1], IIRFilterType.SecondOrder, 2)
    output = filter.execute_block([1.0, 0.0, 1.0, 0.0, 1.0])
    delay = filter.group_delay(0.0)
    _eq(delay, 19.6774211296624)


def test_dot_product_mod_l51():
    """src/dot_product/mod.rs:51"""
    coefs = [1.0, 2.0, 3.0, 4.0, 5.0]
    dp = DotProduct.new(coefs, Direction.REVERSE)


def test_dot_product_mod_l93():
    """src/dot_product/mod.rs:93"""
    coefs = [1.0, 2.0, 3.0, 4.0, 5.0]
    dp = DotProduct.new(coefs, Direction.FORWARD)
    ref_coefs = dp.coefficents()
    _eq(coefs, ref_coefs)


def test_dot_product_mod_l115():
    """src/dot_product/mod.rs:115"""
    coefs = [1.0, 2.0, 3.0, 4.0, 5.0]
    dp = DotProduct.new(coefs, Direction.REVERSE)
    _eq(_len(dp), 5)


def test_dot_product_mod_l132():
    """src/dot_product/mod.rs:132"""
    coefs = [1.0, 2.0, 3.0, 4.0, 5.0]
    dp = DotProduct.new(coefs, Direction.REVERSE)
    _eq(dp.is_empty(), False)


def test_dot_product_execute_l7():
    """src/dot_product/execute.rs:7"""
    coefs = [1.0, 2.0, 3.0, 4.0, 5.0]
    dp = DotProduct.new(coefs, Direction.REVERSE)
    mul = [1.0] * 5
    exe = dp.execute(mul)
    _eq(exe, 15.0)


def test_filter_firdes_mod_l61():
    """src/filter/firdes/mod.rs:61"""
    est = estimate_required_filter_length(0.35, 100.0, EstimationMethod.Herrmann)
    _eq(est, 15)


def test_filter_firdes_mod_l107():
    """src/filter/firdes/mod.rs:107"""
    est = estimate_required_filter_stop_band_attenuation(0.35, 16, EstimationMethod.Herrmann)
    _eq(int(est), 101)


def test_filter_firdes_mod_l158():
    """src/filter/firdes/mod.rs:158"""
    est = (lambda est: (est + 0.005) * 100.0)(estimate_required_filter_transition(101.0, 16, EstimationMethod.Herrmann))
    _eq(int(est), 35)


def test_filter_firdes_mod_l268():
    """src/filter/firdes/mod.rs:268"""
    taps = firdes.firdes_kaiser(8, 0.35, 120.0, 0.0)
    _eq(_len(taps), 8)


def test_filter_firdes_mod_l319():
    """src/filter/firdes/mod.rs:319"""
    taps = firdes.firdes_notch(8, 0.35, 120.0)
    _eq(_len(taps), 17)


def test_filter_firdes_mod_l379():
    """src/filter/firdes/mod.rs:379"""
    taps = firdes.firdes_doppler(51, 0.1, 2.0, 0.0)
    _eq(_len(taps), 51)


def test_filter_firdes_mod_l429():
    """src/filter/firdes/mod.rs:429"""
    taps = firdes_notch(25, 0.2, 30.0)
    auto_corr = filter_autocorrelation(taps, 3)
    rev_auto_corr = filter_autocorrelation(taps, -3)
    _eq(auto_corr, rev_auto_corr)
    _eq(np.float32(auto_corr), np.float32(0.047983058))


def test_filter_firdes_mod_l470():
    """src/filter/firdes/mod.rs:470"""
    h = firdes_kaiser(51, 0.35, 120.0, 0.0)
    g = firdes_notch(25, 0.20, 30.0)
    cross_corr = filter_crosscorrelation(h, g, 0)
    _eq(np.float32(cross_corr), np.float32(0.92825377))


def test_filter_firdes_mod_l539():
    """src/filter/firdes/mod.rs:539"""
    h = firdes_notch(25, 0.20, 30.0)
    rms, max = filter_isi(h, 1, 25)
    _eq(np.float32(rms), np.float32(0.02509764))
    _eq(np.float32(max), np.float32(0.061966006))


def test_filter_firdes_mod_l588():
    """src/filter/firdes/mod.rs:588"""
    h = firdes_notch(25, 0.20, 30.0)
    energy = filter_energy(h, 0.35, 128)
    _eq(np.float32(energy), np.float32(0.3152318))


def test_filter_auto_correlator_mod_l7():
    """src/filter/auto_correlator/mod.rs:7"""
    auto_corr_filter = AutoCorrelator(10, 5, dtype=np.complex128)


def test_filter_auto_correlator_mod_l46():
    """src/filter/auto_correlator/mod.rs:46"""
    auto_corr_filter = AutoCorrelator(10, 5, dtype=np.complex128)


def test_filter_auto_correlator_mod_l68():
    """src/filter/auto_correlator/mod.rs:68"""
    auto_corr = AutoCorrelator(10, 5, dtype=np.complex128)
    auto_corr.push(complex(4.0, 0.0))
    auto_corr.reset()


def test_filter_auto_correlator_mod_l92():
    """src/filter/auto_correlator/mod.rs:92"""
    auto_corr = AutoCorrelator(5, 10, dtype=np.complex128)
    auto_corr.push(complex(4.0, 0.0))


def test_filter_auto_correlator_mod_l120():
    """src/filter/auto_correlator/mod.rs:120"""
    auto_corr = AutoCorrelator(5, 10, dtype=np.complex128)
    window = [complex(2.02, 0.0), complex(4.04, 0.0)]
    auto_corr.write(window)


def test_filter_auto_correlator_mod_l143():
    """src/filter/auto_correlator/mod.rs:143"""
    len = 500
    ivec = [math.cos(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    qvec = [math.sin(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    complex_vec = [complex(x, y) for x, y in zip(ivec, qvec)]
    auto_corr = AutoCorrelator(5, 10, dtype=np.complex128)
    auto_corr.write(complex_vec)
    val = auto_corr.execute()


def test_filter_auto_correlator_mod_l169():
    """src/filter/auto_correlator/mod.rs:169"""
    len = 500
    ivec = [math.cos(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    qvec = [math.sin(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    complex_vec = [complex(x, y) for x, y in zip(ivec, qvec)]
    auto_corr = AutoCorrelator(5, 10, dtype=np.complex128)
    output = auto_corr.execute_block(complex_vec)


def test_filter_auto_correlator_mod_l197():
    """src/filter/auto_correlator/mod.rs:197"""
    len = 500
    ivec = [math.cos(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    qvec = [math.sin(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    complex_vec = [complex(x, y) for x, y in zip(ivec, qvec)]
    auto_corr = AutoCorrelator(5, 10, dtype=np.complex128)
    output = auto_corr.execute_block(complex_vec)
    energy = auto_corr.get_energy()
    _eq(_round(energy * 10000.0), 125.0)


def test_auto_gain_control_mod_l20():
    """src/auto_gain_control/mod.rs:20"""
    len = 500
    ivec = [math.cos(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    qvec = [math.sin(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    complex_vec = [complex(x, y) for x, y in zip(ivec, qvec)]
    agc = AGC()
    agc.squelch_enable()
    agc.squelch_set_threshold(-30.0)
    agc.set_bandwidth(0.02)
    agc_vec = agc.execute_block(complex_vec)
    last_item = agc_vec[_len(agc_vec) - 1]
    val = math.sqrt(last_item.real ** 2.0 + last_item.imag ** 2.0)
    assert val > 0.98 and val < 1.02
    assert agc.get_rssi() < -25.5 and agc.get_rssi() > -26.0


def test_auto_gain_control_mod_l118():
    """src/auto_gain_control/mod.rs:118"""
    len = 500
    ivec = [math.cos(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    qvec = [math.sin(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    complex_vec = [complex(x, y) for x, y in zip(ivec, qvec)]
    agc = AGC()
    agc.squelch_enable()
    agc.squelch_set_threshold(-30.0)
    agc.set_bandwidth(0.01)
    agc_vec = agc.execute_block(complex_vec)
    assert agc.get_signal_level() < 0.05


def test_auto_gain_control_mod_l157():
    """src/auto_gain_control/mod.rs:157"""
    len = 500
    ivec = [math.cos(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    qvec = [math.sin(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    complex_vec = [complex(x, y) for x, y in zip(ivec, qvec)]
    agc = AGC()
    agc.squelch_enable()
    agc.squelch_set_threshold(-30.0)
    agc.set_bandwidth(0.01)
    agc_vec = agc.execute_block(complex_vec)
    assert agc.get_gain() > 1.0
    agc.reset()
    assert agc.get_gain() == 1.0


def test_auto_gain_control_mod_l194():
    """src/auto_gain_control/mod.rs:194"""
    len = 500
    ivec = [math.cos(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    qvec = [math.sin(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    complex_vec = [complex(x, y) for x, y in zip(ivec, qvec)]
    agc = AGC()
    agc.squelch_enable()
    agc.squelch_set_threshold(-30.0)
    agc.set_bandwidth(0.01)
    agc_samp_out = agc.execute(complex_vec[0])
    second_samp = agc.execute(complex_vec[1])
    _eq(agc_samp_out, complex_vec[0])
    assert _plain(second_samp) != _plain(complex_vec[1])


def test_auto_gain_control_mod_l252():
    """src/auto_gain_control/mod.rs:252"""
    len = 500
    ivec = [math.cos(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    qvec = [math.sin(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    complex_vec = [complex(x, y) for x, y in zip(ivec, qvec)]
    agc = AGC()
    agc.squelch_enable()
    agc.squelch_set_threshold(-30.0)
    agc.set_bandwidth(0.01)
    agc_vec = agc.execute_block(complex_vec)
    _eq(_len(agc_vec), _len(complex_vec))
    assert _plain(agc_vec) != _plain(complex_vec)
    _eq(agc_vec[0], complex_vec[0])


def test_auto_gain_control_mod_l291():
    """src/auto_gain_control/mod.rs:291"""
    agc = AGC()
    _eq(agc.is_unlocked(), False)
    agc.lock()
    _eq(agc.is_unlocked(), True)
    agc.unlock()
    _eq(agc.is_unlocked(), False)


def test_auto_gain_control_mod_l311():
    """src/auto_gain_control/mod.rs:311"""
    agc = AGC()
    _eq(agc.is_unlocked(), False)
    agc.lock()
    _eq(agc.is_unlocked(), True)
    agc.unlock()
    _eq(agc.is_unlocked(), False)


def test_auto_gain_control_mod_l330():
    """src/auto_gain_control/mod.rs:330"""
    agc = AGC()
    _eq(agc.is_unlocked(), False)
    agc.lock()
    _eq(agc.is_unlocked(), True)
    agc.unlock()
    _eq(agc.is_unlocked(), False)


def test_auto_gain_control_mod_l349():
    """src/auto_gain_control/mod.rs:349"""
    agc = AGC()
    _eq(agc.get_bandwidth(), 0.1)


def test_auto_gain_control_mod_l365():
    """src/auto_gain_control/mod.rs:365"""
    agc = AGC()
    agc.set_bandwidth(0.01)
    _eq(agc.get_bandwidth(), 0.01)


def test_auto_gain_control_mod_l392():
    """src/auto_gain_control/mod.rs:392"""
    agc = AGC()
    _eq(agc.get_signal_level(), 1.0)


def test_auto_gain_control_mod_l408():
    """src/auto_gain_control/mod.rs:408"""
    agc = AGC()
    agc.set_signal_level(10.0)
    _eq(agc.get_signal_level(), 10.0)


def test_auto_gain_control_mod_l434():
    """src/auto_gain_control/mod.rs:434"""
    agc = AGC()
    _eq(agc.get_rssi(), -0.0)


def test_auto_gain_control_mod_l450():
    """src/auto_gain_control/mod.rs:450"""
    agc = AGC()
    agc.set_rssi(-20.0)
    _eq(agc.get_rssi(), -20.0)


def test_auto_gain_control_mod_l472():
    """src/auto_gain_control/mod.rs:472"""
    agc = AGC()
    _eq(agc.get_gain(), 1.0)


def test_auto_gain_control_mod_l488():
    """src/auto_gain_control/mod.rs:488"""
    agc = AGC()
    agc.set_gain(2.0)
    _eq(agc.get_gain(), 2.0)


def test_auto_gain_control_mod_l510():
    """src/auto_gain_control/mod.rs:510"""
    agc = AGC()
    _eq(agc.get_scale(), 1.0)


def test_auto_gain_control_mod_l526():
    """src/auto_gain_control/mod.rs:526"""
    agc = AGC()
    agc.set_scale(2.0)
    _eq(agc.get_scale(), 2.0)


def test_auto_gain_control_mod_l550():
    """src/auto_gain_control/mod.rs:550"""
    len = 500
    ivec = [math.cos(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    qvec = [math.sin(float(x)) * 0.05 for x in range(int(-len / 2), int(len / 2))]
    complex_vec = [complex(x, y) for x, y in zip(ivec, qvec)]
    agc = AGC()
    agc.squelch_enable()
    agc.squelch_set_threshold(-30.0)
    agc.set_bandwidth(0.01)
    signal_level = agc.init(complex_vec)
    assert signal_level > 0.04999 and signal_level <= 0.05
