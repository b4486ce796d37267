"""sdsp_set_default_algo (include/sdsp.h): a process-wide starting algorithm lets an unchanged
reference-API caller reach the fast kernels.  With the default at AUTO, handles built with no
algorithm argument give the same bits as handles explicitly set to the fast path on long blocks,
and the reference-order bits on short ones; the default is restored to EXACT afterwards."""
import numpy as np
import pytest

import oracle_lib as O
from gpu_util import bits_equal

pytestmark = pytest.mark.gpu

sd = pytest.importorskip("solid_dsp_amd")
from solid_dsp_amd import FIRFilter, DecimatingFIRFilter, IIRFilter, IIRFilterType  # noqa: E402


@pytest.fixture
def default_auto():
    old = sd.get_default_algo()
    sd.set_default_algo(sd.ALGO_AUTO)
    try:
        yield
    finally:
        sd.set_default_algo(old)


def _taps(L, fc):
    return np.sinc(2 * fc * (np.arange(L) - (L - 1) / 2)).astype(np.float32) * np.float32(2 * fc)


def test_default_auto_fir_takes_overlap_save(default_auto):
    h = _taps(256, 0.1)
    x = O.synth(21, 0, 0, 1 << 17, complex_=True)
    f = FIRFilter(h, np.float32(0.2), sample_dtype=np.complex64, host_step=False)
    assert sd.lib().sdsp_fir_get_algo(f._h) == sd.ALGO_AUTO
    g = FIRFilter(h, np.float32(0.2), sample_dtype=np.complex64, host_step=False, algo=sd.ALGO_FFT)
    assert bits_equal(f.execute_block(x), g.execute_block(x))  # long block: overlap-save
    # a short block stays on the reference order: a fresh AUTO handle against an EXACT one
    f2 = FIRFilter(h, np.float32(0.2), sample_dtype=np.complex64, host_step=False)
    e = FIRFilter(h, np.float32(0.2), sample_dtype=np.complex64, host_step=False, algo=sd.ALGO_EXACT)
    assert bits_equal(f2.execute_block(x[:4096]), e.execute_block(x[:4096]))


def test_default_auto_decimator_takes_fma(default_auto):
    h = _taps(256, 1.0 / 64)
    x = O.synth(22, 0, 0, 1 << 17, complex_=True)
    d = DecimatingFIRFilter(h, np.float32(1.0 / 32), 32, sample_dtype=np.complex64, host_step=False)
    f = DecimatingFIRFilter(h, np.float32(1.0 / 32), 32, sample_dtype=np.complex64, host_step=False,
                            algo=sd.ALGO_FMA)
    assert bits_equal(d.execute_block(x), f.execute_block(x))
    e = DecimatingFIRFilter(h, np.float32(1.0 / 32), 32, sample_dtype=np.complex64, host_step=False,
                            algo=sd.ALGO_EXACT)
    d2 = DecimatingFIRFilter(h, np.float32(1.0 / 32), 32, sample_dtype=np.complex64, host_step=False)
    assert bits_equal(d2.execute_block(x[:8192]), e.execute_block(x[:8192]))  # short block: reference order


def test_default_auto_iir_takes_scan(default_auto):
    import json
    import os
    sos = np.array(json.load(open(os.path.join(os.path.dirname(__file__), "golden", "butter8_0p2_sos.json")))["sos"])
    b, a = sos[:, :3].reshape(-1).astype(np.float32), sos[:, 3:].reshape(-1).astype(np.float32)
    x = O.synth(23, 0, 0, 1 << 17, complex_=False)
    f = IIRFilter(b, a, IIRFilterType.SecondOrder, sample_dtype=np.float32)
    g = IIRFilter(b, a, IIRFilterType.SecondOrder, sample_dtype=np.float32, algo=sd.ALGO_FMA)
    assert bits_equal(f.execute_block(x), g.execute_block(x))
    assert f.wscan_mode() == g.wscan_mode() != 0


def test_default_back_to_exact():
    assert sd.get_default_algo() == sd.ALGO_EXACT
    h = _taps(64, 0.1)
    x = O.synth(24, 0, 0, 1 << 17, complex_=True)
    f = FIRFilter(h, np.float32(0.2), sample_dtype=np.complex64, host_step=False)
    assert sd.lib().sdsp_fir_get_algo(f._h) == sd.ALGO_EXACT
    assert bits_equal(f.execute_block(x), O.fir(O.RC32, h, np.float32(0.2)).execute_block(x))
