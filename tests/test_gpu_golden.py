"""Device outputs against the committed restatement fixtures
(tests/golden/vectors_*.npz; parity unpinned by the reference, see
tests/golden/make_golden.py).  Reference-order kernels are bit-identical at the
fixture's precision; FFT and channeliser within their tolerances."""
import os
import sys

import numpy as np
import pytest

from gpu_util import bits_equal, rel_rms

pytestmark = pytest.mark.gpu
sd = pytest.importorskip("solid_dsp_amd")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden as G  # noqa: E402
import oracle_lib as O  # noqa: E402

NAMES = G.names()


@pytest.mark.parametrize("name", [n for n in NAMES if G.load(n)[0] in ("pfb", "interp", "fir")])
def test_filters_bit_identical_to_fixture(name):
    kind, p, a = G.load(name)
    sdt = O._IN_DT[p["dtype"]]
    if kind == "pfb":
        f = sd.PolyPhaseFilterBank(a["taps"], p["M"], a["taps"].dtype.type(p["scale"]), sample_dtype=sdt)
    elif kind == "interp":
        f = sd.InterpolatingFIRFilter(a["taps"], p["M"], sample_dtype=sdt)
    else:
        f = sd.FIRFilter(a["taps"], a["taps"].dtype.type(complex(*p["scale"])), sample_dtype=sdt)
    x, y = a["x"], a["y"]
    h = len(x) // 3  # streamed over two calls
    got = np.concatenate([f.execute_block(x[:h]), f.execute_block(x[h:])])
    assert bits_equal(got, y), name


@pytest.mark.parametrize("name", [n for n in NAMES if n.startswith("fft_")])
@pytest.mark.parametrize("prec", [np.complex64, np.complex128])
def test_fft_matches_fixture(name, prec):
    kind, p, a = G.load(name)
    d = sd.FFTDirection.FORWARD if p["direction"] == 0 else sd.FFTDirection.REVERSE
    y = sd.FFT(p["n"], d, precision=prec).execute(a["x"].astype(prec)[None, :])[0]
    assert rel_rms(y, a["y"]) <= (2e-6 if prec == np.complex64 else 1e-7), name


def test_channeliser_matches_fixture():
    kind, p, a = G.load("chan_m64_k8")
    c = sd.Channelizer(a["taps"].astype(np.float32), p["M"], sample_dtype=np.complex64)
    y = c.execute_block(a["x"].astype(np.complex64)).reshape(-1)
    assert rel_rms(y, a["y"]) <= 1e-6
