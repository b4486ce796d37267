"""The committed restatement fixtures (tests/golden/vectors_*.npz, written by
tests/golden/make_golden.py) against a fresh run of the oracle: the oracle is
pinned to committed data for the rows the reference's tests do not cover
(PFB, interpolator, channeliser, FFT, full-complex FIR).  CPU only."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden as G  # noqa: E402


def test_every_fixture_family_present():
    kinds = {G.load(n)[0] for n in G.names()}
    assert kinds == {"pfb", "interp", "fir", "fft", "chan"}


@pytest.mark.parametrize("name", G.names())
def test_oracle_reproduces_fixture(name):
    kind, params, arrays = G.load(name)
    fresh = G.vector_cases()[name][2]
    for k, v in arrays.items():
        assert v.dtype == fresh[k].dtype and v.shape == fresh[k].shape, (name, k)
        assert v.tobytes() == fresh[k].tobytes(), (name, k)


def test_fft_fixtures_match_numpy():
    for name in G.names():
        kind, p, a = G.load(name)
        if kind != "fft":
            continue
        ref = np.fft.fft(a["x"]) if p["direction"] == 0 else np.fft.ifft(a["x"]) * p["n"]
        assert np.linalg.norm(a["y"] - ref) / np.linalg.norm(ref) < 1e-7, name
