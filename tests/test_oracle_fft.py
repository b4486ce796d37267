"""The FFT restatement (oracle/sdsp_oracle_fft.cpp) against numpy.fft — the
reference has no FFT tests, so this pins the restatement (parity of the
reference FFT is otherwise unpinned).  Also pins the planner's method choice
(src/fft/mod.rs:125-143) and the channeliser composition against a direct
numpy evaluation of SURVEY Appendix A.6."""
import numpy as np
import pytest

import oracle_lib as O

M_DFT, M_MIXED, M_RADER, M_RADER2 = 0, 1, 2, 3


def offt(x, direction):
    L = O.lib()
    h = L.orc_fft_new(len(x), direction)
    assert h
    y = np.zeros(len(x), np.complex128)
    assert L.orc_fft_execute(h, O._ptr(np.ascontiguousarray(x, np.complex128)), O._ptr(y)) == 0
    m = L.orc_fft_method(h)
    L.orc_fft_free(h)
    return y, m


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15, 16, 17, 18, 19, 24, 31, 32, 64,
                               100, 127, 128, 256, 257, 1000, 1024, 4096])
def test_fft_restatement_vs_numpy(n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    for d in (0, 1):
        y, m = offt(x, d)
        ref = np.fft.fft(x) if d == 0 else np.fft.ifft(x) * n
        err = np.linalg.norm(y - ref) / np.linalg.norm(ref)
        # the reference's DFT16 twiddles are truncated to 8 digits (dft/mod.rs:38-45)
        assert err < (1e-7 if n >= 16 and (n & (n - 1) == 0 or m in (M_RADER, M_RADER2)) else 1e-13), (n, d, err)


def test_planner_methods():
    assert offt(np.ones(16), 0)[1] == M_DFT
    assert offt(np.ones(11), 0)[1] == M_DFT
    assert offt(np.ones(1024), 0)[1] == M_MIXED
    assert offt(np.ones(12), 0)[1] == M_MIXED
    assert offt(np.ones(257), 0)[1] == M_RADER     # prime, 256 = 2^8
    assert offt(np.ones(19), 0)[1] == M_RADER2     # prime, 18 not a power of two


def test_channelizer_restatement():
    rng = np.random.default_rng(4)
    M, K, frames = 16, 4, 6
    h = rng.standard_normal(M * K)
    x = rng.standard_normal(M * frames) + 1j * rng.standard_normal(M * frames)
    y = np.zeros(M * frames, np.complex128)
    L = O.lib()
    got = L.orc_channelize(O._ptr(h), len(h), M, O._ptr(x), len(x), O._ptr(y))
    assert got == frames
    y = y.reshape(frames, M)
    for m in range(frames):
        v = np.array([sum(h[p + (K - 1 - i) * M] * x[(m - i) * M + (M - 1 - p)] for i in range(K) if m - i >= 0)
                      for p in range(M)])
        ref = np.fft.fft(v)
        assert np.linalg.norm(y[m] - ref) <= 1e-7 * np.linalg.norm(ref)
