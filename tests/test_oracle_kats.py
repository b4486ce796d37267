"""Pin the CPU restatement (oracle/) to every known-answer doctest the
reference holds for the streaming path.  Exact equality on f64,
exactly as the reference's `assert_eq!` does."""
import math

import numpy as np
import pytest

import oracle_lib as O

C64 = np.complex128


def test_msb_index():  # src/resources/mod.rs:11-17
    assert O.lib().orc_msb_index(1) == 1
    assert O.lib().orc_msb_index(129) == 8
    assert O.lib().orc_msb_index(0) == 0


def _dot(kind, coefs, direction, samples):
    out = np.zeros(2)
    c = np.ascontiguousarray(coefs)
    s = np.ascontiguousarray(samples)
    O.lib().orc_dot_execute(kind, O._ptr(c), len(c), direction, O._ptr(s), len(s), O._dptr(out))
    return out


def test_dot_product_reverse_ones():  # src/dot_product/mod.rs:15, execute.rs:15
    r = _dot(0, np.array([1.0, 2, 3, 4, 5]), 1, np.ones(5))
    assert r[0] == 15.0


def test_dot_product_min_len():  # iterations = min(samples.len(), self.len)  mod.rs:161
    r = _dot(0, np.array([1.0, 2, 3, 4, 5]), 0, np.ones(3))
    assert r[0] == 6.0
    r = _dot(0, np.array([1.0, 2, 3]), 0, np.ones(8))
    assert r[0] == 6.0


def test_fir_execute_kat():  # src/filter/fir/mod.rs:200-206
    f = O.fir(O.RC64, [1.0, 2, 3, 4, 5], 1.0)
    y = f.execute_block(np.array([2.02 + 0j]))
    assert y[0] == complex(10.1, 0.0)


def test_fir_execute_block_kat():  # src/filter/fir/mod.rs:226-232
    f = O.fir(O.RC64, [1.0, 2, 3, 4, 5], 1.0)
    x = np.array([2.02, 4.04, 1.02, 0.23, 9.19], dtype=C64)
    y = f.execute_block(x)
    assert y[4] == complex(60.03, 0.0)


def test_fir_frequency_response_kat():  # src/filter/fir/mod.rs:253-261
    h = O.firdes_notch(25, 0.35, 120.0)
    f = O.fir(O.RR64, h, 1.0)
    r = f.frequency_response(0.0)
    assert round(r.real) == 1.0
    assert r.imag == 0.0


def test_fir_group_delay_kat():  # src/filter/fir/mod.rs:284-291
    h = O.firdes_notch(12, 0.35, 120.0)
    f = O.fir(O.RR64, h, 1.0)
    assert int(f.group_delay(0.0) + 0.5) == 12


def test_decim_execute_kat():  # src/filter/fir/decim.rs:213-219
    d = O.decim(O.RC64, [1.0, 2, 3, 4, 5], 1.0, 2)
    assert len(d.execute_block(np.array([2.02 + 0j]))) == 0
    y = d.execute_block(np.array([4.04 + 0j]))
    assert list(y) == [complex(28.28, 0.0)]


def test_decim_execute_block_kat():  # src/filter/fir/decim.rs:242-248
    d = O.decim(O.RC64, [1.0, 2, 3, 4, 5], 1.0, 2)
    y = d.execute_block(np.array([2.02, 4.04, 1.02, 0.23], dtype=C64))
    assert list(y) == [complex(28.28, 0.0), complex(21.39, 0.0)]


def test_decim_push_write_phase():  # decim.rs:115-118, 136-139
    d = O.decim(O.RC64, [1.0, 2, 3, 4, 5], 1.0, 3)
    d.push(1.0)
    d.write(np.array([2.0, 3.0], dtype=C64))   # ci = 3 % 3 = 0, nothing emitted
    y = d.execute_block(np.array([1.0, 1.0, 1.0], dtype=C64))
    # emits after the 3rd input of the block: window (newest first) = 1,1,1,3,2
    assert list(y) == [complex(5 * 1 + 4 * 1 + 3 * 1 + 2 * 3 + 1 * 2, 0)]


ACTIVE_LAG = (0.02, 1.0 / math.sqrt(2.0), 1000.0)


def test_sos_execute_kat():  # src/filter/iir/sos.rs:85-90
    n, d = O.active_lag(*ACTIVE_LAG)
    err = O.C.c_int(0)
    h = O.lib().orc_sos_new(O._dptr(n), 3, O._dptr(d), 3, O.C.byref(err))
    assert O.lib().orc_sos_execute(h, 1.0) == 0.05816769596076701
    O.lib().orc_sos_free(h)


def test_sos_coef_storage_kat():  # src/filter/iir/sos.rs:127-129, 147-149 (swapped names)
    n, d = O.active_lag(*ACTIVE_LAG)
    err = O.C.c_int(0)
    h = O.lib().orc_sos_new(O._dptr(n), 3, O._dptr(d), 3, O.C.byref(err))
    num2, den3 = np.zeros(2), np.zeros(3)
    O.lib().orc_sos_coefs(h, O._dptr(num2), O._dptr(den3))
    assert num2[1] == 0.99999840000128
    assert den3[1] == 0.003199997440002048
    O.lib().orc_sos_free(h)


def test_sos_group_delay_kat():  # src/filter/iir/sos.rs:206
    n, d = O.active_lag(*ACTIVE_LAG)
    err = O.C.c_int(0)
    h = O.lib().orc_sos_new(O._dptr(n), 3, O._dptr(d), 3, O.C.byref(err))
    assert O.lib().orc_sos_group_delay(h, 0.0) == 17.6774211296624
    O.lib().orc_sos_free(h)


def test_iir_second_order_execute_kat():  # src/filter/iir/mod.rs:262-267
    n, d = O.active_lag(*ACTIVE_LAG)
    f = O.iir(O.RR64, n, d, O.SECOND_ORDER)
    assert f.execute_block(np.array([1.0]))[0] == 0.05816769596076701


IIR_BLOCK = [0.05816769596076701, 0.119535296293297, 0.18410279587774706,
             0.2518701895942824, 0.32283747232307686]


def test_iir_second_order_block_kat():  # src/filter/iir/mod.rs:302-307
    n, d = O.active_lag(*ACTIVE_LAG)
    f = O.iir(O.RR64, n, d, O.SECOND_ORDER)
    y = f.execute_block(np.array([1.0, 0, 1, 0, 1]))
    assert list(y) == IIR_BLOCK


def test_iir_second_order_block_complex():  # same KAT through In = Complex<f64> (mod.rs:302 doc uses f64)
    n, d = O.active_lag(*ACTIVE_LAG)
    f = O.iir(O.RC64, n, d, O.SECOND_ORDER)
    y = f.execute_block(np.array([1.0, 0, 1, 0, 1], dtype=C64))
    assert list(y.real) == IIR_BLOCK
    assert not y.imag.any()


def test_iir_freq_response_quirk():  # src/filter/iir/mod.rs:334 — SecondOrder response is 0
    n, d = O.active_lag(*ACTIVE_LAG)
    f = O.iir(O.RR64, n, d, O.SECOND_ORDER)
    assert f.frequency_response(0.0) == 0j


def test_iir_group_delay_kat():  # src/filter/iir/mod.rs:390
    n, d = O.active_lag(*ACTIVE_LAG)
    f = O.iir(O.RR64, n, d, O.SECOND_ORDER)
    assert f.group_delay(0.0) == 19.6774211296624


def test_iir_normal_matches_second_order_for_one_biquad():
    # A single biquad as Normal DF-II runs the same recurrence (mod.rs:272-279 vs sos.rs:92-114).
    n, d = O.active_lag(*ACTIVE_LAG)
    a = O.iir(O.RR64, n, d, O.NORMAL).execute_block(np.array([1.0, 0, 1, 0, 1]))
    assert np.allclose(a, IIR_BLOCK, rtol=1e-14, atol=0)


def test_decim_iir_kat():  # src/filter/iir/decim.rs:215-219
    n, d = O.active_lag(*ACTIVE_LAG)
    f = O.iir_decim(O.RR64, n, d, O.SECOND_ORDER, 2)
    y = f.execute_block(np.array([1.0, 0, 1, 0, 1]))
    assert list(y) == [0.119535296293297, 0.2518701895942824]


def test_interp_iir_kat():  # src/filter/iir/interp.rs:178-181
    n, d = O.active_lag(*ACTIVE_LAG)
    f = O.iir_interp(O.RR64, n, d, O.SECOND_ORDER, 2)
    y = f.execute_block(np.array([1.0]))
    assert list(y) == [0.05816769596076701, 0.119535296293297]


def test_firdes_lengths():  # src/filter/firdes/mod.rs:278-305, 329-368 doctests
    assert len(O.firdes_kaiser(8, 0.35, 120.0, 0.0)) == 8
    assert len(O.firdes_notch(8, 0.35, 120.0)) == 17


def test_estimate_kats():  # src/filter/firdes/mod.rs:64-69, 110-115, 161-166
    L = O.lib()
    out = O.C.c_size_t(0)
    assert L.orc_estimate_req_filter_len(0.35, 100.0, 1, O.C.byref(out)) == 0
    assert out.value == 15
    assert int(L.orc_estimate_req_filter_as(0.35, 16, 1)) == 101
    assert int((L.orc_estimate_req_filter_df(101.0, 16, 1) + 0.005) * 100.0) == 35


def test_firdes_analysis_kats():
    # src/filter/firdes/mod.rs doctests: firdes_doppler :376-387, filter_autocorrelation :431-441,
    # filter_crosscorrelation :470-485, filter_isi :540-550, filter_energy :589-600 (f32 casts as there)
    L = O.lib()
    d = np.zeros(51)
    L.orc_firdes_doppler(51, 0.1, 2.0, 0.0, O._dptr(d))
    assert len(d) == 51 and np.all(np.isfinite(d))
    h = O.firdes_notch(25, 0.2, 30.0)
    ac = L.orc_filter_autocorrelation(O._dptr(h), len(h), 3)
    assert ac == L.orc_filter_autocorrelation(O._dptr(h), len(h), -3)
    assert np.float32(ac) == np.float32(0.047983058)
    k = O.firdes_kaiser(51, 0.35, 120.0, 0.0)
    assert np.float32(L.orc_filter_crosscorrelation(O._dptr(k), len(k), O._dptr(h), len(h), 0)) == \
        np.float32(0.92825377)
    rms, mx = O.C.c_double(0), O.C.c_double(0)
    L.orc_filter_isi(O._dptr(h), len(h), 1, 25, O.C.byref(rms), O.C.byref(mx))
    assert np.float32(rms.value) == np.float32(0.02509764) and np.float32(mx.value) == np.float32(0.061966006)
    e = O.C.c_double(0)
    assert L.orc_filter_energy(O._dptr(h), len(h), 0.35, 128, O.C.byref(e)) == 0
    assert np.float32(e.value) == np.float32(0.3152318)


def test_errors_mirror_reference():
    with pytest.raises(ValueError, match="1"):
        O.fir(O.RR64, [], 1.0)  # CoefficientsLengthZero  fir/mod.rs:80-82
    with pytest.raises(ValueError, match="2"):
        O.decim(O.RR64, [1.0], 1.0, 0)  # DecimationLessThanOne  decim.rs:30-31
    with pytest.raises(ValueError, match="3"):
        O.interp(O.RR64, [1.0], 0)  # InterpolationLessThanOne interp.rs:30-31
    with pytest.raises(ValueError, match="4"):
        O.pfb(O.RR64, [1.0], 0, 1.0)  # NotEnoughFilters pfb.rs:25-26
    with pytest.raises(ValueError, match="13"):
        O.iir(O.RR64, [1.0, 2, 3], [1.0], O.SECOND_ORDER)  # SecondOrderSectionSizeMismatch
    with pytest.raises(ValueError, match="14"):
        O.iir(O.RR64, [1.0, 2], [1.0, 2], O.SECOND_ORDER)


def test_fir_time_reversed_taps_semantics():
    # y[n] = scale * sum_k h[L-1-k] x[n-k]   (DotProduct REVERSE + newest-first Window)
    rng = np.random.default_rng(1)
    h = rng.standard_normal(7)
    x = rng.standard_normal(40)
    y = O.fir(O.RR64, h, 0.5).execute_block(x)
    ref = np.array([sum(h[6 - k] * x[n - k] for k in range(7) if n - k >= 0) for n in range(40)]) * 0.5
    assert np.allclose(y, ref, rtol=1e-13, atol=1e-15)


def test_pfb_semantics():
    # u_p[n] = sum_{i<K} h[p+(K-1-i)M] x[n-i], K = floor(L/M), no scale (pfb.rs:24-90)
    rng = np.random.default_rng(2)
    M, L = 4, 18   # K = 4, tail taps 16,17 dropped
    h = rng.standard_normal(L)
    x = rng.standard_normal(9)
    y = O.pfb(O.RR64, h, M, 3.0).execute_block(x).reshape(-1, M)
    K = L // M
    for n in range(len(x)):
        for p in range(M):
            ref = sum(h[p + (K - 1 - i) * M] * x[n - i] for i in range(K) if n - i >= 0)
            assert abs(y[n, p] - ref) < 1e-12


def test_interp_pads_in_f32():
    # K = ceil_f32(L/M) and h zero-padded to K*M (interp.rs:35-48)
    rng = np.random.default_rng(3)
    h = rng.standard_normal(10)
    y = O.interp(O.RR64, h, 4).execute_block(np.array([1.0, 0, 0, 0]))
    hp = np.concatenate([h, np.zeros(2)])  # K = 3
    K, M = 3, 4
    for n in range(4):
        for p in range(M):
            i = n
            ref = hp[p + (K - 1 - i) * M] if i < K else 0.0
            assert y[n * M + p] == ref


def test_synth_is_f32_exact_uniform():
    x = O.synth(20250226, 0, 0, 4096)
    assert x.dtype == np.float32
    assert x.min() >= -1.0 and x.max() < 1.0
    # values are k / 2^23 exactly
    k = x.astype(np.float64) * 2 ** 23
    assert np.all(k == np.round(k))
    c = O.synth(20250226, 0, 10, 5, complex_=True)
    s = O.synth(20250226, 0, 20, 10)
    assert np.array_equal(c.view(np.float32), s)
