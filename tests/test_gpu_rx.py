"""MI355X parity of the receive-chain kernels (kern_rx.hip) against the CPU
restatement (oracle/sdsp_oracle_rx.cpp): AutoCorrelator and NCO mixing."""
import math

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

C64, C128 = np.complex64, np.complex128


def _rand(rng, n, dt):
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(dt)


@pytest.mark.parametrize("w,d", [(5, 10), (1, 0), (8, 3), (64, 16), (257, 0), (1500, 7), (2600, 1000), (33, 33)])
@pytest.mark.parametrize("dt", [C128, C64])
def test_acorr_bit_identical_ragged(w, d, dt):
    import solid_dsp_amd as sd
    rng = np.random.default_rng(w * 7 + d)
    x = _rand(rng, 9000, dt)
    g = sd.AutoCorrelator(w, d, dtype=dt)
    o = O.AutoCorr(w, d, dt)
    cuts = [0, 1, 2, 300, 301, 4096, 9000]
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        y = g.execute_block(x[lo:hi])
        r = o.execute_block(x[lo:hi])
        assert y.tobytes() == r.tobytes(), (w, d, lo, hi)
    assert g.execute() == o.execute()
    e, er = g.get_energy(), o.get_energy()
    assert abs(e - er) <= 1e-12 * max(er, 1e-300) + 1e-300, (e, er)


def test_acorr_doctest_and_write_reset():
    import solid_dsp_amd as sd
    xs = np.arange(-250, 250, dtype=np.float64)
    sig = (np.cos(xs) * 0.05 + 1j * (np.sin(xs) * 0.05)).astype(C128)
    g = sd.AutoCorrelator(5, 10)
    y = g.execute_block(sig)
    assert round(g.get_energy() * 10000.0) == 125.0  # auto_correlator/mod.rs:201-211
    assert np.all(y == 0)
    g2 = sd.AutoCorrelator(10, 5)
    o2 = O.AutoCorr(10, 5)
    g2.write(sig[:100])
    o2.write(sig[:100])
    assert g2.execute() == o2.execute()
    g2.push(sig[100])
    o2.write(sig[100:101])
    assert g2.execute() == o2.execute()
    g2.reset()
    assert g2.execute() == 0 and g2.get_energy() == 0.0
    assert str(g2).startswith("AutoCorrelator<f64> [Size=10] [Delay=5]")


def test_acorr_channels_and_device():
    import torch
    import solid_dsp_amd as sd
    rng = np.random.default_rng(11)
    ch, n = 3, 70000
    x = _rand(rng, ch * n, C64).reshape(ch, n)
    g = sd.AutoCorrelator(48, 16, dtype=C64, channels=ch)
    d_in = torch.from_numpy(x).to("cuda")
    d_out = torch.empty_like(d_in)
    g.execute_block_device(d_in, n, d_out, torch.cuda.current_stream())
    torch.cuda.synchronize()
    y = d_out.cpu().numpy()
    for c in range(ch):
        o = O.AutoCorr(48, 16, C64)
        assert y[c].tobytes() == o.execute_block(x[c]).tobytes(), c
    e = g.get_energy()
    ref = [float(np.sum(np.abs(x[c, -48:].astype(C128)) ** 2)) for c in range(ch)]
    assert np.allclose(e, ref, rtol=1e-6)


@pytest.mark.parametrize("w,d,dt", [(64, 16, C64), (130, 120, C64), (64, 16, C128), (9, 0, C64)])
def test_acorr_pipelined_many_tiles(w, d, dt):
    """the persistent pipelined kernel (K, d <= 128): more tiles than resident waves, so every
    wave walks several tiles with the next tile's loads in flight; ragged length, two channels,
    edge tiles on the one-shot kernel -- bit-identical to the restatement"""
    import torch
    import solid_dsp_amd as sd
    rng = np.random.default_rng(w + d)
    ch, n = 2, (1 << 22) + 333
    x = _rand(rng, ch * n, dt).reshape(ch, n)
    g = sd.AutoCorrelator(w, d, dtype=dt, channels=ch)
    d_in = torch.from_numpy(x).to("cuda")
    d_out = torch.empty_like(d_in)
    g.execute_block_device(d_in, n, d_out, torch.cuda.current_stream())
    torch.cuda.synchronize()
    y = d_out.cpu().numpy()
    for c in range(ch):
        o = O.AutoCorr(w, d, dt)
        assert y[c].tobytes() == o.execute_block(x[c]).tobytes(), c


def test_nco_mix_bit_identical_and_state():
    import solid_dsp_amd as sd
    rng = np.random.default_rng(12)
    x = _rand(rng, 50000, C128)
    for down in (False, True):
        g, o = sd.NCO(), O.Nco()
        for f in (g, o):
            f.set_frequency(0.0123)
            f.set_phase(-2.5)
            f.adjust_frequency(1e-3)
            f.adjust_phase(0.25)
        assert g.state() == o.state()
        parts = [(0, 1), (1, 777), (777, 50000)]
        for lo, hi in parts:
            y = g.mix_down_block(x[lo:hi]) if down else g.mix_up_block(x[lo:hi])
            r = o.mix_block(x[lo:hi], down)
            assert y.tobytes() == r.tobytes(), (down, lo, hi)
            assert g.state() == o.state()
        assert g.sincos() == o.sincos()


def test_nco_mix_c32_tolerance_and_pll():
    import solid_dsp_amd as sd
    rng = np.random.default_rng(13)
    x = _rand(rng, 100000, C64)
    g, o = sd.NCO(), O.Nco()
    for f in (g, o):
        f.set_frequency(2 * math.pi * 0.1)
    y = g.mix_up_block(x)
    r = o.mix_block(x.astype(C128))
    rel = np.linalg.norm(y - r) / np.linalg.norm(r)
    assert rel <= 1e-6, rel  # f32 table and product
    with pytest.raises(sd.NCOError):
        g.set_internal_pll_bandwidth(-0.1)
    g.set_internal_pll_bandwidth(0.04)
    assert o.set_pll_bandwidth(0.04) == 0
    g.pll_step(0.3)
    o.pll_step(0.3)
    assert g.state() == o.state()
    assert g.get_frequency() == 0.0 and g.get_phase() == 0.0  # integer-division quirk (nco/mod.rs:69-91)


# ---------------------------------------------------------------- AGC
# The device recurrence calls the gfx950 f64 exp / log / log10 (not glibc's):
# outputs and gains agree with the restatement to a few ulp per step, and the
# loop is contractive, so the bound below holds over thousands of samples.
AGC_RTOL = 1e-12


def _doctest_signal(length=500):
    xs = np.arange(-length // 2, length // 2, dtype=np.float64)
    return (np.cos(xs) * 0.05 + 1j * (np.sin(xs) * 0.05)).astype(C128)


def _agc_pair(bw, squelch=True, timeout=None, channels=1):
    import solid_dsp_amd as sd
    g, o = sd.AGC(channels=channels), O.Agc()
    if squelch:
        g.squelch_enable()
        g.squelch_set_threshold(-30.0)
        o.squelch(1)
        o.squelch_set_threshold(-30.0)
    if timeout is not None:
        g.squelch_set_timeout(timeout)
        o.squelch_set_timeout(timeout)
    g.set_bandwidth(bw)
    o.set_bandwidth(bw)
    return g, o


def _close(y, r):
    return np.max(np.abs(y - r)) <= AGC_RTOL * max(np.max(np.abs(r)), 1e-300)


def test_agc_doctests_on_device():
    """src/auto_gain_control/mod.rs:20-41, :118-135, :157-176, :194-213, :251-271, :550-567"""
    import solid_dsp_amd as sd
    sig = _doctest_signal()
    g, _ = _agc_pair(0.02)
    y = g.execute_block(sig)
    assert 0.98 < abs(y[-1]) < 1.02
    assert -26.0 < g.get_rssi() < -25.5
    g, _ = _agc_pair(0.01)
    y = g.execute_block(sig)
    assert g.get_signal_level() < 0.05 and g.get_gain() > 1.0
    assert len(y) == len(sig) and np.any(y != sig) and y[0] == sig[0]
    g.reset()
    assert g.get_gain() == 1.0 and g.squelch_get_mode() == sd.SquelchMode.ENABLED
    g, _ = _agc_pair(0.01)
    assert g.execute(sig[0]) == sig[0]
    assert g.execute(sig[1]) != sig[1]
    g, _ = _agc_pair(0.01)
    assert 0.04999 < g.init(sig) <= 0.05
    a = sd.AGC()
    assert a.get_bandwidth() == 0.1 and a.get_signal_level() == 1.0 and a.get_rssi() == 0.0
    assert a.get_gain() == 1.0 and a.get_scale() == 1.0 and not a.is_unlocked()
    a.lock()
    assert a.is_unlocked()
    a.unlock()
    a.set_signal_level(10.0)
    assert a.get_signal_level() == 10.0
    a.set_rssi(-20.0)
    assert a.get_rssi() == -20.0
    a.set_gain(2.0)
    a.set_scale(2.0)
    assert a.get_gain() == 2.0 and a.get_scale() == 2.0
    assert str(a).startswith("AGC [Gain=2.00000] [Scale=2.00000]")


def test_agc_errors():
    import solid_dsp_amd as sd
    a = sd.AGC()
    for f, v, code in ((a.set_bandwidth, 1.5, 40), (a.set_bandwidth, -0.01, 40), (a.set_signal_level, 0.0, 41),
                       (a.set_gain, 0.0, 42), (a.set_scale, -1.0, 43)):
        with pytest.raises(sd.AGCError) as e:
            f(v)
        assert e.value.code == code
    with pytest.raises(sd.AGCError) as e:
        a.init(np.zeros(0, C128))
    assert e.value.code == 44


@pytest.mark.parametrize("complex_", [True, False])
def test_agc_vs_restatement_squelch_cycle(complex_):
    """burst, silence past the squelch timeout, second burst: every squelch state,
    ragged block boundaries (not multiples of the 16-sample LDS chunk)"""
    rng = np.random.default_rng(21)
    parts = [0.05 * rng.standard_normal(3000), 1e-9 * np.ones(4000), 0.3 * rng.standard_normal(3000)]
    if complex_:
        parts = [p + 1j * 0.7 * rng.standard_normal(len(p)) * (np.abs(p).mean()) for p in parts]
    x = np.concatenate(parts)
    g, o = _agc_pair(0.05, timeout=37)
    for lo, hi in [(0, 1), (1, 17), (17, 4001), (4001, len(x))]:
        y = g.execute_block(x[lo:hi])
        r = o.execute_block(x[lo:hi])
        assert _close(y, r), (lo, hi)
        assert abs(g.get_gain() - o.get_gain()) <= AGC_RTOL * o.get_gain()
        assert int(g.squelch_get_mode()) == o.get_mode()
        assert g.state().squelch_timer == o.get_timer()


def test_agc_bank_and_device_lock():
    """a 70-channel bank (two 64-lane workgroups, ragged) on device buffers, then locked"""
    import torch
    import solid_dsp_amd as sd
    rng = np.random.default_rng(22)
    ch, n = 70, 2500
    amp = 10.0 ** rng.uniform(-3, 0, ch)
    x = ((rng.standard_normal((ch, n)) + 1j * rng.standard_normal((ch, n))) * amp[:, None]).astype(C128)
    g = sd.AGC(channels=ch)
    g.set_bandwidth(0.02)
    d_in = torch.from_numpy(x).to("cuda")
    d_out = torch.empty_like(d_in)
    g.execute_block_device(d_in, n, d_out, complex_=True, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    y = d_out.cpu().numpy()
    gains = g.get_gain()
    for c in range(ch):
        o = O.Agc()
        o.set_bandwidth(0.02)
        assert _close(y[c], o.execute_block(x[c])), c
        assert abs(gains[c] - o.get_gain()) <= AGC_RTOL * o.get_gain()
    g.lock()
    y2 = g.execute_block(x)
    assert np.array_equal(y2, x * gains[:, None])  # locked: out = input * gain, gain frozen
    assert np.array_equal(g.get_gain(), gains)


def test_agc_long_call_unpipelined_kernel():
    """n >= 2^22 per channel runs agc_kernel (the pipelined kernel's buffer offsets are 32-bit):
    both kernels against the restatement, two channels, n ragged against the chunk"""
    import torch
    import solid_dsp_amd as sd
    rng = np.random.default_rng(23)
    ch, n = 2, (1 << 22) + 5
    x = ((rng.standard_normal((ch, n)) + 1j * rng.standard_normal((ch, n))) * 0.01).astype(C128)
    g = sd.AGC(channels=ch)
    g.set_bandwidth(0.02)
    d_in = torch.from_numpy(x).to("cuda")
    d_out = torch.empty_like(d_in)
    g.execute_block_device(d_in, n, d_out, complex_=True, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    y = d_out.cpu().numpy()
    gains = g.get_gain()
    for c in range(ch):
        o = O.Agc()
        o.set_bandwidth(0.02)
        assert _close(y[c], o.execute_block(x[c])), c
        assert abs(gains[c] - o.get_gain()) <= AGC_RTOL * o.get_gain()


@pytest.mark.parametrize("thr", [-20.0, -20.0 - 1e-12, -20.0 + 1e-12, -19.99999, -20.00001])
def test_agc_squelch_at_threshold(thr):
    """gain pinned exactly at the squelch threshold (x = 0.1, gain 10: E stays 1.0, the
    rssi stays -20): the device's fast threshold test must defer to the reference
    expression there, and agree with it just outside"""
    import solid_dsp_amd as sd
    g, o = sd.AGC(), O.Agc()
    for a in (g, o):
        a.set_rssi(-20.0)
        a.squelch_set_threshold(thr)
        a.squelch_set_timeout(5)
    g.squelch_enable()
    o.squelch(1)
    x = np.full(64, 0.1)
    y, r = g.execute_block(x), o.execute_block(x)
    assert g.get_gain() == o.get_gain() == 10.0
    assert int(g.squelch_get_mode()) == o.get_mode()
    assert y.tobytes() == r.tobytes()


def test_nco_device_unaligned_and_odd():
    """device mixing through 8-byte-aligned (not 16-byte) c32 pointers and odd lengths:
    the kernel's one-sample-per-lane form and the ragged tail"""
    import torch
    import solid_dsp_amd as sd
    rng = np.random.default_rng(14)
    n = 100001
    x = _rand(rng, n + 1, C64)
    d_in = torch.from_numpy(x).to("cuda")
    d_out = torch.zeros_like(d_in)
    for off, m in ((1, n), (0, n), (1, 3)):
        g, o = sd.NCO(), O.Nco()
        for f in (g, o):
            f.set_frequency(0.7)
            f.set_phase(1.1)
        g.mix_block_device(d_in[off:], m, d_out[off:], down=True, precision=0, stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        y = d_out[off:off + m].cpu().numpy()
        r = o.mix_block(x[off:off + m].astype(C128), True)
        assert np.linalg.norm(y - r) / np.linalg.norm(r) <= 1e-6, (off, m)
        assert g.state() == o.state()
