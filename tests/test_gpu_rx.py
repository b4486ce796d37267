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
