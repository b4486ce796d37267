"""CPU checks of the receive-chain restatement (oracle/sdsp_oracle_rx.cpp):
AutoCorrelator (src/filter/auto_correlator/mod.rs) and NCO (src/nco/mod.rs).

Pinned by the reference's own doctest (energy KAT, auto_correlator/mod.rs:201-211)
and by independent pure-Python restatements of the literal Window / NCO code
(small sizes).  Full-complex outputs beyond those are otherwise unpinned by the
reference's tests (it has no output KAT for execute())."""
import math

import numpy as np

import oracle_lib as O


def _doctest_signal(length=500):
    x = np.arange(-length // 2, length // 2, dtype=np.float64)
    return (np.cos(x) * 0.05 + 1j * (np.sin(x) * 0.05)).astype(np.complex128)


def test_acorr_energy_kat():
    # auto_correlator/mod.rs:201-211: new(5, 10), execute_block(500 samples), energy*1e4 rounds to 125
    a = O.AutoCorr(5, 10)
    y = a.execute_block(_doctest_signal())
    assert round(a.get_energy() * 10000.0) == 125.0
    # delay >= window: the delayed Window's to_vec() reads only its zeroed tail
    assert np.all(y == 0)


class _PyWindow:
    """src/window/mod.rs:17-77 literally: cap + delay slots, push shifts cap - 1."""

    def __init__(self, cap, delay):
        self.cap, self.delay = cap, delay
        self.buf = [0j] * (cap + delay)

    def push(self, x):
        self.buf[1:self.cap] = self.buf[0:self.cap - 1]
        self.buf[0] = x

    def to_vec(self):
        return self.buf[self.delay:self.delay + self.cap]


def _py_acorr(x, w, d):
    win, dwin = _PyWindow(w, 0), _PyWindow(w, d)
    out = []
    for s in x:
        s = complex(s)
        win.push(s)
        dwin.push(s.conjugate())
        acc = 0j
        for a, b in zip(win.to_vec(), dwin.to_vec()):
            # num-complex Mul: (ar br - ai bi, ar bi + ai br), separate roundings
            acc = complex(acc.real + (a.real * b.real - a.imag * b.imag), acc.imag + (a.real * b.imag + a.imag * b.real))
        out.append(acc)
    return np.array(out, dtype=np.complex128)


def test_acorr_matches_literal_python():
    rng = np.random.default_rng(3)
    for w, d in [(8, 3), (5, 0), (1, 0), (6, 6), (4, 9), (16, 1)]:
        x = (rng.standard_normal(150) + 1j * rng.standard_normal(150)).astype(np.complex128)
        a = O.AutoCorr(w, d)
        y = a.execute_block(x)
        assert y.tobytes() == _py_acorr(x, w, d).tobytes(), (w, d)
        # execute() without a push repeats the last output
        assert a.execute() == y[-1]


def test_acorr_energy_running_sum():
    rng = np.random.default_rng(4)
    x = (rng.standard_normal(1000) + 1j * rng.standard_normal(1000)).astype(np.complex128)
    a = O.AutoCorr(32, 4)
    a.write(x[:700])
    a.write(x[700:])
    ref = float(np.sum(np.abs(x[-32:]) ** 2))
    assert abs(a.get_energy() - ref) <= 1e-12 * ref
    a.reset()
    assert a.get_energy() == 0.0


def _py_constrain(theta):
    d = theta / (2.0 * math.pi)
    f = d - math.trunc(d)
    if f < 0.0:
        f += 1.0
    return int(f * float(0xFFFFFFFF)) & 0xFFFFFFFF


def test_nco_constrain_and_table():
    L = O.lib()
    for t in [0.0, math.pi, -math.pi / 2, 0.1, -7.3, 1e3, 2 * math.pi, -1e-20]:
        assert L.orc_nco_constrain(t) == _py_constrain(t), t
    n = O.Nco()
    assert n.sincos() == (0.0, 1.0)  # theta 0: sin table[0], cos table[256]
    n.set_phase(math.pi / 2)
    s, c = n.sincos()
    idx = (((_py_constrain(math.pi / 2) + (1 << 21)) & 0xFFFFFFFF) >> 22) & 0x3FF
    assert s == math.sin(2 * math.pi * idx / 1024) and c == math.sin(2 * math.pi * ((idx + 256) & 0x3FF) / 1024)


def test_nco_mix_block_per_sample():
    rng = np.random.default_rng(5)
    x = (rng.standard_normal(300) + 1j * rng.standard_normal(300)).astype(np.complex128)
    n = O.Nco()
    n.set_frequency(0.0123)
    n.set_phase(-2.5)
    th0, dt = n.state()
    y = n.mix_block(x)
    th = th0
    for i in range(len(x)):
        idx = (((th + (1 << 21)) & 0xFFFFFFFF) >> 22) & 0x3FF
        ph = complex(math.sin(2 * math.pi * ((idx + 256) & 0x3FF) / 1024), math.sin(2 * math.pi * idx / 1024))
        v = complex(x[i])
        ref = complex(ph.real * v.real - ph.imag * v.imag, ph.real * v.imag + ph.imag * v.real)
        assert y[i] == ref
        th = (th + dt) & 0xFFFFFFFF
    assert n.state() == (th, dt)


def test_nco_pll_and_bandwidth():
    n = O.Nco()
    assert n.set_pll_bandwidth(-1.0) == 1  # NCOErrorCode::BandwidthOutOfRange
    assert n.set_pll_bandwidth(0.04) == 0
    n.pll_step(0.3)
    th, dt = n.state()
    assert dt == _py_constrain(0.3 * 0.04) and th == _py_constrain(0.3 * math.sqrt(0.04))


# ---------------------------------------------------------------- AGC
def _agc(bw, squelch=True):
    a = O.Agc()
    if squelch:
        a.squelch(1)
        a.squelch_set_threshold(-30.0)
    assert a.set_bandwidth(bw) == 0
    return a


def test_agc_doctest_kats():
    """The reference's doctests (src/auto_gain_control/mod.rs:20-41, :118-135, :157-176,
    :194-213, :251-271, :550-567)."""
    sig = _doctest_signal()
    a = _agc(0.02)
    y = a.execute_block(sig)
    assert 0.98 < abs(y[-1]) < 1.02
    assert -26.0 < a.get_rssi() < -25.5
    a = _agc(0.01)
    y = a.execute_block(sig)
    assert 1.0 / a.get_gain() < 0.05  # get_signal_level
    assert a.get_gain() > 1.0
    a.reset()
    assert a.get_gain() == 1.0
    assert len(y) == len(sig) and np.any(y != sig) and y[0] == sig[0]
    a = _agc(0.01)
    assert a.execute_block(sig[:1])[0] == sig[0]
    assert a.execute_block(sig[1:2])[0] != sig[1]
    a = _agc(0.01)
    rc, level = a.init(sig)
    assert rc == 0 and 0.04999 < level <= 0.05


def test_agc_setters_and_errors():
    a = O.Agc()
    assert a.get_gain() == 1.0 and a.get_rssi() == 0.0  # -0.0 == 0.0
    a.set_rssi(-20.0)
    assert a.get_rssi() == -20.0
    assert a.set_bandwidth(1.5) == 40 and a.set_bandwidth(-0.1) == 40
    assert a.init(np.zeros(0, np.complex128))[0] == 44
    a.set_rssi(400.0)  # gain clamps at 1e-16
    assert a.get_gain() == 1e-16


def _py_agc(x, bw, thr=None, timeout=100, lock=False, scale=1.0):
    """Literal restatement of execute / update_squelch_mode in Python floats."""
    gain, E, alpha, mode, timer = 1.0, 1.0, bw, ("EN" if thr is not None else "DIS"), 0
    out = []
    for v in x:
        o = v * gain
        ee = (o.conjugate() * o).real
        E = (1.0 - alpha) * E + ee * alpha
        if lock:
            out.append(o)
            continue
        if E > 0.000001:
            gain *= math.exp(-0.5 * alpha * math.log(E))
        gain = min(gain, 1000000.0)
        if mode != "DIS":
            hi = math.log10(gain) * -20.0 > thr
            if mode == "EN":
                mode = "RISE" if hi else "EN"
            elif mode == "RISE":
                mode = "HI" if hi else "FALL"
            elif mode == "HI":
                mode = "HI" if hi else "FALL"
            elif mode == "FALL":
                timer = timeout
                mode = "HI" if hi else "LO"
            elif mode == "LO":
                timer -= 1
                mode = "TO" if timer == 0 else ("HI" if hi else "LO")
            elif mode == "TO":
                mode = "EN"
        out.append(v if mode == "EN" else o * scale)
    return np.array(out), gain, E


def test_agc_matches_literal_python():
    """bit-identical to a literal Python restatement (same libm), squelch cycling
    through every state: a burst, silence past the timeout, a second burst."""
    rng = np.random.default_rng(5)
    x = np.concatenate([0.05 * (rng.standard_normal(300) + 1j * rng.standard_normal(300)),
                        1e-9 * np.ones(400, np.complex128),
                        0.2 * (rng.standard_normal(300) + 1j * rng.standard_normal(300))])
    for thr in (-30.0, None):
        a = _agc(0.05, squelch=thr is not None)
        if thr is not None:
            a.squelch_set_timeout(37)
        y = a.execute_block(x)
        ref, g, e = _py_agc(x, 0.05, thr, timeout=37)
        assert y.tobytes() == ref.astype(np.complex128).tobytes()
        assert a.get_gain() == g and a.get_energy() == e
    a = O.Agc()
    a.lock(1)
    xr = rng.standard_normal(100)
    ref, g, e = _py_agc(xr.astype(np.float64), 0.1, lock=True)
    assert a.execute_block(xr).tobytes() == ref.astype(np.float64).tobytes()
