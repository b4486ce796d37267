"""GPU FFT, channeliser and DotProduct parity against the CPU restatement."""
import numpy as np
import pytest

import oracle_lib as O
from gpu_util import bits_equal, rel_rms, to_dev, empty_dev, to_host

pytestmark = pytest.mark.gpu

sd = pytest.importorskip("solid_dsp_amd")
from solid_dsp_amd import FFT, FFTDirection, DotProduct, Direction, Channelizer  # noqa: E402


def offt(x, d):
    L = O.lib()
    h = L.orc_fft_new(len(x), d)
    y = np.zeros(len(x), np.complex128)
    L.orc_fft_execute(h, O._ptr(np.ascontiguousarray(x, np.complex128)), O._ptr(y))
    L.orc_fft_free(h)
    return y


@pytest.mark.parametrize("n", [1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 3, 5, 12, 100, 257, 1000])
@pytest.mark.parametrize("prec", [np.complex64, np.complex128])
def test_fft_vs_restatement(n, prec):
    rng = np.random.default_rng(n)
    batch = 3
    x = (rng.standard_normal((batch, n)) + 1j * rng.standard_normal((batch, n))).astype(prec)
    for d in (FFTDirection.FORWARD, FFTDirection.REVERSE):
        y = FFT(n, d, precision=prec).execute(x)
        for b in range(batch):
            ref = offt(x[b].astype(np.complex128), int(d))
            # f32: single-precision FFT; f64: bounded by the reference's own 8-digit DFT16 twiddles
            tol = 2e-6 if prec == np.complex64 else 1e-7
            assert rel_rms(y[b], ref) <= tol, (n, d, rel_rms(y[b], ref))


@pytest.mark.parametrize("n,method", [(8192, "four-step"), (65536, "four-step"), (1 << 20, "four-step"),
                                      (513, "Bluestein"), (1000, "Bluestein"), (500, "direct DFT"), (4097, "Bluestein"),
                                      (10007, "Bluestein"), (3 * 5 * 7 * 11 * 13, "Bluestein"),
                                      (100003, "Bluestein")])
@pytest.mark.parametrize("prec", [np.complex64, np.complex128])
def test_fft_large_and_any_size(n, method, prec):
    """General sizes: four-step powers of two and Bluestein, both
    directions, batched and in place, vs numpy (f64) and, up to 2^16, the restated
    reference planner (whose DFT16 constants bound the f64 agreement near 1e-7)."""
    import torch
    rng = np.random.default_rng(n)
    batch = 2 if n <= 1 << 16 else 1
    x = (rng.standard_normal((batch, n)) + 1j * rng.standard_normal((batch, n))).astype(prec)
    for d in (FFTDirection.FORWARD, FFTDirection.REVERSE):
        f = FFT(n, d, precision=prec)
        assert f.method == method
        y = f.execute(x)
        xs = x.astype(np.complex128)
        ref = np.fft.fft(xs, axis=-1) if d == FFTDirection.FORWARD else np.fft.ifft(xs, axis=-1) * n
        tol = 5e-6 if prec == np.complex64 else 1e-12
        assert rel_rms(y, ref) <= tol, (n, d, rel_rms(y, ref))
        if n <= 1 << 16:
            assert rel_rms(y[0], offt(xs[0], int(d))) <= (5e-6 if prec == np.complex64 else 1e-7)
        # device, in place
        t = torch.from_numpy(x.copy()).to("cuda")
        f.execute_device(t, t, batch, torch.cuda.current_stream())
        torch.cuda.synchronize()
        assert rel_rms(t.cpu().numpy(), y) <= (1e-6 if prec == np.complex64 else 1e-14)


@pytest.mark.parametrize("d", [FFTDirection.FORWARD, FFTDirection.REVERSE])
def test_fft_2p20_column_pass_lane_forms_agree(d):
    """The 2^20-point column pass loads its strided side in 16-byte lanes when the input is
    16-byte aligned and in 8-byte lanes otherwise (kern_chan1024.hip, fft1024_pipe_body
    LA & 16): the same arithmetic, so the two must agree bit for bit, and with numpy."""
    import torch
    n, batch = 1 << 20, 2
    rng = np.random.default_rng(7)
    x = (rng.standard_normal((batch, n)) + 1j * rng.standard_normal((batch, n))).astype(np.complex64)
    f = FFT(n, d, precision=np.complex64)
    st = torch.cuda.current_stream()
    a = torch.from_numpy(x.reshape(-1)).to("cuda")
    ya = torch.empty_like(a)
    f.execute_device(a, ya, batch, st)
    b = torch.empty(batch * n + 1, dtype=torch.complex64, device="cuda")[1:]  # 8 bytes past alignment
    assert b.data_ptr() % 16 == 8
    b.copy_(a)
    yb = torch.empty_like(a)
    f.execute_device(b, yb, batch, st)
    torch.cuda.synchronize()
    ya, yb = ya.cpu().numpy(), yb.cpu().numpy()
    assert bits_equal(ya, yb)
    xs = x.astype(np.complex128)
    ref = np.fft.fft(xs, axis=-1) if d == FFTDirection.FORWARD else np.fft.ifft(xs, axis=-1) * n
    assert rel_rms(ya.reshape(batch, n), ref) <= 5e-6


def test_fft_errors():
    with pytest.raises(sd.SdspError):
        FFT(0)


@pytest.mark.parametrize("M,K", [(16, 4), (64, 8), (1024, 8)])
def test_channelizer_vs_restatement(M, K):
    rng = np.random.default_rng(M + K)
    h = O.firdes_kaiser(M * K, 0.5 / M, 80.0, 0.0).astype(np.float32)
    frames = 12
    x = O.synth(20250226, 1, 0, M * frames, complex_=True)
    ch = Channelizer(h, M, sample_dtype=np.complex64)
    y = np.concatenate([ch.execute_block(x[: 5 * M]), ch.execute_block(x[5 * M:])])
    ref = np.zeros(M * frames, np.complex128)
    O.lib().orc_channelize(O._ptr(h.astype(np.float64)), len(h), M, O._ptr(x.astype(np.complex128)), len(x),
                           O._ptr(ref))
    ref = ref.reshape(frames, M)
    assert rel_rms(y, ref) <= 1e-6
    assert np.abs(y - ref).max() <= 1e-6 * np.abs(h).sum() * np.abs(x).max() * np.sqrt(M)


def test_channelizer_multistream_device():
    import torch
    M, K, frames, S = 64, 8, 20, 3
    h = O.firdes_kaiser(M * K, 0.5 / M, 80.0, 0.0)
    x = np.stack([O.synth(9, s, 0, M * frames, complex_=True).astype(np.complex128) for s in range(S)])
    ch = Channelizer(h, M, sample_dtype=np.complex128, streams=S)
    d_in = to_dev(x.reshape(-1))
    d_out = empty_dev(S * M * frames, np.complex128)
    assert ch.execute_block_device(d_in, M * frames, d_out, torch.cuda.current_stream()) == frames
    y = to_host(d_out).reshape(S, frames, M)
    for s in range(S):
        ref = np.zeros(M * frames, np.complex128)
        O.lib().orc_channelize(O._ptr(h), len(h), M, O._ptr(x[s]), M * frames, O._ptr(ref))
        assert rel_rms(y[s], ref.reshape(frames, M)) <= 1e-7


@pytest.mark.parametrize("variant,fpb", [(0, 0), (1, 16), (1, 0), (2, 8), (2, 48), (3, 16), (3, 0), (4, 8), (4, 48),
                                         (5, 8), (5, 0), (6, 8), (6, 0)])
@pytest.mark.parametrize("K", [3, 8])
@pytest.mark.parametrize("xcd", [0, 1])
def test_channelizer_1024_streaming_variants(variant, fpb, K, xcd):
    """the streaming M=1024 kernels (1024- and 512-thread workgroups, SDSP_TUNE_CHAN_STREAMING
    1-4; 5 / 6: eight / four frames per round) and the per-frame kernel (0) against the restatement: several streams, workgroup
    boundaries inside a block (warm-up frames), a ragged last round, two blocks (history),
    launch-order and XCD-ordered chunk maps"""
    import torch
    M, S, frames = 1024, 4, 75
    h = O.firdes_kaiser(M * K, 0.5 / M, 80.0, 0.0).astype(np.float32)
    x = np.stack([O.synth(31, s, 0, M * frames, complex_=True) for s in range(S)]).astype(np.complex64)
    ch = Channelizer(h, M, sample_dtype=np.complex64, streams=S)
    assert sd.lib().sdsp_chan_set_tuning(ch._h, 8, variant) == 0
    assert sd.lib().sdsp_chan_set_tuning(ch._h, 9, fpb) == 0
    assert sd.lib().sdsp_chan_set_tuning(ch._h, 15, xcd) == 0
    st = torch.cuda.current_stream()
    y = np.zeros((S, frames, M), np.complex64)
    for a, b in ((0, 32), (32, frames)):
        d_in = to_dev(np.ascontiguousarray(x[:, a * M:b * M]).reshape(-1))
        d_out = empty_dev(S * M * (b - a), np.complex64)
        assert ch.execute_block_device(d_in, M * (b - a), d_out, st) == b - a
        y[:, a:b] = to_host(d_out).reshape(S, b - a, M)
    for s in range(S):
        ref = np.zeros(M * frames, np.complex128)
        O.lib().orc_channelize(O._ptr(h.astype(np.float64)), len(h), M, O._ptr(x[s].astype(np.complex128)),
                               M * frames, O._ptr(ref))
        assert rel_rms(y[s], ref.reshape(frames, M)) <= 1e-6
        # §8d max-abs bound, as in test_channelizer_vs_restatement
        assert np.abs(y[s] - ref.reshape(frames, M)).max() <= 1e-6 * np.abs(h).sum() * np.abs(x[s]).max() * np.sqrt(M)


@pytest.mark.parametrize("variant,fpb", [(1, 16), (2, 8), (3, 16), (4, 8), (5, 8), (6, 8)])
@pytest.mark.parametrize("xcd", [0, 1])
def test_channelizer_1024_persistent_chunk_walk(variant, fpb, xcd):
    """more chunks than resident workgroups: every workgroup walks several chunks
    (per-XCD windows or launch order), each restarting its PFB ring from K-1 warm-up frames"""
    import torch
    M, K, S, frames = 1024, 8, 2, 2100
    h = O.firdes_kaiser(M * K, 0.5 / M, 80.0, 0.0).astype(np.float32)
    x = np.stack([O.synth(77, s, 0, M * frames, complex_=True) for s in range(S)]).astype(np.complex64)
    ch = Channelizer(h, M, sample_dtype=np.complex64, streams=S)
    for key, v in ((8, variant), (9, fpb), (15, xcd)):
        assert sd.lib().sdsp_chan_set_tuning(ch._h, key, v) == 0
    d_out = empty_dev(S * M * frames, np.complex64)
    assert ch.execute_block_device(to_dev(x.reshape(-1)), M * frames, d_out, torch.cuda.current_stream()) == frames
    y = to_host(d_out).reshape(S, frames, M)
    for s in range(S):
        ref = np.zeros(M * frames, np.complex128)
        O.lib().orc_channelize(O._ptr(h.astype(np.float64)), len(h), M, O._ptr(x[s].astype(np.complex128)),
                               M * frames, O._ptr(ref))
        assert rel_rms(y[s], ref.reshape(frames, M)) <= 1e-6
        # §8d max-abs bound, as in test_channelizer_vs_restatement
        assert np.abs(y[s] - ref.reshape(frames, M)).max() <= 1e-6 * np.abs(h).sum() * np.abs(x[s]).max() * np.sqrt(M)


@pytest.mark.parametrize("cdt,sdt,kind", [(np.float64, np.float64, 0), (np.float64, np.complex128, 1),
                                          (np.complex128, np.complex128, 2)])
@pytest.mark.parametrize("direction", [Direction.FORWARD, Direction.REVERSE])
def test_dot_product_bit_parity(cdt, sdt, kind, direction):
    """vs the oracle DotProduct restatement (f64 family), bit for bit"""
    rng = np.random.default_rng(1)
    c = rng.standard_normal(37).astype(cdt)
    if np.dtype(cdt).kind == "c":
        c = c + 1j * rng.standard_normal(37)
    for n in (37, 20, 50):  # iterations = min(samples, len)  (mod.rs:161)
        s = rng.standard_normal(n).astype(sdt)
        if np.dtype(sdt).kind == "c":
            s = s + 1j * rng.standard_normal(n)
        got = DotProduct(c, direction, sample_dtype=sdt).execute(s)
        ref = np.zeros(2)
        O.lib().orc_dot_execute(kind, O._ptr(c), len(c), int(direction), O._ptr(s), n, O._dptr(ref))
        r = ref[0] if kind == 0 else complex(ref[0], ref[1])
        assert bits_equal(np.array([got], dtype=sdt), np.array([r], dtype=sdt))


def test_dot_product_batched_device_f32():
    import torch
    rng = np.random.default_rng(2)
    c = rng.standard_normal(16).astype(np.float32)
    S = (rng.standard_normal((100, 24)) + 1j * rng.standard_normal((100, 24))).astype(np.complex64)
    d_s = to_dev(S.reshape(-1))
    d_o = empty_dev(100, np.complex64)
    DotProduct(c, Direction.REVERSE, sample_dtype=np.complex64).execute_batched_device(
        d_s, 24, 24, 100, d_o, torch.cuda.current_stream())
    got = to_host(d_o)
    ref = (S[:, :16] * c[::-1].astype(np.float64)).sum(axis=1)
    assert rel_rms(got, ref) <= 1e-6


def test_dot_product_kat():  # src/dot_product/mod.rs:15
    assert DotProduct(np.array([1.0, 2, 3, 4, 5]), Direction.REVERSE).execute(np.ones(5)) == 15.0


def test_channelizer_rejects_in_place_and_orders_side_stream_reset():
    import torch
    M, K, frames = 1024, 8, 64
    h = O.firdes_kaiser(M * K, 0.5 / M, 80.0, 0.0).astype(np.float32)
    x = O.synth(12, 0, 0, M * frames, complex_=True).astype(np.complex64)
    ch = Channelizer(h, M, sample_dtype=np.complex64)
    buf = to_dev(np.concatenate([x, x]))
    with pytest.raises(sd.SdspError) as e:
        ch.execute_block_device(buf, M * frames, buf[M:])
    assert e.value.code == 90
    s = torch.cuda.Stream()
    outs = [empty_dev(M * frames, np.complex64) for _ in range(2)]
    with torch.cuda.stream(s):
        ch.execute_block_device(buf[:M * frames], M * frames, outs[0], s)
        ch.reset()  # must wait for the queued block before zeroing the history
        ch.execute_block_device(buf[:M * frames], M * frames, outs[1], s)
    torch.cuda.synchronize()
    assert bits_equal(to_host(outs[0]), to_host(outs[1]))
