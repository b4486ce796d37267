"""Stream ordering of streaming handles and the kernel-variant knobs (MI355X).

ADVICE r03: a block on a caller stream s1, then a block on the handle's own
stream, then blocks on s1 and on a third stream s2, all queued without a host
sync in between, must run in call order -- each reads the delay line (window,
history, IIR state) the previous one wrote.  VERDICT r04 #3: the same chain through
torch's default stream (the legacy null stream, hipStreamLegacy at the C ABI):
legacy -> handle -> s1 -> legacy, which the fences order by a host wait.  The first block is long, so an
unordered launch would start while it is still running.  Every later block is
checked bit for bit against the restatement (EXACT / serial kernels), or within
the §8d tolerance (overlap-save).

The kernel-variant knobs (SDSP_TUNE_*: sdsp_acorr_set_tuning, sdsp_agc_set_tuning,
sdsp_fft_set_tuning) replace the round-3 environment switches: every value
computes the same result, and both branches run in one process here."""
import numpy as np
import pytest

import oracle_lib as O
from gpu_util import bits_equal, rel_rms, to_dev, empty_dev, to_host

pytestmark = pytest.mark.gpu

sd = pytest.importorskip("solid_dsp_amd")
L = sd._lib

C64, C128, F32, F64 = np.complex64, np.complex128, np.float32, np.float64
N1, N2 = 1 << 24, 4096  # the long first block, then three short ones


def _streams():
    import torch
    return torch.cuda.Stream(), torch.cuda.Stream()


ORDERS = ["streams", "legacy"]


def _chain(execute, blocks, nout, dt, order="streams"):
    """Stage every block on the device first (synchronised), then queue them with no host
    sync in between on s1, the handle's stream (None), s1 and s2 ("streams"), or on the
    legacy default stream, the handle's stream, s1 and the legacy stream ("legacy");
    execute(d_in, n, d_out, stream) -> outputs produced.  Returns the host outputs of
    every block."""
    import torch
    s1, s2 = _streams()
    legacy = torch.cuda.default_stream()
    assert legacy.cuda_stream == 0  # mapped to hipStreamLegacy by _lib.stream_handle
    seq = [s1, None, s1, s2] if order == "streams" else [legacy, None, s1, legacy]
    ins = [to_dev(b) for b in blocks]
    outs = [empty_dev(max(nout(len(b)), 1), dt) for b in blocks]
    torch.cuda.synchronize()
    got = [execute(i, len(b), o, st) for i, b, o, st in zip(ins, blocks, outs, seq)]
    torch.cuda.synchronize()
    return [to_host(o)[:m] for o, m in zip(outs, got)]


def _cuts(n0):
    return [0, n0, n0 + N2, n0 + 2 * N2, n0 + 3 * N2]


def _fir_window_ref(o_factory, x, lo, hi, L_):
    """Outputs [lo, hi) of the whole-stream FIR from its (L-1)-sample input window: a fresh
    restatement fed x[lo-L+1, hi) computes the same sums in the same order."""
    a = max(lo - (L_ - 1), 0)
    return o_factory().execute_block(x[a:hi])[lo - a:]


@pytest.mark.parametrize("order", ORDERS)
@pytest.mark.parametrize("algo", ["exact", "fft"])
def test_fir_blocks_across_streams_run_in_call_order(algo, order):
    h = O.firdes_kaiser(64, 0.1, 80.0, 0.0).astype(F32)
    x = O.synth(77, 0, 0, N1 + 3 * N2, complex_=True)
    f = sd.FIRFilter(h, F32(0.2), sample_dtype=C64, algo=sd.ALGO_EXACT if algo == "exact" else sd.ALGO_FFT,
                     host_step=False)
    cuts = _cuts(N1)
    outs = _chain(f.execute_block_device, [x[cuts[k]:cuts[k + 1]] for k in range(4)], lambda n: n, C64, order)
    f.synchronize()
    mk32 = lambda: O.fir(O.RC32, h, F32(0.2))
    mk64 = lambda: O.fir(O.RC64, h.astype(F64), 0.2)
    for k in range(1, 4):
        if algo == "exact":
            assert bits_equal(outs[k], _fir_window_ref(mk32, x, cuts[k], cuts[k + 1], 64)), k
        else:
            ref = _fir_window_ref(mk64, x.astype(C128), cuts[k], cuts[k + 1], 64)
            assert rel_rms(outs[k], ref) <= 1e-6, (k, rel_rms(outs[k], ref))
    if algo == "exact":
        assert bits_equal(outs[0][-N2:], _fir_window_ref(mk32, x, N1 - N2, N1, 64))


@pytest.mark.parametrize("order", ORDERS)
def test_decim_blocks_across_streams_run_in_call_order(order):
    h = O.firdes_kaiser(64, 0.05, 80.0, 0.0).astype(F32)
    M = 8
    x = O.synth(78, 0, 0, N1 + 3 * N2, complex_=True)
    f = sd.DecimatingFIRFilter(h, F32(0.5), M, sample_dtype=C64, algo=sd.ALGO_EXACT, host_step=False)
    cuts = [0, N1 + 3, N1 + N2 + 3, N1 + 2 * N2 + 1, N1 + 3 * N2]  # ragged against M
    phase = [0]

    def nout(n):  # outputs of a block from the phase the previous blocks leave
        k = (phase[0] + n) // M
        phase[0] = (phase[0] + n) % M
        return k

    outs = _chain(f.execute_block_device, [x[cuts[k]:cuts[k + 1]] for k in range(4)], nout, C64, order)
    f.synchronize()
    got = np.concatenate(outs[1:])
    first_out = (cuts[1] + M) // M - 1  # the first output m whose input (m+1)M-1 is >= cuts[1]
    a = (first_out + 1) * M - 64  # its 64-tap window starts here
    a -= a % M  # phase-aligned restart: a fresh decimator's outputs fall on the same inputs
    ref = O.decim(O.RC32, h, F32(0.5), M).execute_block(x[a:])
    skip = first_out - a // M
    assert len(got) == len(ref) - skip
    assert bits_equal(got, ref[skip:])


@pytest.mark.parametrize("order", ORDERS)
def test_pfb_blocks_across_streams_run_in_call_order(order):
    rng = np.random.default_rng(4)
    M, K = 16, 8
    h = rng.standard_normal(M * K).astype(F32)
    n0 = 1 << 20
    x = O.synth(79, 0, 0, n0 + 3 * 512, complex_=True)
    p = sd.PolyPhaseFilterBank(h, M, 1.0, sample_dtype=C64, coef_dtype=F32)
    cuts = [0, n0, n0 + 512, n0 + 1024, n0 + 1536]
    outs = _chain(lambda i, n, o, st: p.execute_block_device(i, n, o, st),
                  [x[cuts[k]:cuts[k + 1]] for k in range(4)], lambda n: n * M, C64, order)
    p.synchronize()
    got = np.concatenate(outs[1:])
    a = cuts[1] - K  # the window needs the last K inputs
    ref = O.pfb(O.RC32, h, M, F32(1.0))
    y = np.concatenate([_pfb_all(ref, v, M) for v in x[a:cuts[4]]])
    assert bits_equal(got, y[K * M:])


def _pfb_all(o, v, M):
    o.push(v)
    return np.array([o.pfb_execute(i) for i in range(M)])


@pytest.mark.parametrize("order", ORDERS)
def test_iir_blocks_across_streams_run_in_call_order(order):
    import json
    import os
    sos = np.array(json.load(open(os.path.join(os.path.dirname(__file__), "golden", "butter8_0p2_sos.json")))["sos"])
    ff = sos[:, :3].reshape(-1)
    fb = sos[:, 3:].reshape(-1)
    n0 = 1 << 20  # the serial recurrence: one lane walks the whole first block
    x = O.synth(80, 0, 0, n0 + 3 * N2).astype(F64)
    f = sd.IIRFilter(ff, fb, sd.IIRFilterType.SecondOrder, sample_dtype=F64, algo=sd.ALGO_EXACT)
    cuts = _cuts(n0)
    outs = _chain(f.execute_block_device, [x[cuts[k]:cuts[k + 1]] for k in range(4)], lambda n: n, F64, order)
    f.synchronize()
    ref = O.iir(O.RR64, ff, fb, 1).execute_block(x)
    for k in range(4):
        assert bits_equal(outs[k], ref[cuts[k]:cuts[k + 1]]), k


@pytest.mark.parametrize("kernel,order", [(0, "streams"), (1, "streams"), (2, "streams"), (0, "legacy")])
def test_acorr_blocks_across_streams_and_kernel_variants(kernel, order):
    """AutoCorrelator(64, 16), c64: the three kernel variants (SDSP_TUNE_ACORR_KERNEL) are
    bit-identical to the restatement, with blocks on three streams in call order"""
    n0 = N1 // 4
    x = O.synth(81, 0, 0, n0 + 3 * N2, complex_=True).astype(C128)
    g = sd.AutoCorrelator(64, 16, dtype=C128)
    g.set_tuning(L.TUNE_ACORR_KERNEL, kernel)
    cuts = _cuts(n0)

    def run(i, n, o, st):
        g.execute_block_device(i, n, o, st)
        return n

    outs = _chain(run, [x[cuts[k]:cuts[k + 1]] for k in range(4)], lambda n: n, C128, order)
    e = g.get_energy()  # the round-4 crash: get_energy on the handle's stream after a legacy-stream block
    g.synchronize()
    got = np.concatenate(outs)
    ref = O.AutoCorr(64, 16, C128).execute_block(x)
    assert got.tobytes() == ref.tobytes()
    assert abs(e - float(np.sum(np.abs(x[-64:]) ** 2))) <= 1e-12 * e
    with pytest.raises(sd.SdspError):
        g.set_tuning(L.TUNE_ACORR_KERNEL, 3)


@pytest.mark.parametrize("order", ORDERS)
def test_chan_blocks_across_streams_run_in_call_order(order):
    """streaming M = 1024 channeliser, two streams: a long first block, then three short
    ones on the chain's streams; each reads the (K-1) M-sample history the previous wrote"""
    from solid_dsp_amd.channelizer import Channelizer
    M, K, S = 1024, 8, 2
    f0 = 2048
    fr = [f0, 16, 8, 24]
    h = O.firdes_kaiser(M * K, 0.5 / M, 80.0, 0.0).astype(F32)
    x = np.stack([O.synth(82, s, 0, M * sum(fr), complex_=True) for s in range(S)]).astype(C64)
    ch = Channelizer(h, M, sample_dtype=C64, streams=S)
    edges = np.cumsum([0] + fr) * M
    blocks = [np.ascontiguousarray(x[:, a:b]).reshape(-1) for a, b in zip(edges[:-1], edges[1:])]

    def run(i, n, o, st):
        return ch.execute_block_device(i, n // S, o, st) * M * S

    outs = _chain(run, blocks, lambda n: n, C64, order)
    ch.synchronize()
    for k in range(1, 4):
        y = outs[k].reshape(S, fr[k], M)
        for s in range(S):
            lo = edges[k] - (K - 1) * M  # a fresh restatement fed the K-1 frames before the block
            ref = np.zeros(edges[k + 1] - lo, C128)
            O.lib().orc_channelize(O._ptr(h.astype(F64)), len(h), M, O._ptr(x[s, lo:edges[k + 1]].astype(C128)),
                                   edges[k + 1] - lo, O._ptr(ref))
            ref = ref.reshape(-1, M)[K - 1:]
            assert rel_rms(y[s], ref) <= 1e-6, (k, s)


@pytest.mark.parametrize("kernel", [0, 1])
def test_agc_kernel_variants_agree(kernel):
    import torch
    from test_gpu_rx import AGC_RTOL, _close
    rng = np.random.default_rng(31)
    ch, n = 65, 3000
    x = ((rng.standard_normal((ch, n)) + 1j * rng.standard_normal((ch, n))) * 0.05).astype(C128)
    g = sd.AGC(channels=ch)
    g.set_tuning(L.TUNE_AGC_KERNEL, kernel)
    g.set_bandwidth(0.05)
    d_in = torch.from_numpy(x).to("cuda")
    d_out = torch.empty_like(d_in)
    g.execute_block_device(d_in, n, d_out, complex_=True, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    y = d_out.cpu().numpy()
    for c in (0, 31, 64):
        o = O.Agc()
        o.set_bandwidth(0.05)
        assert _close(y[c], o.execute_block(x[c])), c
    with pytest.raises(sd.SdspError):
        g.set_tuning(L.TUNE_AGC_KERNEL, 2)


@pytest.mark.parametrize("knob", [(L.TUNE_FFT_WAVE1024, 16), (L.TUNE_FFT_WAVE1024, 1),
                                  (L.TUNE_FFT_WAVE1024, 8),
                                  (L.TUNE_FFT_WAVE1024, 0), (L.TUNE_FFT_GROUP, 1), (L.TUNE_FFT_GROUP, 8)])
def test_fft_pass_kernel_variants_agree(knob):
    """2^20-point c32 four-step FFT on each pass kernel (SDSP_TUNE_FFT_WAVE1024 = 0 runs the
    generic pass, whose group size SDSP_TUNE_FFT_GROUP sets) vs numpy, both directions"""
    rng = np.random.default_rng(5)
    n = 1 << 20
    x = (rng.standard_normal((2, n)) + 1j * rng.standard_normal((2, n))).astype(C64)
    for d in (sd.FFTDirection.FORWARD, sd.FFTDirection.REVERSE):
        f = sd.FFT(n, d, precision=C64)
        f.set_tuning(*knob)
        if knob[0] == L.TUNE_FFT_GROUP:
            f.set_tuning(L.TUNE_FFT_WAVE1024, 0)
        y = f.execute(x)
        xs = x.astype(C128)
        ref = np.fft.fft(xs, axis=-1) if d == sd.FFTDirection.FORWARD else np.fft.ifft(xs, axis=-1) * n
        assert rel_rms(y, ref) <= 5e-6, (knob, d, rel_rms(y, ref))
    with pytest.raises(sd.SdspError):
        f.set_tuning(L.TUNE_FFT_WAVE1024, 2)
