"""Generate the committed golden fixtures (run from the repo root:
`python tests/golden/make_golden.py`).

* butter8_0p2_sos.json -- cfg3's 4-section cascade, scipy.signal.butter(8, 0.2,
  output='sos'), rows [b0 b1 b2 a0 a1 a2].
* butter8_0p01_sos.json -- a narrow-band cascade, scipy.signal.butter(8, 0.01,
  output='sos'): section 0 carries the whole gain (b0 = 3.4e-15), the case the
  wave scan's b0-factored coordinates scale states by ~1/b0 (test_gpu_iir.py).
* vectors_*.npz -- make_vectors(): inputs and expected outputs for the rows the
  reference's own tests do not pin (PolyPhaseFilterBank, InterpolatingFIRFilter,
  the channeliser, FFT, full-complex FIR), computed by the oracle restatement
  (oracle/, test infrastructure) from seeded inputs.  They are "parity unpinned
  by the reference" (DESIGN §2): they freeze the restatement's outputs so the
  device tests (tests/test_gpu_golden.py) and the oracle itself
  (tests/test_golden_fixtures.py) are checked against committed data.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))

SEED = 20250226


def make_butter():
    from scipy import signal
    for wn, name in ((0.2, "butter8_0p2_sos.json"), (0.01, "butter8_0p01_sos.json")):
        sos = signal.butter(8, wn, output="sos")
        with open(os.path.join(HERE, name), "w") as f:
            json.dump({"source": "scipy.signal.butter(8, %g, output='sos')" % wn, "sos": sos.tolist()}, f, indent=1)


def _rand(rng, n, dt):
    if np.dtype(dt).kind == "c":
        return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(dt)
    return rng.standard_normal(n).astype(dt)


def vector_cases():
    """name -> (kind, params, arrays) for every fixture; deterministic."""
    import oracle_lib as O
    rng = np.random.default_rng(SEED)
    cases = {}
    # PolyPhaseFilterBank (pfb.rs:24-90): dtype, L taps, M filters, scale (ignored by execute)
    for name, dt, cdt, sdt, L, M in [("pfb_rc32", O.RC32, np.float32, np.complex64, 18, 4),
                                     ("pfb_cc64", O.CC64, np.complex128, np.complex128, 64, 8)]:
        h, x = _rand(rng, L, cdt), _rand(rng, 300, sdt)
        y = O.pfb(dt, h, M, cdt(3.0)).execute_block(x)
        cases[name] = ("pfb", {"dtype": dt, "M": M, "scale": 3.0}, {"taps": h, "x": x, "y": y})
    # InterpolatingFIRFilter (interp.rs:27-111), incl. the zero-padded ceil_f32(L/M) branches
    for name, dt, cdt, sdt, L, M in [("interp_rc32_k8", O.RC32, np.float32, np.complex64, 256, 32),
                                     ("interp_cc32_pad", O.CC32, np.complex64, np.complex64, 60, 16),
                                     ("interp_rr64", O.RR64, np.float64, np.float64, 10, 4)]:
        h, x = _rand(rng, L, cdt), _rand(rng, 600, sdt)
        y = O.interp(dt, h, M).execute_block(x)
        cases[name] = ("interp", {"dtype": dt, "M": M}, {"taps": h, "x": x, "y": y})
    # full-complex FIR (fir/mod.rs:209-212, num-complex Mul), f32 and f64
    for name, dt, cdt, sdt, L in [("fir_cc32", O.CC32, np.complex64, np.complex64, 63),
                                  ("fir_cc64", O.CC64, np.complex128, np.complex128, 17)]:
        h, x = _rand(rng, L, cdt), _rand(rng, 1000, sdt)
        y = O.fir(dt, h, cdt(0.5 - 0.25j)).execute_block(x)
        cases[name] = ("fir", {"dtype": dt, "scale": [0.5, -0.25]}, {"taps": h, "x": x, "y": y})
    # FFT (fft/mod.rs:123-215): the restated planner (Rader / mixed radix / DFT leaves), both directions
    L_ = O.lib()
    for nfft in (12, 60, 97, 256, 1000, 4096):
        x = _rand(rng, nfft, np.complex128)
        for d in (0, 1):
            h = L_.orc_fft_new(nfft, d)
            y = np.zeros(nfft, np.complex128)
            L_.orc_fft_execute(h, O._ptr(x), O._ptr(y))
            L_.orc_fft_free(h)
            cases[f"fft_{nfft}_{'fwd' if d == 0 else 'rev'}"] = ("fft", {"n": nfft, "direction": d}, {"x": x, "y": y})
    # channeliser (PFB branch layout + FFT FORWARD), M = 64, K = 8, 16 frames
    M = 64
    h = O.firdes_kaiser(8 * M, 1.0 / (2 * M), 80.0, 0.0)
    x = _rand(rng, 16 * M, np.complex128)
    y = np.zeros_like(x)
    L_.orc_channelize(O._ptr(h), len(h), M, O._ptr(x), len(x), O._ptr(y))
    cases["chan_m64_k8"] = ("chan", {"M": M}, {"taps": h, "x": x, "y": y})
    return cases


def make_vectors():
    for name, (kind, params, arrays) in vector_cases().items():
        np.savez_compressed(os.path.join(HERE, f"vectors_{name}.npz"), kind=np.array(kind),
                            params=np.array(json.dumps(params)), **arrays)


def load(name):
    d = np.load(os.path.join(HERE, f"vectors_{name}.npz"))
    return str(d["kind"]), json.loads(str(d["params"])), {k: d[k] for k in d.files if k not in ("kind", "params")}


def names():
    return sorted(f[len("vectors_"):-len(".npz")] for f in os.listdir(HERE) if f.startswith("vectors_"))


if __name__ == "__main__":
    make_butter()
    make_vectors()
