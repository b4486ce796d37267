"""Timing of the generic polyphase filterbank path (shapes the interpolator tile
kernel does not take) -- run once with the product library and once with
PFB_LIB=tools/_build/libsdsp_lab.so (tools/lab.mk: the per-output pfb_kernel) on
the same box; prints one JSON object per shape.  Tools only."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SHAPES = [  # (label, M, K, sample dtype)
    ("c32 M=24 K=10", 24, 10, np.complex64),
    ("f32 M=5 K=64", 5, 64, np.float32),
    ("c64 M=100 K=6", 100, 6, np.complex128),
]


def main(log2n=22, rounds=9):
    import torch
    if os.environ.get("PFB_LIB"):
        import solid_dsp_amd._lib as LL
        LL.LIB_PATH = os.path.join(REPO, os.environ["PFB_LIB"])
    import solid_dsp_amd as sd
    from solid_dsp_amd import PolyPhaseFilterBank
    n = 1 << log2n
    res = {}
    for label, M, K, sdt in SHAPES:
        rng = np.random.default_rng(M * K)
        h = rng.standard_normal(M * K).astype(np.float32 if sdt != np.complex128 else np.float64)
        f = PolyPhaseFilterBank(h, M, sample_dtype=sdt)
        tdt = {np.complex64: torch.complex64, np.float32: torch.float32, np.complex128: torch.complex128}[sdt]
        x = torch.randn(n, dtype=tdt, device="cuda")
        y = torch.empty(n * M, dtype=tdt, device="cuda")
        st = torch.cuda.current_stream()
        for _ in range(3):
            f.execute_block_device(x, n, y, st)
        ts = []
        for _ in range(rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            f.execute_block_device(x, n, y, st)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        sb = np.dtype(sdt).itemsize
        res[label] = {"median_ms": round(ms, 4), "GBps": round(sb * n * (1 + M) / (ms * 1e-3) / 1e9, 1),
                      "lib": os.path.basename(sd._lib.LIB_PATH)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
