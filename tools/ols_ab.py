"""Interleaved in-process A/B of the overlap-save interior kernels on cfg2
(guide §5.4 rule 24: shuffled order every round, median of rounds).

  python tools/ols_ab.py            # one-shot (0) vs persistent packed (1) vs scalar (2)
  OLS_KERNELS=0,1 OLS_ROUNDS=20 python tools/ols_ab.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TUNE_OLS_KERNEL = 14


def main(rounds=int(os.environ.get("OLS_ROUNDS", "12")), log2n=30):
    import torch
    import solid_dsp_amd as sd
    from solid_dsp_amd import FIRFilter
    from solid_dsp_amd.filter import firdes
    n = 1 << log2n
    h = firdes.firdes_kaiser(256, 0.1, 80.0, 0.0).astype(np.float32)
    d_in = torch.empty(n, dtype=torch.complex64, device="cuda")
    sd.lib().sdsp_synth_f32_device(d_in.data_ptr(), 20250226, 0, 0, 2 * n, None)
    kernels = [int(k) for k in os.environ.get("OLS_KERNELS", "0,1,2").split(",")]
    variants = {}
    for k in kernels:
        f = FIRFilter(h, np.float32(0.2), sample_dtype=np.complex64, algo=sd.ALGO_FFT)
        assert sd.lib().sdsp_fir_set_tuning(f._h, TUNE_OLS_KERNEL, k) == 0
        variants[f"kernel{k}"] = f
    s = torch.cuda.current_stream()
    outs = {}
    for k, f in variants.items():
        o = torch.empty_like(d_in)
        f.execute_block_device(d_in, n, o, s)
        outs[k] = np.concatenate([o[: 1 << 22].cpu().numpy(), o[-(1 << 20):].cpu().numpy()]).astype(np.complex128)
        del o
    ref = outs[next(iter(outs))]
    diff = {k: float(np.linalg.norm(v - ref) / np.linalg.norm(ref)) for k, v in outs.items()}
    d_out = torch.empty_like(d_in)
    order = list(variants.items())
    rng = np.random.default_rng(1)
    times = {k: [] for k in variants}
    for _ in range(rounds):
        rng.shuffle(order)
        for k, f in order:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            f.execute_block_device(d_in, n, d_out, s)
            e1.record(s)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1))
    res = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)),
               "GBps": 16.0 * n / (np.median(v) * 1e-3) / 1e9, "rel_diff_vs_first": diff[k]}
           for k, v in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
