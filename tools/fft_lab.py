"""In-process A/B of the four-step 2^20-point pass kernel's cache policy on the cfg8 batch
(256 forward transforms, c32), lab build only (tools/lab.mk: sdsp_lab_set_fft_policy, bit 0
nontemporal loads, bit 1 nontemporal stores), interleaved, BURST back-to-back calls per sample.
  FFT_CASES="0,1,2,3" FFT_BURST=10 python tools/fft_lab.py"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(rounds=int(os.environ.get("FFT_ROUNDS", "9"))):
    import torch
    import solid_dsp_amd._lib as LL
    LL.LIB_PATH = os.path.join(REPO, "tools", "_build", "libsdsp_lab.so")
    import solid_dsp_amd as sd
    from solid_dsp_amd import FFT, FFTDirection
    L = sd.lib()
    N, batch = 1 << 20, 256
    d_in = torch.empty(N * batch, dtype=torch.complex64, device="cuda")
    L.sdsp_synth_f32_device(d_in.data_ptr(), 20250226, 0, 0, 2 * N * batch, None)
    d_out = torch.empty_like(d_in)
    st = torch.cuda.current_stream()
    f = FFT(N, FFTDirection.FORWARD, precision=np.complex64)
    cases = [int(c) for c in os.environ.get("FFT_CASES", "0,1,2,3").split(",")]
    burst = int(os.environ.get("FFT_BURST", "10"))
    ref, agree = None, {}
    for c in cases:
        L.sdsp_lab_set_fft_policy(c)
        f.execute_device(d_in, d_out, batch, st)
        torch.cuda.synchronize()
        y = d_out[-N:].cpu().numpy()
        ref = y if ref is None else ref
        agree[c] = float(np.abs(y - ref).max())
    L.sdsp_lab_set_fft_policy(0)
    for _ in range(40):
        f.execute_device(d_in, d_out, batch, st)
    times = {c: [] for c in cases}
    rng = np.random.default_rng(0)
    for _ in range(rounds):
        for c in rng.permutation(sorted(set(cases))):
            L.sdsp_lab_set_fft_policy(int(c))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(burst):
                f.execute_device(d_in, d_out, batch, st)
            e1.record(st)
            torch.cuda.synchronize()
            times[int(c)].append(e0.elapsed_time(e1) / burst)
    L.sdsp_lab_set_fft_policy(0)
    print(json.dumps({f"policy{c}": {"median_ms": float(np.median(v)), "frac_of_8TBps": 16.0 * N * batch / (np.median(v) * 1e-3) / 8e12,
                                     "max_abs_vs_first": agree[c]} for c, v in times.items()}, indent=1))


if __name__ == "__main__":
    main()
