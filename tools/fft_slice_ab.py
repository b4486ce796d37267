"""Batched 2^20-point c32 FFT (cfg8 shape, 256 transforms): the whole batch in one
call (each four-step pass over 2 GiB, the intermediate through HBM) against the same
batch as consecutive calls of B transforms, whose 8 B-MiB intermediate can stay in the
256 MiB Infinity Cache between the two passes.  Interleaved, medians of ROUNDS.
  FFT_SLICES="0,4,8,16,32" python tools/fft_slice_ab.py   (0 = one call)"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(rounds=int(os.environ.get("FFT_ROUNDS", "9"))):
    import torch
    import solid_dsp_amd as sd
    from solid_dsp_amd import FFT, FFTDirection
    N, batch = 1 << 20, 256
    d_in = torch.empty(N * batch, dtype=torch.complex64, device="cuda")
    sd.lib().sdsp_synth_f32_device(d_in.data_ptr(), 20250226, 0, 0, 2 * N * batch, None)
    d_out = torch.empty_like(d_in)
    st = torch.cuda.current_stream()
    f = FFT(N, FFTDirection.FORWARD, precision=np.complex64)
    slices = [int(v) for v in os.environ.get("FFT_SLICES", "0,4,8,16,32").split(",")]

    def run(b):
        if b == 0:
            f.execute_device(d_in, d_out, batch, st)
            return
        for i in range(0, batch, b):
            f.execute_device(d_in[i * N:(i + b) * N], d_out[i * N:(i + b) * N], b, st)

    ref = None
    agree = {}
    for b in slices:
        run(b)
        torch.cuda.synchronize()
        y = d_out[-N:].cpu().numpy()
        ref = y if ref is None else ref
        agree[b] = float(np.abs(y - ref).max())
    for _ in range(20):
        run(0)
    times = {b: [] for b in slices}
    rng = np.random.default_rng(0)
    for _ in range(rounds):
        for b in rng.permutation(slices):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            run(int(b))
            e1.record(st)
            torch.cuda.synchronize()
            times[int(b)].append(e0.elapsed_time(e1))
    res = {f"slice{b}": {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)),
                         "frac_of_8TBps": 16.0 * N * batch / (np.median(v) * 1e-3) / 8e12, "max_abs_vs_first": agree[b]}
           for b, v in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
