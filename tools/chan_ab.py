"""Interleaved in-process A/B of the channeliser kernels (per-frame chan_kernel vs
the streaming M=1024 kernel, SDSP_TUNE_CHAN_STREAMING) on the cfg5 workload."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(rounds=6):
    import torch
    import solid_dsp_amd as sd
    from solid_dsp_amd import Channelizer
    from solid_dsp_amd.filter import firdes
    M, S, n = 1024, 8, 1 << 24
    h = firdes.firdes_kaiser(8192, 1.0 / 2048, 80.0, 0.0).astype(np.float32)
    d_in = torch.empty(S * n, dtype=torch.complex64, device="cuda")
    for s_ in range(S):
        sd.lib().sdsp_synth_f32_device(d_in[s_ * n:].data_ptr(), 20250226, s_, 0, 2 * n, None)
    st = torch.cuda.current_stream()
    variants, outs = {}, {}
    for fast, fpb in ((0, 0), (1, 32), (1, 64), (1, 128), (1, 256)):
        f = Channelizer(h, M, sample_dtype=np.complex64, streams=S)
        assert sd.lib().sdsp_chan_set_tuning(f._h, 8, fast) == 0
        assert sd.lib().sdsp_chan_set_tuning(f._h, 9, fpb) == 0
        key = f"fast{fast}_fpb{fpb}"
        variants[key] = f
        o = torch.empty_like(d_in)
        f.execute_block_device(d_in, n, o, st)
        torch.cuda.synchronize()
        outs[key] = o.cpu().numpy().astype(np.complex128)
        f.reset()
    a = outs["fast0_fpb0"]
    agree = {k: float(np.linalg.norm(a - b) / np.linalg.norm(a)) for k, b in outs.items()}
    d_out = torch.empty_like(d_in)
    times = {k: [] for k in variants}
    for _ in range(rounds):
        for k, f in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            f.execute_block_device(d_in, n, d_out, st)
            e1.record(st)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1))
    res = {k: {"median_ms": float(np.median(v)), "GBps": 16.0 * S * n / (np.median(v) * 1e-3) / 1e9}
           for k, v in times.items()}
    res["rel_rms_between"] = agree
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
