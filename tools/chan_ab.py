"""Interleaved in-process A/B of the channeliser kernels (per-frame chan_kernel vs
the streaming M=1024 kernels, SDSP_TUNE_CHAN_STREAMING 1 = 1024-thread, 2 = 512-thread) on the cfg5 workload.
  CHAN_CASES="variant:frames_per_block:xcd_order,..." python tools/chan_ab.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(rounds=int(os.environ.get("CHAN_ROUNDS", "9"))):
    import torch
    lab = os.environ.get("CHAN_LAB")  # ablation bits per case (lab build): 1 no FFT, 2 no loads, 4 no stores
    if lab:
        import solid_dsp_amd._lib as LL
        LL.LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "_build",
                                   "libsdsp_lab.so")
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
    cases = os.environ.get("CHAN_CASES", "0:0:0,1:256:0,1:256:1,2:256:1")
    labs = {}
    for c in cases.split(","):
        fast, fpb, xcd, ab = ((int(v) for v in c.split(":")) if c.count(":") == 3 else
                              (*(int(v) for v in c.split(":")), 0))
        f = Channelizer(h, M, sample_dtype=np.complex64, streams=S)
        assert sd.lib().sdsp_chan_set_tuning(f._h, 8, fast) == 0
        assert sd.lib().sdsp_chan_set_tuning(f._h, 9, fpb) == 0
        assert sd.lib().sdsp_chan_set_tuning(f._h, 15, xcd) == 0
        key = f"fast{fast}_fpb{fpb}_xcd{xcd}" + (f"_lab{ab}" if ab else "")
        labs[key] = ab
        variants[key] = f
        if lab:
            sd.lib().sdsp_lab_set_chan_ablation(ab)
        o = torch.empty_like(d_in)
        f.execute_block_device(d_in, n, o, st)
        torch.cuda.synchronize()
        outs[key] = o.cpu().numpy().astype(np.complex128)
        f.reset()
    a = next(iter(outs.values()))
    agree = {k: float(np.linalg.norm(a - b) / np.linalg.norm(a)) for k, b in outs.items()}
    d_out = torch.empty_like(d_in)
    times = {k: [] for k in variants}
    keys = list(variants)
    if lab:
        sd.lib().sdsp_lab_set_chan_ablation(0)
    for _ in range(30):  # clocks settle
        variants[keys[-1]].execute_block_device(d_in, n, d_out, st)
    rng = np.random.default_rng(0)
    burst = int(os.environ.get("CHAN_BURST", "1"))  # > 1: back-to-back calls per sample (sustained, bench-like)
    for _ in range(rounds):
        for k in rng.permutation(keys):
            f = variants[k]
            if lab:
                sd.lib().sdsp_lab_set_chan_ablation(labs[k])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(burst):
                f.execute_block_device(d_in, n, d_out, st)
            e1.record(st)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / burst)
    res = {k: {"median_ms": float(np.median(v)), "GBps": 16.0 * S * n / (np.median(v) * 1e-3) / 1e9}
           for k, v in times.items()}
    res["rel_rms_between"] = agree
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
