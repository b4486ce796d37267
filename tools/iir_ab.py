"""Interleaved in-process A/B of the SOS scan kernels (block scan vs wave scan,
SDSP_TUNE_IIR_WAVE_SCAN) on the cfg3 workload, with agreement between them."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(rounds=int(os.environ.get("IIR_ROUNDS", "8")), log2n=30):
    import torch
    lab = bool(os.environ.get("IIR_LAB"))  # cases "variant:ablation" on the lab build (tools/lab.mk)
    if lab or os.environ.get("IIR_LIB"):  # IIR_LIB: e.g. an older build, same box
        import solid_dsp_amd._lib as LL
        LL.LIB_PATH = os.path.join(REPO, os.environ.get("IIR_LIB") or "tools/_build/libsdsp_lab.so")
    import solid_dsp_amd as sd
    from solid_dsp_amd import IIRFilter, IIRFilterType
    n = 1 << log2n
    sos = np.array(json.load(open(os.path.join(REPO, "tests", "golden", "butter8_0p2_sos.json")))["sos"])
    ff = sos[:, :3].reshape(-1).astype(np.float32)
    fb = sos[:, 3:].reshape(-1).astype(np.float32)
    d_in = torch.empty(n, dtype=torch.float32, device="cuda")
    sd.lib().sdsp_synth_f32_device(d_in.data_ptr(), 20250226, 0, 0, n, None)
    s = torch.cuda.current_stream()
    variants, outs = {}, {}
    abl = {}
    for case in os.environ.get("IIR_CASES", "0,1,2,5").split(","):
        ws, ab = (int(v) for v in (case.split(":") + ["0"])[:2])
        f = IIRFilter(ff, fb, IIRFilterType.SecondOrder, sample_dtype=np.float32, algo=sd.ALGO_FMA)
        sd.lib().sdsp_iir_set_tuning(f._h, 7, ws)
        key = f"wscan{ws}" + (f"_lab{ab}" if ab else "")
        abl[key] = ab
        if lab:
            sd.lib().sdsp_lab_set_iir_ablation(ab)
        variants[key] = f
        o = torch.empty_like(d_in)
        f.execute_block_device(d_in, n, o, s)
        torch.cuda.synchronize()
        outs[key] = (o[: 1 << 22].cpu().numpy().astype(np.float64), o[-(1 << 20):].cpu().numpy().astype(np.float64))
        f.reset()
    a = next(iter(outs.values()))
    agree = {k: max(float(np.linalg.norm(a[i] - b[i]) / np.linalg.norm(a[i])) for i in range(2))
             for k, b in outs.items()}
    d_out = torch.empty_like(d_in)
    times = {k: [] for k in variants}
    keys = list(variants)
    if lab:
        sd.lib().sdsp_lab_set_iir_ablation(0)
    for _ in range(40):  # clocks settle
        variants[keys[-1]].execute_block_device(d_in, n, d_out, s)
    rng = np.random.default_rng(0)
    burst = int(os.environ.get("IIR_BURST", "1"))  # > 1: back-to-back calls per sample (sustained, bench-like)
    for _ in range(rounds):
        for k in rng.permutation(keys):
            f = variants[k]
            if lab:
                sd.lib().sdsp_lab_set_iir_ablation(abl[k])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(burst):
                f.execute_block_device(d_in, n, d_out, s)
            e1.record(s)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / burst)
    res = {k: {"median_ms": float(np.median(v)), "GBps": 8.0 * n / (np.median(v) * 1e-3) / 1e9}
           for k, v in times.items()}
    res["rel_rms_between"] = agree
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
