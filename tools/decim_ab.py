"""Interleaved in-process A/B of the polyphase decimator's lane-group segment
length (SDSP_TUNE_DECIM_SEG) on the cfg4 workload.  Outputs must be bit-identical."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(rounds=8, log2n=30):
    import torch
    import solid_dsp_amd as sd
    from solid_dsp_amd import DecimatingFIRFilter
    from solid_dsp_amd.filter import firdes
    n = 1 << log2n
    h = firdes.firdes_kaiser(256, 1.0 / 64, 80.0, 0.0).astype(np.float32)
    d_in = torch.empty(n, dtype=torch.complex64, device="cuda")
    sd.lib().sdsp_synth_f32_device(d_in.data_ptr(), 20250226, 0, 0, 2 * n, None)
    segs = json.loads(os.environ.get("DECIM_SEGS", "[0, 64, 128, 256, 512, 1024, 4096]"))
    s = torch.cuda.current_stream()
    variants, outs = {}, {}
    for seg in segs:
        f = DecimatingFIRFilter(h, np.float32(1.0 / 32), 32, sample_dtype=np.complex64, algo=sd.ALGO_FMA)
        sd.lib().sdsp_fir_set_tuning(f._h, 6, seg)
        variants[f"seg{seg}"] = f
        o = torch.empty(n // 32, dtype=torch.complex64, device="cuda")
        f.execute_block_device(d_in, n, o, s)
        outs[f"seg{seg}"] = o.cpu().numpy().view(np.uint64)
        f.reset()
    ref = next(iter(outs.values()))
    d_out = torch.empty(n // 32, dtype=torch.complex64, device="cuda")
    times = {k: [] for k in variants}
    for _ in range(rounds):
        for k, f in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            f.execute_block_device(d_in, n, d_out, s)
            e1.record(s)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1))
    bytes_ = 8 * n + 8 * (n // 32)
    res = {k: {"median_ms": float(np.median(v)), "GBps": bytes_ / (np.median(v) * 1e-3) / 1e9,
               "identical": bool(np.array_equal(outs[k], ref))} for k, v in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
