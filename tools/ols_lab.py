"""Interleaved in-process A/B of overlap-save one-shot kernel variants (tools
only): loads tools/_build/libsdsp_lab.so (make -f tools/lab.mk), which carries
extra template instances of fir_ols_os_kernel selected by
sdsp_lab_set_ols_variant.  Shuffled order every round, median of rounds
(guide §5.4 rule 24), after a clock-settling phase.

  OLS_CASES="0,4,4:18432,20::4" OLS_ROUNDS=15 python tools/ols_lab.py
A case is var[:dyn_lds_bytes[:chunk]].  OLS_BURST=B times B back-to-back calls per
sample (the bench's sustained regime) instead of one isolated call.  Variant bits (kern_fir_ols_os.hip): 1
wave-level sync for the two wave-local phase boundaries; 2 no HBM traffic
(ablation); 4 HBM traffic only (ablation); 16 XCDs interleaved in runs of
`chunk` segments instead of contiguous eighths.  dyn_lds pins occupancy
(36 KB static: +18432 -> 3 workgroups per CU, +45056 -> 2).
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(rounds=int(os.environ.get("OLS_ROUNDS", "15")), log2n=30):
    import torch
    import solid_dsp_amd._lib as LL
    LL.LIB_PATH = os.path.join(REPO, "tools", "_build", "libsdsp_lab.so")
    import solid_dsp_amd as sd
    from solid_dsp_amd import FIRFilter
    from solid_dsp_amd.filter import firdes
    L = sd.lib()
    L.sdsp_lab_set_ols_variant.argtypes = [C.c_int, C.c_int, C.c_int]
    L.sdsp_lab_ols_stamps.argtypes = [C.c_void_p]
    if os.environ.get("OLS_HWID"):  # which CU slots the lab tickets use: distinct (XCC_ID, HW_ID[15:8])
        nb = 4096
        hb = torch.zeros(2 * nb, dtype=torch.int32, device="cuda")
        assert L.sdsp_lab_hwid_probe(C.c_void_p(hb.data_ptr()), nb) == 0
        a = hb.cpu().numpy().astype(np.int64).reshape(-1, 2)
        keys = set(((a[:, 0] & 7) << 8 | ((a[:, 1] >> 8) & 255)).tolist())
        print("hwid: %d distinct slots over %d blocks; xcc values %s; hw_id samples %s" % (
            len(keys), nb, sorted(set(a[:, 0].tolist()))[:16], [hex(v) for v in a[:8, 1]]), flush=True)
    n = 1 << log2n
    h = firdes.firdes_kaiser(256, 0.1, 80.0, 0.0).astype(np.float32)
    d_in = torch.empty(n, dtype=torch.complex64, device="cuda")
    L.sdsp_synth_f32_device(d_in.data_ptr(), 20250226, 0, 0, 2 * n, None)
    def parse(c):
        if c == "nco":  # the NCO mix_down of the same buffer (cfg7's kernel), for a side-by-side
            return (-1, 0, 1)
        f = (c.split(":") + ["", ""])[:3]
        return (int(f[0]), int(f[1] or 0), int(f[2] or 1))
    variants = [parse(c) for c in os.environ.get("OLS_CASES", "0,1,2,4").split(",")]
    nco = sd.NCO()
    nco.set_frequency(2 * np.pi * 0.0123)
    f = FIRFilter(h, np.float32(0.2), sample_dtype=np.complex64, algo=sd.ALGO_FFT)
    s = torch.cuda.current_stream()
    d_out = torch.empty_like(d_in)
    outs, diff = {}, {}
    for v in variants:
        if v[0] < 0 or (v[0] < 256 and v[0] & 6) or (v[0] & 131072):
            continue
        L.sdsp_lab_set_ols_variant(*v)
        f.reset()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        f.execute_block_device(d_in, n, d_out, s)
        e1.record(s)
        torch.cuda.synchronize()
        print("first run var%d:%d:%d %.3f ms" % (v + (e0.elapsed_time(e1),)), flush=True)
        outs[v] = np.concatenate([d_out[: 1 << 22].cpu().numpy(), d_out[-(1 << 20):].cpu().numpy()])
    ref = outs.get((0, 0, 1))
    for v, o in outs.items():
        diff[v] = None if ref is None else float(np.linalg.norm(o.astype(np.complex128) - ref) / np.linalg.norm(ref))
    L.sdsp_lab_set_ols_variant(0, 0, 1)
    for _ in range(60):  # ~0.2 s of device time: clocks settle
        f.execute_block_device(d_in, n, d_out, s)
    torch.cuda.synchronize()
    rng = np.random.default_rng(1)
    burst = int(os.environ.get("OLS_BURST", "1"))  # > 1: back-to-back calls per sample (sustained, bench-like)
    times = {v: [] for v in variants}
    order = list(variants)
    for i in range(rounds):
        print("round", i, flush=True)
        rng.shuffle(order)
        for v in order:
            L.sdsp_lab_set_ols_variant(*(v if v[0] >= 0 else (0, 0, 1)))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(burst):
                if v[0] < 0:
                    nco.mix_block_device(d_in, n, d_out, down=True, precision=0, stream=s)
                else:
                    f.execute_block_device(d_in, n, d_out, s)
            e1.record(s)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / burst)
    clocks = {}
    for v in variants:  # in-kernel clock of the stamped variant, after a sustained burst
        if v[0] < 0 or not (v[0] & 262144):
            continue
        L.sdsp_lab_set_ols_variant(*v)
        L.sdsp_lab_ols_stamps_clear()
        for _ in range(max(burst, 20)):
            f.execute_block_device(d_in, n, d_out, s)
        torch.cuda.synchronize()
        st = np.zeros(4 * 8192, dtype=np.uint64)
        assert L.sdsp_lab_ols_stamps(C.c_void_p(st.ctypes.data)) == 0
        st = st.reshape(-1, 4).astype(np.float64)
        ok = st[:, 3] > st[:, 1]
        ghz = (st[ok, 2] - st[ok, 0]) / (st[ok, 3] - st[ok, 1]) * 0.1
        dur_us = (st[ok, 3] - st[ok, 1]) * 0.01
        clocks["var%d:%d:%d" % v] = {"workgroups": int(ok.sum()), "clock_GHz_median": float(np.median(ghz)),
                                     "clock_GHz_p10": float(np.percentile(ghz, 10)),
                                     "clock_GHz_p90": float(np.percentile(ghz, 90)),
                                     "workgroup_us_median": float(np.median(dur_us))}
    if clocks:
        print("in-kernel clock (s_memtime / s_memrealtime x 100 MHz):", json.dumps(clocks, indent=1), flush=True)
    res = {("nco" if v[0] < 0 else "var%d:%d:%d" % v): {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
                       "frac_of_8TBps": 16.0 * n / (np.median(t) * 1e-3) / 8e12,
                       "rel_diff_vs_var0": diff.get(v)} for v, t in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
