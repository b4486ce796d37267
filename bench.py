#!/usr/bin/env python3
"""Benchmarks of the streaming filter engine on MI355X.

Default (the driver's headline, BASELINE.json configs[1]): 256-tap complex-f32
FIR over a 1 GiS synthetic stream per GPU, metric "Msamples/sec 256-tap
complex FIR @1/2/4/8 GPU; % HBM roofline".  One step = one device-resident
FIRFilter::execute_block pass (overlap-save kernel) over the whole channel.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1|2|3|4|5] [--log2n 30] [--algo fft|exact|fma]

Other configs (BASELINE.json configs[2..4]):
  3  4-biquad cascade (scipy butter(8, 0.2) SOS), real f32, 1 GiS, block-parallel scan
  4  M=32 decimator, 256 taps (32 branches x 8), crcf, 1 GiS input per GPU
  5  1024-channel PFB + FFT channeliser, 8 streams x 2^24 samples per GPU
SURVEY §8f rows (build-defined cases, same parity + measurement fields):
  6  AutoCorrelator(64, 16), c32, 2^29 samples
  7  NCO mix_down, c32, 2^30 samples
  8  batched 2^20-point forward FFT (four-step), c32, 2^28 samples
  9  AGC bank, Complex<f64>, 2^18 channels x 2^10 samples
 10  32x interpolating FIR (K = 8), crcf, 2^25 inputs -> 2^30 outputs
 11  IIRFilter<f64, Complex<f64>> active_lag bank (the reference demo's filter), 2^16 channels x 2^12
 12  Normal DF-II IIR, order 2, real f32, 2^30 samples (dense-system wave scan)

With N ranks each rank processes its own independent channel(s) (weak
scaling, no collective in the timed region); RCCL is used afterwards only for
the final gather of every rank's whole output to rank 0, timed separately
(`gather`) and checked there against the f64 restatement.  rank 0 prints one
JSON line.  `--gpus N` under torch.distributed.run must equal WORLD_SIZE;
without a torchrun environment this script (never touching the GPU itself)
spawns the N ranks.  `--dry-run` rehearses launch, timing and gather on the
CPU over gloo.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
SEED = 20250226


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU); outside torch.distributed.run this process spawns them itself")
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", type=int, default=2, choices=list(range(1, 13)))
    p.add_argument("--log2n", type=int, default=30, help="samples per GPU per step (configs 2-4)")
    p.add_argument("--algo", default="fft", choices=["fft", "exact", "fma"], help="config 2 kernel")
    p.add_argument("--cpu-samples", type=int, default=None,
                   help="bounded sample of the same workload timed on the host (oracle restatement)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--no-gather", action="store_true", help="skip the final RCCL gather of every rank's output")
    p.add_argument("--dist", action="store_true",
                   help="run the multi-GPU code path (RCCL process group, barriers, max-over-ranks, the final "
                        "gather and its check) even at world size 1: the RCCL path on a one-GPU box")
    p.add_argument("--no-dropin", action="store_true", help="config 2: skip the drop-in cost figures")
    p.add_argument("--shard", default="channel", choices=["channel", "time"],
                   help="configs 2 and 4: independent channels per rank (default), or one long stream "
                        "time-sharded (rank r filters inputs [r n, (r+1) n) after an (L-1)-input halo)")
    p.add_argument("--settle-ms", type=float, default=150.0,
                   help="untimed steps of the workload before the warm-up, in ms of device time (0: none)")
    p.add_argument("--tune", action="append", default=[], metavar="NAME=VALUE",
                   help="kernel-variant knob on the workload's handle, e.g. FFT_WAVE1024=2 "
                        "(SDSP_TUNE_<NAME>, include/sdsp.h); A/B runs only, the default line uses none")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU-only rehearsal of the rank launch, timing and gather over gloo (no GPU)")
    return p.parse_args()


def load_traffic(config, log2n, algo, kernel=""):
    """(HBM bytes per launch of the dominant kernel, the summary file it came from)
    from the committed PMC pass (profiles/*/pmc_summary_cfg*.json written by
    tools/pmc_summary.py), or (None, None).  The summary must name the kernel this
    run launches (first word of `kernel`)."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*", f"pmc_summary_cfg{config}.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
            if (d.get("log2n") == log2n and d.get("algo", algo) == algo
                    and d.get("kernel", "") and kernel.split()[0].startswith(d["kernel"])):
                return d["hbm_bytes_per_launch"], os.path.relpath(path, REPO)
        except (OSError, ValueError, KeyError):
            pass
    return None, None


def stream_copy_gbps(torch, sd, nbytes=4 << 30, seconds=0.3):
    """Achievable HBM bandwidth on this box: one-shot 16-byte-per-lane device copy
    (read + write bytes / time), repeated for ~`seconds` of device time; the
    median of the second half of the repetitions (the first half lets the clocks
    settle)."""
    a = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    a.fill_(1.0)
    st = torch.cuda.current_stream()
    L = sd.lib()
    L.sdsp_bandwidth_copy_device(a.data_ptr(), b.data_ptr(), nbytes, st.cuda_stream)
    ts = []
    while len(ts) < 8 or (sum(ts) < seconds * 1e3 and len(ts) < 400):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        L.sdsp_bandwidth_copy_device(a.data_ptr(), b.data_ptr(), nbytes, st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    del a, b
    torch.cuda.empty_cache()
    return 2.0 * nbytes / (float(np.median(ts[len(ts) // 2:])) * 1e-3) / 1e9


def settle(w, stream, torch, ms=150.0, chunk=8):
    """Untimed steps of the workload itself, in back-to-back chunks, until `ms` of device
    time: the device's clock / power state takes tens of milliseconds of THIS load to
    settle after the copy phase (tools/steady_probe.py, profiles/r04/lab/: cfg5 runs
    0.44 ms per step for its first ~30 steps, 0.396 from then on for 400 steps; cfg3 1.83
    -> 1.72 ms; cfg2 3.35 -> 3.28), and a timed window of a few steps would otherwise land
    on that transient.  The timed steps that follow are the workload unchanged."""
    from solid_dsp_amd import parallel as P

    def run(k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            w.step(stream)
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1)

    n, t = 0, 0.0
    while True:
        t += run(chunk)
        n += chunk
        # every rank runs the same number of steps (a step may hold a collective: cfg3 --shard time)
        if P.max_over_ranks(float(t < ms), device="cuda") == 0.0:
            return {"steps": n, "ms": round(t, 1)}


def timed_cpu(run_chunk, label, samples, chunk, cores=1):
    """Stream `samples` inputs through CPU filter objects, `chunk` at a time (the
    same synthetic chunk re-fed, so host memory stays bounded).  cores > 1: one
    independent channel per thread (the restatement is C; ctypes releases the GIL),
    each thread streaming samples / cores."""
    reps = max(1, samples // (chunk * cores))
    t0 = time.perf_counter()
    if cores == 1:
        for _ in range(reps):
            run_chunk(0)
    else:
        from concurrent.futures import ThreadPoolExecutor

        def worker(c):
            for _ in range(reps):
                run_chunk(c)
        with ThreadPoolExecutor(cores) as ex:
            list(ex.map(worker, range(cores)))
    dt = time.perf_counter() - t0
    total = reps * chunk * cores
    return {"value": total / dt / 1e6, "unit": "Msamples/sec", "cores": cores, "kind": "port",
            "sample": f"{label}; {total} input samples streamed in {reps} execute_block calls of {chunk}, "
                      f"{cores} thread(s), {dt:.1f} s"}


# --------------------------------------------------------------------------- workloads
class StreamShard:
    """Configs 2 and 4: a stream per rank, or one stream time-sharded over the ranks."""

    def time_sharded(self, args, rank, torch, sd, P_halo, m_per_in=1):
        """input of this rank: its own channel (channel = rank), or with --shard time
        segment `rank` of ONE stream (channel 0) plus the halo of inputs before it
        (parallel.time_segment); the halo block is filtered first in every step and its
        outputs dropped, so the segment's outputs are the single stream's"""
        from solid_dsp_amd import parallel as P
        cs = torch.cuda.current_stream().cuda_stream
        self.shard = getattr(args, "shard", "channel")
        self.halo = 0
        if self.shard != "time":
            sd.lib().sdsp_synth_f32_device(self.d_in.data_ptr(), SEED, rank, 0, 2 * self.n, cs)
            return
        first, self.halo = P.time_segment(self.n, rank, P_halo(P))
        sd.lib().sdsp_synth_f32_device(self.d_in.data_ptr(), SEED, 0, 2 * rank * self.n, 2 * self.n, cs)
        self.d_halo = torch.empty(max(self.halo, 1), dtype=torch.complex64, device="cuda")
        self.d_halo_out = torch.empty(max(self.halo // m_per_in, 1), dtype=torch.complex64, device="cuda")
        if self.halo:
            sd.lib().sdsp_synth_f32_device(self.d_halo.data_ptr(), SEED, 0, 2 * first, 2 * self.halo, cs)
        self.parallelism = ("one stream (channel 0) time-sharded: rank r filters inputs [r n, (r+1) n) after a "
                            f"{P_halo(P)}-input halo, no exchange")

    def step(self, stream):
        if self.halo:  # time-sharded: the delay line from the segment's halo
            self.f.execute_block_device(self.d_halo, self.halo, self.d_halo_out, stream)
        self.f.execute_block_device(self.d_in, self.n, self.d_out, stream)


class Cfg2FIR(StreamShard):
    """256-tap crcf FIR, firdes_kaiser(256, 0.1, 80) taps rounded to f32, scale 0.2."""
    metric = "Msamples/sec 256-tap complex FIR @1/2/4/8 GPU; % HBM roofline"
    taps = 256
    tol = 1e-6

    def __init__(self, args, rank, dev, torch, sd):
        from solid_dsp_amd import FIRFilter
        from solid_dsp_amd.filter import firdes
        self.n = 1 << args.log2n
        self.h = firdes.firdes_kaiser(self.taps, 0.1, 80.0, 0.0).astype(np.float32)
        self.algo = {"fft": sd.ALGO_FFT, "exact": sd.ALGO_EXACT, "fma": sd.ALGO_FMA}[args.algo]
        self.algo_name = args.algo
        self.f = FIRFilter(self.h, np.float32(0.2), sample_dtype=np.complex64, device=dev, algo=self.algo)
        self.make = lambda: FIRFilter(self.h, np.float32(0.2), sample_dtype=np.complex64, device=dev, algo=self.algo)
        self.d_in = torch.empty(self.n, dtype=torch.complex64, device="cuda")
        self.d_out = torch.empty(self.n, dtype=torch.complex64, device="cuda")
        self.time_sharded(args, rank, torch, sd, P_halo=lambda P: P.fir_halo(self.taps))
        self.samples_per_step = self.n
        self.bytes_per_step = 16 * self.n
        self.dtype = "c32 (f32 taps x complex-f32 samples, f32 accumulate)"
        self.kernel = {"fft": "fir_ols_os_kernel<true, false, false> (one-shot XCD-ordered packed-FP32 overlap-save N=4096, "
                              "fused DFT16, one segment per workgroup, 4 workgroups/CU, one halo row compiled in) + "
                              "fir_ols_os_kernel<false, false, true> (the 2 boundary "
                              "segments and the next history, a second launch)",
                       "exact": "fir_direct_kernel<EXACT>",
                       "fma": "fir_direct_kernel<FMA>"}[args.algo]
        self.workload = (f"cfg2: 256-tap crcf FIR, firdes_kaiser(256, 0.1, 80), scale 0.2, 2^{args.log2n} samples "
                         "per channel, device resident")

    def parity(self, stream, rng, windows=4, width=4096):
        """random output windows recomputed on the CPU (f64 restatement) from the L-1 preceding inputs"""
        import oracle_lib as O
        import torch
        g = self.make()
        g.execute_block_device(self.d_in, self.n, self.d_out, stream)
        torch.cuda.synchronize()
        worst = 0.0
        L = self.taps
        for _ in range(windows):
            s = int(rng.integers(L, self.n - width))
            xs = self.d_in[s - (L - 1): s + width].cpu().numpy()
            ys = self.d_out[s: s + width].cpu().numpy()
            ref = O.fir(O.RC64, self.h.astype(np.float64), 0.2).execute_block(xs.astype(np.complex128))[L - 1:]
            worst = max(worst, float(np.linalg.norm(ys - ref) / np.linalg.norm(ref)))
        return worst

    @staticmethod
    def expected(h, r, s, width):
        """outputs [s, s + width) of channel r, recomputed by the f64 restatement from the
        channel's synthetic inputs (parallel.fir_input_window)"""
        import oracle_lib as O
        from solid_dsp_amd import parallel as P
        first, count, drop = P.fir_input_window(s, width, len(h))
        xs = O.synth(SEED, r, first, count, complex_=True).astype(np.complex128)
        return O.fir(O.RC64, np.asarray(h, np.float64), 0.2).execute_block(xs)[drop:]

    def check_gathered(self, big, rng, width=4096):
        """every rank's gathered output (channel = rank): two random windows each; time-sharded:
        windows of the one stream inside every segment and across every segment boundary"""
        from solid_dsp_amd import parallel as P
        if self.shard == "time":
            return P.check_time_sharded(big, lambda g, w: Cfg2FIR.expected(self.h, 0, g, w), rng, width, self.taps)
        return P.check_gathered(big, lambda r, s, w: Cfg2FIR.expected(self.h, r, s, w), rng, width, self.taps,
                                self.n)

    def cpu(self, samples):
        import oracle_lib as O
        x = O.synth(SEED, 0, 0, CPU_CHUNK, complex_=True).astype(np.complex128)
        f = O.fir(O.RC64, self.h.astype(np.float64), 0.2)
        return timed_cpu(lambda c: f.execute_block(x), "FIRFilter<f64, Complex<f64>> restatement (memmove Window + "
                         "to_vec + sequential dot)", samples, CPU_CHUNK)


class Cfg3IIR:
    """4-section SOS cascade, scipy butter(8, 0.2), real f32 stream, block-parallel scan."""
    metric = "Msamples/sec 4-stage IIR biquad cascade (f32, 1 GiS); % HBM roofline"
    tol = 1e-5

    def __init__(self, args, rank, dev, torch, sd):
        from solid_dsp_amd import IIRFilter, IIRFilterType
        sos = np.array(json.load(open(os.path.join(REPO, "tests", "golden", "butter8_0p2_sos.json")))["sos"])
        self.ff = sos[:, :3].reshape(-1).astype(np.float32)
        self.fb = sos[:, 3:].reshape(-1).astype(np.float32)
        self.n = 1 << args.log2n
        self.f = IIRFilter(self.ff, self.fb, IIRFilterType.SecondOrder, sample_dtype=np.float32, device=dev,
                           algo=sd.ALGO_FMA)
        self.d_in = torch.empty(self.n, dtype=torch.float32, device="cuda")
        self.d_out = torch.empty(self.n, dtype=torch.float32, device="cuda")
        self.shard = getattr(args, "shard", "channel")
        self.rank = rank
        cs = torch.cuda.current_stream().cuda_stream
        if self.shard == "time":
            # segment `rank` of ONE stream (channel 0), joined to the segments before it by one
            # exchange of the boundary states (parallel.iir_exclusive_scan)
            from solid_dsp_amd import parallel as P
            sd.lib().sdsp_synth_f32_device(self.d_in.data_ptr(), SEED, 0, rank * self.n, self.n, cs)
            A, _, c, _ = P.sos_state_space(self.ff, self.fb)
            self.Phi = P.state_transition(A, self.n)
            self.W = P.zero_input_length(A, c, self.n)
            self.g = IIRFilter(self.ff, self.fb, IIRFilterType.SecondOrder, sample_dtype=np.float32, device=dev,
                               algo=sd.ALGO_FMA)
            self.d_zero = torch.zeros(self.W, dtype=torch.float32, device="cuda")
            self.d_corr = torch.empty(self.W, dtype=torch.float32, device="cuda")
            self.parallelism = ("one stream (channel 0) time-sharded: rank r filters inputs [r n, (r+1) n) from zero "
                                "state, one all_gather of the 8 boundary-state values, exclusive scan of the states "
                                f"and the zero-input response of the true initial state added to the first {self.W} "
                                "outputs")
        else:
            sd.lib().sdsp_synth_f32_device(self.d_in.data_ptr(), SEED, rank, 0, self.n, cs)
        self.samples_per_step = self.n
        self.bytes_per_step = 8 * self.n
        self.dtype = "f32 (f32 coefficients, real f32 samples)"
        self.kernel = "sos_wscan_kernel<4> (wave-level scan, 128-byte chunks, state-response correction)"
        self.workload = f"cfg3: 4-biquad SOS cascade butter(8, 0.2), real f32, 2^{args.log2n} samples per channel"
        self.algo_name = "scan"

    def step(self, stream):
        if self.shard != "time":
            self.f.execute_block_device(self.d_in, self.n, self.d_out, stream)
            return
        # time shard: the segment from zero state, the boundary-state exchange, the correction
        import torch
        from solid_dsp_amd import parallel as P
        self.f.reset()  # every timed step re-runs the same segment from zero state
        self.f.execute_block_device(self.d_in, self.n, self.d_out, stream)
        s_r, _ = self.f.get_state()  # waits for the block
        init = P.iir_exclusive_scan(P.exchange_states(s_r.astype(np.float64), device="cuda"), self.Phi)[self.rank]
        self.g.set_state(init.astype(np.float32))
        self.g.execute_block_device(self.d_zero, self.W, self.d_corr, stream)
        with torch.cuda.stream(stream):
            self.d_out[: self.W] += self.d_corr

    def parity(self, stream, rng):
        import oracle_lib as O
        import torch
        if self.shard == "time" and self.rank != 0:
            return None  # rank 0 holds the stream's start; the gathered check covers the others
        m = 1 << 20  # the first 2^20 outputs of a fresh pass vs the f64 restatement (IIR: full prefix)
        from solid_dsp_amd import IIRFilter, IIRFilterType
        import solid_dsp_amd as sd
        g = IIRFilter(self.ff, self.fb, IIRFilterType.SecondOrder, sample_dtype=np.float32, algo=sd.ALGO_FMA)
        g.execute_block_device(self.d_in, self.n, self.d_out, stream)
        torch.cuda.synchronize()
        x = self.d_in[:m].cpu().numpy().astype(np.float64)
        y = self.d_out[:m].cpu().numpy()
        ref = O.iir(O.RR64, self.ff.astype(np.float64), self.fb.astype(np.float64), O.SECOND_ORDER).execute_block(x)
        return float(np.linalg.norm(y - ref) / np.linalg.norm(ref))

    def output(self):
        return self.d_out

    # the cascade's state response decays as max|pole|^k = 0.891^k: 0.891^2048 ~ 1e-103, so an
    # output window recomputed from 2048 inputs before it (zero state) equals the whole-stream
    # f64 recurrence far below f32 rounding
    WARM = 2048

    @staticmethod
    def expected(ff, fb, r, s, width):
        """outputs [s, s + width) of channel r in f64: the restatement over the channel's
        synthetic inputs from max(s - WARM, 0), zero state (IIR channel shards)"""
        import oracle_lib as O
        a = max(s - Cfg3IIR.WARM, 0)
        x = O.synth(SEED, r, a, s + width - a).astype(np.float64)
        f = O.iir(O.RR64, np.asarray(ff, np.float64), np.asarray(fb, np.float64), O.SECOND_ORDER)
        return f.execute_block(x)[s - a:]

    @staticmethod
    def check(big, ff, fb, n, rng, width=4096):
        """every rank's gathered output (channel = rank): two random windows each"""
        from solid_dsp_amd import parallel as P
        return P.check_gathered(big, lambda r, s, w: Cfg3IIR.expected(ff, fb, r, s, w), rng, width, 0, n)

    def check_gathered(self, big, rng, width=4096):
        """channel shards: two random windows of every rank's channel; time shards: windows of
        the one stream inside every segment and across every segment boundary"""
        from solid_dsp_amd import parallel as P
        if self.shard == "time":
            return P.check_time_sharded(big, lambda g, w: Cfg3IIR.expected(self.ff, self.fb, 0, g, w), rng, width, 0)
        return Cfg3IIR.check(big, self.ff, self.fb, self.n, rng, width)

    def cpu(self, samples):
        import oracle_lib as O
        x = O.synth(SEED, 0, 0, CPU_CHUNK).astype(np.float64)
        f = O.iir(O.RR64, self.ff.astype(np.float64), self.fb.astype(np.float64), O.SECOND_ORDER)
        return timed_cpu(lambda c: f.execute_block(x), "IIRFilter<f64, f64> SecondOrder restatement", samples,
                         CPU_CHUNK)


class Cfg4Decim(StreamShard):
    """M=32 decimator, firdes_kaiser(256, 1/64, 80) rounded to f32, scale 1/32, crcf."""
    metric = "Msamples/sec 32-branch polyphase decimator (M=32, 8 taps/branch); % HBM roofline"
    tol = 1e-6

    def __init__(self, args, rank, dev, torch, sd):
        from solid_dsp_amd import DecimatingFIRFilter
        from solid_dsp_amd.filter import firdes
        self.n = 1 << args.log2n
        self.h = firdes.firdes_kaiser(256, 1.0 / 64, 80.0, 0.0).astype(np.float32)
        self.f = DecimatingFIRFilter(self.h, np.float32(1.0 / 32), 32, sample_dtype=np.complex64, device=dev,
                                     algo=sd.ALGO_FMA)
        self.d_in = torch.empty(self.n, dtype=torch.complex64, device="cuda")
        self.d_out = torch.empty(self.n // 32 + 1, dtype=torch.complex64, device="cuda")
        self.time_sharded(args, rank, torch, sd, P_halo=lambda P: P.decim_halo(256, 32), m_per_in=32)
        self.samples_per_step = self.n
        self.bytes_per_step = 8 * self.n + 8 * (self.n // 32)
        self.dtype = "c32 (f32 taps x complex-f32 samples)"
        self.kernel = "decim_poly_kernel (column-parallel polyphase, fused multiply-add)"
        self.workload = f"cfg4: M=32 x 8-tap polyphase decimator, crcf, 2^{args.log2n} input samples per channel"
        self.algo_name = "fma"

    def parity(self, stream, rng, width=4096):
        """random windows of outputs recomputed in f64 from the definition
        y[m] = scale * sum_j h[j] x[32m + 31 - 255 + j]  (fresh handle: first output after input 31)"""
        import torch
        from numpy.lib.stride_tricks import sliding_window_view
        from solid_dsp_amd import DecimatingFIRFilter
        import solid_dsp_amd as sd
        g = DecimatingFIRFilter(self.h, np.float32(1.0 / 32), 32, sample_dtype=np.complex64, algo=sd.ALGO_FMA)
        g.execute_block_device(self.d_in, self.n, self.d_out, stream)
        torch.cuda.synchronize()
        h = self.h.astype(np.float64)
        worst = 0.0
        for _ in range(4):
            m = int(rng.integers(8, self.n // 32 - width))
            xs = self.d_in[32 * m - 224: 32 * (m + width)].cpu().numpy().astype(np.complex128)
            ref = sliding_window_view(xs, 256)[::32][:width] @ h / 32.0
            ys = self.d_out[m: m + width].cpu().numpy()
            worst = max(worst, float(np.linalg.norm(ys - ref) / np.linalg.norm(ref)))
        return worst

    def output(self):
        return self.d_out[: self.n // 32]

    @staticmethod
    def expected(h, r, m, width):
        """decimated outputs [m, m + width) of channel r in f64 from the definition
        y[m] = scale sum_j h[j] x[32 m + 31 - 255 + j] (parallel.decim_input_window)"""
        from numpy.lib.stride_tricks import sliding_window_view
        import oracle_lib as O
        from solid_dsp_amd import parallel as P
        first, count = P.decim_input_window(m, width, len(h), 32)
        xs = O.synth(SEED, r, first, count, complex_=True).astype(np.complex128)
        return sliding_window_view(xs, len(h))[::32][:width] @ np.asarray(h, np.float64) / 32.0

    def check_gathered(self, big, rng, width=4096):
        """every rank's gathered decimated output (channel = rank), two random windows each;
        time-sharded: windows of the one stream inside and across the segments"""
        from solid_dsp_amd import parallel as P
        if self.shard == "time":
            return P.check_time_sharded(big, lambda g, w: Cfg4Decim.expected(self.h, 0, g, w), rng, width, 8)
        return P.check_gathered(big, lambda r, m, w: Cfg4Decim.expected(self.h, r, m, w), rng, width, 8,
                                self.n // 32)

    def cpu(self, samples):
        import oracle_lib as O
        x = O.synth(SEED, 0, 0, CPU_CHUNK, complex_=True).astype(np.complex128)
        f = O.decim(O.RC64, self.h.astype(np.float64), 1.0 / 32, 32)
        return timed_cpu(lambda c: f.execute_block(x), "DecimatingFIRFilter<f64, Complex<f64>> restatement",
                         samples, CPU_CHUNK)


class Cfg5Chan:
    """1024-channel PFB + FFT, prototype firdes_kaiser(8192, 1/2048, 80), 8 streams x 2^24 per GPU."""
    metric = "Msamples/sec 1024-channel PFB + FFT channeliser (8 streams/GPU); % HBM roofline"

    def __init__(self, args, rank, dev, torch, sd):
        from solid_dsp_amd import Channelizer
        from solid_dsp_amd.filter import firdes
        self.M, self.S = 1024, 8
        self.n = 1 << 24
        self.h = firdes.firdes_kaiser(8192, 1.0 / 2048, 80.0, 0.0).astype(np.float32)
        self.f = Channelizer(self.h, self.M, sample_dtype=np.complex64, device=dev, streams=self.S)
        self.d_in = torch.empty(self.S * self.n, dtype=torch.complex64, device="cuda")
        self.d_out = torch.empty(self.S * self.n, dtype=torch.complex64, device="cuda")
        from solid_dsp_amd import parallel as P
        for s, ch in enumerate(P.channel_ids(self.S, 1, rank)):  # streams rank*S .. rank*S+S-1
            sd.lib().sdsp_synth_f32_device(self.d_in[s * self.n:].data_ptr(), SEED, ch, 0, 2 * self.n,
                                           torch.cuda.current_stream().cuda_stream)
        self.samples_per_step = self.S * self.n
        self.bytes_per_step = 16 * self.S * self.n
        self.dtype = "c32 (f32 taps x complex-f32 samples)"
        self.kernel = ("chan1024_kernel<8, 1024, prefetch, 8> (streaming PFB in registers, rounds of 8 frames, "
                       "next round's samples requested before this round's stores, packed-FP32 16x16x4 FFT with "
                       "one swizzled LDS transpose and a row-swap DFT4)")
        self.workload = "cfg5: 1024-channel PFB (K=8) + 1024-pt FFT, 8 streams x 2^24 samples per GPU"
        self.algo_name = "chan"

    def step(self, stream):
        self.f.execute_block_device(self.d_in, self.n, self.d_out, stream)

    def parity(self, stream, rng):
        import oracle_lib as O
        import torch
        from solid_dsp_amd import Channelizer
        g = Channelizer(self.h, self.M, sample_dtype=np.complex64, streams=self.S)
        g.execute_block_device(self.d_in, self.n, self.d_out, stream)
        torch.cuda.synchronize()
        fr = 64  # first 64 frames of stream 0
        x = self.d_in[: fr * self.M].cpu().numpy().astype(np.complex128)
        y = self.d_out[: fr * self.M].cpu().numpy()
        ref = np.zeros(fr * self.M, np.complex128)
        O.lib().orc_channelize(O._ptr(self.h.astype(np.float64)), len(self.h), self.M, O._ptr(x), len(x), O._ptr(ref))
        return float(np.linalg.norm(y - ref) / np.linalg.norm(ref))

    def output(self):
        return self.d_out  # [S streams][n]: the rank's streams rank S .. rank S + S - 1

    @staticmethod
    def expected(h, M, ch, s, width):
        """channeliser outputs [s, s + width) of stream ch (frame-major, out[frame][M]) in f64: a
        fresh restatement over the stream's synthetic inputs from K - 1 frames before the
        first frame the window touches (frame m depends on input frames m - K + 1 .. m)"""
        import oracle_lib as O
        K = len(h) // M
        f0, f1 = s // M, -(-(s + width) // M)
        a = max(f0 - (K - 1), 0)
        x = O.synth(SEED, ch, a * M, (f1 - a) * M, complex_=True).astype(np.complex128)
        ref = np.zeros(len(x), np.complex128)
        hh = np.asarray(h, np.float64)
        O.lib().orc_channelize(O._ptr(hh), len(hh), M, O._ptr(x), len(x), O._ptr(ref))
        return ref[s - a * M: s - a * M + width]

    @staticmethod
    def check(big, h, M, S, n, rng, width=8192):
        """every stream of every rank's gathered output (rank r holds streams r S .. r S + S - 1,
        parallel.channel_ids): two random windows each"""
        from solid_dsp_amd import parallel as P
        rows = big.reshape(big.shape[0] * S, n)  # row j = stream j
        return P.check_gathered(rows, lambda j, s, w: Cfg5Chan.expected(h, M, j, s, w), rng, width, 0, n)

    def check_gathered(self, big, rng, width=8192):
        return Cfg5Chan.check(big, self.h, self.M, self.S, self.n, rng, width)

    def cpu(self, samples):
        """8 streams on min(8, host cores) threads, one stream per thread."""
        import oracle_lib as O
        chunk = CPU_CHUNK // self.M * self.M
        cores = max(1, min(self.S, os.cpu_count() or 1))
        xs = [O.synth(SEED, c, 0, chunk, complex_=True).astype(np.complex128) for c in range(cores)]
        outs = [np.zeros(chunk, np.complex128) for _ in range(cores)]
        h = self.h.astype(np.float64)
        # each call is a fresh channeliser over the chunk (the restatement has no carried state)
        return timed_cpu(lambda c: O.lib().orc_channelize(O._ptr(h), len(h), self.M, O._ptr(xs[c]), chunk,
                                                          O._ptr(outs[c])),
                         "channeliser restatement (PFB DotProducts + reference mixed-radix FFT)", samples, chunk,
                         cores)


class Cfg1FIR:
    """cfg1 plumbing case: 63-tap real f32 FIR, firdes_kaiser(63, 0.2, 60), 2^20 samples,
    reference-order EXACT kernel (bit-identical to the f32 restatement)."""
    metric = "Msamples/sec 63-tap real-f32 FIR, 1 MiS (plumbing case)"
    tol = 0

    def __init__(self, args, rank, dev, torch, sd):
        from solid_dsp_amd import FIRFilter
        from solid_dsp_amd.filter import firdes
        self.n = 1 << 20
        self.h = firdes.firdes_kaiser(63, 0.2, 60.0, 0.0).astype(np.float32)
        self.f = FIRFilter(self.h, np.float32(1.0), sample_dtype=np.float32, device=dev, algo=sd.ALGO_EXACT)
        self.d_in = torch.empty(self.n, dtype=torch.float32, device="cuda")
        self.d_out = torch.empty(self.n, dtype=torch.float32, device="cuda")
        sd.lib().sdsp_synth_f32_device(self.d_in.data_ptr(), SEED, rank, 0, self.n,
                                       torch.cuda.current_stream().cuda_stream)
        self.samples_per_step = self.n
        self.bytes_per_step = 8 * self.n
        self.dtype = "f32 (f32 taps x real f32 samples, reference summation order)"
        self.kernel = "fir_direct_kernel<EXACT>"
        self.parity_check = "bit mismatches vs the f32 restatement, whole stream (must be 0)"
        self.workload = "cfg1: 63-tap real f32 FIR, firdes_kaiser(63, 0.2, 60), 2^20 samples"
        self.algo_name = "exact"

    def step(self, stream):
        self.f.execute_block_device(self.d_in, self.n, self.d_out, stream)

    def parity(self, stream, rng):
        """bit-exact against the f32 restatement over the whole stream (fresh handle)"""
        import oracle_lib as O
        import torch
        from solid_dsp_amd import FIRFilter
        import solid_dsp_amd as sd
        g = FIRFilter(self.h, np.float32(1.0), sample_dtype=np.float32, algo=sd.ALGO_EXACT)
        g.execute_block_device(self.d_in, self.n, self.d_out, stream)
        torch.cuda.synchronize()
        x = self.d_in.cpu().numpy()
        y = self.d_out.cpu().numpy()
        ref = O.fir(O.RR32, self.h, np.float32(1.0)).execute_block(x)
        return float(np.count_nonzero(y.view(np.uint32) != ref.view(np.uint32)))

    def cpu(self, samples):
        import oracle_lib as O
        x = O.synth(SEED, 0, 0, CPU_CHUNK).astype(np.float64)
        f = O.fir(O.RR64, self.h.astype(np.float64), 1.0)
        return timed_cpu(lambda c: f.execute_block(x), "FIRFilter<f64, f64> restatement (memmove Window + to_vec + "
                         "sequential dot)", samples, CPU_CHUNK)


class Cfg6ACorr:
    """AutoCorrelator(window 64, delay 16), Complex<f32>, 2^29 samples: one read of x and
    one write of y per sample (src/filter/auto_correlator/mod.rs:181-191)."""
    metric = "Msamples/sec AutoCorrelator(64, 16) execute_block, c32; % HBM roofline"
    tol = 0

    def __init__(self, args, rank, dev, torch, sd):
        self.W, self.D = 64, 16
        self.n = 1 << min(args.log2n, 29)
        self.f = sd.AutoCorrelator(self.W, self.D, dtype=np.complex64, device=dev)
        self.d_in = torch.empty(self.n, dtype=torch.complex64, device="cuda")
        self.d_out = torch.empty(self.n, dtype=torch.complex64, device="cuda")
        sd.lib().sdsp_synth_f32_device(self.d_in.data_ptr(), SEED, rank, 0, 2 * self.n,
                                       torch.cuda.current_stream().cuda_stream)
        self.samples_per_step = self.n
        self.bytes_per_step = 16 * self.n
        self.dtype = "c32 (complex-f32 products and sums, f64 energy)"
        self.kernel = ("acorr_pipe_kernel<float> (persistent one-wave workgroups over tiles of 512 outputs, 8 per lane, the "
                       "next tile's inputs loaded across this tile's sums; LDS-staged conj products) + edge tiles + energy + history")
        self.parity_check = "bit mismatches vs the c32 restatement over the first 2^20 outputs (must be 0)"
        self.workload = f"cfg6: AutoCorrelator(64, 16), c32, 2^{int(np.log2(self.n))} samples per channel"
        self.algo_name = "acorr"

    def step(self, stream):
        self.f.execute_block_device(self.d_in, self.n, self.d_out, stream)

    def parity(self, stream, rng):
        import oracle_lib as O
        import torch
        import solid_dsp_amd as sd
        m = 1 << 20
        g = sd.AutoCorrelator(self.W, self.D, dtype=np.complex64)
        g.execute_block_device(self.d_in, m, self.d_out, stream)
        torch.cuda.synchronize()
        x = self.d_in[:m].cpu().numpy()
        y = self.d_out[:m].cpu().numpy()
        ref = O.AutoCorr(self.W, self.D, np.complex64).execute_block(x)
        return float(np.count_nonzero(y.view(np.uint64) != ref.view(np.uint64)))

    def cpu(self, samples):
        import oracle_lib as O
        chunk = CPU_CHUNK // 4
        x = O.synth(SEED, 0, 0, chunk, complex_=True).astype(np.complex128)
        f = O.AutoCorr(self.W, self.D, np.complex128)
        return timed_cpu(lambda c: f.execute_block(x), "AutoCorrelator<f64> restatement (two Windows, memmove push, "
                         "to_vec + zip sum per sample)", samples, chunk)


class Cfg7NCO:
    """NCO mix_down of a Complex<f32> stream, frequency 2 pi 0.0123 (src/nco/mod.rs:147-172)."""
    metric = "Msamples/sec NCO mix_down, c32; % HBM roofline"

    def __init__(self, args, rank, dev, torch, sd):
        self.n = 1 << args.log2n
        self.freq = 2 * np.pi * 0.0123
        self.f = sd.NCO(device=dev)
        self.f.set_frequency(self.freq)
        self.d_in = torch.empty(self.n, dtype=torch.complex64, device="cuda")
        self.d_out = torch.empty(self.n, dtype=torch.complex64, device="cuda")
        sd.lib().sdsp_synth_f32_device(self.d_in.data_ptr(), SEED, rank, 0, 2 * self.n,
                                       torch.cuda.current_stream().cuda_stream)
        self.samples_per_step = self.n
        self.bytes_per_step = 16 * self.n
        self.dtype = "c32 (f32 copy of the f64 sine table, complex-f32 product)"
        self.kernel = "nco_mix_kernel<float, true> (u32 phase per sample, LDS sine table)"
        self.parity_check = "rel_rms vs the f64 restatement over the first 2^20 outputs (tolerance 1e-6)"
        self.workload = f"cfg7: NCO mix_down, dtheta = constrain(2 pi 0.0123), c32, 2^{args.log2n} samples"
        self.algo_name = "nco"

    def step(self, stream):
        self.f.mix_block_device(self.d_in, self.n, self.d_out, down=True, precision=0, stream=stream)

    def parity(self, stream, rng):
        import oracle_lib as O
        import torch
        import solid_dsp_amd as sd
        m = 1 << 20
        g = sd.NCO()
        g.set_frequency(self.freq)
        g.mix_block_device(self.d_in, m, self.d_out, down=True, precision=0, stream=stream)
        torch.cuda.synchronize()
        x = self.d_in[:m].cpu().numpy().astype(np.complex128)
        y = self.d_out[:m].cpu().numpy()
        o = O.Nco()
        o.set_frequency(self.freq)
        ref = o.mix_block(x, True)
        return float(np.linalg.norm(y - ref) / np.linalg.norm(ref))

    def cpu(self, samples):
        import oracle_lib as O
        x = O.synth(SEED, 0, 0, CPU_CHUNK, complex_=True).astype(np.complex128)
        o = O.Nco()
        o.set_frequency(self.freq)
        return timed_cpu(lambda c: o.mix_block(x, True), "NCO restatement (table lookup + mix_down + step per "
                         "sample, f64)", samples, CPU_CHUNK)


class Cfg8FFT:
    """Batched 2^20-point forward FFT, Complex<f32>, 256 transforms per step (src/fft/mod.rs)."""
    metric = "Msamples/sec batched 2^20-point FFT, c32; % HBM roofline"
    tol = 5e-6

    def __init__(self, args, rank, dev, torch, sd):
        from solid_dsp_amd import FFT, FFTDirection
        self.N = 1 << 20
        self.n = 1 << min(args.log2n, 28)
        self.batch = self.n // self.N
        self.f = FFT(self.N, FFTDirection.FORWARD, precision=np.complex64, device=dev)
        self.d_in = torch.empty(self.n, dtype=torch.complex64, device="cuda")
        self.d_out = torch.empty(self.n, dtype=torch.complex64, device="cuda")
        sd.lib().sdsp_synth_f32_device(self.d_in.data_ptr(), SEED, rank, 0, 2 * self.n,
                                       torch.cuda.current_stream().cuda_stream)
        self.samples_per_step = self.n
        # algorithmic bytes: one read and one write of every sample; the four-step
        # plan makes two passes, so its floor is 2x this
        self.bytes_per_step = 16 * self.n
        self.dtype = "c32 (complex-f32 butterflies, f64-derived twiddles)"
        self.kernel = "fft1024_pipe_kernel x2 (four-step 1024 x 1024 on the wave-level register FFT, 16 transforms per step of a persistent, load-pipelined workgroup per CU; the column pass loads its strided side in 16-byte lanes)"
        self.parity_check = "rel_rms of transform 0 vs numpy f64 (tolerance 5e-6)"
        self.workload = f"cfg8: {self.batch} x 2^20-point forward FFT, c32, out of place"
        self.algo_name = "fft"

    def step(self, stream):
        self.f.execute_device(self.d_in, self.d_out, self.batch, stream)

    def parity(self, stream, rng):
        import torch
        self.step(stream)
        torch.cuda.synchronize()
        x = self.d_in[: self.N].cpu().numpy().astype(np.complex128)
        y = self.d_out[: self.N].cpu().numpy()
        ref = np.fft.fft(x)
        return float(np.linalg.norm(y - ref) / np.linalg.norm(ref))

    def cpu(self, samples):
        import oracle_lib as O
        L = O.lib()
        h = L.orc_fft_new(self.N, 0)
        x = O.synth(SEED, 0, 0, self.N, complex_=True).astype(np.complex128)
        y = np.zeros(self.N, np.complex128)
        try:
            return timed_cpu(lambda c: L.orc_fft_execute(h, O._ptr(x), O._ptr(y)),
                             "FFT restatement (reference mixed-radix planner, f64), one 2^20 transform per call",
                             samples, self.N)
        finally:
            L.orc_fft_free(h)


class Cfg9AGC:
    """AGC bank: 2^18 independent AGC(bandwidth 0.02, squelch -30 dB) channels x 2^10
    Complex<f64> samples (src/auto_gain_control/mod.rs:214-285); one lane per channel."""
    metric = "Msamples/sec AGC execute_block, Complex<f64>, 2^18 channels; % HBM roofline"
    tol = 1e-12

    def __init__(self, args, rank, dev, torch, sd):
        self.ch, self.n = 1 << 18, 1 << 10
        self.f = self._make(sd, dev)
        total = self.ch * self.n
        self.d_in = torch.empty(total, dtype=torch.complex128, device="cuda")
        self.d_out = torch.empty(total, dtype=torch.complex128, device="cuda")
        tmp = torch.empty(2 * total, dtype=torch.float32, device="cuda")
        sd.lib().sdsp_synth_f32_device(tmp.data_ptr(), SEED, rank, 0, 2 * total, torch.cuda.current_stream().cuda_stream)
        self.d_in.copy_(torch.view_as_complex(tmp.view(-1, 2).to(torch.float64) * 0.05))
        del tmp
        self.samples_per_step = total
        self.bytes_per_step = 32 * total
        self.dtype = "c64 (f64 gain recurrence with exp/ln/log10 per sample)"
        self.kernel = "agc_pipe_kernel<true, 16> (one lane per channel, 16-sample LDS runs, next run prefetched)"
        self.parity_check = "max |y - ref| / max |ref| over the first 64 channels vs the f64 restatement (tolerance 1e-12)"
        self.workload = "cfg9: AGC(bw 0.02, squelch -30 dB) bank, 2^18 channels x 2^10 Complex<f64> samples"
        self.algo_name = "agc"

    @staticmethod
    def _make(sd, dev=0):
        f = sd.AGC(channels=1 << 18, device=dev)
        f.set_bandwidth(0.02)
        f.squelch_enable()
        f.squelch_set_threshold(-30.0)
        return f

    def step(self, stream):
        self.f.execute_block_device(self.d_in, self.n, self.d_out, complex_=True, stream=stream)

    def parity(self, stream, rng):
        import oracle_lib as O
        import torch
        import solid_dsp_amd as sd
        g = self._make(sd)
        g.execute_block_device(self.d_in, self.n, self.d_out, complex_=True, stream=stream)
        torch.cuda.synchronize()
        m = 64 * self.n
        x = self.d_in[:m].cpu().numpy().reshape(64, self.n)
        y = self.d_out[:m].cpu().numpy().reshape(64, self.n)
        worst = 0.0
        for c in range(64):
            o = O.Agc()
            o.set_bandwidth(0.02)
            o.squelch(1)
            o.squelch_set_threshold(-30.0)
            r = o.execute_block(x[c])
            worst = max(worst, float(np.max(np.abs(y[c] - r)) / np.max(np.abs(r))))
        return worst

    def cpu(self, samples):
        import oracle_lib as O
        x = (O.synth(SEED, 0, 0, CPU_CHUNK // 4, complex_=True).astype(np.complex128) * 0.05)
        o = O.Agc()
        o.set_bandwidth(0.02)
        o.squelch(1)
        o.squelch_set_threshold(-30.0)
        return timed_cpu(lambda c: o.execute_block(x), "AGC<Complex<f64>> restatement (execute per sample, "
                         "libm exp/ln/log10)", samples, CPU_CHUNK // 4)


class Cfg10Interp:
    """M=32 interpolator, firdes_kaiser(256, 1/64, 80) rounded to f32 (K = 8 taps per branch),
    crcf, 2^25 inputs -> 2^30 outputs per GPU (src/filter/fir/interp.rs:102-111)."""
    metric = "Msamples/sec (outputs) 32x interpolating FIR, 8 taps/branch, crcf; % HBM roofline"
    tol = 1e-6

    def __init__(self, args, rank, dev, torch, sd):
        from solid_dsp_amd import InterpolatingFIRFilter
        from solid_dsp_amd.filter import firdes
        self.M = 32
        self.n = 1 << (args.log2n - 5)
        self.h = firdes.firdes_kaiser(256, 1.0 / 64, 80.0, 0.0).astype(np.float32)
        self.make = lambda d=dev: InterpolatingFIRFilter(self.h, self.M, sample_dtype=np.complex64, device=d)
        self.f = self.make()
        self.d_in = torch.empty(self.n, dtype=torch.complex64, device="cuda")
        self.d_out = torch.empty(self.n * self.M, dtype=torch.complex64, device="cuda")
        sd.lib().sdsp_synth_f32_device(self.d_in.data_ptr(), SEED, rank, 0, 2 * self.n,
                                       torch.cuda.current_stream().cuda_stream)
        self.samples_per_step = self.n * self.M
        self.bytes_per_step = 8 * self.n + 8 * self.n * self.M
        self.dtype = "c32 (f32 taps x complex-f32 samples, reference summation order)"
        self.kernel = "interp_tile_kernel<float, c32, EXACT, 8> (LDS-staged inputs, branch pairs in registers, 16-byte stores)"
        self.parity_check = "rel_rms of 4 random 4096-output windows vs the f64 restatement (tolerance 1e-6)"
        self.workload = f"cfg10: InterpolatingFIRFilter M=32, 256 taps (K=8), crcf, 2^{args.log2n - 5} inputs per channel"
        self.algo_name = "interp"

    def step(self, stream):
        self.f.execute_block_device(self.d_in, self.n, self.d_out, stream)

    def _ref(self, x, j0, count):
        """outputs for inputs j0 .. j0+count-1 from x[j0-7 .. j0+count) in f64 (zero before 0)"""
        import oracle_lib as O
        g = O.interp(O.RC64, self.h.astype(np.float64), self.M)
        return g.execute_block(x.astype(np.complex128))[7 * self.M:]

    def parity(self, stream, rng, windows=4, width=128):
        import torch
        g = self.make()
        g.execute_block_device(self.d_in, self.n, self.d_out, stream)
        torch.cuda.synchronize()
        worst = 0.0
        for _ in range(windows):
            j = int(rng.integers(8, self.n - width))
            xs = self.d_in[j - 7: j + width].cpu().numpy()
            ref = self._ref(xs, j, width)
            ys = self.d_out[j * self.M: (j + width) * self.M].cpu().numpy()
            worst = max(worst, float(np.linalg.norm(ys - ref) / np.linalg.norm(ref)))
        return worst

    def check_gathered(self, big, rng, width=128):
        import oracle_lib as O
        worst = 0.0
        for r in range(big.shape[0]):
            j = int(rng.integers(8, self.n - width))
            xs = O.synth(SEED, r, j - 7, width + 7, complex_=True)
            ys = big[r, j * self.M: (j + width) * self.M].cpu().numpy()
            ref = self._ref(xs, j, width)
            worst = max(worst, float(np.linalg.norm(ys - ref) / np.linalg.norm(ref)))
        return worst

    def cpu(self, samples):
        import oracle_lib as O
        chunk = CPU_CHUNK // self.M
        x = O.synth(SEED, 0, 0, chunk, complex_=True).astype(np.complex128)
        f = O.interp(O.RC64, self.h.astype(np.float64), self.M)
        r = timed_cpu(lambda c: f.execute_block(x), "InterpolatingFIRFilter<f64, Complex<f64>> restatement (push + "
                      "M DotProducts over Window::to_vec per input)", samples // self.M, chunk)
        r["value"] *= self.M  # outputs per second, the metric's unit
        r["sample"] += f"; value counts the {self.M} outputs per input"
        return r


def dropin_costs(torch, sd, h32):
    """What an unchanged Rust caller of the reference pays (not the headline),
    on cfg2's taps: the FIRFilter<f64, Complex<f64>> reference-typed EXACT device path, the
    PCIe-inclusive host-slice execute_block, and per-sample Filter::execute latency."""
    from solid_dsp_amd import FIRFilter
    st = torch.cuda.current_stream()
    out = {}
    # (a) FIRFilter<f64, Complex<f64>> on the device, EXACT (bit-identical to the reference)
    n = 1 << 26
    f = FIRFilter(h32.astype(np.float64), 0.2, sample_dtype=np.complex128, algo=sd.ALGO_EXACT)
    xi = torch.empty(2 * n, dtype=torch.float32, device="cuda")
    sd.lib().sdsp_synth_f32_device(xi.data_ptr(), SEED, 0, 0, 2 * n, st.cuda_stream)
    d_in = torch.view_as_complex(xi.view(-1, 2).to(torch.float64))
    d_out = torch.empty_like(d_in)
    f.execute_block_device(d_in, n, d_out, st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        f.execute_block_device(d_in, n, d_out, st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    out["f64_exact_device"] = {"Msamples_per_s": round(n / dt / 1e6, 1), "ms_per_2^26": round(dt * 1e3, 3),
                               "GBps": round(32 * n / dt / 1e9, 1), "kernel": "fir_direct_kernel<double, c64, EXACT>"}
    del xi, d_in, d_out
    # (a') FIRFilter<f32, Complex<f32>> built with no algorithm while the process default is AUTO
    # (SDSP_DEFAULT_ALGO=auto / sdsp_set_default_algo): an unchanged caller on the headline kernel
    old = sd.get_default_algo()
    sd.set_default_algo(sd.ALGO_AUTO)
    try:
        fa = FIRFilter(h32, np.float32(0.2), sample_dtype=np.complex64)
    finally:
        sd.set_default_algo(old)
    xa = torch.empty(2 * n, dtype=torch.float32, device="cuda")
    sd.lib().sdsp_synth_f32_device(xa.data_ptr(), SEED, 0, 0, 2 * n, st.cuda_stream)
    d_in = torch.view_as_complex(xa.view(-1, 2))
    d_out = torch.empty_like(d_in)
    fa.execute_block_device(d_in, n, d_out, st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        fa.execute_block_device(d_in, n, d_out, st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    out["c32_default_auto_device"] = {"Msamples_per_s": round(n / dt / 1e6, 1), "ms_per_2^26": round(dt * 1e3, 3),
                                      "algo_of_handle": int(sd.lib().sdsp_fir_get_algo(fa._h)),
                                      "note": "FIRFilter<f32, Complex<f32>> created with no set_algo while "
                                              "SDSP_DEFAULT_ALGO=auto: the overlap-save kernel (2^26-sample blocks, "
                                              "host-timed, launch gaps included)"}
    del xa, d_in, d_out, fa
    # (b) host slices through execute_block (H2D + kernel + D2H, pageable numpy buffers)
    for name, dtype, algo, m in [("host_slice_c32_fft", np.complex64, sd.ALGO_FFT, 1 << 25),
                                 ("host_slice_f64_exact", np.complex128, sd.ALGO_EXACT, 1 << 24)]:
        g = FIRFilter(h32.astype(np.float64) if dtype == np.complex128 else h32,
                      0.2 if dtype == np.complex128 else np.float32(0.2), sample_dtype=dtype, algo=algo)
        x = (np.random.default_rng(0).standard_normal(2 * m).astype(np.float32)).view(np.complex64).astype(dtype)
        g.execute_block(x[:4096])
        t0 = time.perf_counter()
        g.execute_block(x)
        dt = time.perf_counter() - t0
        out[name] = {"Msamples_per_s": round(m / dt / 1e6, 1), "samples": m,
                     "note": "PCIe-inclusive: host slice in, host Vec out (pageable buffers)"}
    # (c) per-sample Filter::execute (one launch + one sync, output in host-mapped memory)
    g = FIRFilter(h32.astype(np.float64), 0.2, sample_dtype=np.complex128)
    for _ in range(50):
        g.execute(0.5 + 0.25j)
    k = 2000
    t0 = time.perf_counter()
    for _ in range(k):
        g.execute(0.5 + 0.25j)
    dt = (time.perf_counter() - t0) / k
    out["per_sample_execute"] = {"us_per_call": round(dt * 1e6, 2), "calls": k,
                                 "note": "FIRFilter<f64, Complex<f64>>::execute via the Python binding (ctypes adds "
                                         "~1 us): the host step against the handle's delay line"}
    # the same calls from a compiled caller (what the Rust shim pays): solid_dsp_amd/csrc/step_bench.c,
    # run as a child process (it opens its own device context)
    import subprocess
    exe = os.path.join(REPO, "solid_dsp_amd", "_build", "step_bench")
    try:
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        out["per_sample_c_abi"] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
            {"error": (r.stderr or r.stdout)[-300:]}
        out["per_sample_c_abi"]["note"] = ("C caller: execute / push with the host step (default) and with a "
                                           "device launch per call (SDSP_TUNE_HOST_STEP = 0); the reference's "
                                           "CPU loop takes ~0.36 us per sample (SURVEY §3.1)")
    except (OSError, subprocess.TimeoutExpired, ValueError, IndexError) as e:
        out["per_sample_c_abi"] = {"error": str(e)[-300:]}
    one = np.array([0.5 + 0.25j])
    t0 = time.perf_counter()
    for _ in range(k):
        g.execute_block(one)
    dt = (time.perf_counter() - t0) / k
    out["per_sample_execute_block_n1"] = {"us_per_call": round(dt * 1e6, 2), "calls": k,
                                          "note": "execute_block with one sample (a host block: below the "
                                                  "host-step threshold)"}
    return out


class Cfg11ActiveLag:
    """A bank of IIRFilter<f64, Complex<f64>> SecondOrder on the reference demo's active_lag(0.02,
    1/sqrt 2, 1000) PLL loop filter (src/main.rs:37-40, iirdes/pll/mod.rs:24-99): 2^16 channels x
    2^12 samples, the reference-order serial recurrence (one lane per channel, bit-identical).  The
    cascade integrates its input, so no block-parallel scan applies (DESIGN.md §4 IIR)."""
    metric = "Msamples/sec IIRFilter<f64, Complex<f64>> active_lag bank, reference-order (bit-exact); % HBM roofline"
    tol = 0

    def __init__(self, args, rank, dev, torch, sd):
        from solid_dsp_amd import IIRFilter, IIRFilterType
        from solid_dsp_amd.filter import iirdes
        self.num, self.den = iirdes.pll.active_lag(0.02, 1.0 / np.sqrt(2.0), 1000.0)
        self.ch, self.n = 1 << 16, 1 << 12
        self.make = lambda d=dev: IIRFilter(self.num, self.den, IIRFilterType.SecondOrder, sample_dtype=np.complex128,
                                            device=d, channels=self.ch, algo=sd.ALGO_EXACT)
        self.f = self.make()
        total = self.ch * self.n
        tmp = torch.empty(2 * total, dtype=torch.float32, device="cuda")
        sd.lib().sdsp_synth_f32_device(tmp.data_ptr(), SEED, rank, 0, 2 * total, torch.cuda.current_stream().cuda_stream)
        self.d_in = torch.view_as_complex(tmp.view(-1, 2).to(torch.float64)).contiguous()
        del tmp
        self.d_out = torch.empty_like(self.d_in)
        self.samples_per_step = total
        self.bytes_per_step = 32 * total
        self.dtype = "c64 (f64 coefficients, Complex<f64> samples, reference summation order)"
        self.kernel = "sos_serial_lds_kernel<1, double, c64> (one lane per channel, 1 KB runs per channel staged through LDS)"
        self.parity_check = "bit mismatches vs the f64 restatement over 16 channels (must be 0)"
        self.workload = "cfg11: active_lag IIRFilter<f64, Complex<f64>> bank, 2^16 channels x 2^12 samples"
        self.algo_name = "iir_serial_bank"

    def step(self, stream):
        self.f.execute_block_device(self.d_in, self.n, self.d_out, stream)

    def parity(self, stream, rng):
        import oracle_lib as O
        import torch
        g = self.make()
        g.execute_block_device(self.d_in, self.n, self.d_out, stream)
        torch.cuda.synchronize()
        bad = 0
        for c in range(16):
            x = self.d_in[c * self.n:(c + 1) * self.n].cpu().numpy()
            y = self.d_out[c * self.n:(c + 1) * self.n].cpu().numpy()
            ref = O.iir(O.RC64, self.num, self.den, O.SECOND_ORDER).execute_block(x)
            bad += int(np.count_nonzero(y.view(np.uint64) != ref.view(np.uint64)))
        return float(bad)

    def cpu(self, samples):
        import oracle_lib as O
        x = O.synth(SEED, 0, 0, CPU_CHUNK, complex_=True).astype(np.complex128)
        f = O.iir(O.RC64, self.num, self.den, O.SECOND_ORDER)
        return timed_cpu(lambda c: f.execute_block(x), "IIRFilter<f64, Complex<f64>> SecondOrder restatement "
                         "(active_lag, one channel)", samples, CPU_CHUNK)


class Cfg12Normal:
    """IIRFilter<f32, f32> Normal DF-II (src/filter/iir/mod.rs:272-279) on the first biquad of the
    cfg3 cascade as one polynomial pair, real f32, 2^30 samples: the dense-system wave scan."""
    metric = "Msamples/sec Normal DF-II IIR (order 2, f32, 1 GiS); % HBM roofline"
    tol = 1e-5

    def __init__(self, args, rank, dev, torch, sd):
        from solid_dsp_amd import IIRFilter, IIRFilterType
        sos = np.array(json.load(open(os.path.join(REPO, "tests", "golden", "butter8_0p2_sos.json")))["sos"])
        self.b, self.a = sos[0, :3].astype(np.float32), sos[0, 3:].astype(np.float32)
        self.n = 1 << args.log2n
        self.make = lambda d=dev: IIRFilter(self.b, self.a, IIRFilterType.Normal, sample_dtype=np.float32, device=d,
                                            algo=sd.ALGO_FMA)
        self.f = self.make()
        self.d_in = torch.empty(self.n, dtype=torch.float32, device="cuda")
        self.d_out = torch.empty(self.n, dtype=torch.float32, device="cuda")
        sd.lib().sdsp_synth_f32_device(self.d_in.data_ptr(), SEED, rank, 0, self.n,
                                       torch.cuda.current_stream().cuda_stream)
        self.samples_per_step = self.n
        self.bytes_per_step = 8 * self.n
        self.dtype = "f32 (f32 coefficients, real f32 samples)"
        self.kernel = "sos_wscan_kernel<0, 2, float, float> (dense 2-state system, 256-byte chunks)"
        self.workload = f"cfg12: Normal DF-II order 2 (cfg3's first biquad), real f32, 2^{args.log2n} samples"
        self.algo_name = "normal_scan"

    def step(self, stream):
        self.f.execute_block_device(self.d_in, self.n, self.d_out, stream)

    def parity(self, stream, rng):
        import oracle_lib as O
        import torch
        m = 1 << 20
        g = self.make()
        g.execute_block_device(self.d_in, self.n, self.d_out, stream)
        torch.cuda.synchronize()
        x = self.d_in[:m].cpu().numpy().astype(np.float64)
        y = self.d_out[:m].cpu().numpy()
        ref = O.iir(O.RR64, self.b.astype(np.float64), self.a.astype(np.float64), O.NORMAL).execute_block(x)
        return float(np.linalg.norm(y - ref) / np.linalg.norm(ref))

    def cpu(self, samples):
        import oracle_lib as O
        x = O.synth(SEED, 0, 0, CPU_CHUNK).astype(np.float64)
        f = O.iir(O.RR64, self.b.astype(np.float64), self.a.astype(np.float64), O.NORMAL)
        return timed_cpu(lambda c: f.execute_block(x), "IIRFilter<f64, f64> Normal restatement (Window + two "
                         "DotProducts per sample)", samples, CPU_CHUNK)


WORKLOADS = {1: Cfg1FIR, 2: Cfg2FIR, 3: Cfg3IIR, 4: Cfg4Decim, 5: Cfg5Chan, 6: Cfg6ACorr, 7: Cfg7NCO, 8: Cfg8FFT, 9: Cfg9AGC,
             10: Cfg10Interp, 11: Cfg11ActiveLag, 12: Cfg12Normal}
# bounded CPU samples: about 10-20 s of single-thread work each on a current x86 host
CPU_DEFAULT = {1: 1 << 27, 2: 1 << 26, 3: 1 << 27, 4: 1 << 28, 5: 1 << 32, 6: 1 << 25, 7: 1 << 28, 8: 1 << 24, 9: 1 << 25,
               10: 1 << 30, 11: 1 << 26, 12: 1 << 27}
CPU_CHUNK = 1 << 22


def free_port():
    """a free TCP port on 127.0.0.1 for a rendezvous"""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`--gpus N` outside torch.distributed.run: this parent never initialises the
    GPU; it starts N child ranks of this same script (one per GPU) with
    RANK / WORLD_SIZE / LOCAL_RANK and a 127.0.0.1 rendezvous, waits for all of
    them, stops the rest when one fails, and returns the worst exit status."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc, pending = 0, list(procs)
    while pending:
        for p in list(pending):
            r = p.poll()
            if r is None:
                continue
            pending.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                for q in pending:
                    q.terminate()
        time.sleep(0.1)
    return rc


def dry_run(args, rank, world):
    """CPU-only rehearsal of the N-rank harness over gloo (no GPU): every rank runs
    its own channel (channel = rank) of the chosen workload's math -- config 2 the
    cfg2 FIR, config 4 the cfg4 decimator, both on the f64 restatement standing in
    for the device, stored as c32 like the device output -- the job time is the max
    over ranks, the whole output of every rank is gathered on rank 0 in small chunks
    (parallel.gather_full_to_root, the function the RCCL path calls) and checked there
    by the same check_gathered the GPU run uses.  SDSP_DRYRUN_FAULT=shift makes the
    last rank deliver its output one sample late (the check must then fail)."""
    import torch
    import torch.distributed as dist
    import oracle_lib as O
    from solid_dsp_amd import parallel as P
    if world > 1:
        dist.init_process_group("gloo")
    cfg = args.config if args.config in (2, 3, 4, 5) else 2
    n = 1 << 15
    if cfg == 3:
        sos = np.array(json.load(open(os.path.join(REPO, "tests", "golden", "butter8_0p2_sos.json")))["sos"])
        ff, fb = sos[:, :3].reshape(-1).astype(np.float32), sos[:, 3:].reshape(-1).astype(np.float32)
        run = lambda x: O.iir(O.RR64, ff.astype(np.float64), fb.astype(np.float64), O.SECOND_ORDER).execute_block(x)
        check = lambda big, rng: Cfg3IIR.check(big, ff, fb, n, rng, 2048)
    elif cfg == 5:
        h5 = O.firdes_kaiser(8192, 1.0 / 2048, 80.0, 0.0).astype(np.float32)
        S5, M5 = 2, 1024

        def run5(r):  # the rank's S5 streams, frame-major channeliser outputs, stream after stream
            out = []
            for ch in P.channel_ids(S5, world, r):
                x = O.synth(SEED, ch, 0, n, complex_=True).astype(np.complex128)
                y = np.zeros(n, np.complex128)
                O.lib().orc_channelize(O._ptr(h5.astype(np.float64)), len(h5), M5, O._ptr(x), n, O._ptr(y))
                out.append(y)
            return np.concatenate(out)
        check = lambda big, rng: Cfg5Chan.check(big, h5, M5, S5, n, rng, 4096)
    elif cfg == 2:
        h = O.firdes_kaiser(256, 0.1, 80.0, 0.0).astype(np.float32)
        run = lambda x: O.fir(O.RC64, h.astype(np.float64), 0.2).execute_block(x)
        expected = lambda r, s, w: Cfg2FIR.expected(h, r, s, w)
        lo, hi, width = 256, n, 2048
    else:
        h = O.firdes_kaiser(256, 1.0 / 64, 80.0, 0.0).astype(np.float32)
        run = lambda x: O.decim(O.RC64, h.astype(np.float64), 1.0 / 32, 32).execute_block(x)
        expected = lambda r, m, w: Cfg4Decim.expected(h, r, m, w)
        lo, hi, width = 8, n // 32, 256
    t0 = time.perf_counter()
    if cfg == 3 and args.shard == "time":  # segment `rank` of one stream, one state exchange
        A3, _, c3, _ = P.sos_state_space(ff, fb)
        o = O.iir(O.RR64, ff.astype(np.float64), fb.astype(np.float64), O.SECOND_ORDER)
        y0 = o.execute_block(O.synth(SEED, 0, rank * n, n).astype(np.float64))
        states = P.exchange_states(o.sos_state())
        init = P.iir_exclusive_scan(states, P.state_transition(A3, n))[rank]
        if os.environ.get("SDSP_DRYRUN_FAULT") == "noexchange":
            init = np.zeros_like(init)
        g3 = O.iir(O.RR64, ff.astype(np.float64), fb.astype(np.float64), O.SECOND_ORDER)
        g3.sos_state(init)
        W3 = P.zero_input_length(A3, c3, n)
        y0[:W3] += g3.execute_block(np.zeros(W3))
        y = y0.astype(np.float32)
    elif cfg == 3:
        y = run(O.synth(SEED, rank, 0, n).astype(np.float64)).astype(np.float32)
    elif cfg == 5:
        y = run5(rank).astype(np.complex64)
    elif args.shard == "time":  # segment `rank` of one stream after its halo (the GPU path's StreamShard)
        mpi = 1 if cfg == 2 else 32
        first, hh = P.time_segment(n, rank, P.fir_halo(256) if cfg == 2 else P.decim_halo(256, 32))
        y = run(O.synth(SEED, 0, first, hh + n, complex_=True).astype(np.complex128))[hh // mpi:].astype(np.complex64)
    else:
        y = run(O.synth(SEED, rank, 0, n, complex_=True).astype(np.complex128)).astype(np.complex64)
    if os.environ.get("SDSP_DRYRUN_FAULT") == "shift" and rank == world - 1:
        y = np.concatenate([np.zeros(1, y.dtype), y[:-1]])
    wall = P.max_over_ranks(time.perf_counter() - t0)
    ranks = P.gather_to_root(torch.tensor([rank], dtype=torch.int64), 0)
    big = P.gather_full_to_root(torch.from_numpy(y), 0, chunk_bytes=1 << 14)
    if rank == 0:
        if cfg == 3 and args.shard == "time":
            worst = P.check_time_sharded(big, lambda g, w: Cfg3IIR.expected(ff, fb, 0, g, w),
                                         np.random.default_rng(2), 2048, 0)
        elif cfg in (3, 5):
            worst = check(big, np.random.default_rng(2))
        elif args.shard == "time":
            worst = P.check_time_sharded(big, lambda g, w: expected(0, g, w), np.random.default_rng(2), width, lo)
        else:
            worst = P.check_gathered(big, expected, np.random.default_rng(2), width, lo, hi)
        print(json.dumps({"metric": "dry-run: rank launch + max-over-ranks timing + full gather + gathered-output "
                          "check (gloo, CPU)", "value": world * n / wall / 1e6, "unit": "Msamples/sec",
                          "n_gpus": world, "config": cfg, "shard": args.shard, "ranks": [int(t.item()) for t in ranks],
                          "gather_rows": int(big.shape[0]), "gather_check": worst,
                          "gather_ok": bool(worst <= (1e-5 if cfg == 3 else 1e-6)), "dry_run": True}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    from solid_dsp_amd import parallel as P
    rank, world, local = P.world()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(spawn_ranks(args.gpus))
    if args.gpus is not None and args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.shard == "time" and args.config not in (2, 3, 4):
        sys.exit("bench.py: --shard time applies to configs 2 (FIR), 3 (IIR) and 4 (decimator)")
    if args.dry_run:
        return dry_run(args, rank, world)

    import torch
    import torch.distributed as dist
    use_dist = world > 1 or args.dist
    if use_dist:
        if "MASTER_ADDR" not in os.environ:  # --dist without a launcher: a one-rank rendezvous
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1",
                              LOCAL_RANK="0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    import solid_dsp_amd as sd

    stream = torch.cuda.current_stream()
    w = WORKLOADS[args.config](args, rank, dev, torch, sd)
    for kv in args.tune:
        name, val = kv.split("=")
        w.f.set_tuning(getattr(sd._lib, "TUNE_" + name.upper()), int(val))
    torch.cuda.synchronize()
    # achievable copy bandwidth of this box, measured before the warm-up: it also
    # brings the device out of its idle clocks (~0.3 s of streaming) so the
    # workload's own warm-up steps are not spent on the clock ramp
    copy_gbps = stream_copy_gbps(torch, sd)
    settled = settle(w, stream, torch, ms=args.settle_ms) if args.settle_ms > 0 else None

    for _ in range(args.warmup):
        w.step(stream)
    torch.cuda.synchronize()

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        starts[k].record(stream)
        w.step(stream)
        ends[k].record(stream)
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    wall = time.perf_counter() - t0
    ev_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    wall = P.max_over_ranks(wall, device="cuda")  # the job runs as long as its slowest rank

    # final gather over RCCL (timed separately, not part of `value`): every rank's
    # whole output to rank 0, checked there against the f64 restatement
    gather = None
    if use_dist and not args.no_gather:
        piece = w.output() if hasattr(w, "output") else w.d_out
        torch.cuda.synchronize()
        dist.barrier()
        tg = time.perf_counter()
        big = P.gather_full_to_root(piece, 0)
        torch.cuda.synchronize()
        g_ms = (time.perf_counter() - tg) * 1e3
        nbytes = world * piece.numel() * piece.element_size()
        gather = {"ms": round(g_ms, 2), "bytes": nbytes, "GBps_into_root": round(nbytes / (g_ms * 1e-3) / 1e9, 1),
                  "check": None}
        if rank == 0 and not args.no_parity and hasattr(w, "check_gathered"):
            gather["check"] = w.check_gathered(big, np.random.default_rng(2))
        del big
        torch.cuda.empty_cache()

    parity = None
    if not args.no_parity and rank == 0:
        parity = w.parity(stream, np.random.default_rng(1))

    if rank == 0:
        ms_per_step = wall * 1e3 / args.steps
        value = world * w.samples_per_step * args.steps / wall / 1e6
        kern_ms = float(np.mean(ev_ms))
        achieved = w.bytes_per_step / (kern_ms * 1e-3) / 1e9
        tol = getattr(w, "tol", 1e-6)
        parity_ok = parity is None or parity <= tol
        if gather and gather["check"] is not None:
            parity_ok = parity_ok and gather["check"] <= tol
        traffic, traffic_src = load_traffic(args.config, args.log2n, w.algo_name, w.kernel)
        out = {
            "metric": w.metric,
            "value": round(value, 1),
            "unit": "Msamples/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup, "settle": settled,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": w.dtype,
            "data": ("synthetic SplitMix64 stream (seed 20250226, channel = rank), device generated"
                     if getattr(w, "shard", "channel") != "time" else
                     "synthetic SplitMix64 stream (seed 20250226, one channel; rank r generates its segment and halo), "
                     "device generated"),
            "config": {"workload": w.workload, "samples_per_step_per_gpu": w.samples_per_step,
                       "kernel": w.kernel, **({"tuning": args.tune} if args.tune else {}),
                       "parallelism": getattr(w, "parallelism", None) or f"channels sharded, independent per GPU x {world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel_ms": round(kern_ms, 4), "kernel_ms_median": round(float(np.median(ev_ms)), 4),
                         "kernel_ms_min": round(float(np.min(ev_ms)), 4),
                         "algorithmic_bytes_per_launch": w.bytes_per_step,
                         "stream_copy_GBps": round(copy_gbps, 1), "frac_of_stream_copy": round(achieved / copy_gbps, 4)},
            "parity": {"check": getattr(w, "parity_check", "rel_rms vs the f64 restatement"),
                       "value": parity, "tolerance": tol, "ok": parity_ok},
            "gather": gather,
        }
        # the drop-in costs and the CPU baseline belong to the single-GPU line (rank 0 at N = 1)
        if args.config == 2 and not args.no_dropin and world == 1:
            out["dropin"] = dropin_costs(torch, sd, w.h)
        if not args.no_cpu and world == 1:
            cb = w.cpu(args.cpu_samples or CPU_DEFAULT[args.config])
            cb["host_nproc"] = os.cpu_count()
            cb["host_affinity_cpus"] = len(os.sched_getaffinity(0))
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
        if not parity_ok:
            print(f"bench.py: parity {parity} (gather check {gather and gather['check']}) exceeds tolerance {tol}",
                  file=sys.stderr)
    if world > 1:
        dist.destroy_process_group()
    if rank == 0 and not parity_ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
