"""Per-step kernel time of one bench workload over a long back-to-back run, to see
whether the short timed window of bench.py sits on a transient (clock / power
controller) rather than on the steady state.  Prints the per-step event times of
STEPS consecutive steps after the bench's own copy-phase warm-up, then the same
workload with a host sync and a PAUSE_MS idle gap between steps.
  python tools/steady_probe.py --config 5 [--steps 400] [--pause-ms 1]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", type=int, default=5)
    p.add_argument("--steps", type=int, default=400)
    p.add_argument("--pause-ms", type=float, default=1.0)
    p.add_argument("--no-copy", action="store_true", help="skip the bench's copy phase before the run")
    a = p.parse_args()
    import torch
    import bench
    import solid_dsp_amd as sd
    sys.argv = [sys.argv[0], f"--config={a.config}"]
    args = bench.parse()
    torch.cuda.set_device(0)
    w = bench.WORKLOADS[a.config](args, 0, torch.cuda.current_device(), torch, sd)
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    copy = None if a.no_copy else bench.stream_copy_gbps(torch, sd)

    def run(n, pause):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for e0, e1 in ev:
            e0.record(st)
            w.step(st)
            e1.record(st)
            if pause is not None:
                torch.cuda.synchronize()
                time.sleep(pause * 1e-3)
        torch.cuda.synchronize()
        return [e0.elapsed_time(e1) for e0, e1 in ev]

    back = run(a.steps, None)
    paused = run(min(a.steps, 200), a.pause_ms)
    q = lambda v: {"median": float(np.median(v)), "min": float(np.min(v)), "p90": float(np.percentile(v, 90))}
    blocks = [float(np.median(back[i:i + 20])) for i in range(0, len(back), 20)]
    print(json.dumps({"config": a.config, "copy_GBps": copy, "back_to_back": q(back), "median_per_20_steps": blocks,
                      "first_25": back[:25], "paused": q(paused), "pause_ms": a.pause_ms}, indent=1))


if __name__ == "__main__":
    main()
