"""Effective clock and instruction counts per sample of the sustained dispatches of a
bench run profiled with one rocprofv3 --pmc pass plus --kernel-trace (tools only).

Effective clock = GRBM_GUI_ACTIVE / 8 / dispatch wall time (MI355X_MICROARCH.md,
"DVFS give-back": rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs).  SQ_INSTS_*
count wave-level instructions; per sample = counter / samples per dispatch.

  python tools/clock_summary.py gpurun_out/X_clock_cfg2 fir_ols_os --samples 1073741824 --last 100
"""
import argparse
import csv
import glob
import json
import os
import statistics


def load(d, kernel):
    trace = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel in r["Kernel_Name"]:
                    trace[r["Dispatch_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    ctr = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel in r["Kernel_Name"]:
                    c = ctr.setdefault(r["Dispatch_Id"], {})
                    c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return trace, ctr


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace_dir")
    p.add_argument("kernel")
    p.add_argument("--samples", type=float, required=True, help="samples (outputs) per dispatch")
    p.add_argument("--last", type=int, default=100)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    trace, ctr = load(a.trace_dir, a.kernel)
    ids = sorted((k for k in ctr if k in trace), key=lambda k: trace[k][0])[-a.last:]
    if not ids:
        raise SystemExit(f"no {a.kernel} dispatches with counters and trace in {a.trace_dir}")
    wall = [(trace[k][1] - trace[k][0]) * 1e-9 for k in ids]
    out = {"kernel": a.kernel, "source": a.trace_dir, "dispatches": len(ids),
           "wall_ms_median": statistics.median(wall) * 1e3}
    names = sorted(set().union(*(ctr[k].keys() for k in ids)))
    for n in names:
        vals = [ctr[k].get(n, 0.0) for k in ids]
        out[n + "_median"] = statistics.median(vals)
        if n.startswith("SQ_INSTS_"):
            out[n + "_per_sample"] = statistics.median(vals) / a.samples
    if "GRBM_GUI_ACTIVE" in names:
        ghz = [ctr[k]["GRBM_GUI_ACTIVE"] / 8.0 / w / 1e9 for k, w in zip(ids, wall)]
        out["effective_clock_GHz_median"] = statistics.median(ghz)
        out["effective_clock_GHz_min"] = min(ghz)
        out["effective_clock_GHz_max"] = max(ghz)
    s = json.dumps(out, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
