"""Per-kernel statistics of the TIMED dispatches of one bench run, from a
rocprofv3 --kernel-trace CSV (the --stats summary averages every dispatch,
warm-ups included).

  python tools/prof_summary.py gpurun_out/X_prof_cfg2 fir_ols_os --skip 5 --out profiles/r02/kernel_timed_cfg2.json

--skip = the bench's --warmup (plus any untimed dispatches before the timed
region); --take = its --steps (the parity/gather legs after it are dropped).  Since
round 4 the bench settles for ~150 ms of untimed steps first: tools/gpu_round.sh
profiles with --no-parity --no-dropin and takes --last 20.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace_dir")
    p.add_argument("kernel")
    p.add_argument("--skip", type=int, default=0)
    p.add_argument("--take", type=int, default=None)
    p.add_argument("--last", type=int, default=None,
                   help="the last N dispatches instead (bench runs with an untimed settle phase and "
                        "no legs after the timed region: --no-parity --no-dropin)")
    p.add_argument("--out", default=None)
    a = p.parse_args()
    files = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    timed = d[-a.last:] if a.last else d[a.skip: a.skip + a.take if a.take else None]
    if not timed:
        raise SystemExit(f"no timed {a.kernel} dispatches in {a.trace_dir}")
    out = {"kernel": rows[0]["Kernel_Name"].split("(")[0], "source": a.trace_dir, "dispatches_total": len(d),
           "skipped_warmup": len(d) - len(timed) if a.last else a.skip, "timed": len(timed), "avg_ms": statistics.mean(timed),
           "median_ms": statistics.median(timed), "min_ms": min(timed), "max_ms": max(timed),
           "all_ms": [round(x, 4) for x in d],
           "vgpr": rows[0].get("VGPR_Count"), "lds_bytes": rows[0].get("LDS_Block_Size"),
           "scratch": rows[0].get("Scratch_Size"), "grid": [rows[0].get("Grid_Size_X"), rows[0].get("Grid_Size_Y")]}
    s = json.dumps(out, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
