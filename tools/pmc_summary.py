"""Summarise rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) for the
dominant kernel of one bench config into profiles/<round>/pmc_summary_cfg<N>.json.

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE, both reported in KiB.  The
factor 2 is the gfx950 correction of MI355X_MICROARCH.md (HBM section): FETCH_SIZE
counts 64 B per 128-B memory-side read request of a wide coalesced stream.

  python tools/pmc_summary.py --config 2 --kernel fir_ols4096 --log2n 30 --algo fft \
      --fetch gpurun_out/X_pmc_fetch_cfg2 --write gpurun_out/X_pmc_write_cfg2 --out profiles/r01
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_dispatch(d, counter, kernel):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter and kernel in row["Kernel_Name"]:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", type=int, required=True)
    p.add_argument("--kernel", required=True)
    p.add_argument("--log2n", type=int, default=30)
    p.add_argument("--algo", required=True)
    p.add_argument("--fetch", required=True)
    p.add_argument("--write", required=True)
    p.add_argument("--algorithmic-bytes", type=float, default=None)
    p.add_argument("--out", required=True)
    p.add_argument("--label", default=None, help="kernel name to record (default: --kernel); bench.py matches "
                                                   "it as a prefix of the kernel it launches")
    a = p.parse_args()
    fk = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    wk = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    if not fk or not wk:
        raise SystemExit(f"no {a.kernel} dispatches with counters in {a.fetch} / {a.write}")
    fetch_b = 2.0 * statistics.median(fk) * 1024.0
    write_b = statistics.median(wk) * 1024.0
    out = {
        "config": a.config, "kernel": a.label or a.kernel, "dispatch_match": a.kernel, "log2n": a.log2n, "algo": a.algo,
        "dispatches": {"fetch": len(fk), "write": len(wk)},
        "fetch_size_kib_median": statistics.median(fk), "write_size_kib_median": statistics.median(wk),
        "hbm_read_bytes_per_launch": fetch_b, "hbm_write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "correction": "read bytes = 2 x FETCH_SIZE (gfx950, MI355X_MICROARCH.md HBM section); KiB -> bytes",
    }
    if a.algorithmic_bytes:
        out["algorithmic_bytes_per_launch"] = a.algorithmic_bytes
        out["traffic_over_algorithmic"] = (fetch_b + write_b) / a.algorithmic_bytes
    os.makedirs(a.out, exist_ok=True)
    path = os.path.join(a.out, f"pmc_summary_cfg{a.config}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
