"""Median per-dispatch SQ counters per kernel (template instance) from rocprofv3 --pmc CSV dirs.
  python tools/pmc_table.py gpurun_out/labpmc_1 gpurun_out/labpmc_2 --kernel fir_ols_os"""
import argparse
import collections
import csv
import glob
import os
import statistics


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dirs", nargs="+")
    p.add_argument("--kernel", default="")
    a = p.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if a.kernel not in k:
                    continue
                k = k.split("(")[0]
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {statistics.median(v):16.0f}  (n={len(v)})")


if __name__ == "__main__":
    main()
