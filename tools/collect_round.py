"""Copy one tools/gpu_round.sh session (gpurun_out/<TAG>_*) into profiles/<round>/:
bench lines, `rocprofv3 --kernel-trace --stats` kernel summaries and the PMC HBM
traffic summaries (tools/pmc_summary.py) of each config's dominant kernel.

  python tools/collect_round.py --tag r01c --out profiles/r01
"""
import argparse
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# dispatch name to match (the interior kernel of cfg2: its boundary launch is a second
# instance of the same template), the algo tag, and the label bench.py matches
LABEL = {2: "fir_ols_os"}
KERNEL = {2: ("fir_ols_os_kernel<true, false, false>", "fft"), 3: ("sos_wscan", "scan"),
          4: ("decim_poly_kernel", "fma"), 5: ("chan1024_kernel", "chan"),
          6: ("acorr_pipe_kernel", "acorr"), 7: ("nco_mix_kernel", "nco"), 8: ("fft1024_pipe", "fft"), 9: ("agc_pipe_kernel", "agc"),
          10: ("interp_tile", "interp"), 11: ("sos_serial", "iir_serial_bank"), 12: ("sos_wscan", "normal_scan")}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tag", required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--configs", default="2 3 4 5")
    a = p.parse_args()
    g = os.path.join(REPO, "gpurun_out")
    os.makedirs(a.out, exist_ok=True)
    for c in map(int, a.configs.split()):
        log = os.path.join(g, f"{a.tag}_bench_cfg{c}.log")
        line = [ln for ln in open(log) if ln.startswith("{")][-1]
        d = json.loads(line)
        with open(os.path.join(a.out, f"bench_cfg{c}.json"), "w") as f:
            f.write(line)
        stats = os.path.join(g, f"{a.tag}_prof_cfg{c}", "run_kernel_stats.csv")
        if os.path.exists(stats):
            shutil.copy(stats, os.path.join(a.out, f"kernel_stats_cfg{c}.csv"))
        timed = os.path.join(g, f"{a.tag}_kernel_timed_cfg{c}.json")
        if os.path.exists(timed):
            shutil.copy(timed, os.path.join(a.out, f"kernel_timed_cfg{c}.json"))
        fetch = os.path.join(g, f"{a.tag}_pmc_fetch_cfg{c}")
        write = os.path.join(g, f"{a.tag}_pmc_write_cfg{c}")
        if c in KERNEL and os.path.isdir(fetch) and os.path.isdir(write):
            k, algo = KERNEL[c]
            subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), "--config", str(c),
                            "--kernel", k, "--algo", algo, "--fetch", fetch, "--write", write,
                            "--algorithmic-bytes", str(d["roofline"]["algorithmic_bytes_per_launch"]),
                            "--out", a.out] + (["--label", LABEL[c]] if c in LABEL else []), check=True)
        print(f"cfg{c}: {d['ms_per_step']} ms/step, frac {d['roofline']['frac']}, "
              f"of copy {d['roofline'].get('frac_of_stream_copy')}")


if __name__ == "__main__":
    main()
