"""Per-phase instruction table of the one-shot overlap-save kernel (tools only; VERDICT r05 #1
"itemise before changing anything").  The kernel is straight-line code -- every wave executes
each instruction once -- so static counts per phase are the per-wave-segment dynamic counts.
Phases are cut at the s_nop 7 / s_nop 6 / s_nop M markers of the lab instance ABL 64 (ABL 88 =
the product's 24 + markers, tools/lab/ols_lab.hip); the product instance is counted alongside
to show the markers do not change the totals.

  python tools/ols_phase_table.py tools/_build/lab/ols_lab.o [--json OUT]
"""
import json
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kinfo  # noqa: E402

PHASES = ["setup + loads", "P1 DFT16 + W4096", "P2 DFT16 + W256", "P3 DFT16 . H . IDFT16 + W256*",
          "P4 IDFT16", "P5 W4096* + IDFT16 + stores"]


def cat(op):
    if op in ("s_nop",):
        return "SALU nop"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith(("v_pk_fma", "v_pk_mul", "v_pk_add")):
        return "VALU packed"
    if op.startswith("v_"):
        return "VALU other"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("buffer_load", "global_load")):
        return "VMEM load"
    if op.startswith(("buffer_store", "global_store")):
        return "VMEM store"
    if op.startswith("s_"):
        return "SALU"
    return "other"


def disasm(obj, pattern):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run([sys.executable, kinfo.__file__, obj, pattern, "--asm", out], check=True, capture_output=True)
        return open(out).read().splitlines()


def ops(lines):
    res = []
    for l in lines:
        m = re.match(r"\s+([a-z_0-9]+)(\s+[^/]*)?", l)
        if m and not l.strip().startswith(("//", ";", ".")) and re.match(r"[sv]_|ds_|buffer_|global_|flat_", m.group(1)):
            res.append((m.group(1), (m.group(2) or "").strip()))
    return res


def split(seq):
    phases, cur, i = [], [], 0
    while i < len(seq):
        op, arg = seq[i]
        if op == "s_nop" and arg == "7" and i + 2 < len(seq) and seq[i + 1] == ("s_nop", "6") and seq[i + 2][0] == "s_nop":
            phases.append(cur)
            cur = []
            i += 3
            continue
        cur.append(op)
        i += 1
    phases.append(cur)
    return phases


def table(phases):
    rows = []
    for name, ph in zip(PHASES, phases):
        c = {}
        for op in ph:
            k = cat(op)
            c[k] = c.get(k, 0) + 1
        rows.append({"phase": name, **c, "total": len(ph)})
    return rows


def main():
    obj = sys.argv[1]
    marked = ops(disasm(obj, r"fir_ols_os_kernelILi88ELb0"))
    prod = ops(disasm(obj, r"fir_ols_os_kernelILi24ELb0"))
    phases = split(marked)
    assert len(phases) == 6, len(phases)
    rows = table(phases)
    tot_m = {}
    for r in rows:
        for k, v in r.items():
            if k != "phase":
                tot_m[k] = tot_m.get(k, 0) + v
    tot_p = table([[op for op, _ in prod]] + [[]] * 5)[0]
    cols = ["VALU packed", "VALU other", "SALU", "SALU nop", "waitcnt", "LDS", "VMEM load", "VMEM store", "barrier",
            "total"]
    print("| phase | " + " | ".join(cols) + " |")
    print("|---|" + "---|" * len(cols))
    for r in rows:
        print("| %s | " % r["phase"] + " | ".join(str(r.get(c, 0)) for c in cols) + " |")
    print("| all phases (marked build) | " + " | ".join(str(tot_m.get(c, 0)) for c in cols) + " |")
    print("| product instance <24> | " + " | ".join(str(tot_p.get(c, 0)) for c in cols) + " |")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump({"phases": rows, "marked_total": tot_m, "product_total": tot_p,
                       "note": "static counts per wave and segment (straight-line kernel)"}, f, indent=1)


if __name__ == "__main__":
    main()
