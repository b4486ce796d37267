"""Register / LDS / scratch use of the gfx950 kernels in a HIP object or shared library
(tools only): `python tools/kinfo.py OBJ [name-regex] [--asm OUT.s]`.  Reads the code
object's metadata notes (llvm-readelf --notes); --asm also writes the disassembly of the
matching kernels."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from check_chan_asm import LLVM  # noqa: E402


def code_object(obj, d):
    fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "co.o")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"],
                   check=True, capture_output=True)
    return co


def main():
    obj = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ".")
    asm_out = sys.argv[sys.argv.index("--asm") + 1] if "--asm" in sys.argv else None
    with tempfile.TemporaryDirectory() as d:
        co = code_object(obj, d)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
        cur = {}
        for line in notes.splitlines():
            m = re.match(r"\s+- \.(\w+):\s+(.*)$", line) or re.match(r"\s+\.(\w+):\s+(.*)$", line)
            if not m:
                continue
            k, v = m.group(1), m.group(2)
            if k == "args":
                continue
            cur[k] = v
            if k == "wavefront_size" and "name" in cur:
                pass
            if k == "vgpr_spill_count" and "name" in cur and pat.search(cur["name"]):
                print("%-90s vgpr=%s agpr=%s sgpr=%s lds=%s scratch=%s spill(v/s)=%s/%s" % (
                    cur["name"][:90], cur.get("vgpr_count"), cur.get("agpr_count"), cur.get("sgpr_count"),
                    cur.get("group_segment_fixed_size"), cur.get("private_segment_fixed_size"),
                    cur.get("vgpr_spill_count"), cur.get("sgpr_spill_count")))
        if asm_out:
            text = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                                  capture_output=True, text=True).stdout
            keep, out = False, []
            for line in text.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
                if m:
                    keep = bool(pat.search(m.group(1)))
                if keep:
                    out.append(line)
            open(asm_out, "w").write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
