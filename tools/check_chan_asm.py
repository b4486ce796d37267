"""Build-time check of the streaming channeliser's untracked prefetch.

chan1024_kernel<K, 1024, PF = true, R = 8> issues each round's input loads as inline
asm `buffer_load_dwordx2 ... offen` (invisible to the compiler's waitcnt tracking) and
waits for them with a hand-placed `s_waitcnt vmcnt(16)` after the round's sixteen
stores.  That is correct only if the compiled code (a) never touches the loads'
destination VGPRs before a wait that provably covers them -- a `vmcnt(N)` with at
least N vector-memory operations issued after the loads on that path -- and (b)
never spills (scratch traffic is counted by vmcnt too and would move the counts).
GCN has no interlock on VMEM results, so a register allocation that breaks either
would silently read stale registers.  This script disassembles the gfx950 code
object of kern_chan1024.o and proves both properties on every path, for every
instance of the kernel that uses the asm loads; `make` runs it after building the
object and tests/test_capi.py runs it again.

    python tools/check_chan_asm.py solid_dsp_amd/_build/obj/kern_chan1024.o
"""
import os
import re
import subprocess
import sys
import tempfile

def _llvm_bin():
    """the ROCm LLVM tools (llvm-objcopy, clang-offload-bundler, llvm-objdump): from ROCM_PATH,
    else next to HIPCC's ROCm, else /opt/rocm (the build must not assume one prefix)"""
    cands = []
    if os.environ.get("ROCM_PATH"):
        cands.append(os.path.join(os.environ["ROCM_PATH"], "llvm", "bin"))
    hipcc = os.environ.get("HIPCC")
    if hipcc:
        cands.append(os.path.join(os.path.dirname(os.path.dirname(os.path.realpath(hipcc))), "llvm", "bin"))
    cands.append("/opt/rocm/llvm/bin")
    for c in cands:
        if all(os.path.exists(os.path.join(c, t)) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")):
            return c
    sys.exit("check_chan_asm: llvm-objcopy / clang-offload-bundler / llvm-objdump not found under " + ", ".join(cands) +
             " (set ROCM_PATH)")


LLVM = _llvm_bin()
KERNEL = re.compile(r"^([0-9a-f]+) <(_Z\w*chan1024_kernelILi(\d)ELi1024ELb1ELi8ELi0EE\w*)>:$")
INSN = re.compile(r"^\s+([a-z_0-9]+)(.*?)\s*//\s*([0-9A-F]+):")
TARGET = re.compile(r"<\w+\+0x([0-9a-f]+)>")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
VMEM = ("buffer_", "global_", "flat_", "scratch_")
BRANCH_COND = ("s_cbranch_",)


def disassemble(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "co.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"],
                       check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                              capture_output=True, text=True).stdout


def kernels(text):
    """{mangled name: [(addr, mnemonic, operands, branch target addr or None)]}"""
    out, cur, base = {}, None, 0
    for line in text.splitlines():
        m = KERNEL.match(line)
        if m:
            base, cur = int(m.group(1), 16), []
            out[m.group(2)] = cur
            continue
        if cur is None:
            continue
        if not line.strip():
            cur = None
            continue
        m = INSN.match(line)
        if m:
            t = TARGET.search(line)
            cur.append((int(m.group(3), 16), m.group(1), m.group(2), base + int(t.group(1), 16) if t else None))
    return out


def vregs(ops):
    s = set()
    for a, b, c in VREG.findall(ops):
        if c:
            s.add(int(c))
        else:
            s.update(range(int(a), int(b) + 1))
    return s


SREG = re.compile(r"^\s*s\[(\d+):(\d+)\]|^\s*s(\d+)\b")


def step_consts(mn, ops, consts, vcc):
    """the few scalar facts the structured-CFG flag branches need: SGPR pairs set to 0 / -1
    by s_mov_b64, and vcc = exec & (~)s[a:b] from them (exec is non-zero in a running wave).
    Returns (consts, vcc); vcc is 0, 'nz' or None (unknown)."""
    dst = ops.split(",")[0].strip()
    consts = dict(consts)
    m = re.match(r"s\[(\d+):(\d+)\]", dst)
    if mn == "s_mov_b64" and m:
        imm = ops.split(",")[1].strip()
        consts.pop(int(m.group(1)), None)
        if imm in ("0", "-1"):
            consts[int(m.group(1))] = int(imm)
        return consts, vcc
    if dst == "vcc" and mn in ("s_andn2_b64", "s_and_b64"):
        src = [o.strip() for o in ops.split(",")[1:]]
        if src[0] == "exec":
            sm = re.match(r"s\[(\d+):(\d+)\]", src[1])
            c = consts.get(int(sm.group(1))) if sm else None
            if c is None:
                return consts, None
            on = (c == 0) if mn == "s_andn2_b64" else (c == -1)
            return consts, ("nz" if on else 0)
        return consts, None
    if dst == "vcc" or (mn.startswith("v_cmp") and mn.endswith("_e32")) or "vcc" in dst:
        vcc = None
    sm = SREG.match(" " + dst)
    if mn.startswith("s_") and sm:
        lo = int(sm.group(1) or sm.group(3))
        hi = int(sm.group(2) or sm.group(3))
        for r in list(consts):
            if r <= hi and lo <= r + 1:
                consts.pop(r)
    return consts, vcc


def check_kernel(insns):
    """[] when safe, else a list of problems"""
    probs = [f"scratch instruction at {a:#x}: {mn}" for a, mn, _, _ in insns if mn.startswith("scratch_")]
    index = {a: i for i, (a, _, _, _) in enumerate(insns)}
    groups, i = [], 0
    while i < len(insns):  # runs of >= 8 `buffer_load_dwordx2 ... offen` (the asm loads)
        j = i
        while j < len(insns) and insns[j][1] == "buffer_load_dwordx2" and "offen" in insns[j][2]:
            j += 1
        if j - i >= 8:
            groups.append((i, j))
        i = max(j, i + 1)
    if len(groups) < 2:
        probs.append(f"expected the prologue and loop asm-load groups, found {len(groups)}")
    for g0, g1 in groups:
        for ld in range(g0, g1):  # each load on its own: a wait may cover only the group's first loads
            dest = vregs(insns[ld][2].split(",")[0])
            # DFS over (instruction index, VMEM ops issued since the load): a path is done at a
            # wait vmcnt(N) with N <= issued (the load has landed) or at s_endpgm
            stack, seen = [(ld + 1, 0, (), None)], set()
            while stack:
                k, cnt, cst, vcc = stack.pop()
                consts = dict(cst)
                while k < len(insns):
                    key = (k, cnt, tuple(sorted(consts.items())), vcc)
                    if key in seen:
                        break
                    seen.add(key)
                    a, mn, ops, tgt = insns[k]
                    if mn == "s_waitcnt" and "vmcnt(" in ops:
                        n = int(re.search(r"vmcnt\((\d+)\)", ops).group(1))
                        if n <= cnt:
                            break  # covered
                    if mn == "s_endpgm":
                        break
                    used = vregs(ops) & dest
                    if used:
                        probs.append(f"load at {insns[ld][0]:#x}: v{sorted(used)} used at {a:#x} ({mn}) after "
                                     f"{cnt} VMEM ops, before a covering wait")
                        break
                    if mn.startswith(VMEM):
                        cnt = min(cnt + 1, 64)
                    if mn == "s_branch":
                        k = index[tgt]
                        continue
                    if mn.startswith(BRANCH_COND) and tgt is not None:
                        taken = {"s_cbranch_vccnz": {0: False, "nz": True}, "s_cbranch_vccz": {0: True, "nz": False}}
                        t = taken.get(mn, {}).get(vcc)
                        if t is True:
                            k = index[tgt]
                            continue
                        if t is None:
                            stack.append((index[tgt], cnt, tuple(sorted(consts.items())), vcc))
                        k += 1
                        continue
                    consts, vcc = step_consts(mn, ops, consts, vcc)
                    k += 1
    return probs


def main(obj):
    ks = kernels(disassemble(obj))
    if not ks:
        print("check_chan_asm: no chan1024_kernel<K, 1024, true, 8> instance found", file=sys.stderr)
        return 1
    bad = 0
    for name, insns in sorted(ks.items()):
        probs = check_kernel(insns)
        for p in probs:
            print(f"check_chan_asm: {name}: {p}", file=sys.stderr)
        bad += bool(probs)
    if not bad:
        print(f"check_chan_asm: {len(ks)} kernel instances: asm-loaded registers untouched until a covering "
              "vmcnt wait on every path, no scratch")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "solid_dsp_amd/_build/obj/kern_chan1024.o"))
