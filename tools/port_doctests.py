"""Port the reference's doctests of the hot path (the files of SURVEY §8a that the
shim replaces):

 * rust/solid-sdsp/tests/reference_doctests.rs: every ```-fenced example of a doc
   comment becomes one #[test] against the `solid` shim crate, body unchanged
   (needs cargo, absent from this image);
 * tests/test_gpu_reference_doctests.py: the same examples
   translated statement by statement to the Python mirror of the same C ABI
   (solid_dsp_amd), so each doctest's calls and asserted literals run on the
   MI355X under `pytest -m gpu`.  The translation covers the Rust subset these
   doctests use (let / tuple bindings, turbofish constructors, unwrap, Complex::new,
   vec!, assert_eq! / assert!, match Ok(..), tuple fields, casts); a statement
   outside it raises, so every doctest is either translated or reported.

Run in this container (it reads /root/reference); the generated files are committed.

    python tools/port_doctests.py
"""
import os
import re

REF = "/root/reference/src"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "rust", "solid-sdsp", "tests", "reference_doctests.rs")
OUT_PY = os.path.join(REPO, "tests", "test_gpu_reference_doctests.py")
FILES = ["filter/fir/mod.rs", "filter/fir/decim.rs", "filter/fir/interp.rs", "filter/fir/pfb.rs",
         "filter/iir/mod.rs", "filter/iir/sos.rs", "filter/iir/decim.rs", "filter/iir/interp.rs",
         "dot_product/mod.rs", "dot_product/execute.rs",
         # the rest of the shim's surface (firdes, AutoCorrelator, NCO, AGC)
         "filter/firdes/mod.rs", "filter/auto_correlator/mod.rs", "nco/mod.rs", "auto_gain_control/mod.rs"]
# files whose module-level (//!) examples are ported too
MODULE_DOC = {"filter/auto_correlator/mod.rs", "nco/mod.rs", "auto_gain_control/mod.rs"}


def doctests(path, module_doc=False):
    """```-fenced examples of the doc comments; a fence left open when its doc comment
    ends is closed there, as rustdoc does (auto_gain_control/mod.rs:310-319)"""
    lines = open(path).read().splitlines()
    out, cur, start, inside = [], None, 0, False
    for n, l in enumerate(lines, 1):
        s = l.strip()
        marker = "///" if s.startswith("///") else "//!" if module_doc and s.startswith("//!") else None
        if marker is None:
            if inside and s:  # blank lines stay inside a doc comment (decim.rs:272)
                inside = False
                out.append((start, cur))
            continue
        body = s[3:]
        if body.startswith(" "):
            body = body[1:]
        if body.startswith("```"):
            if not inside:
                inside, cur, start = True, [], n
            else:
                inside = False
                out.append((start, cur))
            continue
        if inside:
            cur.append(body)
    return out


# ---------------------------------------------------------------- Rust subset -> Python
_DT = {"f64": "np.float64", "f32": "np.float32", "Complex<f64>": "np.complex128", "Complex<f32>": "np.complex64"}


def _statements(body):
    """split a doctest body into top-level statements (';' outside brackets / braces);
    `use` lines dropped"""
    text = "\n".join(l for l in body if not l.strip().startswith(("use ", "//")))
    out, depth, cur = [], 0, ""
    for ch in text:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == ";" and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return [" ".join(st.split()) for st in out if st.strip()]


def _close_paren(s, i):
    """index of the ')' matching the '(' at s[i]"""
    depth = 0
    for j in range(i, len(s)):
        depth += s[j] == "("
        depth -= s[j] == ")"
        if depth == 0:
            return j
    raise ValueError("unbalanced: " + s)


def _turbofish(s):
    """Type::<Coef, In>::new(args) -> Type.new(args, coef_dtype=..., sample_dtype=...)"""
    pat = re.compile(r"(\w+)::<(\w+(?:<\w+>)?), (\w+(?:<\w+>)?)>::new\(")
    while True:
        m = pat.search(s)
        if not m:
            return s
        j = _close_paren(s, m.end() - 1)
        kw = ", coef_dtype=%s, sample_dtype=%s" % (_DT[m.group(2)], _DT[m.group(3)])
        s = s[:m.start()] + m.group(1) + ".new(" + s[m.end():j] + kw + s[j:]


def _expr(e):
    e = re.sub(r"match (.+?) \{ Ok\((\w+)\) => \2, _ => (?:vec!\(\)|0|0\.0) \}", r"\1", e)
    e = re.sub(r"match (.+?) \{ Ok\((\w+)\) => (.+?), _ => 0\.0 \}", r"(lambda \2: \3)(\1)", e)
    # the AGC / AutoCorrelator doctests' test tone and its Complex zip
    e = re.sub(r"\((-?\w+)/(\d+)\.\.(\w+)/(\d+)\)\.map\(\|(\w+)\| \(\5 as f64\)\.(cos|sin)\(\) \* ([\d.]+)\)"
               r"\.collect\(\)", r"[math.\6(float(\5)) * \7 for \5 in range(int(\1 / \2), int(\3 / \4))]", e)
    e = re.sub(r"(\w+)\.iter\(\)\.zip\((\w+)\.iter\(\)\)\.map\(\|\(&(\w+), &(\w+)\)\| Complex::new\(\3, \4\)\)"
               r"\.collect\(\)", r"[complex(\3, \4) for \3, \4 in zip(\1, \2)]", e)
    e = re.sub(r"\bAutoCorrelator::<(f64|f32)>::new\(([^()]*)\)",
               lambda m: "AutoCorrelator(%s, dtype=%s)" % (m.group(2), _DT["Complex<%s>" % m.group(1)]), e)
    e = re.sub(r"\b(AGC|NCO)::new\(\)", r"\1()", e)
    e = e.replace(" && ", " and ")
    e = _turbofish(e)
    e = e.replace(".unwrap()", "").replace(".to_vec()", "")
    e = e.replace("either::Either::Right(", "(").replace("either::Either::Left(", "(")
    e = re.sub(r"Filter::(\w+)\(&?(\w+), ", r"\2.\1(", e)
    e = re.sub(r"(?:solid::filter::)?iirdes::pll::", "iirdes.pll.", e)
    e = re.sub(r"(?:solid::filter::)?firdes::", "firdes.", e)
    e = e.replace("Complex::new(", "complex(")
    e = re.sub(r"vec!\[([^\[\];]*); (\w+)\]", r"[\1] * \2", e)
    e = e.replace("vec![", "[").replace("vec!()", "[]")
    e = re.sub(r"\((\d+)f64\)\.sqrt\(\)", r"math.sqrt(\1.0)", e)
    e = re.sub(r"\b(\d+)f64\b", r"\1.0", e)
    e = re.sub(r"\b(\w+)::new\(", r"\1.new(", e)
    e = re.sub(r"\b(\w+)::(\w+)", r"\1.\2", e)
    e = re.sub(r"(^|[(,\s])&(?=[\w\[(])", r"\1", e)
    e = re.sub(r"(^|[(,\s])\*(?=\w)", r"\1", e)
    e = re.sub(r"(?<=[A-Za-z_)\]])\.(\d+)\b", r"[\1]", e)
    e = re.sub(r"\(([^()]*)\) as usize", r"int(\1)", e)
    e = re.sub(r"\(([^()]*)\)\.abs\(\)", r"abs(\1)", e)
    e = re.sub(r"([\w.]+)\.re\.round\(\)", r"_round(\1.real)", e)
    e = re.sub(r"\.re\b", ".real", e)
    e = re.sub(r"\.im\b", ".imag", e)
    e = re.sub(r"\b(\w+)\.len\(\)", r"_len(\1)", e)
    e = re.sub(r"\b(\w+) as usize\b", r"int(\1)", e)
    e = re.sub(r"\(([^()]*)\)\.round\(\)", r"_round(\1)", e)
    e = re.sub(r"([\w.]+)\.powf\(([\d.]+)\)", r"\1 ** \2", e)
    e = re.sub(r"\(([^()]*)\)\.sqrt\(\)", r"math.sqrt(\1)", e)
    e = re.sub(r"\bfalse\b", "False", e)
    e = re.sub(r"\btrue\b", "True", e)
    if "::" in e or "!" in e.replace("!=", "") or "&" in e:
        raise ValueError("outside the translated subset: " + e)
    return e


def to_python(body):
    out = []
    for st in _statements(body):
        m = re.match(r"let (?:mut )?\((\w+), (\w+)\) = (.+)$", st)
        if m:
            out.append("%s, %s = %s" % (m.group(1), m.group(2), _expr(m.group(3))))
            continue
        m = re.match(r"let (?:mut )?(\w+)(?:\s*: [^=]+)? = (.+)$", st)
        if m:
            out.append("%s = %s" % (m.group(1), _expr(m.group(2))))
            continue
        m = re.match(r"assert_eq!\((.+) as f32, (.+)\)$", st)
        if m:  # an f32 comparison: both sides rounded to f32, as Rust compares them
            out.append("_eq(np.float32(%s), np.float32(%s))" % (_expr(m.group(1)), _expr(m.group(2))))
            continue
        m = re.match(r"assert!\((\w+(?:\[\d+\])?) != (\w+(?:\[\d+\])?)\)$", st)
        if m:  # Vec / Complex inequality, compared as values
            out.append("assert _plain(%s) != _plain(%s)" % (_expr(m.group(1)), _expr(m.group(2))))
            continue
        m = re.match(r"assert_eq!\((.+)\)$", st)
        if m:
            out.append("_eq(%s)" % _expr(m.group(1)))
            continue
        m = re.match(r"assert!\((.+)\)$", st)
        if m:
            out.append("assert %s" % _expr(m.group(1)))
            continue
        out.append(_expr(st))
    return out


PY_HEAD = '''"""The reference's doctests of the hot path (juliantos/solid-dsp src/filter/{fir,iir,firdes}/*.rs,
src/filter/auto_correlator, src/dot_product/*.rs, src/nco, src/auto_gain_control), translated statement by statement by tools/port_doctests.py to the
Python mirror of the C ABI (solid_dsp_amd) and run on the MI355X: every call goes through
libsdsp.so, and each asserted literal is the reference's, compared exactly as Rust's
assert_eq! compares (f64 / Complex<f64> equality).  Generated -- edit the porter, not this file."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sd = pytest.importorskip("solid_dsp_amd")
from solid_dsp_amd import (FIRFilter, DecimatingFIRFilter, InterpolatingFIRFilter, PolyPhaseFilterBank,  # noqa
                           IIRFilter, IIRFilterType, SecondOrderFilter, DecimatingIIRFilter, InterpolatingIIRFilter,
                           DotProduct, Direction, AGC, NCO, AutoCorrelator)
from solid_dsp_amd.filter import firdes, iirdes  # noqa: E402
from solid_dsp_amd.filter.firdes import *  # noqa: E402,F401,F403


def _plain(v):
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, (list, tuple)):
        return [_plain(u) for u in v]
    if isinstance(v, np.generic):
        return v.item()
    return v


def _eq(a, b):
    """assert_eq!: exact equality, element by element for sequences"""
    pa, pb = _plain(a), _plain(b)
    assert pa == pb, (pa, pb)


def _len(x):
    return x.len() if hasattr(x, "len") and callable(x.len) else len(x)


def _round(v):  # f64::round: half away from zero
    return math.floor(v + 0.5) if v >= 0 else -math.floor(-v + 0.5)
'''


_CTOR = re.compile(r"\b(FIRFilter|DecimatingFIRFilter)\.new\(")


def _with_host_step(line):
    """add host_step=host_step to every FIRFilter / DecimatingFIRFilter constructor call"""
    out, i = "", 0
    for m in _CTOR.finditer(line):
        j = _close_paren(line, m.end() - 1)
        out += line[i:j] + ", host_step=host_step)"
        i = j + 1
    return out + line[i:]


def main():
    parts = ["// Generated by tools/port_doctests.py from the reference's doc comments (juliantos/solid-dsp",
             "// src/filter/{fir,iir,firdes}/*.rs, src/filter/auto_correlator, src/dot_product/*.rs, src/nco,",
             "// src/auto_gain_control): each doctest, body unchanged, as an",
             "// integration test of this crate -- the drop-in must pass the reference's own examples.",
             "// Needs libsdsp.so and a gfx950 device at run time (cargo test).", "",
             "#![allow(unused_imports, unused_variables, unused_mut)]", ""]
    total = 0
    for f in FILES:
        tag = f.replace("/", "_").replace(".rs", "")
        for start, body in doctests(os.path.join(REF, f), f in MODULE_DOC):
            total += 1
            parts.append("/// src/%s:%d" % (f, start))
            parts.append("#[test]")
            parts.append("fn %s_l%d() {" % (tag, start))
            parts += ["    " + b if b else "" for b in body]
            parts.append("}")
            parts.append("")
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as fh:
        fh.write("\n".join(parts))
    print("%d doctests -> %s" % (total, OUT))
    py = [PY_HEAD]
    for f in FILES:
        tag = f.replace("/", "_").replace(".rs", "")
        for start, body in doctests(os.path.join(REF, f), f in MODULE_DOC):
            lines = to_python(body)
            # FIR / decimator doctests also run with host_step=False, so the
            # reference's literals reach the HIP kernels (fir_step_kernel, the block kernels),
            # not only the host step that short blocks and per-sample calls default to
            dev = [_with_host_step(ln) for ln in lines]
            py.append("")
            if dev != lines:
                py.append('@pytest.mark.parametrize("host_step", [None, False])')
                py.append("def test_%s_l%d(host_step):" % (tag, start))
                lines = dev
            else:
                py.append("def test_%s_l%d():" % (tag, start))
            py.append('    """src/%s:%d"""' % (f, start))
            py += ["    " + ln for ln in lines] or ["    pass"]
            py.append("")
    with open(OUT_PY, "w") as fh:
        fh.write("\n".join(py))
    print("%d doctests -> %s" % (total, OUT_PY))


if __name__ == "__main__":
    main()
