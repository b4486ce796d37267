"""Public-API signatures of Rust sources (tools and tests only): every `pub fn`
with its generic parameter names, parameter list and return type, every `fn` of a
`pub trait`, every `pub struct` / `pub enum` with its variants.  Used by
tests/test_rust_shim_api.py to hold the shim (rust/solid-sdsp) to the reference's
API, and to regenerate tests/golden/reference_api.json from /root/reference:

    python tools/rust_api.py /root/reference/src > tests/golden/reference_api.json
"""
import json
import os
import re
import sys

# reference file (relative to src/) -> shim file (relative to rust/solid-sdsp/src/), and whether
# the shim must declare exactly the reference's `pub fn`s ("eq") or a subset of them ("sub")
FILES = {
    "filter/mod.rs": ("filter/mod.rs", "eq"),
    "filter/fir/mod.rs": ("filter/fir/mod.rs", "eq"),
    "filter/fir/decim.rs": ("filter/fir/decim.rs", "eq"),
    "filter/fir/interp.rs": ("filter/fir/interp.rs", "eq"),
    "filter/fir/pfb.rs": ("filter/fir/pfb.rs", "eq"),
    "filter/iir/mod.rs": ("filter/iir/mod.rs", "eq"),
    "filter/iir/sos.rs": ("filter/iir/sos.rs", "eq"),
    "filter/iir/decim.rs": ("filter/iir/decim.rs", "eq"),
    "filter/iir/interp.rs": ("filter/iir/interp.rs", "eq"),
    "dot_product/mod.rs": ("dot_product/mod.rs", "eq"),
    "dot_product/execute.rs": ("dot_product/execute.rs", "eq"),
    "filter/iirdes/pll/mod.rs": ("filter/iirdes/pll/mod.rs", "eq"),
    "filter/firdes/mod.rs": ("filter/firdes/mod.rs", "eq"),
    "filter/firdes/filter_traits.rs": ("filter/firdes/filter_traits.rs", "eq"),
    "filter/auto_correlator/mod.rs": ("filter/auto_correlator/mod.rs", "eq"),
    "nco/mod.rs": ("nco/mod.rs", "eq"),
    "auto_gain_control/mod.rs": ("auto_gain_control/mod.rs", "eq"),
    "fft/mod.rs": ("fft.rs", "eq"),
}


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return "\n".join(l.split("//")[0] if not l.lstrip().startswith("//") else "" for l in src.splitlines())


def _balanced(s, i, open_c, close_c):
    """s[i] == open_c; index just past the matching close_c"""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == open_c:
            depth += 1
        elif s[j] == close_c:
            depth -= 1
            if depth == 0:
                return j + 1
    raise ValueError("unbalanced")


def _norm(t):
    t = re.sub(r"\s+", " ", t).strip().rstrip(",").strip()
    t = re.sub(r"\s*([<>(),&:\[\];])\s*", r"\1", t)
    t = t.replace(",)", ")").replace(",>", ">").replace(",]", "]")
    return t.replace("mut", "mut ").replace("dyn", "dyn ").replace("mut  ", "mut ").replace("dyn  ", "dyn ")


def _generic_names(g):
    if not g:
        return ""
    inner = g[1:-1]
    parts, depth, cur = [], 0, ""
    for ch in inner:
        if ch in "<([":
            depth += 1
        elif ch in ">)]":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    parts.append(cur)
    return "<" + ",".join(p.split(":")[0].strip() for p in parts if p.strip()) + ">"


def _fn_at(src, m):
    """parse `fn NAME<G>(PARAMS) -> RET` starting at match m (group 'name')"""
    i = m.end()
    gen = ""
    if src[i:i + 1] == "<":
        j = _balanced(src, i, "<", ">")
        gen = src[i:j]
        i = j
    while src[i].isspace():
        i += 1
    assert src[i] == "(", src[m.start():i + 20]
    j = _balanced(src, i, "(", ")")
    params = src[i + 1:j - 1]
    rest = src[j:]
    ret = ""
    mm = re.match(r"\s*->\s*", rest)
    if mm:
        k = mm.end()
        depth = 0
        while k < len(rest):
            ch = rest[k]
            if ch in "<([":
                depth += 1
            elif ch in ">)]":
                if ch == ">" and rest[k - 1] == "-":
                    pass
                else:
                    depth -= 1
            if depth == 0 and (ch in "{;" or rest.startswith("where", k)):
                break
            k += 1
        ret = rest[mm.end():k]
    return {"name": m.group("name"), "generics": _generic_names(gen), "params": _norm(params), "ret": _norm(ret)}


def api(path):
    src = _strip_comments(open(path).read())
    out = {"pub_fn": [], "trait_fn": [], "types": {}}
    for m in re.finditer(r"\bpub\s+fn\s+(?P<name>\w+)", src):
        out["pub_fn"].append(_fn_at(src, m))
    for m in re.finditer(r"\bpub\s+trait\s+(\w+)[^{]*\{", src):
        body_end = _balanced(src, m.end() - 1, "{", "}")
        body = src[m.end():body_end - 1]
        for f in re.finditer(r"\bfn\s+(?P<name>\w+)", body):
            d = _fn_at(body, f)
            d["trait"] = m.group(1)
            out["trait_fn"].append(d)
    for m in re.finditer(r"\bpub\s+(struct|enum)\s+(\w+)", src):
        kind, name = m.group(1), m.group(2)
        variants = []
        if kind == "enum":
            k = src.index("{", m.end())
            body = src[k + 1:_balanced(src, k, "{", "}") - 1]
            variants = [v.strip().split("(")[0].split("{")[0].strip() for v in body.split(",") if v.strip()]
        out["types"][name] = {"kind": kind, "variants": variants}
    out["pub_fn"].sort(key=lambda d: (d["name"], d["params"]))
    out["trait_fn"].sort(key=lambda d: (d["trait"], d["name"]))
    return out


def reference_api(ref_src):
    return {f: api(os.path.join(ref_src, f)) for f in FILES}


if __name__ == "__main__":
    json.dump(reference_api(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src"), sys.stdout, indent=1,
              sort_keys=True)
    sys.stdout.write("\n")
