"""The Rust shim (rust/solid-sdsp, §8f row 1) declares the reference's public API
of the hot path exactly: for every file of src/filter/{fir,iir}/*, src/filter/mod.rs,
src/filter/firdes/*, src/filter/auto_correlator, src/dot_product/*, src/filter/iirdes/pll,
src/fft/mod.rs, src/nco and src/auto_gain_control, the same `pub fn` names, generic
parameters, parameter lists (names and types) and return types, the same trait
methods and the same public structs / enums with the same variants.  The reference's
signatures are pinned in tests/golden/reference_api.json (tools/rust_api.py); when
/root/reference is present the fixture is regenerated and must be unchanged.
(No cargo in this image: the shim is checked as source, not compiled.)"""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import rust_api as R  # noqa: E402

FIXTURE = os.path.join(REPO, "tests", "golden", "reference_api.json")
SHIM = os.path.join(REPO, "rust", "solid-sdsp", "src")
REF = "/root/reference/src"


def _key(d):
    return (d["name"], d["generics"], d["params"], d["ret"])


@pytest.fixture(scope="module")
def ref_api():
    with open(FIXTURE) as f:
        return json.load(f)


def test_fixture_matches_reference(ref_api):
    if not os.path.isdir(REF):
        pytest.skip("reference sources not present (the committed fixture pins the API)")
    assert R.reference_api(REF) == ref_api


@pytest.mark.parametrize("ref_file", sorted(R.FILES))
def test_shim_pub_fns(ref_api, ref_file):
    shim_file, mode = R.FILES[ref_file]
    shim = R.api(os.path.join(SHIM, shim_file))
    want = set(map(_key, ref_api[ref_file]["pub_fn"]))
    have = set(map(_key, shim["pub_fn"]))
    assert not (have - want), ("declared by the shim, not by the reference", sorted(have - want))
    if mode == "eq":
        assert not (want - have), ("missing from the shim", sorted(want - have))


@pytest.mark.parametrize("ref_file", sorted(R.FILES))
def test_shim_traits_and_types(ref_api, ref_file):
    shim_file, mode = R.FILES[ref_file]
    shim = R.api(os.path.join(SHIM, shim_file))
    for trait in {d["trait"] for d in ref_api[ref_file]["trait_fn"]}:
        want = {_key(d) for d in ref_api[ref_file]["trait_fn"] if d["trait"] == trait}
        have = {_key(d) for d in shim["trait_fn"] if d["trait"] == trait}
        assert want == have, (trait, want ^ have)
    if mode == "eq":
        for name, t in ref_api[ref_file]["types"].items():
            assert shim["types"].get(name) == t, (name, t, shim["types"].get(name))


def test_shim_binds_declared_symbols_only():
    """every extern fn of src/sys.rs is an SDSP_API symbol of include/sdsp.h"""
    import re
    hdr = open(os.path.join(REPO, "include", "sdsp.h")).read()
    declared = set(re.findall(r"SDSP_API\s+[^;(]*?\b(sdsp_\w+)\s*\(", hdr))
    sysrs = open(os.path.join(SHIM, "sys.rs")).read()
    bound = set(re.findall(r"pub fn (sdsp_\w+)\s*\(", sysrs))
    assert bound and not (bound - declared), sorted(bound - declared)


# C type of include/sdsp.h -> the Rust FFI type it must be declared as
_C_SCALAR = {"int": "c_int", "size_t": "usize", "double": "f64", "float": "f32", "uint64_t": "u64",
             "uint32_t": "u32", "int32_t": "i32", "char": "c_char", "void": "c_void",
             "ptrdiff_t": "isize"}


def _c_to_rust(ctype):
    """'const sdsp_fir*' -> '*const sdsp_fir', 'double*' -> '*mut f64', 'sdsp_fir**' ->
    '*mut *mut sdsp_fir', 'int' -> 'c_int'"""
    import re
    t = " ".join(ctype.replace("*", " * ").split())
    const = t.startswith("const ")
    if const:
        t = t[len("const "):]
    stars = t.count("*")
    base = t.replace("*", "").strip()
    base = _C_SCALAR.get(base, base)
    if stars == 0:
        return base
    inner = ("*const " if const else "*mut ") + base
    for _ in range(stars - 1):
        inner = "*mut " + inner
    return re.sub(r"\s+", " ", inner)


def _header_prototypes():
    import re
    hdr = open(os.path.join(REPO, "include", "sdsp.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    protos = {}
    for m in re.finditer(r"SDSP_API\s+([^;]*?)\b(sdsp_\w+)\s*\(([^)]*)\)\s*;", hdr, flags=re.S):
        ret, name, params = m.group(1).strip(), m.group(2), " ".join(m.group(3).split())
        args = []
        if params and params != "void":
            for p in params.split(","):
                p = p.strip()
                pm = re.match(r"(.*?)(\w+)$", p)
                args.append(_c_to_rust(pm.group(1).strip()))
        protos[name] = (None if ret == "void" else _c_to_rust(ret), args)
    return protos


def _sys_rs_decls():
    import re
    src = open(os.path.join(SHIM, "sys.rs")).read()
    decls = {}
    for m in re.finditer(r"pub fn (sdsp_\w+)\s*\(([^)]*)\)\s*(?:->\s*([^;]+))?;", src, flags=re.S):
        name, params, ret = m.group(1), " ".join(m.group(2).split()), m.group(3)
        args = []
        if params.strip():
            for p in params.split(","):
                if p.strip():
                    args.append(" ".join(p.split(":", 1)[1].split()))
        decls[name] = (ret.strip() if ret else None, args)
    return decls


def test_shim_extern_types_match_header():
    """every extern fn of src/sys.rs declares exactly the parameter and
    return types of its include/sdsp.h prototype (size_t = usize, int = c_int, const T* =
    *const T, T* = *mut T, handles by their opaque struct)"""
    protos, decls = _header_prototypes(), _sys_rs_decls()
    assert len(decls) >= 60
    bad = []
    for name, (ret, args) in decls.items():
        want_ret, want_args = protos[name]
        if ret != want_ret or args != want_args:
            bad.append((name, (ret, args), (want_ret, want_args)))
    assert not bad, bad


def test_c_to_rust_type_map():
    assert _c_to_rust("const sdsp_fir*") == "*const sdsp_fir"
    assert _c_to_rust("sdsp_fir**") == "*mut *mut sdsp_fir"
    assert _c_to_rust("double *") == "*mut f64"
    assert _c_to_rust("const void*") == "*const c_void"
    assert _c_to_rust("size_t") == "usize"
