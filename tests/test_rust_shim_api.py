"""The Rust shim (rust/solid-sdsp, §8f row 1) declares the reference's public API
of the hot path exactly: for every file of src/filter/{fir,iir}/*, src/filter/mod.rs,
src/dot_product/* and src/filter/iirdes/pll, the same `pub fn` names, generic
parameters, parameter lists (names and types) and return types, the same trait
methods and the same public structs / enums with the same variants; firdes offers a
subset of the reference's functions with identical signatures.  The reference's
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
