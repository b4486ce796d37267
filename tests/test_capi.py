"""CPU-side checks of the C-ABI boundary: libsdsp.so builds for gfx950, loads,
and exports every symbol include/sdsp.h declares.  No compute calls (there is
no GPU here and the library has no CPU path)."""
import os
import re
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "sdsp.h")


def declared_symbols():
    text = open(HDR).read()
    return sorted(set(re.findall(r"SDSP_API\s+[\w\s\*]+?\b(sdsp_\w+)\s*\(", text)))


def test_header_declares_api():
    syms = declared_symbols()
    assert "sdsp_fir_create" in syms and "sdsp_fir_execute_block_device" in syms
    assert len(syms) > 40


def test_library_exports_every_declared_symbol():
    import solid_dsp_amd as sd
    so = sd.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (sdsp_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_library_has_gfx950_code_object():
    import solid_dsp_amd as sd
    data = open(sd.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle target id in .hip_fatbin


def test_no_device_fails_loudly():
    import solid_dsp_amd as sd
    if sd.device_count() > 0:
        pytest.skip("device present")
    with pytest.raises(sd.SdspError) as e:
        sd.FIRFilter(np.ones(4), 1.0)
    assert e.value.code == 101  # SDSP_E_NO_DEVICE: no CPU fallback


def test_host_design_matches_oracle():
    """Host-side design functions of the library (not the hot path) vs the oracle restatement."""
    import oracle_lib as O
    from solid_dsp_amd.filter import firdes, iirdes
    from solid_dsp_amd import group_delay as gd
    for args in [(63, 0.2, 60.0, 0.0), (256, 0.1, 80.0, 0.0), (256, 1 / 64, 80.0, 0.0), (8, 0.35, 120.0, 0.25)]:
        assert np.array_equal(firdes.firdes_kaiser(*args), O.firdes_kaiser(*args))
    assert np.array_equal(firdes.firdes_notch(25, 0.35, 120.0), O.firdes_notch(25, 0.35, 120.0))
    n, d = iirdes.pll.active_lag(0.02, 1 / np.sqrt(2), 1000.0)
    on, od = O.active_lag(0.02, 1 / np.sqrt(2), 1000.0)
    assert np.array_equal(n, on) and np.array_equal(d, od)
    h = O.firdes_notch(12, 0.35, 120.0)
    err = O.C.c_int(0)
    assert gd.fir_group_delay(h, 0.1) == O.lib().orc_fir_group_delay(O._dptr(h), len(h), 0.1, O.C.byref(err))
    with pytest.raises(firdes.FirdesError):
        firdes.firdes_kaiser(8, 0.7, 60.0)


def test_cfg5_prototype_design_is_finite():
    from solid_dsp_amd.filter import firdes
    h = firdes.firdes_kaiser(8192, 1 / 2048, 80.0, 0.0)
    assert np.all(np.isfinite(h)) and abs(h.sum() - 1024) < 5


def test_rust_shim_binds_only_declared_symbols():
    """rust/solid-sdsp/src/sys.rs (the uncompiled Rust side of the boundary) declares
    only entry points that include/sdsp.h exports."""
    import re
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(repo, "include", "sdsp.h")).read()
    declared = set(re.findall(r"SDSP_API[^;(]*?\b(sdsp_\w+)\s*\(", hdr))
    rs = open(os.path.join(repo, "rust", "solid-sdsp", "src", "sys.rs")).read()
    bound = set(re.findall(r"pub fn (sdsp_\w+)\s*\(", rs))
    assert bound and not (bound - declared), sorted(bound - declared)
