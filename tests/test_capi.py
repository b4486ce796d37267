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


def test_firdes_full_set_matches_oracle_and_kats():
    """VERDICT r05 missing #2: the rest of solid::filter::firdes (src/filter/firdes/mod.rs:46-640)
    in the product's design.cpp -- bit-equal to the oracle restatement on a sweep of arguments, the
    reference's doctest KATs through libsdsp.so, and the reference's error codes."""
    import oracle_lib as O
    from solid_dsp_amd.filter import firdes as F
    L = O.lib()
    M = F.EstimationMethod
    # KATs (doctests :64-69, :110-115, :161-166, :431-441, :470-485, :540-550, :589-600)
    assert F.estimate_required_filter_length(0.35, 100.0, M.Herrmann) == 15
    assert int(F.estimate_required_filter_stop_band_attenuation(0.35, 16, M.Herrmann)) == 101
    assert int((F.estimate_required_filter_transition(101.0, 16, M.Herrmann) + 0.005) * 100.0) == 35
    assert len(F.firdes_doppler(51, 0.1, 2.0, 0.0)) == 51
    h = F.firdes_notch(25, 0.2, 30.0)
    assert F.filter_autocorrelation(h, 3) == F.filter_autocorrelation(h, -3)
    assert np.float32(F.filter_autocorrelation(h, 3)) == np.float32(0.047983058)
    k = F.firdes_kaiser(51, 0.35, 120.0, 0.0)
    assert np.float32(F.filter_crosscorrelation(k, h, 0)) == np.float32(0.92825377)
    rms, mx = F.filter_isi(h, 1, 25)
    assert np.float32(rms) == np.float32(0.02509764) and np.float32(mx) == np.float32(0.061966006)
    assert np.float32(F.filter_energy(h, 0.35, 128)) == np.float32(0.3152318)
    # bit equality with the restatement
    for method in (M.Kaiser, M.Herrmann):
        for df, as_ in [(0.35, 100.0), (0.05, 60.0), (0.2, 120.0), (0.01, 30.0), (0.5, 106.0)]:
            out = O.C.c_size_t(0)
            assert L.orc_estimate_req_filter_len(df, as_, int(method), O.C.byref(out)) == 0
            assert F.estimate_required_filter_length(df, as_, method) == out.value
        for df, n in [(0.35, 16), (0.1, 63), (0.02, 256)]:
            assert F.estimate_required_filter_stop_band_attenuation(df, n, method) == \
                L.orc_estimate_req_filter_as(df, n, int(method))
        for as_, n in [(101.0, 16), (60.0, 63), (80.0, 256)]:
            assert F.estimate_required_filter_transition(as_, n, method) == L.orc_estimate_req_filter_df(as_, n, int(method))
    for args in [(51, 0.1, 2.0, 0.0), (64, 0.03, 0.5, 0.7), (7, 0.25, 10.0, 1.2), (1, 0.1, 2.0, 0.0)]:
        ref = np.zeros(args[0])
        L.orc_firdes_doppler(*args, O._dptr(ref))
        assert np.array_equal(F.firdes_doppler(*args), ref, equal_nan=True), args
    g = F.firdes_kaiser(20, 0.2, 60.0, 0.0)
    for lag in (-60, -51, -50, -19, -3, 0, 1, 7, 31, 32, 50, 51, 80):
        assert F.filter_autocorrelation(k, lag) == L.orc_filter_autocorrelation(O._dptr(k), len(k), lag)
        for a, b in ((k, g), (g, k), (h, k)):
            assert F.filter_crosscorrelation(a, b, lag) == \
                L.orc_filter_crosscorrelation(O._dptr(a), len(a), O._dptr(b), len(b), lag), (len(a), len(b), lag)
    for sps, delay in ((1, 25), (2, 12), (5, 5), (3, 3)):
        rr, rm = O.C.c_double(0), O.C.c_double(0)
        L.orc_filter_isi(O._dptr(h), len(h), sps, delay, O.C.byref(rr), O.C.byref(rm))
        assert F.filter_isi(h, sps, delay) == (rr.value, rm.value)
    for fc, nfft in ((0.35, 128), (0.1, 64), (0.0, 7), (0.5, 33)):
        e = O.C.c_double(0)
        assert L.orc_filter_energy(O._dptr(k), len(k), fc, nfft, O.C.byref(e)) == 0
        assert F.filter_energy(k, fc, nfft) == e.value
    # FirdesErrorCode (firdes/mod.rs:17-44): Bandwidth, StopBandLevel, FilterSize, FFTSize
    for call, code in [(lambda: F.estimate_required_filter_length(0.6, 60.0, M.Kaiser), 1),
                       (lambda: F.estimate_required_filter_length(0.2, 0.0, M.Herrmann), 2),
                       (lambda: F.estimate_required_filter_length_kaiser(-0.1, 60.0), 1),
                       (lambda: F.estimate_required_filter_length_herrmann(0.1, -1.0), 2),
                       (lambda: F.estimate_required_filter_stop_band_attenuation(0.7, 16, M.Kaiser), 1),
                       (lambda: F.estimate_required_filter_transition(-5.0, 16, M.Herrmann), 2),
                       (lambda: F.filter_energy(h, 0.6, 128), 1),
                       (lambda: F.filter_energy([], 0.2, 128), 5),
                       (lambda: F.filter_energy(h, 0.2, 0), 6)]:
        with pytest.raises(F.FirdesError) as e:
            call()
        assert e.value.code == code


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


# ---------------------------------------------------------------- channeliser asm-load proof
def _chk():
    import importlib.util
    spec = importlib.util.spec_from_file_location("check_chan_asm", os.path.join(REPO, "tools", "check_chan_asm.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_chan_asm_loads_are_covered_in_the_built_object():
    """the untracked prefetch of chan1024_kernel<K, 1024, true, 8> is read only after
    a provably covering vmcnt wait on every path, with no scratch (tools/check_chan_asm.py,
    also run by the Makefile)"""
    obj = os.path.join(REPO, "solid_dsp_amd", "_build", "obj", "kern_chan1024.o")
    if not os.path.exists(obj):
        pytest.skip("libsdsp not built")
    assert _chk().main(obj) == 0


def test_chan_asm_checker_flags_unsafe_code():
    m = _chk()
    ld = [(0x10 + 8 * i, "buffer_load_dwordx2", f" v[{2 * i}:{2 * i + 1}], v40, s[0:3], 0 offen", None)
          for i in range(8)]
    pro = ld + [(0x60, "s_waitcnt", " vmcnt(0)", None)]  # a prologue group, waited at once
    base = 0x100
    loop = [(base + 8 * i, mn, ops, None) for i, (mn, ops) in enumerate(
        [("buffer_load_dwordx2", f" v[{2 * i}:{2 * i + 1}], v40, s[0:3], 0 offen") for i in range(8)]
        + [("buffer_store_dwordx2", " v[20:21], v41, s[4:7], 0 offen nt")] * 16
        + [("s_waitcnt", " vmcnt(16)"), ("v_mov_b64_e32", " v[30:31], v[14:15]"), ("s_endpgm", "")])]
    assert m.check_kernel(pro + loop) == []
    early = loop[:8] + loop[8:8 + 15] + loop[24:]  # one store short: vmcnt(16) no longer covers
    assert m.check_kernel(pro + early)
    use = loop[:8] + [(0x200, "v_add_f32_e32", " v50, v3, v4", None)] + loop[8:]  # before any wait
    assert m.check_kernel(pro + use)
    spill = pro + loop[:-1] + [(0x300, "scratch_store_dword", " off, v1, s0", None), loop[-1]]
    assert m.check_kernel(spill)
    # per load: a wait that covers only the group's first loads releases only their registers
    two = [(0x400 + 8 * i, "buffer_load_dwordx2", f" v[{2 * i}:{2 * i + 1}], v40, s[0:3], 0 offen", None)
           for i in range(16)]
    wait8 = [(0x500, "s_waitcnt", " vmcnt(8)", None)]
    first = [(0x508, "v_mov_b64_e32", " v[50:51], v[2:3]", None)]
    second = [(0x508, "v_mov_b64_e32", " v[50:51], v[18:19]", None)]
    end = [(0x510, "s_waitcnt", " vmcnt(0)", None), (0x518, "s_endpgm", "", None)]
    assert m.check_kernel(pro + two + wait8 + first + end) == []
    assert m.check_kernel(pro + two + wait8 + second + end)


def test_default_algo_knob_and_environment():
    """sdsp_set_default_algo / SDSP_DEFAULT_ALGO (no device work: the knob is host state)"""
    import sys
    import solid_dsp_amd as sd
    lib = sd.lib()
    old = lib.sdsp_get_default_algo()
    try:
        assert lib.sdsp_set_default_algo(3) == 90  # FFT is not a default for every handle type
        assert lib.sdsp_set_default_algo(-1) == 90 and lib.sdsp_set_default_algo(7) == 90
        for a in (sd.ALGO_AUTO, sd.ALGO_FMA, sd.ALGO_EXACT):
            assert lib.sdsp_set_default_algo(a) == 0 and lib.sdsp_get_default_algo() == a
    finally:
        lib.sdsp_set_default_algo(old)
    code = "import solid_dsp_amd as sd; print(sd.get_default_algo())"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for env, want in (("auto", 0), ("FMA", 2), ("exact", 1), ("bogus", 1), (None, 1)):
        e = dict(os.environ)
        e.pop("SDSP_DEFAULT_ALGO", None)
        if env is not None:
            e["SDSP_DEFAULT_ALGO"] = env
        out = subprocess.run([sys.executable, "-c", code], cwd=root, env=e, capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr
        assert int(out.stdout.strip().splitlines()[-1]) == want, (env, out.stdout)
