"""World-size-2 gloo tests (CPU) of the multi-GPU harness in
solid_dsp_amd/parallel.py: channel sharding, max-over-ranks timing and the
final gather that bench.py performs over RCCL.  Each rank filters its own
channels with the oracle restatement (no GPU here); rank 0 checks the gathered
result against a single-process run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_lib as O
        from solid_dsp_amd import parallel as P
        r, w, _ = P.world()
        assert (r, w) == (rank, world)
        h = O.firdes_kaiser(64, 0.1, 80.0, 0.0)
        n = 4096
        outs = []
        for ch in P.channel_ids(2, w, r):  # weak scaling: 2 channels per rank
            x = O.synth(20250226, ch, 0, n, complex_=True).astype(np.complex128)
            outs.append(O.fir(O.RC64, h, 0.2).execute_block(x))
        piece = torch.from_numpy(np.stack(outs).view(np.float64).copy())
        t = P.max_over_ranks(1.0 + rank)  # slowest rank wins
        got = P.gather_to_root(piece, 0)
        if rank == 0:
            q.put((t, [g.numpy() for g in got]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_shard_maps():
    from solid_dsp_amd import parallel as P
    assert P.shard(8, 2, 0) == [0, 2, 4, 6] and P.shard(8, 2, 1) == [1, 3, 5, 7]
    all_ids = sorted(i for r in range(3) for i in P.shard(10, 3, r))
    assert all_ids == list(range(10))
    assert P.channel_ids(8, 8, 3) == list(range(24, 32))
    with pytest.raises(ValueError):
        P.shard(4, 2, 2)


def test_world2_gloo_shard_time_gather():
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O
    O.lib()  # build before forking
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    # read the result before joining: a worker cannot exit while its queue
    # payload is still in the pipe
    pc = mp.spawn(_worker, args=(2, port, q), nprocs=2, join=False)
    t, got = q.get(timeout=120)
    while not pc.join(timeout=60):
        pass
    assert t == 2.0
    h = O.firdes_kaiser(64, 0.1, 80.0, 0.0)
    for rank in range(2):
        arr = got[rank].view(np.complex128)
        for j, ch in enumerate([rank * 2, rank * 2 + 1]):
            x = O.synth(20250226, ch, 0, 4096, complex_=True).astype(np.complex128)
            ref = O.fir(O.RC64, h, 0.2).execute_block(x)
            assert np.array_equal(arr[j], ref)


def _full_gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, REPO)
        from solid_dsp_amd import parallel as P
        out = torch.arange(1000, dtype=torch.float64) + 1e4 * rank  # ragged last chunk (1000 % 96 != 0)
        big = P.gather_full_to_root(out, 0, chunk_bytes=96 * 8)
        if rank == 0:
            q.put(big.numpy())
        else:
            assert big is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_world2_gloo_full_gather_chunks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.spawn(_full_gather_worker, args=(2, _free_port(), q), nprocs=2, join=False)
    big = q.get(timeout=120)
    while not pc.join(timeout=60):
        pass
    assert big.shape == (2, 1000)
    for r in range(2):
        assert np.array_equal(big[r], np.arange(1000) + 1e4 * r)


@pytest.mark.parametrize("shard", ["channel", "time"])
@pytest.mark.parametrize("config,fault", [(2, ""), (4, ""), (2, "shift"), (4, "shift"), (3, ""), (3, "shift"),
                                          (3, "noexchange"), (5, ""), (5, "shift")])
def test_bench_gpus2_dry_run_checks_gathered_output(config, fault, shard):
    """`bench.py --gpus 2 --dry-run` launches two ranks itself, runs the config's
    workload math per channel (the f64 restatement standing in for the device),
    gathers every rank's whole complex output over gloo with the function the RCCL
    path uses, and checks it with the same check_gathered: a rank whose output is one
    sample late must fail the check.  --shard time: one stream
    time-sharded, each rank's segment after its halo, checked inside and across the
    segment boundaries (check_time_sharded); config 3 time-sharded joins its segments with
    the one all_gather of boundary states (parallel.iir_exclusive_scan) -- without that
    exchange (SDSP_DRYRUN_FAULT=noexchange) the check must fail."""
    import json
    import subprocess
    import sys
    if config == 5 and shard == "time":
        pytest.skip("config 5 shards by stream only")
    if fault == "noexchange" and shard != "time":
        pytest.skip("the boundary-state exchange belongs to the IIR time shard")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["SDSP_DRYRUN_FAULT"] = fault
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run", "--config",
                        str(config), "--shard", shard], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["ranks"] == [0, 1] and line["config"] == config
    assert line["shard"] == shard
    assert line["gather_rows"] == 2
    if fault:
        assert not line["gather_ok"] and line["gather_check"] > 1e-3
    else:
        # configs 2 / 4 / 5: the f64 restatement stored as c32 (<= 1e-6); config 3 stores f32 (<= 1e-5)
        assert line["gather_ok"] and line["gather_check"] <= (1e-5 if config == 3 else 1e-6)


def test_input_windows_match_streaming_outputs():
    """parallel.fir_input_window / decim_input_window: a zero-state run over the
    window's inputs reproduces the streaming outputs of the whole channel"""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O
    from solid_dsp_amd import parallel as P
    x = O.synth(7, 3, 0, 6000, complex_=True).astype(np.complex128)
    h = O.firdes_kaiser(40, 0.1, 80.0, 0.0)
    full = O.fir(O.RC64, h, 0.2).execute_block(x)
    for s, w in [(39, 100), (1000, 17), (5900, 100)]:
        first, count, drop = P.fir_input_window(s, w, len(h))
        got = O.fir(O.RC64, h, 0.2).execute_block(x[first:first + count])[drop:]
        assert np.array_equal(got, full[s:s + w])
    with pytest.raises(ValueError):
        P.fir_input_window(10, 5, 40)
    hd = O.firdes_kaiser(48, 1.0 / 16, 80.0, 0.0)
    M = 8
    fd = O.decim(O.RC64, hd, 1.0, M).execute_block(x)
    from numpy.lib.stride_tricks import sliding_window_view
    for m, w in [(5, 20), (100, 7), (600, 140)]:
        first, count = P.decim_input_window(m, w, len(hd), M)
        ref = sliding_window_view(x[first:first + count], len(hd))[::M][:w] @ hd
        assert np.allclose(ref, fd[m:m + w], rtol=0, atol=1e-12)
    with pytest.raises(ValueError):
        P.decim_input_window(2, 4, 48, 8)


def test_time_sharded_segments_reproduce_the_single_stream():
    """SURVEY §8e time-sharding: three segments of one stream, each filtered by a fresh
    handle after its halo (parallel.time_segment, fir_halo / decim_halo), concatenate to
    the single stream's outputs bit for bit (FIR and decimator restatements), and
    check_time_sharded passes them and flags a boundary off by one sample"""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O
    from solid_dsp_amd import parallel as P
    n, R = 4096, 3
    x = O.synth(11, 0, 0, R * n, complex_=True).astype(np.complex128)
    h = O.firdes_kaiser(64, 0.1, 80.0, 0.0)
    for M in (1, 8):
        mk = (lambda: O.fir(O.RC64, h, 0.5)) if M == 1 else (lambda: O.decim(O.RC64, h, 0.5, M))
        full = mk().execute_block(x)
        halo = P.fir_halo(len(h)) if M == 1 else P.decim_halo(len(h), M)
        assert halo % M == 0 and halo >= len(h) - 1
        segs = []
        for r in range(R):
            first, hh = P.time_segment(n, r, halo)
            assert first == r * n - hh and (r > 0 or hh == 0)
            segs.append(mk().execute_block(x[first:(r + 1) * n])[hh // M:])
        assert all(len(sg) == n // M for sg in segs)
        big = np.stack(segs)
        assert np.array_equal(big.reshape(-1), full)
        exp = lambda g, w: full[g:g + w]
        assert P.check_time_sharded(big, exp, np.random.default_rng(0), 64 // M * 4, 0) == 0.0
        bad = big.copy()
        bad[1] = np.concatenate([segs[0][-1:], segs[1][:-1]])  # segment 1 one output late
        assert P.check_time_sharded(bad, exp, np.random.default_rng(0), 64 // M * 4, 0) > 1e-3


def test_check_gathered_flags_a_shifted_row():
    from solid_dsp_amd import parallel as P
    n = 5000
    rows = np.stack([np.exp(1j * 0.01 * (np.arange(n) + 100 * r)) for r in range(3)]).astype(np.complex64)
    expected = lambda r, s, w: np.exp(1j * 0.01 * (np.arange(s, s + w) + 100 * r))
    assert P.check_gathered(rows, expected, np.random.default_rng(0), 256, 0, n) < 1e-6
    bad = rows.copy()
    bad[2] = np.roll(bad[2], 1)
    assert P.check_gathered(bad, expected, np.random.default_rng(0), 256, 1, n) > 1e-3


def test_world2_gloo_full_gather_complex():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.spawn(_full_gather_complex_worker, args=(2, _free_port(), q), nprocs=2, join=False)
    big = q.get(timeout=120)
    while not pc.join(timeout=60):
        pass
    assert big.shape == (2, 999) and big.dtype == np.complex64
    for r in range(2):
        assert np.array_equal(big[r], (np.arange(999) + 1j * (np.arange(999) + 1e4 * r)).astype(np.complex64))


def _full_gather_complex_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, REPO)
        from solid_dsp_amd import parallel as P
        out = torch.complex(torch.arange(999, dtype=torch.float32), torch.arange(999, dtype=torch.float32) + 1e4 * rank)
        big = P.gather_full_to_root(out, 0, chunk_bytes=100 * 8 + 4)  # odd chunk: pairs must not split
        if rank == 0:
            q.put(big.numpy())
        else:
            assert big is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_bench_rejects_gpus_world_mismatch():
    import subprocess
    import sys
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


@pytest.mark.parametrize("case", ["butter8", "active_lag"])
def test_iir_time_shard_exchange_reproduces_the_single_stream(case):
    """SURVEY §8e IIR time shard on the f64 restatement: three segments of one stream, each
    run from zero state; the exclusive scan of their final states (Phi = A^n) gives each
    segment's true initial state, and adding its zero-input response reproduces the single
    stream -- for the decaying butter(8) cascade and for the reference demo's active_lag PLL
    filter, whose integrator state never decays (zero_input_length = the whole segment)"""
    import json
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as O
    from solid_dsp_amd import parallel as P
    if case == "butter8":
        sos = np.array(json.load(open(os.path.join(REPO, "tests", "golden", "butter8_0p2_sos.json")))["sos"])
        ff, fb = sos[:, :3].reshape(-1), sos[:, 3:].reshape(-1)
    else:
        ff, fb = O.active_lag(0.02, 1 / np.sqrt(2.0), 1000.0)
    n, R = 6000, 3  # butter8: the zero-input response is below rounding after 4096 samples
    x = O.synth(5, 0, 0, R * n).astype(np.float64)
    full = O.iir(O.RR64, ff, fb, O.SECOND_ORDER).execute_block(x)
    A, b, c, d = P.sos_state_space(ff, fb)
    W = P.zero_input_length(A, c, n)
    assert (W < n) == (case == "butter8")
    ys, states = [], []
    for r in range(R):
        o = O.iir(O.RR64, ff, fb, O.SECOND_ORDER)
        ys.append(o.execute_block(x[r * n:(r + 1) * n]))
        states.append(o.sos_state())
    inits = P.iir_exclusive_scan(states, P.state_transition(A, n))
    got = []
    for r in range(R):
        g = O.iir(O.RR64, ff, fb, O.SECOND_ORDER)
        g.sos_state(inits[r])
        y = ys[r].copy()
        y[:W] += g.execute_block(np.zeros(W))
        got.append(y)
    got = np.concatenate(got)
    scale = np.abs(full).max()
    # butter8: rounding only.  active_lag's states run ~1e6 x its output and A^n of its
    # double pole at z = 1 grows with n, so the re-associated sum (any split of one stream)
    # is ~1e-7 relative -- the conditioning the wave scan refuses such cascades for
    tol = 1e-12 if case == "butter8" else 1e-6
    assert np.abs(got - full).max() <= tol * scale, np.abs(got - full).max() / scale
    # the state-space model is the recurrence: one step from a random state
    rng = np.random.default_rng(1)
    st = rng.standard_normal(2 * (len(ff) // 3))
    o = O.iir(O.RR64, ff, fb, O.SECOND_ORDER)
    o.sos_state(st)
    y1 = o.execute_block(np.array([0.7]))[0]
    assert np.allclose(o.sos_state(), A @ st + b * 0.7, rtol=1e-12, atol=1e-12)
    assert np.isclose(y1, c @ st + d * 0.7, rtol=1e-12, atol=1e-12)
    # without the exchange the segment boundaries are wrong
    bad = np.concatenate(ys)
    assert np.abs(bad - full).max() > 1e-6 * scale


def test_world2_gloo_state_exchange():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.spawn(_state_exchange_worker, args=(2, _free_port(), q), nprocs=2, join=False)
    got = q.get(timeout=120)
    while not pc.join(timeout=60):
        pass
    assert len(got) == 2
    for r in range(2):
        assert np.array_equal(got[r], np.arange(8) + 100.0 * r)


def _state_exchange_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, REPO)
        from solid_dsp_amd import parallel as P
        got = P.exchange_states(np.arange(8) + 100.0 * rank)
        if rank == 0:
            q.put([np.asarray(g) for g in got])
        dist.barrier()
    finally:
        dist.destroy_process_group()
