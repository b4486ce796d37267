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


def test_bench_gpus2_spawns_two_ranks():
    """`bench.py --gpus 2` outside torchrun launches two ranks itself (dry run: gloo, CPU)."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["ranks"] == [0, 1]
    assert line["gather_rows"] == 2 and line["gather_ok"]


def test_bench_rejects_gpus_world_mismatch():
    import subprocess
    import sys
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
