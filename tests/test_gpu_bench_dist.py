"""The multi-GPU code path of bench.py on the MI355X (the RCCL path had only run
over gloo on the CPU).  `bench.py --dist` runs a world of one rank through exactly the code the
driver's N-GPU runs take -- `init_process_group("nccl")`, the barriers around the timed region,
the all_reduce MAX of the wall time, the chunked RCCL gather of the whole output into rank 0
(`parallel.gather_full_to_root`, complex outputs as interleaved real pairs) and the gathered
output's check against the f64 restatement (`check_gathered`) -- on a real device.  The
N >= 2 scaling runs are the driver's (one 8-GPU node); the N = 2 logic is covered over gloo in
tests/test_parallel_gloo.py."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("config,extra", [(2, ["--log2n", "24"]), (3, ["--log2n", "24"]),
                                          (3, ["--log2n", "24", "--shard", "time"]), (4, ["--log2n", "24"]),
                                          (5, [])])
def test_bench_rccl_path_one_rank(config, extra):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dist", "--config", str(config),
                        "--steps", "2", "--warmup", "1", "--no-cpu", "--no-dropin", "--settle-ms", "0"] + extra,
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    g = line["gather"]
    assert g is not None and g["bytes"] > 0
    assert g["check"] is not None and g["check"] <= 1e-5, g
    assert line["parity"]["ok"], line["parity"]
