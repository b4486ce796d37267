#!/bin/bash
# r03n: time-sharding on the device (one GPU: segments after their halos), bench --shard time on one rank,
# then the LDS bank-conflict probe
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -m gpu -x -q -k "time_sharded" --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_r03n.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r03n.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --config 4 --shard time --steps 10 --warmup 3 --no-cpu > gpurun_out/r03n_cfg4_time.json 2>&1 || exit $?
tail -1 gpurun_out/r03n_cfg4_time.json | cut -c1-300
bash tools/gpu_r03m.sh
