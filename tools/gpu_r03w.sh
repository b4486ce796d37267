#!/bin/bash
# r03w: receive-chain tests (pipelined AutoCorrelator by default), then the cfg6 measurement pass
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_r03w.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_r03w.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 CONFIGS="6" TAG=r03w bash tools/gpu_round.sh
