#!/bin/bash
# r03e: host-step parity tests, then the untracked-load slot lab
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "host_step or caller_stream" > gpurun_out/pytest_r03e.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r03e.log; [ $rc -eq 0 ] || exit $rc
OLS_CASES="0,260:0:4,308,308:0:4,308:0:8,276:0:4" OLS_ROUNDS=9 bash tools/gpu_lab.sh slot8
