#!/bin/bash
# r03x: rx tests (XCD-ordered pipelined AutoCorrelator), cfg6 A/B against the launch-order walk
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_r03x.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_r03x.log; [ $rc -eq 0 ] || exit $rc
OLD=tools/_build/libsdsp_old.so CONFIGS="6" REPS=3 bash tools/lib_ab.sh r03x
