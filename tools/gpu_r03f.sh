#!/bin/bash
# r03f: IIR wave-scan parity, cfg3/cfg12 A/B (scalar Cr), OLS nontemporal-store lab
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_iir.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_r03f.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r03f.log; [ $rc -eq 0 ] || exit $rc
OLD=tools/_build/libsdsp_old.so CONFIGS="3 12" REPS=2 bash tools/lib_ab.sh r03f || exit $?
OLS_CASES="0,128,4,132" OLS_ROUNDS=9 bash tools/gpu_lab.sh ntst
