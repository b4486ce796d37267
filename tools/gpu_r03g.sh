#!/bin/bash
# r03g: parity of the kernels with nontemporal stores, A/B vs the r03 start build, IIR lab ablations
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_fir.py tests/test_gpu_golden.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_r03g.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r03g.log; [ $rc -eq 0 ] || exit $rc
OLD=tools/_build/libsdsp_old.so CONFIGS="2 7 10" REPS=2 bash tools/lib_ab.sh r03g || exit $?
IIR_LAB=1 IIR_CASES="1:0,1:24,1:7,1:512,1:1024,1:519" timeout -k 10 300 python -u tools/iir_ab.py > gpurun_out/iir_lab_r03g.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/iir_lab_r03g.log | tail -40; exit $rc
