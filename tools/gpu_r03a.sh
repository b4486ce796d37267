#!/bin/bash
# round-3 GPU pass: FIR tests (host step), then the slot-kernel ticket lab
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fir.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fir_r03b.log 2>&1
rc=$?; tail -5 gpurun_out/fir_r03b.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
OLS_CASES="0,4,260,260:0:4,260:0:8,276,276:0:4,276:0:8" OLS_ROUNDS=7 tools/gpu_lab.sh slot6
