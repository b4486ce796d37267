#!/bin/bash
# r03p: IIR lab ablations per wave-scan variant (HBM-only 7, compute-only 24) and tiles per wave (bits 8-11)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
IIR_LAB=1 IIR_CASES="${IIR_CASES:-1:0,2:0,6:0,1:7,2:7,6:7,1:24,2:24,6:24,6:256,6:512,6:1024}" timeout -k 10 400 python -u tools/iir_ab.py > gpurun_out/r03p_iir_lab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03p_iir_lab.log | grep -B1 median_ms | grep -v "^--"; exit $rc
