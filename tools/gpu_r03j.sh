#!/bin/bash
# r03j: cfg2 A/B: r03 NT-store build vs merged pmul asm (fewer s_nop) vs + no ds_read2 merges; OLS parity first
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -m gpu -x -q -k "ols or fft or cfg2 or fma" --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_r03j.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r03j.log; [ $rc -eq 0 ] || exit $rc
LIBS="tools/_build/libsdsp_old.so solid_dsp_amd/_build/libsdsp.so tools/_build/libsdsp_nord2.so" CONFIGS="2" REPS=3 bash tools/libs_ab.sh r03j
