#!/bin/bash
# r03y: FFT tests (branch-free next-group loads), then cfg8 A/B over the pass kernel's prefetch depth
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fft.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_r03y.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_r03y.log; [ $rc -eq 0 ] || exit $rc
LIBS="tools/_build/libsdsp_head.so solid_dsp_amd/_build/libsdsp.so tools/_build/libsdsp_pre12.so tools/_build/libsdsp_pre8.so tools/_build/libsdsp_pre4.so" \
  CONFIGS="8" REPS=2 bash tools/libs_ab.sh r03y
