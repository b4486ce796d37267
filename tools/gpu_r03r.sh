#!/bin/bash
# r03r: FFT/channeliser tests, then cfg8 A/B (old build vs twiddle-prefetch pass kernel) and the
# channeliser's 8-frame rounds (SDSP_TUNE_CHAN_STREAMING 5) against the default (3)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fft.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_r03r.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r03r.log; [ $rc -eq 0 ] || exit $rc
OLD=tools/_build/libsdsp_old.so CONFIGS="8" REPS=3 bash tools/lib_ab.sh r03r || exit $?
CHAN_CASES="3:0:1,5:0:1,5:128:1,5:256:1" CHAN_ROUNDS=15 timeout -k 10 300 python -u tools/chan_ab.py > gpurun_out/r03r_chan.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03r_chan.log; exit $rc
