#!/bin/bash
# r03s: channeliser tests (variants 5/6: 8 / 4 frames per round), then cfg5 A/B of the variants
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fft.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_r03s.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r03s.log; [ $rc -eq 0 ] || exit $rc
CHAN_CASES="3:0:1,5:0:1,6:0:1,5:64:1,6:64:1,6:256:1" CHAN_ROUNDS=15 timeout -k 10 300 python -u tools/chan_ab.py > gpurun_out/r03s_chan.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03s_chan.log; exit $rc
