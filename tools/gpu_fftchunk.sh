#!/bin/bash
# cfg8 sweep of the four-step FFT's batch chunking (SDSP_FFT_CHUNK transforms per pass pair; the
# runtime knob existed only for this experiment and was removed after it: logs in profiles/r03/lab/fft_chunk/)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/fftchunk
SDSP_FFT_CHUNK=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fft.py -m gpu > gpurun_out/fftchunk/pytest_chunk1.log 2>&1 || { tail -5 gpurun_out/fftchunk/pytest_chunk1.log; exit 9; }
tail -1 gpurun_out/fftchunk/pytest_chunk1.log
for rep in 1 2; do
for c in 0 4 8 16 32 64; do
  SDSP_FFT_CHUNK=$c timeout -k 10 200 python bench.py --config 8 --steps 20 --warmup 5 --no-cpu --no-parity > gpurun_out/fftchunk/c${c}_r${rep}.log 2>&1 || exit 9
  python -c "
import json
l = [x for x in open('gpurun_out/fftchunk/c${c}_r${rep}.log') if x.startswith('{')][-1]
d = json.loads(l); print('chunk $c rep $rep', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
done
