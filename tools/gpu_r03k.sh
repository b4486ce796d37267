#!/bin/bash
# r03k: FFT parity with the pipelined pass kernel (blocked four-step intermediate), then cfg8 pipe vs one-shot (SDSP_FFT_WAVE1024=1)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fft.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_r03k.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r03k.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 16; do
    SDSP_FFT_WAVE1024=$v timeout -k 10 200 python bench.py --config 8 --steps 20 --warmup 5 --no-cpu > gpurun_out/r03k_cfg8_v${v}_r$r.json 2>&1 || exit 9
    python -c "
import json
d = json.loads([x for x in open('gpurun_out/r03k_cfg8_v${v}_r$r.json') if x.startswith('{')][-1]); r = d['roofline']
print('cfg8 v$v rep$r', d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('parity'))"
  done
done
