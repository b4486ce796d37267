#!/bin/bash
# r03q: IIR tests with real-f32 scans on 128-byte chunks by default, cfg3 / cfg12 bench lines
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_iir.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_r03q.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r03q.log; [ $rc -eq 0 ] || exit $rc
for c in 3 12; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu > gpurun_out/r03q_cfg$c.json 2>&1 || exit $?
  python -c "
import json
d = json.loads([x for x in open('gpurun_out/r03q_cfg$c.json') if x.startswith('{')][-1]); r = d['roofline']
print('cfg$c', d['ms_per_step'], r['kernel_ms'], r['frac'], r['frac_of_stream_copy'], d['parity'])"
done
