#!/bin/bash
# r03v: AutoCorrelator tests on the default path and with the pipelined kernel (SDSP_ACORR_PIPE=1),
# then cfg6 A/B: pipelined vs staged one-shot
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_r03v.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_r03v.log; [ $rc -eq 0 ] || exit $rc
SDSP_ACORR_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_r03v_pipe.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_r03v_pipe.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in pipe stage; do
    if [ $v = pipe ]; then export SDSP_ACORR_PIPE=1; else unset SDSP_ACORR_PIPE; fi
    timeout -k 10 200 python bench.py --config 6 --steps 20 --warmup 5 --no-cpu > gpurun_out/r03v_cfg6_${v}_r$r.log 2>&1 || exit 9
    python -c "
import json
d = json.loads([x for x in open('gpurun_out/r03v_cfg6_${v}_r$r.log') if x.startswith('{')][-1]); r = d['roofline']
print('cfg6 $v rep$r', d['ms_per_step'], r['kernel_ms'], r['frac'], d['parity'])"
  done
done
