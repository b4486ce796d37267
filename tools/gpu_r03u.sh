#!/bin/bash
# r03u: AutoCorrelator tests (LDS-staged input), then cfg6 A/B: staged vs two loads per product
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_r03u.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r03u.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in stage nostage; do
    if [ $v = nostage ]; then export SDSP_ACORR_NOSTAGE=1; else unset SDSP_ACORR_NOSTAGE; fi
    timeout -k 10 200 python bench.py --config 6 --steps 20 --warmup 5 --no-cpu --no-parity > gpurun_out/r03u_cfg6_${v}_r$r.log 2>&1 || exit 9
    python -c "
import json
d = json.loads([x for x in open('gpurun_out/r03u_cfg6_${v}_r$r.log') if x.startswith('{')][-1]); r = d['roofline']
print('cfg6 $v rep$r', d['ms_per_step'], r['kernel_ms'], r['frac'])"
  done
done
