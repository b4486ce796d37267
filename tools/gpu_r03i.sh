#!/bin/bash
# r03i: IIR parity incl. the exact-carry bound, then cfg3/cfg12 bench lines
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_iir.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_r03i.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r03i.log; [ $rc -eq 0 ] || exit $rc
for c in 3 12; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > gpurun_out/bench_r03i_cfg$c.json 2> gpurun_out/bench_r03i_cfg$c.err || exit $?
  tail -1 gpurun_out/bench_r03i_cfg$c.json | cut -c1-400
done
