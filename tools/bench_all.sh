#!/bin/bash
# all bench configs, one process each, stop at the first fault-like exit
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${TAG:-b}
for c in ${CONFIGS:-2 3 4 5}; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-10} --warmup 3 > gpurun_out/${TAG}_cfg$c.log 2>&1
  rc=$?; echo "cfg$c rc=$rc"; tail -1 gpurun_out/${TAG}_cfg$c.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
