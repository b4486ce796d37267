#!/bin/bash
# quick GPU iteration: gpu tests + bench (+ optional bw calibration)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-q}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
run() { local name=$1; local lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/${TAG}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-4} gpurun_out/${TAG}_$name.log; ok $rc || exit $rc; }
run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run bench 300 python bench.py --steps 10 --warmup 3 --no-cpu
[ -n "$BW" ] && run bw 120 python tools/bw_calib.py
echo done
