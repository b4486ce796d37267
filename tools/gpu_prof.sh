#!/bin/bash
# GPU session: tests, bench, STREAM calibration, rocprofv3 kernel stats + PMC
# passes.  Stops at the first fault-like exit status.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-s2}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
run() { local name=$1; local lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/${TAG}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/${TAG}_$name.log; ok $rc || exit $rc; }
if [ -z "$SKIP_TESTS" ]; then run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider; fi
run bench 300 python bench.py --steps 10 --warmup 3 --cpu-samples 4000000
run bw 120 python tools/bw_calib.py
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu --no-parity
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python bench.py --steps 3 --warmup 1 --no-cpu --no-parity
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python bench.py --steps 3 --warmup 1 --no-cpu --no-parity
echo done
