#!/bin/bash
# GPU session 1: parity tests, smoke, short bench.  Stops at the first fault-like exit.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/s1_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/s1_pytest.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/s1_smoke.log
ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-samples 2000000 > gpurun_out/s1_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/s1_bench.log
