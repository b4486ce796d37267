#!/bin/bash
# round-3: the whole GPU suite, the default bench line, then the slot-kernel lab
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r03d.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu_r03d.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03d.json 2> gpurun_out/bench_r03d.err
rc=$?; tail -c 3000 gpurun_out/bench_r03d.json; echo "bench rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
OLS_CASES="0,4,260,260:0:4,260:0:8,276,276:0:4,276:0:8" OLS_ROUNDS=9 tools/gpu_lab.sh slot7
