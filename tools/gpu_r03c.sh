#!/bin/bash
# round-3: the whole GPU suite, then the default bench line
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r03c.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu_r03c.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03c.json 2> gpurun_out/bench_r03c.err
rc=$?; tail -c 3000 gpurun_out/bench_r03c.json; echo "bench rc=$rc"; exit $rc
