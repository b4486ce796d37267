#!/bin/bash
# r03o: IIR wave-scan variants incl. 128-byte chunks without register prefetch (4 waves/SIMD), parity + cfg3 A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_iir.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_r03o.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r03o.log; [ $rc -eq 0 ] || exit $rc
IIR_CASES="1,2,6" timeout -k 10 300 python -u tools/iir_ab.py > gpurun_out/r03o_iir_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03o_iir_ab.log | tail -30; exit $rc
