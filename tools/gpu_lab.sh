#!/bin/bash
# one lab A/B pass on the GPU box: tools/gpu_lab.sh TAG  (env OLS_VARIANTS / OLS_ROUNDS pass through)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-lab}
timeout -k 10 300 python -u tools/ols_lab.py > gpurun_out/${TAG}.log 2>&1
rc=$?; echo "lab rc=$rc"; cat gpurun_out/${TAG}.log | grep -v amdgpu.ids; exit $rc
