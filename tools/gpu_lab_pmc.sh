#!/bin/bash
# SQ counter passes over lab variants (one rocprofv3 --pmc run per pass):
#   OLS_CASES="0,2" tools/gpu_lab_pmc.sh TAG
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-labpmc}
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  OLS_ROUNDS=${OLS_ROUNDS:-2} timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_$i -o run -- python tools/ols_lab.py > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_$i.log; exit $rc; }
done
echo done
