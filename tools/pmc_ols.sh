#!/bin/bash
# SQ counter passes over the default overlap-save kernel (one variant, few launches)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
export OLS_VARIANTS="[[0,1,0,0,0]]"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_ols$i -o run -- python tools/ols_ab.py > gpurun_out/pmc_ols$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -3 gpurun_out/pmc_ols$i.log
  [ $rc -eq 0 ] || exit $rc
done
