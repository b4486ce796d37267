#!/bin/bash
# SQ counter passes over overlap-save kernel variants (one variant per process, few launches).
#   VARIANTS="name:json name:json ..."  (json = tools/ols_ab.py OLS_VARIANTS list with one entry)
#   PASSES="counters;counters;..."      (default: the two SQ passes below)
#   LIST=1                              also write `rocprofv3 -L` to gpurun_out/counters.txt
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-"scalar:[[0,1,0,0]]"}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM"
PASSES=${PASSES:-"$P1;$P2"}
if [ -n "$LIST" ]; then
  timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo "list rc=$?"
fi
IFS=';' read -ra PL <<< "$PASSES"
for v in $VARIANTS; do
  name=${v%%:*}
  export OLS_VARIANTS=${v#*:}
  i=0
  for P in "${PL[@]}"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_ols_${name}_$i -o run -- python tools/ols_ab.py > gpurun_out/pmc_ols_${name}_$i.log 2>&1
    rc=$?; echo "$name pass $i rc=$rc"; tail -2 gpurun_out/pmc_ols_${name}_$i.log
    [ $rc -eq 0 ] || exit $rc
  done
done
echo done
