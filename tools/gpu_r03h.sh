#!/bin/bash
# r03h: parity after the nontemporal stores, A/B vs the r03 start build, SQ counters of the cfg3 wave scan
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_iir.py tests/test_gpu_fir.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_r03h.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r03h.log; [ $rc -eq 0 ] || exit $rc
OLD=tools/_build/libsdsp_old.so CONFIGS="6 9 11" REPS=2 bash tools/lib_ab.sh r03h || exit $?
OLD=tools/_build/libsdsp_old.so REPS=2 bash tools/exact_ab.sh r03h || exit $?
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAIT_ANY GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d gpurun_out/r03h_sq_cfg3_$i -o run -- python bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-parity > gpurun_out/r03h_sq_cfg3_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r03h_sq_cfg3_$i.log; exit $rc; }
done
python tools/pmc_table.py gpurun_out/r03h_sq_cfg3_1 gpurun_out/r03h_sq_cfg3_2 --kernel sos_wscan
