#!/bin/bash
# Round measurement session: GPU tests, then per config the bench line (the
# driver's --steps 20 --warmup 5), a rocprofv3 kernel-trace/stats pass of the
# same command (timed dispatches summarised by tools/prof_summary.py) and two
# PMC passes (FETCH_SIZE, WRITE_SIZE, separate runs).  Stops at the first
# fault-like exit status.   CONFIGS="2 10" TAG=r02b bash tools/gpu_round.sh
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
run() { local name=$1; local lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/${TAG}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-2} gpurun_out/${TAG}_$name.log; ok $rc || exit $rc; }
declare -A KERN=([1]=fir_direct [2]="fir_ols_os_kernel<true, false, false>" [3]=sos_wscan [4]=decim_poly [5]=chan1024 [6]=acorr_pipe [7]=nco_mix [8]=fft1024_pipe [9]=agc_pipe [10]=interp_tile [11]=sos_serial [12]=sos_wscan)
if [ -z "$SKIP_TESTS" ]; then run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider; fi
for c in ${CONFIGS:-2 3 4 5}; do
  run bench_cfg$c 300 python bench.py --config $c --steps 20 --warmup 5
  run prof_cfg$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_cfg$c -o run -- python bench.py --config $c --steps 20 --warmup 5 --no-cpu --no-parity --no-dropin
  python tools/prof_summary.py gpurun_out/${TAG}_prof_cfg$c "${KERN[$c]}" --last 20 --out gpurun_out/${TAG}_kernel_timed_cfg$c.json > /dev/null 2>&1 || echo "prof_summary cfg$c failed"
  if [ -z "$SKIP_PMC" ]; then
    run pmc_fetch_cfg$c 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch_cfg$c -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-parity --no-dropin --settle-ms 0
    run pmc_write_cfg$c 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write_cfg$c -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-parity --no-dropin --settle-ms 0
  fi
done
echo done
