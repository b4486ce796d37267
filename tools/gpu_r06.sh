#!/bin/bash
# round-6 GPU steps: TAG [steps...]; each step under its own limit, stop at the first failure
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-r06}; shift
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/${TAG}_$name.log 2>&1; local rc=$?;
        echo "== $name rc=$rc"; grep -v amdgpu.ids gpurun_out/${TAG}_$name.log | tail -${TAILN:-30}; return $rc; }
for step in "$@"; do
  case $step in
    olsab) run olsab 240 env OLS_CASES="${OLS_CASES:-24,67108888}" OLS_BURST=${OLS_BURST:-20} OLS_ROUNDS=${OLS_ROUNDS:-10} python -u tools/ols_lab.py || exit $?;;
    iirnew) run iirnew 300 python -u -m pytest tests/test_gpu_iir.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "tiny_leading_b0 or zero_b0" || exit $?;;
    doctests) run doctests 300 python -u -m pytest tests/test_gpu_reference_doctests.py tests/test_gpu_rx.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?;;
    olsiso) run olsiso 240 env OLS_CASES="${OLS_CASES:-24,67108888}" OLS_BURST=1 OLS_ROUNDS=${OLS_ROUNDS_ISO:-30} python -u tools/ols_lab.py || exit $?;;
    firtests) run firtests 300 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?;;
    clock2) run clock2 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES \
              --kernel-trace --output-format csv -d gpurun_out/${TAG}_clock_cfg2 -o run -- \
              python bench.py --config 2 --steps 60 --warmup 5 --no-cpu --no-parity --no-dropin || exit $?;;
    clock) for c in ${CLOCK_CFGS:-6 9}; do
             run clock_cfg$c 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES \
               --kernel-trace --output-format csv -d gpurun_out/${TAG}_clock_cfg$c -o run -- \
               python bench.py --config $c --steps 40 --warmup 5 --no-cpu --no-parity --no-dropin || exit $?
           done;;
    deftests) run deftests 300 python -u -m pytest tests/test_gpu_default_algo.py tests/test_gpu_fir.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?;;
    ffttests) run ffttests 300 python -u -m pytest tests/test_gpu_fft.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?;;
    iirtests) run iirtests 400 python -u -m pytest tests/test_gpu_iir.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?;;
    libab) OLD=${OLD:-tools/_build/libsdsp_old.so} CONFIGS="${AB_CONFIGS:-3 12}" REPS=${REPS:-3} run libab 900 bash tools/lib_ab.sh ${TAG}_ab || exit $?;;
    gputests) run gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?;;
    bench) run bench 300 python bench.py --steps 20 --warmup 5 || exit $?;;
    *) echo "unknown step $step"; exit 2;;
  esac
done
