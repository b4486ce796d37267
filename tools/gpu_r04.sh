#!/bin/bash
# Round-4 GPU session steps: STEPS="pytest olsab bench ..." TAG=r04x tools/gpu_r04.sh
# Every step runs under its own time limit; the script stops at the first failure.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${TAG:-r04}
run() {
    local name=$1 lim=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -"${TAILN:-6}" "gpurun_out/${TAG}_$name.log"
    [ $rc -eq 0 ] || exit $rc
}
for s in ${STEPS:-pytest}; do
    case $s in
        pytest) run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        pytest_new) run pytest_new 600 python -u -m pytest ${TESTS:-tests/test_gpu_streams.py} -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        olsab) OLS_ROUNDS=${ROUNDS:-15} OLS_CASES=${OLS_CASES:-0,256,4,260} run olsab 600 python -u tools/ols_lab.py ;;
        olsburst) OLS_BURST=${BURST:-20} OLS_ROUNDS=${BROUNDS:-6} OLS_CASES=${OLS_CASES:-0,256,4,260} run olsburst 600 python -u tools/ols_lab.py ;;
        iirab) IIR_LAB=1 IIR_CASES=${IIR_CASES:-0,0:4} run iirab 600 python -u tools/iir_ab.py ;;
        iirburst) IIR_BURST=${BURST:-20} IIR_LAB=1 IIR_CASES=${IIR_CASES:-0,0:4} run iirburst 600 python -u tools/iir_ab.py ;;
        chanab) run chanab 600 python -u tools/chan_ab.py ;;
        chanburst) CHAN_BURST=${BURST:-40} run chanburst 600 python -u tools/chan_ab.py ;;
        copyprobe) run copyprobe 300 tools/_build/copy_shape_probe ;;
        fftslice) run fftslice 300 python -u tools/fft_slice_ab.py ;;
        fftlab) run fftlab 300 python -u tools/fft_lab.py ;;
        nocopy*) run "$s" 300 python -u tools/steady_probe.py --config "${s#nocopy}" --steps 400 --no-copy ;;
        steady*) run "$s" 300 python -u tools/steady_probe.py --config "${s#steady}" --steps 400 ;;
        bench) run bench 300 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} ;;
        bench_cfg*) run "$s" 300 python -u bench.py --config "${s#bench_cfg}" --steps 20 --warmup 5 --no-cpu ;;
        # tune8_<NAME>_<VALUE>: config 8 with one kernel-variant knob
        tune8_*) t=${s#tune8_}; run "$s" 300 python -u bench.py --config 8 --steps 20 --warmup 5 --no-cpu \
                     --tune "${t%_*}=${t##*_}" ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo done
