#!/bin/bash
# Round-5 GPU session steps: STEPS="pytest olsab bench ..." TAG=r05x tools/gpu_r05.sh
# Every step runs under its own time limit; the script stops at the first failure.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${TAG:-r05}
export TMPDIR=/tmp
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
        # iirpmc: one PMC pass (SQ instruction counts) over the lab ablations in IIR_CASES
        iirpmc) IIR_LAB=1 IIR_CASES=${IIR_CASES:-2,2:1,2:2,2:4,2:7} run iirpmc 300 rocprofv3 --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES} \
                --output-format csv -d gpurun_out/${TAG}_iirpmc -o run -- python -u tools/iir_ab.py ;;
        iirburst) IIR_BURST=${BURST:-20} IIR_LAB=1 IIR_CASES=${IIR_CASES:-0,0:4} run iirburst 600 python -u tools/iir_ab.py ;;
        chanab) run chanab 600 python -u tools/chan_ab.py ;;
        chanburst) CHAN_BURST=${BURST:-40} run chanburst 600 python -u tools/chan_ab.py ;;
        # libab_cfg<N>: alternating whole bench lines of the builds in LIBS (tools/libs_ab.sh)
        libab_cfg*) CONFIGS=${s#libab_cfg} run "$s" 900 bash tools/libs_ab.sh ${TAG}_$s ;;
        # proflib_cfg<N>: a kernel-trace / stats profile of the bench under every build in LIBS
        proflib_cfg*) c=${s#proflib_cfg}; for lib in $LIBS; do b=$(basename $lib .so)
                run "${s}_$b" 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${s}_$b -o run -- \
                    python tools/bench_lib.py $lib --config $c --steps 20 --warmup 5 --no-cpu --no-parity --no-dropin; done ;;
        # fftprof: the cfg8 pass kernels per case in FFT_CASES (kernel trace), then the stride probe
        fftprof) FFT_ROUNDS=${FROUNDS:-5} run fftprof 300 rocprofv3 --kernel-trace --stats --output-format csv \
                     -d gpurun_out/${TAG}_fftprof -o run -- python -u tools/fft_lab.py
                 run strideprobe 200 tools/_build/stride_probe ;;
        fenceprobe) run fenceprobe 120 tools/_build/fence_probe 3 ;;
        copyprobe) run copyprobe 300 tools/_build/copy_shape_probe ;;
        fftslice) run fftslice 300 python -u tools/fft_slice_ab.py ;;
        fftlab) run fftlab 300 python -u tools/fft_lab.py ;;
        nocopy*) run "$s" 300 python -u tools/steady_probe.py --config "${s#nocopy}" --steps 400 --no-copy ;;
        steady*) run "$s" 300 python -u tools/steady_probe.py --config "${s#steady}" --steps 400 ;;
        bench) run bench 300 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} ;;
        # bench_tune_<NAME>_<VALUE>: the default config with one tuning key (e.g. bench_tune_OLS_KERNEL_3)
        bench_tune_*) t=${s#bench_tune_}; run "$s" 300 python -u bench.py --steps 20 --warmup 5 --no-cpu \
                     --tune "${t%_*}=${t##*_}" ${BENCH_ARGS:-} ;;
        bench_cfg*) run "$s" 300 python -u bench.py --config "${s#bench_cfg}" --steps 20 --warmup 5 --no-cpu ;;
        # tune8_<NAME>_<VALUE>: config 8 with one kernel-variant knob
        tune8_*) t=${s#tune8_}; run "$s" 300 python -u bench.py --config 8 --steps 20 --warmup 5 --no-cpu \
                     --tune "${t%_*}=${t##*_}" ;;
        # clock_cfg<N>: effective clock (GRBM_GUI_ACTIVE / 8 / wall) and SQ instruction counts of the
        # bench's sustained dispatches, one PMC pass (tools/clock_summary.py)
        clock_cfg*) c=${s#clock_cfg}
            run "$s" 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES \
                --kernel-trace --output-format csv -d gpurun_out/${TAG}_clock_cfg$c -o run -- \
                python bench.py --config $c --steps ${CSTEPS:-60} --warmup 5 --no-cpu --no-parity --no-dropin ;;
        # olspmc_<COUNTER>: one PMC pass over the lab variants in OLS_CASES (traffic per variant)
        olspmc_*) k=${s#olspmc_}
            OLS_ROUNDS=2 run "$s" 300 rocprofv3 --pmc $k --output-format csv -d gpurun_out/${TAG}_$s -o run -- \
                python tools/ols_lab.py ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo done
