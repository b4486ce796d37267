#!/bin/bash
# A/B/... of several libsdsp.so builds on bench configs, interleaved (tools only):
#   LIBS="tools/_build/libsdsp_old.so solid_dsp_amd/_build/libsdsp.so" CONFIGS="2" REPS=3 bash tools/libs_ab.sh TAG
# Each run is a separate bench.py process (--no-cpu --no-parity) with solid_dsp_amd._lib.LIB_PATH
# pointed at one build; prints ms_per_step / kernel_ms / frac per run.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-ab}
for c in ${CONFIGS:-2}; do
  for r in $(seq ${REPS:-2}); do
    for lib in $LIBS; do
      b=$(basename $lib .so)
      timeout -k 10 200 python -c "
import runpy, sys
import solid_dsp_amd._lib as L
L.LIB_PATH = '$lib'
sys.argv = ['bench.py', '--config', '$c', '--steps', '20', '--warmup', '5', '--no-cpu', '--no-parity']
runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/${TAG}_cfg${c}_r${r}_$b.log 2>&1 || exit 9
      python -c "
import json
l = [x for x in open('gpurun_out/${TAG}_cfg${c}_r${r}_$b.log') if x.startswith('{')][-1]
d = json.loads(l); r = d['roofline']
print('cfg$c rep$r $b', d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('frac_of_stream_copy'))"
    done
  done
done
