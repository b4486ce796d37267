#!/bin/bash
# A/B of two builds of libsdsp.so on bench configs, alternating (tools only):
#   OLD=tools/_build/libsdsp_old.so CONFIGS="4 9 11" REPS=2 bash tools/lib_ab.sh TAG
# Runs bench.py --no-cpu --no-parity with solid_dsp_amd._lib.LIB_PATH pointed at each
# build in turn and prints ms_per_step / kernel_ms per run.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-ab}
for c in ${CONFIGS:-4}; do
  for r in $(seq ${REPS:-2}); do
    for lib in "$OLD" solid_dsp_amd/_build/libsdsp.so; do
      timeout -k 10 200 python -c "
import runpy, sys
import solid_dsp_amd._lib as L
L.LIB_PATH = '$lib'
sys.argv = ['bench.py', '--config', '$c', '--steps', '20', '--warmup', '5', '--no-cpu', '--no-parity']
runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/${TAG}_cfg${c}_r${r}_$(basename $lib .so).log 2>&1 || exit 9
      python -c "
import json
l = [x for x in open('gpurun_out/${TAG}_cfg${c}_r${r}_$(basename $lib .so).log') if x.startswith('{')][-1]
d = json.loads(l); r = d['roofline']
print('cfg$c rep$r $(basename $lib .so)', d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('frac_of_stream_copy'))"
    done
  done
done
