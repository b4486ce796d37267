#!/bin/bash
# A/B of two libsdsp.so builds on the EXACT FIR / decimator paths (tools/exact_paths.py)
# and the generic PFB shapes (tools/pfb_ab.py), alternating.  Tools only.
#   OLD=tools/_build/libsdsp_old.so REPS=2 bash tools/exact_ab.sh TAG
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${1:-eab}
for r in $(seq ${REPS:-2}); do
  for lib in "$OLD" solid_dsp_amd/_build/libsdsp.so; do
    b=$(basename $lib .so)
    timeout -k 10 200 python -c "
import runpy, sys
import solid_dsp_amd._lib as L
L.LIB_PATH = '$lib'
runpy.run_path('tools/exact_paths.py', run_name='__main__')" > gpurun_out/${TAG}_exact_r${r}_$b.log 2>&1 || exit 9
    echo "exact rep$r $b $(grep '^{' gpurun_out/${TAG}_exact_r${r}_$b.log)"
    PFB_LIB=$lib timeout -k 10 200 python tools/pfb_ab.py > gpurun_out/${TAG}_pfb_r${r}_$b.log 2>&1 || exit 9
    echo "pfb rep$r $b"; grep '^{' gpurun_out/${TAG}_pfb_r${r}_$b.log
  done
done
