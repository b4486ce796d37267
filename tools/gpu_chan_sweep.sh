# cfg5 channeliser knob sweep (SDSP_TUNE_CHAN_STREAMING x SDSP_TUNE_CHAN_FRAMES_PER_BLOCK),
# alternating bench lines:  gpurun -- 'bash tools/gpu_chan_sweep.sh'
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for r in 1 2; do
  for v in ${VARS:-5 3 6}; do
    for f in ${FPBS:-0 64 128 192}; do
      timeout -k 10 200 python bench.py --config 5 --steps 20 --warmup 5 --no-cpu --no-parity \
        --tune CHAN_STREAMING=$v --tune CHAN_FRAMES_PER_BLOCK=$f > gpurun_out/chansw_${v}_${f}_r$r.log 2>&1 || exit 9
      python -c "
import json
l=[x for x in open('gpurun_out/chansw_${v}_${f}_r$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('var $v fpb $f rep$r', d['ms_per_step'], r['kernel_ms'], r['frac'])"
    done
  done
done
