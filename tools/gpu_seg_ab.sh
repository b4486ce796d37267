# cfg4 decimator: outputs per lane group (SDSP_TUNE_DECIM_SEG) A/B, alternating bench lines
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for r in 1 2; do
  for seg in ${SEGS:-256 512 1024}; do
    timeout -k 10 200 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu --no-parity --no-dropin --tune DECIM_SEG=$seg \
      > gpurun_out/segab_${seg}_r$r.log 2>&1 || exit 9
    python -c "
import json
l=[x for x in open('gpurun_out/segab_${seg}_r$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('seg $seg rep$r', d['ms_per_step'], r['kernel_ms'], r['frac'])"
  done
done
