#!/bin/bash
# r03l: per-pass kernel times of cfg8 (blocked intermediate) under rocprofv3 kernel trace
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03l_prof_cfg8 -o run -- python bench.py --config 8 --steps 10 --warmup 3 --no-cpu --no-parity > gpurun_out/r03l.log 2>&1 || exit $?
python -c "
import csv, glob
for f in glob.glob('gpurun_out/r03l_prof_cfg8/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'fft' in r['Name']: print(r['Name'][:110], r['Calls'], r['AverageNs'])
"
