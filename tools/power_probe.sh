#!/bin/bash
# Power and clocks while one bench workload runs back to back (tools only):
#   tools/power_probe.sh CONFIG [STEPS]
# Starts tools/steady_probe.py on the workload and samples `amd-smi metric` (power,
# clocks, temperature) every half second while it runs; output under gpurun_out/.
cd "$(dirname "$0")/.."
cfg=${1:-2}
steps=${2:-1500}
mkdir -p gpurun_out
out=gpurun_out/power_cfg${cfg}
timeout -k 10 240 python -u tools/steady_probe.py --config "$cfg" --steps "$steps" --no-copy > "$out.steady.log" 2>&1 &
pid=$!
for i in $(seq 1 60); do
    kill -0 "$pid" 2>/dev/null || break
    echo "== sample $i $(date +%T.%N)" >> "$out.smi.log"
    timeout 10 /opt/rocm/bin/amd-smi metric -g 0 -p -c -t >> "$out.smi.log" 2>&1
    sleep 0.5
done
wait "$pid"
rc=$?
echo "steady_probe rc=$rc"
exit $rc
