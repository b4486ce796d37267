#!/bin/bash
# r03m: LDS bank conflicts per phase of the cfg2 image layout (tools/lds_probe.hip), timing + SQ counters
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 tools/_build/lds_probe > gpurun_out/r03m_lds_probe.log 2>&1 || exit $?
cat gpurun_out/r03m_lds_probe.log
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv \
    -d gpurun_out/r03m_pmc -o run -- tools/_build/lds_probe > gpurun_out/r03m_pmc.log 2>&1 || exit $?
python tools/pmc_table.py gpurun_out/r03m_pmc --kernel probe
