#!/bin/bash
# iteration session: given test files + optional extra python tool.  Stops at the first fault-like exit.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${TAG:-it}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
run() { local name=$1; local lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/${TAG}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-6} gpurun_out/${TAG}_$name.log; ok $rc || exit $rc; }
run pytest 900 python -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider -x
if [ -n "$TOOL" ]; then TAILN=40 run tool 400 python $TOOL; fi
echo done
