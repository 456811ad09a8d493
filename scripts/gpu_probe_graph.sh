#!/bin/bash
# the captured fork/join probe (scripts/probes/graph_event_probe.hip, built on the
# CPU side with hipcc) in each mode, one process per mode, each under its own time limit; stops at
# the first failure.  Output: gpurun_out/graph_probe.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out; mkdir -p $OUT
for mode in ${MODES:-eager separate nocapfork capture shared cache}; do
  timeout -k 10 60 ./scripts/probes/graph_event_probe $mode ${ITERS:-20000} >> $OUT/graph_probe.log 2>&1
  rc=$?; echo "mode $mode rc=$rc" | tee -a $OUT/graph_probe.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
