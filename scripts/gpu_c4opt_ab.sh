#!/bin/bash
# c4opt (batched L-BFGS, small line-search batches) with and without the lane kernels / chains.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c4ab_${1:-a}; mkdir -p $OUT
for mode in default nochain nolane default2; do
  ( [ $mode = nochain ] && export GRAPE_NO_CHAIN=1; [ $mode = nolane ] && export GRAPE_NO_LANE=1
    timeout -k 10 300 python bench.py --workload c4opt --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths > $OUT/$mode.log 2>&1 )
  rc=$?; echo "$mode rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python -c "import json; d=json.loads([l for l in open('$OUT/$mode.log') if l.startswith('{')][-1]); print('  $mode', round(d['value'], 1))"
done
