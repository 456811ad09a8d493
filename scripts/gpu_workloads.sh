#!/bin/bash
# Every bench workload once (1 GPU), JSON lines into gpurun_out/workloads_TAG/.
#   bash scripts/gpu_workloads.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-wl}; OUT=gpurun_out/workloads_$TAG; mkdir -p $OUT
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
for w in c3 c5 c5err c4opt c2-closure; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths > $OUT/$w.log 2>&1
  rc=$?; echo "$w rc=$rc"
  if faulted $OUT/$w.log; then echo FAULT; exit 99; fi
  [ $rc -ne 0 ] && { tail -5 $OUT/$w.log; exit $rc; }
  grep '^{' $OUT/$w.log | tail -1 > $OUT/$w.json
  python -c "import json; d=json.load(open('$OUT/$w.json')); print('  $w', round(d['value'], 1), d['unit'], 'frac', round(d.get('roofline', {}).get('frac', 0), 3))"
done
