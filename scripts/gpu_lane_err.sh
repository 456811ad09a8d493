#!/bin/bash
# Lane exponentials with error sources: parity, GPU suite, C3 A/B (lane vs row groups).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-le}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py -x -v -s --timeout 120 --timeout-method thread > $OUT/lane_$TAG.log 2>&1
rc=$?; echo "lane tests rc=$rc"; grep -E "oracle|FAIL|Error" $OUT/lane_$TAG.log | tail -20
if faulted $OUT/lane_$TAG.log; then echo FAULT; exit 99; fi
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -2 $OUT/pytest_gpu_$TAG.log
if faulted $OUT/pytest_gpu_$TAG.log; then echo FAULT; exit 99; fi
[ $rc -ne 0 ] && exit $rc
for mode in lane row; do
  if [ $mode = row ]; then export GRAPE_NO_LANE=1; fi
  timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths > $OUT/bench_c3_${mode}_$TAG.log 2>&1
  rc=$?; echo "c3 $mode rc=$rc"; grep '^{' $OUT/bench_c3_${mode}_$TAG.log | tail -1 | head -c 300; echo
  [ $rc -ne 0 ] && exit $rc
done
exit 0
