#!/bin/bash
# Lane-matrix kernels: parity (bitwise vs the row groups + oracle), full GPU suite, A/B bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-lane}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py -x -v -s --timeout 120 --timeout-method thread > $OUT/lane_$TAG.log 2>&1
rc=$?; echo "lane tests rc=$rc"; grep -E "PASS|FAIL|Error|oracle" $OUT/lane_$TAG.log | tail -20
if faulted $OUT/lane_$TAG.log; then echo FAULT; exit 99; fi
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 $OUT/pytest_gpu_$TAG.log
if faulted $OUT/pytest_gpu_$TAG.log; then echo FAULT; exit 99; fi
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths > $OUT/bench_lane_$TAG.log 2>&1
rc=$?; echo "bench lane rc=$rc"; tail -c 1500 $OUT/bench_lane_$TAG.log | head -c 700; echo
[ $rc -ne 0 ] && exit $rc
GRAPE_NO_LANE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths > $OUT/bench_rowgroup_$TAG.log 2>&1
rc=$?; echo "bench rowgroup rc=$rc"; tail -c 1500 $OUT/bench_rowgroup_$TAG.log | head -c 700; echo
exit $rc
