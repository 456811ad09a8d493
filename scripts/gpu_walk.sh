#!/bin/bash
# Round 3: chunk-walk correctness first (new kernels), then the A/B timing, then the other
# sector / lane / parity tests.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
TAG=${1:-walk}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_walk.py -x -v --timeout 200 --timeout-method thread > "$OUT/walk_tests_$TAG.log" 2>&1
rc=$?; echo "walk tests rc=$rc"; tail -30 "$OUT/walk_tests_$TAG.log"
faulted "$OUT/walk_tests_$TAG.log" && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u scripts/probes/walk_ab.py ${AB_ARGS:-} > "$OUT/walk_ab_$TAG.log" 2>&1
rc2=$?; echo "walk ab rc=$rc2"; cat "$OUT/walk_ab_$TAG.log" | tail -5
faulted "$OUT/walk_ab_$TAG.log" && { echo FAULT; exit 99; }
[ $rc2 -ne 0 ] && exit $rc2
[ -n "${NO_MORE:-}" ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_sectors.py tests/test_gpu_lane.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$OUT/more_tests_$TAG.log" 2>&1
rc3=$?; echo "more tests rc=$rc3"; tail -15 "$OUT/more_tests_$TAG.log"
exit $rc3
