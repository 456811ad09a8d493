#!/bin/bash
# Selected GPU test files (TESTS, default: the general-H0 and walk tests) in one pytest process,
# then optionally the C2 profile (PROFILE=TAG: scripts/gpu_profile.sh with BATCH=32768).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-tests}
TESTS=${TESTS:-tests/test_gpu_general_h0.py tests/test_gpu_walk.py}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 700 python -u -m pytest $TESTS -x -v --timeout 200 --timeout-method thread > "$OUT/tests_$TAG.log" 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/tests_$TAG.log" | tail -40
faulted "$OUT/tests_$TAG.log" && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && exit $rc
if [ -n "${PROFILE:-}" ]; then
  BATCH=32768 bash scripts/gpu_profile.sh "$PROFILE" || exit $?
  grep -o '"value": [0-9.]*' "$OUT/${PROFILE}_bench.json" | head -1
fi
exit 0
