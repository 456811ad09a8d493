#!/bin/bash
# Chain kernels: lane parity tests, then kernel stats with and without the per-lane chains.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
TAG=${1:-cab}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_sectors.py -x -q --timeout 120 --timeout-method thread > $OUT/chain_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/chain_tests_$TAG.log
if faulted $OUT/chain_tests_$TAG.log; then echo FAULT; exit 99; fi
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for mode in chain nochain; do
  [ $mode = nochain ] && export GRAPE_NO_CHAIN=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${mode}_$TAG" -o run -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-host-paths > "$OUT/prof_${mode}_$TAG.log" 2>&1
  rc=$?; echo "$mode rc=$rc"; grep '^{' "$OUT/prof_${mode}_$TAG.log" | tail -1 | head -c 120; echo
  [ $rc -ne 0 ] && exit $rc
done
exit 0
