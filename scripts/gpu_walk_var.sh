#!/bin/bash
# Walk tests on the default build, then the A/B probe under rocprof for each tuning variant
# in tunelibs/ (GRAPE_LIB selects the library).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-var}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 500 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_sectors.py -x -v --timeout 200 --timeout-method thread > "$OUT/walk_tests_$TAG.log" 2>&1
rc=$?; echo "walk tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error" "$OUT/walk_tests_$TAG.log" | tail -8
faulted "$OUT/walk_tests_$TAG.log" && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
for lib in $ROOT/robustgrape_amd/libgrape.so $ROOT/tunelibs/*.so; do
  v=$(basename $lib .so)
  GRAPE_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_$v" -o run -- \
      python3 "$ROOT/scripts/probes/walk_ab.py" --opts 0 --steps 6 > "$OUT/ab_${TAG}_$v.log" 2>&1
  rc=$?; echo "$v rc=$rc $(grep evals_per_s $OUT/ab_${TAG}_$v.log | cut -c1-120)"
  faulted "$OUT/ab_${TAG}_$v.log" && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && exit $rc
done
exit 0
