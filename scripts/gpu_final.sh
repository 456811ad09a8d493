#!/bin/bash
# End-of-round check on one MI355X: the whole GPU test suite (one pytest process), smoke(), the
# default bench line, then the rocprof kernel-trace stats and the PMC passes of the same bench
# command (scripts/gpu_profile.sh).  Each GPU step has its own time limit; the script stops at the
# first failure.  Outputs under gpurun_out/final_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-final}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > $OUT/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $OUT/${TAG}_tests.log
  faulted $OUT/${TAG}_tests.log && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc
if [ -z "${SKIP_BENCH:-}" ]; then
  timeout -k 10 600 python bench.py > $OUT/${TAG}_bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; faulted $OUT/${TAG}_bench.log && { echo FAULT; exit 99; }; [ $rc -ne 0 ] && exit $rc
  grep '^{' $OUT/${TAG}_bench.log | tail -1 | cut -c1-300
fi
if [ -z "${SKIP_PROFILE:-}" ]; then
  BATCH=32768 bash scripts/gpu_profile.sh ${TAG}_c2 || exit $?
fi
exit 0
