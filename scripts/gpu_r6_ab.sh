#!/bin/bash
# Round 6: the gauge / walk / eval1 parity tests on the in-tree build, then C2 A/B of build variants
# (abvar/libgrape_<v>.so, "base" = in-tree).  bash scripts/gpu_r6_ab.sh TAG v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; TAG=$1; shift
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $O/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.log
  faulted $O/${TAG}_tests.log && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && exit $rc
fi
STEPS=${STEPS:-20} BENCH_ARGS="--no-whole-matrix --no-c4-strong ${BENCH_ARGS:-}" bash scripts/gpu_ab_c2.sh $TAG "$@"
