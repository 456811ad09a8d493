#!/bin/bash
# The whole GPU suite on the default build (captured calls do not fork), then again with every
# plan's captured small calls forking the second sector class (GRAPE_GRAPH_FORK=1, the
# GRAPE_OPT_GRAPH_FORK path) under Python's faulthandler, so a host crash names its test and stack.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-fork}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
SKIP_BENCH=1 SKIP_PROFILE=1 bash scripts/gpu_final.sh ${TAG}_default || exit $?
GRAPE_GRAPH_FORK=1 timeout -k 10 600 python -X faulthandler -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread > $OUT/${TAG}_forked_tests.log 2>&1
rc=$?; echo "forked suite rc=$rc"; tail -3 $OUT/${TAG}_forked_tests.log
faulted $OUT/${TAG}_forked_tests.log && { echo FAULT; exit 99; }
exit $rc
