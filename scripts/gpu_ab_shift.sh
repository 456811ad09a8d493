#!/bin/bash
# Diagonal-shift A/B (grape_walk.hpp GRAPE_WALK_SHIFT): every GPU test on the in-tree build, then
# C2 and C3 bench lines for base / noshift / base.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/shift_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/shift_tests.log
faulted $O/shift_tests.log && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ab_c2.sh shift base noshift base || exit $?
BENCH_ARGS="--workload c3" STEPS=5 bash scripts/gpu_ab_c2.sh shiftc3 base noshift || exit $?
