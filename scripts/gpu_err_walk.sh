#!/bin/bash
# Image-walk tests (error sources through the chunk walks), then optionally the C3 workload
# (BENCH=1) and its rocprof kernel stats (PROF=TAG).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-errwalk}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
TESTS=${TESTS:-tests/test_gpu_walk_err.py}
timeout -k 10 600 python -u -m pytest $TESTS -x -v -s --timeout 300 --timeout-method thread > "$OUT/tests_$TAG.log" 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|imgwalk" "$OUT/tests_$TAG.log" | tail -60
faulted "$OUT/tests_$TAG.log" && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && exit $rc
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths ${BENCH_ARGS:-} > "$OUT/c3_$TAG.log" 2>&1
  rc=$?; echo "c3 rc=$rc"; faulted "$OUT/c3_$TAG.log" && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && { tail -5 "$OUT/c3_$TAG.log"; exit $rc; }
  grep '^{' "$OUT/c3_$TAG.log" | tail -1 > "$OUT/c3_$TAG.json"
  python -c "import json; d=json.load(open('$OUT/c3_$TAG.json')); print('c3', round(d['value']), d['kernels_ms_per_step'])"
fi
if [ -n "${PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$PROF" -o run -- \
    python3 "$ROOT/bench.py" --workload c3 --steps 5 --warmup 1 --no-cpu-baseline --no-host-paths ${BENCH_ARGS:-} > "$OUT/rocprof_$PROF.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  cut -d, -f1-4 "$OUT/prof_$PROF/run_kernel_stats.csv" | head -16
fi
exit 0
