#!/bin/bash
# One GPU validation pass: parity tests, smoke, bench, rocprof kernel trace.
# Stops at the first step that does not end with 0 (tests: 0 or 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r01}
STEPS=${STEPS:-20}
# a runtime fault can leave the exit code at 0 or 1: treat its message as fatal
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }

timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu_$TAG.log"
if faulted "$OUT/pytest_gpu_$TAG.log"; then echo "GPU FAULT in pytest"; exit 99; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "${TESTS_ONLY:-}" ] && exit $rc

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke_$TAG.log"
if faulted "$OUT/smoke_$TAG.log"; then echo "GPU FAULT in smoke"; exit 99; fi
if [ $rc -ne 0 ]; then exit $rc; fi

timeout -k 10 400 python bench.py --steps "$STEPS" --warmup 3 > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench_$TAG.log"
if faulted "$OUT/bench_$TAG.log"; then echo "GPU FAULT in bench"; exit 99; fi
[ $rc -ne 0 ] && exit $rc

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths > "$OUT/rocprof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/rocprof_$TAG.log"
find "$OUT/prof_$TAG" -name "*stats*" | head
exit $rc
