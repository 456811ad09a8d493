#!/bin/bash
# Parity tests on the default build, then bench every library variant in $VARIANT_DIR (default build_variants/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-tune}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > $OUT/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_$TAG.log
  if faulted $OUT/pytest_$TAG.log; then echo FAULT; exit 99; fi
  [ $rc -ne 0 ] && exit $rc
fi
shopt -s nullglob
for lib in robustgrape_amd/libgrape.so ${VARIANT_DIR:-build_variants}/*.so; do
  name=$(basename $lib .so)
  GRAPE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-paths ${BENCH_ARGS:-} > $OUT/bench_${TAG}_$name.log 2>&1
  rc=$?; echo "$name rc=$rc"
  if faulted $OUT/bench_${TAG}_$name.log; then echo FAULT; exit 99; fi
  [ $rc -ne 0 ] && { tail -5 $OUT/bench_${TAG}_$name.log; continue; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_${TAG}_$name.log').read().strip().splitlines()[-1]); print('  %-14s %10.0f evals/s  frac=%.3f  ' % ('$name', d['value'], d['roofline']['frac']), {k: round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items() if v})"
done
