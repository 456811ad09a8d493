#!/bin/bash
# A/B of build variants (abvar/libgrape_<v>.so; "base" = the in-tree build) on C2: optional walk
# parity tests per variant (TESTS=1), then one bench line each.  bash scripts/gpu_ab_c2.sh tag v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; TAG=$1; shift
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
for v in "$@"; do
  if [ "$v" = base ]; then unset GRAPE_LIB; else export GRAPE_LIB=$PWD/abvar/libgrape_$v.so; fi
  if [ -n "${TESTS:-}" ]; then
    timeout -k 10 300 python -u -m pytest ${TESTFILE:-tests/test_gpu_walk.py} -x -q --timeout 120 --timeout-method thread > $O/ab_tests_${TAG}_$v.log 2>&1
    rc=$?; echo "$v tests rc=$rc"; tail -2 $O/ab_tests_${TAG}_$v.log
    faulted $O/ab_tests_${TAG}_$v.log && { echo FAULT; exit 99; }
    [ $rc -ne 0 ] && exit $rc
  fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host-paths ${BENCH_ARGS:-} > $O/ab_${TAG}_$v.log 2>&1
  rc=$?; faulted $O/ab_${TAG}_$v.log && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && { echo "bench $v rc=$rc"; tail -5 $O/ab_${TAG}_$v.log; exit $rc; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/ab_${TAG}_$v.log') if l.startswith('{')][-1])
k = d.get('kernels_ms_per_pass') or d.get('kernels_ms_per_step', {}); print('$v', round(d['value']), {n: round(x, 3) for n, x in k.items()}, round(d['roofline']['frac'], 3) if 'roofline' in d else d.get('kernels_frac'))
"
done
