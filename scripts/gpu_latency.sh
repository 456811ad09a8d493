#!/bin/bash
# Latency work: full GPU tests, the single-evaluation probe + kernel trace, one bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); TAG=${1:-a}; OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread ${TESTS_K:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu_$TAG.log"
  faulted "$OUT/pytest_gpu_$TAG.log" && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && exit $rc
fi
bash scripts/gpu_single_prof.sh $TAG || exit $?
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; faulted "$OUT/bench_$TAG.log" && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && { tail -5 "$OUT/bench_$TAG.log"; exit $rc; }
python3 -c "
import json
d=json.loads([l for l in open('$OUT/bench_$TAG.log') if l.startswith('{')][-1])
print('C2', round(d['value']), 'single', d.get('single_eval',{}).get('value'), d.get('single_eval',{}).get('latency_ms_median'), 'c4', {k:(round(v['value']),round(v['ms_per_step'],4)) for k,v in d.get('c4_points',{}).items() if isinstance(v,dict)})
"
