#!/bin/bash
# A/B of plan options on one workload, interleaved: bash scripts/gpu_opts_ab.sh TAG WORKLOAD opt1 opt2 ...
# (each option value is passed as --plan-options; the list may repeat values: A B A B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; TAG=$1; WL=$2; shift 2
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
i=0
for v in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --workload $WL --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host-paths \
      --no-whole-matrix --plan-options $v ${BENCH_ARGS:-} > $O/opts_${TAG}_${i}_$v.log 2>&1
  rc=$?; faulted $O/opts_${TAG}_${i}_$v.log && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && { echo "bench $v rc=$rc"; tail -5 $O/opts_${TAG}_${i}_$v.log; exit $rc; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/opts_${TAG}_${i}_$v.log') if l.startswith('{')][-1])
k = d.get('kernels_ms_per_pass') or d.get('kernels_ms_per_step', {}); print('opt=$v', round(d['value']), {n: round(x, 3) for n, x in k.items()}, round(d['roofline']['frac'], 3) if 'roofline' in d else '')
"
done
