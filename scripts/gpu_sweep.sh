#!/bin/bash
# Bench one library over several batch sizes: gpu_sweep.sh TAG LIB "B1 B2 ..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=$1; LIB=$2; BATCHES=$3
for bsz in $BATCHES; do
  GRAPE_LIB=$PWD/$LIB timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths --batch $bsz > $OUT/sweep_${TAG}_$bsz.log 2>&1
  rc=$?
  if grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|core dumped" $OUT/sweep_${TAG}_$bsz.log; then echo FAULT; exit 99; fi
  [ $rc -ne 0 ] && { echo "B=$bsz rc=$rc"; tail -3 $OUT/sweep_${TAG}_$bsz.log; exit $rc; }
  python -c "import json; d=json.loads(open('$OUT/sweep_${TAG}_$bsz.log').read().strip().splitlines()[-1]); print('  %-8s B=%-5d %10.0f evals/s ' % ('$TAG', $bsz, d['value']), {k: round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items() if v})"
done
