#!/bin/bash
# A/B of the working tree against another checkout with its own built library (abvar/<name>/, e.g. a
# `git worktree` of HEAD): one bench line each, alternating.  bash scripts/gpu_ab_tree.sh tag name cur name cur ...
# ("cur" = this tree).  BENCH_ARGS / STEPS as in gpu_ab_c2.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; O=$ROOT/gpurun_out; mkdir -p $O; TAG=$1; shift
for v in "$@"; do
  if [ "$v" = cur ]; then d=$ROOT; else d=$ROOT/abvar/$v; fi
  (cd $d && timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host-paths ${BENCH_ARGS:-} > $O/abt_${TAG}_$v.log 2>&1)
  rc=$?
  grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" $O/abt_${TAG}_$v.log && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && { echo "bench $v rc=$rc"; tail -5 $O/abt_${TAG}_$v.log; exit $rc; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/abt_${TAG}_$v.log') if l.startswith('{')][-1])
k = d.get('kernels_ms_per_pass') or d.get('kernels_ms_per_step', {}); print('$v', round(d['value']), {n: round(x, 3) for n, x in k.items()}, round(d['roofline']['frac'], 3) if 'roofline' in d else d.get('kernels_frac'))
"
done
