#!/bin/bash
# A/B of exponential-kernel build variants (abvar/libgrape_<v>.so; "base" = the in-tree build)
# on C2 and C3: bash scripts/ab_lowexp.sh v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then unset GRAPE_LIB; else export GRAPE_LIB=$PWD/abvar/libgrape_$v.so; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths > $O/ab_c2_$v.log 2>&1 || { echo "bench c2 $v failed"; tail -5 $O/ab_c2_$v.log; exit 1; }
  timeout -k 10 300 python bench.py --workload c3 --steps 6 --warmup 2 --no-cpu-baseline --no-host-paths > $O/ab_c3_$v.log 2>&1 || { echo "bench c3 $v failed"; exit 1; }
  python3 -c "
import json
for w in ('c2','c3'):
    d=json.loads([l for l in open('$O/ab_'+w+'_$v.log') if l.startswith('{')][-1])
    print('$v', w, round(d['value']), {k: round(x,2) for k,x in d['kernels_ms_per_step'].items()}, round(d['roofline']['frac'],3))
"
done
