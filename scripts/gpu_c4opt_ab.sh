#!/bin/bash
# c4opt A/B: plan options / scan widths of the optimiser's plan, one bench line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c4ab_${1:-a}; mkdir -p $OUT
for cfg in ${CFGS:-0,0 128,0 0,8 128,8}; do  # plan options,scan waves
  set -- ${cfg/,/ }
  timeout -k 10 200 python bench.py --workload c4opt --steps 10 --warmup 2 --plan-options $1 --scan-waves $2 > $OUT/o$1_w$2.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/o$1_w$2.log; exit $rc; }
  grep '^{' $OUT/o$1_w$2.log | tail -1 > $OUT/o$1_w$2.json
  python -c "import json; d=json.load(open('$OUT/o$1_w$2.json')); print('options $1 scan $2:', round(d['value']), 'ms/it', round(d['ms_per_step'], 3), d['optimizer'])"
done
