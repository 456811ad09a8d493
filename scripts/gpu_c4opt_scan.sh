#!/bin/bash
# c4opt: the optimiser's plan at 8- vs 16-wave scans (plan options, scan waves), one bench line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${CFGS:-0_8 0_16 128_16 0_8}; do
  o=${c%_*}; w=${c#*_}
  timeout -k 10 200 python bench.py --workload c4opt --steps 10 --warmup 2 --plan-options $o --scan-waves $w > gpurun_out/c4o_$c.log 2>&1 || { tail -5 gpurun_out/c4o_$c.log; exit 1; }
  grep '^{' gpurun_out/c4o_$c.log | tail -1 > gpurun_out/c4o_$c.json
  python -c "import json; d=json.load(open('gpurun_out/c4o_$c.json')); print('$c', round(d['value']), round(d['ms_per_step'], 3), d.get('optimizer'))"
done
