#!/bin/bash
# C2 device-pass sizes: one bench line per --chunk (evaluations per device pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${CHUNKS:-16384 32768 65536 131072}; do
  timeout -k 10 300 python bench.py --chunk $c --batch ${BATCH:-262144} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host-paths --no-whole-matrix > gpurun_out/c2pass_$c.log 2>&1 || { tail -5 gpurun_out/c2pass_$c.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/c2pass_$c.log') if l.startswith('{')][-1]); print('$c', round(d['value']), {k: round(v, 3) for k, v in d['kernels_ms_per_pass'].items()}, round(d['roofline']['frac'], 3))"
done
