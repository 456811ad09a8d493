#!/bin/bash
# C3 device-pass sizes (image walk): one bench line per --chunk, then rocprof at PROF_CHUNK.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/c3sweep_${1:-a}; mkdir -p "$OUT"
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
for c in ${CHUNKS:-2048 4096 8192 16384}; do
  timeout -k 10 300 python bench.py --workload c3 --batch ${BATCH:-16384} --chunk $c --steps 5 --warmup 1 --no-cpu-baseline --no-host-paths > "$OUT/c3_$c.log" 2>&1
  rc=$?; faulted "$OUT/c3_$c.log" && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && { tail -5 "$OUT/c3_$c.log"; exit $rc; }
  grep '^{' "$OUT/c3_$c.log" | tail -1 > "$OUT/c3_$c.json"
  python -c "import json; d=json.load(open('$OUT/c3_$c.json')); print('chunk $c', round(d['value']), {k: round(v, 2) for k, v in d['kernels_ms_per_step'].items()})"
done
if [ -n "${PROF_CHUNK:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --workload c3 --batch ${BATCH:-16384} --chunk $PROF_CHUNK --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths > "$OUT/rocprof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
  cut -d, -f1-4 "$OUT/prof/run_kernel_stats.csv" | head -16
fi
exit 0
