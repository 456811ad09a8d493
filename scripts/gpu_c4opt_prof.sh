#!/bin/bash
# Where the optimiser's time goes: the torch-profiler probe and a rocprof kernel trace of c4opt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/c4opt_${1:-a}; mkdir -p "$OUT"
timeout -k 10 300 python scripts/probes/opt_profile.py ${B:-1024} > "$OUT/opt_profile.log" 2>&1
rc=$?; echo "probe rc=$rc"; head -3 "$OUT/opt_profile.log"; [ $rc -ne 0 ] && { tail -20 "$OUT/opt_profile.log"; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$ROOT/bench.py" --workload c4opt --steps 10 --warmup 2 > "$OUT/bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench.log"; exit $rc; }
grep '^{' "$OUT/bench.log" | tail -1 | cut -c1-400
exit 0
