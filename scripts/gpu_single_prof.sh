#!/bin/bash
# Where a single evaluation's time goes: the probe's wall clock, then its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/single_${1:-a}; mkdir -p "$OUT"
timeout -k 10 120 python scripts/probes/single_probe.py > "$OUT/probe.log" 2>&1
rc=$?; echo "probe rc=$rc"; tail -2 "$OUT/probe.log"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
CALLS=200 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$ROOT/scripts/probes/single_probe.py" > "$OUT/rocprof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$OUT/rocprof.log"
exit $rc
