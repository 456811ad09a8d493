#!/bin/bash
# Per-instantiation kernel times, lane-matrix vs row-group kernels (rocprofv3 kernel stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
TAG=${1:-lp}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_lane_$TAG" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths > "$OUT/prof_lane_$TAG.log" 2>&1
rc=$?; echo "lane rc=$rc"; [ $rc -ne 0 ] && exit $rc
export GRAPE_NO_LANE=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_row_$TAG" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths > "$OUT/prof_row_$TAG.log" 2>&1
rc=$?; echo "row rc=$rc"; exit $rc
