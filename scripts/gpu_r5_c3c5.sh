#!/bin/bash
# Round-5 C3 / C5 evidence on one MI355X: the C3 bench under rocprofv3 (kernel stats, HBM PMC
# passes, instruction mix), the full C5 bench (with its CPU baseline), and the dense engine's
# MFMA / LDS PMC passes.  Every step under its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
TAG=${1:-r5}
BATCH=${C3_PASS:-8192} bash scripts/gpu_profile.sh ${TAG}c3 --workload c3 || exit $?
BATCH=${C3_PASS:-8192} BENCH_EXTRA="--workload c3" bash scripts/gpu_pmc_mix.sh ${TAG}c3mix || exit $?
timeout -k 10 420 python -u bench.py --workload c5 > $OUT/${TAG}c5_bench.log 2>&1 || { tail -5 $OUT/${TAG}c5_bench.log; exit 1; }
tail -c 400 $OUT/${TAG}c5_bench.log
bash scripts/gpu_pmc_dense.sh ${TAG}c5pmc || exit $?
exit 0
