#!/bin/bash
# Round-3 batch: full GPU tests, c4opt A/B, C3 rocprof + HBM PMC at the bench pass size, C2
# instruction-mix PMC passes.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-b}
TESTS_ONLY=1 bash scripts/gpu_round.sh $TAG || exit $?
bash scripts/gpu_c4opt_ab.sh $TAG || exit $?
BATCH=8192 bash scripts/gpu_profile.sh c3_$TAG --workload c3 || exit $?
BENCH_ARGS="--no-whole-matrix" bash scripts/gpu_pmc.sh c2mix_$TAG || exit $?
python3 scripts/pmc_summary.py gpurun_out/c2mix_${TAG}_p1 gpurun_out/c2mix_${TAG}_p2 gpurun_out/c2mix_${TAG}_p5 --batch 32768 > gpurun_out/c2mix_${TAG}.txt
echo batch done
