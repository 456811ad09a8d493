#!/bin/bash
# Round-5 measurements on one MI355X: C2 and C3 with the phase-covariant walks (default) against the
# per-step exponentials (GRAPE_OPT_NO_GAUGE = 8192) in one call, then the default bench line with
# every leg, then the rocprofv3 kernel-trace stats + PMC HBM passes + instruction mix of C2.
#   bash scripts/gpu_r5_perf.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r5p}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
run() {  # name, timeout, args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py "$@" > $OUT/${TAG}_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; faulted $OUT/${TAG}_$name.log && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && { tail -5 $OUT/${TAG}_$name.log; exit $rc; }
  grep '^{' $OUT/${TAG}_$name.log | tail -1 | python3 -c "import sys,json; d=json.load(sys.stdin); print('  value', d['value'], 'ms/step', d['ms_per_step'], {k: round(v, 4) for k, v in d.get('kernels_ms_per_pass', d.get('kernels_ms_per_step', {})).items()})"
}
Q="--no-cpu-baseline --no-host-paths --no-whole-matrix --no-c4-strong"
run c2_gauge 300 --steps 50 $Q
run c2_nogauge 300 --steps 50 $Q --plan-options 8192
run c2_gauge_b 300 --steps 50 $Q
run c3_gauge 300 --workload c3 --steps 20 $Q
run c3_nogauge 300 --workload c3 --steps 20 $Q --plan-options 8192
run c2_full 600
[ -n "${SKIP_PROFILE:-}" ] && exit 0
BATCH=32768 bash scripts/gpu_profile.sh ${TAG}_c2 || exit $?
BATCH=32768 bash scripts/gpu_pmc_mix.sh ${TAG}_c2mix || exit $?
exit 0
