#!/bin/bash
# Walk tests, then a kernel trace and two PMC passes over the walk A/B probe, then the other
# sector / lane / parity tests.  Stops at the first failing GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-walkprof}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_walk.py -x -v --timeout 200 --timeout-method thread > "$OUT/walk_tests_$TAG.log" 2>&1
rc=$?; echo "walk tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error" "$OUT/walk_tests_$TAG.log" | tail -25
faulted "$OUT/walk_tests_$TAG.log" && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$ROOT/scripts/probes/walk_ab.py" --opts ${AB_OPTS:-0,32} --steps 4 > "$OUT/rocprof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/rocprof_$TAG.log"
faulted "$OUT/rocprof_$TAG.log" && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && exit $rc
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --kernel-trace --output-format csv -d "$OUT/pmc_${TAG}_p$i" -o run -- \
      python3 "$ROOT/scripts/probes/walk_ab.py" --opts 0 --steps 1 --batch 32768 > "$OUT/pmc_${TAG}_p$i.log" 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"
  faulted "$OUT/pmc_${TAG}_p$i.log" && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && exit $rc
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY
SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU GRBM_GUI_ACTIVE
GROUPS
cd "$ROOT"
[ -n "${NO_MORE:-}" ] && exit 0
timeout -k 10 700 python -u -m pytest tests/test_gpu_sectors.py tests/test_gpu_lane.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$OUT/more_tests_$TAG.log" 2>&1
rc3=$?; echo "more tests rc=$rc3"; tail -15 "$OUT/more_tests_$TAG.log"
exit $rc3
