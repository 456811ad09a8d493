#!/bin/bash
# Round-6 baseline legs on one MI355X: c4opt (device optimiser), C3 with its latency legs, the
# ar_cz-shaped single evaluation.  Each GPU step has its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; TAG=${1:-r6base}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
run() {  # name, limit, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/${TAG}_$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; faulted $O/${TAG}_$n.log && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && { tail -5 $O/${TAG}_$n.log; exit $rc; }
  grep '^{' $O/${TAG}_$n.log | tail -1 | cut -c1-400
}
for leg in ${LEGS:-arcz c3 c4opt}; do
  case $leg in
    arcz) run arcz 200 --workload arcz ;;
    c3) run c3 300 --workload c3 --steps 10 --warmup 2 --no-cpu-baseline ;;
    c4opt) run c4opt 300 --workload c4opt --steps 20 --warmup 5 ;;
    c2) run c2 300 --steps 20 --warmup 3 --no-cpu-baseline --no-whole-matrix ${C2ARGS:-} ;;
  esac
done
exit 0
