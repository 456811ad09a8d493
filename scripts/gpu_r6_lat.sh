#!/bin/bash
# Round 6 latency legs: parity tests (TESTS), then per build variant (abvar/libgrape_<v>.so, "base" =
# in-tree) the ar_cz single evaluation, c4opt and C2 at small device passes.  Each GPU step has its own
# limit; stop at the first failure.   bash scripts/gpu_r6_lat.sh TAG v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O; TAG=$1; shift
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.log
  faulted $O/${TAG}_tests.log && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && exit $rc
fi
run() {  # variant leg limit args...
  local v=$1 n=$2 t=$3; shift 3
  timeout -k 10 $t python bench.py "$@" > $O/${TAG}_${v}_$n.log 2>&1
  local rc=$?; faulted $O/${TAG}_${v}_$n.log && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && { echo "$v $n rc=$rc"; tail -5 $O/${TAG}_${v}_$n.log; exit $rc; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/${TAG}_${v}_$n.log') if l.startswith('{')][-1])
se=d.get('single_eval') or {}
print('$v', '$n', round(d['value']), round(d.get('ms_per_step', 0), 4), se.get('latency_ms_median'), se.get('c_entry_latency_ms_median'))
"
}
for v in "$@"; do
  if [ "$v" = base ]; then unset GRAPE_LIB; else export GRAPE_LIB=$PWD/abvar/libgrape_$v.so; fi
  for leg in ${LEGS:-arcz c4opt c2k1 c2k4}; do
    case $leg in
      arcz) run $v arcz 200 --workload arcz --no-cpu-baseline ;;
      c3) run $v c3 300 --workload c3 --steps 10 --warmup 2 --no-cpu-baseline ;;
      c3p16) run $v c3p16 300 --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths --chunk 16384 ;;
      c3p4) run $v c3p4 300 --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths --chunk 4096 ;;
      c4opt) run $v c4opt 300 --workload c4opt --steps 20 --warmup 5 ;;
      c5) run $v c5 300 --workload c5 --steps 30 --warmup 3 --no-cpu-baseline --no-host-paths ;;
      c5err) run $v c5err 300 --workload c5err --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths ;;
      c4optw0) run $v c4optw0 300 --workload c4opt --steps 20 --warmup 5 --scan-waves 0 ;;
      c2k2) run $v c2k2 300 --chunk 2048 --batch 65536 --steps 20 --warmup 3 --no-cpu-baseline --no-host-paths --no-whole-matrix --no-c4-strong ;;
      c2k1) run $v c2k1 300 --chunk 1024 --batch 65536 --steps 20 --warmup 3 --no-cpu-baseline --no-host-paths --no-whole-matrix --no-c4-strong ;;
      c2k4) run $v c2k4 300 --chunk 4096 --batch 65536 --steps 20 --warmup 3 --no-cpu-baseline --no-host-paths --no-whole-matrix --no-c4-strong ;;
    esac
  done
done
exit 0
