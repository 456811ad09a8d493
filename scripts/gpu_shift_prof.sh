#!/bin/bash
# Per-kernel A/B of the diagonal shift: walk tests on the in-tree build, then rocprofv3 kernel
# stats of a short C2 bench for base / noshift / base (GRAPE_LIB selects the variant library).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); O=$ROOT/gpurun_out; mkdir -p $O
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|hipErrorLaunchFailure|core dumped" "$1"; }
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/shiftp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/shiftp_tests.log
faulted $O/shiftp_tests.log && { echo FAULT; exit 99; }
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
n=0
for v in base noshift base; do
  n=$((n+1))
  if [ "$v" = base ]; then unset GRAPE_LIB; else export GRAPE_LIB=$ROOT/abvar/libgrape_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/shiftp_${n}_$v" -o run -- \
      python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths > "$O/shiftp_${n}_$v.log" 2>&1
  rc=$?; faulted "$O/shiftp_${n}_$v.log" && { echo FAULT; exit 99; }
  [ $rc -ne 0 ] && { echo "rocprof $v rc=$rc"; exit $rc; }
  f=$(find "$O/shiftp_${n}_$v" -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "k_walk_(fwd|grad)<" "$f" | awk -F'",' '{split($2,a,","); printf "%s %.3f ms\n", substr($1,2,45), a[3]/1e6}'
  grep -o '"value": [0-9.]*' "$O/shiftp_${n}_$v.log" | head -1
done
