#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench command, then separate PMC passes
# (FETCH_SIZE / WRITE_SIZE, kernel-trace only) summarised to HBM bytes per launch.
#   bash scripts/gpu_profile.sh TAG [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
TAG=${1:-prof}; shift || true
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-host-paths --no-whole-matrix --no-c4-strong $*"
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|core dumped" "$1"; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG}_stats -o run -- \
    python3 $ROOT/bench.py $ARGS > $OUT/${TAG}_stats.log 2>&1
rc=$?; echo "stats rc=$rc"; faulted $OUT/${TAG}_stats.log && { echo FAULT; exit 99; }; [ $rc -ne 0 ] && exit $rc
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/${TAG}_pmc$i -o run -- \
      python3 $ROOT/bench.py $ARGS > $OUT/${TAG}_pmc$i.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; faulted $OUT/${TAG}_pmc$i.log && { echo FAULT; exit 99; }; [ $rc -ne 0 ] && exit $rc
done
python3 $ROOT/scripts/pmc_summary.py $OUT/${TAG}_pmc1 $OUT/${TAG}_pmc2 --batch ${BATCH:-1024} --json $OUT/${TAG}_pmc.json > $OUT/${TAG}_pmc.txt
grep '^{' $OUT/${TAG}_stats.log | tail -1 > $OUT/${TAG}_bench.json
echo done
