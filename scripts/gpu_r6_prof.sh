#!/bin/bash
# Round 6 profiling on one MI355X: the C2 instruction-mix PMC passes (scripts/gpu_pmc_mix.sh), then
# rocprofv3 kernel-trace stats of the latency legs (ar_cz single evaluation, c4opt).  Each GPU step has
# its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
TAG=${1:-r6prof}
faulted() { grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault|core dumped" "$1"; }
# keep what comes back small (gpurun merges at most 64 MiB): per-dispatch traces and counter rows are
# summarised, then removed; the rocprof stats tables stay
prune() { find "$1" -name "*kernel_trace.csv" -delete 2>/dev/null; find "$1" -name "*counter_collection.csv" -delete 2>/dev/null
          find "$1" -name "*.db" -delete 2>/dev/null; find "$1" -name "*agent_info.csv" -delete 2>/dev/null; true; }
for leg in ${LEGS:-mix arcz c4opt}; do
  case $leg in
    mix) BATCH=32768 bash scripts/gpu_pmc_mix.sh ${TAG}_mix || exit $?; for d in $OUT/${TAG}_mix_p*; do prune $d; done ;;
    c2stats) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $OUT/${TAG}_c2 -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-paths \
          --no-whole-matrix --no-c4-strong > $OUT/${TAG}_c2.log 2>&1); rc=$?; echo "c2 stats rc=$rc"
          faulted $OUT/${TAG}_c2.log && exit 99; [ $rc -ne 0 ] && exit $rc; prune $OUT/${TAG}_c2 ;;
    c3stats) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $OUT/${TAG}_c3 -o run -- python3 $ROOT/bench.py --workload c3 --steps 6 --warmup 2 --no-cpu-baseline --no-host-paths > $OUT/${TAG}_c3.log 2>&1)
          rc=$?; echo "c3 stats rc=$rc"; faulted $OUT/${TAG}_c3.log && exit 99; [ $rc -ne 0 ] && exit $rc; prune $OUT/${TAG}_c3 ;;
    c3mix) BATCH=8192 BENCH_EXTRA="--workload c3" bash scripts/gpu_pmc_mix.sh ${TAG}_c3mix || exit $?; for d in $OUT/${TAG}_c3mix_p*; do prune $d; done ;;
    arcz) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $OUT/${TAG}_arcz -o run -- python3 $ROOT/bench.py --workload arcz --no-cpu-baseline > $OUT/${TAG}_arcz.log 2>&1)
          rc=$?; echo "arcz rc=$rc"; faulted $OUT/${TAG}_arcz.log && exit 99; [ $rc -ne 0 ] && exit $rc; prune $OUT/${TAG}_arcz ;;
    c4opt) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $OUT/${TAG}_c4opt -o run -- python3 $ROOT/bench.py --workload c4opt --steps 20 --warmup 5 > $OUT/${TAG}_c4opt.log 2>&1)
          rc=$?; echo "c4opt rc=$rc"; faulted $OUT/${TAG}_c4opt.log && exit 99; [ $rc -ne 0 ] && exit $rc; prune $OUT/${TAG}_c4opt ;;
  esac
done
exit 0
