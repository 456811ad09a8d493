#!/bin/bash
# Instruction-mix PMC passes of the default bench (one counter group per rocprofv3 run, kernel
# trace only), summarised by scripts/pmc_mix.py into gpurun_out/TAG_mix.json (the bench reads the
# committed copy, profiles/pmc_mix_latest.json, for its roofline's executed-FP64 field).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
TAG=${1:-mix}
cd /tmp && export TMPDIR=/tmp
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" \
             "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $group --kernel-trace --output-format csv -d $OUT/${TAG}_p$i -o run -- \
      python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths --no-whole-matrix --no-c4-strong ${BENCH_EXTRA:-} > $OUT/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault" $OUT/${TAG}_p$i.log; then echo FAULT; exit 99; fi
  [ $rc -ne 0 ] && { tail -5 $OUT/${TAG}_p$i.log; exit $rc; }
done
python3 $ROOT/scripts/pmc_mix.py $OUT/$TAG --json $OUT/${TAG}_mix.json --batch ${BATCH:-32768} > $OUT/${TAG}_mix.txt
cat $OUT/${TAG}_mix.txt
exit 0
