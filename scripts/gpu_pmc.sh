#!/bin/bash
# PMC counter passes (one --pmc group per pass, kernel-trace only; no sys/runtime trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
TAG=${1:-pmc}
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/${TAG}_counters.txt 2>&1 || true
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $group --kernel-trace --output-format csv -d $OUT/${TAG}_p$i -o run -- \
      python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-paths ${BENCH_ARGS:-} > $OUT/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  if grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault" $OUT/${TAG}_p$i.log; then echo FAULT; exit 99; fi
  [ $rc -ne 0 ] && { tail -5 $OUT/${TAG}_p$i.log; }
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY
SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE
GROUPS
exit 0
