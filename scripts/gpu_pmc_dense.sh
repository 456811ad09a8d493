#!/bin/bash
# PMC passes for the dense (MFMA) engine on the C5 bench: MFMA busy, LDS, waits.
#   bash scripts/gpu_pmc_dense.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD; OUT=$ROOT/gpurun_out; mkdir -p $OUT
TAG=${1:-pmcd}
cd /tmp && export TMPDIR=/tmp
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $group --kernel-trace --output-format csv -d $OUT/${TAG}_p$i -o run -- \
      python3 $ROOT/bench.py --workload ${WORKLOAD:-c5} --batch 16 --steps 2 --warmup 1 --no-cpu-baseline --no-host-paths > $OUT/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  if grep -qE "HSA_STATUS_ERROR|illegal memory access|Memory access fault" $OUT/${TAG}_p$i.log; then echo FAULT; exit 99; fi
  [ $rc -ne 0 ] && { tail -5 $OUT/${TAG}_p$i.log; exit $rc; }
done <<GROUPS
SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE
GROUPS
exit 0
