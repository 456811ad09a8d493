#!/bin/bash
# Round-5 check on one MI355X: the GPU suite + smoke (gpu_final.sh without the profile), then the
# dense-engine FD-noise probe for the in-tree library (Gauss 3M) and the 4M variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r5}
SKIP_PROFILE=1 SKIP_BENCH=${SKIP_BENCH:-} bash scripts/gpu_final.sh $TAG || exit $?
timeout -k 10 600 python -u scripts/probes/fd_exact_probe.py --gpu > $OUT/${TAG}_fd_exact.log 2>&1 || { tail -5 $OUT/${TAG}_fd_exact.log; exit 1; }
tail -5 $OUT/${TAG}_fd_exact.log | cut -c1-400
timeout -k 10 300 python -u scripts/probes/dense_fd_noise.py 3m > $OUT/${TAG}_noise_3m.log 2>&1 || { tail -5 $OUT/${TAG}_noise_3m.log; exit 1; }
tail -1 $OUT/${TAG}_noise_3m.log
if [ -f robustgrape_amd/libgrape_4m.so ]; then
  GRAPE_LIB=robustgrape_amd/libgrape_4m.so timeout -k 10 300 python -u scripts/probes/dense_fd_noise.py 4m \
      > $OUT/${TAG}_noise_4m.log 2>&1 || { tail -5 $OUT/${TAG}_noise_4m.log; exit 1; }
  tail -1 $OUT/${TAG}_noise_4m.log
fi
exit 0
