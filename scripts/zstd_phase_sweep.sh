#!/bin/bash
# GPU step: compress time of the Zstd entropy kernel cut after each phase (BITAR_ZSTD_STOP
# variants built beforehand by: for k in 1 2 3 4 5; do scripts/build_variant.sh zs$k -DBITAR_ZSTD_STOP=$k; done)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for k in ${PHASES:-1 2 3 4 5}; do
  echo "phase $k"
  mkdir -p gpurun_out
  BITAR_HIP_LIB=$PWD/bitar_amd/lib/variants/libbitar_hip_zs$k.so timeout -k 10 120 python scripts/kernel_bench.py --codec zstd --kinds ${KINDS:-2} --reps 2 > gpurun_out/zs$k.log 2>&1 || { tail -20 gpurun_out/zs$k.log; exit 1; }
  grep compress_ms gpurun_out/zs$k.log
done
