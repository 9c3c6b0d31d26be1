#!/bin/bash
# GPU step: Zstd decode time of executor variants (scripts/build_variant.sh zh1..3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for k in ${VARIANTS:-zh1 zh2 zh3}; do
  echo "variant $k"
  BITAR_HIP_LIB=$PWD/bitar_amd/lib/variants/libbitar_hip_$k.so timeout -k 10 120 python scripts/kernel_bench.py --codec zstd --kinds ${KINDS:-2} --reps 2 > gpurun_out/$k.log 2>&1 || { tail -20 gpurun_out/$k.log; exit 1; }
  grep decompress_ms gpurun_out/$k.log
done
