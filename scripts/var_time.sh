#!/bin/bash
# GPU step: kernel_bench with each library variant of $VARIANTS (scripts/build_variant.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in $VARIANTS; do
  echo "== $v"
  BITAR_HIP_LIB=$PWD/bitar_amd/lib/variants/libbitar_hip_$v.so timeout -k 10 120 python scripts/kernel_bench.py --codec ${CODEC:-zstd} --kinds ${KINDS:-2} --reps 2 || exit 1
done
