#!/bin/bash
# GPU step: DEFLATE decode timing over the lane decoder's segments per wave
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for L in ${LANES:-16 8 4 32}; do
  echo "== lanes $L"
  BITAR_HIP_INFLATE_LANES=$L timeout -k 10 120 python scripts/kernel_bench.py --codec ${CODEC:-deflate} --kinds ${KINDS:-1,2} --reps 3 || exit 1
done
