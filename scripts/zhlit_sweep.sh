#!/bin/bash
# GPU step: Zstd kind-2 decode time over zstd_hlit_kernel's segments per wave (4 / 8 / 16)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for hs in 16 8 4; do
  echo "BITAR_HIP_HLIT_SEGS=$hs"
  BITAR_HIP_HLIT_SEGS=$hs timeout -k 10 200 python -u scripts/kernel_bench.py --codec zstd --kinds ${KINDS:-2} --reps 2 || exit 1
done
