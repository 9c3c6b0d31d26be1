#!/bin/bash
# GPU step: DEFLATE decode time over inflate_lanes_kernel's lanes per wave, at two input sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for b in ${SIZES:-268435456 1073741824}; do
  for l in ${LANES:-1 2 4 8}; do
    echo "bytes=$b lanes=$l"
    BITAR_HIP_INFLATE_LANES=$l timeout -k 10 120 python scripts/kernel_bench.py --codec deflate --kinds ${KINDS:-1} --bytes $b --reps 2 || exit 1
  done
done
