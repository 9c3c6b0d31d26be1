#!/bin/bash
# GPU step: LZ4 kernel timing of every lz4 variant library, interleaved twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in 1 2; do
for lib in bitar_amd/lib/variants/libbitar_hip_lz4_*.so; do
  echo "== $lib"
  BITAR_HIP_LIB=$lib timeout -k 10 120 python scripts/kernel_bench.py --codec lz4 --kinds ${KINDS:-1,2} --reps 5 || exit 1
done
done
