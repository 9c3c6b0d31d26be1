#!/bin/bash
# GPU step: kernel timing of every variant library (bitar_amd/lib/variants), interleaved twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in 1 2; do
for lib in bitar_amd/lib/variants/libbitar_hip_*.so; do
  for c in ${CODECS:-lz4}; do
    echo "== $lib $c"
    BITAR_HIP_LIB=$lib timeout -k 10 120 python scripts/kernel_bench.py --codec $c --kinds ${KINDS:-1,2} --reps ${REPS:-3} || exit 1
  done
done
done
