#!/bin/bash
# GPU step: compress parity of the shipped library, then compress/decompress timing of every
# variant library (bitar_amd/lib/variants), LZ4 and DEFLATE, interleaved twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_deflate.py -x -q -m gpu \
  --timeout 120 --timeout-method thread || exit 1
for rep in 1 2; do
for lib in bitar_amd/lib/variants/libbitar_hip_*.so; do
  for c in ${CODECS:-lz4 deflate}; do
    echo "== $lib $c"
    BITAR_HIP_LIB=$lib timeout -k 10 120 python scripts/kernel_bench.py --codec $c --kinds ${KINDS:-1,2} --reps 5 || exit 1
  done
done
done
