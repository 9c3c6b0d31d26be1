#!/bin/bash
# GPU step: compress parity of a variant library (VAR=name under bitar_amd/lib/variants), then
# compress/decompress timing of the shipped library and the variant, interleaved twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=bitar_amd/lib/variants/libbitar_hip_$VAR.so
BITAR_HIP_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_deflate.py tests/test_gpu_zstd.py -x -q -m gpu \
  --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
for rep in 1 2; do
for lib in bitar_amd/lib/libbitar_hip.so $V; do
  for c in ${CODECS:-lz4}; do
    echo "== $lib $c"
    BITAR_HIP_LIB=$lib timeout -k 10 120 python scripts/kernel_bench.py --codec $c --kinds ${KINDS:-1,2} --reps 5 || exit 1
  done
done
done
