#!/bin/bash
# GPU-box step: parity of variant $V (compress bit-exact vs the oracle, every codec on the
# window parse), then an interleaved A/B against the in-tree library:
#   V=chain3 CODECS="lz4 zstd deflate" KINDS=1,2,5,6 scripts/gpu_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
lib=$PWD/bitar_amd/lib/variants/libbitar_hip_$V.so
if [ -z "$NO_TESTS" ]; then
  BITAR_HIP_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_deflate.py tests/test_gpu_zstd.py \
    -x -q --timeout 200 --timeout-method thread -k "${TEST_K:-compress and not 1gib and not full_size}" > gpurun_out/ab_tests_$V.log 2>&1 \
    || { echo "variant tests failed"; tail -30 gpurun_out/ab_tests_$V.log; exit 1; }
  tail -2 gpurun_out/ab_tests_$V.log
fi
for codec in ${CODECS:-lz4}; do
  VARIANTS="cur $V" CODEC=$codec KINDS=${KINDS:-1,2,5,6} ROUNDS=${ROUNDS:-2} scripts/ab.sh > gpurun_out/ab_${V}_$codec.txt 2>&1 || { echo "ab failed"; tail -20 gpurun_out/ab_${V}_$codec.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab_${V}_$codec.txt
done
