#!/bin/bash
# GPU-box step: DEFLATE GPU tests, A/B of $VARIANTS (kernel_bench, fixed and dynamic DEFLATE at
# 59460-B segments, kinds $KINDS), stock decode of each variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_mutations.py -x -q -m gpu \
  --timeout 300 --timeout-method thread -k "deflate or inflate or Deflate" > gpurun_out/t_d.log 2>&1 || { tail -30 gpurun_out/t_d.log; exit 1; }
tail -n 1 gpurun_out/t_d.log
: > gpurun_out/ab.txt
for c in deflate deflate_dyn; do
  VARIANTS="${VARIANTS:-head cur}" ROUNDS=2 CODEC=$c KINDS=${KINDS:-1,2} KB_ARGS="--seg 59460" scripts/ab.sh >> gpurun_out/ab.txt 2>&1 || exit 1
done
for v in ${VARIANTS:-head cur}; do
  if [ "$v" = cur ]; then lib=bitar_amd/lib/libbitar_hip.so; else lib=bitar_amd/lib/variants/libbitar_hip_$v.so; fi
  BITAR_HIP_LIB=$lib timeout -k 10 300 python bench.py --only stock --steps 10 --warmup 3 --no-cpu-baseline --no-qp2 \
    > gpurun_out/bst_$v.json 2> gpurun_out/bst_$v.err || exit 1
done
