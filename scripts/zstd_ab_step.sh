#!/bin/bash
# GPU-box step: Zstd GPU tests, A/B of $VARIANTS (kernel_bench, Zstd kinds 1/2/5/6), stock
# decode of each variant, and the headline stream-count sweep ($SWEEP=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_mutations.py -x -q -m gpu \
  --timeout 200 --timeout-method thread -k "zstd or Zstd" > gpurun_out/t_z.log 2>&1 || { tail -30 gpurun_out/t_z.log; exit 1; }
tail -n 1 gpurun_out/t_z.log
VARIANTS="${VARIANTS:-base cur}" ROUNDS=2 CODEC=zstd KINDS=${KINDS:-1,2,5,6} scripts/ab.sh > gpurun_out/ab.txt 2>&1 || exit 1
for v in ${VARIANTS:-base cur}; do
  if [ "$v" = cur ]; then lib=bitar_amd/lib/libbitar_hip.so; else lib=bitar_amd/lib/variants/libbitar_hip_$v.so; fi
  BITAR_HIP_LIB=$lib timeout -k 10 300 python bench.py --only stock --steps 10 --warmup 3 --no-cpu-baseline \
    > gpurun_out/bst_$v.json 2> gpurun_out/bst_$v.err || exit 1
done
if [ -n "$SWEEP" ]; then timeout -k 10 300 python scripts/stream_sweep.py > gpurun_out/ss.txt 2>&1 || exit 1; fi
