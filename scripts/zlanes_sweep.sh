#!/bin/bash
# GPU-box step: zstd kernel sweep over zstd_lanes_kernel widths (BITAR_HIP_ZSTD_LANES)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LANES:-16 32 64 0}; do
  echo "== lanes $L"
  BITAR_HIP_ZSTD_LANES=$L timeout -k 10 300 python scripts/kernel_bench.py --codec zstd --kinds ${KINDS:-1,2,6,0} --reps 2 2>&1 | grep -v amdgpu.ids || exit 1
done
