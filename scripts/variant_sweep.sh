#!/bin/bash
# GPU-box step: kernel sweep for the default library and every built variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/variants.txt
for lib in bitar_amd/lib/libbitar_hip.so $(ls bitar_amd/lib/variants/*.so 2>/dev/null); do
  echo "== $lib" >> gpurun_out/variants.txt
  BITAR_HIP_LIB=$PWD/$lib timeout -k 10 300 python scripts/kernel_bench.py --kinds ${KINDS:-1,2,6} --codec ${CODEC:-lz4} >> gpurun_out/variants.txt 2>&1 || { echo "failed: $lib"; cat gpurun_out/variants.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/variants.txt
