#!/bin/bash
# GPU step: dynamic-DEFLATE compress timing of the shipped library and the no-emission variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in "" skipwin; do
  lib=bitar_amd/lib/libbitar_hip.so; [ -n "$v" ] && lib=bitar_amd/lib/variants/libbitar_hip_$v.so
  echo "== ${v:-shipped}"
  BITAR_HIP_LIB=$lib timeout -k 10 120 python scripts/kernel_bench.py --codec deflate_dyn --kinds ${KINDS:-1,2} || exit 1
done
