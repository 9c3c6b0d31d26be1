#!/bin/bash
# GPU-box step: parity tests then per-kind kernel sweeps (stop at first failure)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_tests.sh && \
timeout -k 10 300 python scripts/kernel_bench.py --kinds ${KINDS:-0,1,2,5,6} > gpurun_out/kb_lz4.txt 2>&1 && \
timeout -k 10 300 python scripts/kernel_bench.py --codec deflate --kinds ${DKINDS:-1,2} > gpurun_out/kb_dfl.txt 2>&1
rc=$?
cat gpurun_out/kb_lz4.txt gpurun_out/kb_dfl.txt 2>/dev/null
exit $rc
