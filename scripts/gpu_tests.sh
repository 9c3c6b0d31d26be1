#!/bin/bash
# GPU-box step: parity tests (each GPU step under its own time limit; stop at first failure)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -x -q -m gpu ${PYTEST_K:+-k "$PYTEST_K"} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -40 gpurun_out/pytest_gpu.log
exit $rc
