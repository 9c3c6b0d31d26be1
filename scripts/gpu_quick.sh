#!/bin/bash
# GPU step: selected parity tests (PYTEST_K / FILES), then kernel timing of the shipped library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-400} python -u -m pytest ${FILES:-tests} -x -q -m gpu ${PYTEST_K:+-k "$PYTEST_K"} \
  --timeout 300 --timeout-method thread > gpurun_out/quick.log 2>&1
rc=$?
tail -5 gpurun_out/quick.log
[ $rc = 0 ] || exit $rc
for c in ${CODECS:-lz4}; do
  timeout -k 10 200 python scripts/kernel_bench.py --codec $c --kinds ${KINDS:-1,2} || exit 1
done
