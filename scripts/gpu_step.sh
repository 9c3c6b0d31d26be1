#!/bin/bash
# GPU step for iterations: optional parity tests (PYTEST_K / FILES, optional BITAR_HIP_LIB), then
# the given commands, each under its own time limit; stop at the first failure.
# usage: bash scripts/gpu_step.sh "cmd1" "cmd2" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$PYTEST_K$FILES" ]; then
  timeout -k 10 600 python -u -m pytest ${FILES:-tests} -x -q -m gpu --timeout 300 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/step_pytest.log 2>&1
  rc=$?
  tail -3 gpurun_out/step_pytest.log
  [ $rc = 0 ] || exit $rc
fi
for c in "$@"; do
  echo "== $c"
  timeout -k 10 300 bash -c "$c" || { echo "step failed: $c"; exit 1; }
done
