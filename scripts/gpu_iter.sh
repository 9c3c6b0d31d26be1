#!/bin/bash
# GPU-box iteration step: optional focused tests, then a per-kernel sweep.
#   PYTEST_K  pytest -k filter for the gpu tests (skip tests if empty)
#   KB_ARGS   arguments to scripts/kernel_bench.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "$PYTEST_K" --timeout 300 \
    --timeout-method thread > gpurun_out/iter_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/iter_tests.log; exit 1; }
  tail -3 gpurun_out/iter_tests.log
fi
timeout -k 10 600 python -u scripts/kernel_bench.py ${KB_ARGS} 2>&1 | tee gpurun_out/iter_kb.log
