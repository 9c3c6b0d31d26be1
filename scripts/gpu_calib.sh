#!/bin/bash
# GPU-box step: the PMC calibration passes (scripts/calib/pmc_calib.hip, built in-tree at
# scripts/calib/build/pmc_calib): one --pmc pass per counter, each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d gpurun_out/calib_$ctr -o pmc --output-format csv -- \
    scripts/calib/build/pmc_calib > gpurun_out/calib_$ctr.log 2>&1 || { echo "calib $ctr failed"; tail -20 gpurun_out/calib_$ctr.log; exit 1; }
done
find gpurun_out/calib_* -name "*.csv" | head
