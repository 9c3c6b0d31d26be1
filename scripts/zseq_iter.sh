#!/bin/bash
# GPU iteration step for the two-phase Zstd sequence path: zstd parity tests, then decode
# timing with the record path on and off, then a kernel trace of the record path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_zstd.py -x -q -m gpu ${PYTEST_K:+-k "$PYTEST_K"} --timeout 200 \
  --timeout-method thread > gpurun_out/zseq_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/zseq_tests.log; exit 1; }
tail -3 gpurun_out/zseq_tests.log
fi
for sq in 1 0; do
  echo "BITAR_HIP_ZSTD_SEQ=$sq"
  BITAR_HIP_ZSTD_SEQ=$sq timeout -k 10 200 python -u scripts/kernel_bench.py --codec zstd --kinds ${KINDS:-1,2,5,6} || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/zseq_prof -o trace --output-format csv -- \
  python3 scripts/kernel_bench.py --codec zstd --kinds 2 > gpurun_out/zseq_prof.log 2>&1 || { echo prof failed; tail gpurun_out/zseq_prof.log; exit 1; }
f=$(find gpurun_out/zseq_prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -12
