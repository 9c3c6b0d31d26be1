#!/bin/bash
# GPU-box step: smoke + bench (+ optional rocprofv3 kernel-trace/stats and PMC passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo bench failed; tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o trace --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-secondary ${BENCH_ARGS} > gpurun_out/prof_${TAG}.log 2>&1 || { echo prof failed; tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${TAG}_$ctr -o pmc --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 ${BENCH_ARGS} > gpurun_out/pmc_${TAG}_$ctr.log 2>&1 || { echo pmc $ctr failed; tail -30 gpurun_out/pmc_${TAG}_$ctr.log; exit 1; }
  done
  find gpurun_out/prof_${TAG} gpurun_out/pmc_${TAG}_* -name "*.csv" | head -20
fi
