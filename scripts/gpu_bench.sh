#!/bin/bash
# GPU-box step: smoke + bench (+ optional rocprofv3 kernel-trace/stats and PMC passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
if [ -z "$NO_BENCH" ]; then  # (NO_BENCH=1: profile passes only, e.g. a second call)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo bench failed; tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
fi
if [ -n "$PROFILE" ]; then
  # one kernel-trace pass and one pass per PMC counter for each leg on its own (--only), so a
  # kernel's averages never mix launches of different legs (the record-batch leg also runs
  # lz4_compress_kernel, the stock-decode leg lz4_decompress_kernel, ...)
  for leg in ${PROF_LEGS:-headline zstd deflate deflate_dyn recordbatch lz4_arrow}; do
    # lz4_arrow: the headline job itself on the kind-2 input (the same grid as the headline,
    # so it gets a run of its own in which it IS the headline)
    if [ "$leg" = lz4_arrow ]; then LEGARGS="--kind 2 --only none"; else LEGARGS="--only $leg"; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$leg -o trace --output-format csv -- \
      python3 bench.py $LEGARGS ${BENCH_ARGS} > gpurun_out/prof_${TAG}_$leg.log 2>&1 || { echo prof $leg failed; tail -30 gpurun_out/prof_${TAG}_$leg.log; exit 1; }
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/pmc_${TAG}_${leg}_$ctr -o pmc --output-format csv -- \
        python3 bench.py $LEGARGS --steps 2 --warmup 1 ${BENCH_ARGS} > gpurun_out/pmc_${TAG}_${leg}_$ctr.log 2>&1 || { echo pmc $leg $ctr failed; tail -30 gpurun_out/pmc_${TAG}_${leg}_$ctr.log; exit 1; }
    done
  done
  find gpurun_out/prof_${TAG}_* gpurun_out/pmc_${TAG}_* -name "*stats.csv" | head -20
fi
