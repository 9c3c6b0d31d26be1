#!/bin/bash
# GPU step: Zstd decode timing over the two-phase path's knobs, then one kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for sd in ${SDS:-16 8 4}; do
  echo "BITAR_HIP_SEQDEC_SEGS=$sd"
  BITAR_HIP_SEQDEC_SEGS=$sd timeout -k 10 200 python -u scripts/kernel_bench.py --codec zstd --kinds ${KINDS:-2} --reps 2 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/zseq_prof -o trace --output-format csv -- \
  python3 scripts/kernel_bench.py --codec zstd --kinds 2 --reps 2 > gpurun_out/zseq_prof.log 2>&1 || { echo prof failed; tail gpurun_out/zseq_prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/zseq_prof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
