#!/bin/bash
# GPU step: kernel trace of the stock-stream decode leg (bench.py --only stock)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/stockprof -o trace --output-format csv -- \
  python3 bench.py --only stock --steps 3 --warmup 1 > gpurun_out/stockprof.log 2>&1 || { tail -20 gpurun_out/stockprof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/stockprof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'bitar' in r['Name']:
        print(r['Name'].split('(')[0][-45:], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
