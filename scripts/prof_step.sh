#!/bin/bash
# GPU step: kernel-trace stats of one command (rocprofv3), the rows matching $GREP printed.
# usage: GREP='seg_|lz4' bash scripts/prof_step.sh python scripts/kernel_bench.py --codec lz4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_step
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o run --output-format csv -- "$@" > gpurun_out/prof_step.log 2>&1 || { tail -5 gpurun_out/prof_step.log; exit 1; }
f=$(find gpurun_out/prof_step -name '*kernel_stats.csv' | head -1)
python3 - "$f" "${GREP:-.}" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Name"]):
        print(f'{float(r["AverageNs"])/1e3:10.1f} us  x{r["Calls"]:>4}  {r["Name"][:70]}')
PY
