#!/bin/bash
# GPU step: one rocprofv3 --pmc pass (counters in $PMC) over one command; per-kernel sums of
# each counter for the kernels matching $GREP.
# usage: PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY" GREP=seqdec bash scripts/pmc_step.sh python ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_step
timeout -s KILL 120 rocprofv3 --pmc $PMC -d gpurun_out/pmc_step -o pmc --output-format csv -- "$@" > gpurun_out/pmc_step.log 2>&1 || { tail -5 gpurun_out/pmc_step.log; exit 1; }
f=$(find gpurun_out/pmc_step -name '*counter_collection.csv' | head -1)
python3 - "$f" "${GREP:-.}" <<'PY'
import csv, re, sys, collections
tot = collections.defaultdict(float); disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Kernel_Name"]):
        k = r["Kernel_Name"][:40]
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for (k, c), v in sorted(tot.items()):
    print(f"{k:40s} {c:24s} {v / max(1, len(disp[k])):16.4g} per dispatch")
PY
