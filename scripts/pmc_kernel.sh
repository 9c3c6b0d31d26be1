#!/bin/bash
# GPU step: one SQ PMC pass over scripts/kernel_bench.py (args passed through), per-kernel
# averages printed.  usage: bash scripts/pmc_kernel.sh TAG "COUNTERS" kernel_bench-args...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; ctrs=$2; shift 2
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc $ctrs -d gpurun_out/pmck_$tag -o pmc --output-format csv -- \
  python3 scripts/kernel_bench.py --reps 1 "$@" > gpurun_out/pmck_$tag.log 2>&1 || { tail -20 gpurun_out/pmck_$tag.log; exit 1; }
python3 - "$tag" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/pmck_{tag}/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].split("::")[-1][:40]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: "%.4g" % (sum(v) / len(v)) for c, v in d.items()})
PY
