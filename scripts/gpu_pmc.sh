#!/bin/bash
# GPU-box step: PMC counter passes (one rocprofv3 --pmc run per counter group) over one kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-pmc}
ARGS=${ARGS:-"--kind 5 --codec lz4 --which decompress"}
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/${TAG}_$i -o pmc --output-format csv -- python3 scripts/prof_one.py $ARGS > gpurun_out/${TAG}_$i.log 2>&1 || { echo "pmc group $i failed"; tail -20 gpurun_out/${TAG}_$i.log; exit 1; }
done
python3 - "$TAG" "$i" <<'PY'
import csv, glob, sys
tag, n = sys.argv[1], int(sys.argv[2])
for k in range(1, n + 1):
    for f in glob.glob(f"gpurun_out/{tag}_{k}/**/*counter_collection.csv", recursive=True):
        agg = {}
        for r in csv.DictReader(open(f)):
            if "bitar_hip" not in r["Kernel_Name"]:
                continue
            key = (r["Kernel_Name"].split("(")[0], r["Counter_Name"])
            agg.setdefault(key, []).append(float(r["Counter_Value"]))
        for (kn, c), v in sorted(agg.items()):
            print(f"{kn:40s} {c:28s} {sum(v)/len(v):16.1f}")
PY
