#!/bin/bash
# GPU-box step: two SQ passes (instruction mix; issue / wait breakdown) over scripts/prof_one.py
# $ARGS, summarised per kernel (millions).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-sq3}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
k=0
for C in "$P1" "$P2"; do
  k=$((k+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/${TAG}_$k -o pmc --output-format csv -- \
    python3 scripts/prof_one.py $ARGS > gpurun_out/${TAG}_$k.log 2>&1 || { echo "pass $k failed"; tail -20 gpurun_out/${TAG}_$k.log; exit 1; }
  python3 - gpurun_out/${TAG}_$k/pmc_counter_collection.csv <<'PY'
import csv, sys
agg = {}
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "bitar_hip" not in k:
        continue
    agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in d.items()})
PY
done
