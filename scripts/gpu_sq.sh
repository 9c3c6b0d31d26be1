#!/bin/bash
# GPU-box step: SQ instruction-mix counters of the headline kernels (one --pmc pass), or of
# ARGS for scripts/prof_one.py (e.g. ARGS="--kind 5 --codec lz4 --which compress").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-sq}
if [ -n "$ARGS" ]; then PROG="scripts/prof_one.py $ARGS"; else PROG="bench.py --only headline --steps 2 --warmup 1 ${BENCH_ARGS}"; fi
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH \
  -d gpurun_out/$TAG -o pmc --output-format csv -- python3 $PROG \
  > gpurun_out/$TAG.log 2>&1 || { echo "sq pass failed"; tail -20 gpurun_out/$TAG.log; exit 1; }
python3 - gpurun_out/$TAG/pmc_counter_collection.csv <<'PY'
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
