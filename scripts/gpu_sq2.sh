#!/bin/bash
# GPU-box step: SQ stall breakdown (one --pmc pass) of the kernels of $PROG (default: the Zstd
# kernel bench on kind 2): waves, VALU / SALU / LDS instructions, wave cycles split into
# issuing (ACTIVE_INST_ANY), parked on waitcnt (WAIT_ANY) and issue-stalled (WAIT_INST_ANY).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-sq2}
PROG=${PROG:-scripts/kernel_bench.py --codec zstd --kinds 2 --reps 1}
CTRS=${CTRS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY}
timeout -s KILL 300 rocprofv3 --pmc $CTRS \
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
    print(k, {c: round(sum(v) / len(v) / 1e6, 3) for c, v in d.items()})
PY
