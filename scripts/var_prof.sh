#!/bin/bash
# GPU step: per-kernel average durations (rocprofv3 --kernel-trace --stats) of every variant
# library under scripts/kernel_bench.py; KFILTER selects the kernels printed
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for lib in bitar_amd/lib/variants/libbitar_hip_*.so; do
  v=$(basename $lib .so)
  BITAR_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/vp_$v -o t --output-format csv -- \
    python3 scripts/kernel_bench.py --codec ${CODEC:-zstd} --kinds ${KINDS:-2} --reps 2 > gpurun_out/vp_$v.log 2>&1 || { tail -5 gpurun_out/vp_$v.log; exit 1; }
  echo "== $v $(grep -h '"kind"' gpurun_out/vp_$v.log | tr '\n' ' ')"
  python3 - "$v" "${KFILTER:-hlit}" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/vp_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in sys.argv[2].split(",")):
        print("  ", r["Name"].split("(")[0][-40:], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
done
