#!/bin/bash
# GPU step: kernel trace of Zstd kind-2 decode for library variants (scripts/build_variant.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VARIANTS:-nost nw4}; do
  BITAR_HIP_LIB=bitar_amd/lib/variants/libbitar_hip_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    -d gpurun_out/hv_$v -o trace --output-format csv -- python3 scripts/kernel_bench.py --codec zstd \
    --kinds 2 --reps 1 > gpurun_out/hv_$v.log 2>&1 || { tail gpurun_out/hv_$v.log; exit 1; }
  echo "== $v"
  python3 - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f'gpurun_out/hv_{sys.argv[1]}/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'zstd' in r['Name']:
        print(r['Name'][:45], round(float(r['AverageNs']) / 1e6, 3))
PY
done
