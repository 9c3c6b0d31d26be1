#!/bin/bash
# GPU step: Zstd decode timing over the hlit / handoff segments per wave ("HLIT:HANDOFF" pairs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for p in ${PAIRS:-16:16 4:16 8:16 16:4 16:8 4:4}; do
  echo "== $p"
  BITAR_HIP_HLIT_SEGS=${p%:*} BITAR_HIP_HANDOFF_LANES=${p#*:} timeout -k 10 120 \
    python scripts/kernel_bench.py --codec zstd --kinds ${KINDS:-2,1} --reps 3 || exit 1
done
