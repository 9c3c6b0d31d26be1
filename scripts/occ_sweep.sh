#!/bin/bash
# GPU step: LZ4 kernel time at 1 GiB and 4 GiB for the shipped library and the occupancy-cap
# variants (VARS), kinds KINDS -- the 4 GiB run approximates steady-state throughput, the
# difference is the kernel's ramp / drain
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for lib in bitar_amd/lib/libbitar_hip.so ${VARS}; do
  for b in 1073741824 4294967296; do
    echo "== $lib $b"
    BITAR_HIP_LIB=$lib timeout -k 10 120 python scripts/kernel_bench.py --codec lz4 --kinds ${KINDS:-1,2} --reps 3 --bytes $b || exit 1
  done
done
