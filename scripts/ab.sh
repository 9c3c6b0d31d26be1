#!/bin/bash
# A/B on one box: kernel_bench.py over the variants named in $VARIANTS ("old" = bitar_amd/lib/
# variants/libbitar_hip_old.so, "cur" = the in-tree build), interleaved $ROUNDS times.
# usage: VARIANTS="old cur" CODEC=lz4 KINDS=1,2 scripts/ab.sh > gpurun_out/ab.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS:-old cur}; do
    if [ "$v" = cur ]; then lib=bitar_amd/lib/libbitar_hip.so; else lib=bitar_amd/lib/variants/libbitar_hip_$v.so; fi
    echo "== $v"
    BITAR_HIP_LIB=$lib timeout -k 10 120 python scripts/kernel_bench.py --codec ${CODEC:-lz4} --kinds ${KINDS:-1,2} --reps ${REPS:-5} ${KB_ARGS} || exit 1
  done
done
