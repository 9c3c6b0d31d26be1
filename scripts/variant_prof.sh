#!/bin/bash
# GPU-box step: rocprofv3 kernel stats of prof_one.py under each library in $VARIANTS
# ("cur" = the in-tree build), $CODEC / $WHICH / $KINDS; prints the per-kernel averages.
# usage: VARIANTS="cur norep" CODEC=zstd WHICH=compress KINDS="2 1" scripts/variant_prof.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/vp
for k in ${KINDS:-2}; do
  for v in ${VARIANTS:-cur}; do
    if [ "$v" = cur ]; then lib=bitar_amd/lib/libbitar_hip.so; else lib=bitar_amd/lib/variants/libbitar_hip_$v.so; fi
    d=gpurun_out/vp/${v}_k$k
    BITAR_HIP_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run -- \
      python3 scripts/prof_one.py --codec ${CODEC:-zstd} --which ${WHICH:-compress} --kind $k \
      --bytes $((1 << 30)) --reps ${REPS:-5} > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
    echo "== $v kind $k"
    python3 scripts/kstats.py $d | head -${TOP:-8}
  done
done
