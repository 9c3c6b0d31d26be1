set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do for v in far4k far8k cur far32k; do
  if [ $v = cur ]; then lib=bitar_amd/lib/libbitar_hip.so; else lib=bitar_amd/lib/variants/libbitar_hip_$v.so; fi
  echo -n "$v "; BITAR_HIP_LIB=$lib timeout -k 10 200 python scripts/stock_bench.py --codec lz4 --kind 1 2>/dev/null | grep codec || exit 1
done; done
