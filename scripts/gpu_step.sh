set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VARIANTS="cur w6 o256 w6o256" CODEC=lz4 KINDS=1,2,5,6 ROUNDS=2 bash scripts/ab.sh > gpurun_out/ab11.txt 2>&1 && grep -h "==\|kind" gpurun_out/ab11.txt | cut -c1-100
