set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_tests.sh > /dev/null || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
VARIANTS="head cur" CODEC=lz4 KINDS=0,1,2,5,6 ROUNDS=2 bash scripts/ab.sh > gpurun_out/ab7.txt 2>&1 || { tail gpurun_out/ab7.txt; exit 1; }
VARIANTS="head cur" CODEC=zstd KINDS=2 ROUNDS=2 bash scripts/ab.sh >> gpurun_out/ab7.txt 2>&1 || { tail gpurun_out/ab7.txt; exit 1; }
VARIANTS="head cur" CODEC=deflate KINDS=1 ROUNDS=2 bash scripts/ab.sh >> gpurun_out/ab7.txt 2>&1 || { tail gpurun_out/ab7.txt; exit 1; }
grep -h "==\|kind" gpurun_out/ab7.txt | cut -c1-110
