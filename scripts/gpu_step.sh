set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_tests.sh > /dev/null || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
VARIANTS="old cur" CODEC=lz4 KINDS=0,1,2,5,6 ROUNDS=2 bash scripts/ab.sh > gpurun_out/ab1.txt 2>&1 || { tail gpurun_out/ab1.txt; exit 1; }
cat gpurun_out/ab1.txt
