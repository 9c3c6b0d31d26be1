set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_collisions.py tests/test_gpu_fullsize.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/la.log 2>&1 && echo "tests ok" && grep -E "passed|failed" gpurun_out/la.log | tail -1 && VARIANTS="nola cur" CODEC=lz4 KINDS=0,1,2,5,6 ROUNDS=2 bash scripts/ab.sh > gpurun_out/ab10.txt 2>&1 && VARIANTS="nola cur" CODEC=deflate KINDS=1 ROUNDS=2 bash scripts/ab.sh >> gpurun_out/ab10.txt 2>&1 && grep -h "==\|kind" gpurun_out/ab10.txt | cut -c1-110
