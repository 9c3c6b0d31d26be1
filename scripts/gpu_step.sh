set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_tests.sh > /dev/null || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
VARIANTS="head cur" CODEC=zstd KINDS=1,2,5,6 ROUNDS=2 bash scripts/ab.sh > gpurun_out/ab6.txt 2>&1 || { tail gpurun_out/ab6.txt; exit 1; }
grep -h "==\|kind" gpurun_out/ab6.txt | cut -c1-110
BITAR_HIP_LIB=bitar_amd/lib/variants/libbitar_hip_noredo.so timeout -k 10 600 python -m pytest tests/test_gpu_fullsize.py tests/test_gpu_lz4.py -x -q -m gpu > gpurun_out/noredo_tests.log 2>&1; echo "noredo tests rc=$?"; tail -3 gpurun_out/noredo_tests.log
VARIANTS="head noredo" CODEC=lz4 KINDS=1,2,5,6 ROUNDS=2 bash scripts/ab.sh > gpurun_out/ab5.txt 2>&1 || { tail gpurun_out/ab5.txt; exit 1; }
grep -h "==\|kind" gpurun_out/ab5.txt | cut -c1-110
