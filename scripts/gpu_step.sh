set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python scripts/coll_debug.py ZSTD > gpurun_out/coll_cur.txt 2>&1; echo "rc=$?"
grep -v "same_as_oracle True first_diff -1 oracle_decodes_gpu_frame True" gpurun_out/coll_cur.txt | head -8
timeout -k 10 600 python -m pytest tests/test_gpu_collisions.py -x -q -m gpu > gpurun_out/coll.log 2>&1; echo "collision tests rc=$?"; tail -2 gpurun_out/coll.log
BITAR_HIP_LIB=bitar_amd/lib/variants/libbitar_hip_redo.so timeout -k 10 600 python -m pytest tests/test_gpu_collisions.py -x -q -m gpu > gpurun_out/coll_redo.log 2>&1; echo "redo collision tests rc=$?"; tail -2 gpurun_out/coll_redo.log
bash scripts/gpu_tests.sh > /dev/null || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
