set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_collisions.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fuzz.log 2>&1 && echo "fuzz ok" && grep -E "passed|failed" gpurun_out/fuzz.log | tail -2 && bash scripts/gpu_tests.sh > /dev/null && tail -2 gpurun_out/pytest_gpu.log
