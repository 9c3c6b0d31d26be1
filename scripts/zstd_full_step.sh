mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_mutations.py tests/test_gpu_fullsize.py tests/test_gpu_job.py -x -q -m gpu --timeout 300 --timeout-method thread -k "zstd or Zstd" > gpurun_out/t_z.log 2>&1 || { tail -40 gpurun_out/t_z.log; exit 1; }
tail -n 1 gpurun_out/t_z.log
VARIANTS="head cur" scripts/zstd_ab_step.sh > /dev/null 2>&1 || { echo ab failed; exit 1; }
