: > gpurun_out/ab.txt
for r in 1 2; do for v in f512 cur; do
  if [ $v = cur ]; then lib=bitar_amd/lib/libbitar_hip.so; else lib=bitar_amd/lib/variants/libbitar_hip_$v.so; fi
  echo "== $v" >> gpurun_out/ab.txt
  BITAR_HIP_LIB=$lib timeout -k 10 120 python scripts/kernel_bench.py --codec deflate --kinds 1,2,5,6 --seg 59460 --reps 3 >> gpurun_out/ab.txt 2>&1 || exit 1
done; done
timeout -k 10 500 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_mutations.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_d.log 2>&1; rc=$?; tail -n 1 gpurun_out/t_d.log; exit $rc
