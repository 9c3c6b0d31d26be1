bash scripts/gpu_tests.sh || exit 1
for lib in bitar_amd/lib/libbitar_hip.so bitar_amd/lib/variants/libbitar_hip_d8k.so; do
  echo "== $lib"
  BITAR_HIP_LIB=$PWD/$lib BITAR_HIP_ZSTD_LANES=0 timeout -k 10 300 python scripts/kernel_bench.py --kinds 1,2 --codec zstd || exit 1
  BITAR_HIP_LIB=$PWD/$lib BITAR_HIP_INFLATE_LANES=0 timeout -k 10 300 python scripts/kernel_bench.py --kinds 1,2 --codec deflate || exit 1
done
