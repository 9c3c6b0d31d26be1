#!/bin/bash
# Build a tuning variant of libbitar_hip.so: scripts/build_variant.sh NAME "-DKNOB=V ..."
# -> bitar_amd/lib/variants/libbitar_hip_NAME.so (select it with BITAR_HIP_LIB=...)
set -e
cd "$(dirname "$0")/../bitar_amd"
name=$1; defs=$2
mkdir -p build_$name lib/variants
for f in runtime lz4_decompress inflate inflate_fixed compress util_kernels zstd_decompress zstd_compress zstd_lanes inflate_lanes deflate_dyn checksum lz4_chain zstd_seq; do
  extra=""
  case $f in  # (the Makefile's per-file scheduler; FLAGS_<file> below overrides)
    lz4_decompress) extra="-mllvm -amdgpu-sched-strategy=max-ilp";;
    zstd_seq) extra="-mllvm -amdgpu-sched-strategy=max-ilp -DBITAR_DEC_RING=2048";;
    zstd_lanes) extra="-mllvm -amdgpu-sched-strategy=max-memory-clause";;
    zstd_compress) extra="-DBITAR_EMIT_WAVES=8 -mllvm -amdgpu-sched-strategy=max-ilp";;
    deflate_dyn) extra="-mllvm -amdgpu-sched-strategy=max-ilp";;
    compress) extra="-mllvm -amdgpu-sched-strategy=max-ilp";;
    inflate) extra="-DBITAR_DEC_RING=2048";;
    inflate_fixed) extra="-DBITAR_DEC_RING=1024 -DBITAR_INFL_WAVES=8";;
    zstd_decompress) extra="-DBITAR_DEC_RING=2048 -DBITAR_ZSD_WAVES=3";;
  esac
  eval "extra=\${FLAGS_$f:-\$extra}"  # FLAGS_<file>="..." replaces a file's extra flags
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics $extra $defs -c csrc/$f.hip -o build_$name/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/variants/libbitar_hip_$name.so build_$name/*.o
rm -rf build_$name
echo lib/variants/libbitar_hip_$name.so
