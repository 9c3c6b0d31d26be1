#!/bin/bash
# Build libbitar_hip variants that differ only in lz4_decompress.hip:
# scripts/build_lz4_variants.sh DIR  (DIR/*.hip -> bitar_amd/lib/variants/libbitar_hip_lz4_<name>.so)
set -e
cd "$(dirname "$0")/../bitar_amd"
dir=$1
mkdir -p build_lzv lib/variants
for f in runtime inflate compress util_kernels zstd_decompress zstd_compress zstd_lanes inflate_lanes deflate_dyn checksum lz4_chain zstd_seq; do
  [ -f build_lzv/$f.o ] || /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics -c csrc/$f.hip -o build_lzv/$f.o &
done
wait
for v in $dir/*.hip; do
  name=$(basename $v .hip)
  cp $v csrc/_lzv_tmp_$name.hip
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics -c csrc/_lzv_tmp_$name.hip -o build_lzv/V_$name.o
  rm csrc/_lzv_tmp_$name.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/variants/libbitar_hip_lz4_$name.so $(ls build_lzv/*.o | grep -v /V_) build_lzv/V_$name.o
  echo lib/variants/libbitar_hip_lz4_$name.so
done
rm -rf build_lzv
