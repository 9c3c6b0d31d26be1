// pmc_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the
// access patterns of this engine's kernels (MI355X_MICROARCH.md "HBM": only 16-B-per-lane
// streaming reads / writes are calibrated there).  Each kernel moves a KNOWN byte count
// (1 GiB, far past the 256 MiB Infinity Cache) in one pattern:
//   read16      16 B per lane, each wave instruction 1 KiB contiguous (window / ring refills)
//   write16     16 B per lane, 1 KiB contiguous per wave instruction (ring flushes)
//   read8_lane  lane-owned streams, 8 B per lane per load, sequential within a lane
//               (inflate_lanes_kernel / zstd_hlit_kernel bit readers), at 2 M / 128 K / 16 K
//               concurrent streams (grid sizes 2097152 / 131072 / 16384 threads)
//   write8_lane lane-owned streams, 8 B per lane per store (zstd_hlit_kernel, inflate_lanes)
//   write1      1 B per lane, 64 B contiguous per wave instruction (flush heads / tails)
//   read1       1 B per lane, 64 B contiguous per wave instruction (byte gathers)
// usage: pmc_calib [bytes]   (prints the kernels' byte counts; run it under
//        rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>


__global__ __launch_bounds__(256) void read16(const uint4* __restrict__ in, uint64_t n16,
                                              uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) {
    const uint4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;  // (never: keeps the loads)
}

__global__ __launch_bounds__(256) void write16(uint4* __restrict__ out, uint64_t n16) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull)
    out[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

// lane-owned streams: thread t owns bytes [t * per, (t + 1) * per)
__global__ __launch_bounds__(256) void read8_lane(const uint64_t* __restrict__ in, uint64_t per8,
                                                  uint32_t* __restrict__ sink) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t* p = in + t * per8;
  uint64_t acc = 0;
  for (uint64_t k = 0; k < per8; ++k) acc ^= p[k];
  if (acc == 0x9E3779B97F4A7C15ull) sink[0] = (uint32_t)acc;
}

__global__ __launch_bounds__(256) void write8_lane(uint64_t* __restrict__ out, uint64_t per8) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  uint64_t* p = out + t * per8;
  for (uint64_t k = 0; k < per8; ++k) p[k] = t ^ k;
}

__global__ __launch_bounds__(256) void write1(uint8_t* __restrict__ out, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    out[i] = (uint8_t)i;
}

__global__ __launch_bounds__(256) void read1(const uint8_t* __restrict__ in, uint64_t n,
                                             uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    acc += in[i];
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1ull << 30);
  uint8_t* a = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&a, n));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 1, n));
  CK(hipDeviceSynchronize());
  const uint32_t grid = 8192;  // 2 M threads
  const uint64_t threads = grid * 256ull;
  const uint64_t per8 = n / 8 / threads;  // 8-B words per lane-owned stream (2 M streams)
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read16, dim3(grid), dim3(256), 0, 0, (const uint4*)a, n / 16, sink);
    hipLaunchKernelGGL(write16, dim3(grid), dim3(256), 0, 0, (uint4*)a, n / 16);
    // lane-owned streams at three concurrencies: 2 M streams of 512 B, 128 K of 8 KiB, 16 K
    // of 64 KiB (the decoders run ~16 K-64 K lane streams per GiB)
    for (uint32_t g : {grid, grid / 16, grid / 128}) {
      const uint64_t p8 = n / 8 / (g * 256ull);
      hipLaunchKernelGGL(read8_lane, dim3(g), dim3(256), 0, 0, (const uint64_t*)a, p8, sink);
      hipLaunchKernelGGL(write8_lane, dim3(g), dim3(256), 0, 0, (uint64_t*)a, p8);
    }
    hipLaunchKernelGGL(write1, dim3(grid), dim3(256), 0, 0, a, n);
    hipLaunchKernelGGL(read1, dim3(grid), dim3(256), 0, 0, (const uint8_t*)a, n, sink);
  }
  CK(hipDeviceSynchronize());
  std::printf("{\"bytes\": %llu, \"lane_stream_bytes\": %llu}\n", (unsigned long long)n,
              (unsigned long long)(per8 * 8 * threads));
  CK(hipFree(a));
  CK(hipFree(sink));
  return 0;
}
