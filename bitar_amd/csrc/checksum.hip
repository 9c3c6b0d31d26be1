// checksum.hip -- per-segment CRC32 / Adler32 of uncompressed data (gfx950), one wavefront
// per segment: the rte_comp_checksum_type the reference configures into its xforms
// (src/include/config.h:169-182, src/config.cc:83-105: CRC32, ADLER32, or both with CRC32 in
// the low and Adler32 in the high 32 bits, DPDK's RTE_COMP_CHECKSUM_CRC32_ADLER32 layout).
// DPDK computes them over the uncompressed side of an op: the input of a compress, the
// output of a decompress.
//
// The segment is cut into 64 equal chunks, one per lane; each lane runs the byte loop over
// its chunk (CRC32 with a 1 KiB LDS table; Adler32 as plain and position-weighted sums), and
// the chunks are combined in GF(2) (crc(A||B) = x^(8|B|) * crc(A) + crc(B) mod P, zlib's
// crc32_combine) and modulo 65521.
#include "wave.hip.h"

namespace bitar_hip {

namespace cks {

constexpr uint32_t kPoly = 0xEDB88320u;  // reflected CRC-32 (zlib)
constexpr uint32_t kBase = 65521u;       // Adler-32 modulus

// a * b mod P in the reflected representation (zlib multmodp)
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) p ^= b;
    b = b & 1u ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}
// x^(8 n) mod P
__device__ __forceinline__ uint32_t x8nmodp(uint32_t n) {
  uint32_t p = 1u << 31;    // x^0
  uint32_t sq = 1u << 23;   // x^8
  while (n) {
    if (n & 1u) p = multmodp(sq, p);
    sq = multmodp(sq, sq);
    n >>= 1;
  }
  return p;
}

}  // namespace cks

// kind: 1 CRC32, 2 Adler32, 3 both (CRC32 | Adler32 << 32).  Segment i: lens ? lens[i] bytes
// (BITAR_HIP_SEGMENT_ERROR -> sum 0) : min(seg, n - i*seg) bytes, at data + i*seg.
__global__ __launch_bounds__(64) void checksum_kernel(uint32_t kind,
                                                      const uint8_t* __restrict__ data,
                                                      uint64_t n, uint32_t seg,
                                                      const uint32_t* __restrict__ lens,
                                                      uint32_t nseg, uint64_t* __restrict__ sums) {
  using namespace cks;
  __shared__ uint32_t table[256];
  const uint32_t i = blockIdx.x;
  if (i >= nseg) return;
  const uint32_t lane = lane_id();
  uint32_t len;
  if (lens) {
    len = lens[i];
    if (len == 0xFFFFFFFFu) {
      if (lane == 0) sums[i] = 0;
      return;
    }
    if (len > seg) len = seg;
  } else {
    const uint64_t off = (uint64_t)i * seg;
    len = (uint32_t)(n - off < seg ? n - off : seg);
  }
  const GMEM uint8_t* p = global_ptr(data + (uint64_t)i * seg);
  for (uint32_t k = lane; k < 256; k += kWave) {
    uint32_t c = k;
    for (int b = 0; b < 8; ++b) c = c & 1u ? (c >> 1) ^ kPoly : c >> 1;
    table[k] = c;
  }
  lds_order();
  // chunk of this lane: [c0, c1)
  const uint32_t chunk = (len + kWave - 1) / kWave;
  const uint32_t c0 = lane * chunk < len ? lane * chunk : len;
  const uint32_t c1 = c0 + chunk < len ? c0 + chunk : len;
  uint32_t crc = 0xFFFFFFFFu;
  uint32_t a = 0, b = 0;  // Adler sums of the chunk: plain, and weighted by (chunk end - k)
  for (uint32_t k = c0; k < c1; ++k) {
    const uint32_t x = p[k];
    crc = table[(crc ^ x) & 0xFFu] ^ (crc >> 8);
    a += x;
    b += a;
    if (((k - c0) & 255u) == 255u) {  // keep the sums far from 2^32
      a %= kBase;
      b %= kBase;
    }
  }
  crc ^= 0xFFFFFFFFu;
  a %= kBase;
  b %= kBase;
  // CRC: total = XOR over chunks of x^(8 * bytes after the chunk) * crc(chunk)
  const uint32_t after = len - c1;
  uint32_t part = c1 > c0 ? multmodp(x8nmodp(after), crc) : 0u;
  for (uint32_t d = 1; d < 64; d <<= 1) part ^= (uint32_t)__shfl_xor((int)part, (int)d, 64);
  // Adler: A = 1 + sum(bytes); B = len + sum over chunks of (b_j + a_j * bytes after it)
  uint64_t bb = ((uint64_t)b + (uint64_t)a * (after % kBase)) % kBase;
  uint64_t aa = a;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    aa += (uint64_t)__shfl_xor((long long)aa, (int)d, 64);
    bb += (uint64_t)__shfl_xor((long long)bb, (int)d, 64);
  }
  const uint32_t A = (uint32_t)((1 + aa) % kBase);
  const uint32_t B = (uint32_t)((len % kBase + bb) % kBase);
  const uint32_t adler = (B << 16) | A;
  if (lane == 0) {
    const uint64_t v = kind == 1 ? (uint64_t)part : kind == 2 ? (uint64_t)adler
                                                               : (uint64_t)part | ((uint64_t)adler << 32);
    sums[i] = v;
  }
}

}  // namespace bitar_hip
