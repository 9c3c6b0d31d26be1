// arrow_codec.cc -- arrow::util::Codec adapters (ZSTD, LZ4_FRAME) over the C ABI.
// See include/bitar/arrow_codec.h for the stream layouts.  Every payload byte is compressed
// and decompressed on the device; the host only walks frame / block headers (sizes) and
// writes the 7-byte LZ4 frame header and EndMark.
#include "bitar/arrow_codec.h"

#include <arrow/status.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "bitar_hip.h"
#include "hip_ctx.h"

namespace bitar {

namespace {

constexpr uint32_t kSeg = 65536;  // segment = Zstd frame content = LZ4 frame block
constexpr uint32_t kZstdMagic = 0xFD2FB528u, kLz4fMagic = 0x184D2204u;

uint32_t Rd32(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

// XXH32 (the LZ4 frame descriptor's header checksum is its second byte; header bytes only)
uint32_t Xxh32(const uint8_t* p, size_t n, uint32_t seed) {
  constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                     P5 = 374761393u;
  auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
  size_t i = 0;
  uint32_t h;
  if (n >= 16) {
    uint32_t v[4] = {seed + P1 + P2, seed + P2, seed, seed - P1};
    for (; i + 16 <= n; i += 16)
      for (int k = 0; k < 4; ++k) v[k] = rotl(v[k] + Rd32(p + i + 4 * k) * P2, 13) * P1;
    h = rotl(v[0], 1) + rotl(v[1], 7) + rotl(v[2], 12) + rotl(v[3], 18);
  } else {
    h = seed + P5;
  }
  h += static_cast<uint32_t>(n);
  for (; i + 4 <= n; i += 4) h = rotl(h + Rd32(p + i) * P3, 17) * P4;
  for (; i < n; ++i) h = rotl(h + p[i] * P5, 11) * P1;
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

// one segment of a compressed stream: csize bytes at offset; raw = stored (LZ4 frame);
// content = its decompressed size when the header states it (Zstd), else 0
struct Piece {
  uint64_t offset;
  uint32_t csize;
  uint32_t content;
  bool raw;
};

// one frame of a stock stream (the unit the stock writers emit per buffer)
struct Frame {
  uint64_t offset = 0, csize = 0;  // the whole frame
  uint64_t content = 0;            // declared content size (has_content)
  bool has_content = false;
  bool linked = false;             // LZ4: blocks depend on the previous ones
  bool content_checksum = false;   // LZ4: XXH32 of the content follows the EndMark
  uint32_t checksum = 0;
  std::vector<Piece> blocks;       // LZ4 data blocks
};

class HipCodec : public arrow::util::Codec {
 public:
  HipCodec(arrow::Compression::type type, int device, bitar_hip_ctx* ctx)
      : type_(type), device_(device), ctx_(ctx) {}
  ~HipCodec() override {
    for (void* p : {d_in_, d_slab_, d_sizes_, d_off_, d_frame_, d_out_, d_srcs_, d_aux_})
      if (p) bitar_hip_free(ctx_, p);
    bitar_hip_close(ctx_);
  }

  int minimum_compression_level() const override { return 1; }
  int maximum_compression_level() const override { return 1; }
  int default_compression_level() const override { return 1; }
  int compression_level() const override { return 1; }
  arrow::Compression::type compression_type() const override { return type_; }

  int64_t MaxCompressedLen(int64_t input_len, const uint8_t*) override {
    const uint64_t nseg = (static_cast<uint64_t>(input_len) + kSeg - 1) / kSeg;
    if (type_ == arrow::Compression::ZSTD)
      return static_cast<int64_t>(9 + nseg * bitar_hip_slot_size(BITAR_HIP_CODEC_ZSTD, kSeg));
    return static_cast<int64_t>(7 + nseg * (4 + kSeg) + 4);
  }

  arrow::Result<std::shared_ptr<arrow::util::Compressor>> MakeCompressor() override {
    return arrow::Status::NotImplemented("streaming compression on the HIP codec");
  }
  arrow::Result<std::shared_ptr<arrow::util::Decompressor>> MakeDecompressor() override {
    return arrow::Status::NotImplemented("streaming decompression on the HIP codec");
  }

  arrow::Result<int64_t> Compress(int64_t input_len, const uint8_t* input,
                                  int64_t output_buffer_len, uint8_t* output) override;
  arrow::Result<int64_t> Decompress(int64_t input_len, const uint8_t* input,
                                    int64_t output_buffer_len, uint8_t* output) override;

 private:
  // grow-only HBM scratch
  arrow::Status Reserve(void*& p, uint64_t& cap, uint64_t bytes) {
    if (bytes <= cap) return arrow::Status::OK();
    if (p) bitar_hip_free(ctx_, p);
    p = nullptr;
    cap = 0;
    BITAR_ABI(bitar_hip_alloc(ctx_, bytes, &p), "bitar_hip_alloc");
    cap = bytes;
    return arrow::Status::OK();
  }
  bool OnDevice(const void* p) const {
    int kind = 0, dev = -1;
    return bitar_hip_pointer_info(p, &kind, &dev) == 0 && kind == 2 && dev == device_;
  }
  arrow::Status Copy(void* dst, const void* src, uint64_t n) {
    if (n) BITAR_ABI(bitar_hip_memcpy(ctx_, dst, src, n, nullptr), "bitar_hip_memcpy");
    return arrow::Status::OK();
  }
  arrow::Status Sync() {
    BITAR_ABI(bitar_hip_sync(ctx_, nullptr), "segment codec");
    return arrow::Status::OK();
  }
  arrow::Result<std::vector<Frame>> WalkZstd(const uint8_t* p, uint64_t n) const;
  arrow::Result<std::vector<Frame>> WalkLz4f(const uint8_t* p, uint64_t n) const;
  arrow::Result<int64_t> DecompressZstd(const std::vector<Frame>& frames, const uint8_t* d_in,
                                        int64_t output_buffer_len, uint8_t* output);
  arrow::Result<int64_t> DecompressLz4f(const std::vector<Frame>& frames, const uint8_t* d_in,
                                        uint64_t n, int64_t output_buffer_len, uint8_t* output);
  // the frame's independent 64 KiB blocks, in parallel, to dout; returns the content size
  arrow::Result<uint64_t> Lz4Independent(const Frame& f, const uint8_t* d_in, uint8_t* dout);

  arrow::Compression::type type_;
  int device_;
  bitar_hip_ctx* ctx_;
  std::mutex mu_;  // one stream per codec; Arrow may share a codec between threads
  void *d_in_ = nullptr, *d_slab_ = nullptr, *d_sizes_ = nullptr, *d_off_ = nullptr,
       *d_frame_ = nullptr, *d_out_ = nullptr, *d_srcs_ = nullptr, *d_aux_ = nullptr;
  uint64_t c_in_ = 0, c_slab_ = 0, c_sizes_ = 0, c_off_ = 0, c_frame_ = 0, c_out_ = 0,
           c_srcs_ = 0, c_aux_ = 0;
};

arrow::Result<int64_t> HipCodec::Compress(int64_t input_len, const uint8_t* input,
                                          int64_t output_buffer_len, uint8_t* output) {
  const std::lock_guard<std::mutex> lock(mu_);
  if (input_len < 0) return arrow::Status::Invalid("negative input length");
  if (output_buffer_len < MaxCompressedLen(input_len, input))
    return arrow::Status::Invalid("output buffer smaller than MaxCompressedLen");
  const uint64_t n = static_cast<uint64_t>(input_len);
  const uint64_t nseg = (n + kSeg - 1) / kSeg;
  const bool zstd = type_ == arrow::Compression::ZSTD;
  const bool out_dev = OnDevice(output);
  // LZ4 frame header: magic, FLG (version 01, independent blocks), BD (64 KiB blocks), HC
  uint8_t hdr[7] = {0x04, 0x22, 0x4D, 0x18, 0x60, 0x40, 0};
  hdr[6] = static_cast<uint8_t>((Xxh32(hdr + 4, 2, 0) >> 8) & 0xFF);
  const uint64_t head = zstd ? 0 : sizeof hdr;
  if (n == 0) {
    // an empty stream: one empty frame (Zstd: single segment, content size 0, one empty
    // last raw block), or the LZ4 frame header + EndMark
    static const uint8_t kEmptyZstd[9] = {0x28, 0xB5, 0x2F, 0xFD, 0x20, 0x00, 0x01, 0x00, 0x00};
    uint8_t lz4[11];
    std::memcpy(lz4, hdr, 7);
    std::memset(lz4 + 7, 0, 4);
    const uint8_t* src = zstd ? kEmptyZstd : lz4;
    const uint64_t len = zstd ? sizeof kEmptyZstd : sizeof lz4;
    if (out_dev) ARROW_RETURN_NOT_OK(Copy(output, src, len));
    else std::memcpy(output, src, len);
    return static_cast<int64_t>(len);
  }
  const uint32_t codec = zstd ? BITAR_HIP_CODEC_ZSTD : BITAR_HIP_CODEC_LZ4;
  const uint64_t stride = bitar_hip_slot_size(codec, kSeg);
  const void* d_in = input;
  if (!OnDevice(input)) {
    ARROW_RETURN_NOT_OK(Reserve(d_in_, c_in_, n));
    ARROW_RETURN_NOT_OK(Copy(d_in_, input, n));
    d_in = d_in_;
  }
  ARROW_RETURN_NOT_OK(Reserve(d_slab_, c_slab_, nseg * stride));
  ARROW_RETURN_NOT_OK(Reserve(d_sizes_, c_sizes_, nseg * 4));
  ARROW_RETURN_NOT_OK(Reserve(d_aux_, c_aux_, nseg * 4));
  ARROW_RETURN_NOT_OK(Reserve(d_off_, c_off_, (nseg + 1) * 8));
  ARROW_RETURN_NOT_OK(Reserve(d_frame_, c_frame_, head + nseg * (stride > kSeg + 4 ? stride : kSeg + 4) + 4));
  auto* sizes = static_cast<uint32_t*>(d_sizes_);
  auto* offs = static_cast<uint64_t*>(d_off_);
  auto* frame = static_cast<uint8_t*>(d_frame_);
  BITAR_ABI(bitar_hip_compress(ctx_, nullptr, codec, d_in, n, kSeg, d_slab_, stride, sizes),
            "bitar_hip_compress");
  if (zstd) {
    BITAR_ABI(bitar_hip_pack(ctx_, nullptr, d_slab_, stride, sizes, static_cast<uint32_t>(nseg),
                             offs, frame),
              "bitar_hip_pack");
  } else {
    BITAR_ABI(bitar_hip_pack_lz4f(ctx_, nullptr, d_in, n, kSeg, d_slab_, stride, sizes,
                                  static_cast<uint32_t*>(d_aux_), offs, frame + head),
              "bitar_hip_pack_lz4f");
  }
  ARROW_RETURN_NOT_OK(Sync());
  uint64_t body = 0;
  ARROW_RETURN_NOT_OK(Copy(&body, offs + nseg, sizeof body));
  ARROW_RETURN_NOT_OK(Sync());
  const uint64_t total = head + body + (zstd ? 0 : 4);
  if (total > static_cast<uint64_t>(output_buffer_len))
    return arrow::Status::CapacityError("compressed stream exceeds the output buffer");
  if (out_dev) {
    if (!zstd) ARROW_RETURN_NOT_OK(Copy(output, hdr, head));
    ARROW_RETURN_NOT_OK(Copy(output + head, frame + head, body));
    if (!zstd) {
      static const uint8_t kEnd[4] = {0, 0, 0, 0};
      ARROW_RETURN_NOT_OK(Copy(output + head + body, kEnd, 4));
    }
  } else {
    if (!zstd) std::memcpy(output, hdr, head);
    ARROW_RETURN_NOT_OK(Copy(output + head, frame + head, body));
    if (!zstd) std::memset(output + head + body, 0, 4);
  }
  ARROW_RETURN_NOT_OK(Sync());
  return static_cast<int64_t>(total);
}

// Zstandard frames (any content size; a frame without one only as the stream's single
// frame, sized by the caller's output buffer)
arrow::Result<std::vector<Frame>> HipCodec::WalkZstd(const uint8_t* p, uint64_t n) const {
  std::vector<Frame> v;
  uint64_t pos = 0;
  while (pos < n) {
    Frame f;
    f.offset = pos;
    if (n - pos < 6 || Rd32(p + pos) != kZstdMagic)
      return arrow::Status::NotImplemented("not a Zstandard frame at offset ", pos);
    pos += 4;
    const uint32_t fhd = p[pos++];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1u, did_flag = fhd & 3u;
    if (fhd & 8u) return arrow::Status::Invalid("Zstandard frame with reserved bit set");
    if (did_flag) return arrow::Status::NotImplemented("Zstandard dictionaries");
    if (!single) pos += 1;
    const uint32_t fsz = fcs_flag == 0 ? (single ? 1u : 0u) : fcs_flag == 1 ? 2u
                         : fcs_flag == 2 ? 4u : 8u;
    if (pos + fsz > n) return arrow::Status::Invalid("truncated Zstandard frame header");
    for (uint32_t k = 0; k < fsz; ++k) f.content |= uint64_t(p[pos + k]) << (8 * k);
    if (fsz == 2) f.content += 256;
    f.has_content = fsz != 0;
    pos += fsz;
    for (bool last = false; !last;) {
      if (pos + 3 > n) return arrow::Status::Invalid("truncated Zstandard block header");
      const uint32_t bh = uint32_t(p[pos]) | uint32_t(p[pos + 1]) << 8 | uint32_t(p[pos + 2]) << 16;
      last = bh & 1u;
      const uint32_t type = (bh >> 1) & 3u, bsz = bh >> 3;
      if (type == 3) return arrow::Status::Invalid("reserved Zstandard block type");
      pos += 3 + (type == 1 ? 1u : bsz);
    }
    if ((fhd >> 2) & 1u) pos += 4;  // content checksum (verified on the device)
    if (pos > n) return arrow::Status::Invalid("truncated Zstandard frame");
    f.csize = pos - f.offset;
    v.push_back(f);
  }
  return v;
}

// LZ4 frames: version 01, blocks of <= 64 KiB (independent or linked), optional block
// checksums, content size and content checksum (both checksums verified here: XXH32)
arrow::Result<std::vector<Frame>> HipCodec::WalkLz4f(const uint8_t* p, uint64_t n) const {
  std::vector<Frame> v;
  uint64_t pos = 0;
  while (pos < n) {
    Frame f;
    f.offset = pos;
    if (n - pos < 7 || Rd32(p + pos) != kLz4fMagic)
      return arrow::Status::NotImplemented("not an LZ4 frame at offset ", pos);
    const uint32_t flg = p[pos + 4], bd = p[pos + 5];
    if ((flg >> 6) != 1) return arrow::Status::Invalid("LZ4 frame version");
    f.linked = !((flg >> 5) & 1);
    const bool block_cks = (flg >> 4) & 1;
    f.content_checksum = (flg >> 2) & 1;
    if (flg & 1) return arrow::Status::NotImplemented("LZ4 dictionary id");
    if (((bd >> 4) & 7) != 4) return arrow::Status::NotImplemented("LZ4 blocks larger than 64 KiB");
    const bool has_size = (flg >> 3) & 1;
    const uint64_t dlen = 2 + (has_size ? 8 : 0);
    if (pos + 4 + dlen + 1 > n) return arrow::Status::Invalid("truncated LZ4 frame header");
    if (((Xxh32(p + pos + 4, dlen, 0) >> 8) & 0xFF) != p[pos + 4 + dlen])
      return arrow::Status::Invalid("LZ4 frame header checksum");
    if (has_size) {
      f.has_content = true;
      for (int k = 0; k < 8; ++k) f.content |= uint64_t(p[pos + 6 + k]) << (8 * k);
    }
    pos += 4 + dlen + 1;
    for (;;) {
      if (pos + 4 > n) return arrow::Status::Invalid("truncated LZ4 frame");
      const uint32_t bs = Rd32(p + pos);
      pos += 4;
      if (bs == 0) break;  // EndMark
      const uint32_t len = bs & 0x7FFFFFFFu;
      if (len > kSeg || pos + len > n) return arrow::Status::Invalid("bad LZ4 block size");
      if (block_cks) {
        if (pos + len + 4 > n) return arrow::Status::Invalid("truncated LZ4 block checksum");
        if (Xxh32(p + pos, len, 0) != Rd32(p + pos + len))
          return arrow::Status::IOError("LZ4 block checksum mismatch");
      }
      f.blocks.push_back({pos, len, 0, (bs >> 31) != 0});
      pos += len + (block_cks ? 4 : 0);
    }
    if (f.content_checksum) {
      if (pos + 4 > n) return arrow::Status::Invalid("truncated LZ4 content checksum");
      f.checksum = Rd32(p + pos);
      pos += 4;
    }
    f.csize = pos - f.offset;
    v.push_back(std::move(f));
  }
  return v;
}

arrow::Result<int64_t> HipCodec::Decompress(int64_t input_len, const uint8_t* input,
                                            int64_t output_buffer_len, uint8_t* output) {
  const std::lock_guard<std::mutex> lock(mu_);
  if (input_len < 0 || output_buffer_len < 0) return arrow::Status::Invalid("negative length");
  const uint64_t n = static_cast<uint64_t>(input_len);
  const bool zstd = type_ == arrow::Compression::ZSTD;
  const bool in_dev = OnDevice(input);
  // the header walk needs the bytes on the host
  std::vector<uint8_t> host;
  const uint8_t* hp = input;
  if (in_dev) {
    host.resize(n);
    ARROW_RETURN_NOT_OK(Copy(host.data(), input, n));
    ARROW_RETURN_NOT_OK(Sync());
    hp = host.data();
  }
  std::vector<Frame> frames;
  if (zstd) {
    ARROW_ASSIGN_OR_RAISE(frames, WalkZstd(hp, n));
  } else {
    ARROW_ASSIGN_OR_RAISE(frames, WalkLz4f(hp, n));
  }
  if (frames.empty()) return 0;
  const uint8_t* d_in = input;
  if (!in_dev) {
    ARROW_RETURN_NOT_OK(Reserve(d_in_, c_in_, n + 16));
    ARROW_RETURN_NOT_OK(Copy(d_in_, input, n));
    d_in = static_cast<const uint8_t*>(d_in_);
  }
  if (zstd) return DecompressZstd(frames, d_in, output_buffer_len, output);
  return DecompressLz4f(frames, d_in, n, output_buffer_len, output);
}

// Zstandard: every frame is one segment of the wave decoder; segments are as large as the
// largest frame (frames of 64 KiB, the shape this codec writes, are the common case)
arrow::Result<int64_t> HipCodec::DecompressZstd(const std::vector<Frame>& frames,
                                                const uint8_t* d_in, int64_t output_buffer_len,
                                                uint8_t* output) {
  const uint64_t nfr = frames.size();
  const uint64_t cap = static_cast<uint64_t>(output_buffer_len);
  // Declared content sizes come from untrusted headers: their sum must fit the caller's
  // buffer BEFORE anything is reserved (a frame without one: only as the single frame, sized
  // by the output buffer).
  uint64_t declared = 0;
  for (const Frame& f : frames) {
    if (!f.has_content && nfr > 1)
      return arrow::Status::NotImplemented("Zstandard frames without content size");
    const uint64_t c = f.has_content ? f.content : cap;
    if (c > (1ull << 30)) return arrow::Status::NotImplemented("Zstandard frame larger than 1 GiB");
    declared += c;
    if (declared > cap)
      return arrow::Status::Invalid("declared Zstandard content exceeds the output buffer (",
                                    output_buffer_len, ")");
  }
  // Frames are decoded in groups of consecutive frames, one launch each; a group's staging
  // is (frames) x (its largest frame), kept within the declared total + 64 KiB, so mixed
  // frame sizes never reserve more than about the output itself (equal-size frames, what
  // this codec writes: one group).
  const uint64_t budget = declared + kSeg;
  auto rnd = [](uint64_t c) { return std::max<uint64_t>((c + 15) & ~15ull, 16); };
  uint64_t total = 0;
  for (uint64_t g0 = 0; g0 < nfr;) {
    uint64_t g1 = g0, seg = 0;
    while (g1 < nfr) {
      const uint64_t c = rnd(frames[g1].has_content ? frames[g1].content : cap);
      const uint64_t s2 = std::max(seg, c);
      if (g1 > g0 && ((g1 - g0 + 1) * s2 > budget || g1 - g0 + 1 > 0x7FFFFFFFull)) break;
      seg = s2;
      ++g1;
    }
    const uint64_t nseg = g1 - g0;
    std::vector<const uint8_t*> srcs(nseg);
    std::vector<uint32_t> csz(nseg);
    for (uint64_t i = 0; i < nseg; ++i) {
      const Frame& f = frames[g0 + i];
      if (f.csize > 0xFFFFFFFFull) return arrow::Status::Invalid("Zstandard frame over 4 GiB");
      srcs[i] = d_in + f.offset;
      csz[i] = static_cast<uint32_t>(f.csize);
    }
    ARROW_RETURN_NOT_OK(Reserve(d_srcs_, c_srcs_, nseg * sizeof(void*)));
    ARROW_RETURN_NOT_OK(Reserve(d_sizes_, c_sizes_, nseg * 4));
    ARROW_RETURN_NOT_OK(Reserve(d_off_, c_off_, nseg * 4));  // produced sizes
    ARROW_RETURN_NOT_OK(Reserve(d_out_, c_out_, nseg * seg));
    ARROW_RETURN_NOT_OK(Copy(d_srcs_, srcs.data(), nseg * sizeof(void*)));
    ARROW_RETURN_NOT_OK(Copy(d_sizes_, csz.data(), nseg * 4));
    auto* dout = static_cast<uint8_t*>(d_out_);
    BITAR_ABI(bitar_hip_decompress(ctx_, nullptr, BITAR_HIP_CODEC_ZSTD,
                                   reinterpret_cast<const void* const*>(d_srcs_),
                                   static_cast<const uint32_t*>(d_sizes_),
                                   static_cast<uint32_t>(nseg), static_cast<uint32_t>(seg), dout,
                                   nseg * seg, static_cast<uint32_t*>(d_off_)),
              "bitar_hip_decompress");
    std::vector<uint32_t> prod(nseg);
    ARROW_RETURN_NOT_OK(Copy(prod.data(), d_off_, nseg * 4));
    ARROW_RETURN_NOT_OK(Sync());
    for (uint64_t i = 0; i < nseg; ++i) {
      const Frame& f = frames[g0 + i];
      if (f.has_content && prod[i] != f.content)
        return arrow::Status::IOError("Zstandard frame ", g0 + i, " decoded to a wrong size");
      if (total + prod[i] > cap)
        return arrow::Status::Invalid("decompressed size exceeds the output buffer (",
                                      output_buffer_len, ")");
      // frame i's output sits at i * seg: gather them back to back
      ARROW_RETURN_NOT_OK(Copy(output + total, dout + i * seg, prod[i]));
      total += prod[i];
    }
    ARROW_RETURN_NOT_OK(Sync());
    g0 = g1;
  }
  return static_cast<int64_t>(total);
}

arrow::Result<uint64_t> HipCodec::Lz4Independent(const Frame& f, const uint8_t* d_in,
                                                 uint8_t* dout) {
  const uint64_t nseg = f.blocks.size();
  if (nseg == 0) return 0;
  // a stored block decodes as an empty one (a lone 0x00 token) and is copied after
  ARROW_RETURN_NOT_OK(Reserve(d_aux_, c_aux_, 16));
  static const uint8_t kEmptyBlock[16] = {0};
  ARROW_RETURN_NOT_OK(Copy(d_aux_, kEmptyBlock, 16));
  const uint8_t* empty = static_cast<const uint8_t*>(d_aux_);
  std::vector<const uint8_t*> srcs(nseg);
  std::vector<uint32_t> csz(nseg);
  for (uint64_t i = 0; i < nseg; ++i) {
    const bool raw = f.blocks[i].raw;
    srcs[i] = raw ? empty : d_in + f.blocks[i].offset;
    csz[i] = raw ? 1u : f.blocks[i].csize;
  }
  ARROW_RETURN_NOT_OK(Reserve(d_srcs_, c_srcs_, nseg * sizeof(void*)));
  ARROW_RETURN_NOT_OK(Reserve(d_sizes_, c_sizes_, nseg * 4));
  ARROW_RETURN_NOT_OK(Reserve(d_off_, c_off_, nseg * 4));  // produced sizes
  ARROW_RETURN_NOT_OK(Copy(d_srcs_, srcs.data(), nseg * sizeof(void*)));
  ARROW_RETURN_NOT_OK(Copy(d_sizes_, csz.data(), nseg * 4));
  BITAR_ABI(bitar_hip_decompress(ctx_, nullptr, BITAR_HIP_CODEC_LZ4,
                                 reinterpret_cast<const void* const*>(d_srcs_),
                                 static_cast<const uint32_t*>(d_sizes_),
                                 static_cast<uint32_t>(nseg), kSeg, dout, nseg * kSeg,
                                 static_cast<uint32_t*>(d_off_)),
            "bitar_hip_decompress");
  for (uint64_t i = 0; i < nseg; ++i)
    if (f.blocks[i].raw)
      ARROW_RETURN_NOT_OK(Copy(dout + i * kSeg, d_in + f.blocks[i].offset, f.blocks[i].csize));
  ARROW_RETURN_NOT_OK(Sync());
  std::vector<uint32_t> prod(nseg);
  ARROW_RETURN_NOT_OK(Copy(prod.data(), d_off_, nseg * 4));
  ARROW_RETURN_NOT_OK(Sync());
  uint64_t total = 0;
  for (uint64_t i = 0; i < nseg; ++i) {
    const uint32_t got = f.blocks[i].raw ? f.blocks[i].csize : prod[i];
    if (i + 1 < nseg && got != kSeg)
      return arrow::Status::NotImplemented("LZ4 frame blocks of other than 64 KiB");
    total += got;
  }
  return total;
}

// LZ4 frames in order: independent blocks decode in parallel (one segment each), linked
// ones in order on one wavefront (bitar_hip_lz4_chain); content checksums checked (XXH32)
arrow::Result<int64_t> HipCodec::DecompressLz4f(const std::vector<Frame>& frames,
                                                const uint8_t* d_in, uint64_t n,
                                                int64_t output_buffer_len, uint8_t* output) {
  const uint64_t cap = static_cast<uint64_t>(output_buffer_len);
  uint64_t most = 0;  // staging: the output, plus a full last block of slack
  for (const Frame& f : frames) most += f.blocks.size() * kSeg;
  ARROW_RETURN_NOT_OK(Reserve(d_out_, c_out_, std::max<uint64_t>(std::min(most, cap + kSeg), 16)));
  auto* dout = static_cast<uint8_t*>(d_out_);
  uint64_t total = 0;
  for (const Frame& f : frames) {
    uint64_t got = 0;
    if (f.blocks.empty()) {
      got = 0;
    } else if (!f.linked) {
      if (total + f.blocks.size() * kSeg > c_out_)
        return arrow::Status::Invalid("LZ4 stream exceeds the output buffer");
      ARROW_ASSIGN_OR_RAISE(got, Lz4Independent(f, d_in, dout + total));
    } else {
      // the kernel takes 32-bit offsets: relative to the frame, whose size must fit
      if (f.csize > 0xFFFFFFFFull)
        return arrow::Status::NotImplemented("linked-block LZ4 frame over 4 GiB");
      std::vector<uint32_t> tab(2 * f.blocks.size());
      for (size_t b = 0; b < f.blocks.size(); ++b) {
        tab[2 * b] = static_cast<uint32_t>(f.blocks[b].offset - f.offset);
        tab[2 * b + 1] = f.blocks[b].csize | (f.blocks[b].raw ? 0x80000000u : 0u);
      }
      ARROW_RETURN_NOT_OK(Reserve(d_srcs_, c_srcs_, tab.size() * 4));
      ARROW_RETURN_NOT_OK(Reserve(d_off_, c_off_, 4));
      ARROW_RETURN_NOT_OK(Copy(d_srcs_, tab.data(), tab.size() * 4));
      BITAR_ABI(bitar_hip_lz4_chain(ctx_, nullptr, d_in + f.offset, static_cast<uint32_t>(f.csize),
                                    static_cast<const uint32_t*>(d_srcs_),
                                    static_cast<uint32_t>(f.blocks.size()), dout + total,
                                    c_out_ - total, static_cast<uint32_t*>(d_off_)),
                "bitar_hip_lz4_chain");
      ARROW_RETURN_NOT_OK(Sync());
      uint32_t prod = 0;
      ARROW_RETURN_NOT_OK(Copy(&prod, d_off_, 4));
      ARROW_RETURN_NOT_OK(Sync());
      got = prod;
    }
    if (f.has_content && got != f.content)
      return arrow::Status::IOError("LZ4 frame decoded to a wrong size");
    if (total + got > cap)
      return arrow::Status::Invalid("decompressed size exceeds the output buffer (",
                                    output_buffer_len, ")");
    if (f.content_checksum) {
      std::vector<uint8_t> back(got);
      ARROW_RETURN_NOT_OK(Copy(back.data(), dout + total, got));
      ARROW_RETURN_NOT_OK(Sync());
      if (Xxh32(back.data(), got, 0) != f.checksum)
        return arrow::Status::IOError("LZ4 content checksum mismatch");
    }
    total += got;
  }
  ARROW_RETURN_NOT_OK(Copy(output, dout, total));
  ARROW_RETURN_NOT_OK(Sync());
  return static_cast<int64_t>(total);
}

}  // namespace

arrow::Result<std::unique_ptr<arrow::util::Codec>> MakeArrowCodec(arrow::Compression::type type,
                                                                  int device) {
  if (type != arrow::Compression::ZSTD && type != arrow::Compression::LZ4_FRAME)
    return arrow::Status::NotImplemented("HIP codec for ",
                                         arrow::util::Codec::GetCodecAsString(type));
  bitar_hip_config cfg{1, 0};
  bitar_hip_ctx* ctx = nullptr;
  BITAR_ABI(bitar_hip_open(device, &cfg, &ctx), "bitar_hip_open");
  return std::unique_ptr<arrow::util::Codec>(new HipCodec(type, device, ctx));
}

}  // namespace bitar
