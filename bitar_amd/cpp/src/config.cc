// config.cc -- Configuration::ToString (reference src/config.cc:40-47, 77-81).
#include "bitar/config.h"

#include <sstream>

namespace bitar {

std::string_view ToString(Codec c) {
  switch (c) {
    case Codec::DEFLATE: return "DEFLATE";
    case Codec::LZ4: return "LZ4";
    case Codec::ZSTD: return "ZSTD";
  }
  return "UNKNOWN";
}

std::string_view ToString(HuffmanEncoding h) {
  switch (h) {
    case HuffmanEncoding::DEFAULT: return "DEFAULT";
    case HuffmanEncoding::FIXED: return "FIXED";
    case HuffmanEncoding::DYNAMIC: return "DYNAMIC";
  }
  return "UNKNOWN";
}

std::string_view ToString(ChecksumType c) {
  switch (c) {
    case ChecksumType::NONE: return "NONE";
    case ChecksumType::CRC32: return "CRC32";
    case ChecksumType::ADLER32: return "ADLER32";
    case ChecksumType::CRC32_ADLER32: return "CRC32_ADLER32";
  }
  return "UNKNOWN";
}

template <typename Class, typename Enable>
std::string Configuration<Class, Enable>::ToString() const {
  std::ostringstream os;
  os << "burst_size: " << burst_size_ << ", max_sgl_segs: " << max_sgl_segs_
     << ", decompressed_seg_size: " << decompressed_seg_size_
     << ", compressed_seg_size: " << compressed_seg_size_
     << ", window_size: " << static_cast<int>(window_size_)
     << ", huffman_enc: " << bitar::ToString(huffman_enc_) << ", codec: " << bitar::ToString(codec_)
     << ", level: " << static_cast<int>(level_);
  return os.str();
}

template class Configuration<Class_HIP_GFX950>;

std::string HipConfiguration::ToString() const {
  return "{ " + Configuration<Class_HIP_GFX950>::ToString() +
         ", checksum_type: " + std::string(bitar::ToString(checksum_type_)) + " }";
}

}  // namespace bitar
