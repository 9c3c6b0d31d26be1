// bitar/config.h -- device configuration (reference src/include/config.h:37-185).
//
// Same setters/getters and slot-sizing rule as the reference's Configuration<Class>; the
// DPDK rte_comp_xform / rte_comp_huffman / rte_comp_checksum_type types are replaced by
// plain enums, and the driver class MLX5_PCI by HIP_GFX950 (one MI355X = one device).
#pragma once

#include <cstdint>
#include <limits>
#include <string>
#include <string_view>
#include <type_traits>

namespace bitar {

namespace internal {

static inline constexpr auto kExpanseRatio = 1.1;  // reference config.h:41
// The reference caps segments at (65535 - RTE_PKTMBUF_HEADROOM) / 1.1 = 59460
// (config.h:42-47); kept for the uint16 API, the HIP engine also takes 65536 through
// set_decompressed_seg_size32.
static inline constexpr std::uint32_t kMaxMbufDataSize =
    std::numeric_limits<std::uint16_t>::max() - 128;
static inline constexpr std::uint32_t kMinSegSize = 8;
static inline constexpr std::uint32_t kMaxSegSize =
    static_cast<std::uint16_t>(kMaxMbufDataSize / kExpanseRatio);
static inline constexpr std::uint32_t kMaxSegSize32 = 65536;
static inline constexpr std::uint32_t kDefaultSegSize = 2048;
static inline constexpr std::uint16_t kMaxPreallocateSlots = 65535;

enum class DriverClass : std::int8_t { HIP_GFX950 };

template <typename EnumClass, typename Constant>
using IsEnumConstant = std::enable_if_t<std::is_enum_v<EnumClass> &&
                                        std::is_same_v<decltype(Constant::value), const EnumClass>>;

}  // namespace internal

using Class_HIP_GFX950 =
    std::integral_constant<internal::DriverClass, internal::DriverClass::HIP_GFX950>;

/// The segment codec (the reference hard-codes RTE_COMP_ALGO_DEFLATE, config.cc:86-88;
/// ZSTD is DPDK's RTE_COMP_ALGO_ZSTD-shaped option, BASELINE configs[5]).
enum class Codec : std::uint8_t { DEFLATE = 1, LZ4 = 2, ZSTD = 3 };
/// rte_comp_huffman
enum class HuffmanEncoding : std::uint8_t { DEFAULT = 0, FIXED = 1, DYNAMIC = 2 };
/// rte_comp_checksum_type
enum class ChecksumType : std::uint8_t { NONE = 0, CRC32 = 1, ADLER32 = 2, CRC32_ADLER32 = 3 };

std::string_view ToString(Codec c);
std::string_view ToString(HuffmanEncoding h);
std::string_view ToString(ChecksumType c);

template <typename Class,
          typename = internal::IsEnumConstant<internal::DriverClass, Class>>
class Configuration {
 public:
  Configuration() { UpdateCompressedSegSize(); }
  Configuration(const Configuration&) = default;
  Configuration(Configuration&&) noexcept = default;
  Configuration& operator=(const Configuration&) = default;
  Configuration& operator=(Configuration&&) noexcept = default;
  virtual ~Configuration() = default;

  [[nodiscard]] virtual std::string ToString() const;
  [[nodiscard]] virtual std::string_view type_name() const noexcept = 0;

  /// Ops per burst.  The HIP engine launches one kernel per call over every segment, so the
  /// value is validated (> 0) and reported but does not cut launches.
  [[nodiscard]] auto burst_size() const noexcept { return burst_size_; }
  void set_burst_size(std::uint16_t burst_size) { burst_size_ = burst_size; }

  /// Segments chained per op (SGL, reference default 1).  k > 1: the k segments of an op are
  /// compressed as one stream and spread over k slots (device.cc, chained ops).
  [[nodiscard]] auto max_sgl_segs() const noexcept { return max_sgl_segs_; }
  void set_max_sgl_segs(std::uint16_t max_sgl_segs) { max_sgl_segs_ = max_sgl_segs; }

  /// Bytes of uncompressed data per segment.
  [[nodiscard]] std::uint32_t decompressed_seg_size() const noexcept {
    return decompressed_seg_size_;
  }
  void set_decompressed_seg_size(std::uint16_t decompressed_seg_size) {
    decompressed_seg_size_ = decompressed_seg_size;
    UpdateCompressedSegSize();
  }
  /// 32-bit form for 64 KiB segments (BASELINE's chunk size), which uint16 cannot express.
  void set_decompressed_seg_size32(std::uint32_t decompressed_seg_size) {
    decompressed_seg_size_ = decompressed_seg_size;
    UpdateCompressedSegSize();
  }

  /// The reference's slot size for compressed output (config.cc:59-73).  The HIP engine's
  /// slots are max(this, the codec's worst-case bound), see CompressDevice::slot_size().
  [[nodiscard]] std::uint32_t compressed_seg_size() const noexcept {
    return compressed_seg_size_;
  }

  /// log2 of the sliding window; 0 = the device maximum.
  [[nodiscard]] auto window_size() const noexcept { return window_size_; }
  void set_window_size(std::uint8_t window_size) { window_size_ = window_size; }

  [[nodiscard]] auto huffman_enc() const noexcept { return huffman_enc_; }
  void set_huffman_enc(HuffmanEncoding huffman_enc) { huffman_enc_ = huffman_enc; }

  /// Output slots preallocated per device (the reference's memzones).
  [[nodiscard]] auto max_preallocate_memzones() const noexcept {
    return max_preallocate_memzones_;
  }
  void set_max_preallocate_memzones(std::uint16_t n) { max_preallocate_memzones_ = n; }

  [[nodiscard]] auto codec() const noexcept { return codec_; }
  void set_codec(Codec codec) { codec_ = codec; }

  /// Compression level, 1..9 (rte_comp_compress_xform.level; the reference always sets 1,
  /// config.cc:86-88).  LZ4: 1 = the fast parse, >= 2 = the wide parse (16 KiB history, the
  /// ratio operating point, BITAR_HIP_CODEC_LZ4_WIDE).  DEFLATE and ZSTD have one level.
  [[nodiscard]] auto level() const noexcept { return level_; }
  void set_level(std::uint8_t level) { level_ = level; }

 private:
  /// Configuration::UpdateCompressedSegSize (reference config.cc:59-73): the highest set bit
  /// of 2*seg, or seg*1.1 when that exceeds 32 KiB.
  void UpdateCompressedSegSize() noexcept {
    const auto lower_bound = static_cast<std::uint32_t>(decompressed_seg_size_ << 1U);
    std::uint32_t num = 1U << 17;
    while (num && (num & lower_bound) == 0) num >>= 1U;
    compressed_seg_size_ =
        num > (65536U >> 1U)
            ? static_cast<std::uint32_t>(static_cast<double>(decompressed_seg_size_) *
                                         internal::kExpanseRatio)
            : num;
  }

  std::uint16_t burst_size_ = 32;
  std::uint16_t max_sgl_segs_ = 1U;
  std::uint32_t decompressed_seg_size_ = internal::kDefaultSegSize;
  std::uint32_t compressed_seg_size_{};
  std::uint8_t window_size_ = 0U;
  HuffmanEncoding huffman_enc_ = HuffmanEncoding::DYNAMIC;  // reference config.h:151
  std::uint16_t max_preallocate_memzones_ = 1024;
  Codec codec_ = Codec::DEFLATE;
  std::uint8_t level_ = 1;
};

static inline constexpr std::string_view kHipConfigurationTypeName{"hip_gfx950"};

/// Configuration of an MI355X compress device (the BlueFieldConfiguration analogue,
/// reference config.h:155-183).
class HipConfiguration : public Configuration<Class_HIP_GFX950> {
 public:
  [[nodiscard]] std::string_view type_name() const noexcept override {
    return kHipConfigurationTypeName;
  }
  [[nodiscard]] std::string ToString() const override;

  [[nodiscard]] auto checksum_type() const noexcept { return checksum_type_; }
  void set_checksum_type(ChecksumType checksum_type) { checksum_type_ = checksum_type; }

  static HipConfiguration Defaults() { return {}; }

 private:
  ChecksumType checksum_type_ = ChecksumType::NONE;
};

}  // namespace bitar
