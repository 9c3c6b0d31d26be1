// bitar/device.h -- the compress device (reference src/include/device.h:53-242).
//
// Same public surface as the reference's CompressDevice<Class>: Initialize, Compress,
// Decompress, Recycle, LcoreOf, device_id, num_qps.  One device = one MI355X; a queue pair
// = one HIP stream + its staging buffers; one call = one kernel launch over every segment
// (the enqueue/dequeue burst loop of device.cc:204-235 disappears into the grid).
// Device work goes through the C ABI of libbitar_hip.so (include/bitar_hip.h).
#pragma once

#include <arrow/result.h>
#include <arrow/status.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_set>
#include <vector>

#include "bitar/config.h"
#include "bitar/type_fwd.h"

namespace arrow {
class Buffer;
class ResizableBuffer;
}  // namespace arrow

struct bitar_hip_ctx;

namespace bitar {

namespace internal {

enum class DeviceState { kUndefined = 1U << 0U, kConfigured = 1U << 1U, kStarted = 1U << 2U };

struct QueuePairMemory;  // per-queue-pair stream + staging (memory.cc analogue)
class DeviceMemory;      // pool of output slots in HBM (memory.cc:120-228 analogue)

}  // namespace internal

template <typename Class,
          typename = internal::IsEnumConstant<internal::DriverClass, Class>>
class CompressDevice {
 public:
  CompressDevice(const CompressDevice&) = delete;
  CompressDevice& operator=(const CompressDevice&) = delete;
  CompressDevice& operator=(CompressDevice&&) = delete;

  /// \brief Initialize this compress device with a corresponding type of configuration.
  virtual arrow::Status Initialize(std::unique_ptr<Configuration<Class>> configuration);

  /// \brief Compress a buffer via the \p queue_pair_id
  /// \return one buffer per segment: non-owning views of device-owned HBM slots
  ///         (is_cpu() == false), valid until Recycle() or device destruction.
  ///
  /// The input may live in HBM of this device (read in place) or in host memory (staged to
  /// HBM on the queue pair's stream first).
  arrow::Result<BufferVector> Compress(std::uint16_t queue_pair_id,
                                       const std::shared_ptr<arrow::Buffer>& decompressed_buffer);

  /// \brief Decompress buffers via the \p queue_pair_id into \p decompressed_buffer, whose
  /// capacity must be >= compressed_buffers.size() * decompressed_seg_size(); segment i
  /// lands at offset i * decompressed_seg_size() and the buffer is resized to the total.
  arrow::Status Decompress(std::uint16_t queue_pair_id, const BufferVector& compressed_buffers,
                           const std::unique_ptr<arrow::ResizableBuffer>& decompressed_buffer);

  /// \brief Return the output slots behind buffers returned by Compress().
  /// \return the number of buffers recycled
  std::size_t Recycle(const BufferVector& buffers);

  /// \brief The worker ("lcore") id that runs async calls of \p queue_pair_id.
  [[nodiscard]] auto LcoreOf(std::uint16_t queue_pair_id) const {
    return worker_lcores_.at(queue_pair_id);
  }

  [[nodiscard]] auto device_id() const noexcept { return device_id_; }

  [[nodiscard]] std::uint16_t num_qps() const noexcept {
    return static_cast<std::uint16_t>(worker_lcores_.size());
  }

  /// HIP extras: bytes per output slot, and the hipStream_t of a queue pair.
  [[nodiscard]] std::uint64_t slot_size() const noexcept { return slot_size_; }
  [[nodiscard]] void* stream(std::uint16_t queue_pair_id) const;
  /// log2 of the farthest match distance the configured encoder emits (12; 14 for the wide
  /// LZ4 parse), set by Initialize.  configuration's window_size() is what was requested (or
  /// this value when 0 was), as in the reference.
  [[nodiscard]] std::uint8_t encoder_window() const noexcept { return encoder_window_; }

  /// \brief Per-segment checksums of the last Compress (over its input) or Decompress (over
  /// its output) on \p queue_pair_id, when the configuration asks for a checksum type: the
  /// values DPDK leaves in rte_comp_op::input_chksum / output_chksum (CRC32 in bits 0..31,
  /// Adler32 in bits 32..63 for CRC32_ADLER32).  Empty when no checksum is configured.
  [[nodiscard]] const std::vector<std::uint64_t>& checksums(std::uint16_t queue_pair_id) const;

  virtual ~CompressDevice();

 protected:
  CompressDevice(std::uint8_t device_id, std::vector<std::uint32_t> worker_lcores);

  /// \brief Validate the configuration for this compress device.
  virtual arrow::Status ValidateConfiguration();

  [[nodiscard]] const std::unique_ptr<Configuration<Class>>& configuration() const noexcept {
    return configuration_;
  }

  virtual arrow::Status set_configuration(std::unique_ptr<Configuration<Class>> configuration);

  /// The checksum to compute per segment (BITAR_HIP_CHECKSUM_*), 0 for none.
  [[nodiscard]] virtual std::uint32_t checksum_kind() const { return 0; }

  [[nodiscard]] auto state() const noexcept { return state_; }
  void set_state(internal::DeviceState state) { state_ = state; }

 private:
  arrow::Status PreAllocateMemory();
  /// State / range / busy checks; on OK the queue pair is marked busy until the call ends.
  arrow::Status EntryGuard(std::uint16_t queue_pair_id);
  void Leave(std::uint16_t queue_pair_id);

  const std::uint8_t device_id_;
  const std::vector<std::uint32_t> worker_lcores_;

  std::unique_ptr<Configuration<Class>> configuration_;
  internal::DeviceState state_{internal::DeviceState::kUndefined};

  bitar_hip_ctx* ctx_ = nullptr;
  std::uint64_t slot_size_ = 0;
  std::uint8_t encoder_window_ = 0;
  std::unique_ptr<internal::DeviceMemory> device_memory_;
  std::vector<std::unique_ptr<internal::QueuePairMemory>> qp_memory_;
};

class DeviceManager {
 public:
  DeviceManager(const DeviceManager&) = delete;
  DeviceManager& operator=(const DeviceManager&) = delete;

  static DeviceManager* Instance();

  template <typename Class, typename = internal::IsEnumConstant<internal::DriverClass, Class>>
  arrow::Result<CompressDevice<Class>*> Create(std::uint8_t device_id,
                                               std::vector<std::uint32_t> worker_lcores);

 private:
  DeviceManager() = default;
  ~DeviceManager() = default;
};

using HipGfx950CompressDevice = CompressDevice<Class_HIP_GFX950>;

template <>
arrow::Result<HipGfx950CompressDevice*> DeviceManager::Create<Class_HIP_GFX950>(
    std::uint8_t device_id, std::vector<std::uint32_t> worker_lcores);

/// An MI355X compress device (the BlueFieldCompressDevice analogue, device.h:221-241).
class HipCompressDevice : public HipGfx950CompressDevice {
  using CompressDevice::CompressDevice;

 public:
  HipCompressDevice(const HipCompressDevice&) = delete;
  HipCompressDevice& operator=(const HipCompressDevice&) = delete;
  ~HipCompressDevice() override = default;

 protected:
  arrow::Status ValidateConfiguration() override;
  arrow::Status set_configuration(
      std::unique_ptr<Configuration<Class_HIP_GFX950>> configuration) override;
  [[nodiscard]] std::uint32_t checksum_kind() const override;

  friend arrow::Result<HipGfx950CompressDevice*>
  DeviceManager::Create<Class_HIP_GFX950>(std::uint8_t, std::vector<std::uint32_t>);
};

}  // namespace bitar
