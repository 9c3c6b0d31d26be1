// bitar/util.h -- asynchronous Compress / Decompress (reference src/include/util.h:43-236).
//
// rte_eal_remote_launch onto a pinned lcore becomes a launch onto a persistent worker
// thread of this process (one per queue pair, ids from CompressDevice::LcoreOf), and
// rte_eal_wait_lcore becomes WaitLcore.  The callback contracts are the reference's.
#pragma once

#include <arrow/result.h>
#include <arrow/status.h>

#include <cstdint>
#include <memory>

#include "bitar/config.h"
#include "bitar/device.h"
#include "bitar/type_fwd.h"

namespace bitar {

static inline constexpr auto kAsyncReturnOK = 2;

template <typename Class, typename Callback,
          typename = internal::IsEnumConstant<internal::DriverClass, Class>>
struct CompressParam {
  /// result_callback: int(std::uint8_t device_id, std::uint16_t queue_pair_id,
  ///                      arrow::Result<bitar::BufferVector>&& result)
  /// Its return value is what WaitLcore() yields.  Held by reference (util.h:69-72): the
  /// caller keeps every argument alive until WaitLcore returns.
  CompressParam(const std::unique_ptr<bitar::CompressDevice<Class>>& device,
                std::uint16_t queue_pair_id,
                const std::shared_ptr<arrow::Buffer>& decompressed_buffer,
                const Callback& result_callback)
      : device_{device},
        queue_pair_id_{queue_pair_id},
        decompressed_buffer_{decompressed_buffer},
        result_callback_{result_callback} {}

  const std::unique_ptr<bitar::CompressDevice<Class>>& device_;
  const std::uint16_t queue_pair_id_{};
  const std::shared_ptr<arrow::Buffer>& decompressed_buffer_;
  const Callback& result_callback_;
};

template <typename Class, typename Callback,
          typename = internal::IsEnumConstant<internal::DriverClass, Class>>
struct DecompressParam {
  /// result_callback: int(std::uint8_t device_id, std::uint16_t queue_pair_id,
  ///                      const arrow::Status& status)
  DecompressParam(const std::unique_ptr<bitar::CompressDevice<Class>>& device,
                  std::uint16_t queue_pair_id, const BufferVector& compressed_buffers,
                  const std::unique_ptr<arrow::ResizableBuffer>& decompressed_buffer,
                  const Callback& result_callback)
      : device_{device},
        queue_pair_id_{queue_pair_id},
        compressed_buffers_{compressed_buffers},
        decompressed_buffer_{decompressed_buffer},
        result_callback_{result_callback} {}

  const std::unique_ptr<bitar::CompressDevice<Class>>& device_;
  const std::uint16_t queue_pair_id_{};
  const BufferVector& compressed_buffers_;
  const std::unique_ptr<arrow::ResizableBuffer>& decompressed_buffer_;
  const Callback& result_callback_;
};

namespace internal {

using LcoreFunction = int (*)(void*);

/// rte_eal_remote_launch: run fn(arg) on worker `lcore_id`; 0, or -EBUSY if it is running.
int RemoteLaunch(LcoreFunction fn, void* arg, std::uint32_t lcore_id);

template <typename Class, typename Callback,
          typename = internal::IsEnumConstant<internal::DriverClass, Class>>
int LcoreCompressFunc(void* compress_param) {
  auto* param = static_cast<CompressParam<Class, Callback>*>(compress_param);
  auto&& result = param->device_->Compress(param->queue_pair_id_, param->decompressed_buffer_);
  return param->result_callback_(param->device_->device_id(), param->queue_pair_id_,
                                 std::move(result));
}

template <typename Class, typename Callback,
          typename = internal::IsEnumConstant<internal::DriverClass, Class>>
int LcoreDecompressFunc(void* decompress_param) {
  auto* param = static_cast<DecompressParam<Class, Callback>*>(decompress_param);
  auto&& status = param->device_->Decompress(param->queue_pair_id_, param->compressed_buffers_,
                                             param->decompressed_buffer_);
  return param->result_callback_(param->device_->device_id(), param->queue_pair_id_, status);
}

}  // namespace internal

/// rte_eal_wait_lcore: block until worker `lcore_id` is idle and return the value the last
/// launched function returned (0 if nothing was launched).
int WaitLcore(std::uint32_t lcore_id);

/// \brief Asynchronously call CompressDevice<Class>::Compress on the queue pair's worker.
/// \return 0 if started, or -EBUSY if that worker is still running.
template <typename Class, typename Callback,
          typename = internal::IsEnumConstant<internal::DriverClass, Class>>
int CompressAsync(const std::unique_ptr<CompressParam<Class, Callback>>& param) {
  return internal::RemoteLaunch(internal::LcoreCompressFunc<Class, Callback>, param.get(),
                                param->device_->LcoreOf(param->queue_pair_id_));
}

/// \brief Asynchronously call CompressDevice<Class>::Decompress on the queue pair's worker.
template <typename Class, typename Callback,
          typename = internal::IsEnumConstant<internal::DriverClass, Class>>
int DecompressAsync(const std::unique_ptr<DecompressParam<Class, Callback>>& param) {
  return internal::RemoteLaunch(internal::LcoreDecompressFunc<Class, Callback>, param.get(),
                                param->device_->LcoreOf(param->queue_pair_id_));
}

}  // namespace bitar
