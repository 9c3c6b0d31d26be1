// bitar/type_fwd.h -- the compressed-frame container (reference src/include/type_fwd.h:32).
#pragma once

#include <arrow/buffer.h>

#include <memory>
#include <vector>

namespace bitar {

/// One compressed segment per element: non-owning views into device-owned output slots
/// (valid until CompressDevice::Recycle or device destruction).
using BufferVector = std::vector<std::unique_ptr<arrow::Buffer>>;

}  // namespace bitar
