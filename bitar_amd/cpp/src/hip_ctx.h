// hip_ctx.h -- process-wide helper contexts of the C ABI (one per device) used by the memory
// pools and the arrow::MemoryManager, plus status translation.  Internal header.
#pragma once

#include <arrow/status.h>

#include <string>

#include "bitar_hip.h"

namespace bitar::internal {

/// Lazily opened context on `device` (one stream), never closed before exit.
arrow::Result<bitar_hip_ctx*> HelperContext(int device);

/// negated arrow::StatusCode from the C ABI -> arrow::Status
inline arrow::Status FromAbi(int rc, const std::string& what) {
  if (rc == 0) return arrow::Status::OK();
  return arrow::Status::FromArgs(static_cast<arrow::StatusCode>(-rc), what, ": ",
                                 bitar_hip_last_error());
}

#define BITAR_ABI(expr, what) ARROW_RETURN_NOT_OK(::bitar::internal::FromAbi((expr), (what)))

}  // namespace bitar::internal
