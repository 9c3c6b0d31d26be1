// bitar/arrow_codec.h -- arrow::util::Codec adapters over the MI355X engine (SURVEY.md §8f
// rank 2: the Arrow IPC body-compression hook the reference demo leaves commented out,
// apps/demo_app.cc:148-150).
//
//   auto codec = bitar::MakeArrowCodec(arrow::Compression::ZSTD);          // or LZ4_FRAME
//   auto opts = arrow::ipc::IpcWriteOptions::Defaults();
//   opts.codec = std::shared_ptr<arrow::util::Codec>(std::move(*codec));
//   // ... arrow::ipc::MakeStreamWriter(sink, schema, opts): bodies compressed on the GPU
//
// Compress cuts the input into 64 KiB segments, compresses them on the device and writes a
// standard stream any Arrow / libzstd / liblz4 reader decodes:
//   ZSTD       one Zstandard frame per segment, concatenated (RFC 8878 allows a stream of
//              frames; ZSTD_decompress and Arrow's ZSTD codec decode it whole);
//   LZ4_FRAME  one LZ4 frame (version 01, independent blocks, 64 KiB maximum block size, no
//              checksums) whose data blocks are the segments (a block that does not shrink
//              is stored uncompressed, as the frame format requires).
// Decompress walks the frame / block headers on the host (sizes only, no decoding) and
// decodes every segment on the device.  It takes what Compress writes and any other stream
// of the same shape (Zstd frames stating a content size of 64 KiB, except the last <= 64
// KiB; LZ4 frames with independent blocks of <= 64 KiB); anything else -- linked LZ4
// blocks, bigger Zstd frames, dictionaries, checksums it cannot verify on the device -- is
// NotImplemented, never a silent CPU fallback.  Host and HBM buffers are both accepted
// (host data is staged through HBM).  Streaming compressors are NotImplemented.
#pragma once

#include <arrow/result.h>
#include <arrow/util/compression.h>

#include <memory>

namespace bitar {

/// A Codec for arrow::Compression::ZSTD or LZ4_FRAME on HIP device `device`.
arrow::Result<std::unique_ptr<arrow::util::Codec>> MakeArrowCodec(
    arrow::Compression::type type, int device = 0);

}  // namespace bitar
