/*
 * bitar_hip.h -- the C-ABI boundary of the MI355X segment codec engine (libbitar_hip.so).
 *
 * Plain pointers and sizes only; no Arrow, torch or HIP types in the signatures
 * (hipStream_t travels as void*).  Every entry point returns 0 or a negated
 * arrow::StatusCode, the convention the reference carries in an int
 * (reference src/include/util.h:157-205).
 *
 * Each function names the reference interface it replaces.  The reference drives a
 * BlueField-2 DEFLATE engine through DPDK compressdev; here one HIP kernel launch
 * replaces a whole enqueue/dequeue burst loop, and a HIP stream replaces a queue pair.
 */
#ifndef BITAR_HIP_H_
#define BITAR_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BITAR_HIP_ABI_VERSION 3

/* negated arrow::StatusCode */
enum bitar_hip_status {
  BITAR_HIP_OK = 0,
  BITAR_HIP_OUT_OF_MEMORY = -1,
  BITAR_HIP_INVALID = -4,
  BITAR_HIP_IO_ERROR = -5,
  BITAR_HIP_CAPACITY_ERROR = -6,
  BITAR_HIP_CANCELLED = -8,
  BITAR_HIP_UNKNOWN_ERROR = -9,
  BITAR_HIP_NOT_IMPLEMENTED = -10
};

/* Codec of one segment op.  DEFLATE = raw RFC 1951 stream per segment, the reference's
 * frame (reference src/config.cc:83-105, memory.cc:110).  LZ4 = raw LZ4 block per segment
 * (the north-star codec).  ZSTD = one RFC 8878 Zstandard frame per segment (the DPDK
 * RTE_COMP_ALGO_ZSTD path of reference src/config.cc:83-105 / BASELINE configs[5]). */
enum bitar_hip_codec {
  BITAR_HIP_CODEC_LZ4 = 1,
  BITAR_HIP_CODEC_DEFLATE = 2,         /* fixed-Huffman blocks (HuffmanEncoding::FIXED) */
  BITAR_HIP_CODEC_ZSTD = 3,
  BITAR_HIP_CODEC_DEFLATE_DYNAMIC = 4, /* dynamic Huffman (HuffmanEncoding::DYNAMIC, the
                                          reference default, config.h:151); decoded like
                                          DEFLATE.  Compress runs two kernels through a
                                          stream-ordered scratch allocation. */
  BITAR_HIP_CODEC_LZ4_WIDE = 5         /* LZ4 blocks from the wide parse: 16 KiB history (match
                                          distance <= 14848), 4096-entry table -- the ratio
                                          operating point, within a few % of liblz4's ratio
                                          at a lower speed; the streams are ordinary LZ4 blocks
                                          (decoded like LZ4).  The C++ front-end selects it for
                                          Codec::LZ4 at level() >= 2 (bitar/config.h). */
};

/* Per-segment marker written into sizes[] / produced[] when that segment's op failed
 * (malformed stream, or output larger than its slot: the reference's
 * RTE_COMP_OP_STATUS_OUT_OF_SPACE_*, device.cc:512-520). */
#define BITAR_HIP_SEGMENT_ERROR 0xFFFFFFFFu

/* Largest segment a kernel accepts (LZ4 offsets are 16-bit; the reference caps segments
 * at kMaxSegSize = 59460, config.h:41-47). */
#define BITAR_HIP_MAX_SEG_SIZE 65536u

typedef struct bitar_hip_ctx bitar_hip_ctx;

typedef struct {
  uint32_t num_streams; /* queue pairs: one HIP stream each (driver.cc:100-157 lcore map) */
  uint32_t flags;       /* BITAR_HIP_FLAG_* (0: the default decoders, no path counters) */
} bitar_hip_config;

/* bitar_hip_config.flags: the context's initial decoder options (bitar_hip_decoder_options);
 * every context keeps its own, so engines with different settings run side by side. */
#define BITAR_HIP_FLAG_INFLATE_WAVE_ONLY 0x1u /* no lane inflater in front of inflate_kernel
                                                 (the default since round 3; the flag also
                                                 overrides BITAR_HIP_INFLATE_LANES) */
#define BITAR_HIP_FLAG_ZSTD_WAVE_ONLY 0x2u    /* no lane Zstd decoder in front of the wave one */
#define BITAR_HIP_FLAG_ZSTD_LANE_EXEC 0x4u    /* handed-off sequence sections: lane executor */
#define BITAR_HIP_FLAG_COUNT_PATHS 0x8u       /* count decoder path entries (see below) */
#define BITAR_HIP_FLAG_PLAIN_ORDER 0x10u      /* calls dispatch segment i as workgroup i
                                                 (default, from 2048 segments: estimated most
                                                 expensive first; the output is identical) */
#define BITAR_HIP_FLAG_ZSTD_SERIAL 0x20u      /* Zstd decode: the Huffman literal streams and
                                                 the sequences' phase A one after the other on
                                                 the call's stream (default: side by side, the
                                                 literals on a paired stream; same output) */

/* Number of visible gfx950 devices.  Replaces rte_compressdev_devices_get() in
 * CompressDriver::ListAvailableDeviceIds (reference src/driver.cc:173-190). */
int bitar_hip_device_count(int* count);

/* Open a device context with cfg->num_streams streams.  Replaces
 * CompressDevice::Initialize: configure + queue_pair_setup + start
 * (reference src/device.cc:114-154). */
int bitar_hip_open(int device, const bitar_hip_config* cfg, bitar_hip_ctx** out);

/* Release streams and device state.  Replaces ~CompressDevice (device.cc:329-343). */
int bitar_hip_close(bitar_hip_ctx* ctx);

/* The hipStream_t behind queue pair `qp` (returned as void*). */
int bitar_hip_stream(bitar_hip_ctx* ctx, uint32_t qp, void** stream);

/* Device ordinal of the context. */
int bitar_hip_device(bitar_hip_ctx* ctx, int* device);

/* Worst-case compressed bytes of one segment of `seg` bytes (LZ4_compressBound /
 * fixed-Huffman bound), rounded up to 256 B.  Plays the role of compressed_seg_size
 * (reference src/config.cc:59-73): the stride of output slots in a slab. */
uint64_t bitar_hip_slot_size(uint32_t codec, uint32_t seg);

/* Largest match distance the encoder of `codec` emits (0 for an unknown codec): the reach of
 * its sliding window, 2560 for the fast parses of LZ4 / DEFLATE / Zstd and 14848 for the
 * wide LZ4 parse.  The front-end reports ceil(log2) of it as the configured window_size
 * (the reference sets the device maximum, src/device.cc:389-393; its streams are valid for
 * any window at least this large, and the decoders accept the full 32 KiB / 64 KiB). */
uint32_t bitar_hip_max_distance(uint32_t codec);

/* HBM / pinned-host allocations on the context's device.  Replace the memzone reservation
 * of RtememzoneAllocator::AllocateAligned / rte_malloc (reference src/memory_pool.cc:70-188).
 * Device allocations are 256-B aligned. */
int bitar_hip_alloc(bitar_hip_ctx* ctx, uint64_t bytes, void** ptr);
int bitar_hip_free(bitar_hip_ctx* ctx, void* ptr);
int bitar_hip_host_alloc(bitar_hip_ctx* ctx, uint64_t bytes, void** ptr);
int bitar_hip_host_free(bitar_hip_ctx* ctx, void* ptr);

/* Asynchronous copy in any direction on `stream`.  In every call `stream` is a hipStream_t;
 * NULL is the HIP default stream, queue-pair streams come from bitar_hip_stream(). */
int bitar_hip_memcpy(bitar_hip_ctx* ctx, void* dst, const void* src, uint64_t bytes,
                     void* stream);

/* Compress n bytes at d_in (device memory) as ceil(n/seg) independent segments.
 * Segment i is written to d_slab + i*slot_stride and d_sizes[i] receives its compressed
 * size.  Asynchronous on `stream`.  n == 0 launches nothing.
 * Replaces one CompressDevice::Compress call: the AssembleFrom / EnqueueBurst /
 * DequeueBurst loop over bursts of segments (reference src/device.cc:156-238,
 * src/memory.cc:350-430).  slot_stride must be >= bitar_hip_slot_size(codec, seg); d_slab
 * and slot_stride must be 16-B aligned. */
int bitar_hip_compress(bitar_hip_ctx* ctx, void* stream, uint32_t codec, const void* d_in,
                       uint64_t n, uint32_t seg, void* d_slab, uint64_t slot_stride,
                       uint32_t* d_sizes);

/* Same, but segment i goes to its own slot d_dsts[i] (a device array of device pointers,
 * each 16-B aligned with room for slot_capacity >= bitar_hip_slot_size(codec, seg) bytes).
 * The form the slot pool of the C++ front-end uses: its free slots are not contiguous
 * (DeviceMemory::Take, reference src/memory.cc:160-189). */
int bitar_hip_compress_scattered(bitar_hip_ctx* ctx, void* stream, uint32_t codec,
                                 const void* d_in, uint64_t n, uint32_t seg,
                                 void* const* d_dsts, uint64_t slot_capacity, uint32_t* d_sizes);

/* Decompress nseg segments.  d_srcs[i] (a device array of device pointers) holds
 * d_sizes[i] compressed bytes; segment i inflates into d_out + i*seg and d_produced[i]
 * receives its size.  Requires capacity >= nseg*seg, else BITAR_HIP_CAPACITY_ERROR
 * (reference device.cc:248-254).  seg <= 65536, except for Zstd: <= 2^30, so that a whole
 * stock frame of any content size can be one segment.  Asynchronous on `stream`.
 * Replaces one CompressDevice::Decompress call (reference src/device.cc:240-318,
 * src/memory.cc:432-505). */
int bitar_hip_decompress(bitar_hip_ctx* ctx, void* stream, uint32_t codec,
                         const void* const* d_srcs, const uint32_t* d_sizes, uint32_t nseg,
                         uint32_t seg, void* d_out, uint64_t capacity, uint32_t* d_produced);

/* Same, with segment i at d_slab + i*slot_stride (the layout bitar_hip_compress writes). */
int bitar_hip_decompress_slab(bitar_hip_ctx* ctx, void* stream, uint32_t codec,
                              const void* d_slab, uint64_t slot_stride,
                              const uint32_t* d_sizes, uint32_t nseg, uint32_t seg,
                              void* d_out, uint64_t capacity, uint32_t* d_produced);

/* Compress n bytes of HOST memory (pinned or pageable) at h_in with the PCIe link and the
 * kernels overlapped: the input is copied into d_stage (device memory, >= n bytes) in chunks
 * of whole segments (about 1/8 of the call, >= 32 MiB) on a copy stream paired with
 * `stream`, and each chunk is compressed on `stream` as soon as it has landed, so a call
 * takes about the link time plus one chunk's compress.  The output is a slab (d_slab, as
 * bitar_hip_compress) or scattered slots (d_dsts with d_slab NULL, as
 * bitar_hip_compress_scattered; slot_stride is then the slots' capacity).  Asynchronous on
 * `stream`; bitar_hip_sync(stream) covers the copies too.  Replaces the zero-copy attach of
 * host input slices the BlueField DMAs from (reference src/memory.cc:380-399,
 * rte_mem_virt2iova at 388). */
int bitar_hip_compress_host(bitar_hip_ctx* ctx, void* stream, uint32_t codec, const void* h_in,
                            uint64_t n, uint32_t seg, void* d_stage, void* d_slab,
                            void* const* d_dsts, uint64_t slot_stride, uint32_t* d_sizes);

/* Decompress into HOST memory: the segments decode into d_stage (device memory, >= nseg*seg
 * bytes) in chunks, and each decoded chunk is copied to h_out on the paired copy stream while
 * the next one decodes; nseg*seg bytes land at h_out (capacity >= nseg*seg, else
 * BITAR_HIP_CAPACITY_ERROR).  Otherwise as bitar_hip_decompress; bitar_hip_sync(stream)
 * covers the copies.  Replaces decompression into host-memory output slices (reference
 * src/memory.cc:482-493). */
int bitar_hip_decompress_host(bitar_hip_ctx* ctx, void* stream, uint32_t codec,
                              const void* const* d_srcs, const uint32_t* d_sizes, uint32_t nseg,
                              uint32_t seg, void* d_stage, void* h_out, uint64_t capacity,
                              uint32_t* d_produced);

/* Wait for `stream` and return BITAR_HIP_IO_ERROR if a segment op launched on THAT stream
 * failed since its last sync (each stream has its own sticky device-side error word, read
 * and cleared in stream order, so concurrent queue pairs never see each other's failures).
 * NULL waits for the default stream and the context's queue pairs and reports / clears
 * their words only: a foreign stream's word (e.g. a torch side stream) is left to a sync of
 * that stream, which reports it exactly once.  Replaces the
 * completion polling of DequeueBurst + GetErrorCount (reference src/device.cc:84-110,
 * 490-535). */
int bitar_hip_sync(bitar_hip_ctx* ctx, void* stream);

/* Exclusive prefix sum of d_sizes (nseg entries) into d_offsets (nseg+1 entries), then
 * gather each slot into one contiguous frame at d_frame (d_frame may be NULL to compute
 * offsets only).  Builds the packed frame / global frame index.  A size
 * above slot_stride (BITAR_HIP_SEGMENT_ERROR of a failed op) packs as 0 bytes and makes the
 * next bitar_hip_sync of `stream` return BITAR_HIP_IO_ERROR; slot_stride may be 0 only when
 * d_frame is NULL. */
int bitar_hip_pack(bitar_hip_ctx* ctx, void* stream, const void* d_slab, uint64_t slot_stride,
                   const uint32_t* d_sizes, uint32_t nseg, uint64_t* d_offsets, void* d_frame);

/* LZ4 frame with LINKED blocks (LZ4 frame format Block_Independence = 0, the liblz4 and
 * Arrow LZ4_FRAME default): the blocks of ONE frame decode in order on one wavefront, each
 * block's matches reaching into the output of the blocks before it.  d_blocks holds nblocks
 * pairs {offset of the block's data in d_src, size | 1u << 31 for a stored block}; the
 * output goes to d_out (capacity bytes) and *d_produced receives its total size, or
 * BITAR_HIP_SEGMENT_ERROR (then the next sync returns BITAR_HIP_IO_ERROR).  Asynchronous on
 * `stream`.  Frame / block checksums are the caller's (XXH32).  Used by the Arrow util::Codec
 * adapter for stock IPC bodies. */
int bitar_hip_lz4_chain(bitar_hip_ctx* ctx, void* stream, const void* d_src, uint32_t src_len,
                        const uint32_t* d_blocks, uint32_t nblocks, void* d_out,
                        uint64_t capacity, uint32_t* d_produced);

/* Batched device-to-device copy: entry i moves d_sizes[i] bytes from d_srcs[i] to d_dsts[i]
 * (device arrays of n device pointers / sizes; any alignment, ranges must not overlap).
 * Asynchronous on `stream`.  The front-end's chained operations (max_sgl_segs > 1) use it to
 * spread one op's compressed stream over its pool slots and to join a chained input: the
 * mbuf chains the reference builds with rte_pktmbuf_chain (src/memory.cc:60-100, 380-425,
 * 459-500). */
int bitar_hip_copy_batch(bitar_hip_ctx* ctx, void* stream, const void* const* d_srcs,
                         void* const* d_dsts, const uint32_t* d_sizes, uint32_t n);

/* The data blocks of an LZ4 frame (LZ4 frame format, block independence) from LZ4 segments
 * of n input bytes (d_in, segment size seg <= 65536, so the frame's maximum block size is
 * 64 KiB): block i = LE32 size + the compressed block, or LE32(len | 1<<31) + the raw input
 * slice when the block did not shrink.  d_framed (nseg uint32) receives the framed sizes,
 * d_offsets (nseg+1 uint64) their exclusive prefix sum; d_frame may be NULL to size only.
 * The frame header and EndMark are the caller's.  Used by the Arrow util::Codec adapter
 * (arrow::Compression::LZ4_FRAME, the Arrow IPC body codec). */
int bitar_hip_pack_lz4f(bitar_hip_ctx* ctx, void* stream, const void* d_in, uint64_t n,
                        uint32_t seg, const void* d_slab, uint64_t slot_stride,
                        const uint32_t* d_sizes, uint32_t* d_framed, uint64_t* d_offsets,
                        void* d_frame);

/* Deterministic synthetic input (SplitMix64-based; kinds as in the oracle's bo_fill:
 * 0 random, 1 Silesia-style mix, 2 Arrow record-batch body, 3 constant, 4 periodic,
 * 5 int64 small-range only, 6 log text only). */
int bitar_hip_fill(bitar_hip_ctx* ctx, void* stream, int kind, uint64_t seed, void* d_out,
                   uint64_t n);

/* Bytes [offset, offset + n) of the same deterministic stream (offset a multiple of 64), so
 * a rank can generate just the batches of a job it was dealt. */
int bitar_hip_fill_at(bitar_hip_ctx* ctx, void* stream, int kind, uint64_t seed,
                      uint64_t offset, void* d_out, uint64_t n);

/* Checksum types (rte_comp_checksum_type, reference src/include/config.h:169-182). */
enum bitar_hip_checksum_kind {
  BITAR_HIP_CHECKSUM_CRC32 = 1,         /* zlib / ISO-HDLC CRC-32 */
  BITAR_HIP_CHECKSUM_ADLER32 = 2,       /* RFC 1950 Adler-32 */
  BITAR_HIP_CHECKSUM_CRC32_ADLER32 = 3  /* CRC-32 in bits 0..31, Adler-32 in bits 32..63 */
};

/* Per-segment checksum of uncompressed data -- what the reference's xforms ask the engine to
 * compute over an op's uncompressed side (checksum_type in compress_xform / decompress_xform,
 * reference src/config.cc:83-105): segment i starts at d_data + i*seg and holds d_lens[i]
 * bytes (a decompress's d_produced; BITAR_HIP_SEGMENT_ERROR gives 0), or, with d_lens NULL,
 * min(seg, n - i*seg) bytes (a compress's input; then nseg must be ceil(n / seg)).
 * d_sums[i] (uint64) receives the checksum.  Asynchronous on `stream`. */
int bitar_hip_checksum(bitar_hip_ctx* ctx, void* stream, uint32_t kind, const void* d_data,
                       uint64_t n, uint32_t seg, const uint32_t* d_lens, uint32_t nseg,
                       uint64_t* d_sums);

/* Decoder selection of one context.  The decoders are interchangeable (every one accepts and
 * rejects exactly what the oracle does); the options pick which kernels run, for tests and
 * tuning.  No reference counterpart: the BlueField engine has one decoder. */
typedef struct {
  uint32_t inflate_lanes; /* segments per wave of inflate_lanes_kernel: 4, 8, 16 or 32;
                             0 = inflate_kernel (one wave per segment) alone */
  uint32_t zstd_lanes;    /* segments per wave of zstd_lanes_kernel: 8, 16, 32 or 64; 0 = off */
  uint32_t zstd_seq;      /* 1 = handed-off sequence sections run zstd_seqdec_kernel +
                             zstd_exec_kernel; 0 = the lane executor (zstd_handoff_kernel) */
  uint32_t count_paths;   /* 1 = count path entries (bitar_hip_path_counters) */
} bitar_hip_decoder_options;

int bitar_hip_get_decoder_options(bitar_hip_ctx* ctx, bitar_hip_decoder_options* opt);
/* Takes effect for calls made after it returns (calls already queued keep their kernels). */
int bitar_hip_set_decoder_options(bitar_hip_ctx* ctx, const bitar_hip_decoder_options* opt);

/* Path counters (counted while count_paths is on): how many segments reached each stage of
 * the decoders, so tests can show that their inputs exercised the path they target. */
enum bitar_hip_path_counter {
  BITAR_HIP_PATH_INFLATE_WAVE = 0,       /* segments decoded by inflate_kernel */
  BITAR_HIP_PATH_INFLATE_WAVE_REJECT = 1,/*   ... of which rejected */
  BITAR_HIP_PATH_INFLATE_BATCH_SEGS = 2, /*   ... that ran >= 1 multi-symbol batch */
  BITAR_HIP_PATH_INFLATE_BATCHES = 3,    /* batches run by inflate_kernel */
  BITAR_HIP_PATH_ZSTD_WAVE = 4,          /* segments decoded by zstd_decompress_kernel */
  BITAR_HIP_PATH_ZSTD_HANDED = 5,        /*   ... that handed their last block over */
  BITAR_HIP_PATH_ZSTD_SEQDEC = 6,        /* handed segments taken by zstd_seqdec_kernel */
  BITAR_HIP_PATH_ZSTD_SEQDEC_REJECT = 7, /*   ... rejected there */
  BITAR_HIP_PATH_ZSTD_EXEC = 8,          /* segments executed by zstd_exec_kernel */
  BITAR_HIP_PATH_ZSTD_EXEC_REJECT = 9,   /*   ... rejected there */
  BITAR_HIP_PATH_LZ4_FAR = 10,           /* segments deferred to the far-history LZ4 kernel */
  /* 11..15: LZ4 batch-path diagnostics, filled only by a library built with
     -DBITAR_LZ4D_PROFILE=1 (scripts/build_variant.sh): batches, their output bytes,
     sequences decoded by the general path, batches whose walk ended at the parsed lanes'
     end, batches whose walk ended at an ineligible sequence */
  BITAR_HIP_PATH_LZ4_BATCHES = 11,
  BITAR_HIP_PATH_LZ4_BATCH_BYTES = 12,
  BITAR_HIP_PATH_LZ4_GENERAL_SEQS = 13,
  BITAR_HIP_PATH_LZ4_STOP_PARSE = 14,
  BITAR_HIP_PATH_LZ4_STOP_INELIGIBLE = 15,
  BITAR_HIP_PATH_COUNT = 16
};

/* Wait for the device, copy min(n, BITAR_HIP_PATH_COUNT) counters to out (host memory) and
 * reset them. */
int bitar_hip_path_counters(bitar_hip_ctx* ctx, uint64_t* out, uint32_t n);

/* Where `ptr` lives: *kind = 0 pageable host, 1 pinned host, 2 device memory (then *device
 * is its ordinal).  Replaces rte_mem_virt2iova() residency assumptions (memory.cc:388). */
int bitar_hip_pointer_info(const void* ptr, int* kind, int* device);

/* Thread-local text of the last error returned on this thread. */
const char* bitar_hip_last_error(void);

/* ABI version (BITAR_HIP_ABI_VERSION). */
int bitar_hip_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* BITAR_HIP_H_ */
