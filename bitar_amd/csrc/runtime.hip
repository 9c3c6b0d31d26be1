// runtime.hip -- the C-ABI of libbitar_hip.so (include/bitar_hip.h).
//
// A context = one gfx950 device + N HIP streams (queue pairs) + a sticky device error word.
// Every entry point validates shapes on the host before launching, so a kernel never sees a
// grid or a size it does not assume (one wave per segment, seg <= 65536).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bitar_hip.h"
#include "order.hip.h"
#include "zstd_hand.hip.h"
#include "zstd_layout.hip.h"

namespace bitar_hip {
template <uint32_t RING, uint32_t HLOG>
__global__ void lz4_compress_kernel(const uint8_t*, uint64_t, uint32_t, uint8_t*, uint64_t,
                                    uint8_t* const*, uint32_t*, uint32_t*, const uint32_t*);
template <bool FARK>
__global__ void lz4_decompress_kernel(const uint8_t* const*, const uint8_t*, uint64_t,
                                      const uint32_t*, uint32_t, uint32_t, uint8_t*, uint32_t*,
                                      uint32_t*, unsigned long long*, const uint32_t*);
__global__ void seg_cost_kernel(const uint8_t*, uint64_t, uint32_t, uint32_t, uint32_t*);
__global__ void order_hist_kernel(const uint32_t*, const uint32_t*, uint32_t, uint32_t, uint32_t,
                                  uint32_t*);
__global__ void order_scatter_kernel(const uint32_t*, const uint32_t*, uint32_t, uint32_t, uint32_t,
                                     uint32_t, const uint32_t*, uint32_t*);
__global__ void deflate_compress_kernel(const uint8_t*, uint64_t, uint32_t, uint8_t*, uint64_t,
                                        uint8_t* const*, uint32_t*, uint32_t*, const uint32_t*);
__global__ void inflate_kernel(const uint8_t* const*, const uint8_t*, uint64_t,
                               const uint32_t*, uint32_t, uint32_t, uint8_t*, uint32_t*,
                               uint32_t*, uint32_t, unsigned long long*, const uint32_t*);
__global__ void inflate_fixed_kernel(const uint8_t* const*, const uint8_t*, uint64_t,
                               const uint32_t*, uint32_t, uint32_t, uint8_t*, uint32_t*,
                               uint32_t*, uint32_t, unsigned long long*, const uint32_t*);
template <uint32_t L>
__global__ void inflate_lanes_kernel(const uint8_t* const*, const uint8_t*, uint64_t,
                                     const uint32_t*, uint32_t, uint32_t, uint8_t*, uint32_t*);
__global__ void zstd_parse_kernel(const uint8_t*, uint64_t, uint32_t, uint8_t*, uint64_t, uint2*, const uint32_t*);
__global__ void zstd_entropy_kernel(const uint8_t*, uint64_t, uint32_t, uint8_t*, uint64_t,
                                    const uint2*, uint8_t*, uint64_t, const uint32_t*);
__global__ void zstd_walk_kernel(const uint8_t*, uint64_t, uint32_t, uint32_t, uint8_t*, uint64_t,
                                 const uint32_t*);
__global__ void walk_key_kernel(const uint2*, uint32_t, uint32_t*);
__global__ void zstd_emit_kernel(const uint8_t*, uint64_t, uint32_t, const uint8_t*, uint64_t,
                                 uint8_t*, uint64_t, uint8_t* const*, uint32_t*, const uint8_t*,
                                 uint64_t, const uint32_t*);
__global__ void zstd_decompress_kernel(const uint8_t* const*, const uint8_t*, uint64_t,
                                       const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                       uint32_t*, uint32_t*, uint32_t, uint8_t*,
                                       unsigned long long*, const uint32_t*, uint32_t);
template <uint32_t S, uint32_t B>
__global__ void zstd_hlit_kernel(const uint8_t* const*, const uint8_t*, uint64_t,
                                 const uint32_t*, uint32_t, uint32_t, uint8_t*, uint32_t*,
                                 const uint8_t*, uint32_t*, const uint32_t*);
__global__ void hand_key_kernel(const uint32_t*, const uint8_t*, uint32_t, uint32_t, uint32_t*);
template <uint32_t L>
__global__ void zstd_handoff_kernel(const uint8_t* const*, const uint8_t*, uint64_t,
                                    const uint32_t*, uint32_t, uint32_t, uint8_t*, uint32_t*,
                                    const uint8_t*, uint32_t*);
template <uint32_t L, uint32_t B>
__global__ void zstd_seqdec_kernel(const uint8_t* const*, const uint8_t*, uint64_t,
                                   const uint32_t*, uint32_t, uint32_t, uint32_t*, uint8_t*,
                                   uint64_t*, uint32_t, uint32_t*, unsigned long long*, const uint32_t*);
__global__ void zstd_exec_kernel(const uint8_t* const*, const uint8_t*, uint64_t, uint32_t,
                                 uint32_t, uint8_t*, uint32_t*, const uint8_t*,
                                 const uint64_t*, uint32_t, uint32_t*, unsigned long long*, const uint32_t*);
template <uint32_t L>
__global__ void zstd_lanes_kernel(const uint8_t* const*, const uint8_t*, uint64_t,
                                  const uint32_t*, uint32_t, uint32_t, uint8_t*, uint32_t*);
__global__ void deflate_dyn_parse_kernel(const uint8_t*, uint64_t, uint32_t, uint8_t*, uint64_t,
                                         uint32_t*, const uint32_t*);
__global__ void deflate_dyn_emit_kernel(const uint8_t*, uint64_t, uint32_t, const uint8_t*,
                                        uint64_t, uint8_t*, uint64_t, uint8_t* const*, uint32_t*,
                                        uint32_t*, const uint32_t*);
__global__ void checksum_kernel(uint32_t, const uint8_t*, uint64_t, uint32_t, const uint32_t*,
                                uint32_t, uint64_t*);
__global__ void scan_sizes_kernel(const uint32_t*, uint32_t, uint64_t, uint64_t*, uint32_t*);
__global__ void pack_kernel(const uint8_t*, uint64_t, const uint32_t*, const uint64_t*, uint32_t,
                            uint8_t*);
__global__ void fill_kernel(int, uint64_t, uint64_t, uint8_t*, uint64_t);
__global__ void lz4_chain_kernel(const uint8_t*, uint32_t, const uint32_t*, uint32_t, uint8_t*,
                                 uint32_t, uint32_t*, uint32_t*);
__global__ void copy_batch_kernel(const uint8_t* const*, uint8_t* const*, const uint32_t*, uint32_t);
__global__ void lz4f_sizes_kernel(const uint32_t*, uint32_t, uint64_t, uint32_t, uint32_t*);
__global__ void lz4f_pack_kernel(const uint8_t*, uint64_t, uint32_t, const uint8_t*, uint64_t,
                                 const uint32_t*, const uint64_t*, uint32_t, uint8_t*);
}  // namespace bitar_hip

// Error words: one sticky uint32 per stream (bit0 decode error, bit1 slot overflow, bit2 a
// failed segment handed to pack).  Word 0 serves the NULL stream, word q+1 queue pair q, and
// further words are handed out on first use to foreign streams (e.g. torch's current
// stream), so a failure on one queue pair is never reported by -- or cleared by -- another
// (the reference reports errors per queue pair: device.cc:84-110, 512-520).
constexpr uint32_t kErrWords = 1024;

struct bitar_hip_ctx {
  int device = -1;
  std::vector<hipStream_t> streams;
  uint32_t* d_err = nullptr;  // kErrWords words
  unsigned long long* d_stats = nullptr;  // BITAR_HIP_PATH_COUNT path counters
  // decoder options (bitar_hip_decoder_options), per context
  std::atomic<uint32_t> inflate_lanes{4}, zstd_lanes{16}, zstd_seq{1}, count_paths{0};
  std::atomic<uint32_t> zstd_fork{1};  // Zstd literals beside phase A (decompress_impl)
  std::atomic<uint32_t> cost_order{1};  // LZ4: dispatch the estimated most expensive segments first
  std::mutex mu;              // guards `words` and `order_scratch`
  std::vector<std::pair<hipStream_t, uint32_t>> words;  // stream -> error word index
  // cost-ordered dispatch scratch of the context's own streams (and the default stream),
  // cached per (stream, slot) and reused in stream order (a call holds its entry's mutex from
  // the sort's launch to the last launch that reads it); foreign streams get per-call scratch
  struct OrderScratch {
    hipStream_t stream;
    int slot;
    void* p = nullptr;
    uint64_t cap = 0;
    std::mutex m;
    OrderScratch(hipStream_t s, int k) : stream(s), slot(k) {}
  };
  std::list<OrderScratch> order_scratch;
  // host-memory calls (bitar_hip_compress_host / _decompress_host): the copy stream paired
  // with each caller stream, created on first use
  std::vector<std::pair<hipStream_t, hipStream_t>> copy_streams;
  // per caller stream: a stream for kernels forked off it (Zstd literals beside sequences)
  std::vector<std::pair<hipStream_t, hipStream_t>> aux_streams;
};

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(e == hipErrorOutOfMemory ? BITAR_HIP_OUT_OF_MEMORY : BITAR_HIP_UNKNOWN_ERROR,
              std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr, what)                       \
  do {                                            \
    hipError_t _e = (expr);                       \
    if (_e != hipSuccess) return hip_fail(_e, what); \
  } while (0)

int enter(bitar_hip_ctx* ctx) {
  if (!ctx) return fail(BITAR_HIP_INVALID, "null context");
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  return 0;
}

// NULL is the HIP default stream (the usual HIP convention); queue-pair streams come from
// bitar_hip_stream().
hipStream_t pick_stream(bitar_hip_ctx*, void* stream) {
  return reinterpret_cast<hipStream_t>(stream);
}

constexpr uint32_t kMaxSeg = BITAR_HIP_MAX_SEG_SIZE;
constexpr uint32_t kMaxZstdFrame = 1u << 30;

// Calls whose kernels need per-segment scratch (dynamic DEFLATE and Zstd compress, Zstd
// decode) run in chunks of at most kChunkSegs segments (2 GiB of 64 KiB segments: every
// chunk still fills the chip many times over) over ONE scratch allocation sized for a chunk,
// so a call's scratch is bounded whatever its size.  Chunks are balanced (a 18059-segment
// call is one chunk, a 65536-segment call two of 32768).
constexpr uint64_t kChunkSegs = 32768;
struct Chunks {
  uint64_t size;
  explicit Chunks(uint64_t nseg) {
    const uint64_t k = (nseg + kChunkSegs - 1) / kChunkSegs;
    size = k ? (nseg + k - 1) / k : 1;
  }
};
// The device pool's cached stream-ordered memory above this is returned to the driver at
// the next synchronisation (a chunk of Zstd compress scratch is ~12 GB; steady-state calls
// stay below this and never touch the driver).
constexpr uint64_t kPoolKeepBytes = 24ull << 30;

// index of the error word of `stream`; words run out only after 1000+ distinct foreign
// streams, after which they share the NULL stream's word (still correct, merely coarser)
uint32_t word_index(bitar_hip_ctx* ctx, hipStream_t stream) {
  if (!stream) return 0;
  for (uint32_t q = 0; q < ctx->streams.size(); ++q)
    if (ctx->streams[q] == stream) return q + 1;
  std::lock_guard<std::mutex> g(ctx->mu);
  for (auto& w : ctx->words)
    if (w.first == stream) return w.second;
  const uint32_t next = (uint32_t)(ctx->streams.size() + 1 + ctx->words.size());
  if (next >= kErrWords) return 0;
  ctx->words.emplace_back(stream, next);
  return next;
}

uint32_t* err_word(bitar_hip_ctx* ctx, hipStream_t stream) {
  return ctx->d_err + word_index(ctx, stream);
}

int sync_error(uint32_t err) {
  if (!err) return 0;
  if (err & 2u) return fail(BITAR_HIP_IO_ERROR, "Compress data output is larger than allocated buffer");
  if (err & 4u) return fail(BITAR_HIP_IO_ERROR, "pack: a segment's size exceeds its slot (failed op)");
  return fail(BITAR_HIP_IO_ERROR, "Some operations have failed");
}

}  // namespace

static void init_options(bitar_hip_ctx* ctx, uint32_t flags);
static void free_order_scratch(bitar_hip_ctx* ctx);

extern "C" {

int bitar_hip_abi_version(void) { return BITAR_HIP_ABI_VERSION; }

const char* bitar_hip_last_error(void) { return g_last_error.c_str(); }

int bitar_hip_device_count(int* count) {
  if (!count) return fail(BITAR_HIP_INVALID, "null count");
  *count = 0;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e == hipErrorNoDevice || n == 0) return 0;
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  int gfx950 = 0;
  for (int d = 0; d < n; ++d) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) == hipSuccess &&
        std::strncmp(prop.gcnArchName, "gfx950", 6) == 0)
      ++gfx950;
  }
  *count = gfx950;
  return 0;
}

int bitar_hip_open(int device, const bitar_hip_config* cfg, bitar_hip_ctx** out) {
  if (!out) return fail(BITAR_HIP_INVALID, "null out");
  *out = nullptr;
  const uint32_t nstreams = cfg && cfg->num_streams ? cfg->num_streams : 1;
  if (nstreams > 64) return fail(BITAR_HIP_INVALID, "num_streams must be in [1, 64]");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (device < 0 || device >= n) return fail(BITAR_HIP_INVALID, "no such device");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(BITAR_HIP_NOT_IMPLEMENTED,
                std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950");
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  auto* ctx = new bitar_hip_ctx();
  ctx->device = device;
  for (uint32_t q = 0; q < nstreams; ++q) {
    hipStream_t s;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess) {
      bitar_hip_close(ctx);
      return hip_fail(e, "hipStreamCreate");
    }
    ctx->streams.push_back(s);
  }
  // stream-ordered scratch (dynamic-Huffman DEFLATE) comes from the device's default pool;
  // keep its memory cached between calls instead of returning it at every sync
  {
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
      uint64_t keep = kPoolKeepBytes;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
    (void)hipGetLastError();
  }
  init_options(ctx, cfg ? cfg->flags : 0u);
  hipError_t e = hipMalloc(&ctx->d_err, kErrWords * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(ctx->d_err, 0, kErrWords * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&ctx->d_stats, BITAR_HIP_PATH_COUNT * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(ctx->d_stats, 0, BITAR_HIP_PATH_COUNT * sizeof(unsigned long long));
  if (e != hipSuccess) {
    bitar_hip_close(ctx);
    return hip_fail(e, "error word");
  }
  *out = ctx;
  return 0;
}

int bitar_hip_close(bitar_hip_ctx* ctx) {
  if (!ctx) return 0;
  if (hipSetDevice(ctx->device) == hipSuccess) {
    for (auto s : ctx->streams) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
    (void)hipDeviceSynchronize();  // (order scratch may sit on foreign streams)
    free_order_scratch(ctx);
    for (auto& cs : ctx->copy_streams) (void)hipStreamDestroy(cs.second);
    ctx->copy_streams.clear();
    for (auto& cs : ctx->aux_streams) (void)hipStreamDestroy(cs.second);
    ctx->aux_streams.clear();
    if (ctx->d_err) (void)hipFree(ctx->d_err);
    if (ctx->d_stats) (void)hipFree(ctx->d_stats);
  }
  delete ctx;
  return 0;
}

int bitar_hip_stream(bitar_hip_ctx* ctx, uint32_t qp, void** stream) {
  if (!ctx || !stream) return fail(BITAR_HIP_INVALID, "null argument");
  if (qp >= ctx->streams.size()) return fail(BITAR_HIP_INVALID, "queue pair out of range");
  *stream = ctx->streams[qp];
  return 0;
}

int bitar_hip_device(bitar_hip_ctx* ctx, int* device) {
  if (!ctx || !device) return fail(BITAR_HIP_INVALID, "null argument");
  *device = ctx->device;
  return 0;
}

uint64_t bitar_hip_slot_size(uint32_t codec, uint32_t seg) {
  uint64_t bound;
  if (codec == BITAR_HIP_CODEC_LZ4 || codec == BITAR_HIP_CODEC_LZ4_WIDE)
    bound = (uint64_t)seg + seg / 255u + 16u;           // LZ4_compressBound
  else if (codec == BITAR_HIP_CODEC_DEFLATE || codec == BITAR_HIP_CODEC_DEFLATE_DYNAMIC)
    bound = ((uint64_t)seg * 9 + 7) / 8 + 16u;          // fixed Huffman, 9 bits/literal
  else if (codec == BITAR_HIP_CODEC_ZSTD)  // oracle bo_zstd_bound: one block, raw if larger
    bound = (uint64_t)seg + 7u + 3u + 8u + 512u;
  else
    return 0;
  return (bound + 255u) & ~(uint64_t)255u;
}

uint32_t bitar_hip_max_distance(uint32_t codec) {
  // the window-scan parse verifies candidates in its LDS input ring, which runs up to 1536 B
  // ahead of the scan: a 4 KiB ring (window_parse.hip.h kMaxDist) for the fast parses of LZ4,
  // DEFLATE and Zstd, a 16 KiB ring for the wide LZ4 parse (compress.hip, lz4_wide)
  switch (codec) {
    case BITAR_HIP_CODEC_LZ4:
    case BITAR_HIP_CODEC_DEFLATE:
    case BITAR_HIP_CODEC_DEFLATE_DYNAMIC:
    case BITAR_HIP_CODEC_ZSTD: return 4096u - 1536u;
    case BITAR_HIP_CODEC_LZ4_WIDE: return 16384u - 1536u;
    default: return 0;
  }
}

int bitar_hip_alloc(bitar_hip_ctx* ctx, uint64_t bytes, void** ptr) {
  if (int r = enter(ctx)) return r;
  if (!ptr) return fail(BITAR_HIP_INVALID, "null ptr");
  HIP_TRY(hipMalloc(ptr, bytes ? bytes : 1), "hipMalloc");
  return 0;
}

int bitar_hip_free(bitar_hip_ctx* ctx, void* ptr) {
  if (int r = enter(ctx)) return r;
  HIP_TRY(hipFree(ptr), "hipFree");
  return 0;
}

int bitar_hip_host_alloc(bitar_hip_ctx* ctx, uint64_t bytes, void** ptr) {
  if (int r = enter(ctx)) return r;
  if (!ptr) return fail(BITAR_HIP_INVALID, "null ptr");
  HIP_TRY(hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault), "hipHostMalloc");
  return 0;
}

int bitar_hip_host_free(bitar_hip_ctx* ctx, void* ptr) {
  if (int r = enter(ctx)) return r;
  HIP_TRY(hipHostFree(ptr), "hipHostFree");
  return 0;
}

int bitar_hip_memcpy(bitar_hip_ctx* ctx, void* dst, const void* src, uint64_t bytes,
                     void* stream) {
  if (int r = enter(ctx)) return r;
  if (!bytes) return 0;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, pick_stream(ctx, stream)),
          "hipMemcpyAsync");
  return 0;
}

// Cost-ordered dispatch (util_kernels.hip, seg_order_kernel): a launch of one wave per segment
// ends with a drain of about one segment's duration, longest when expensive segments come
// last.  For calls of at least kOrderMinSegs segments the LZ4 kernels take their segments in
// the order of an estimated cost key, most expensive first.  Measured (1 GiB, kind 1 = 1 MiB
// regions of columns / text / random data): see DESIGN.md 4.1.
extern "C++" {
constexpr uint32_t kOrderMinSegs = 2048;
struct SegOrder {
  bitar_hip_ctx::OrderScratch* e = nullptr;
  std::unique_lock<std::mutex> held;
  void* transient = nullptr;  // a foreign stream's scratch (freed by release(), stream-ordered)
  hipStream_t tstream = nullptr;
  uint32_t* order = nullptr;  // null: plain order
  // order = argsort of the keys: keys[i] written by `key` (a launch), or -- csizes given --
  // the compressed sizes' key computed by the sort itself (decompress; seg: the segment size).
  // slot: which of the stream's cached scratch areas (a call holding two orders at once
  // uses slots 0 and 1).  The scratch is allocated once per stream and grown on demand, so
  // steady-state calls queue no allocation.
  template <class F>
  int make(bitar_hip_ctx* ctx, hipStream_t s, uint32_t nseg, const uint32_t* csizes, F key,
           uint32_t seg = 0, int slot = 0) {
    if (!ctx->cost_order.load(std::memory_order_relaxed) || nseg < kOrderMinSegs) return 0;
    const uint32_t tile = bitar_hip::order_tile(nseg);
    const uint32_t ntiles = (nseg + tile - 1) / tile;
    const uint64_t need = 8ull * nseg + 4ull * bitar_hip::kOrderBins * ntiles + 64;
    bool own = s == nullptr;
    for (hipStream_t q : ctx->streams) own = own || q == s;
    if (!own) {
      // a foreign stream (e.g. a torch side stream): no cache entry, which would pin HBM for
      // the context's life and be inherited by a later stream reusing the handle -- the
      // scratch is allocated and freed in this stream's order by this call
      if (hipMallocAsync(&transient, need, s) != hipSuccess) {
        (void)hipGetLastError();
        transient = nullptr;
        return 0;  // (an optimisation only: the call runs in plain order)
      }
      tstream = s;
    } else {
      {
        std::lock_guard<std::mutex> g(ctx->mu);
        for (auto& x : ctx->order_scratch)
          if (x.stream == s && x.slot == slot) e = &x;
        if (!e) e = &ctx->order_scratch.emplace_back(s, slot);
      }
      held = std::unique_lock<std::mutex>(e->m);
      if (e->cap < need) {
        // (an optimisation only: without scratch the call runs in plain order)
        if (e->p) (void)hipFreeAsync(e->p, s);
        e->p = nullptr;
        e->cap = 0;
        const uint64_t cap = (need + (1u << 20) - 1) & ~(uint64_t)((1u << 20) - 1);
        if (hipMallocAsync(&e->p, cap, s) != hipSuccess) {
          (void)hipGetLastError();
          e->p = nullptr;
          held.unlock();
          return 0;
        }
        e->cap = cap;
      }
    }
    order = static_cast<uint32_t*>(transient ? transient : e->p);
    uint32_t* keys = csizes ? nullptr : order + nseg;
    auto* hist = reinterpret_cast<uint32_t*>(
        (reinterpret_cast<uintptr_t>(order + 2ull * nseg) + 15) & ~(uintptr_t)15);
    if (keys) key(keys);
    hipLaunchKernelGGL(bitar_hip::order_hist_kernel, dim3(ntiles), dim3(64), 0, s, keys, csizes,
                       seg, nseg, tile, hist);
    hipLaunchKernelGGL(bitar_hip::order_scatter_kernel, dim3(ntiles), dim3(64), 0, s, keys,
                       csizes, seg, nseg, tile, ntiles, hist, order);
    return 0;
  }
  // after the last launch that reads the order has been queued
  int release() {
    if (held.owns_lock()) held.unlock();
    if (transient) (void)hipFreeAsync(transient, tstream);
    transient = nullptr;
    return 0;
  }
  ~SegOrder() { release(); }
};

// the context's cached order scratch, freed at close (after its streams are idle)
static void free_order_scratch(bitar_hip_ctx* ctx) {
  std::lock_guard<std::mutex> g(ctx->mu);
  for (auto& x : ctx->order_scratch)
    if (x.p) (void)hipFree(x.p);
  ctx->order_scratch.clear();
}
}  // extern "C++"

static int compress_impl(bitar_hip_ctx* ctx, void* stream, uint32_t codec, const void* d_in,
                         uint64_t n, uint32_t seg, void* d_slab, uint64_t slot_stride,
                         void* const* d_dsts, uint32_t* d_sizes) {
  if (int r = enter(ctx)) return r;
  if (codec != BITAR_HIP_CODEC_LZ4 && codec != BITAR_HIP_CODEC_DEFLATE &&
      codec != BITAR_HIP_CODEC_ZSTD && codec != BITAR_HIP_CODEC_DEFLATE_DYNAMIC &&
      codec != BITAR_HIP_CODEC_LZ4_WIDE)
    return fail(BITAR_HIP_NOT_IMPLEMENTED, "unknown codec");
  if (seg == 0 || seg > kMaxSeg) return fail(BITAR_HIP_INVALID, "seg must be in [1, 65536]");
  if (n == 0) return 0;  // empty input -> no segments (reference device.cc:161-164)
  if (!d_in || (!d_slab && !d_dsts) || !d_sizes) return fail(BITAR_HIP_INVALID, "null buffer");
  if (slot_stride < bitar_hip_slot_size(codec, seg))
    return fail(BITAR_HIP_INVALID, "slot size below the worst-case bound");
  if (d_slab && (((uintptr_t)d_slab & 15u) != 0 || (slot_stride & 15u) != 0))
    return fail(BITAR_HIP_INVALID, "d_slab and slot_stride must be 16-B aligned");
  const uint64_t nseg = (n + seg - 1) / seg;
  if (nseg > 0x7FFFFFFFull) return fail(BITAR_HIP_INVALID, "too many segments");
  hipStream_t s = pick_stream(ctx, stream);
  const auto* in = static_cast<const uint8_t*>(d_in);
  auto* slab = static_cast<uint8_t*>(d_slab);
  auto* dsts = reinterpret_cast<uint8_t* const*>(d_dsts);
  // cost-ordered dispatch of the segments of [cin, cin + nb): key = distinct byte values in
  // a 128-byte sample of each segment (incompressible segments, which the parses skip
  // through and whose stored form is a copy, show the most)
  auto cost_order = [&](SegOrder& o, const uint8_t* cin, uint64_t nb, uint32_t cn) {
    return o.make(ctx, s, cn, nullptr, [&](uint32_t* keys) {
      hipLaunchKernelGGL(bitar_hip::seg_cost_kernel, dim3((cn + 15) / 16), dim3(64), 0, s,
                         cin, nb, seg, cn, keys);
    });
  };
  if (codec == BITAR_HIP_CODEC_LZ4 || codec == BITAR_HIP_CODEC_LZ4_WIDE) {
    SegOrder ord;
    if (int r = cost_order(ord, in, n, (uint32_t)nseg)) return r;
    if (codec == BITAR_HIP_CODEC_LZ4)
      hipLaunchKernelGGL((bitar_hip::lz4_compress_kernel<4096, 10>), dim3((uint32_t)nseg),
                         dim3(64), 0, s, in, n, seg, slab, slot_stride, dsts, d_sizes,
                         err_word(ctx, s), ord.order);
    else
      hipLaunchKernelGGL((bitar_hip::lz4_compress_kernel<16384, 12>), dim3((uint32_t)nseg),
                         dim3(64), 0, s, in, n, seg, slab, slot_stride, dsts, d_sizes,
                         err_word(ctx, s), ord.order);
    if (int r = ord.release()) return r;
  }
  else if (codec == BITAR_HIP_CODEC_DEFLATE) {
    SegOrder ord;
    if (int r = cost_order(ord, in, n, (uint32_t)nseg)) return r;
    hipLaunchKernelGGL(bitar_hip::deflate_compress_kernel, dim3((uint32_t)nseg), dim3(64), 0, s,
                       in, n, seg, slab, slot_stride, dsts, d_sizes, err_word(ctx, s), ord.order);
    if (int r = ord.release()) return r;
  }
  else if (codec == BITAR_HIP_CODEC_DEFLATE_DYNAMIC) {
    // pass 1 (parse -> records + histograms) and pass 2 (codes + emit) through a
    // stream-ordered scratch per segment (deflate_dyn.hip): 2 KiB plan + the literal stream
    // (<= seg bytes, 16-B aligned) + 8-byte match records (<= seg / 4: matches are >= 4
    // bytes); the per-window form (BITAR_DYN_BULK 0) needs 2 KiB + 16 KiB of window masks +
    // 4-byte records, within the same stride.  Large calls run in chunks of <= kChunkSegs
    // segments over one scratch allocation, so scratch is bounded whatever the call's size.
    const uint64_t scr_old = bitar_hip_slot_size(BITAR_HIP_CODEC_DEFLATE, seg) + 2048u + 16384u;
    const uint64_t scr_bulk = 2048u + ((seg + 15u) & ~15ull) + 8u * ((uint64_t)seg / 4u + 64u);
    const uint64_t scr_stride = ((scr_old > scr_bulk ? scr_old : scr_bulk) + 15u) & ~15ull;
    const Chunks ch(nseg);
    void* scratch = nullptr;
    HIP_TRY(hipMallocAsync(&scratch, ch.size * scr_stride, s), "scratch allocation");
    auto* scr = static_cast<uint8_t*>(scratch);
    for (uint64_t c0 = 0; c0 < nseg; c0 += ch.size) {
      const uint64_t cn = nseg - c0 < ch.size ? nseg - c0 : ch.size;
      const uint64_t cb = c0 * seg, nb = n - cb < cn * seg ? n - cb : cn * seg;
      uint8_t* cslab = slab ? slab + c0 * slot_stride : nullptr;
      uint8_t* const* cdsts = dsts ? dsts + c0 : nullptr;
      SegOrder ord;
      if (int r = cost_order(ord, in + cb, nb, (uint32_t)cn)) return r;
      hipLaunchKernelGGL(bitar_hip::deflate_dyn_parse_kernel, dim3((uint32_t)cn), dim3(64), 0, s,
                         in + cb, nb, seg, scr, scr_stride, err_word(ctx, s), ord.order);
      hipLaunchKernelGGL(bitar_hip::deflate_dyn_emit_kernel, dim3((uint32_t)cn), dim3(64), 0, s,
                         in + cb, nb, seg, static_cast<const uint8_t*>(scr), scr_stride, cslab,
                         slot_stride, cdsts, d_sizes + c0, err_word(ctx, s), ord.order);
      if (int r = ord.release()) return r;
    }
    const hipError_t le = hipGetLastError();
    HIP_TRY(hipFreeAsync(scratch, s), "scratch release");
    HIP_TRY(le, "compress launch");
  }
  else {
    // pass 1 (parse -> literals + sequence records) and pass 2 (entropy coding) through a
    // stream-ordered scratch: per segment the literal area + records (zstd_compress.hip),
    // then {nlit, nseq} per segment
    const uint64_t scr_stride = bitar_hip::zse::scratch_stride(seg);
    // + the chain-walk scratch (zstd_layout.hip.h: a 5000-byte header with the record, the
    // literal codes and the FSE tables, then 10 bytes per sequence and 12 per step of <= 64)
    const uint64_t w_stride = bitar_hip::zse::walk_stride(seg);
    const Chunks ch(nseg);
    void* scratch = nullptr;
    HIP_TRY(hipMallocAsync(&scratch, ch.size * (scr_stride + 8u + w_stride), s),
            "scratch allocation");
    auto* scr = static_cast<uint8_t*>(scratch);
    auto* meta = reinterpret_cast<uint2*>(scr + ch.size * scr_stride);
    auto* wscr = scr + ch.size * scr_stride + ch.size * 8u;
    for (uint64_t c0 = 0; c0 < nseg; c0 += ch.size) {
      const uint64_t cn = nseg - c0 < ch.size ? nseg - c0 : ch.size;
      const uint64_t cb = c0 * seg, nb = n - cb < cn * seg ? n - cb : cn * seg;
      uint8_t* cslab = slab ? slab + c0 * slot_stride : nullptr;
      uint8_t* const* cdsts = dsts ? dsts + c0 : nullptr;
      const uint8_t* cin = in + cb;
      SegOrder ord;
      if (int r = cost_order(ord, cin, nb, (uint32_t)cn)) return r;
      hipLaunchKernelGGL(bitar_hip::zstd_parse_kernel, dim3((uint32_t)cn), dim3(64), 0, s, cin,
                         nb, seg, scr, scr_stride, meta, ord.order);
      hipLaunchKernelGGL(bitar_hip::zstd_entropy_kernel, dim3((uint32_t)cn), dim3(64), 0, s, cin,
                         nb, seg, scr, scr_stride, meta, wscr, w_stride, ord.order);
      SegOrder word;  // (the walk's order: sequence counts, most first)
      if (int r = word.make(ctx, s, (uint32_t)cn, nullptr, [&](uint32_t* keys) {
            hipLaunchKernelGGL(bitar_hip::walk_key_kernel, dim3((uint32_t)((cn + 63) / 64)),
                               dim3(64), 0, s, meta, (uint32_t)cn, keys);
          }, 0, 1))
        return r;
      hipLaunchKernelGGL(bitar_hip::zstd_walk_kernel, dim3((uint32_t)((cn + 3) / 4)), dim3(64),
                         0, s, scr, scr_stride, seg, (uint32_t)cn, wscr, w_stride, word.order);
      if (int r = word.release()) return r;
      hipLaunchKernelGGL(bitar_hip::zstd_emit_kernel, dim3((uint32_t)cn), dim3(64), 0, s, cin, nb,
                         seg, scr, scr_stride, cslab, slot_stride, cdsts, d_sizes + c0, wscr,
                         w_stride, ord.order);
      if (int r = ord.release()) return r;
    }
    const hipError_t le = hipGetLastError();
    HIP_TRY(hipFreeAsync(scratch, s), "scratch release");
    HIP_TRY(le, "compress launch");
  }
  HIP_TRY(hipGetLastError(), "compress launch");
  return 0;
}

int bitar_hip_compress(bitar_hip_ctx* ctx, void* stream, uint32_t codec, const void* d_in,
                       uint64_t n, uint32_t seg, void* d_slab, uint64_t slot_stride,
                       uint32_t* d_sizes) {
  if (n && !d_slab) return fail(BITAR_HIP_INVALID, "null d_slab");
  return compress_impl(ctx, stream, codec, d_in, n, seg, d_slab, slot_stride, nullptr, d_sizes);
}

int bitar_hip_compress_scattered(bitar_hip_ctx* ctx, void* stream, uint32_t codec,
                                 const void* d_in, uint64_t n, uint32_t seg,
                                 void* const* d_dsts, uint64_t slot_capacity, uint32_t* d_sizes) {
  if (n && !d_dsts) return fail(BITAR_HIP_INVALID, "null d_dsts");
  return compress_impl(ctx, stream, codec, d_in, n, seg, nullptr, slot_capacity, d_dsts,
                       d_sizes);
}

int bitar_hip_pointer_info(const void* ptr, int* kind, int* device) {
  if (!kind || !device) return fail(BITAR_HIP_INVALID, "null argument");
  *kind = 0;
  *device = -1;
  if (!ptr) return 0;
  hipPointerAttribute_t a;
  hipError_t e = hipPointerGetAttributes(&a, ptr);
  if (e != hipSuccess) {  // unknown to HIP: ordinary pageable host memory
    (void)hipGetLastError();
    return 0;
  }
  if (a.type == hipMemoryTypeDevice) {
    *kind = 2;
    *device = a.device;
  } else if (a.type == hipMemoryTypeHost && a.devicePointer == ptr) {
    // pinned host memory the device reaches at the same address (hipHostMalloc, torch
    // pin_memory): kernels may read it in place.  Memory pinned by hipHostRegister can have
    // another device address; it is reported as pageable (kind 0), so callers stage it with a
    // copy (hipMemcpyDefault) instead of handing its host address to a kernel.
    *kind = 1;
    *device = a.device;
  }
  return 0;
}

// Decoder options: per context (bitar_hip_decoder_options).  The environment variables
// BITAR_HIP_INFLATE_LANES / BITAR_HIP_ZSTD_LANES / BITAR_HIP_ZSTD_SEQ (tuning runs) set the
// defaults a context starts from; cfg->flags override them at open.
static uint32_t zstd_lanes_from(long x) {
  return x <= 0 ? 0u : x >= 64 ? 64u : x >= 32 ? 32u : x >= 16 ? 16u : 8u;
}
static uint32_t inflate_lanes_from(long x) {
  return x <= 0 ? 0u : x >= 32 ? 32u : x >= 16 ? 16u : x >= 8 ? 8u : 4u;
}
static long env_long(const char* name, long dflt) {
  const char* e = std::getenv(name);
  return e ? std::strtol(e, nullptr, 10) : dflt;
}

// Zstd: zstd_hlit_kernel on a stream of its own, beside zstd_seqdec_kernel (both latency-bound
// with about one wave per SIMD, and independent: the sequences need no literal).  Per
// context: BITAR_HIP_FLAG_ZSTD_SERIAL (or BITAR_HIP_ZSTD_FORK=0) queues them one after the
// other; BITAR_HIP_ZSTD_FORK=2 (timing runs) puts phase A on the side stream instead.
static uint32_t zstd_fork_env() {
  static const uint32_t v = (uint32_t)env_long("BITAR_HIP_ZSTD_FORK", 1);
  return v > 2 ? 1u : v;
}

static void init_options(bitar_hip_ctx* ctx, uint32_t flags) {
  // The lane inflater in front of the wave inflater is off by default since the wave
  // inflater's batches take far matches (round 3): 1 GiB fixed-Huffman decode, wave alone vs
  // 4 lanes per wave in front: kind 1 11.6 / 14.1 ms, kind 2 12.4 / 17.6, kind 5 13.3 / 12.6,
  // kind 6 11.7 / 8.9 (the lanes win long-match data only; splitting segments between the
  // two by compression ratio was slower than either: the launches run one after the other).
  // Dynamic blocks always take the wave inflater.  inflate_lanes = 4 keeps the lane form.
  ctx->inflate_lanes = flags & BITAR_HIP_FLAG_INFLATE_WAVE_ONLY
                           ? 0u : inflate_lanes_from(env_long("BITAR_HIP_INFLATE_LANES", 0));
  ctx->zstd_lanes = flags & BITAR_HIP_FLAG_ZSTD_WAVE_ONLY
                        ? 0u : zstd_lanes_from(env_long("BITAR_HIP_ZSTD_LANES", 16));
  ctx->zstd_seq = flags & BITAR_HIP_FLAG_ZSTD_LANE_EXEC ? 0u : env_long("BITAR_HIP_ZSTD_SEQ", 1) != 0;
  ctx->zstd_fork = flags & BITAR_HIP_FLAG_ZSTD_SERIAL ? 0u : zstd_fork_env();
  ctx->count_paths = (flags & BITAR_HIP_FLAG_COUNT_PATHS) ? 1u : 0u;
  ctx->cost_order = (flags & BITAR_HIP_FLAG_PLAIN_ORDER) ? 0u : env_long("BITAR_HIP_COST_ORDER", 1) != 0;
}

// the counters' device pointer for a launch, null (= not counted) unless count_paths is on
static unsigned long long* stats_of(bitar_hip_ctx* ctx) {
  return ctx->count_paths.load(std::memory_order_relaxed) ? ctx->d_stats : nullptr;
}

extern "C" int bitar_hip_get_decoder_options(bitar_hip_ctx* ctx, bitar_hip_decoder_options* opt) {
  if (!ctx || !opt) return fail(BITAR_HIP_INVALID, "null argument");
  opt->inflate_lanes = ctx->inflate_lanes.load();
  opt->zstd_lanes = ctx->zstd_lanes.load();
  opt->zstd_seq = ctx->zstd_seq.load();
  opt->count_paths = ctx->count_paths.load();
  return 0;
}

extern "C" int bitar_hip_set_decoder_options(bitar_hip_ctx* ctx,
                                             const bitar_hip_decoder_options* opt) {
  if (!ctx || !opt) return fail(BITAR_HIP_INVALID, "null argument");
  ctx->inflate_lanes = inflate_lanes_from((long)opt->inflate_lanes);
  ctx->zstd_lanes = zstd_lanes_from((long)opt->zstd_lanes);
  ctx->zstd_seq = opt->zstd_seq ? 1u : 0u;
  ctx->count_paths = opt->count_paths ? 1u : 0u;
  return 0;
}

extern "C" int bitar_hip_path_counters(bitar_hip_ctx* ctx, uint64_t* out, uint32_t n) {
  if (int r = enter(ctx)) return r;
  if (!out && n) return fail(BITAR_HIP_INVALID, "null out");
  HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
  unsigned long long v[BITAR_HIP_PATH_COUNT];
  HIP_TRY(hipMemcpy(v, ctx->d_stats, sizeof(v), hipMemcpyDeviceToHost), "read path counters");
  HIP_TRY(hipMemset(ctx->d_stats, 0, sizeof(v)), "reset path counters");
  for (uint32_t k = 0; k < n && k < BITAR_HIP_PATH_COUNT; ++k) out[k] = v[k];
  return 0;
}

// segments per wave of zstd_hlit_kernel / zstd_handoff_kernel / zstd_seqdec_kernel (4 / 8 /
// 16): tuning knobs BITAR_HIP_HLIT_SEGS, BITAR_HIP_HANDOFF_LANES, BITAR_HIP_SEQDEC_SEGS, read once
static uint32_t pow2_knob(const char* name, uint32_t dflt) {
  const long x = env_long(name, (long)dflt);
  return x >= 16 ? 16u : x >= 8 ? 8u : 4u;
}
static uint32_t hlit_segs() {
  static const uint32_t v = pow2_knob("BITAR_HIP_HLIT_SEGS", 16);
  return v;
}
// (tuning knob: 1 puts the forked single-block literal kernel on the side stream after the
// multi-block one instead of on the caller's stream after phase A)
#ifndef BITAR_HLIT1_SIDE
#define BITAR_HLIT1_SIDE 0
#endif
static uint32_t seqdec_segs() {
  static const uint32_t v = pow2_knob("BITAR_HIP_SEQDEC_SEGS", 16);
  return v;
}
static uint32_t handoff_lanes() {
  static const uint32_t v = pow2_knob("BITAR_HIP_HANDOFF_LANES", 16);
  return v;
}

// the stream paired with the caller's stream s in `list` (created on first use; null if that
// fails)
static hipStream_t side_stream_for(bitar_hip_ctx* ctx,
                                   std::vector<std::pair<hipStream_t, hipStream_t>>& list,
                                   hipStream_t s) {
  std::lock_guard<std::mutex> g(ctx->mu);
  for (auto& cs : list)
    if (cs.first == s) return cs.second;
  hipStream_t c = nullptr;
  if (hipStreamCreateWithFlags(&c, hipStreamNonBlocking) != hipSuccess) return nullptr;
  list.emplace_back(s, c);
  return c;
}
static int stream_after(hipStream_t b, hipStream_t a);


static int decompress_impl(bitar_hip_ctx* ctx, void* stream, uint32_t codec,
                           const void* const* d_srcs, const void* d_slab, uint64_t stride,
                           const uint32_t* d_sizes, uint32_t nseg, uint32_t seg, void* d_out,
                           uint64_t capacity, uint32_t* d_produced) {
  if (int r = enter(ctx)) return r;
  // the caller's FIXED hint picks the inflater built for fixed-Huffman streams (9 / 8-bit
  // fast tables, more waves per CU; any stream still decodes, inflate_fixed.hip)
  const bool fixed_hint = codec == BITAR_HIP_CODEC_DEFLATE;
  if (codec == BITAR_HIP_CODEC_DEFLATE_DYNAMIC) codec = BITAR_HIP_CODEC_DEFLATE;  // same format
  if (codec == BITAR_HIP_CODEC_LZ4_WIDE) codec = BITAR_HIP_CODEC_LZ4;              // same format
  if (codec != BITAR_HIP_CODEC_LZ4 && codec != BITAR_HIP_CODEC_DEFLATE &&
      codec != BITAR_HIP_CODEC_ZSTD)
    return fail(BITAR_HIP_NOT_IMPLEMENTED, "unknown codec");
  if (nseg == 0) return 0;  // reference device.cc:244-246
  // Zstd: a segment may be a whole stock frame of up to kMaxZstdFrame bytes (the wave
  // decoder reads far history from HBM; the Arrow adapter decodes stock IPC bodies so)
  const uint32_t max_seg = codec == BITAR_HIP_CODEC_ZSTD ? kMaxZstdFrame : kMaxSeg;
  if (seg == 0 || seg > max_seg)
    return fail(BITAR_HIP_INVALID, "seg must be in [1, " + std::to_string(max_seg) + "]");
  if (capacity < (uint64_t)nseg * seg)  // reference device.cc:248-254
    return fail(BITAR_HIP_CAPACITY_ERROR,
                "The decompressed_buffer is required to be >= " +
                    std::to_string((uint64_t)nseg * seg) + " bytes");
  if (!d_sizes || !d_out || !d_produced || (!d_srcs && !d_slab))
    return fail(BITAR_HIP_INVALID, "null buffer");
  if (nseg > 0x7FFFFFFFu) return fail(BITAR_HIP_INVALID, "too many segments");
  hipStream_t s = pick_stream(ctx, stream);
  unsigned long long* const stats = stats_of(ctx);
  const auto* srcs = reinterpret_cast<const uint8_t* const*>(d_srcs);
  const auto* slab = static_cast<const uint8_t*>(d_slab);
  auto* out = static_cast<uint8_t*>(d_out);
  if (codec == BITAR_HIP_CODEC_LZ4)
  {
    // near-history kernel over every segment, then the far-history kernel over the segments
    // it deferred (lz4_decompress.hip)
    // cost key: the coded size, largest first; incompressible segments (copies) last
    SegOrder ord;
    if (int r = ord.make(ctx, s, nseg, d_sizes, [](uint32_t*) {}, seg)) return r;
    hipLaunchKernelGGL(bitar_hip::lz4_decompress_kernel<false>, dim3(nseg), dim3(64), 0, s, srcs,
                       slab, stride, d_sizes, nseg, seg, out, d_produced, err_word(ctx, s),
                       stats, ord.order);
    hipLaunchKernelGGL(bitar_hip::lz4_decompress_kernel<true>, dim3(nseg), dim3(64), 0, s, srcs,
                       slab, stride, d_sizes, nseg, seg, out, d_produced, err_word(ctx, s),
                       stats, ord.order);
    if (int r = ord.release()) return r;
  }
  else if (codec == BITAR_HIP_CODEC_DEFLATE) {
    // lane-per-segment decoder for stored / fixed-Huffman streams first; the wave decoder
    // then takes the segments it deferred (inflate_lanes.hip)
    const uint32_t L = ctx->inflate_lanes.load(std::memory_order_relaxed);
    if (L) {
      const dim3 g((nseg + L - 1) / L);
#define BITAR_INFL_LANES(N)                                                                  \
  hipLaunchKernelGGL(bitar_hip::inflate_lanes_kernel<N>, g, dim3(64), 0, s, srcs, slab, stride, \
                     d_sizes, nseg, seg, out, d_produced)
      if (L == 32) BITAR_INFL_LANES(32);
      else if (L == 16) BITAR_INFL_LANES(16);
      else if (L == 8) BITAR_INFL_LANES(8);
      else BITAR_INFL_LANES(4);
#undef BITAR_INFL_LANES
    }
    SegOrder ord;
    if (int r = ord.make(ctx, s, nseg, d_sizes, [](uint32_t*) {}, seg)) return r;
    hipLaunchKernelGGL(fixed_hint ? bitar_hip::inflate_fixed_kernel : bitar_hip::inflate_kernel,
                       dim3(nseg), dim3(64), 0, s, srcs, slab, stride, d_sizes, nseg, seg, out,
                       d_produced, err_word(ctx, s), L ? 1u : 0u, stats, ord.order);
    if (int r = ord.release()) return r;
  }
  else {
    // lane-per-segment decoder first; the wave-per-segment decoder then takes the segments it
    // deferred (zstd_lanes.hip)
    const uint32_t L = ctx->zstd_lanes.load(std::memory_order_relaxed);
    if (L) {
      const dim3 g((nseg + L - 1) / L);
      if (L == 64)
        hipLaunchKernelGGL(bitar_hip::zstd_lanes_kernel<64>, g, dim3(64), 0, s, srcs, slab,
                           stride, d_sizes, nseg, seg, out, d_produced);
      else if (L == 32)
        hipLaunchKernelGGL(bitar_hip::zstd_lanes_kernel<32>, g, dim3(64), 0, s, srcs, slab,
                           stride, d_sizes, nseg, seg, out, d_produced);
      else if (L == 16)
        hipLaunchKernelGGL(bitar_hip::zstd_lanes_kernel<16>, g, dim3(64), 0, s, srcs, slab,
                           stride, d_sizes, nseg, seg, out, d_produced);
      else
        hipLaunchKernelGGL(bitar_hip::zstd_lanes_kernel<8>, g, dim3(64), 0, s, srcs, slab,
                           stride, d_sizes, nseg, seg, out, d_produced);
    }
    // The wave decoder hands the sequence sections of its frames' last blocks over through a
    // stream-ordered scratch (zstd_hand.hip.h: kStride bytes per segment); segments <= 64 KiB
    // then run FSE chains -> records (zstd_seqdec_kernel, rcap 8-byte records per segment)
    // -> output (zstd_exec_kernel), the rest the lane executor.  Both scratch buffers are
    // allocated before any kernel is queued, once, for a chunk of <= kChunkSegs segments.
    const Chunks ch(nseg);
    const bool seq = ctx->zstd_seq.load(std::memory_order_relaxed) && seg <= 65536;
    const uint32_t rcap = seg / 3 + 1;  // every valid frame (matches are >= 3 bytes)
    void* hscr = nullptr;
    void* recs = nullptr;
    HIP_TRY(hipMallocAsync(&hscr, ch.size * bitar_hip::zhand::kStride, s), "scratch allocation");
    if (seq) {
      const hipError_t e = hipMallocAsync(&recs, ch.size * rcap * 8, s);
      if (e != hipSuccess) {
        (void)hipFreeAsync(hscr, s);
        return hip_fail(e, "scratch allocation");
      }
    }
    uint8_t* hs = static_cast<uint8_t*>(hscr);
    auto* rp = static_cast<uint64_t*>(recs);
    uint32_t* ew = err_word(ctx, s);
    const uint32_t hs_n = hlit_segs(), ho_n = handoff_lanes(), sd = seqdec_segs();
    for (uint64_t c0 = 0; c0 < nseg; c0 += ch.size) {
      const uint32_t cn = (uint32_t)(nseg - c0 < ch.size ? nseg - c0 : ch.size);
      const uint8_t* const* csrcs = srcs ? srcs + c0 : nullptr;
      const uint8_t* cslab = slab ? slab + c0 * stride : nullptr;
      const uint32_t* csz = d_sizes + c0;
      uint8_t* cout = out + c0 * seg;
      uint32_t* cprod = d_produced + c0;
      SegOrder ord;  // (cost key: the compressed size; allocation failure = plain order)
      (void)ord.make(ctx, s, cn, csz, [](uint32_t*) {}, seg);
      // (multi-block hand-offs -- every block of this engine's frames -- need the two-phase
      // sequence path; the lane executor takes last blocks only)
      hipLaunchKernelGGL(bitar_hip::zstd_decompress_kernel, dim3(cn), dim3(64), 0, s, csrcs,
                         cslab, stride, csz, cn, seg, cout, cprod, ew, L ? 1u : 0u, hs, stats,
                         ord.order, seq ? 1u : 0u);
#define BITAR_ZSTD_TAIL(K, N)                                                                 \
  hipLaunchKernelGGL(bitar_hip::K<N>, dim3((cn + N - 1) / N), dim3(64), 0, s, csrcs, cslab, stride, \
                     csz, cn, seg, cout, cprod, hs, ew)
  // (the multi-block kernels (B > 1) take units of 4 blocks: 2 cn of them)
#define BITAR_HLIT(N, B, O)                                                                   \
  hipLaunchKernelGGL((bitar_hip::zstd_hlit_kernel<N, B>), dim3(((B > 1 ? 2 : 1) * cn + N - 1) / N), \
                     dim3(64), 0, s, csrcs, cslab, stride, csz, cn, seg, cout, cprod, hs, ew, O)
      // the literal streams beside the sequences' phase A: one of the two on the aux stream
      // (zstd_fork 1: the literals there, launched first; 2: phase A there, first)
      // the multi-block lane kernels take their segments most expensive first (by sequences /
      // by literals: the column types of a record batch alternate in runs of segments, and
      // index order would give whole CUs the same kind of segment)
      SegOrder oseq, olit;
      if (seq) {
        (void)oseq.make(ctx, s, 2 * cn, nullptr, [&](uint32_t* keys) {
          hipLaunchKernelGGL(bitar_hip::hand_key_kernel, dim3((2 * cn + 63) / 64), dim3(64), 0, s,
                             cprod, hs, cn, 0u, keys);
        }, 0, 1);
        (void)olit.make(ctx, s, 2 * cn, nullptr, [&](uint32_t* keys) {
          hipLaunchKernelGGL(bitar_hip::hand_key_kernel, dim3((2 * cn + 63) / 64), dim3(64), 0, s,
                             cprod, hs, cn, 1u, keys);
        }, 0, 2);
      }
      const uint32_t fork = seq ? ctx->zstd_fork.load(std::memory_order_relaxed) : 0u;
      hipStream_t a = fork ? side_stream_for(ctx, ctx->aux_streams, s) : nullptr;
      if (a && stream_after(a, s)) a = nullptr;
      // single-block hand-offs (16 segments x 4 streams / chains per wave) and, with the
      // two-phase path, the multi-block ones (4 segments x 4 blocks x 4 per wave).  Forked
      // (fork 1), the single-block literal kernel goes on the caller's stream after phase A:
      // ahead of the multi-block literals on the side stream, its 36 KiB workgroups -- which
      // exit at once on this engine's multi-block frames -- waited for CU room behind phase A,
      // and the multi-block literals behind them (1 GiB kind 2: 1.3 ms on the call's path).
      const bool split = a && fork == 1;
      auto hlit1 = [&](hipStream_t s) {
        if (hs_n == 4) BITAR_HLIT(4, 1, nullptr);
        else if (hs_n == 8) BITAR_HLIT(8, 1, nullptr);
        else BITAR_HLIT(16, 1, nullptr);
      };
      auto hlit = [&](hipStream_t s) {
        if (!split) hlit1(s);
        if (seq) BITAR_HLIT(4, 4, olit.order);
        if (split && BITAR_HLIT1_SIDE) hlit1(s);
      };
      auto seqdec = [&](hipStream_t s) {
#define BITAR_SEQDEC(N, B, O)                                                                 \
  hipLaunchKernelGGL((bitar_hip::zstd_seqdec_kernel<N, B>), dim3(((B > 1 ? 2 : 1) * cn + N - 1) / N), \
                     dim3(64), 0, s, csrcs, cslab, stride, csz, cn, seg, cprod, hs, rp, rcap, ew, \
                     stats, O)
        if (sd == 4) BITAR_SEQDEC(4, 1, nullptr);
        else if (sd == 8) BITAR_SEQDEC(8, 1, nullptr);
        else BITAR_SEQDEC(16, 1, nullptr);
        BITAR_SEQDEC(4, 4, oseq.order);
#undef BITAR_SEQDEC
      };
      if (a && fork == 2) {
        seqdec(a);
        hlit(s);
      } else {
        hlit(a ? a : s);
        if (seq) seqdec(s);
        if (split && !BITAR_HLIT1_SIDE) hlit1(s);
      }
      if (seq) {
        if (a && stream_after(s, a)) (void)hipStreamSynchronize(a);  // (join failed: wait here)
        hipLaunchKernelGGL(bitar_hip::zstd_exec_kernel, dim3(cn), dim3(64), 0, s, csrcs, cslab,
                           stride, cn, seg, cout, cprod, hs, rp, rcap, ew, stats, ord.order);
      }
      (void)ord.release();
      (void)oseq.release();
      (void)olit.release();
      if (ho_n == 4) BITAR_ZSTD_TAIL(zstd_handoff_kernel, 4);
      else if (ho_n == 8) BITAR_ZSTD_TAIL(zstd_handoff_kernel, 8);
      else BITAR_ZSTD_TAIL(zstd_handoff_kernel, 16);
#undef BITAR_ZSTD_TAIL
#undef BITAR_HLIT
    }
    const hipError_t le = hipGetLastError();
    if (recs) (void)hipFreeAsync(recs, s);
    HIP_TRY(hipFreeAsync(hscr, s), "scratch release");
    HIP_TRY(le, "decompress launch");
  }
  HIP_TRY(hipGetLastError(), "decompress launch");
  return 0;
}

int bitar_hip_decompress(bitar_hip_ctx* ctx, void* stream, uint32_t codec,
                         const void* const* d_srcs, const uint32_t* d_sizes, uint32_t nseg,
                         uint32_t seg, void* d_out, uint64_t capacity, uint32_t* d_produced) {
  if (nseg && !d_srcs) return fail(BITAR_HIP_INVALID, "null d_srcs");
  return decompress_impl(ctx, stream, codec, d_srcs, nullptr, 0, d_sizes, nseg, seg, d_out,
                         capacity, d_produced);
}

int bitar_hip_decompress_slab(bitar_hip_ctx* ctx, void* stream, uint32_t codec,
                              const void* d_slab, uint64_t slot_stride,
                              const uint32_t* d_sizes, uint32_t nseg, uint32_t seg,
                              void* d_out, uint64_t capacity, uint32_t* d_produced) {
  if (nseg && !d_slab) return fail(BITAR_HIP_INVALID, "null d_slab");
  return decompress_impl(ctx, stream, codec, nullptr, d_slab, slot_stride, d_sizes, nseg, seg,
                         d_out, capacity, d_produced);
}

// ---- host-memory calls: the PCIe link and the kernels overlapped ---------------------------
// The caller's stream s and a copy stream paired with it: the copy stream first waits for
// everything queued on s (the staging area may still be read by an earlier call), then per
// chunk of whole segments one copy + one event, and s waits on each chunk's event before the
// chunk's kernels (compress) -- or the copy stream waits on the chunk's decode before copying
// it out (decompress).  s finally waits on the copy stream, so a sync of s covers the call.
static hipStream_t copy_stream_for(bitar_hip_ctx* ctx, hipStream_t s) {
  return side_stream_for(ctx, ctx->copy_streams, s);
}

// b waits for what is queued on a now
static int stream_after(hipStream_t b, hipStream_t a) {
  hipEvent_t e;
  HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  hipError_t r = hipEventRecord(e, a);
  if (r == hipSuccess) r = hipStreamWaitEvent(b, e, 0);
  (void)hipEventDestroy(e);  // (released once recorded work completes)
  HIP_TRY(r, "stream ordering");
  return 0;
}

// chunks of whole segments: about 1/8 of the call, at least 32 MiB
static uint64_t host_chunk_segs(uint64_t nseg, uint32_t seg) {
  uint64_t c = (nseg + 7) / 8;
  const uint64_t lo = ((32ull << 20) + seg - 1) / seg;
  return c < lo ? lo : c;
}

int bitar_hip_compress_host(bitar_hip_ctx* ctx, void* stream, uint32_t codec, const void* h_in,
                            uint64_t n, uint32_t seg, void* d_stage, void* d_slab,
                            void* const* d_dsts, uint64_t slot_stride, uint32_t* d_sizes) {
  if (int r = enter(ctx)) return r;
  if (n == 0) return 0;
  if (!h_in || !d_stage || (!d_slab && !d_dsts) || !d_sizes)
    return fail(BITAR_HIP_INVALID, "null buffer");
  if (seg == 0 || seg > kMaxSeg) return fail(BITAR_HIP_INVALID, "seg must be in [1, 65536]");
  const hipStream_t s = pick_stream(ctx, stream);
  const hipStream_t c = copy_stream_for(ctx, s);
  if (!c) return fail(BITAR_HIP_UNKNOWN_ERROR, "copy stream");
  if (int r = stream_after(c, s)) return r;
  const uint64_t nseg = (n + seg - 1) / seg, per = host_chunk_segs(nseg, seg);
  auto* stage = static_cast<uint8_t*>(d_stage);
  const auto* src = static_cast<const uint8_t*>(h_in);
  auto* slab = static_cast<uint8_t*>(d_slab);
  for (uint64_t c0 = 0; c0 < nseg; c0 += per) {
    const uint64_t cn = nseg - c0 < per ? nseg - c0 : per;
    const uint64_t off = c0 * seg, nb = n - off < cn * seg ? n - off : cn * seg;
    HIP_TRY(hipMemcpyAsync(stage + off, src + off, nb, hipMemcpyDefault, c), "stage input");
    if (int r = stream_after(s, c)) return r;
    if (int r = compress_impl(ctx, s, codec, stage + off, nb, seg,
                              slab ? slab + c0 * slot_stride : nullptr, slot_stride,
                              d_dsts ? d_dsts + c0 : nullptr, d_sizes + c0))
      return r;
  }
  return 0;
}

int bitar_hip_decompress_host(bitar_hip_ctx* ctx, void* stream, uint32_t codec,
                              const void* const* d_srcs, const uint32_t* d_sizes, uint32_t nseg,
                              uint32_t seg, void* d_stage, void* h_out, uint64_t capacity,
                              uint32_t* d_produced) {
  if (int r = enter(ctx)) return r;
  if (nseg == 0) return 0;
  if (capacity < (uint64_t)nseg * seg)  // reference device.cc:248-254
    return fail(BITAR_HIP_CAPACITY_ERROR, "The decompressed_buffer is required to be >= " +
                                              std::to_string((uint64_t)nseg * seg) + " bytes");
  if (!d_srcs || !d_sizes || !d_stage || !h_out || !d_produced)
    return fail(BITAR_HIP_INVALID, "null buffer");
  if (seg == 0 || seg > kMaxSeg) return fail(BITAR_HIP_INVALID, "seg must be in [1, 65536]");
  const hipStream_t s = pick_stream(ctx, stream);
  const hipStream_t c = copy_stream_for(ctx, s);
  if (!c) return fail(BITAR_HIP_UNKNOWN_ERROR, "copy stream");
  if (int r = stream_after(c, s)) return r;  // (h_out / d_stage users queued before)
  const uint64_t per = host_chunk_segs(nseg, seg);
  auto* stage = static_cast<uint8_t*>(d_stage);
  auto* out = static_cast<uint8_t*>(h_out);
  for (uint64_t c0 = 0; c0 < nseg; c0 += per) {
    const uint64_t cn = nseg - c0 < per ? nseg - c0 : per;
    if (int r = decompress_impl(ctx, s, codec, d_srcs + c0, nullptr, 0, d_sizes + c0,
                                (uint32_t)cn, seg, stage + c0 * seg, cn * seg, d_produced + c0))
      return r;
    if (int r = stream_after(c, s)) return r;
    HIP_TRY(hipMemcpyAsync(out + c0 * seg, stage + c0 * seg, cn * seg, hipMemcpyDefault, c),
            "output copy");
  }
  return stream_after(s, c);
}

int bitar_hip_sync(bitar_hip_ctx* ctx, void* stream) {
  if (int r = enter(ctx)) return r;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (s) {
    // this stream's word only: read and clear it in stream order, so work queued on other
    // streams (other queue pairs) can neither be reported here nor lose its error
    uint32_t* w = err_word(ctx, s);
    uint32_t err = 0;
    HIP_TRY(hipMemcpyAsync(&err, w, sizeof(err), hipMemcpyDeviceToHost, s), "read error word");
    HIP_TRY(hipMemsetAsync(w, 0, sizeof(err), s), "clear error word");
    HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
    return sync_error(err);
  }
  // NULL: the default stream and this context's queue pairs (not other contexts' or other
  // libraries' streams).  Only their words (0 = the default stream, 1..num_streams) are read
  // and cleared: a foreign stream's word belongs to a sync of that stream, since work still
  // running there could set it after this read and lose its error at the clear.
  HIP_TRY(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
  for (hipStream_t q : ctx->streams) HIP_TRY(hipStreamSynchronize(q), "hipStreamSynchronize");
  const size_t nw = ctx->streams.size() + 1;
  std::vector<uint32_t> words(nw);
  HIP_TRY(hipMemcpy(words.data(), ctx->d_err, nw * sizeof(uint32_t), hipMemcpyDeviceToHost),
          "read error words");
  uint32_t err = 0;
  for (uint32_t x : words) err |= x;
  if (err) HIP_TRY(hipMemset(ctx->d_err, 0, nw * sizeof(uint32_t)), "clear error words");
  return sync_error(err);
}

int bitar_hip_pack(bitar_hip_ctx* ctx, void* stream, const void* d_slab, uint64_t slot_stride,
                   const uint32_t* d_sizes, uint32_t nseg, uint64_t* d_offsets, void* d_frame) {
  if (int r = enter(ctx)) return r;
  if (!d_sizes || !d_offsets) return fail(BITAR_HIP_INVALID, "null buffer");
  if (d_frame && nseg && (!d_slab || slot_stride == 0))
    return fail(BITAR_HIP_INVALID, "null slab or zero slot stride");
  hipStream_t s = pick_stream(ctx, stream);
  // sizes above the slot stride (a failed op's SEGMENT_ERROR) pack as 0 bytes and flag the
  // stream's error word, so the next sync reports IOError instead of copying out of bounds
  const uint64_t limit = slot_stride ? slot_stride : (uint64_t)BITAR_HIP_SEGMENT_ERROR - 1;
  hipLaunchKernelGGL(bitar_hip::scan_sizes_kernel, dim3(1), dim3(1024), 0, s, d_sizes, nseg,
                     limit, d_offsets, err_word(ctx, s));
  HIP_TRY(hipGetLastError(), "scan launch");
  if (d_frame && nseg) {
    hipLaunchKernelGGL(bitar_hip::pack_kernel, dim3(nseg), dim3(64), 0, s,
                       static_cast<const uint8_t*>(d_slab), slot_stride, d_sizes, d_offsets,
                       nseg, static_cast<uint8_t*>(d_frame));
    HIP_TRY(hipGetLastError(), "pack launch");
  }
  return 0;
}

int bitar_hip_lz4_chain(bitar_hip_ctx* ctx, void* stream, const void* d_src, uint32_t src_len,
                        const uint32_t* d_blocks, uint32_t nblocks, void* d_out,
                        uint64_t capacity, uint32_t* d_produced) {
  if (int r = enter(ctx)) return r;
  if (!d_src || !d_blocks || !d_out || !d_produced) return fail(BITAR_HIP_INVALID, "null buffer");
  if (capacity > 0xFFFFFFFFull) capacity = 0xFFFFFFFFull;
  hipStream_t s = pick_stream(ctx, stream);
  hipLaunchKernelGGL(bitar_hip::lz4_chain_kernel, dim3(1), dim3(64), 0, s,
                     static_cast<const uint8_t*>(d_src), src_len, d_blocks, nblocks,
                     static_cast<uint8_t*>(d_out), (uint32_t)capacity, d_produced,
                     err_word(ctx, s));
  HIP_TRY(hipGetLastError(), "lz4 chain launch");
  return 0;
}

int bitar_hip_copy_batch(bitar_hip_ctx* ctx, void* stream, const void* const* d_srcs,
                         void* const* d_dsts, const uint32_t* d_sizes, uint32_t n) {
  if (int r = enter(ctx)) return r;
  if (n == 0) return 0;
  if (!d_srcs || !d_dsts || !d_sizes) return fail(BITAR_HIP_INVALID, "null buffer");
  hipStream_t s = pick_stream(ctx, stream);
  hipLaunchKernelGGL(bitar_hip::copy_batch_kernel, dim3(n), dim3(64), 0, s,
                     reinterpret_cast<const uint8_t* const*>(d_srcs),
                     reinterpret_cast<uint8_t* const*>(d_dsts), d_sizes, n);
  HIP_TRY(hipGetLastError(), "copy batch launch");
  return 0;
}

int bitar_hip_pack_lz4f(bitar_hip_ctx* ctx, void* stream, const void* d_in, uint64_t n,
                        uint32_t seg, const void* d_slab, uint64_t slot_stride,
                        const uint32_t* d_sizes, uint32_t* d_framed, uint64_t* d_offsets,
                        void* d_frame) {
  if (int r = enter(ctx)) return r;
  if (seg == 0 || seg > kMaxSeg) return fail(BITAR_HIP_INVALID, "seg must be in [1, 65536]");
  const uint64_t nseg64 = (n + seg - 1) / seg;
  if (nseg64 > 0x7FFFFFFFull) return fail(BITAR_HIP_INVALID, "too many segments");
  const uint32_t nseg = (uint32_t)nseg64;
  if (!d_sizes || !d_framed || !d_offsets) return fail(BITAR_HIP_INVALID, "null buffer");
  hipStream_t s = pick_stream(ctx, stream);
  if (nseg) {
    hipLaunchKernelGGL(bitar_hip::lz4f_sizes_kernel, dim3((nseg + 255) / 256), dim3(256), 0, s,
                       d_sizes, nseg, n, seg, d_framed);
    HIP_TRY(hipGetLastError(), "lz4f sizes launch");
  }
  hipLaunchKernelGGL(bitar_hip::scan_sizes_kernel, dim3(1), dim3(1024), 0, s, d_framed, nseg,
                     (uint64_t)BITAR_HIP_SEGMENT_ERROR - 1, d_offsets, err_word(ctx, s));
  HIP_TRY(hipGetLastError(), "scan launch");
  if (d_frame && nseg) {
    if (!d_slab || !d_in) return fail(BITAR_HIP_INVALID, "null input or slab");
    hipLaunchKernelGGL(bitar_hip::lz4f_pack_kernel, dim3(nseg), dim3(64), 0, s,
                       static_cast<const uint8_t*>(d_in), n, seg,
                       static_cast<const uint8_t*>(d_slab), slot_stride, d_sizes, d_offsets,
                       nseg, static_cast<uint8_t*>(d_frame));
    HIP_TRY(hipGetLastError(), "lz4f pack launch");
  }
  return 0;
}

int bitar_hip_checksum(bitar_hip_ctx* ctx, void* stream, uint32_t kind, const void* d_data,
                       uint64_t n, uint32_t seg, const uint32_t* d_lens, uint32_t nseg,
                       uint64_t* d_sums) {
  if (int r = enter(ctx)) return r;
  if (kind < BITAR_HIP_CHECKSUM_CRC32 || kind > BITAR_HIP_CHECKSUM_CRC32_ADLER32)
    return fail(BITAR_HIP_INVALID, "checksum kind must be CRC32, ADLER32 or CRC32_ADLER32");
  if (seg == 0 || seg > kMaxSeg) return fail(BITAR_HIP_INVALID, "seg must be in [1, 65536]");
  if (!d_lens && nseg != (uint32_t)((n + seg - 1) / seg))
    return fail(BITAR_HIP_INVALID, "nseg must be ceil(n / seg) without a length array");
  if (!nseg) return 0;
  if (!d_data || !d_sums) return fail(BITAR_HIP_INVALID, "null buffer");
  hipLaunchKernelGGL(bitar_hip::checksum_kernel, dim3(nseg), dim3(64), 0, pick_stream(ctx, stream),
                     kind, static_cast<const uint8_t*>(d_data), n, seg, d_lens, nseg, d_sums);
  HIP_TRY(hipGetLastError(), "checksum launch");
  return 0;
}

int bitar_hip_fill_at(bitar_hip_ctx* ctx, void* stream, int kind, uint64_t seed,
                      uint64_t offset, void* d_out, uint64_t n) {
  if (int r = enter(ctx)) return r;
  if (offset & 63u) return fail(BITAR_HIP_INVALID, "fill offset must be a multiple of 64");
  if (!n) return 0;
  if (!d_out) return fail(BITAR_HIP_INVALID, "null buffer");
  const uint64_t lines = (n + 63) / 64;
  uint64_t blocks = (lines + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(bitar_hip::fill_kernel, dim3((uint32_t)blocks), dim3(256), 0,
                     pick_stream(ctx, stream), kind, seed, offset,
                     static_cast<uint8_t*>(d_out), n);
  HIP_TRY(hipGetLastError(), "fill launch");
  return 0;
}

int bitar_hip_fill(bitar_hip_ctx* ctx, void* stream, int kind, uint64_t seed, void* d_out,
                   uint64_t n) {
  return bitar_hip_fill_at(ctx, stream, kind, seed, 0, d_out, n);
}

}  // extern "C"
