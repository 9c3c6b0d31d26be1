// device.cc -- CompressDevice on an MI355X (reference src/device.cc + src/memory.cc).
//
// Reference flow per call: AssembleFrom (mbufs per segment, memzone slots) -> EnqueueBurst
// -> DequeueBurst (busy-poll) -> callback, repeated per burst of <= 32 ops
// (device.cc:156-318, memory.cc:350-505).  Here: take one slot per segment from the HBM slot
// pool, upload the slot-address table, launch ONE kernel over every segment on the queue
// pair's stream, read back the per-segment sizes, sync.  Errors map as in the reference:
// per-op failure / OUT_OF_SPACE -> IOError, busy queue pair -> Cancelled, capacity ->
// CapacityError, bad state/range -> Invalid.
#include "bitar/device.h"

#include <arrow/buffer.h>
#include <arrow/util/logging.h>

#include <algorithm>
#include <cstring>
#include <stack>

#include "bitar/hip_device.h"
#include "bitar_hip.h"
#include "hip_ctx.h"

namespace bitar {

namespace internal {

static constexpr std::uint32_t kMinPreallocateSlots = 20;  // reference memory.h:51

// Pool of compressed-output slots (DeviceMemory, reference memory.cc:120-228): a LIFO free
// stack of slot addresses carved from HBM chunks, an occupied flag per slot (the reference's
// occupied set, as a flag array: a 16384-segment call takes and returns 16384 slots, and a
// hash-set node per slot cost ~1 ms of host time per call), growth on demand.
class DeviceMemory {
 public:
  DeviceMemory(bitar_hip_ctx* ctx, std::uint64_t slot_size) : ctx_(ctx), slot_size_(slot_size) {}
  ~DeviceMemory() {
    for (auto& c : chunks_) (void)bitar_hip_free(ctx_, c.base);
  }

  arrow::Status Preallocate(std::uint32_t n) { return Grow(n); }

  // n slots (the reference takes one memzone per segment, memory.cc:405-425)
  arrow::Status Take(std::uint32_t n, std::vector<std::uint8_t*>* out) {
    const std::lock_guard<std::mutex> lock(mutex_);
    if (free_.size() < n) {
      ARROW_RETURN_NOT_OK(GrowLocked(std::max<std::uint32_t>(
          n - static_cast<std::uint32_t>(free_.size()), kGrowSlots)));
    }
    out->resize(n);
    for (std::uint32_t i = 0; i < n; ++i) {
      std::uint8_t* a = free_.back();
      free_.pop_back();
      (*out)[i] = a;
      *Flag(a) = 1;
    }
    return arrow::Status::OK();
  }

  // 1 if addr is the start of an occupied slot (returned to the pool), else 0
  std::size_t Put(const std::uint8_t* addr) {
    const std::lock_guard<std::mutex> lock(mutex_);
    return PutLocked(addr);
  }

  // every slot of `buffers`, last to first (one lock for the whole call)
  std::size_t PutBuffers(const BufferVector& buffers) {
    const std::lock_guard<std::mutex> lock(mutex_);
    std::size_t count = 0;
    for (auto it = std::crbegin(buffers); it != std::crend(buffers); ++it)
      count += PutLocked(reinterpret_cast<const std::uint8_t*>((*it)->address()));
    return count;
  }

  void PutAll(const std::vector<std::uint8_t*>& slots) {
    const std::lock_guard<std::mutex> lock(mutex_);
    for (auto* s : slots) PutLocked(s);
  }

 private:
  static constexpr std::uint32_t kGrowSlots = 256;
  struct Chunk {
    std::uint8_t* base;
    std::uint64_t n;
    std::vector<std::uint8_t> occupied;
  };

  // the occupied flag of the slot starting at addr, nullptr if addr starts no slot
  std::uint8_t* Flag(const std::uint8_t* addr) {
    // chunks_ is sorted by base: the last chunk starting at or below addr
    auto it = std::upper_bound(chunks_.begin(), chunks_.end(), addr,
                               [](const std::uint8_t* a, const Chunk& c) { return a < c.base; });
    if (it == chunks_.begin()) return nullptr;
    Chunk& c = *(it - 1);
    const std::uint64_t off = static_cast<std::uint64_t>(addr - c.base);
    if (off % slot_size_ || off / slot_size_ >= c.n) return nullptr;
    return &c.occupied[off / slot_size_];
  }

  std::size_t PutLocked(const std::uint8_t* addr) {
    std::uint8_t* f = Flag(addr);
    if (!f || !*f) return 0;
    *f = 0;
    free_.push_back(const_cast<std::uint8_t*>(addr));
    return 1;
  }

  arrow::Status Grow(std::uint32_t n) {
    const std::lock_guard<std::mutex> lock(mutex_);
    return GrowLocked(n);
  }
  arrow::Status GrowLocked(std::uint32_t n) {
    if (!chunks_.empty())
      ARROW_LOG(WARNING) << "Allocating output slots in the critical path (" << n << " slots)";
    void* p = nullptr;
    BITAR_ABI(bitar_hip_alloc(ctx_, slot_size_ * n, &p), "slot pool");
    auto* base = static_cast<std::uint8_t*>(p);
    Chunk c{base, n, std::vector<std::uint8_t>(n, 0)};
    chunks_.insert(std::upper_bound(chunks_.begin(), chunks_.end(), base,
                                    [](const std::uint8_t* a, const Chunk& x) { return a < x.base; }),
                   std::move(c));
    for (std::uint32_t i = n; i-- > 0;) free_.push_back(base + slot_size_ * i);
    return arrow::Status::OK();
  }

  bitar_hip_ctx* ctx_;
  const std::uint64_t slot_size_;
  std::vector<Chunk> chunks_;  // sorted by base
  std::vector<std::uint8_t*> free_;
  std::mutex mutex_;
};

// A compressed output: a non-owning view of one HBM slot (memory.cc:211-228) whose size is
// set once the kernel's sizes are back -- so the views are built while the kernel runs.
class SlotBuffer : public arrow::Buffer {
 public:
  SlotBuffer(const std::uint8_t* data, std::shared_ptr<arrow::MemoryManager> mm)
      : arrow::Buffer(data, 0, std::move(mm)) {}
  void set_size(std::int64_t n) {
    size_ = n;
    capacity_ = n;
  }
};

// Per-queue-pair stream and staging (QueuePairMemory, reference memory.cc:237-348): pinned
// host tables of slot addresses / sizes, their device copies, and an HBM staging area for
// host-resident inputs and outputs.
struct QueuePairMemory {
  bitar_hip_ctx* ctx = nullptr;
  void* stream = nullptr;
  std::atomic<bool> busy{false};
  std::uint64_t* h_ptrs = nullptr;
  std::uint32_t* h_sizes = nullptr;
  std::uint64_t* d_ptrs = nullptr;
  std::uint32_t* d_sizes = nullptr;
  std::uint32_t* d_prod = nullptr;
  std::size_t table_cap = 0;
  void* d_stage = nullptr;
  std::uint64_t stage_cap = 0;
  std::uint64_t* d_sums = nullptr;  // per-segment checksums (device, then pinned host)
  std::uint64_t* h_sums = nullptr;
  std::size_t sums_cap = 0;
  std::vector<std::uint64_t> checksums;  // of the last call
  void* d_chain = nullptr;  // chained ops (max_sgl_segs > 1): one stream per op
  std::uint64_t chain_cap = 0;
  // what d_ptrs[0, ptr_mirror.size()) holds: a steady-state caller gets its slots back in the
  // same order every call (LIFO pool, Recycle last to first), so the slot-pointer table of a
  // compress call -- and of the decompress call over those slots -- is usually already on the
  // device and its copy is skipped
  std::vector<std::uint64_t> ptr_mirror;

  // d_ptrs[0, n) <- h_ptrs[0, n) on the queue pair's stream, unless d_ptrs already holds them
  int UploadPtrs(std::uint32_t n) {
    if (ptr_mirror.size() >= n && std::memcmp(ptr_mirror.data(), h_ptrs, 8ull * n) == 0) return 0;
    const int rc = bitar_hip_memcpy(ctx, d_ptrs, h_ptrs, 8ull * n, stream);
    if (rc == 0) ptr_mirror.assign(h_ptrs, h_ptrs + n);
    else ptr_mirror.clear();
    return rc;
  }

  ~QueuePairMemory() {
    if (!ctx) return;
    if (h_ptrs) (void)bitar_hip_host_free(ctx, h_ptrs);
    if (h_sizes) (void)bitar_hip_host_free(ctx, h_sizes);
    if (d_ptrs) (void)bitar_hip_free(ctx, d_ptrs);
    if (d_sizes) (void)bitar_hip_free(ctx, d_sizes);
    if (d_prod) (void)bitar_hip_free(ctx, d_prod);
    if (d_stage) (void)bitar_hip_free(ctx, d_stage);
    if (d_sums) (void)bitar_hip_free(ctx, d_sums);
    if (h_sums) (void)bitar_hip_host_free(ctx, h_sums);
    if (d_chain) (void)bitar_hip_free(ctx, d_chain);
  }

  arrow::Status Chain(std::uint64_t bytes) {
    if (bytes <= chain_cap) return arrow::Status::OK();
    if (d_chain) (void)bitar_hip_free(ctx, d_chain);
    d_chain = nullptr;
    chain_cap = 0;
    BITAR_ABI(bitar_hip_alloc(ctx, bytes, &d_chain), "qp chain scratch");
    chain_cap = bytes;
    return arrow::Status::OK();
  }

  arrow::Status Sums(std::size_t n) {
    if (n <= sums_cap) return arrow::Status::OK();
    if (d_sums) (void)bitar_hip_free(ctx, d_sums);
    if (h_sums) (void)bitar_hip_host_free(ctx, h_sums);
    d_sums = nullptr;
    h_sums = nullptr;
    sums_cap = 0;
    const std::size_t cap = std::max<std::size_t>(n, 1024);
    void* p = nullptr;
    BITAR_ABI(bitar_hip_alloc(ctx, cap * 8, &p), "checksum table");
    d_sums = static_cast<std::uint64_t*>(p);
    BITAR_ABI(bitar_hip_host_alloc(ctx, cap * 8, &p), "checksum table");
    h_sums = static_cast<std::uint64_t*>(p);
    sums_cap = cap;
    return arrow::Status::OK();
  }

  arrow::Status Tables(std::size_t n) {
    if (n <= table_cap) return arrow::Status::OK();
    std::size_t cap = std::max<std::size_t>(n, 2 * table_cap);
    if (h_ptrs) (void)bitar_hip_host_free(ctx, h_ptrs);
    if (h_sizes) (void)bitar_hip_host_free(ctx, h_sizes);
    if (d_ptrs) (void)bitar_hip_free(ctx, d_ptrs);
    if (d_sizes) (void)bitar_hip_free(ctx, d_sizes);
    if (d_prod) (void)bitar_hip_free(ctx, d_prod);
    h_ptrs = nullptr;
    h_sizes = nullptr;
    d_ptrs = nullptr;
    d_sizes = nullptr;
    d_prod = nullptr;
    table_cap = 0;
    ptr_mirror.clear();
    void* p = nullptr;
    BITAR_ABI(bitar_hip_host_alloc(ctx, cap * 8, &p), "qp tables");
    h_ptrs = static_cast<std::uint64_t*>(p);
    BITAR_ABI(bitar_hip_host_alloc(ctx, cap * 4, &p), "qp tables");
    h_sizes = static_cast<std::uint32_t*>(p);
    BITAR_ABI(bitar_hip_alloc(ctx, cap * 8, &p), "qp tables");
    d_ptrs = static_cast<std::uint64_t*>(p);
    BITAR_ABI(bitar_hip_alloc(ctx, cap * 4, &p), "qp tables");
    d_sizes = static_cast<std::uint32_t*>(p);
    BITAR_ABI(bitar_hip_alloc(ctx, cap * 4, &p), "qp tables");
    d_prod = static_cast<std::uint32_t*>(p);
    table_cap = cap;
    return arrow::Status::OK();
  }

  arrow::Status Stage(std::uint64_t bytes) {
    if (bytes <= stage_cap) return arrow::Status::OK();
    if (d_stage) (void)bitar_hip_free(ctx, d_stage);
    d_stage = nullptr;
    stage_cap = 0;
    BITAR_ABI(bitar_hip_alloc(ctx, bytes, &d_stage), "qp staging");
    stage_cap = bytes;
    return arrow::Status::OK();
  }
};

namespace {

// true if `addr` is HBM of `device` (buffers of our memory manager short-cut the query)
bool OnDevice(const arrow::Buffer& b, int device) {
  const auto& mm = b.memory_manager();
  if (mm && !mm->is_cpu() && mm->device()->device_type() == arrow::DeviceAllocationType::kROCM)
    return mm->device()->device_id() == device;
  int kind = 0, dev = -1;
  if (bitar_hip_pointer_info(reinterpret_cast<const void*>(b.address()), &kind, &dev) != 0)
    return false;
  return kind == 2 && dev == device;
}

bool OnDevice(std::uint64_t address, int device) {
  int kind = 0, dev = -1;
  if (bitar_hip_pointer_info(reinterpret_cast<const void*>(address), &kind, &dev) != 0)
    return false;
  return kind == 2 && dev == device;
}

// DEFLATE + FIXED -> fixed-Huffman blocks; DEFLATE + DYNAMIC (the reference default,
// config.h:151) or DEFAULT (the PMD's choice) -> dynamic Huffman
template <typename Cfg>
std::uint32_t AbiCodec(const Cfg& c) {
  switch (c.codec()) {
    case Codec::LZ4: return c.level() >= 2 ? BITAR_HIP_CODEC_LZ4_WIDE : BITAR_HIP_CODEC_LZ4;
    case Codec::ZSTD: return BITAR_HIP_CODEC_ZSTD;
    default:
      return c.huffman_enc() == HuffmanEncoding::FIXED ? BITAR_HIP_CODEC_DEFLATE
                                                      : BITAR_HIP_CODEC_DEFLATE_DYNAMIC;
  }
}

}  // namespace

}  // namespace internal

template <typename Class, typename Enable>
arrow::Status CompressDevice<Class, Enable>::Initialize(
    std::unique_ptr<Configuration<Class>> configuration) {
  if (state_ != internal::DeviceState::kUndefined)
    return arrow::Status::Invalid("Compress device ", +device_id_, " is already initialized");
  ARROW_RETURN_NOT_OK(set_configuration(std::move(configuration)));
  ARROW_RETURN_NOT_OK(ValidateConfiguration());
  ARROW_RETURN_NOT_OK(PreAllocateMemory());
  set_state(internal::DeviceState::kStarted);
  return arrow::Status::OK();
}

template <typename Class, typename Enable>
arrow::Status CompressDevice<Class, Enable>::PreAllocateMemory() {
  bitar_hip_config cfg{num_qps(), 0};
  BITAR_ABI(bitar_hip_open(device_id_, &cfg, &ctx_), "Device configuration failed");
  set_state(internal::DeviceState::kConfigured);
  const auto codec = internal::AbiCodec(*configuration_);
  const std::uint32_t seg = configuration_->decompressed_seg_size();
  slot_size_ = std::max<std::uint64_t>(bitar_hip_slot_size(codec, seg),
                                       (configuration_->compressed_seg_size() + 255u) & ~255u);
  device_memory_ = std::make_unique<internal::DeviceMemory>(ctx_, slot_size_);
  ARROW_RETURN_NOT_OK(device_memory_->Preallocate(configuration_->max_preallocate_memzones()));
  for (std::uint16_t qp = 0; qp < num_qps(); ++qp) {
    auto m = std::make_unique<internal::QueuePairMemory>();
    m->ctx = ctx_;
    BITAR_ABI(bitar_hip_stream(ctx_, qp, &m->stream), "queue pair stream");
    ARROW_RETURN_NOT_OK(m->Tables(1024));
    qp_memory_.push_back(std::move(m));
  }
  return arrow::Status::OK();
}

template <typename Class, typename Enable>
arrow::Status CompressDevice<Class, Enable>::EntryGuard(std::uint16_t queue_pair_id) {
  if (ARROW_PREDICT_FALSE(state_ != internal::DeviceState::kStarted)) {
    return arrow::Status::Invalid("Compress device ", +device_id_,
                                  " has not started. [Current state: ",
                                  static_cast<int>(state_), "]");
  }
  if (ARROW_PREDICT_FALSE(queue_pair_id >= num_qps())) {
    return arrow::Status::Invalid("queue_pair_id must be in the range of [0, ", num_qps(), ")");
  }
  bool expected = false;  // atomic, unlike the reference's pending-ops hint (device.cc:456)
  if (!qp_memory_[queue_pair_id]->busy.compare_exchange_strong(expected, true)) {
    return arrow::Status::Cancelled("Queue pair ", queue_pair_id, " of compress device ",
                                    +device_id_, " is busy");
  }
  return arrow::Status::OK();
}

template <typename Class, typename Enable>
void CompressDevice<Class, Enable>::Leave(std::uint16_t queue_pair_id) {
  qp_memory_[queue_pair_id]->busy.store(false);
}

template <typename Class, typename Enable>
void* CompressDevice<Class, Enable>::stream(std::uint16_t queue_pair_id) const {
  return queue_pair_id < qp_memory_.size() ? qp_memory_[queue_pair_id]->stream : nullptr;
}

template <typename Class, typename Enable>
const std::vector<std::uint64_t>& CompressDevice<Class, Enable>::checksums(
    std::uint16_t queue_pair_id) const {
  static const std::vector<std::uint64_t> kNone;
  return queue_pair_id < qp_memory_.size() ? qp_memory_[queue_pair_id]->checksums : kNone;
}

template <typename Class, typename Enable>
arrow::Result<BufferVector> CompressDevice<Class, Enable>::Compress(
    std::uint16_t queue_pair_id, const std::shared_ptr<arrow::Buffer>& decompressed_buffer) {
  BufferVector compressed_buffers;
  if (ARROW_PREDICT_FALSE(decompressed_buffer == nullptr || decompressed_buffer->size() == 0)) {
    return compressed_buffers;  // reference device.cc:161-164
  }
  ARROW_RETURN_NOT_OK(EntryGuard(queue_pair_id));
  auto* m = qp_memory_[queue_pair_id].get();
  struct Guard {
    CompressDevice* d;
    std::uint16_t qp;
    ~Guard() { d->Leave(qp); }
  } guard{this, queue_pair_id};

  const std::uint32_t seg = configuration_->decompressed_seg_size();
  const auto n = static_cast<std::uint64_t>(decompressed_buffer->size());
  const auto nseg = static_cast<std::uint32_t>((n + seg - 1) / seg);
  const auto codec = internal::AbiCodec(*configuration_);

  // input: read HBM in place; host memory (the reference attaches it zero-copy, 380-399) is
  // staged into HBM chunk by chunk with each chunk's compress overlapping the next one's
  // copy (bitar_hip_compress_host)
  const void* h_in = reinterpret_cast<const void*>(decompressed_buffer->address());
  const void* d_in = h_in;
  const bool host_in = !internal::OnDevice(*decompressed_buffer, device_id_);
  if (host_in) {
    ARROW_RETURN_NOT_OK(m->Stage(n));
    d_in = m->d_stage;
  }

  std::vector<std::uint8_t*> slots;
  ARROW_RETURN_NOT_OK(device_memory_->Take(nseg, &slots));
  auto release = [&](const arrow::Status& st) {  // ReleaseAll (device.cc:537-542)
    device_memory_->PutAll(slots);
    return st;
  };
  auto failed = [&](int rc) {
    m->ptr_mirror.clear();  // (a failed stream: the table's copy may not have landed)
    return release(internal::FromAbi(
        rc, "Failed to compress via queue pair " + std::to_string(queue_pair_id) +
                " of compress device " + std::to_string(device_id_)));
  };
  // an op covers k segments (max_sgl_segs, reference memory.cc:359-399); k == 1 compresses
  // each segment straight into its slot, k > 1 compresses the op as one stream into the
  // queue pair's chain scratch and then spreads it over the op's slots (the dst mbuf chain,
  // memory.cc:401-425), slot_size() bytes per slot
  const std::uint32_t k = configuration_->max_sgl_segs();
  const std::uint64_t opseg = std::uint64_t{k} * seg;
  const auto nops = static_cast<std::uint32_t>((n + opseg - 1) / opseg);
  const std::uint64_t stride = k > 1 ? bitar_hip_slot_size(codec, static_cast<std::uint32_t>(opseg)) : 0;
  auto st = m->Tables(k > 1 ? 2ull * nseg + nops : nseg);
  if (st.ok() && k > 1) st = m->Chain(stride * nops);
  if (!st.ok()) return release(st);
  int rc = 0;
  if (k == 1) {
    for (std::uint32_t i = 0; i < nseg; ++i)
      m->h_ptrs[i] = static_cast<std::uint64_t>(reinterpret_cast<uintptr_t>(slots[i]));
    rc = m->UploadPtrs(nseg);
    const auto* dsts = reinterpret_cast<void* const*>(m->d_ptrs);
    if (rc == 0 && host_in)
      rc = bitar_hip_compress_host(ctx_, m->stream, codec, h_in, n, seg, m->d_stage, nullptr,
                                   dsts, slot_size_, m->d_sizes);
    else if (rc == 0)
      rc = bitar_hip_compress_scattered(ctx_, m->stream, codec, d_in, n, seg, dsts, slot_size_,
                                        m->d_sizes);
  } else {
    if (host_in) rc = bitar_hip_memcpy(ctx_, m->d_stage, h_in, n, m->stream);
    if (rc == 0)
      rc = bitar_hip_compress(ctx_, m->stream, codec, d_in, n, static_cast<std::uint32_t>(opseg),
                              m->d_chain, stride, m->d_sizes);
  }
  if (rc == 0) rc = bitar_hip_memcpy(ctx_, m->h_sizes, m->d_sizes, 4ull * nops, m->stream);
  auto mm = hip_memory_manager(device_id_);
  if (rc == 0 && k == 1) {
    // the output views, built while the kernel runs (their sizes are set after the sync)
    compressed_buffers.reserve(nseg);
    for (std::uint32_t i = 0; i < nseg; ++i)
      compressed_buffers.emplace_back(std::make_unique<internal::SlotBuffer>(slots[i], mm));
  }
  // the checksum of the uncompressed input of each op (DPDK input_chksum of a compress op)
  const std::uint32_t ck = checksum_kind();
  if (rc == 0 && ck) {
    st = m->Sums(nops);
    if (!st.ok()) return release(st);
    rc = bitar_hip_checksum(ctx_, m->stream, ck, d_in, n, static_cast<std::uint32_t>(opseg),
                            nullptr, nops, m->d_sums);
    if (rc == 0) rc = bitar_hip_memcpy(ctx_, m->h_sums, m->d_sums, 8ull * nops, m->stream);
  }
  if (rc == 0) rc = bitar_hip_sync(ctx_, m->stream);
  if (rc != 0) return failed(rc);
  m->checksums.assign(m->h_sums, ck ? m->h_sums + nops : m->h_sums);
  for (std::uint32_t j = 0; j < nops; ++j) {
    const std::uint64_t cap = (k == 1 ? 1 : std::min<std::uint64_t>(k, nseg - std::uint64_t{j} * k)) * slot_size_;
    if (m->h_sizes[j] == BITAR_HIP_SEGMENT_ERROR || m->h_sizes[j] > cap)
      return release(arrow::Status::IOError("Compress data output is larger than allocated buffer"));
  }
  if (k == 1) {
    for (std::uint32_t i = 0; i < nseg; ++i)
      static_cast<internal::SlotBuffer*>(compressed_buffers[i].get())->set_size(m->h_sizes[i]);
    return compressed_buffers;
  }
  compressed_buffers.reserve(nseg);
  // spread op j's stream over its slots: slot i of the op holds bytes [i*L, (i+1)*L); the
  // op's trailing slots may stay empty and are returned as empty buffers, so that Decompress
  // regroups exactly k buffers per op (the reference returns only the non-empty ones,
  // device.cc:183-195, and then groups by k regardless)
  const std::uint64_t L = slot_size_;
  std::vector<std::uint32_t> piece(nseg, 0);
  std::uint32_t e = 0;
  auto* chain = static_cast<std::uint8_t*>(m->d_chain);
  for (std::uint32_t i = 0; i < nseg; ++i) {
    const std::uint32_t j = i / k;
    const std::uint64_t at = std::uint64_t{i % k} * L;
    const std::uint64_t size = m->h_sizes[j];
    piece[i] = static_cast<std::uint32_t>(size > at ? std::min(L, size - at) : 0);
    if (piece[i] == 0) continue;
    m->h_ptrs[e] = reinterpret_cast<std::uint64_t>(chain + j * stride + at);
    m->h_ptrs[nseg + e] = reinterpret_cast<std::uint64_t>(slots[i]);
    m->h_sizes[nops + e] = piece[i];
    ++e;
  }
  m->ptr_mirror.clear();
  rc = bitar_hip_memcpy(ctx_, m->d_ptrs, m->h_ptrs, 16ull * nseg, m->stream);
  if (rc == 0) rc = bitar_hip_memcpy(ctx_, m->d_sizes, m->h_sizes + nops, 4ull * e, m->stream);
  if (rc == 0)
    rc = bitar_hip_copy_batch(ctx_, m->stream, reinterpret_cast<const void* const*>(m->d_ptrs),
                              reinterpret_cast<void* const*>(m->d_ptrs + nseg), m->d_sizes, e);
  if (rc == 0) rc = bitar_hip_sync(ctx_, m->stream);
  if (rc != 0) return failed(rc);
  for (std::uint32_t i = 0; i < nseg; ++i)
    compressed_buffers.emplace_back(std::make_unique<arrow::Buffer>(slots[i], piece[i], mm));
  return compressed_buffers;
}

template <typename Class, typename Enable>
arrow::Status CompressDevice<Class, Enable>::Decompress(
    std::uint16_t queue_pair_id, const BufferVector& compressed_buffers,
    const std::unique_ptr<arrow::ResizableBuffer>& decompressed_buffer) {
  if (ARROW_PREDICT_FALSE(compressed_buffers.empty())) return arrow::Status::OK();
  const std::uint32_t seg = configuration_->decompressed_seg_size();
  const auto min_capacity = static_cast<std::int64_t>(compressed_buffers.size() * seg);
  if (decompressed_buffer == nullptr || decompressed_buffer->capacity() < min_capacity) {
    return arrow::Status::CapacityError("The decompressed_buffer is required to be >= ",
                                        min_capacity, " bytes");  // device.cc:248-254
  }
  ARROW_RETURN_NOT_OK(EntryGuard(queue_pair_id));
  auto* m = qp_memory_[queue_pair_id].get();
  struct Guard {
    CompressDevice* d;
    std::uint16_t qp;
    ~Guard() { d->Leave(qp); }
  } guard{this, queue_pair_id};

  const auto nseg = static_cast<std::uint32_t>(compressed_buffers.size());
  const auto codec = internal::AbiCodec(*configuration_);
  // op j decompresses buffers [j*k, (j+1)*k) as one stream into k segments of the output
  // (max_sgl_segs = k, reference memory.cc:432-505); k > 1 first joins the op's buffers in
  // the queue pair's chain scratch (the src mbuf chain)
  const std::uint32_t k = configuration_->max_sgl_segs();
  const std::uint64_t opseg = std::uint64_t{k} * seg;
  const std::uint32_t nops = (nseg + k - 1) / k, nfull = nseg / k, tail = nseg % k;
  ARROW_RETURN_NOT_OK(m->Tables(k > 1 ? 2ull * nseg + nops : 3ull * nseg));

  // sources: HBM buffers in place; host buffers staged behind the output area -- pinned ones
  // (the HipHost / Rtememzone pool) gathered by ONE copy kernel reading host memory over the
  // link, pageable ones by a copy each (memory.cc:459-500 attaches them zero-copy)
  std::uint64_t host_bytes = 0;
  std::vector<std::uint8_t> where(nseg);  // 2 HBM, 1 pinned host, 0 pageable host
  const arrow::MemoryManager* own_mm = hip_memory_manager(device_id_).get();
  for (std::uint32_t i = 0; i < nseg; ++i) {
    const auto& b = *compressed_buffers[i];
    // (our own slot views: their memory manager says so without a query)
    if (b.memory_manager().get() == own_mm || internal::OnDevice(b, device_id_)) {
      where[i] = 2;
      continue;
    }
    int kind = 0, dev = -1;
    (void)bitar_hip_pointer_info(reinterpret_cast<const void*>(b.address()), &kind, &dev);
    where[i] = kind == 1 ? 1 : 0;
    host_bytes += (static_cast<std::uint64_t>(b.size()) + 15) & ~15ull;
  }
  const auto out_addr = decompressed_buffer->mutable_address();
  const bool out_on_dev = internal::OnDevice(out_addr, device_id_);
  const std::uint64_t out_bytes = out_on_dev ? 0 : static_cast<std::uint64_t>(min_capacity);
  if (host_bytes + out_bytes) ARROW_RETURN_NOT_OK(m->Stage(host_bytes + out_bytes));
  auto* stage = static_cast<std::uint8_t*>(m->d_stage);
  std::uint64_t off = out_bytes;
  std::uint32_t ngather = 0;  // pinned sources: table entries at [nseg, 3 nseg)
  for (std::uint32_t i = 0; i < nseg; ++i) {
    const auto& b = compressed_buffers[i];
    if (static_cast<std::uint64_t>(b->size()) >= BITAR_HIP_SEGMENT_ERROR)
      return arrow::Status::Invalid("compressed buffer ", i, " is too large");
    m->h_sizes[i] = static_cast<std::uint32_t>(b->size());
    if (where[i] == 2) {
      m->h_ptrs[i] = b->address();
      continue;
    }
    if (where[i] == 1 && k == 1) {
      m->h_ptrs[nseg + ngather] = b->address();
      m->h_ptrs[2ull * nseg + ngather] = reinterpret_cast<std::uint64_t>(stage + off);
      m->h_sizes[nseg + ngather] = static_cast<std::uint32_t>(b->size());
      ++ngather;
    } else {
      BITAR_ABI(bitar_hip_memcpy(ctx_, stage + off, reinterpret_cast<const void*>(b->address()),
                                 static_cast<std::uint64_t>(b->size()), m->stream),
                "stage compressed input");
    }
    m->h_ptrs[i] = reinterpret_cast<std::uint64_t>(stage + off);
    off += (static_cast<std::uint64_t>(b->size()) + 15) & ~15ull;
  }
  if (ngather) {
    if (m->ptr_mirror.size() > nseg) m->ptr_mirror.resize(nseg);
    BITAR_ABI(bitar_hip_memcpy(ctx_, m->d_ptrs + nseg, m->h_ptrs + nseg, 8ull * ngather, m->stream),
              "tables");
    BITAR_ABI(bitar_hip_memcpy(ctx_, m->d_ptrs + 2ull * nseg, m->h_ptrs + 2ull * nseg,
                               8ull * ngather, m->stream), "tables");
    BITAR_ABI(bitar_hip_memcpy(ctx_, m->d_sizes + nseg, m->h_sizes + nseg, 4ull * ngather,
                               m->stream), "tables");
    BITAR_ABI(bitar_hip_copy_batch(ctx_, m->stream,
                                   reinterpret_cast<const void* const*>(m->d_ptrs + nseg),
                                   reinterpret_cast<void* const*>(m->d_ptrs + 2ull * nseg),
                                   m->d_sizes + nseg, ngather),
              "gather compressed input");
  }
  void* d_out = out_on_dev ? reinterpret_cast<void*>(out_addr) : m->d_stage;
  int rc = 0;
  std::uint32_t nunits = nseg;  // ops, one produced size / checksum each
  std::uint64_t unit = seg;
  bool out_copied = false;  // the output already went to host memory (decompress_host)
  if (k == 1) {
    BITAR_ABI(m->UploadPtrs(nseg), "tables");
    BITAR_ABI(bitar_hip_memcpy(ctx_, m->d_sizes, m->h_sizes, 4ull * nseg, m->stream), "tables");
    const auto* srcs = reinterpret_cast<const void* const*>(m->d_ptrs);
    if (!out_on_dev) {  // host output: decode chunks, each copied out while the next decodes
      rc = bitar_hip_decompress_host(ctx_, m->stream, codec, srcs, m->d_sizes, nseg, seg, d_out,
                                     reinterpret_cast<void*>(out_addr),
                                     static_cast<std::uint64_t>(min_capacity), m->d_prod);
      out_copied = true;
    } else {
      rc = bitar_hip_decompress(ctx_, m->stream, codec, srcs, m->d_sizes, nseg, seg, d_out,
                                static_cast<std::uint64_t>(min_capacity), m->d_prod);
    }
  } else {
    nunits = nops;
    unit = opseg;
    // op j's stream = its buffers back to back at chain + base_j (16-B aligned bases)
    std::uint64_t total = 0;
    std::vector<std::uint64_t> base(nops);
    for (std::uint32_t j = 0; j < nops; ++j) {
      base[j] = total;
      std::uint64_t len = 0;
      for (std::uint32_t i = j * k; i < std::min(nseg, (j + 1) * k); ++i) len += m->h_sizes[i];
      if (len >= BITAR_HIP_SEGMENT_ERROR)
        return arrow::Status::Invalid("compressed op ", j, " is too large");
      m->h_sizes[nseg + j] = static_cast<std::uint32_t>(len);
      total = (total + len + 15) & ~15ull;
    }
    ARROW_RETURN_NOT_OK(m->Chain(std::max<std::uint64_t>(total, 16)));
    auto* chain = static_cast<std::uint8_t*>(m->d_chain);
    for (std::uint32_t j = 0; j < nops; ++j) {
      std::uint64_t at = base[j];
      m->h_ptrs[2ull * nseg + j] = reinterpret_cast<std::uint64_t>(chain + at);
      for (std::uint32_t i = j * k; i < std::min(nseg, (j + 1) * k); ++i) {
        m->h_ptrs[nseg + i] = reinterpret_cast<std::uint64_t>(chain + at);
        at += m->h_sizes[i];
      }
    }
    m->ptr_mirror.clear();
    BITAR_ABI(bitar_hip_memcpy(ctx_, m->d_ptrs, m->h_ptrs, 8ull * (2ull * nseg + nops), m->stream),
              "tables");
    BITAR_ABI(bitar_hip_memcpy(ctx_, m->d_sizes, m->h_sizes, 4ull * (nseg + nops), m->stream),
              "tables");
    const auto* ops = reinterpret_cast<const void* const*>(m->d_ptrs + 2ull * nseg);
    rc = bitar_hip_copy_batch(ctx_, m->stream, reinterpret_cast<const void* const*>(m->d_ptrs),
                              reinterpret_cast<void* const*>(m->d_ptrs + nseg), m->d_sizes, nseg);
    if (rc == 0 && nfull)
      rc = bitar_hip_decompress(ctx_, m->stream, codec, ops, m->d_sizes + nseg, nfull,
                                static_cast<std::uint32_t>(opseg), d_out, nfull * opseg, m->d_prod);
    if (rc == 0 && tail)  // the last op covers the remaining tail < k buffers
      rc = bitar_hip_decompress(ctx_, m->stream, codec, ops + nfull, m->d_sizes + nseg + nfull, 1,
                                tail * seg, static_cast<std::uint8_t*>(d_out) + nfull * opseg,
                                std::uint64_t{tail} * seg, m->d_prod + nfull);
  }
  if (rc == 0)
    rc = bitar_hip_memcpy(ctx_, m->h_sizes, m->d_prod, 4ull * nunits, m->stream);
  // the checksum of the decompressed output of each op (DPDK output_chksum)
  const std::uint32_t ck = checksum_kind();
  if (rc == 0 && ck) {
    ARROW_RETURN_NOT_OK(m->Sums(nunits));
    rc = bitar_hip_checksum(ctx_, m->stream, ck, d_out, static_cast<std::uint64_t>(min_capacity),
                            static_cast<std::uint32_t>(unit), m->d_prod, nunits, m->d_sums);
    if (rc == 0) rc = bitar_hip_memcpy(ctx_, m->h_sums, m->d_sums, 8ull * nunits, m->stream);
  }
  if (rc == 0 && !out_on_dev && !out_copied)
    rc = bitar_hip_memcpy(ctx_, reinterpret_cast<void*>(out_addr), d_out,
                          static_cast<std::uint64_t>(min_capacity), m->stream);
  if (rc == 0) rc = bitar_hip_sync(ctx_, m->stream);
  if (rc == 0) m->checksums.assign(m->h_sums, ck ? m->h_sums + nunits : m->h_sums);
  if (rc != 0) {
    m->ptr_mirror.clear();
    return internal::FromAbi(rc, "Failed to decompress via queue pair " +
                                     std::to_string(queue_pair_id) + " of compress device " +
                                     std::to_string(device_id_));
  }
  std::int64_t total = 0;
  for (std::uint32_t i = 0; i < nunits; ++i) {
    if (m->h_sizes[i] == BITAR_HIP_SEGMENT_ERROR)
      return arrow::Status::IOError("Some operations have failed");
    total += m->h_sizes[i];
  }
  // Don't shrink the buffer (reference device.cc:312-315)
  ARROW_UNUSED(decompressed_buffer->Resize(total, false));
  return arrow::Status::OK();
}

template <typename Class, typename Enable>
std::size_t CompressDevice<Class, Enable>::Recycle(const BufferVector& buffers) {
  if (!device_memory_) return 0;
  return device_memory_->PutBuffers(buffers);
}

template <typename Class, typename Enable>
CompressDevice<Class, Enable>::~CompressDevice() {
  qp_memory_.clear();
  device_memory_.reset();
  if (ctx_) bitar_hip_close(ctx_);
  ctx_ = nullptr;
  set_state(internal::DeviceState::kUndefined);
}

template <typename Class, typename Enable>
CompressDevice<Class, Enable>::CompressDevice(std::uint8_t device_id,
                                              std::vector<std::uint32_t> worker_lcores)
    : device_id_(device_id), worker_lcores_(std::move(worker_lcores)) {}

template <typename Class, typename Enable>
arrow::Status CompressDevice<Class, Enable>::ValidateConfiguration() {
  // device capabilities: <= 64 queue pairs, chained ops of <= 64 KiB (max_sgl_segs * seg),
  // the encoder's window, fixed or dynamic Huffman (reference device.cc:352-415, 566-574)
  constexpr std::uint16_t kMaxQueuePairs = 64;
  if (num_qps() == 0 || num_qps() > kMaxQueuePairs) {
    return arrow::Status::Invalid("The requested number of queue pairs (", num_qps(),
                                  ") exceeds the maximum (", kMaxQueuePairs,
                                  ") allowed for device ", +device_id_);
  }
  if (configuration_->burst_size() == 0)
    return arrow::Status::Invalid("Burst size must be greater than 0");
  if (configuration_->codec() != Codec::DEFLATE && configuration_->codec() != Codec::LZ4 &&
      configuration_->codec() != Codec::ZSTD)
    return arrow::Status::NotImplemented("Compress device ", +device_id_,
                                         " does not support the codec");
  if (configuration_->max_sgl_segs() < 1) configuration_->set_max_sgl_segs(1);
  // chained ops: an op of max_sgl_segs segments is one stream, so it must fit a segment
  // kernel (the reference asks the PMD for RTE_COMP_FF_OOP_SGL_IN_SGL_OUT, device.cc:377-380)
  if (std::uint64_t{configuration_->max_sgl_segs()} * configuration_->decompressed_seg_size() >
      internal::kMaxSegSize32) {
    return arrow::Status::Invalid("Compress device does not support chained mbufs of more than ",
                                  internal::kMaxSegSize32, " bytes per operation.");
  }
  if (configuration_->decompressed_seg_size() < internal::kMinSegSize ||
      configuration_->decompressed_seg_size() > internal::kMaxSegSize32) {
    return arrow::Status::Invalid("decompressed_seg_size is not in the range of [",
                                  internal::kMinSegSize, ", ", internal::kMaxSegSize32, "]");
  }
  // level: LZ4 1..9 (>= 2 selects the wide parse); DEFLATE and ZSTD have one level, so any
  // other value is refused rather than ignored (the reference always sets 1)
  if (configuration_->level() < 1 || configuration_->level() > 9)
    return arrow::Status::Invalid("level is not in the range of [1, 9]");
  if (configuration_->codec() != Codec::LZ4 && configuration_->level() != 1)
    return arrow::Status::Invalid("level is not in the range of [1, 1] for this codec");
  // window log (reference device.cc:389-393): 0 asks for the device's maximum, which here is
  // the reach of the encoder this configuration runs (bitar_hip_max_distance: 2560 B -> 2^12,
  // the wide LZ4 parse 14848 B -> 2^14); a requested window is validated and kept as the
  // reference keeps it.  Any window from the reach up to the format's maximum (DEFLATE 2^15,
  // LZ4 / single-segment Zstd 2^16) is honoured -- every stream the encoder writes is valid for
  // it, and the decoders take the format's full window -- a smaller one is refused.
  // encoder_window() reports the reach whatever was requested.
  const std::uint32_t reach = bitar_hip_max_distance(internal::AbiCodec(*configuration_));
  std::uint8_t window = 1;
  while ((1u << window) < reach) ++window;
  encoder_window_ = window;
  const std::uint8_t max_window = configuration_->codec() == Codec::DEFLATE ? 15 : 16;
  if (configuration_->window_size() == 0) {
    configuration_->set_window_size(window);
  } else if (configuration_->window_size() < window || configuration_->window_size() > max_window) {
    return arrow::Status::Invalid("window_size is not in the range of [", +window, ", ",
                                  +max_window, "]");
  }
  if (configuration_->max_preallocate_memzones() < internal::kMinPreallocateSlots) {
    return arrow::Status::Invalid("max_preallocate_memzones (",
                                  configuration_->max_preallocate_memzones(),
                                  ") is not in the range of [", internal::kMinPreallocateSlots,
                                  ", ", internal::kMaxPreallocateSlots, "]");
  }
  return arrow::Status::OK();
}

template <typename Class, typename Enable>
arrow::Status CompressDevice<Class, Enable>::set_configuration(
    std::unique_ptr<Configuration<Class>> configuration) {
  if (!configuration) return arrow::Status::Invalid("null configuration");
  configuration_ = std::move(configuration);
  return arrow::Status::OK();
}

template class CompressDevice<Class_HIP_GFX950>;

DeviceManager* DeviceManager::Instance() {
  static DeviceManager instance;
  return &instance;
}

template <>
arrow::Result<HipGfx950CompressDevice*> DeviceManager::Create<Class_HIP_GFX950>(
    std::uint8_t device_id, std::vector<std::uint32_t> worker_lcores) {
  return new HipCompressDevice(device_id, std::move(worker_lcores));
}

arrow::Status HipCompressDevice::ValidateConfiguration() {
  const auto* hip_configuration = dynamic_cast<HipConfiguration*>(configuration().get());
  if (ARROW_PREDICT_FALSE(hip_configuration == nullptr))
    return arrow::Status::Invalid("Invalid configuration for HipCompressDevice");
  // every rte_comp_checksum_type is supported (checksum.hip); see checksums()
  return HipGfx950CompressDevice::ValidateConfiguration();
}

std::uint32_t HipCompressDevice::checksum_kind() const {
  const auto* c = dynamic_cast<const HipConfiguration*>(configuration().get());
  if (!c) return 0;
  switch (c->checksum_type()) {
    case ChecksumType::CRC32: return BITAR_HIP_CHECKSUM_CRC32;
    case ChecksumType::ADLER32: return BITAR_HIP_CHECKSUM_ADLER32;
    case ChecksumType::CRC32_ADLER32: return BITAR_HIP_CHECKSUM_CRC32_ADLER32;
    default: return 0;
  }
}

arrow::Status HipCompressDevice::set_configuration(
    std::unique_ptr<Configuration<Class_HIP_GFX950>> configuration) {
  if (!configuration) return arrow::Status::Invalid("null configuration");
  if (configuration->type_name() != kHipConfigurationTypeName) {
    return arrow::Status::Invalid("Configuration of type ", configuration->type_name(),
                                  " cannot be applied to compress device of type ",
                                  kHipConfigurationTypeName);
  }
  return HipGfx950CompressDevice::set_configuration(std::move(configuration));
}

}  // namespace bitar
