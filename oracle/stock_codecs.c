/*
 * stock_codecs.c -- the STOCK third-party codecs (liblz4 1.9.3, zlib 1.2.11, libzstd 1.4.x of
 * this image), segment-parallel on host threads.  TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * Used by bench.py (cpu_baseline leg: the CPU baseline the reference's software path would
 * be -- zlib raw DEFLATE level 1 at 59460-B segments is the reference's codec,
 * reference src/config.cc:83-105 + apps/app_common.h:39; liblz4 default at 64 KiB is the
 * north-star codec; and the host-side preparation of stock streams that the GPU decoders
 * are timed on) and by the tests (stock streams for GPU decode parity).  The product never
 * links it.
 *
 * Threading mirrors the reference's lcores: `threads` POSIX threads, static
 * round-robin over segments; every segment is one independent stateless op
 * (reference src/memory.cc:110).
 */
#include <lz4.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>
#include <zstd.h>

enum { SC_LZ4 = 1, SC_DEFLATE = 2, SC_ZSTD = 3 };

typedef struct {
  int codec, level, compress, tid, threads;
  const uint8_t* in;
  uint64_t n;
  uint32_t seg, nseg;
  uint8_t* slab;
  uint64_t stride;
  uint32_t* sizes;
  uint8_t* out;
  int err;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  z_stream zs;
  int zinit = 0;
  ZSTD_CCtx* cc = NULL;
  ZSTD_DCtx* dc = NULL;
  memset(&zs, 0, sizeof(zs));
  if (j->codec == SC_DEFLATE) {
    zinit = j->compress ? deflateInit2(&zs, j->level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY)
                        : inflateInit2(&zs, -15);
    if (zinit != Z_OK) { j->err = -1; return NULL; }
  } else if (j->codec == SC_ZSTD) {
    if (j->compress) cc = ZSTD_createCCtx(); else dc = ZSTD_createDCtx();
  }
  for (uint32_t i = (uint32_t)j->tid; i < j->nseg; i += (uint32_t)j->threads) {
    const uint64_t off = (uint64_t)i * j->seg;
    const uint32_t len = (uint32_t)(j->n - off < j->seg ? j->n - off : j->seg);
    uint8_t* slot = j->slab + (uint64_t)i * j->stride;
    if (j->compress) {
      const uint8_t* src = j->in + off;
      uint64_t c = 0;
      if (j->codec == SC_LZ4) {
        int r = LZ4_compress_default((const char*)src, (char*)slot, (int)len, (int)j->stride);
        if (r <= 0) { j->err = -1; break; }
        c = (uint64_t)r;
      } else if (j->codec == SC_DEFLATE) {
        deflateReset(&zs);
        zs.next_in = (Bytef*)src;
        zs.avail_in = len;
        zs.next_out = slot;
        zs.avail_out = (uInt)j->stride;
        if (deflate(&zs, Z_FINISH) != Z_STREAM_END) { j->err = -1; break; }
        c = zs.total_out;
      } else {
        size_t r = ZSTD_compressCCtx(cc, slot, j->stride, src, len, j->level);
        if (ZSTD_isError(r)) { j->err = -1; break; }
        c = r;
      }
      j->sizes[i] = (uint32_t)c;
    } else {
      /* capacity: this segment's own length (the last one may be short; libzstd >= 1.5
       * may stage literals in the tail of dst up to the capacity it is given) */
      uint8_t* dst = j->out + off;
      const uint32_t csz = j->sizes[i];
      uint64_t p = 0;
      if (j->codec == SC_LZ4) {
        int r = LZ4_decompress_safe((const char*)slot, (char*)dst, (int)csz, (int)len);
        if (r < 0) { j->err = -1; break; }
        p = (uint64_t)r;
      } else if (j->codec == SC_DEFLATE) {
        inflateReset(&zs);
        zs.next_in = slot;
        zs.avail_in = csz;
        zs.next_out = dst;
        zs.avail_out = (uInt)len;
        if (inflate(&zs, Z_FINISH) != Z_STREAM_END) { j->err = -1; break; }
        p = zs.total_out;
      } else {
        size_t r = ZSTD_decompressDCtx(dc, dst, len, slot, csz);
        if (ZSTD_isError(r)) { j->err = -1; break; }
        p = r;
      }
      if (p != len) { j->err = -1; break; }
    }
  }
  if (j->codec == SC_DEFLATE) {
    if (j->compress) deflateEnd(&zs); else inflateEnd(&zs);
  }
  if (cc) ZSTD_freeCCtx(cc);
  if (dc) ZSTD_freeDCtx(dc);
  return NULL;
}

static int run(job_t* tmpl, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 4096) threads = 4096;
  job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  if (!jobs || !th) { free(jobs); free(th); return -1; }
  int err = 0;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = *tmpl;
    jobs[t].tid = t;
    jobs[t].threads = threads;
    if (threads == 1) worker(&jobs[t]);
    else if (pthread_create(&th[t], NULL, worker, &jobs[t]) != 0) { err = -1; threads = t; break; }
  }
  if (threads > 1 || err)
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  for (int t = 0; t < threads; ++t) if (jobs[t].err) err = jobs[t].err;
  free(jobs);
  free(th);
  return err;
}

/* Worst-case compressed size of one segment of n bytes. */
uint64_t sc_bound(int codec, uint32_t n) {
  if (codec == SC_LZ4) return (uint64_t)LZ4_compressBound((int)n);
  if (codec == SC_DEFLATE) return (uint64_t)compressBound(n) + 64;
  if (codec == SC_ZSTD) return (uint64_t)ZSTD_compressBound(n);
  return 0;
}

/* Compress ceil(n/seg) segments of `in` into slab slots of `stride` bytes; sizes[i] gets
 * each compressed size.  level: zlib / zstd level (ignored for LZ4 = LZ4_compress_default). */
int sc_compress(int codec, int level, const uint8_t* in, uint64_t n, uint32_t seg,
                uint8_t* slab, uint64_t stride, uint32_t* sizes, int threads) {
  job_t j;
  memset(&j, 0, sizeof(j));
  j.codec = codec; j.level = level; j.compress = 1;
  j.in = in; j.n = n; j.seg = seg; j.nseg = (uint32_t)((n + seg - 1) / seg);
  j.slab = slab; j.stride = stride; j.sizes = sizes;
  return run(&j, threads);
}

/* Decompress the slab back into out (n bytes, segment i at i*seg); every segment must
 * decode to its full length. */
int sc_decompress(int codec, const uint8_t* slab, uint64_t stride, const uint32_t* sizes,
                  uint64_t n, uint32_t seg, uint8_t* out, int threads) {
  job_t j;
  memset(&j, 0, sizeof(j));
  j.codec = codec; j.compress = 0;
  j.n = n; j.seg = seg; j.nseg = (uint32_t)((n + seg - 1) / seg);
  j.slab = (uint8_t*)slab; j.stride = stride; j.sizes = (uint32_t*)sizes; j.out = out;
  return run(&j, threads);
}
