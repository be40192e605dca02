// pipe.cpp — end-to-end decode from host memory (include/mtblx.h, mtblx_pipe_decode): an
// mtbl file in host memory in, the caller's host byte slices out, i.e. the PCIe-inclusive
// rate BASELINE.json's north_star asks for beside the device-resident one.
//
// Reference path it replaces, per data block (ReaderIntoIter::next -> block_at_index ->
// Reader::block -> Block::init -> BlockIter scan):
//   Reader::block       /root/reference/src/reader.rs:140-175   framing, crc32c, decompress
//   decompress          src/compression.rs:57-68 (snappy :116-119)   -> host, this file
//   Block::init + scan  src/block.rs:16-238                          -> device, decode.hip
// (framing and the checksum are the caller's: the directory holds each block's stored-content
// window, as mtblx_block_dir / mtblx_writer_block_dir produce it, and mtblx_crc32c_blocks
// verifies stored bytes on the device.)
//
// Consecutive blocks are cut into chunks.  Each chunk goes through
//   host   stage into a pinned slot: nothing for a pinned uncompressed source (the H2D reads
//          the file in place), a parallel copy for a pageable one, parallel snappy
//          decompression for CompressionType::Snappy
//   s_h2d  directory + bytes, host -> device
//   s_dec  mtblx_decode_blocks, then the chunk totals -> pinned host
// With MTBLX_PIPE_DEVICE_SNAPPY a snappy file crosses PCIe as stored (compressed) and is
// decompressed on the device (mtblx_snappy_decompress_dev, snappy_dev.hip) right before the
// decode, on s_dec: the host stage is then the same as for an uncompressed file.
//   s_d2h  rebase of the chunk's per-block bases to file-global ones, then every output ->
//          the caller's host arrays at the running offsets
// with kSlots chunks in flight, so the host stage of chunk i+1, the H2D and decode of chunk i
// and the D2H of chunk i-1 overlap (H2D and D2H use separate DMA engines).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "mtblx.h"
#include "bounds.h"
#include "mtblx_host.h"


namespace {

constexpr int kSlots = 3;

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// persistent host workers for the staging stage (copies / decompression)
class Pool {
 public:
  explicit Pool(uint32_t n) : n_(std::max<uint32_t>(1, n)) {
    for (uint32_t t = 1; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& x : th_) x.join();
  }
  uint32_t size() const { return n_; }
  // f(t, n) on every worker t in [0, n) (t = 0 is the caller); returns when all are done
  void run(const std::function<void(uint32_t, uint32_t)>& f) {
    if (n_ == 1) {
      f(0, 1);
      return;
    }
    {
      std::lock_guard<std::mutex> l(mu_);
      job_ = &f;
      left_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    f(0, n_);
    std::unique_lock<std::mutex> l(mu_);
    done_.wait(l, [&] { return left_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(uint32_t t) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(uint32_t, uint32_t)>* j;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        j = job_;
      }
      (*j)(t, n_);
      std::lock_guard<std::mutex> l(mu_);
      if (--left_ == 0) done_.notify_one();
    }
  }
  uint32_t n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(uint32_t, uint32_t)>* job_ = nullptr;
  uint64_t gen_ = 0;
  uint32_t left_ = 0;
  bool stop_ = false;
};

inline uint64_t up256(uint64_t x) { return (x + 255) & ~255ull; }

struct Caps {
  uint64_t in = 0, blocks = 0, rec = 0, keys = 0, vals = 0;
};

// output capacities for a chunk of `in` uncompressed bytes in `blocks` blocks: every entry
// has a >= 3-byte header and its value bytes come from the block; keys can exceed the input
// (shared prefixes), so 2x is a starting point and an overflowing chunk is re-run exactly
Caps caps_for(uint64_t in, uint64_t blocks) {
  Caps c;
  c.in = in;
  c.blocks = blocks;
  c.rec = in / 3 + blocks + 1;
  c.keys = 2 * in + 4096;
  c.vals = in + 64;
  return c;
}

struct Slot {
  uint8_t* h = nullptr;       // pinned staging: dir (off u64[blocks] | len u32[blocks]) | dir2 | data
  uint8_t* d = nullptr;       // device copy of the staging layout
  uint8_t* du = nullptr;      // device snappy: decompressed blocks (16-byte aligned starts)
  uint8_t* dz = nullptr;      // device snappy: dec_len u32[blocks] | status i32[blocks]
  int32_t* hz = nullptr;      // device snappy: pinned copy of the status
  uint8_t* dout = nullptr;    // device outputs
  uint64_t* htot = nullptr;   // pinned chunk totals [4]
  Caps cap;
  mtblx_decoded o{};
  hipEvent_t e_h2d = nullptr, e_dec0 = nullptr, e_dec = nullptr, e_d2h = nullptr;
  bool busy = false;          // e_d2h pending for a previous chunk
  uint64_t dir_bytes() const { return up256(cap.blocks * 12); }
  // dir2 (device snappy): decompressed layout dst_off u64[blocks] | dst_len u32[blocks]
  uint64_t data_at() const { return 2 * dir_bytes(); }
  uint64_t du_bytes() const { return cap.in + 16 * cap.blocks + 64; }
};

__global__ void k_rebase(uint64_t* rb, uint64_t* kb, uint64_t* vb, uint32_t n, uint64_t r0, uint64_t k0,
                         uint64_t v0) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    rb[i] += r0;
    kb[i] += k0;
    vb[i] += v0;
  }
}

struct Chunk {
  uint32_t b0, nb;
  uint64_t lo, hi;     // uncompressed: file range holding the chunk's blocks
  uint64_t ubytes;     // uncompressed content bytes (packed, snappy)
  uint32_t maxlen;
};

}  // namespace

struct mtblx_pipe {
  uint64_t chunk_bytes = 64ull << 20;
  uint32_t max_blocks = 1u << 16;
  int dev = 0;
  int dev_snappy = 2;   // MTBLX_PIPE_DEVICE_SNAPPY: 0 host, 1 device, 2 auto (= the device, measured faster on both)
  hipStream_t s_h2d = nullptr, s_dec = nullptr, s_d2h = nullptr;
  Slot slot[kSlots];
  void* ws = nullptr;
  size_t ws_bytes = 0;
  Pool pool;
  uint32_t threads;
  explicit mtblx_pipe(uint32_t nthreads) : pool(nthreads), threads(nthreads) {}
};

namespace {

void free_outputs(Slot& s) {
  if (s.dout) (void)hipFree(s.dout);
  s.dout = nullptr;
}

int alloc_outputs(Slot& s, const Caps& c) {
  free_outputs(s);
  uint64_t off = 0;
  auto take = [&](uint64_t n) {
    const uint64_t o = off;
    off += up256(n ? n : 1);
    return o;
  };
  const uint64_t o_nrec = take(4 * c.blocks), o_st = take(4 * c.blocks), o_rb = take(8 * c.blocks),
                 o_kb = take(8 * c.blocks), o_vb = take(8 * c.blocks), o_tot = take(32), o_ke = take(4 * c.rec),
                 o_ve = take(4 * c.rec), o_k = take(c.keys), o_v = take(c.vals);
  if (hipMalloc(&s.dout, off) != hipSuccess) return MTBLX_E_HIP;
  uint8_t* b = s.dout;
  s.o.nrec = reinterpret_cast<uint32_t*>(b + o_nrec);
  s.o.status = reinterpret_cast<int32_t*>(b + o_st);
  s.o.rec_base = reinterpret_cast<uint64_t*>(b + o_rb);
  s.o.key_base = reinterpret_cast<uint64_t*>(b + o_kb);
  s.o.val_base = reinterpret_cast<uint64_t*>(b + o_vb);
  s.o.totals = reinterpret_cast<uint64_t*>(b + o_tot);
  s.o.key_end = reinterpret_cast<uint32_t*>(b + o_ke);
  s.o.val_end = reinterpret_cast<uint32_t*>(b + o_ve);
  s.o.keys = b + o_k;
  s.o.vals = b + o_v;
  s.o.rec_cap = c.rec;
  s.o.keys_cap = c.keys;
  s.o.vals_cap = c.vals;
  s.cap.rec = c.rec;
  s.cap.keys = c.keys;
  s.cap.vals = c.vals;
  return MTBLX_OK;
}

void free_slot(Slot& s) {
  if (s.h) (void)hipHostFree(s.h);
  if (s.d) (void)hipFree(s.d);
  free_outputs(s);
  if (s.htot) (void)hipHostFree(s.htot);
  if (s.hz) (void)hipHostFree(s.hz);
  if (s.du) (void)hipFree(s.du);
  if (s.dz) (void)hipFree(s.dz);
  for (hipEvent_t* e : {&s.e_h2d, &s.e_dec0, &s.e_dec, &s.e_d2h})
    if (*e) (void)hipEventDestroy(*e);
  s = Slot();
}

int alloc_slot(Slot& s, const Caps& c) {
  free_slot(s);
  s.cap = c;
  const uint64_t inb = s.data_at() + c.in + 64;
  if (hipHostMalloc(reinterpret_cast<void**>(&s.h), inb, hipHostMallocDefault) != hipSuccess) return MTBLX_E_HIP;
  if (hipMalloc(reinterpret_cast<void**>(&s.d), inb) != hipSuccess) return MTBLX_E_HIP;
  if (hipHostMalloc(reinterpret_cast<void**>(&s.htot), 32, hipHostMallocDefault) != hipSuccess) return MTBLX_E_HIP;
  if (hipHostMalloc(reinterpret_cast<void**>(&s.hz), 4 * c.blocks + 4, hipHostMallocDefault) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&s.du), s.du_bytes()) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&s.dz), 8 * c.blocks + 8) != hipSuccess)
    return MTBLX_E_HIP;
  if (hipEventCreateWithFlags(&s.e_h2d, hipEventDisableTiming) != hipSuccess) return MTBLX_E_HIP;
  if (hipEventCreateWithFlags(&s.e_d2h, hipEventDisableTiming) != hipSuccess) return MTBLX_E_HIP;
  if (hipEventCreate(&s.e_dec0) != hipSuccess || hipEventCreate(&s.e_dec) != hipSuccess) return MTBLX_E_HIP;
  return alloc_outputs(s, c);
}

bool host_pinned(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

}  // namespace

extern "C" mtblx_pipe* mtblx_pipe_new(uint64_t chunk_bytes, uint32_t max_blocks, uint32_t threads) {
  if (mtblx_device_ok() != 1) return nullptr;
  mtblx_pipe* p = new mtblx_pipe(threads ? threads : 16);
  if (chunk_bytes) p->chunk_bytes = chunk_bytes;
  if (max_blocks) p->max_blocks = max_blocks;
  (void)hipGetDevice(&p->dev);
  bool ok = hipStreamCreateWithFlags(&p->s_h2d, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&p->s_dec, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&p->s_d2h, hipStreamNonBlocking) == hipSuccess;
  const Caps c = caps_for(p->chunk_bytes + 16ull * p->max_blocks + 64, p->max_blocks);
  for (int i = 0; ok && i < kSlots; ++i) ok = alloc_slot(p->slot[i], c) == MTBLX_OK;
  p->ws_bytes = mtblx_decode_workspace_bytes(p->max_blocks);
  ok = ok && hipMalloc(&p->ws, p->ws_bytes) == hipSuccess && hipMemset(p->ws, 0, p->ws_bytes) == hipSuccess;
  if (!ok) {
    mtblx_pipe_free(p);
    return nullptr;
  }
  return p;
}

extern "C" void mtblx_pipe_free(mtblx_pipe* p) {
  if (!p) return;
  (void)hipSetDevice(p->dev);
  for (hipStream_t s : {p->s_h2d, p->s_dec, p->s_d2h})
    if (s) (void)hipStreamSynchronize(s);
  for (auto& s : p->slot) free_slot(s);
  if (p->ws) (void)hipFree(p->ws);
  for (hipStream_t s : {p->s_h2d, p->s_dec, p->s_d2h})
    if (s) (void)hipStreamDestroy(s);
  delete p;
}

extern "C" int mtblx_pipe_decode(mtblx_pipe* p, const uint8_t* file, uint64_t file_len, uint32_t compression,
                                 const uint64_t* blk_off, const uint32_t* blk_len, uint32_t nblk,
                                 const mtblx_decoded* out, mtblx_pipe_stats* stats) {
  if (!p || !out || (nblk && (!file || !blk_off || !blk_len)) || compression > 5) return MTBLX_E_INVAL;
  if (nblk && (!out->nrec || !out->rec_base || !out->key_base || !out->val_base || !out->status || !out->totals))
    return MTBLX_E_INVAL;
  if (compression >= 2) {
    // Zlib / Zstd (and Lz4 / Lz4hc, every block Err): the decompressed lengths are not in the
    // stored bytes, so the whole directory is decompressed first on the host (16 threads,
    // codecs_host.cpp), then streamed as CompressionType::None; failed blocks are
    // MTBLX_ST_DECOMPRESS (Reader::block's Err(Error::Io), src/reader.rs:166)
    const double t0 = now_s();
    std::vector<uint64_t> doff(nblk ? nblk : 1), dlen(nblk ? nblk : 1);
    std::vector<int32_t> zst(nblk ? nblk : 1);
    uint8_t* dbuf = nullptr;
    mtblx_decompress_blocks(compression, file, blk_off, blk_len, nblk, p->threads, &dbuf, doff.data(), dlen.data(),
                            zst.data());
    if (!dbuf) return MTBLX_E_INVAL;
    std::vector<uint32_t> dl(nblk ? nblk : 1);
    uint64_t dtotal = 0;
    for (uint32_t b = 0; b < nblk; ++b) {
      if (dlen[b] > 0xFFFFFFFFull) { free(dbuf); return MTBLX_E_INVAL; }   // >= 4 GiB decompressed block
      dl[b] = (uint32_t)dlen[b];
      dtotal = std::max(dtotal, doff[b] + dlen[b]);
    }
    const double t_dz = now_s() - t0;
    const int rc = mtblx_pipe_decode(p, dbuf, dtotal, 0, doff.data(), dl.data(), nblk, out, stats);
    if (rc == MTBLX_OK) {
      uint32_t bad = 0;
      for (uint32_t b = 0; b < nblk; ++b)
        if (zst[b] != MTBLX_CODEC_OK) { out->status[b] = MTBLX_ST_DECOMPRESS; ++bad; }
      if (stats) {
        stats->stage_seconds += t_dz;
        stats->seconds += t_dz;
        stats->decompress_errors = bad;
      }
    }
    free(dbuf);
    return rc;
  }
  if (hipSetDevice(p->dev) != hipSuccess) return MTBLX_E_HIP;
  const double t_start = now_s();
  mtblx_pipe_stats st{};
  for (uint32_t b = 0; b < nblk; ++b)
    if (blk_off[b] > file_len || blk_len[b] > file_len - blk_off[b]) return MTBLX_E_INVAL;

  // ---- plan: uncompressed lengths, chunk cuts ----
  std::vector<uint64_t> ulen(nblk);
  std::vector<uint8_t> zerr(nblk, 0);
  for (uint32_t b = 0; b < nblk; ++b) {
    if (compression == 0) {
      ulen[b] = blk_len[b];
    } else {
      uint64_t u = 0;
      if (mtblx_snappy_uncompressed_len(file + blk_off[b], blk_len[b], &u) != MTBLX_SNAPPY_OK || u > 0xFFFFFFFFull) {
        zerr[b] = 1;
        u = 0;
      }
      ulen[b] = u;
    }
  }
  // stored bytes H2D + device decompression (mtblx_snappy_decompress_dev) or host decompression.
  // auto = the device: the stored bytes cross PCIe once and the host stage vanishes.  It wins on
  // poorly compressed blocks (cfg5, ~1x: 28.5-32 vs 27 GiB/s end to end) and, since
  // k_snappy_lanes (~320 GB/s of output), on compressible ones too (the bench line's 4.58x
  // stream: 21.1 vs 13.4 GiB/s end to end).  (Round 2's auto kept streams that
  // expand > 2x on the host, when the device decompressor ran ~170 GB/s.)
  const bool dz_mode = compression == 1 && p->dev_snappy != 0;
  const bool ranged = compression == 0 || dz_mode;
  std::vector<Chunk> chunks;
  Caps need;
  for (uint32_t b = 0; b < nblk;) {
    Chunk c{b, 0, blk_off[b], blk_off[b], 0, 0};
    while (b < nblk && c.nb < p->max_blocks) {
      const uint64_t u = ulen[b];
      const uint64_t nhi = std::max(c.hi, blk_off[b] + blk_len[b]);
      const uint64_t range = nhi - std::min(c.lo, blk_off[b]);
      const uint64_t span = compression == 0 ? range
                            : dz_mode   ? std::max<uint64_t>(range, c.ubytes + u + 16ull * (c.nb + 1))
                                        : c.ubytes + u;
      if (c.nb > 0 && span > p->chunk_bytes) break;
      // chunks shipped as stored are one contiguous file range: blocks must be in file order
      if (ranged && c.nb > 0 && blk_off[b] < c.hi) break;
      c.lo = std::min(c.lo, blk_off[b]);
      c.hi = nhi;
      c.ubytes += u;
      c.maxlen = (uint32_t)std::max<uint64_t>(c.maxlen, u);
      ++c.nb;
      ++b;
    }
    const uint64_t in = compression == 0 ? c.hi - c.lo
                        : dz_mode   ? std::max<uint64_t>(c.hi - c.lo, c.ubytes + 16ull * c.nb)
                                    : c.ubytes;
    need.in = std::max(need.in, in);
    st.block_bytes += c.ubytes;
    chunks.push_back(c);
  }
  // grow the slots for an oversize chunk (a single block larger than chunk_bytes)
  if (need.in > p->slot[0].cap.in) {
    for (hipStream_t s : {p->s_h2d, p->s_dec, p->s_d2h}) (void)hipStreamSynchronize(s);
    const Caps c = caps_for(need.in, p->max_blocks);
    for (auto& s : p->slot)
      if (alloc_slot(s, c) != MTBLX_OK) return MTBLX_E_HIP;
  }
  const bool pinned_src = ranged && nblk && host_pinned(file);

  uint64_t R = 0, K = 0, V = 0, flags = 0;
  std::vector<std::pair<uint32_t, uint32_t>> skipped;   // chunks whose outputs did not fit `out`
  int rc = MTBLX_OK;

  // ---- stage + H2D + decode of chunk i ----
  auto enqueue = [&](size_t i) -> int {
    Slot& s = p->slot[i % kSlots];
    const Chunk& c = chunks[i];
    if (s.busy) {   // the slot's previous chunk: its D2H (hence its decode) must be complete
      if (hipEventSynchronize(s.e_d2h) != hipSuccess) return MTBLX_E_HIP;
      s.busy = false;
    }
    const double t0 = now_s();
    uint64_t* doff = reinterpret_cast<uint64_t*>(s.h);
    uint32_t* dlen = reinterpret_cast<uint32_t*>(s.h + 8 * s.cap.blocks);
    uint8_t* hdata = s.h + s.data_at();
    uint64_t* zoff = reinterpret_cast<uint64_t*>(s.h + s.dir_bytes());            // dz_mode: dst_off
    uint32_t* zlen = reinterpret_cast<uint32_t*>(s.h + s.dir_bytes() + 8 * s.cap.blocks);   // dst_len
    uint64_t ubytes = 0;
    const uint8_t* src = hdata;
    uint64_t bytes;
    if (ranged) {
      for (uint32_t j = 0; j < c.nb; ++j) {
        doff[j] = blk_off[c.b0 + j] - c.lo;
        dlen[j] = blk_len[c.b0 + j];
      }
      if (dz_mode) {   // the decompressed layout: 16-byte aligned starts, lengths from the preambles
        for (uint32_t j = 0; j < c.nb; ++j) {
          const uint32_t u = zerr[c.b0 + j] ? 0u : (uint32_t)ulen[c.b0 + j];
          zoff[j] = ubytes;
          zlen[j] = u;
          ubytes += (u + 15ull) & ~15ull;
        }
      }
      bytes = c.hi - c.lo;
      if (pinned_src) {
        src = file + c.lo;
      } else {
        p->pool.run([&](uint32_t t, uint32_t n) {
          const uint64_t a = bytes * t / n, e = bytes * (t + 1) / n;
          memcpy(hdata + a, file + c.lo + a, e - a);
        });
      }
    } else {
      uint64_t pos = 0;
      for (uint32_t j = 0; j < c.nb; ++j) {
        doff[j] = pos;
        dlen[j] = (uint32_t)ulen[c.b0 + j];
        pos += ulen[c.b0 + j];
      }
      bytes = pos;
      p->pool.run([&](uint32_t t, uint32_t n) {
        const uint32_t j0 = (uint32_t)((uint64_t)c.nb * t / n), j1 = (uint32_t)((uint64_t)c.nb * (t + 1) / n);
        for (uint32_t j = j0; j < j1; ++j) {
          const uint32_t b = c.b0 + j;
          if (zerr[b]) continue;
          uint64_t got = 0;
          const int r = mtblx_snappy_decompress(file + blk_off[b], blk_len[b], hdata + doff[j], ulen[b], &got);
          if (r != MTBLX_SNAPPY_OK || got != ulen[b]) {
            zerr[b] = 1;   // distinct bytes per thread
            dlen[j] = 0;   // decoded as an empty content (INVALID_BLOCK), reported as DECOMPRESS
          }
        }
      });
    }
    st.stage_seconds += now_s() - t0;
    hipStream_t sh = p->s_h2d, sd = p->s_dec;
    const uint64_t lens_at = 8 * s.cap.blocks;
    for (int half = 0; half < (dz_mode ? 2 : 1); ++half) {
      const uint64_t h0 = half * s.dir_bytes();
      if (hipMemcpyAsync(s.d + h0, s.h + h0, 8ull * c.nb, hipMemcpyHostToDevice, sh) != hipSuccess ||
          hipMemcpyAsync(s.d + h0 + lens_at, s.h + h0 + lens_at, 4ull * c.nb, hipMemcpyHostToDevice, sh) != hipSuccess)
        return MTBLX_E_HIP;
      st.h2d_bytes += 12ull * c.nb;
    }
    if (bytes && hipMemcpyAsync(s.d + s.data_at(), src, bytes, hipMemcpyHostToDevice, sh) != hipSuccess)
      return MTBLX_E_HIP;
    st.h2d_bytes += bytes;
    if (hipEventRecord(s.e_h2d, sh) != hipSuccess || hipStreamWaitEvent(sd, s.e_h2d, 0) != hipSuccess)
      return MTBLX_E_HIP;
    mtblx_block_batch in{s.d + s.data_at(), bytes ? bytes : 1, reinterpret_cast<const uint64_t*>(s.d),
                         reinterpret_cast<const uint32_t*>(s.d + 8 * s.cap.blocks), c.nb, c.maxlen};
    (void)hipEventRecord(s.e_dec0, sd);
    if (dz_mode) {   // Reader::block's decompression (src/reader.rs:166-170) on the device
      uint32_t* dec_len = reinterpret_cast<uint32_t*>(s.dz);
      int32_t* zst = reinterpret_cast<int32_t*>(s.dz + 4 * s.cap.blocks);
      const uint64_t* d_zoff = reinterpret_cast<const uint64_t*>(s.d + s.dir_bytes());
      const uint32_t* d_zlen = reinterpret_cast<const uint32_t*>(s.d + s.dir_bytes() + lens_at);
      int rz = mtblx_snappy_decompress_dev(s.d + s.data_at(), in.blk_off, in.blk_len, c.nb, s.du, d_zoff, d_zlen,
                                           c.maxlen, zst, dec_len, sd);
      if (rz != MTBLX_OK) return rz;
      if (hipMemcpyAsync(s.hz, zst, 4ull * c.nb, hipMemcpyDeviceToHost, sd) != hipSuccess) return MTBLX_E_HIP;
      in = mtblx_block_batch{s.du, std::max<uint64_t>(ubytes, 1), d_zoff, dec_len, c.nb, c.maxlen};
    }
    int r = mtblx_decode_blocks(&in, &s.o, p->ws, p->ws_bytes, sd);
    if (r != MTBLX_OK) return r;
    if (hipMemcpyAsync(s.htot, s.o.totals, 32, hipMemcpyDeviceToHost, sd) != hipSuccess) return MTBLX_E_HIP;
    if (hipEventRecord(s.e_dec, sd) != hipSuccess) return MTBLX_E_HIP;
    return MTBLX_OK;
  };

  // ---- outputs of chunk i -> the caller's arrays ----
  auto drain = [&](size_t i) -> int {
    Slot& s = p->slot[i % kSlots];
    const Chunk& c = chunks[i];
    if (hipEventSynchronize(s.e_dec) != hipSuccess) return MTBLX_E_HIP;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, s.e_dec0, s.e_dec) == hipSuccess) st.decode_ms += ms;
    if (dz_mode)   // device decompression failures: Err(Error::Io), the block decoded as empty
      for (uint32_t j = 0; j < c.nb; ++j) {
        if (s.hz[j] == MTBLX_SNAPPY_TIMEOUT) return MTBLX_E_TIMEOUT;   // an internal wait gave up
        if (s.hz[j] != MTBLX_SNAPPY_OK) zerr[c.b0 + j] = 1;
      }
    uint64_t nr = s.htot[0], kb = s.htot[1], vb = s.htot[2];
    if (s.htot[3] & 3ull) {
      // bit 0: the slot's output capacity was too small (keys far longer than the block bytes):
      // totals hold the exact sizes, so grow the slot and decode the chunk again.
      // bit 1: the launch's look-back timed out (mtblx.h): its outputs are discarded and the
      // chunk is decoded again as a fresh launch; a second timeout fails the call.
      Caps c2 = s.cap;
      if (s.htot[3] & 1ull) {
        c2.rec = std::max(c2.rec, nr + 1);
        c2.keys = std::max(c2.keys, kb + 64);
        c2.vals = std::max(c2.vals, vb + 64);
      }
      const bool grow = (s.htot[3] & 1ull) != 0;
      if (hipStreamSynchronize(p->s_d2h) != hipSuccess || (grow && alloc_outputs(s, c2) != MTBLX_OK))
        return MTBLX_E_HIP;
      mtblx_block_batch in{s.d + s.data_at(), std::max<uint64_t>(compression == 0 ? c.hi - c.lo : c.ubytes, 1),
                           reinterpret_cast<const uint64_t*>(s.d),
                           reinterpret_cast<const uint32_t*>(s.d + 8 * s.cap.blocks), c.nb, c.maxlen};
      if (dz_mode)
        in = mtblx_block_batch{s.du, s.du_bytes(), reinterpret_cast<const uint64_t*>(s.d + s.dir_bytes()),
                               reinterpret_cast<const uint32_t*>(s.dz), c.nb, c.maxlen};
      int r = mtblx_decode_blocks(&in, &s.o, p->ws, p->ws_bytes, p->s_dec);
      if (r != MTBLX_OK) return r;
      if (hipMemcpyAsync(s.htot, s.o.totals, 32, hipMemcpyDeviceToHost, p->s_dec) != hipSuccess ||
          hipEventRecord(s.e_dec, p->s_dec) != hipSuccess || hipEventSynchronize(s.e_dec) != hipSuccess)
        return MTBLX_E_HIP;
      nr = s.htot[0];
      kb = s.htot[1];
      vb = s.htot[2];
      if (s.htot[3] & 2ull) return MTBLX_E_TIMEOUT;
    }
    flags |= s.htot[3] & ~1ull;
    hipStream_t so = p->s_d2h;
    if (hipStreamWaitEvent(so, s.e_dec, 0) != hipSuccess) return MTBLX_E_HIP;
    const bool fits = R + nr <= out->rec_cap && K + kb <= out->keys_cap && V + vb <= out->vals_cap &&
                      (!nr || (out->key_end && out->val_end)) && (!kb || out->keys) && (!vb || out->vals);
    MTBLX_LAUNCH((s.o.rec_base, s.o.key_base, s.o.val_base), k_rebase, dim3((c.nb + 255) / 256), dim3(256), 0, so, s.o.rec_base, s.o.key_base, s.o.val_base,
                       c.nb, R, K, V);
    auto d2h = [&](void* dst, const void* srcp, uint64_t n) {
      st.d2h_bytes += n;
      return n == 0 || hipMemcpyAsync(dst, srcp, n, hipMemcpyDeviceToHost, so) == hipSuccess;
    };
    bool ok = d2h(out->nrec + c.b0, s.o.nrec, 4ull * c.nb) && d2h(out->status + c.b0, s.o.status, 4ull * c.nb) &&
              d2h(out->rec_base + c.b0, s.o.rec_base, 8ull * c.nb) &&
              d2h(out->key_base + c.b0, s.o.key_base, 8ull * c.nb) &&
              d2h(out->val_base + c.b0, s.o.val_base, 8ull * c.nb);
    if (fits) {
      ok = ok && d2h(out->key_end + R, s.o.key_end, 4 * nr) && d2h(out->val_end + R, s.o.val_end, 4 * nr) &&
           d2h(out->keys + K, s.o.keys, kb) && d2h(out->vals + V, s.o.vals, vb);
    } else {
      skipped.emplace_back(c.b0, c.nb);
      flags |= 1ull;
    }
    if (!ok || hipEventRecord(s.e_d2h, so) != hipSuccess) return MTBLX_E_HIP;
    s.busy = true;
    R += nr;
    K += kb;
    V += vb;
    return MTBLX_OK;
  };

  for (size_t i = 0; i < chunks.size() && rc == MTBLX_OK; ++i) {
    rc = enqueue(i);
    if (rc == MTBLX_OK && i > 0) rc = drain(i - 1);
  }
  if (rc == MTBLX_OK && !chunks.empty()) rc = drain(chunks.size() - 1);
  for (hipStream_t s : {p->s_h2d, p->s_dec, p->s_d2h})
    if (hipStreamSynchronize(s) != hipSuccess) rc = MTBLX_E_HIP;
  for (auto& s : p->slot) s.busy = false;
  if (rc != MTBLX_OK) return rc;
  // per-block outcomes the device could not know
  for (const auto& sk : skipped)
    for (uint32_t j = 0; j < sk.second; ++j) out->status[sk.first + j] = MTBLX_ST_OVERFLOW;
  for (uint32_t b = 0; b < nblk; ++b)
    if (zerr[b]) {
      out->status[b] = MTBLX_ST_DECOMPRESS;
      ++st.decompress_errors;
    }
  out->totals[0] = R;
  out->totals[1] = K;
  out->totals[2] = V;
  out->totals[3] = flags;
  st.chunks = (uint32_t)chunks.size();
  st.seconds = now_s() - t_start;
  if (stats) *stats = st;
  return MTBLX_OK;
}

extern "C" int mtblx_pipe_set(mtblx_pipe* p, int option, int64_t value) {
  if (!p) return MTBLX_E_INVAL;
  if (option == MTBLX_PIPE_DEVICE_SNAPPY) {
    if (value < 0 || value > 2) return MTBLX_E_INVAL;
    p->dev_snappy = (int)value;
    return MTBLX_OK;
  }
  return MTBLX_E_INVAL;
}

extern "C" int mtblx_host_alloc(void** p, uint64_t bytes) {
  if (!p) return MTBLX_E_INVAL;
  return hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
extern "C" int mtblx_host_free(void* p) { return hipHostFree(p) == hipSuccess ? MTBLX_OK : MTBLX_E_HIP; }
extern "C" int mtblx_host_register(void* p, uint64_t bytes) {
  return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
extern "C" int mtblx_host_unregister(void* p) { return hipHostUnregister(p) == hipSuccess ? MTBLX_OK : MTBLX_E_HIP; }
