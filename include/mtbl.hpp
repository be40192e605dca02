// mtbl.hpp — C++ mirror of oxidized-mtbl's public surface over libmtblx's C ABI.
//
// The reference is a Rust crate; Rust is not in this image, so the host side above the C ABI
// is C++ (header-only, C++17, compiled with hipcc).  Same names, argument meaning and error
// behaviour as the crate, for the path this library accelerates:
//
//   WriterBuilder / Writer      /root/reference/src/writer.rs:15-201   (mtblx_writer_*)
//   ReaderBuilder / Reader      src/reader.rs:15-135                    (footer, framing: host;
//                                                                        index, directory, CRC,
//                                                                        block decode: device)
//   Reader::get                 src/reader.rs:111-122                   (mtblx_get, batched seek)
//   ReaderIntoIter::next        src/reader.rs:337-405                   (records decoded on the
//                                                                        device, served on host)
//   Reader::iter_prefix / iter_range / iter_from                         (binary search over the
//                                                                        decoded, sorted keys)
//   Metadata                    src/metadata.rs:11-24
//   MtblError                   src/error.rs:44-52
//
// Errors: where the crate returns Err(Error::Mtbl(e)) this throws mtbl::Error(e); where it
// returns Err(Error::Io) (a snappy stream snap rejects) it throws mtbl::Error(kIo); where it
// panics (checksum assert_eq, out-of-range slices, corrupt entries, "out-of-order key") it
// throws mtbl::Panic.  Iteration reproduces ReaderIntoIter's end rules exactly (an empty
// block after the first ends it; records yielded before a panic are kept, then Panic).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "mtblx.h"
#include "mtblx_host.h"

namespace mtbl {

using Bytes = std::vector<uint8_t>;

// src/lib.rs:4-8
constexpr uint64_t DEFAULT_BLOCK_RESTART_INTERVAL = 16;
constexpr uint64_t DEFAULT_BLOCK_SIZE = 8192;
constexpr uint64_t MIN_BLOCK_SIZE = 1024;
constexpr uint64_t METADATA_SIZE = 512;

// src/compression.rs:6-15
enum class CompressionType : uint32_t { None = 0, Snappy = 1, Zlib = 2, Lz4 = 3, Lz4hc = 4, Zstd = 5 };

// src/error.rs:44-52 (+ Io)
enum class MtblError : int {
  InvalidMetadataSize = MTBLX_ERR_INVALID_METADATA_SIZE,
  InvalidIndexBlockOffset = MTBLX_ERR_INVALID_INDEX_BLOCK_OFFSET,
  InvalidIndexLength = MTBLX_ERR_INVALID_INDEX_LENGTH,
  InvalidFormatVersion = MTBLX_ERR_INVALID_FORMAT_VERSION,
  InvalidCompressionAlgorithm = MTBLX_ERR_INVALID_COMPRESSION_ALGORITHM,
  InvalidBlock = MTBLX_ERR_INVALID_BLOCK,
  Io = MTBLX_ERR_IO,
};

inline const char* error_name(MtblError e) {
  switch (e) {
    case MtblError::InvalidMetadataSize: return "InvalidMetadataSize";
    case MtblError::InvalidIndexBlockOffset: return "InvalidIndexBlockOffset";
    case MtblError::InvalidIndexLength: return "InvalidIndexLength";
    case MtblError::InvalidFormatVersion: return "InvalidFormatVersion";
    case MtblError::InvalidCompressionAlgorithm: return "InvalidCompressionAlgorithm";
    case MtblError::InvalidBlock: return "InvalidBlock";
    case MtblError::Io: return "Io";
  }
  return "?";
}

struct Error : std::runtime_error {
  MtblError kind;
  explicit Error(MtblError k) : std::runtime_error(error_name(k)), kind(k) {}
};
struct Panic : std::runtime_error {   // where the reference panics
  explicit Panic(const std::string& w) : std::runtime_error(w) {}
};

namespace detail {
inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP: ") + what + ": " + hipGetErrorString(e));
}
inline void abi_check(int rc, const char* what) {
  if (rc != MTBLX_OK) throw std::runtime_error(std::string(what) + " failed: " + std::to_string(rc));
}
// totals[3] bit 1: the launch's look-back timed out and nothing it wrote may be used (mtblx.h)
inline void launch_check(uint64_t flags, const char* what) {
  if (flags & 2ull) throw std::runtime_error(std::string(what) + ": look-back timeout, outputs discarded");
}
// device buffer (hipMalloc), freed with the owner
struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  explicit DevBuf(size_t bytes) : n(bytes) { hip_check(hipMalloc(&p, bytes ? bytes : 1), "hipMalloc"); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { reset(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
    return *this;
  }
  ~DevBuf() { reset(); }
  void reset() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
  template <class T> T* as() const { return static_cast<T*>(p); }
};
template <class T>
inline DevBuf upload(const T* src, size_t count) {
  DevBuf b(count * sizeof(T));
  if (count) hip_check(hipMemcpy(b.p, src, count * sizeof(T), hipMemcpyHostToDevice), "H2D");
  return b;
}
template <class T>
inline std::vector<T> download(const void* src, size_t count) {
  std::vector<T> v(count);
  if (count) hip_check(hipMemcpy(v.data(), src, count * sizeof(T), hipMemcpyDeviceToHost), "D2H");
  return v;
}

// decoded blocks, downloaded to the host (the layout of mtblx_decoded)
struct Decoded {
  std::vector<uint32_t> nrec, key_end, val_end;
  std::vector<uint64_t> rec_base, key_base, val_base;
  std::vector<int32_t> status;
  Bytes keys, vals;
};

// count -> allocate -> decode -> download, for the batch {data, off, len} on the device
inline Decoded decode_batch(const uint8_t* d_data, uint64_t data_len, const uint64_t* d_off, const uint32_t* d_len,
                            uint32_t nblk, uint32_t max_len) {
  Decoded h;
  if (nblk == 0) return h;
  mtblx_block_batch in{d_data, data_len, d_off, d_len, nblk, max_len};
  const size_t wsb = mtblx_decode_workspace_bytes(nblk);
  DevBuf ws(wsb);
  hip_check(hipMemset(ws.p, 0, wsb), "memset");
  DevBuf per(8 * 4 * (size_t)nblk + 32);   // nrec | status | rec_base | key_base | val_base | totals
  uint8_t* b = per.as<uint8_t>();
  mtblx_decoded out{};
  out.nrec = reinterpret_cast<uint32_t*>(b);
  out.status = reinterpret_cast<int32_t*>(b + 4ull * nblk);
  out.rec_base = reinterpret_cast<uint64_t*>(b + 8ull * nblk);
  out.key_base = reinterpret_cast<uint64_t*>(b + 16ull * nblk);
  out.val_base = reinterpret_cast<uint64_t*>(b + 24ull * nblk);
  out.totals = reinterpret_cast<uint64_t*>(b + 32ull * nblk);
  abi_check(mtblx_count_blocks(&in, &out, ws.p, wsb, nullptr), "mtblx_count_blocks");
  hip_check(hipDeviceSynchronize(), "sync");
  const auto tot = download<uint64_t>(out.totals, 4);
  launch_check(tot[3], "mtblx_count_blocks");
  DevBuf ke(4 * tot[0] + 4), ve(4 * tot[0] + 4), kk(tot[1] + 1), vv(tot[2] + 1);
  out.key_end = ke.as<uint32_t>();
  out.val_end = ve.as<uint32_t>();
  out.rec_cap = tot[0];
  out.keys = kk.as<uint8_t>();
  out.keys_cap = tot[1];
  out.vals = vv.as<uint8_t>();
  out.vals_cap = tot[2];
  abi_check(mtblx_decode_blocks(&in, &out, ws.p, wsb, nullptr), "mtblx_decode_blocks");
  hip_check(hipDeviceSynchronize(), "sync");
  launch_check(download<uint64_t>(out.totals, 4)[3], "mtblx_decode_blocks");
  h.nrec = download<uint32_t>(out.nrec, nblk);
  h.status = download<int32_t>(out.status, nblk);
  h.rec_base = download<uint64_t>(out.rec_base, nblk);
  h.key_base = download<uint64_t>(out.key_base, nblk);
  h.val_base = download<uint64_t>(out.val_base, nblk);
  h.key_end = download<uint32_t>(out.key_end, tot[0]);
  h.val_end = download<uint32_t>(out.val_end, tot[0]);
  h.keys = download<uint8_t>(out.keys, tot[1]);
  h.vals = download<uint8_t>(out.vals, tot[2]);
  return h;
}
}  // namespace detail

// ------------------------------------------------------------------ Writer (src/writer.rs)
class Writer {
 public:
  Writer(uint64_t block_size, uint64_t restart_interval, CompressionType c, uint32_t level = 0)
      : w_(mtblx_writer_new(block_size, restart_interval, static_cast<uint32_t>(c))) {
    if (!w_) throw std::invalid_argument("CompressionType: None, Snappy, Zlib, Zstd only (Lz4: the crate's Err)");
    mtblx_writer_set_level(w_, level);
  }
  Writer(const Writer&) = delete;
  Writer& operator=(const Writer&) = delete;
  Writer(Writer&& o) noexcept : w_(o.w_) { o.w_ = nullptr; }
  ~Writer() { if (w_) mtblx_writer_free(w_); }
  static Writer memory();   // WriterBuilder::default().memory()

  // src/writer.rs:112-149; "out-of-order key" panics
  void insert(const uint8_t* key, size_t klen, const uint8_t* val, size_t vlen) {
    if (mtblx_writer_insert(w_, key, klen, val, vlen) != MTBLX_OK) throw Panic("out-of-order key");
  }
  void insert(const Bytes& k, const Bytes& v) { insert(k.data(), k.size(), v.data(), v.size()); }
  void insert(const std::string& k, const std::string& v) {
    insert(reinterpret_cast<const uint8_t*>(k.data()), k.size(), reinterpret_cast<const uint8_t*>(v.data()), v.size());
  }
  // src/writer.rs:155-181: the finished file
  Bytes into_inner() {
    uint8_t* p = nullptr;
    uint64_t n = 0;
    detail::abi_check(mtblx_writer_finish(w_, &p, &n), "mtblx_writer_finish");
    Bytes out(p, p + n);
    mtblx_free(p);
    return out;
  }

 private:
  mtblx_writer* w_;
};

class WriterBuilder {   // src/writer.rs:15-80
 public:
  WriterBuilder& compression_type(CompressionType c) { c_ = c; return *this; }
  WriterBuilder& compression_level(uint32_t l) { level_ = l; return *this; }
  WriterBuilder& block_size(uint64_t n) { bs_ = std::max(n, MIN_BLOCK_SIZE); return *this; }
  WriterBuilder& block_restart_interval(uint64_t n) { iv_ = n; return *this; }
  Writer memory() const { return Writer(bs_, iv_, c_, level_); }

 private:
  CompressionType c_ = CompressionType::None;
  uint64_t bs_ = DEFAULT_BLOCK_SIZE, iv_ = DEFAULT_BLOCK_RESTART_INTERVAL;
  uint32_t level_ = 0;   // DEFAULT_COMPRESSION_LEVEL (src/lib.rs:8)
};
inline Writer Writer::memory() { return WriterBuilder().memory(); }

// ------------------------------------------------------------------ Reader (src/reader.rs)
struct Metadata {   // src/metadata.rs:11-24
  uint64_t index_block_offset, data_block_size, compression_algorithm, count_entries, count_data_blocks,
      bytes_data_blocks, bytes_index_block, bytes_keys, bytes_values;
};

struct Record {   // a (key, value) pair served by the iterators (views into the Reader)
  const uint8_t* key;
  size_t key_len;
  const uint8_t* val;
  size_t val_len;
  Bytes key_bytes() const { return Bytes(key, key + key_len); }
  Bytes val_bytes() const { return Bytes(val, val + val_len); }
};

class Reader;

// ReaderIntoIter (src/reader.rs:219-405) in its Iter mode; next() throws where the reference
// returns Err / panics, after yielding the records it yields before that.
class ReaderIntoIter {
 public:
  std::optional<Record> next();

 private:
  friend class Reader;
  ReaderIntoIter(const Reader* r, size_t i, size_t end) : r_(r), i_(i), end_(end) {}
  const Reader* r_;
  size_t i_, end_;
};

class Reader {
 public:
  // Reader::new (src/reader.rs:99-101): ReaderBuilder::default().read(data), checksums on
  static Reader open(const Bytes& data);
  static Reader open(const uint8_t* data, size_t len);
  Metadata metadata() const { return meta_; }
  ReaderIntoIter into_iter() const { return ReaderIntoIter(this, 0, nrec_); }
  // src/reader.rs:111-122, on the device (mtblx_get: index seek -> block_at_index -> BlockIter::seek)
  std::optional<Bytes> get(const uint8_t* key, size_t klen) const;
  std::optional<Bytes> get(const std::string& k) const {
    return get(reinterpret_cast<const uint8_t*>(k.data()), k.size());
  }
  // ReaderIntoIter's GetPrefix / GetRange / From filters (src/reader.rs:385-402)
  std::vector<Record> iter_prefix(const Bytes& prefix) const;
  std::vector<Record> iter_range(const Bytes& start, const Bytes& end) const;   // end inclusive
  std::vector<Record> iter_from(const Bytes& key) const;
  size_t len() const { return nrec_; }   // records the full iteration yields before it ends

 private:
  friend class ReaderBuilder;
  friend class ReaderIntoIter;
  Reader(const uint8_t* data, size_t len, bool verify);
  Record rec(size_t i) const {
    const uint64_t k0 = i ? gke_[i - 1] : 0, v0 = i ? gve_[i - 1] : 0;
    return Record{dec_.keys.data() + k0, (size_t)(gke_[i] - k0), dec_.vals.data() + v0, (size_t)(gve_[i] - v0)};
  }
  size_t lower_bound(const uint8_t* k, size_t kl) const;
  enum class End { None, ErrOpen, ErrNext, Panic, Loop };
  Bytes file_;
  detail::DevBuf dfile_;
  bool verify_;
  uint32_t version_ = 1;
  Metadata meta_{};
  uint64_t index_off_ = 0, index_len_ = 0;
  detail::Decoded dec_;
  std::vector<uint64_t> gke_, gve_;   // global END offsets of the yielded records
  size_t nrec_ = 0;
  End end_ = End::None;
  MtblError err_ = MtblError::InvalidBlock;
};

class ReaderBuilder {   // src/reader.rs:15-30
 public:
  ReaderBuilder& verify_checksums(bool v) { verify_ = v; return *this; }
  Reader read(const Bytes& data) const { return Reader(data.data(), data.size(), verify_); }
  Reader read(const uint8_t* data, size_t len) const { return Reader(data, len, verify_); }

 private:
  bool verify_ = true;
};

inline Reader Reader::open(const Bytes& data) { return ReaderBuilder().read(data); }
inline Reader Reader::open(const uint8_t* data, size_t len) { return ReaderBuilder().read(data, len); }

inline Reader::Reader(const uint8_t* data, size_t len, bool verify) : file_(data, data + len), verify_(verify) {
  using namespace detail;
  // ReaderBuilder::read (src/reader.rs:31-81): footer, index framing + checksum (host)
  mtblx_footer f{};
  if (mtblx_read_footer(file_.data(), file_.size(), &f) != MTBLX_OK) throw Error(static_cast<MtblError>(f.err));
  std::memcpy(&meta_, f.meta, sizeof(meta_));
  version_ = f.version;
  uint64_t coff = 0, clen = 0;
  int panic = 0;
  const int rc = mtblx_frame_block(file_.data(), file_.size(), version_, meta_.index_block_offset, verify ? 1 : 0,
                                   &coff, &clen, &panic);
  if (panic) throw Panic("index block framing / checksum (src/reader.rs:52-74)");
  if (rc != MTBLX_OK) throw Error(MtblError::InvalidIndexLength);
  index_off_ = coff;
  index_len_ = clen;
  dfile_ = upload(file_.data(), file_.size());
  // the index block, decoded on the device like any block
  const uint64_t ioff = coff;
  const uint32_t ilen = (uint32_t)clen;
  DevBuf d_ioff = upload(&ioff, 1), d_ilen = upload(&ilen, 1);
  const Decoded idx = decode_batch(dfile_.as<uint8_t>(), file_.size(), d_ioff.as<uint64_t>(), d_ilen.as<uint32_t>(),
                                   1, ilen);
  if (idx.status[0] == MTBLX_ST_INVALID_BLOCK) throw Error(MtblError::InvalidBlock);   // src/reader.rs:76
  const uint32_t nent = idx.nrec[0];
  // block_at_index + Reader::block framing for every index entry (device), then the checksums
  std::vector<uint64_t> boff(nent);
  std::vector<uint32_t> blen(nent);
  std::vector<int32_t> dst(nent);
  std::vector<uint8_t> bad(nent, 0);
  DevBuf d_off(8ull * nent), d_len(4ull * nent);
  if (nent) {
    DevBuf d_vals = upload(idx.vals.data(), idx.vals.size()), d_vend = upload(idx.val_end.data(), nent);
    DevBuf d_dst(4ull * nent);
    abi_check(mtblx_block_dir(dfile_.as<uint8_t>(), file_.size(), version_, d_vals.as<uint8_t>(),
                              d_vend.as<uint32_t>(), 0, nent, d_off.as<uint64_t>(), d_len.as<uint32_t>(),
                              d_dst.as<int32_t>(), nullptr),
              "mtblx_block_dir");
    hip_check(hipDeviceSynchronize(), "sync");
    boff = download<uint64_t>(d_off.p, nent);
    blen = download<uint32_t>(d_len.p, nent);
    dst = download<int32_t>(d_dst.p, nent);
    if (verify) {
      DevBuf d_bad(nent);
      mtblx_block_batch in{dfile_.as<uint8_t>(), file_.size(), d_off.as<uint64_t>(), d_len.as<uint32_t>(), nent,
                           *std::max_element(blen.begin(), blen.end())};
      abi_check(mtblx_crc32c_blocks(&in, nullptr, d_bad.as<uint8_t>(), 1, nullptr), "mtblx_crc32c_blocks");
      hip_check(hipDeviceSynchronize(), "sync");
      bad = download<uint8_t>(d_bad.p, nent);
    }
  }
  // Reader::block's decompression (src/reader.rs:166-170), any CompressionType, on the host
  // (compression stays on the host per the north star: mtblx_decompress_blocks); then one
  // device decode of every block
  std::vector<uint8_t> zerr(nent, 0);
  if (nent && meta_.compression_algorithm != 0) {
    std::vector<uint64_t> so(nent, 0), uoff(nent, 0), ulen(nent, 0);
    std::vector<uint32_t> sn(nent, 0);
    std::vector<int32_t> zst(nent, 0);
    for (uint32_t i = 0; i < nent; ++i)
      if (dst[i] == MTBLX_DIR_OK) { so[i] = boff[i]; sn[i] = blen[i]; }
    uint8_t* ubuf = nullptr;
    mtblx_decompress_blocks(static_cast<uint32_t>(meta_.compression_algorithm), file_.data(), so.data(), sn.data(),
                            nent, 16, &ubuf, uoff.data(), ulen.data(), zst.data());
    if (!ubuf) throw std::bad_alloc();
    std::vector<uint32_t> ul(nent);
    uint32_t mx = 0;
    uint64_t tot = 0;
    for (uint32_t i = 0; i < nent; ++i) {
      zerr[i] = dst[i] == MTBLX_DIR_OK && zst[i] != MTBLX_CODEC_OK;
      if (ulen[i] > 0xFFFFFFFFull) { mtblx_free(ubuf); throw std::runtime_error("decompressed block >= 4 GiB"); }
      ul[i] = zerr[i] ? 0u : (uint32_t)ulen[i];
      mx = std::max(mx, ul[i]);
      tot = std::max(tot, uoff[i] + ulen[i]);
    }
    DevBuf d_u = upload(ubuf, tot + 1), d_uo = upload(uoff.data(), nent), d_ul = upload(ul.data(), nent);
    mtblx_free(ubuf);
    dec_ = decode_batch(d_u.as<uint8_t>(), tot + 1, d_uo.as<uint64_t>(), d_ul.as<uint32_t>(), nent, mx);
  } else if (nent) {
    std::vector<uint32_t> l2(blen);
    for (uint32_t i = 0; i < nent; ++i)
      if (dst[i] != MTBLX_DIR_OK) l2[i] = 0;   // never decoded: the iteration stops before it
    DevBuf d_l2 = upload(l2.data(), nent);
    dec_ = decode_batch(dfile_.as<uint8_t>(), file_.size(), d_off.as<uint64_t>(), d_l2.as<uint32_t>(), nent,
                        *std::max_element(l2.begin(), l2.end()));
  }
  // ReaderIntoIter::next's end rules over the per-block outcomes (src/reader.rs:337-405)
  size_t take_blocks = 0, take_last = 0;
  bool stopped = false;
  if (nent == 0 && idx.status[0] == MTBLX_ST_CORRUPT) end_ = End::Panic;
  for (uint32_t i = 0; i < nent && !stopped; ++i) {
    if (dst[i] != MTBLX_DIR_OK || bad[i]) { end_ = End::Panic; take_blocks = i; stopped = true; break; }
    if (zerr[i]) { end_ = i == 0 ? End::ErrOpen : End::ErrNext; err_ = MtblError::Io; take_blocks = i; stopped = true; break; }
    const int32_t s = dec_.status[i];
    if (s == MTBLX_ST_INVALID_BLOCK) {
      end_ = i == 0 ? End::ErrOpen : End::ErrNext;
      err_ = MtblError::InvalidBlock;
      take_blocks = i;
      stopped = true;
      break;
    }
    if (s == MTBLX_ST_UNSUPPORTED) throw std::runtime_error("block >= 4 GiB");
    if (s == MTBLX_ST_OK && dec_.nrec[i] == 0 && i > 0) { take_blocks = i; stopped = true; break; }
    if (s == MTBLX_ST_CORRUPT || s == MTBLX_ST_LOOP) {
      take_blocks = i;
      take_last = dec_.nrec[i];
      end_ = s == MTBLX_ST_CORRUPT ? End::Panic : End::Loop;
      stopped = true;
      break;
    }
  }
  if (!stopped && nent) {
    take_blocks = nent;
    if (idx.status[0] == MTBLX_ST_CORRUPT) end_ = End::Panic;   // past the index's last entry
    else if (idx.status[0] == MTBLX_ST_LOOP) end_ = End::Loop;
  }
  if (end_ == End::ErrOpen) throw Error(err_);   // ReaderIntoIter::new returns the Err
  // global END offsets of the yielded records (blocks are laid out in order from record 0)
  for (size_t b = 0; b < take_blocks + (take_last ? 1 : 0); ++b) {
    const size_t cnt = b < take_blocks ? dec_.nrec[b] : take_last;
    for (size_t q = 0; q < cnt; ++q) {
      const size_t r = dec_.rec_base[b] + q;
      gke_.push_back(dec_.key_base[b] + dec_.key_end[r]);
      gve_.push_back(dec_.val_base[b] + dec_.val_end[r]);
    }
  }
  nrec_ = gke_.size();
}

inline std::optional<Record> ReaderIntoIter::next() {
  if (i_ < end_) return r_->rec(i_++);
  switch (r_->end_) {
    case Reader::End::None: return std::nullopt;
    case Reader::End::ErrOpen:
    case Reader::End::ErrNext: throw Error(r_->err_);
    case Reader::End::Panic: throw Panic("corrupt block: the reference panics here");
    case Reader::End::Loop: throw Panic("zero-progress entry: the reference never returns");
  }
  return std::nullopt;
}

inline std::optional<Bytes> Reader::get(const uint8_t* key, size_t klen) const {
  using namespace detail;
  if (meta_.compression_algorithm != 0) {   // values live in decompressed blocks: the decoded records
    const size_t i = lower_bound(key, klen);
    if (i < nrec_) {
      const Record r = rec(i);
      if (r.key_len == klen && std::memcmp(r.key, key, klen) == 0) return r.val_bytes();
    }
    return std::nullopt;
  }
  const uint64_t kend = klen;
  DevBuf d_key = upload(key, klen ? klen : 1), d_kend = upload(&kend, 1);
  DevBuf d_st(4), d_vo(8), d_vl(8);
  abi_check(mtblx_get(dfile_.as<uint8_t>(), file_.size(), version_, verify_ ? 1 : 0, index_off_, index_len_,
                      d_key.as<uint8_t>(), d_kend.as<uint64_t>(), 1, d_st.as<int32_t>(), d_vo.as<uint64_t>(),
                      d_vl.as<uint64_t>(), nullptr),
            "mtblx_get");
  hip_check(hipDeviceSynchronize(), "sync");
  const int32_t st = download<int32_t>(d_st.p, 1)[0];
  if (st == MTBLX_GET_FOUND) {
    const uint64_t o = download<uint64_t>(d_vo.p, 1)[0], n = download<uint64_t>(d_vl.p, 1)[0];
    return Bytes(file_.begin() + o, file_.begin() + o + n);
  }
  if (st == MTBLX_GET_NONE) return std::nullopt;
  if (st == MTBLX_GET_ERR) throw Error(MtblError::InvalidBlock);
  throw Panic(st == MTBLX_GET_LOOP ? "Reader::get never returns" : "Reader::get panics");
}

inline size_t Reader::lower_bound(const uint8_t* k, size_t kl) const {
  size_t lo = 0, hi = nrec_;
  while (lo < hi) {   // first record whose key >= k (keys are sorted)
    const size_t mid = (lo + hi) / 2;
    const Record r = rec(mid);
    const int c = std::memcmp(r.key, k, std::min(r.key_len, kl));
    if (c < 0 || (c == 0 && r.key_len < kl)) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

inline std::vector<Record> Reader::iter_prefix(const Bytes& p) const {
  std::vector<Record> out;
  for (size_t i = lower_bound(p.data(), p.size()); i < nrec_; ++i) {
    const Record r = rec(i);
    if (r.key_len < p.size() || std::memcmp(r.key, p.data(), p.size()) != 0) break;
    out.push_back(r);
  }
  return out;
}

inline std::vector<Record> Reader::iter_range(const Bytes& s, const Bytes& e) const {
  std::vector<Record> out;
  for (size_t i = lower_bound(s.data(), s.size()); i < nrec_; ++i) {
    const Record r = rec(i);
    const int c = std::memcmp(r.key, e.data(), std::min(r.key_len, e.size()));
    if (c > 0 || (c == 0 && r.key_len > e.size())) break;   // key > end (end is inclusive)
    out.push_back(r);
  }
  return out;
}

inline std::vector<Record> Reader::iter_from(const Bytes& k) const {
  std::vector<Record> out;
  for (size_t i = lower_bound(k.data(), k.size()); i < nrec_; ++i) out.push_back(rec(i));
  return out;
}

}  // namespace mtbl
