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
//   ReaderIntoIter::next / seek src/reader.rs:219-405                   (device seek + decode of the
//   Reader::into_iter / iter_prefix / iter_range / iter_from             blocks the iteration reaches,
//                                                                        records served on the host)
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
#include <memory>
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
// one query of mtblx_block_seek_batch, or -- kbuf allocated: the iterator's key past 64 KiB --
// of mtblx_block_seek_batch_kbuf with the key in kbuf
// (vsrc allocated: mtblx_block_seek_batch_ex, the value bytes left to mtblx_copy_ranges)
inline int block_seek_call(const uint8_t* base, const DevBuf& key, const DevBuf& kend, const DevBuf& q, const DevBuf& k,
                           uint64_t keys_cap, const DevBuf& v, uint64_t vals_cap, const DevBuf& ke, const DevBuf& ve,
                           const DevBuf& kc, uint64_t rec_cap, const DevBuf& kbuf, const DevBuf& vsrc) {
  const auto* kk = static_cast<const uint8_t*>(key.p);
  const auto* kn = static_cast<const uint64_t*>(kend.p);
  auto* qq = static_cast<mtblx_block_seek*>(q.p);
  if (vsrc.p)
    return mtblx_block_seek_batch_ex(base, kk, kn, 1, qq, k.as<uint8_t>(), keys_cap, v.as<uint8_t>(), vals_cap,
                                     ke.as<uint64_t>(), ve.as<uint64_t>(), kc.as<uint64_t>(), rec_cap,
                                     kbuf.p ? kbuf.as<uint8_t>() : nullptr, kbuf.p ? kbuf.n : 0, vsrc.as<uint64_t>(),
                                     nullptr);
  if (kbuf.p)
    return mtblx_block_seek_batch_kbuf(base, kk, kn, 1, qq, k.as<uint8_t>(), keys_cap, v.as<uint8_t>(), vals_cap,
                                       ke.as<uint64_t>(), ve.as<uint64_t>(), kc.as<uint64_t>(), rec_cap,
                                       kbuf.as<uint8_t>(), kbuf.n, nullptr);
  return mtblx_block_seek_batch(base, kk, kn, 1, qq, k.as<uint8_t>(), keys_cap, v.as<uint8_t>(), vals_cap,
                                ke.as<uint64_t>(), ve.as<uint64_t>(), kc.as<uint64_t>(), rec_cap, nullptr);
}
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

// a key (possibly empty: one readable zero byte) on the device
inline DevBuf upload_key(const Bytes& k) {
  static const uint8_t zero = 0;
  return k.empty() ? upload(&zero, 1) : upload(k.data(), k.size());
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
    // Lz4 / Lz4hc build a writer whose data-block flushes return Err (Error(Io) below), as the
    // crate's do; NULL = an unknown type, or Zstd without libzstd.so.1 on this host
    if (!w_) throw std::invalid_argument("CompressionType: unknown, or Zstd without libzstd.so.1");
    mtblx_writer_set_level(w_, level);
  }
  Writer(const Writer&) = delete;
  Writer& operator=(const Writer&) = delete;
  Writer(Writer&& o) noexcept : w_(o.w_) { o.w_ = nullptr; }
  ~Writer() { if (w_) mtblx_writer_free(w_); }
  static Writer memory();   // WriterBuilder::default().memory()

  // src/writer.rs:112-149: "out-of-order key" panics; a flush whose compressor returns Err is
  // Err(Io) (the record is not inserted), and the insert after it panics on the data block's
  // `assert!(!self.finished)` (src/block_builder.rs:51)
  void insert(const uint8_t* key, size_t klen, const uint8_t* val, size_t vlen) {
    check(mtblx_writer_insert(w_, key, klen, val, vlen));
  }
  void insert(const Bytes& k, const Bytes& v) { insert(k.data(), k.size(), v.data(), v.size()); }
  void insert(const std::string& k, const std::string& v) {
    insert(reinterpret_cast<const uint8_t*>(k.data()), k.size(), reinterpret_cast<const uint8_t*>(v.data()), v.size());
  }
  // src/writer.rs:155-181: the finished file
  Bytes into_inner() {
    uint8_t* p = nullptr;
    uint64_t n = 0;
    check(mtblx_writer_finish(w_, &p, &n));
    Bytes out(p, p + n);
    mtblx_free(p);
    return out;
  }

 private:
  static void check(int rc) {
    if (rc == MTBLX_OK) return;
    if (rc == MTBLX_E_IO) throw Error(MtblError::Io);
    if (rc == MTBLX_E_FORMAT) throw Panic("out-of-order key");
    throw Panic("BlockBuilder::add: assertion failed (or the writer already panicked)");
  }
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

// ReaderIntoIter (src/reader.rs:219-405): built by Reader::into_iter (new), iter_from
// (new_from), iter_prefix (new_get_prefix), iter_range (new_get_range); next() and the
// mid-iteration seek() (:302-335).  The device seeks and decodes (mtblx_index_seek_batch,
// mtblx_block_seek_batch, mtblx_entry_offsets, mtblx_decode_blocks over the blocks the
// iteration reaches, in growing chunks); the host keeps the reference's state: first, valid,
// the index position and block_offset (0 from the constructors, never updated by next(), so a
// seek landing on a block at that offset re-seeks the block the iterator holds, with that
// iterator's key capacity).  seek() re-seeks the LIVE index iterator (:303) and seeks the data
// block to the landed index entry's key (`key` is shadowed at :305).  On a regular index block
// (mtblx_entry_offsets) the index position is a directory entry; on a corrupt one (read with
// verification off) the live index iterator is driven on the device with
// mtblx_block_seek_batch (seek with its key capacity, early return kept, resume), on the scan
// chain or off it.  next() returns a view valid until the next next()/seek(); it throws Error
// where the reference returns Some(Err) (the iterator is then exhausted), Panic where it
// panics or never returns.
class ReaderIntoIter {
 public:
  std::optional<Record> next();
  bool seek(const Bytes& key);   // Ok(true), or throws
  bool seek(const std::string& k) { return seek(Bytes(k.begin(), k.end())); }
  // drain into owned (key, value) pairs
  std::vector<std::pair<Bytes, Bytes>> collect() {
    std::vector<std::pair<Bytes, Bytes>> out;
    while (auto r = next()) out.emplace_back(r->key_bytes(), r->val_bytes());
    return out;
  }

 private:
  friend class Reader;
  enum Kind { kIter = 0, kGet = 1, kPrefix = 2, kRange = 3 };
  struct Content {   // a block's content on the device (decompressed copy for compressed files)
    std::shared_ptr<detail::DevBuf> own;
    const uint8_t* base = nullptr;
    uint64_t off = 0, len = 0;
  };
  struct Bi {        // one BlockIter: the records it yields from its position on (host copies)
    Content c;
    Bytes keys, vals;
    std::vector<uint64_t> ke, ve;   // END offsets
    int end = MTBLX_EMIT_END;       // after the last record
    std::vector<uint64_t> kcaps;    // key capacity at each record (empty + !kcaps_known: replay)
    bool kcaps_known = false;
    uint64_t kcap_end = 0;
    size_t pos = 0;
    std::optional<Bytes> last_val;  // val of the last entry a seek parsed
    size_t n() const { return ke.size(); }
    Record rec(size_t i) const {
      const uint64_t k0 = i ? ke[i - 1] : 0, v0 = i ? ve[i - 1] : 0;
      return Record{keys.data() + k0, (size_t)(ke[i] - k0), vals.data() + v0, (size_t)(ve[i] - v0)};
    }
  };
  struct Loaded {    // a block as next() loads it: an outcome code or the Bi
    int code = 0;    // 0 ok, 1 panic (framing / checksum), 2 Err(Io), 3 Err(InvalidBlock), 4 >= 4 GiB
    Bi bi;
  };
  struct IxList {    // the live index iterator of an irregular index: the records next() visits
    Bi b;            // from its position on (b.pos), emitted by mtblx_block_seek_batch
    uint64_t stop_off = 0;
    int64_t ord0 = -1;   // directory entry of record 0 when on the scan chain, else -1
    bool valid() const { return b.pos < b.n(); }
    uint64_t kcap() const { return valid() ? b.kcaps[b.pos] : b.kcap_end; }
  };
  static constexpr uint64_t kIxEmit = 256;   // index records per emission
  struct EmitResult {
    mtblx_block_seek res;
    Bi b;
  };
  ReaderIntoIter(const Reader* r, Kind t, Bytes k) : r_(r), type_(t), k_(std::move(k)) {}
  void init_iter();
  void init_from(const Bytes& key);
  Bi load(size_t i);
  // BlockIter::seek / seek_to_first / resume on one block content, no status checks
  static EmitResult emit(const Content& c, const Bytes* key, int first, uint64_t kcap, uint64_t max_records,
                         uint64_t resume_off = 0);
  static Bi seek_block(const Content& c, const Bytes* key, uint64_t kcap);   // key null: seek_to_first
  uint64_t kcap_now(Bi& b);
  void ix_seek(const Bytes& key);
  bool ix_next();
  Bi ix_load();
  IxList ix_list(EmitResult&& e, int64_t ord0) const;
  const Reader* r_;
  Kind type_;
  Bytes k_;
  uint64_t block_offset_ = 0;
  bool first_ = true, valid_ = true;
  std::optional<Bi> bi_;
  int64_t e_ = -1;                  // index position, -1: the index iterator is invalid
  std::optional<IxList> ix_;        // irregular index: the live index iterator
  size_t chunk0_ = 0, grow_ = 1;
  std::vector<Loaded> chunk_;
  size_t vchunk0_ = 0;              // irregular index: prefetched blocks of ix_ (by record)
  std::vector<Loaded> vchunk_;
};

class Reader {
 public:
  // Reader::new (src/reader.rs:99-101): ReaderBuilder::default().read(data), checksums on
  static Reader open(const Bytes& data);
  static Reader open(const uint8_t* data, size_t len);
  Metadata metadata() const { return meta_; }
  uint32_t file_version() const { return version_; }   // Metadata::file_version: 0 FormatV1, 1 FormatV2
  // Reader::into_iter (src/reader.rs:124-126)
  ReaderIntoIter into_iter() const {
    ReaderIntoIter it(this, ReaderIntoIter::kIter, {});
    it.init_iter();
    return it;
  }
  // src/reader.rs:111-122, on the device (mtblx_get: index seek -> block_at_index -> BlockIter::seek)
  std::optional<Bytes> get(const uint8_t* key, size_t klen) const;
  std::optional<Bytes> get(const std::string& k) const {
    return get(reinterpret_cast<const uint8_t*>(k.data()), k.size());
  }
  // src/reader.rs:128-138: seek-based, touching only the blocks the iteration reaches
  ReaderIntoIter iter_from(const Bytes& key) const { return make(ReaderIntoIter::kIter, key, key); }
  ReaderIntoIter iter_prefix(const Bytes& prefix) const { return make(ReaderIntoIter::kPrefix, prefix, prefix); }
  ReaderIntoIter iter_range(const Bytes& start, const Bytes& end) const {   // end inclusive
    return make(ReaderIntoIter::kRange, start, end);
  }
  size_t len() const;   // records the full iteration yields before it ends (decodes the file once)

 private:
  friend class ReaderBuilder;
  friend class ReaderIntoIter;
  Reader(const uint8_t* data, size_t len, bool verify);
  ReaderIntoIter make(ReaderIntoIter::Kind t, const Bytes& seek_key, const Bytes& k) const {
    ReaderIntoIter it(this, t, k);
    it.init_from(seek_key);
    return it;
  }
  mtblx_index_seek index_seek(const Bytes& key) const;
  Bytes index_key(size_t i) const {   // separator key of directory entry i
    const uint32_t a = i ? ikend_[i - 1] : 0;
    return Bytes(ikeys_.begin() + a, ikeys_.begin() + ikend_[i]);
  }
  void index_chain() const;
  bool regular() const { index_chain(); return regular_; }
  std::optional<size_t> chain_ordinal(uint64_t entry) const;
  size_t ordinal(uint64_t entry) const;
  ReaderIntoIter::Content index_content() const {
    return ReaderIntoIter::Content{nullptr, dfile_.as<uint8_t>(), index_off_, index_len_};
  }
  ReaderIntoIter::Content seek_content(const mtblx_index_seek& s) const;
  ReaderIntoIter::Content value_content(const Bytes& value) const;
  struct Framing {   // block_at_index + Reader::block framing of some index entries
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    std::vector<int32_t> st;
    std::vector<uint64_t> block_off;   // the block offset (for contents >= 4 GiB)
  };
  Framing frame_values(const std::vector<Bytes>& values) const;
  std::vector<ReaderIntoIter::Loaded> load_range(size_t i0, size_t i1) const;
  std::vector<ReaderIntoIter::Loaded> load_framed(const Framing& f) const;
  void load_big(uint64_t block_off, ReaderIntoIter::Loaded& L) const;
  void load_content(const ReaderIntoIter::Content& c, ReaderIntoIter::Loaded& L) const;
  Bytes file_;
  detail::DevBuf dfile_;
  bool verify_;
  uint32_t version_ = 1;
  Metadata meta_{};
  uint64_t index_off_ = 0, index_len_ = 0;
  uint32_t nent_ = 0;
  int32_t index_status_ = MTBLX_ST_OK;
  std::vector<uint64_t> boff_;
  std::vector<uint32_t> blen_;
  std::vector<int32_t> dst_;
  Bytes ikeys_;                  // the index block's keys (separators) and END offsets
  std::vector<uint32_t> ikend_;
  detail::DevBuf d_off_, d_len_;
  std::vector<std::pair<uint32_t, uint64_t>> big_;   // entries whose content is >= 4 GiB: block offset
  mutable std::vector<uint64_t> eoffs_;
  mutable bool eoffs_known_ = false, regular_ = false;
  mutable std::optional<size_t> len_;
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
  nent_ = idx.nrec[0];
  index_status_ = idx.status[0];
  ikeys_ = idx.keys;
  ikend_.assign(idx.key_end.begin(), idx.key_end.begin() + nent_);
  // block_at_index + Reader::block framing for every index entry (device); checksums are
  // checked per block when the iteration loads it
  boff_.assign(nent_, 0);
  blen_.assign(nent_, 0);
  dst_.assign(nent_, 0);
  d_off_ = DevBuf(8ull * nent_);
  d_len_ = DevBuf(4ull * nent_);
  if (nent_) {
    DevBuf d_vals = upload(idx.vals.data(), idx.vals.size()), d_vend = upload(idx.val_end.data(), nent_);
    DevBuf d_dst(4ull * nent_);
    abi_check(mtblx_block_dir(dfile_.as<uint8_t>(), file_.size(), version_, d_vals.as<uint8_t>(),
                              d_vend.as<uint32_t>(), 0, nent_, d_off_.as<uint64_t>(), d_len_.as<uint32_t>(),
                              d_dst.as<int32_t>(), nullptr),
              "mtblx_block_dir");
    hip_check(hipDeviceSynchronize(), "sync");
    boff_ = download<uint64_t>(d_off_.p, nent_);
    blen_ = download<uint32_t>(d_len_.p, nent_);
    dst_ = download<int32_t>(d_dst.p, nent_);
    for (uint32_t i = 0; i < nent_; ++i) {   // block_at_index's offset of >= 4 GiB blocks (host)
      if (dst_[i] != MTBLX_DIR_UNSUPPORTED) continue;
      const uint32_t v0 = i ? idx.val_end[i - 1] : 0;
      uint64_t o = 0;
      mtblx_varint_decode64(idx.vals.data() + v0, idx.val_end[i] - v0, &o);
      big_.emplace_back(i, o);
    }
  }
}

// blocks [i0, i1) as next() loads them: Reader::block (framing, checksum, host decompression
// -- compression stays on the host per the north star) + one device decode of the range
inline std::vector<ReaderIntoIter::Loaded> Reader::load_range(size_t i0, size_t i1) const {
  Framing f;
  f.off.assign(boff_.begin() + i0, boff_.begin() + i1);
  f.len.assign(blen_.begin() + i0, blen_.begin() + i1);
  f.st.assign(dst_.begin() + i0, dst_.begin() + i1);
  f.block_off.assign(i1 - i0, 0);
  for (const auto& e : big_)
    if (e.first >= i0 && e.first < i1) f.block_off[e.first - i0] = e.second;
  return load_framed(f);
}

// block_at_index + Reader::block framing of arbitrary index values on the device (mtblx_block_dir)
inline Reader::Framing Reader::frame_values(const std::vector<Bytes>& values) const {
  using namespace detail;
  const uint32_t n = (uint32_t)values.size();
  Framing f;
  Bytes blob;
  std::vector<uint32_t> vend(n);
  for (uint32_t i = 0; i < n; ++i) {
    blob.insert(blob.end(), values[i].begin(), values[i].end());
    vend[i] = (uint32_t)blob.size();
  }
  if (blob.empty()) blob.push_back(0);
  DevBuf d_v = upload(blob.data(), blob.size()), d_ve = upload(vend.data(), n);
  DevBuf d_o(8ull * n), d_l(4ull * n), d_s(4ull * n);
  abi_check(mtblx_block_dir(dfile_.as<uint8_t>(), file_.size(), version_, d_v.as<uint8_t>(), d_ve.as<uint32_t>(), 0, n,
                            d_o.as<uint64_t>(), d_l.as<uint32_t>(), d_s.as<int32_t>(), nullptr),
            "mtblx_block_dir");
  hip_check(hipDeviceSynchronize(), "sync");
  f.off = download<uint64_t>(d_o.p, n);
  f.len = download<uint32_t>(d_l.p, n);
  f.st = download<int32_t>(d_s.p, n);
  f.block_off.assign(n, 0);
  for (uint32_t i = 0; i < n; ++i)
    if (f.st[i] == MTBLX_DIR_UNSUPPORTED) mtblx_varint_decode64(values[i].data(), values[i].size(), &f.block_off[i]);
  return f;
}

inline std::vector<ReaderIntoIter::Loaded> Reader::load_framed(const Framing& f) const {
  using namespace detail;
  const uint32_t n = (uint32_t)f.off.size();
  std::vector<ReaderIntoIter::Loaded> out(n);
  std::vector<uint8_t> bad(n, 0);
  std::vector<uint32_t> l2(f.len);
  for (uint32_t i = 0; i < n; ++i)
    if (f.st[i] != MTBLX_DIR_OK) l2[i] = 0;   // never decoded: the iteration stops before it
  DevBuf d_l2 = upload(l2.data(), n), d_off = upload(f.off.data(), n);
  const uint64_t* d_o = d_off.as<uint64_t>();
  const uint32_t mx = n ? *std::max_element(l2.begin(), l2.end()) : 0;
  if (verify_ && n) {
    DevBuf d_bad(n);
    mtblx_block_batch in{dfile_.as<uint8_t>(), file_.size(), d_o, d_l2.as<uint32_t>(), n, mx};
    abi_check(mtblx_crc32c_blocks(&in, nullptr, d_bad.as<uint8_t>(), 1, nullptr), "mtblx_crc32c_blocks");
    hip_check(hipDeviceSynchronize(), "sync");
    bad = download<uint8_t>(d_bad.p, n);
  }
  std::vector<uint8_t> zerr(n, 0);
  std::shared_ptr<DevBuf> ubuf;
  std::vector<uint64_t> uoff(n, 0);
  std::vector<uint32_t> ul(n, 0);
  std::vector<uint64_t> ulen(n, 0);
  Decoded dec;
  if (meta_.compression_algorithm != 0) {
    std::vector<uint64_t> so(n, 0);
    std::vector<uint32_t> sn(n, 0);
    std::vector<int32_t> zst(n, 0);
    for (uint32_t i = 0; i < n; ++i)
      if (f.st[i] == MTBLX_DIR_OK && !bad[i]) { so[i] = f.off[i]; sn[i] = f.len[i]; }
    uint8_t* hb = nullptr;
    mtblx_decompress_blocks(static_cast<uint32_t>(meta_.compression_algorithm), file_.data(), so.data(), sn.data(), n,
                            16, &hb, uoff.data(), ulen.data(), zst.data());
    if (!hb) throw std::bad_alloc();
    uint32_t umx = 0;
    uint64_t tot = 0;
    for (uint32_t i = 0; i < n; ++i) {
      zerr[i] = sn[i] && zst[i] != MTBLX_CODEC_OK;
      // a content >= 4 GiB stays out of the batch (u32 lengths): the emitting seek decodes it below
      ul[i] = zerr[i] || ulen[i] > 0xFFFFFFFFull ? 0u : (uint32_t)ulen[i];
      umx = std::max(umx, ul[i]);
      tot = std::max(tot, uoff[i] + ulen[i]);
    }
    ubuf = std::make_shared<DevBuf>(tot + 1);
    if (tot) hip_check(hipMemcpy(ubuf->p, hb, tot, hipMemcpyHostToDevice), "H2D");
    mtblx_free(hb);
    DevBuf d_uo = upload(uoff.data(), n), d_ul = upload(ul.data(), n);
    dec = decode_batch(ubuf->as<uint8_t>(), tot + 1, d_uo.as<uint64_t>(), d_ul.as<uint32_t>(), n, umx);
  } else {
    dec = decode_batch(dfile_.as<uint8_t>(), file_.size(), d_o, d_l2.as<uint32_t>(), n, mx);
  }
  for (uint32_t i = 0; i < n; ++i) {
    auto& L = out[i];
    if (f.st[i] == MTBLX_DIR_UNSUPPORTED) {   // content >= 4 GiB (u64 restart array)
      load_big(f.block_off[i], L);
      continue;
    }
    if (f.st[i] != MTBLX_DIR_OK || bad[i]) { L.code = 1; continue; }
    if (zerr[i]) { L.code = 2; continue; }
    if (ubuf && ulen[i] > 0xFFFFFFFFull) {   // decompressed content >= 4 GiB (u64 restart array)
      load_content(ReaderIntoIter::Content{ubuf, ubuf->as<uint8_t>(), uoff[i], ulen[i]}, L);
      continue;
    }
    const int32_t s = dec.status[i];
    if (s == MTBLX_ST_INVALID_BLOCK) { L.code = 3; continue; }
    if (s == MTBLX_ST_UNSUPPORTED) { L.code = 4; continue; }
    auto& b = L.bi;
    if (ubuf) b.c = ReaderIntoIter::Content{ubuf, ubuf->as<uint8_t>(), uoff[i], ul[i]};
    else b.c = ReaderIntoIter::Content{nullptr, dfile_.as<uint8_t>(), f.off[i], f.len[i]};
    b.end = s == MTBLX_ST_CORRUPT ? MTBLX_EMIT_PANIC : s == MTBLX_ST_LOOP ? MTBLX_EMIT_LOOP : MTBLX_EMIT_END;
    const uint64_t r0 = dec.rec_base[i], kb = dec.key_base[i], vb = dec.val_base[i];
    uint64_t kend = 0, vend = 0;
    for (uint32_t q = 0; q < dec.nrec[i]; ++q) {
      kend = dec.key_end[r0 + q];
      vend = dec.val_end[r0 + q];
      b.ke.push_back(kend);
      b.ve.push_back(vend);
    }
    b.keys.assign(dec.keys.begin() + kb, dec.keys.begin() + kb + kend);
    b.vals.assign(dec.vals.begin() + vb, dec.vals.begin() + vb + vend);
  }
  return out;
}

// Reader::block + Block::init + the scan of a block >= 4 GiB: framing and checksum on the host
// (mtblx_frame_block), the scan on the device (the emitting block seek, seek_to_first)
inline void Reader::load_big(uint64_t boff, ReaderIntoIter::Loaded& L) const {
  using namespace detail;
  uint64_t coff = 0, clen = 0;
  int panic = 0;
  if (mtblx_frame_block(file_.data(), file_.size(), version_, boff, verify_ ? 1 : 0, &coff, &clen, &panic) != MTBLX_OK) {
    L.code = 1;
    return;
  }
  if (meta_.compression_algorithm == 0) {
    load_content(ReaderIntoIter::Content{nullptr, dfile_.as<uint8_t>(), coff, clen}, L);
    return;
  }
  uint8_t* hb = nullptr;   // src/reader.rs:166-170 on the host, any size
  uint64_t un = 0;
  if (mtblx_decompress(static_cast<uint32_t>(meta_.compression_algorithm), file_.data() + coff, clen, &hb, &un) !=
      MTBLX_CODEC_OK) {
    if (hb) mtblx_free(hb);
    L.code = 2;
    return;
  }
  auto buf = std::make_shared<DevBuf>(un + 1);
  if (un) hip_check(hipMemcpy(buf->p, hb, un, hipMemcpyHostToDevice), "H2D");
  mtblx_free(hb);
  load_content(ReaderIntoIter::Content{buf, buf->as<uint8_t>(), 0, un}, L);
}

// Block::init + seek_to_first + the records of one content (any size) on the device
inline void Reader::load_content(const ReaderIntoIter::Content& c, ReaderIntoIter::Loaded& L) const {
  try {
    L.bi = ReaderIntoIter::seek_block(c, nullptr, 0);
  } catch (const Error&) {
    L.code = 3;
  } catch (const Panic&) {
    L.code = 1;
  }
}

inline size_t Reader::len() const {
  if (!len_) {
    ReaderIntoIter it = into_iter();
    size_t n = 0;
    try {
      while (it.next()) ++n;
    } catch (const std::exception&) {   // the records before an Err / panic count
    }
    len_ = n;
  }
  return *len_;
}

inline mtblx_index_seek Reader::index_seek(const Bytes& key) const {
  using namespace detail;
  const uint64_t kend = key.size();
  DevBuf d_key = upload_key(key), d_kend = upload(&kend, 1);
  DevBuf d_out(sizeof(mtblx_index_seek));
  abi_check(mtblx_index_seek_batch(dfile_.as<uint8_t>(), file_.size(), version_, verify_ ? 1 : 0, index_off_,
                                   index_len_, d_key.as<uint8_t>(), d_kend.as<uint64_t>(), 1,
                                   d_out.as<mtblx_index_seek>(), nullptr),
            "mtblx_index_seek_batch");
  hip_check(hipDeviceSynchronize(), "sync");
  return download<mtblx_index_seek>(d_out.p, 1)[0];
}

// the index scan chain's entry offsets and whether the index block is regular (mtblx.h)
inline void Reader::index_chain() const {
  using namespace detail;
  if (eoffs_known_) return;
  const uint64_t cap = index_len_ / 3 + 1;   // an entry takes >= 3 bytes
  DevBuf d_offs(8ull * cap), d_cnt(8), d_reg(4);
  abi_check(mtblx_entry_offsets(dfile_.as<uint8_t>() + index_off_, index_len_, d_offs.as<uint64_t>(), cap,
                                d_cnt.as<uint64_t>(), d_reg.as<uint32_t>(), nullptr),
            "mtblx_entry_offsets");
  hip_check(hipDeviceSynchronize(), "sync");
  const uint64_t cnt = std::min<uint64_t>(download<uint64_t>(d_cnt.p, 1)[0], cap);
  eoffs_ = download<uint64_t>(d_offs.p, cnt);
  regular_ = download<uint32_t>(d_reg.p, 1)[0] == 1 && index_status_ == MTBLX_ST_OK;
  eoffs_known_ = true;
}

inline std::optional<size_t> Reader::chain_ordinal(uint64_t entry) const {
  index_chain();
  const auto it = std::lower_bound(eoffs_.begin(), eoffs_.end(), entry);
  if (it == eoffs_.end() || *it != entry) return std::nullopt;
  return (size_t)(it - eoffs_.begin());
}

inline size_t Reader::ordinal(uint64_t entry) const {   // a regular index's landing
  const auto o = chain_ordinal(entry);
  if (!o || *o >= nent_) throw std::runtime_error("index seek landed off the directory of a regular index");
  return *o;
}

// Reader::block (src/reader.rs:139-175) at the offset an index value names: framing and
// checksum (host), decompression (host) -> the content BlockIter reads; throws like the crate
inline ReaderIntoIter::Content Reader::value_content(const Bytes& value) const {
  using namespace detail;
  uint64_t boff = 0;
  if (mtblx_varint_decode64(value.data(), value.size(), &boff) < 0) throw Panic("varint_decode64 of the index value");
  uint64_t coff = 0, clen = 0;
  int panic = 0;
  mtblx_frame_block(file_.data(), file_.size(), version_, boff, verify_ ? 1 : 0, &coff, &clen, &panic);
  if (panic) throw Panic("Reader::block: framing / checksum");
  if (meta_.compression_algorithm == 0) return ReaderIntoIter::Content{nullptr, dfile_.as<uint8_t>(), coff, clen};
  uint8_t* out = nullptr;
  uint64_t n = 0;
  if (mtblx_decompress(static_cast<uint32_t>(meta_.compression_algorithm), file_.data() + coff, clen, &out, &n) !=
      MTBLX_CODEC_OK)
    throw Error(MtblError::Io);
  auto own = std::make_shared<DevBuf>(upload(out, n ? n : 1));
  mtblx_free(out);
  return ReaderIntoIter::Content{own, own->as<uint8_t>(), 0, n};
}

inline ReaderIntoIter::Content Reader::seek_content(const mtblx_index_seek& s) const {
  using namespace detail;
  if (s.block_status == MTBLX_SEEK_PANIC) throw Panic("Reader::block");
  if (meta_.compression_algorithm == 0) {
    if (s.block_status == MTBLX_SEEK_ERR) throw Error(MtblError::InvalidBlock);
    if (s.block_status == MTBLX_SEEK_UNSUPPORTED) throw std::runtime_error("index seek: unexpected block status");
    return ReaderIntoIter::Content{nullptr, dfile_.as<uint8_t>(), s.data_off, s.data_len};
  }
  // compressed: decompress on the host, Block::init runs on the result (mtblx_block_seek_batch)
  uint8_t* out = nullptr;
  uint64_t n = 0;
  if (mtblx_decompress(static_cast<uint32_t>(meta_.compression_algorithm), file_.data() + s.data_off, s.data_len, &out,
                       &n) != MTBLX_CODEC_OK)
    throw Error(MtblError::Io);
  auto own = std::make_shared<DevBuf>(upload(out, n ? n : 1));
  mtblx_free(out);
  return ReaderIntoIter::Content{own, own->as<uint8_t>(), 0, n};
}

inline ReaderIntoIter::EmitResult ReaderIntoIter::emit(const Content& c, const Bytes* key, int first, uint64_t kcap,
                                                       uint64_t max_records, uint64_t resume_off) {
  using namespace detail;
  mtblx_block_seek q{};
  q.data_off = c.off;
  q.data_len = c.len;
  q.kcap = kcap;
  q.max_records = max_records;
  q.first = first;
  q.resume_off = resume_off;
  // output sized exactly from a first counting pass when the block is big (>= 4 GiB blocks)
  const bool big = c.len > (64ull << 20);
  uint64_t rec_cap = std::min<uint64_t>(max_records, big ? 4096 : c.len / 3 + 1),
           keys_cap = big ? 1 << 20 : 2 * c.len + 64, vals_cap = big ? 1 << 20 : c.len + 16;
  const Bytes none;
  const uint64_t kend = key ? key->size() : 0;
  DevBuf d_key = upload_key(key ? *key : none), d_kend = upload(&kend, 1);
  DevBuf kbuf;   // allocated once a key runs past the 64 KiB LDS key
  for (int attempt = 0; attempt < 4; ++attempt) {
    DevBuf d_q = upload(&q, 1), d_k(keys_cap + 1), d_v(vals_cap + 1), d_ke(8 * rec_cap + 8), d_ve(8 * rec_cap + 8),
        d_kc(8 * rec_cap + 8);
    DevBuf d_vs = big ? DevBuf(8 * rec_cap + 8) : DevBuf();   // big blocks: values moved by the whole grid
    abi_check(block_seek_call(c.base, d_key, d_kend, d_q, d_k, keys_cap, d_v, vals_cap, d_ke, d_ve, d_kc, rec_cap, kbuf,
                              d_vs),
              "mtblx_block_seek_batch");
    hip_check(hipDeviceSynchronize(), "sync");
    EmitResult r;
    r.res = download<mtblx_block_seek>(d_q.p, 1)[0];
    if (r.res.status == MTBLX_SEEK_UNSUPPORTED && !kbuf.p) {   // any key this iterator can build fits
      kbuf = DevBuf(kend + c.len + 64);
      continue;
    }
    if (r.res.end == MTBLX_EMIT_OVERFLOW) {
      rec_cap = r.res.nrec;
      keys_cap = r.res.key_bytes;
      vals_cap = r.res.val_bytes;
      continue;
    }
    Bi& b = r.b;
    b.c = c;
    b.end = r.res.end;
    b.ke = download<uint64_t>(d_ke.p, r.res.nrec);
    b.ve = download<uint64_t>(d_ve.p, r.res.nrec);
    b.kcaps = download<uint64_t>(d_kc.p, r.res.nrec);
    b.kcaps_known = true;
    b.kcap_end = r.res.kcap;
    b.keys = download<uint8_t>(d_k.p, r.res.key_bytes);
    if (big && r.res.nrec) {   // the values: mtblx_copy_ranges from the block content
      const std::vector<uint64_t> vs = download<uint64_t>(d_vs.p, r.res.nrec);
      std::vector<uint64_t> so(r.res.nrec), dofs(r.res.nrec), ln(r.res.nrec), cb(r.res.nrec);
      uint64_t prev = 0, chunks = 0;
      for (uint64_t i = 0; i < r.res.nrec; ++i) {
        so[i] = c.off + vs[i];
        dofs[i] = prev;
        ln[i] = b.ve[i] - prev;
        cb[i] = chunks;
        chunks += (ln[i] + 15) / 16;
        prev = b.ve[i];
      }
      DevBuf d_so = upload(so.data(), so.size()), d_do = upload(dofs.data(), dofs.size()),
             d_ln = upload(ln.data(), ln.size()), d_cb = upload(cb.data(), cb.size());
      abi_check(mtblx_copy_ranges(c.base, d_so.as<uint64_t>(), d_v.as<uint8_t>(), d_do.as<uint64_t>(),
                                  d_ln.as<uint64_t>(), d_cb.as<uint64_t>(), (uint32_t)r.res.nrec, chunks, nullptr),
                "mtblx_copy_ranges");
      hip_check(hipDeviceSynchronize(), "sync");
    }
    b.vals = download<uint8_t>(d_v.p, r.res.val_bytes);
    if (r.res.has_val) b.last_val = download<uint8_t>(c.base + c.off + r.res.last_voff, r.res.last_vlen);
    return r;
  }
  throw std::runtime_error("mtblx_block_seek_batch: output sizes did not converge");
}

inline ReaderIntoIter::Bi ReaderIntoIter::seek_block(const Content& c, const Bytes* key, uint64_t kcap) {
  EmitResult r = emit(c, key, key ? 0 : 1, kcap, ~0ull >> 2);
  if (r.res.status == MTBLX_SEEK_ERR) throw Error(MtblError::InvalidBlock);
  if (r.res.status == MTBLX_SEEK_PANIC) throw Panic("BlockIter::seek");
  if (r.res.status == MTBLX_SEEK_LOOP) throw Panic("BlockIter::seek never returns");
  if (r.res.status == MTBLX_SEEK_UNSUPPORTED) throw std::runtime_error("emitting seek: key buffer too small");
  return std::move(r.b);
}

// the key Vec's capacity of the held iterator now (parse_next_key's END leaves it unchanged)
inline uint64_t ReaderIntoIter::kcap_now(Bi& b) {
  using namespace detail;
  if (b.n() == 0) return b.kcap_end;
  if (!b.kcaps_known) {   // records from the bulk decoder: replay seek_to_first + next on the device
    mtblx_block_seek q{};
    q.data_off = b.c.off;
    q.data_len = b.c.len;
    q.max_records = b.n();
    q.first = 1;
    const uint64_t kend = 0;
    const uint8_t z = 0;
    DevBuf d_key = upload(&z, 1), d_kend = upload(&kend, 1), d_q = upload(&q, 1);
    // only the key capacities are needed: the value bytes are deferred (vsrc) and never moved
    DevBuf d_k(2 * b.c.len + 65), d_v, d_ke(8 * b.n() + 8), d_ve(8 * b.n() + 8), d_kc(8 * b.n() + 8),
        d_vs(8 * b.n() + 8);
    DevBuf kbuf;
    for (int attempt = 0; attempt < 2; ++attempt) {
      abi_check(block_seek_call(b.c.base, d_key, d_kend, d_q, d_k, 2 * b.c.len + 64, d_v, b.c.len + 16, d_ke, d_ve, d_kc,
                                b.n(), kbuf, d_vs),
                "mtblx_block_seek_batch");
      hip_check(hipDeviceSynchronize(), "sync");
      if (download<mtblx_block_seek>(d_q.p, 1)[0].status != MTBLX_SEEK_UNSUPPORTED || kbuf.p) break;
      kbuf = DevBuf(b.c.len + 64);   // a key past 64 KiB: again with the key in device memory
      hip_check(hipMemcpy(d_q.p, &q, sizeof(q), hipMemcpyHostToDevice), "H2D");
    }
    b.kcaps = download<uint64_t>(d_kc.p, b.n());
    b.kcaps_known = true;
  }
  return b.kcaps[std::min(b.pos, b.n() - 1)];
}

inline ReaderIntoIter::Bi ReaderIntoIter::load(size_t i) {
  if (chunk_.empty() || i < chunk0_ || i >= chunk0_ + chunk_.size()) {
    const size_t n = std::min<size_t>(r_->nent_ - i, grow_);
    grow_ = std::min<size_t>(2 * grow_, 256);
    chunk_ = r_->load_range(i, i + n);
    chunk0_ = i;
  }
  Loaded& L = chunk_[i - chunk0_];
  switch (L.code) {
    case 1: throw Panic("Reader::block: framing / checksum");
    case 2: throw Error(MtblError::Io);
    case 3: throw Error(MtblError::InvalidBlock);
    case 4: throw std::runtime_error("block >= 4 GiB");
  }
  return L.bi;
}

inline ReaderIntoIter::IxList ReaderIntoIter::ix_list(EmitResult&& e, int64_t ord0) const {
  if (e.res.status == MTBLX_SEEK_PANIC) throw Panic("index seek");
  if (e.res.status == MTBLX_SEEK_LOOP) throw Panic("index seek never returns");
  if (e.res.status == MTBLX_SEEK_UNSUPPORTED) throw std::runtime_error("emitting seek: key buffer too small");
  IxList l;
  l.b = std::move(e.b);
  l.stop_off = e.res.stop_off;
  l.ord0 = ord0;
  return l;
}

inline void ReaderIntoIter::init_iter() {   // new (src/reader.rs:231-254)
  if (r_->nent_ == 0) {
    if (r_->index_status_ == MTBLX_ST_CORRUPT) throw Panic("index block: first entry");
    if (!r_->regular()) ix_ = IxList{};
    return;
  }
  if (r_->regular()) {
    e_ = 0;
  } else {   // the scan's own chain = the directory, with its key capacities
    ix_ = ix_list(emit(r_->index_content(), nullptr, 1, 0, kIxEmit), 0);
  }
  bi_ = load(0);
}

inline void ReaderIntoIter::init_from(const Bytes& key) {   // new_from (src/reader.rs:256-279)
  if (!r_->regular()) {   // a fresh live index iterator, seeked
    ix_ = IxList{};
    ix_seek(key);
    if (!ix_->valid()) return;
    bi_ = seek_block(r_->value_content(ix_->b.rec(ix_->b.pos).val_bytes()), &key, 0);
    return;
  }
  const mtblx_index_seek s = r_->index_seek(key);
  if (s.status == MTBLX_SEEK_PANIC) throw Panic("index seek");
  if (s.status == MTBLX_SEEK_LOOP) throw Panic("index seek never returns");
  if (!s.valid) return;
  e_ = (int64_t)r_->ordinal(s.entry);
  bi_ = seek_block(r_->seek_content(s), &key, 0);
}

// index_iter.seek(key) on the live iterator of an irregular index (src/block.rs:154-194)
inline void ReaderIntoIter::ix_seek(const Bytes& key) {
  EmitResult e = emit(r_->index_content(), &key, 0, ix_->kcap(), kIxEmit);
  if (e.res.status == MTBLX_SEEK_OK && e.res.early) return;   // corrupt restart: the old position stays
  int64_t ord0 = -1;
  if (e.res.status == MTBLX_SEEK_OK && e.res.nrec) {
    const auto o = r_->chain_ordinal(e.res.entry);
    if (o) ord0 = (int64_t)*o;
  }
  ix_ = ix_list(std::move(e), ord0);
  vchunk_.clear();
}

// index_iter.next() (src/block.rs:196-202) on the live iterator
inline bool ReaderIntoIter::ix_next() {
  IxList& ix = *ix_;
  if (!ix.valid()) return false;
  if (ix.b.pos + 1 < ix.b.n()) { ++ix.b.pos; return true; }
  if (ix.b.end == MTBLX_EMIT_END) { ix.b.pos = ix.b.n(); return false; }
  if (ix.b.end == MTBLX_EMIT_PANIC) throw Panic("index block: next entry");
  if (ix.b.end == MTBLX_EMIT_LOOP) return true;   // a zero-progress entry: the same record again
  // EMIT_MAX: the entry after the last record, parsed from that record's key and capacity
  const Bytes k = ix.b.rec(ix.b.n() - 1).key_bytes();
  EmitResult e = emit(r_->index_content(), &k, 2, ix.b.kcaps.back(), kIxEmit, ix.stop_off);
  if (e.res.status == MTBLX_SEEK_PANIC) throw Panic("index block: next entry");
  const int64_t ord0 = ix.ord0 < 0 ? -1 : ix.ord0 + (int64_t)ix.b.n();
  ix_ = ix_list(std::move(e), ord0);
  vchunk_.clear();
  return ix_->valid();
}

// block_at_index of the live index iterator's record (Reader::block + seek_to_first)
inline ReaderIntoIter::Bi ReaderIntoIter::ix_load() {
  const IxList& ix = *ix_;
  const size_t pos = ix.b.pos;
  if (ix.ord0 >= 0 && (size_t)ix.ord0 + pos < r_->nent_) return load((size_t)ix.ord0 + pos);
  if (vchunk_.empty() || pos < vchunk0_ || pos >= vchunk0_ + vchunk_.size()) {
    const size_t n = std::min<size_t>(ix.b.n() - pos, grow_);
    grow_ = std::min<size_t>(2 * grow_, 256);
    std::vector<Bytes> vals;
    for (size_t q = pos; q < pos + n; ++q) vals.push_back(ix.b.rec(q).val_bytes());
    vchunk_ = r_->load_framed(r_->frame_values(vals));
    vchunk0_ = pos;
  }
  Loaded& L = vchunk_[pos - vchunk0_];
  switch (L.code) {
    case 1: throw Panic("Reader::block: framing / checksum");
    case 2: throw Error(MtblError::Io);
    case 3: throw Error(MtblError::InvalidBlock);
    case 4: throw std::runtime_error("block >= 4 GiB");
  }
  return L.bi;
}

inline std::optional<Record> ReaderIntoIter::next() {   // src/reader.rs:337-405
  if (!valid_ || !bi_) return std::nullopt;
  Bi* b = &*bi_;
  if (!first_ && b->pos < b->n()) ++b->pos;   // bi.next()
  first_ = false;
  if (b->pos == b->n() && b->end == MTBLX_EMIT_PANIC) throw Panic("BlockIter::next / get");
  if (b->pos == b->n() && b->end == MTBLX_EMIT_LOOP) throw Panic("zero-progress entry: the reference never returns");
  if (b->pos == b->n()) {
    valid_ = false;
    if (ix_) {                                // irregular index: the live index iterator
      if (!ix_next()) return std::nullopt;
      Bi nb = ix_load();                      // Some(Err(e)) throws; valid stays false
      bi_ = std::move(nb);
    } else {
      if (e_ < 0) return std::nullopt;
      if ((size_t)e_ + 1 >= r_->nent_) {       // index_iter.next() past the last entry
        e_ = -1;
        if (r_->index_status_ == MTBLX_ST_CORRUPT) throw Panic("index block: next entry");
        if (r_->index_status_ == MTBLX_ST_LOOP) throw Panic("index block never returns");
        return std::nullopt;
      }
      ++e_;
      Bi nb = load((size_t)e_);                // Some(Err(e)) throws; valid stays false
      bi_ = std::move(nb);
    }
    b = &*bi_;
    if (b->n() == 0 && b->end == MTBLX_EMIT_PANIC) throw Panic("BlockIter::seek_to_first / get");
    if (b->n() == 0) return std::nullopt;
    valid_ = true;
  }
  const Record rec = b->rec(b->pos);
  const size_t kl = k_.size();
  if (type_ == kGet) {
    valid_ = rec.key_len == kl && (kl == 0 || std::memcmp(rec.key, k_.data(), kl) == 0);
  } else if (type_ == kPrefix) {
    valid_ = rec.key_len >= kl && (kl == 0 || std::memcmp(rec.key, k_.data(), kl) == 0);
  } else if (type_ == kRange) {
    const size_t m = std::min(rec.key_len, kl);
    const int c = m ? std::memcmp(rec.key, k_.data(), m) : 0;
    valid_ = !(c > 0 || (c == 0 && rec.key_len > kl));
  }
  if (!valid_) return std::nullopt;
  return rec;
}

// src/reader.rs:302-335: the block is seeked to the landed index entry's key (:305 shadows `key`)
inline bool ReaderIntoIter::seek(const Bytes& key) {
  Bytes ikey;
  uint64_t new_off = 0;
  std::optional<mtblx_index_seek> s;
  if (ix_) {                        // irregular index: the live index iterator
    ix_seek(key);
    if (!ix_->valid()) {
      valid_ = false;
      return true;
    }
    const Record ir = ix_->b.rec(ix_->b.pos);
    ikey = ir.key_bytes();
    if (mtblx_varint_decode64(ir.val, ir.val_len, &new_off) < 0) throw Panic("varint_decode64 of the index value");
  } else {
    s = r_->index_seek(key);
    if (s->status == MTBLX_SEEK_PANIC) throw Panic("index seek");
    if (s->status == MTBLX_SEEK_LOOP) throw Panic("index seek never returns");
    if (!s->valid) {   // past the last key: next() returns None
      valid_ = false;
      e_ = -1;
      return true;
    }
    e_ = (int64_t)r_->ordinal(s->entry);
    ikey = r_->index_key((size_t)e_);
    new_off = s->block_off;
  }
  if (block_offset_ != new_off) {
    block_offset_ = new_off;   // updated before the load (:322)
    Bi nb = seek_block(s ? r_->seek_content(*s) : r_->value_content(ix_->b.rec(ix_->b.pos).val_bytes()), &ikey, 0);
    bi_ = std::move(nb);
  } else if (bi_) {                 // the held block, whatever it is
    Bi nb = seek_block(bi_->c, &ikey, kcap_now(*bi_));
    bi_ = std::move(nb);
  }
  first_ = true;
  valid_ = true;
  return true;
}

inline std::optional<Bytes> Reader::get(const uint8_t* key, size_t klen) const {
  using namespace detail;
  if (meta_.compression_algorithm != 0) {   // values live in decompressed blocks: the seek iterator
    ReaderIntoIter it(this, ReaderIntoIter::kGet, Bytes(key, key + klen));
    it.init_from(Bytes(key, key + klen));
    std::optional<Bytes> held = it.bi_ ? it.bi_->last_val : std::nullopt;
    try {
      auto r = it.next();
      if (!r) return std::nullopt;
      return r->val_bytes();
    } catch (const Error&) {
      // next() returned Some(Err): Reader::get returns the OLD block iterator's val
      // (src/reader.rs:111-122, :376-379), or None
      return held;
    }
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

}  // namespace mtbl
