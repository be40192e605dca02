// host.cpp — host-side mirror of the reference's file layer, around the device codec.
//
//   Writer / WriterBuilder   /root/reference/src/writer.rs:15-265
//   BlockBuilder             src/block_builder.rs:1-104 (host build of block bytes)
//   Metadata                 src/metadata.rs:27-79
//   Reader framing           src/reader.rs:31-81, :140-175 (footer, index, block framing, CRC)
//   crc32c                   crate crc32c 0.4 (SSE4.2 crc32 instruction)
//
// Block DECODE never happens here: the reader hands every block (index block included)
// to the device decoder (decode.hip) through mtblx_decode_blocks.
#include <nmmintrin.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "mtblx.h"
#include "mtblx_host.h"

int mtblx_compress_vec(uint32_t c, uint32_t level, const uint8_t* src, uint64_t n, std::vector<uint8_t>& out);

namespace {

inline void wr32(uint8_t* p, uint32_t v) { memcpy(p, &v, 4); }
inline void wr64(uint8_t* p, uint64_t v) { memcpy(p, &v, 8); }
inline uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

// varint_encode32 / varint_encode64 (src/varint.rs:12-42, :63-76)
inline uint32_t venc32(uint8_t* b, uint32_t v) {
  uint32_t i = 0;
  while (v >= 128) { b[i++] = (uint8_t)(v | 128); v >>= 7; }
  b[i] = (uint8_t)v;
  return i + 1;
}
inline uint32_t venc64(uint8_t* b, uint64_t v) {
  uint32_t i = 0;
  while (v >= 128) { b[i++] = (uint8_t)(v | 128); v >>= 7; }
  b[i] = (uint8_t)v;
  return i + 1;
}

// varint_decode64 (src/varint.rs:78-97 delegating to :44-61).  -1 = reference panics.
int vdec64(const uint8_t* d, uint64_t len, uint64_t* out) {
  if (len == 0) return -1;
  uint32_t win = len < 10 ? (uint32_t)len : 10u, l = 0;
  for (uint32_t i = 0; i < win; ++i)
    if (!(d[i] & 0x80)) { l = i + 1; break; }
  if (l < 5) {  // varint_decode32 semantics, window of 5
    uint32_t w5 = len < 5 ? (uint32_t)len : 5u, l5 = 0;
    for (uint32_t i = 0; i < w5; ++i)
      if (!(d[i] & 0x80)) { l5 = i + 1; break; }
    uint32_t v = d[0] & 0x7f;
    if (l5 > 1) v |= (uint32_t)(d[1] & 0x7f) << 7;
    if (l5 > 2) v |= (uint32_t)(d[2] & 0x7f) << 14;
    if (l5 > 3) v |= (uint32_t)(d[3] & 0x7f) << 21;
    if (l5 > 4) v |= (uint32_t)d[4] << 28;
    *out = v;
    return (int)l5;
  }
  uint64_t v = 0;
  for (uint32_t i = 0; i < l; ++i) v |= (uint64_t)(d[i] & 0x7f) << (7 * i);
  *out = v;
  return (int)l;
}

int cmp_bytes(const uint8_t* a, size_t al, const uint8_t* b, size_t bl) {
  size_t m = std::min(al, bl);
  int c = m ? memcmp(a, b, m) : 0;
  if (c) return c < 0 ? -1 : 1;
  return al < bl ? -1 : (al > bl ? 1 : 0);
}

// ---------------- BlockBuilder (src/block_builder.rs) ----------------
struct BlockBuilder {
  size_t interval;
  std::vector<uint8_t> buf;
  std::vector<uint8_t> last_key;
  std::vector<uint64_t> restarts{0};
  size_t counter = 0;
  bool finished = false;
  explicit BlockBuilder(size_t iv) : interval(iv) { buf.reserve(1 << 16); }
  void reset() { buf.clear(); last_key.clear(); restarts.assign(1, 0); counter = 0; finished = false; }
  bool empty() const { return buf.empty(); }
  size_t estimate() const { return buf.size() + restarts.size() * (buf.size() > 0xFFFFFFFFull ? 8 : 4) + 4; }
  bool add(const uint8_t* k, size_t kl, const uint8_t* v, size_t vl) {
    if (!(counter <= interval) || finished) return false;  // asserts (:50-51)
    size_t shared = 0;
    if (counter < interval) {
      size_t m = std::min(last_key.size(), kl);
      while (shared < m && last_key[shared] == k[shared]) ++shared;
    } else {
      restarts.push_back(buf.size());
      counter = 0;
    }
    uint8_t t[15];
    uint32_t n = venc32(t, (uint32_t)shared);
    n += venc32(t + n, (uint32_t)(kl - shared));
    n += venc32(t + n, (uint32_t)vl);
    buf.insert(buf.end(), t, t + n);
    buf.insert(buf.end(), k + shared, k + kl);
    buf.insert(buf.end(), v, v + vl);
    last_key.assign(k, k + kl);
    ++counter;
    return true;
  }
  // finish (:85-104): content = entries | restarts (u32, u64 past 4 GiB) | count u32
  void finish(std::vector<uint8_t>& out) {
    bool r64 = buf.size() > 0xFFFFFFFFull;
    uint8_t t[8];
    for (uint64_t r : restarts) {
      if (r64) { wr64(t, r); buf.insert(buf.end(), t, t + 8); }
      else { wr32(t, (uint32_t)r); buf.insert(buf.end(), t, t + 4); }
    }
    wr32(t, (uint32_t)restarts.size());
    buf.insert(buf.end(), t, t + 4);
    out.swap(buf);   // mem::replace: the builder keeps an empty buffer until reset()
    buf.clear();
    finished = true;
  }
};

// bytes_shortest_separator (src/writer.rs:239-265); false = reference assert fires
bool shortest_separator(std::vector<uint8_t>& s, const uint8_t* l, size_t ll) {
  size_t min_len = std::min(s.size(), ll), di = 0;
  while (di < min_len && s[di] == l[di]) ++di;
  if (di >= min_len) return true;
  uint8_t db = s[di];
  if (db < 255 && (uint8_t)(db + 1) < l[di]) {
    s[di] = db + 1;
    s.resize(di + 1);
  } else if (di < (min_len >= 2 ? min_len - 2 : 0)) {
    uint16_t us = (uint16_t)(s[di] << 8 | s[di + 1]);
    uint16_t ul = (uint16_t)(l[di] << 8 | l[di + 1]);
    uint16_t ub = (uint16_t)(us + 1);
    if (us <= ub && ub <= ul) {  // write_u16 on a Vec APPENDS (:260)
      s.push_back((uint8_t)(ub >> 8));
      s.push_back((uint8_t)ub);
    }
  }
  return cmp_bytes(s.data(), s.size(), l, ll) < 0;
}

}  // namespace

extern "C" uint32_t mtblx_crc32c(const uint8_t* d, uint64_t n) {
  uint64_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, d, 8);
    c = _mm_crc32_u64(c, w);
    d += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *d++);
  return c32 ^ 0xFFFFFFFFu;
}

// ---------------- Writer (src/writer.rs) ----------------
struct mtblx_writer {
  uint64_t meta[9] = {0};  // footer order, src/metadata.rs:61-79
  uint32_t compression = 0;
  uint32_t level = 0;        // WriterBuilder::compression_level (DEFAULT_COMPRESSION_LEVEL = 0)
  BlockBuilder data, index;
  std::vector<uint8_t> last_key;
  uint64_t last_offset = 0, pending_offset = 0;
  bool pending_index_entry = false;
  bool poisoned = false;
  std::vector<uint8_t> out;
  std::vector<uint8_t> scratch, zbuf;
  std::vector<uint64_t> blk_off;  // stored-content offset of each data block (block directory)
  std::vector<uint32_t> blk_len;
  std::vector<uint32_t> blk_nrec;
  uint32_t cur_nrec = 0;
  mtblx_writer(uint64_t bs, uint64_t iv, uint32_t comp) : data(iv), index(iv) {
    meta[1] = std::max<uint64_t>(bs, 1024);  // WriterBuilder::block_size clamps (:43-46)
    meta[2] = comp;
    compression = comp;
  }
  // write_block (:203-237): data blocks are compressed with the file's compression type
  // (:214), the index block never (into_inner passes CompressionType::None, :165-173); the
  // checksum covers the STORED bytes (:217-218).  A compressor Err (Lz4 / Lz4hc: "unsupported",
  // src/compression.rs:70-81; a codec failure) returns at the `?` of :214 (MTBLX_E_IO) after
  // BlockBuilder::finish has already taken the block's bytes and set `finished`
  // (src/block_builder.rs:85-104): nothing is written, the pending block's records are lost, and
  // the next insert panics on the builder's !finished assert -- as the reference does.
  int write_block(BlockBuilder& b, bool is_data, uint64_t& written) {
    b.finish(scratch);
    const std::vector<uint8_t>* stored = &scratch;
    if (is_data && compression != 0) {   // compress (src/compression.rs:70-81), codecs_host.cpp
      if (mtblx_compress_vec(compression, level, scratch.data(), scratch.size(), zbuf) != MTBLX_CODEC_OK)
        return MTBLX_E_IO;
      stored = &zbuf;
    }
    uint8_t hdr[14];
    uint32_t ll = venc64(hdr, stored->size());
    wr32(hdr + ll, mtblx_crc32c(stored->data(), stored->size()));
    out.insert(out.end(), hdr, hdr + ll + 4);
    if (is_data) {
      blk_off.push_back(out.size());
      blk_len.push_back((uint32_t)stored->size());
      blk_nrec.push_back(cur_nrec);
      cur_nrec = 0;
    }
    out.insert(out.end(), stored->begin(), stored->end());
    written = ll + 4 + stored->size();
    last_offset = pending_offset;
    pending_offset += written;
    b.reset();
    return MTBLX_OK;
  }
  int flush() {  // (:183-200): MTBLX_OK, MTBLX_E_IO (Err), MTBLX_E_FORMAT (the assert panics)
    if (data.empty()) return MTBLX_OK;
    if (pending_index_entry) return MTBLX_E_FORMAT;
    uint64_t written = 0;
    const int r = write_block(data, true, written);
    if (r != MTBLX_OK) return r;
    meta[5] += written;
    meta[4] += 1;
    pending_index_entry = true;
    return MTBLX_OK;
  }
};

extern "C" mtblx_writer* mtblx_writer_new(uint64_t block_size, uint64_t restart_interval, uint32_t compression) {
  // CompressionType 0..5.  Lz4 / Lz4hc build a writer whose first data-block flush returns Err
  // "unsupported" (src/compression.rs:70-81): MTBLX_E_IO from insert / finish.  Zstd needs
  // libzstd.so.1 on this host (the crate bundles it): NULL without it.
  if (compression > 5 || (compression == 5 && !mtblx_codec_available(compression))) return nullptr;
  return new mtblx_writer(block_size, restart_interval, compression);
}

extern "C" int mtblx_writer_set_level(mtblx_writer* w, uint32_t level) {
  if (!w) return MTBLX_E_INVAL;
  w->level = level;
  return MTBLX_OK;
}

extern "C" void mtblx_writer_free(mtblx_writer* w) { delete w; }

extern "C" int mtblx_writer_insert(mtblx_writer* w, const uint8_t* k, uint64_t kl, const uint8_t* v, uint64_t vl) {
  if (!w || w->poisoned) return MTBLX_E_INVAL;
  if (w->meta[3] > 0 && cmp_bytes(k, kl, w->last_key.data(), w->last_key.size()) <= 0) {
    w->poisoned = true;  // panic!("out-of-order key") (:119-123)
    return MTBLX_E_FORMAT;
  }
  if (w->data.estimate() + 15 + kl + vl >= w->meta[1]) {  // (:125-130)
    const int r = w->flush();
    if (r == MTBLX_E_IO) return r;   // Err: this record is not inserted; the flushed block is lost
    if (r != MTBLX_OK) { w->poisoned = true; return r; }
  }
  if (w->pending_index_entry) {  // (:132-138)
    if (!shortest_separator(w->last_key, k, kl)) { w->poisoned = true; return MTBLX_E_FORMAT; }
    uint8_t enc[10];
    uint32_t el = venc64(enc, w->last_offset);
    if (!w->index.add(w->last_key.data(), w->last_key.size(), enc, el)) { w->poisoned = true; return MTBLX_E_FORMAT; }
    w->pending_index_entry = false;
  }
  w->last_key.assign(k, k + kl);
  w->meta[3] += 1;
  w->meta[7] += kl;
  w->meta[8] += vl;
  // BlockBuilder::add's asserts (:50-51) -- `!finished` fires on the insert after a flush whose
  // compressor returned Err (the builder's buffer was moved out and never reset): a panic
  if (!w->data.add(k, kl, v, vl)) { w->poisoned = true; return MTBLX_E_INVAL; }
  w->cur_nrec += 1;
  return MTBLX_OK;
}

extern "C" int mtblx_writer_insert_batch(mtblx_writer* w, const uint8_t* keys, const uint64_t* key_end,
                                         const uint8_t* vals, const uint64_t* val_end, uint64_t n) {
  uint64_t k0 = 0, v0 = 0;
  for (uint64_t i = 0; i < n; ++i) {
    int r = mtblx_writer_insert(w, keys + k0, key_end[i] - k0, vals + v0, val_end[i] - v0);
    if (r) return r;
    k0 = key_end[i];
    v0 = val_end[i];
  }
  return MTBLX_OK;
}

extern "C" int mtblx_writer_finish(mtblx_writer* w, uint8_t** out, uint64_t* out_len) {  // into_inner (:155-181)
  if (!w || w->poisoned || !out || !out_len) return MTBLX_E_INVAL;
  const int r = w->flush();
  if (r != MTBLX_OK) return r;
  if (w->pending_index_entry) {
    uint8_t enc[10];
    uint32_t el = venc64(enc, w->last_offset);
    if (!w->index.add(w->last_key.data(), w->last_key.size(), enc, el)) return MTBLX_E_FORMAT;
    w->pending_index_entry = false;
  }
  w->meta[0] = w->pending_offset;
  uint64_t written = 0;
  w->write_block(w->index, false, written);   // CompressionType::None: cannot fail
  w->meta[6] += written;
  uint8_t md[512];
  memset(md, 0, sizeof(md));
  for (int i = 0; i < 9; ++i) wr64(md + 8 * i, w->meta[i]);
  wr32(md + 508, 0x4D54424Cu);
  w->out.insert(w->out.end(), md, md + 512);
  *out_len = w->out.size();
  *out = (uint8_t*)malloc(w->out.size());
  if (!*out) return MTBLX_E_INVAL;
  memcpy(*out, w->out.data(), w->out.size());
  w->poisoned = true;  // writer consumed
  return MTBLX_OK;
}

extern "C" uint64_t mtblx_writer_block_count(const mtblx_writer* w) { return w ? w->blk_off.size() : 0; }
extern "C" int mtblx_writer_block_dir(const mtblx_writer* w, uint64_t* blk_off, uint32_t* blk_len,
                                      uint32_t* blk_nrec) {
  if (!w) return MTBLX_E_INVAL;
  std::copy(w->blk_off.begin(), w->blk_off.end(), blk_off);
  std::copy(w->blk_len.begin(), w->blk_len.end(), blk_len);
  if (blk_nrec) std::copy(w->blk_nrec.begin(), w->blk_nrec.end(), blk_nrec);
  return MTBLX_OK;
}

extern "C" void mtblx_free(void* p) { free(p); }

// ---------------- Reader framing (src/reader.rs:31-81, :140-175) ----------------
extern "C" int mtblx_read_footer(const uint8_t* d, uint64_t len, mtblx_footer* f) {
  memset(f, 0, sizeof(*f));
  if (len < 512) return f->err = MTBLX_ERR_INVALID_METADATA_SIZE, MTBLX_E_FORMAT;
  const uint8_t* m = d + len - 512;
  uint32_t magic = rd32(m + 508);  // metadata.rs:28-33
  if (magic == 0x77846676u) f->version = 0;
  else if (magic == 0x4D54424Cu) f->version = 1;
  else return f->err = MTBLX_ERR_INVALID_FORMAT_VERSION, MTBLX_E_FORMAT;
  for (int i = 0; i < 9; ++i) f->meta[i] = rd64(m + 8 * i);
  if (f->meta[2] > 5) return f->err = MTBLX_ERR_INVALID_COMPRESSION_ALGORITHM, MTBLX_E_FORMAT;
  uint64_t max_off = len - 512 - 13;  // wrapping, as the reference (:46)
  if (f->meta[0] > max_off) return f->err = MTBLX_ERR_INVALID_INDEX_BLOCK_OFFSET, MTBLX_E_FORMAT;
  return MTBLX_OK;
}

// Parse the framing of the block at file offset `off` (Reader::block, :140-164).
// Returns 0 and the stored-content window, or MTBLX_E_FORMAT (reference would panic:
// out-of-range slice / CRC assert) with *panic = 1.
extern "C" int mtblx_frame_block(const uint8_t* d, uint64_t len, uint32_t version, uint64_t off, int verify,
                                 uint64_t* content_off, uint64_t* content_len, int* panic) {
  *panic = 1;
  if (!(off < len)) return MTBLX_E_FORMAT;
  uint64_t ll, sz;
  if (version == 0) {
    if (off + 4 > len) return MTBLX_E_FORMAT;
    ll = 4;
    sz = rd32(d + off);
  } else {
    int k = vdec64(d + off, len - off, &sz);
    if (k < 0) return MTBLX_E_FORMAT;
    ll = (uint64_t)k;
  }
  uint64_t start = off + ll + 4;
  if (start > len || sz > len - start) return MTBLX_E_FORMAT;
  if (verify && rd32(d + off + ll) != mtblx_crc32c(d + start, sz)) return MTBLX_E_FORMAT;
  *content_off = start;
  *content_len = sz;
  *panic = 0;
  return MTBLX_OK;
}

extern "C" int mtblx_varint_decode64(const uint8_t* d, uint64_t len, uint64_t* out) { return vdec64(d, len, out); }
