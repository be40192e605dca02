// snappy_host.cpp — host snappy "raw" codec for CompressionType::Snappy.
//
// The reference wraps the `snap` crate (1.x, raw format, no framing):
//   snappy_decompress   /root/reference/src/compression.rs:116-119  snap::raw::Decoder::decompress_vec
//   snappy_compress     src/compression.rs:126-130                   snap::raw::Encoder::compress_vec
// Reader::block decompresses every data block after its CRC check (src/reader.rs:166-170) and
// write_block compresses every data block before framing it (src/writer.rs:213-214); the index
// block is always stored uncompressed (src/writer.rs:165-173).  Per BASELINE.json north_star
// compression stays on the host: this file is that host stage, written in-repo so the GPU box
// does not depend on a system libsnappy.
//
// Format (snappy format_description.txt): varint32 uncompressed length, then elements
//   tag&3 == 0  literal   len-1 = tag>>2 (< 60) or the next 1..4 LE bytes (tag>>2 = 60..63)
//   tag&3 == 1  copy      len = 4 + ((tag>>2)&7), offset = (tag>>5)<<8 | next byte
//   tag&3 == 2  copy      len = 1 + (tag>>2),     offset = next 2 LE bytes
//   tag&3 == 3  copy      len = 1 + (tag>>2),     offset = next 4 LE bytes
// A copy's offset must be 1 .. bytes produced so far; copies may overlap their own output.
// Decompression is format-defined, so any conforming decoder yields the reference's bytes.
// Compressed bytes are NOT pinned to the reference (no test pins them); they
// only have to be valid snappy (tests cross-check with libsnappy where the image has it).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "mtblx.h"
#include "mtblx_host.h"

namespace {

inline uint32_t ld16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }
inline uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint64_t ld64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

// varint32 preamble; returns bytes used, 0 on error (unterminated / more than 32 bits)
inline uint32_t read_len(const uint8_t* s, uint64_t n, uint64_t& out) {
  uint64_t v = 0;
  for (uint32_t i = 0; i < 5 && i < n; ++i) {
    v |= (uint64_t)(s[i] & 0x7f) << (7 * i);
    if (!(s[i] & 0x80)) {
      if (v > 0xFFFFFFFFull) return 0;
      out = v;
      return i + 1;
    }
  }
  return 0;
}

// decode the element stream [s, se) into exactly dst[0 .. want)
int decode_body(const uint8_t* s, const uint8_t* se, uint8_t* dst, uint64_t want) {
  uint8_t* d = dst;
  uint8_t* const de = dst + want;
  while (s < se) {
    const uint32_t tag = *s++;
    uint64_t len, off;
    if ((tag & 3) == 0) {  // literal
      len = (tag >> 2) + 1;
      if (len > 60) {
        const uint32_t nb = (uint32_t)len - 60;
        if ((uint64_t)(se - s) < nb) return MTBLX_SNAPPY_CORRUPT;
        uint64_t l = 0;
        for (uint32_t i = 0; i < nb; ++i) l |= (uint64_t)s[i] << (8 * i);
        s += nb;
        len = l + 1;
      }
      if ((uint64_t)(se - s) < len || (uint64_t)(de - d) < len) return MTBLX_SNAPPY_CORRUPT;
      memcpy(d, s, len);
      d += len;
      s += len;
      continue;
    }
    if ((tag & 3) == 1) {
      if (se - s < 1) return MTBLX_SNAPPY_CORRUPT;
      len = 4 + ((tag >> 2) & 7);
      off = ((uint64_t)(tag >> 5) << 8) | *s++;
    } else if ((tag & 3) == 2) {
      if (se - s < 2) return MTBLX_SNAPPY_CORRUPT;
      len = 1 + (tag >> 2);
      off = ld16(s);
      s += 2;
    } else {
      if (se - s < 4) return MTBLX_SNAPPY_CORRUPT;
      len = 1 + (tag >> 2);
      off = ld32(s);
      s += 4;
    }
    if (off == 0 || off > (uint64_t)(d - dst) || (uint64_t)(de - d) < len) return MTBLX_SNAPPY_CORRUPT;
    const uint8_t* src = d - off;
    if (off >= len) {
      memcpy(d, src, len);
    } else {
      for (uint64_t i = 0; i < len; ++i) d[i] = src[i];  // overlapping copy: byte order matters
    }
    d += len;
  }
  return d == de ? MTBLX_SNAPPY_OK : MTBLX_SNAPPY_CORRUPT;
}

// ---------------- compressor: greedy LZ77 over 64 KiB fragments, 14-bit hash ----------------
constexpr uint32_t kFrag = 1u << 16;
constexpr int kHashBits = 14;

inline uint32_t hash4(uint32_t x) { return (x * 0x1e35a7bdu) >> (32 - kHashBits); }

inline uint8_t* emit_literal(uint8_t* o, const uint8_t* s, uint32_t len) {
  const uint32_t n = len - 1;
  if (n < 60) {
    *o++ = (uint8_t)(n << 2);
  } else {
    const uint32_t nb = n < (1u << 8) ? 1 : n < (1u << 16) ? 2 : n < (1u << 24) ? 3 : 4;
    *o++ = (uint8_t)((59 + nb) << 2);
    for (uint32_t i = 0; i < nb; ++i) *o++ = (uint8_t)(n >> (8 * i));
  }
  memcpy(o, s, len);
  return o + len;
}

inline uint8_t* emit_copy_upto64(uint8_t* o, uint32_t off, uint32_t len) {  // 4 <= len <= 64
  if (len < 12 && off < 2048) {
    *o++ = (uint8_t)(1 | ((len - 4) << 2) | ((off >> 8) << 5));
    *o++ = (uint8_t)off;
  } else {
    *o++ = (uint8_t)(2 | ((len - 1) << 2));
    *o++ = (uint8_t)off;
    *o++ = (uint8_t)(off >> 8);
  }
  return o;
}

inline uint8_t* emit_copy(uint8_t* o, uint32_t off, uint32_t len) {
  while (len >= 68) { o = emit_copy_upto64(o, off, 64); len -= 64; }
  if (len > 64) { o = emit_copy_upto64(o, off, 60); len -= 60; }
  return emit_copy_upto64(o, off, len);
}

uint8_t* compress_fragment(const uint8_t* in, uint32_t n, uint8_t* o, uint16_t* table) {
  const uint8_t* lit = in;
  if (n >= 15) {
    memset(table, 0, sizeof(uint16_t) << kHashBits);
    const uint8_t* const limit = in + n - 4;   // last position a 4-byte match can start
    const uint8_t* ip = in + 1;
    uint32_t skip = 32;
    while (ip <= limit) {
      const uint32_t cur = ld32(ip);
      const uint32_t h = hash4(cur);
      const uint8_t* cand = in + table[h];
      table[h] = (uint16_t)(ip - in);
      if (cand < ip && ld32(cand) == cur) {
        if (ip > lit) o = emit_literal(o, lit, (uint32_t)(ip - lit));
        const uint8_t* e = in + n;
        const uint8_t* a = ip + 4;
        const uint8_t* b = cand + 4;
        while (a + 8 <= e && ld64(a) == ld64(b)) { a += 8; b += 8; }
        while (a < e && *a == *b) { ++a; ++b; }
        o = emit_copy(o, (uint32_t)(ip - cand), (uint32_t)(a - ip));
        ip = a;
        lit = ip;
        skip = 32;
        if (ip <= limit) table[hash4(ld32(ip - 1))] = (uint16_t)(ip - 1 - in);
        continue;
      }
      ip += skip++ >> 5;   // accelerate through incompressible input
    }
  }
  if (lit < in + n) o = emit_literal(o, lit, (uint32_t)(in + n - lit));
  return o;
}

}  // namespace

extern "C" uint64_t mtblx_snappy_max_compressed_len(uint64_t n) { return 32 + n + n / 6; }

extern "C" int mtblx_snappy_uncompressed_len(const uint8_t* src, uint64_t n, uint64_t* out) {
  uint64_t v = 0;
  if (!src || !out || !read_len(src, n, v)) return MTBLX_SNAPPY_CORRUPT;
  *out = v;
  return MTBLX_SNAPPY_OK;
}

extern "C" int mtblx_snappy_decompress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap,
                                       uint64_t* out_len) {
  uint64_t want = 0;
  const uint32_t h = src ? read_len(src, n, want) : 0;
  if (!h) return MTBLX_SNAPPY_CORRUPT;
  if (want > cap) return MTBLX_SNAPPY_TOO_SMALL;
  if (out_len) *out_len = want;
  return decode_body(src + h, src + n, dst, want);
}

extern "C" int mtblx_snappy_compress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out_len) {
  if (n > 0xFFFFFFFFull || cap < mtblx_snappy_max_compressed_len(n)) return MTBLX_SNAPPY_TOO_SMALL;
  uint8_t* o = dst;
  uint64_t v = n;
  while (v >= 128) { *o++ = (uint8_t)(v | 128); v >>= 7; }
  *o++ = (uint8_t)v;
  std::vector<uint16_t> table(1u << kHashBits);
  for (uint64_t p = 0; p < n; p += kFrag) {
    const uint32_t len = (uint32_t)std::min<uint64_t>(kFrag, n - p);
    o = compress_fragment(src + p, len, o, table.data());
  }
  *out_len = (uint64_t)(o - dst);
  return MTBLX_SNAPPY_OK;
}

extern "C" uint64_t mtblx_snappy_decompress_blocks(const uint8_t* file, const uint64_t* blk_off,
                                                   const uint32_t* blk_len, uint8_t* dst, const uint64_t* dst_off,
                                                   const uint64_t* dst_len, int32_t* st, uint64_t nblk,
                                                   uint32_t threads) {
  std::atomic<uint64_t> bad{0};
  auto work = [&](uint64_t b0, uint64_t b1) {
    uint64_t nb = 0;
    for (uint64_t b = b0; b < b1; ++b) {
      uint64_t got = 0;
      int r = mtblx_snappy_decompress(file + blk_off[b], blk_len[b], dst + dst_off[b], dst_len[b], &got);
      if (r == MTBLX_SNAPPY_OK && got != dst_len[b]) r = MTBLX_SNAPPY_CORRUPT;
      if (st) st[b] = r;
      nb += r != MTBLX_SNAPPY_OK;
    }
    bad += nb;
  };
  threads = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(threads, nblk ? nblk : 1));
  if (threads == 1) {
    work(0, nblk);
  } else {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < threads; ++t) th.emplace_back(work, nblk * t / threads, nblk * (t + 1) / threads);
    for (auto& x : th) x.join();
  }
  return bad.load();
}
