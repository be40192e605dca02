// codecs_host.cpp — host block (de)compression for every CompressionType of the crate
// (/root/reference/src/compression.rs:57-81).  The north star keeps compression on the host.
//
//   None    borrowed as is                                   (:59)
//   Snappy  in-repo raw codec (snappy_host.cpp)              (:116-130, crate snap 1.x raw)
//   Zlib    zlib inflate / deflate, zlib-wrapped streams     (:85-106, crate flate2 1.x
//           ZlibDecoder::read_to_end / ZlibEncoder): the system zlib (linked)
//   Zstd    libzstd streaming                                (:140-156, crate zstd 0.5.1
//           stream::copy_decode / copy_encode, which wrap the C libzstd): libzstd.so.1,
//           loaded at run time (MTBLX_CODEC_UNSUPPORTED -> Error::Io if it is absent)
//   Lz4 / Lz4hc  Err("unsupported ... decompression")     (:63-67) -> MTBLX_CODEC_UNSUPPORTED
//
// Compressed bytes are not pinned to the crate's encoders (flate2 defaults to
// miniz_oxide, the zstd crate to its own bundled libzstd); decompression is format-defined.
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "mtblx.h"
#include "mtblx_host.h"

namespace {

// ---- zlib (flate2's ZlibDecoder over a byte slice: inflate until the stream ends; bytes after
// the end are never read; input exhausted first -> UnexpectedEof -> Err) ----
int zlib_decompress(const uint8_t* src, uint64_t n, std::vector<uint8_t>& out) {
  z_stream z;
  memset(&z, 0, sizeof z);
  if (inflateInit(&z) != Z_OK) return MTBLX_CODEC_CORRUPT;
  out.clear();
  uint64_t in_left = n;
  const uint8_t* in = src;
  int r = Z_OK;
  uint8_t buf[1 << 16];
  while (r != Z_STREAM_END) {
    if (z.avail_in == 0) {
      const uInt take = (uInt)std::min<uint64_t>(in_left, 1u << 30);
      z.next_in = const_cast<Bytef*>(in);
      z.avail_in = take;
      in += take;
      in_left -= take;
    }
    z.next_out = buf;
    z.avail_out = sizeof buf;
    r = inflate(&z, Z_NO_FLUSH);
    out.insert(out.end(), buf, buf + (sizeof buf - z.avail_out));
    if (r == Z_STREAM_END) break;
    if (r != Z_OK && r != Z_BUF_ERROR) { inflateEnd(&z); return MTBLX_CODEC_CORRUPT; }
    if (r == Z_BUF_ERROR && z.avail_in == 0 && in_left == 0) { inflateEnd(&z); return MTBLX_CODEC_CORRUPT; }
  }
  inflateEnd(&z);
  return MTBLX_CODEC_OK;
}

// flate2's ZlibEncoder streams any length; zlib's avail_in / avail_out are 32-bit, so the input
// is fed in pieces of <= 1 GiB (Z_NO_FLUSH), then Z_FINISH, the output grown as needed
int zlib_compress(uint32_t level, const uint8_t* src, uint64_t n, std::vector<uint8_t>& out) {
  z_stream z;
  memset(&z, 0, sizeof z);
  if (deflateInit(&z, (int)std::min<uint32_t>(level, 9)) != Z_OK) return MTBLX_CODEC_CORRUPT;
  constexpr uint64_t kPiece = 1ull << 30;
  out.resize(std::min<uint64_t>(deflateBound(&z, (uLong)std::min<uint64_t>(n, kPiece)) + 64, n + (1u << 20)) + 64);
  uint64_t in_left = n, done = 0;
  int r = Z_OK;
  for (;;) {
    if (z.avail_in == 0 && in_left) {
      const uint64_t take = std::min(in_left, kPiece);
      z.next_in = const_cast<Bytef*>(src + (n - in_left));
      z.avail_in = (uInt)take;
      in_left -= take;
    }
    if (out.size() - done < (1u << 16)) out.resize(out.size() + std::max<uint64_t>(out.size() / 2, 1u << 20));
    z.next_out = out.data() + done;
    z.avail_out = (uInt)std::min<uint64_t>(out.size() - done, kPiece);
    const uInt before = z.avail_out;
    r = deflate(&z, in_left == 0 ? Z_FINISH : Z_NO_FLUSH);
    done += before - z.avail_out;
    if (r == Z_STREAM_END) break;
    if (r != Z_OK && r != Z_BUF_ERROR) break;
  }
  out.resize(done);
  deflateEnd(&z);
  return r == Z_STREAM_END ? MTBLX_CODEC_OK : MTBLX_CODEC_CORRUPT;
}

// ---- zstd: libzstd.so.1 at run time (the stable streaming API only) ----
struct ZBufIn { const void* src; size_t size; size_t pos; };
struct ZBufOut { void* dst; size_t size; size_t pos; };
struct Zstd {
  void* (*createDStream)();
  size_t (*freeDStream)(void*);
  size_t (*initDStream)(void*);
  size_t (*decompressStream)(void*, ZBufOut*, ZBufIn*);
  unsigned (*isError)(size_t);
  size_t (*compress)(void*, size_t, const void*, size_t, int);
  size_t (*compressBound)(size_t);
  bool ok = false;
};

const Zstd& zstd() {
  static Zstd z;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    z.createDStream = reinterpret_cast<void* (*)()>(dlsym(h, "ZSTD_createDStream"));
    z.freeDStream = reinterpret_cast<size_t (*)(void*)>(dlsym(h, "ZSTD_freeDStream"));
    z.initDStream = reinterpret_cast<size_t (*)(void*)>(dlsym(h, "ZSTD_initDStream"));
    z.decompressStream = reinterpret_cast<size_t (*)(void*, ZBufOut*, ZBufIn*)>(dlsym(h, "ZSTD_decompressStream"));
    z.isError = reinterpret_cast<unsigned (*)(size_t)>(dlsym(h, "ZSTD_isError"));
    z.compress = reinterpret_cast<size_t (*)(void*, size_t, const void*, size_t, int)>(dlsym(h, "ZSTD_compress"));
    z.compressBound = reinterpret_cast<size_t (*)(size_t)>(dlsym(h, "ZSTD_compressBound"));
    z.ok = z.createDStream && z.freeDStream && z.initDStream && z.decompressStream && z.isError && z.compress &&
           z.compressBound;
  });
  return z;
}

// zstd::stream::copy_decode: every frame until the input ends; a frame cut short -> Err
int zstd_decompress(const uint8_t* src, uint64_t n, std::vector<uint8_t>& out) {
  const Zstd& Z = zstd();
  if (!Z.ok) return MTBLX_CODEC_UNSUPPORTED;
  out.clear();
  void* ds = Z.createDStream();
  if (!ds) return MTBLX_CODEC_CORRUPT;
  size_t r = Z.initDStream(ds);
  if (Z.isError(r)) { Z.freeDStream(ds); return MTBLX_CODEC_CORRUPT; }
  ZBufIn in{src, (size_t)n, 0};
  uint8_t buf[1 << 16];
  size_t last = 0;   // 0 = at a frame boundary
  while (in.pos < in.size) {
    ZBufOut o{buf, sizeof buf, 0};
    last = Z.decompressStream(ds, &o, &in);
    if (Z.isError(last)) { Z.freeDStream(ds); return MTBLX_CODEC_CORRUPT; }
    out.insert(out.end(), buf, buf + o.pos);
    if (o.pos == 0 && in.pos == in.size) break;
  }
  // flush what the decoder still holds for a completed frame
  for (int k = 0; k < 1 << 20 && last != 0; ++k) {
    ZBufOut o{buf, sizeof buf, 0};
    last = Z.decompressStream(ds, &o, &in);
    if (Z.isError(last)) { Z.freeDStream(ds); return MTBLX_CODEC_CORRUPT; }
    out.insert(out.end(), buf, buf + o.pos);
    if (o.pos == 0) break;
  }
  Z.freeDStream(ds);
  return last == 0 ? MTBLX_CODEC_OK : MTBLX_CODEC_CORRUPT;   // input ended inside a frame
}

int zstd_compress(uint32_t level, const uint8_t* src, uint64_t n, std::vector<uint8_t>& out) {
  const Zstd& Z = zstd();
  if (!Z.ok) return MTBLX_CODEC_UNSUPPORTED;
  out.resize(Z.compressBound((size_t)n));
  const size_t r = Z.compress(out.data(), out.size(), src, (size_t)n, (int)level);
  if (Z.isError(r)) return MTBLX_CODEC_CORRUPT;
  out.resize(r);
  return MTBLX_CODEC_OK;
}

int snappy_decompress(const uint8_t* src, uint64_t n, std::vector<uint8_t>& out) {
  uint64_t u = 0;
  if (mtblx_snappy_uncompressed_len(src, n, &u) != MTBLX_SNAPPY_OK || u > (1ull << 40)) return MTBLX_CODEC_CORRUPT;
  out.resize(u);
  uint64_t got = 0;
  const int r = mtblx_snappy_decompress(src, n, out.data(), u, &got);
  return (r == MTBLX_SNAPPY_OK && got == u) ? MTBLX_CODEC_OK : MTBLX_CODEC_CORRUPT;
}

int decompress_vec(uint32_t c, const uint8_t* src, uint64_t n, std::vector<uint8_t>& out) {
  switch (c) {
    case 0: out.assign(src, src + n); return MTBLX_CODEC_OK;
    case 1: return snappy_decompress(src, n, out);
    case 2: return zlib_decompress(src, n, out);
    case 5: return zstd_decompress(src, n, out);
    default: return MTBLX_CODEC_UNSUPPORTED;   // Lz4 / Lz4hc (:63-67), anything else
  }
}

}  // namespace

int mtblx_compress_vec(uint32_t c, uint32_t level, const uint8_t* src, uint64_t n, std::vector<uint8_t>& out) {
  switch (c) {
    case 0: out.assign(src, src + n); return MTBLX_CODEC_OK;
    case 1: {
      out.resize(mtblx_snappy_max_compressed_len(n));
      uint64_t zl = 0;
      if (mtblx_snappy_compress(src, n, out.data(), out.size(), &zl) != MTBLX_SNAPPY_OK) return MTBLX_CODEC_CORRUPT;
      out.resize(zl);
      return MTBLX_CODEC_OK;
    }
    case 2: return zlib_compress(level, src, n, out);
    case 5: return zstd_compress(level, src, n, out);
    default: return MTBLX_CODEC_UNSUPPORTED;
  }
}

extern "C" int mtblx_codec_available(uint32_t compression) {
  if (compression == 5) return zstd().ok ? 1 : 0;
  return compression <= 2 ? 1 : 0;
}

extern "C" int mtblx_decompress(uint32_t compression, const uint8_t* src, uint64_t n, uint8_t** out,
                                uint64_t* out_len) {
  if (!out || !out_len || (n && !src)) return MTBLX_E_INVAL;
  std::vector<uint8_t> v;
  const int r = decompress_vec(compression, src, n, v);
  *out = nullptr;
  *out_len = 0;
  if (r != MTBLX_CODEC_OK) return r;
  *out = static_cast<uint8_t*>(malloc(v.size() ? v.size() : 1));
  if (!*out) return MTBLX_E_INVAL;
  if (!v.empty()) memcpy(*out, v.data(), v.size());
  *out_len = v.size();
  return MTBLX_CODEC_OK;
}

extern "C" int mtblx_compress(uint32_t compression, uint32_t level, const uint8_t* src, uint64_t n, uint8_t** out,
                              uint64_t* out_len) {
  if (!out || !out_len || (n && !src)) return MTBLX_E_INVAL;
  std::vector<uint8_t> v;
  const int r = mtblx_compress_vec(compression, level, src, n, v);
  *out = nullptr;
  *out_len = 0;
  if (r != MTBLX_CODEC_OK) return r;
  *out = static_cast<uint8_t*>(malloc(v.size() ? v.size() : 1));
  if (!*out) return MTBLX_E_INVAL;
  if (!v.empty()) memcpy(*out, v.data(), v.size());
  *out_len = v.size();
  return MTBLX_CODEC_OK;
}

extern "C" uint64_t mtblx_decompress_blocks(uint32_t compression, const uint8_t* file, const uint64_t* blk_off,
                                            const uint32_t* blk_len, uint64_t nblk, uint32_t threads, uint8_t** dst,
                                            uint64_t* dst_off, uint64_t* dst_len, int32_t* st) {
  if (!dst || !dst_off || !dst_len) return nblk ? nblk : 1;
  *dst = nullptr;
  std::vector<std::vector<uint8_t>> parts(nblk);
  std::atomic<uint64_t> bad{0};
  auto work = [&](uint64_t b0, uint64_t b1) {
    uint64_t nb = 0;
    for (uint64_t b = b0; b < b1; ++b) {
      const int r = decompress_vec(compression, file + blk_off[b], blk_len[b], parts[b]);
      if (r != MTBLX_CODEC_OK) parts[b].clear();
      if (st) st[b] = r;
      nb += r != MTBLX_CODEC_OK;
    }
    bad += nb;
  };
  threads = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(threads ? threads : 16, nblk ? nblk : 1));
  if (threads == 1) {
    work(0, nblk);
  } else {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < threads; ++t) th.emplace_back(work, nblk * t / threads, nblk * (t + 1) / threads);
    for (auto& x : th) x.join();
  }
  uint64_t total = 0;
  for (uint64_t b = 0; b < nblk; ++b) {
    dst_off[b] = total;
    dst_len[b] = parts[b].size();
    total += (parts[b].size() + 15) & ~15ull;
  }
  *dst = static_cast<uint8_t*>(malloc(total ? total : 16));
  if (!*dst) return nblk ? nblk : 1;
  auto cp = [&](uint64_t b0, uint64_t b1) {
    for (uint64_t b = b0; b < b1; ++b)
      if (!parts[b].empty()) memcpy(*dst + dst_off[b], parts[b].data(), parts[b].size());
  };
  if (threads == 1) {
    cp(0, nblk);
  } else {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < threads; ++t) th.emplace_back(cp, nblk * t / threads, nblk * (t + 1) / threads);
    for (auto& x : th) x.join();
  }
  return bad.load();
}
