// reader.hip — MI355X (gfx950) index block -> data-block directory.
//
// The reference walks the index block one entry at a time (ReaderIntoIter::next,
// /root/reference/src/reader.rs:337-405) and, per entry, decodes the data block offset
// from the entry's value and frames the block:
//   block_at_index   src/reader.rs:177-186   varint_decode64(value) -> file offset
//   Reader::block    src/reader.rs:139-174   assert offset < len; varint64 (V2) / u32 (V1)
//                                            content length; crc32c; content slice
// Here the index block is first decoded like any other block (mtblx_decode_blocks), then
// one thread per entry does the offset decode + framing for every entry at once.  The CRC
// and Block::init checks of Reader::block are done by mtblx_crc32c_blocks (framed) and by
// the decode kernel's per-block status, over the directory this kernel writes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "bounds.h"
#include "devinfo.h"
#include "crc_dev.h"
#include "mtblx.h"

namespace mtblx_rd {

// varint_length_packed over d[0..n) (src/varint.rs:1-10): 0 if no terminator
__device__ __forceinline__ uint32_t length_packed(const uint8_t* d, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) {
    MTBLX_CHK(d + i, 1);
    if (!(d[i] & 0x80u)) return (uint32_t)i + 1;
  }
  return 0;
}

// varint_decode64 on the slice d[0..n) (src/varint.rs:78-97 with varint_decode32 :44-61).
// Returns the consumed length (0 = unterminated), or -1 where the reference panics
// (n == 0: it indexes data[0]; fewer than 4 bytes on the 64-bit path: data[1..3]).
__device__ __forceinline__ int dec64(const uint8_t* d, uint64_t n, uint64_t& v) {
  if (n == 0) return -1;
  MTBLX_CHK(d, 1);
  const uint32_t l = length_packed(d, n < 10 ? n : 10);
  if (l < 5) {
    const uint32_t l32 = length_packed(d, n < 5 ? n : 5);
    uint32_t val = d[0] & 0x7fu;
    if (l32 > 1) val |= (uint32_t)(d[1] & 0x7fu) << 7;
    if (l32 > 2) val |= (uint32_t)(d[2] & 0x7fu) << 14;
    if (l32 > 3) val |= (uint32_t)(d[3] & 0x7fu) << 21;
    if (l32 > 4) val |= (uint32_t)d[4] << 28;
    v = val;
    return (int)l32;
  }
  MTBLX_CHK(d, l);
  uint64_t val = (uint64_t)(d[0] & 0x7fu) | ((uint64_t)(d[1] & 0x7fu) << 7) | ((uint64_t)(d[2] & 0x7fu) << 14) |
                 ((uint64_t)(d[3] & 0x7fu) << 21);
  uint32_t shift = 28;
  for (uint32_t i = 4; i < l; ++i) {
    val |= (uint64_t)(d[i] & 0x7fu) << shift;
    shift += 7;
  }
  v = val;
  return (int)l;
}

__global__ void k_block_dir(const uint8_t* file, uint64_t file_len, uint32_t version, const uint8_t* vals,
                            const uint32_t* val_end, uint64_t val_base, uint32_t nent, uint64_t* blk_off,
                            uint32_t* blk_len, int32_t* dir_st) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nent) return;
  MTBLX_CHK(val_end + i, 4);
  if (i) MTBLX_CHK(val_end + i - 1, 4);
  const uint64_t v0 = val_base + (i ? val_end[i - 1] : 0u), v1 = val_base + val_end[i];
  uint64_t off = 0, start = 0, sz = 0;
  int32_t st = MTBLX_DIR_OK;
  // block_at_index: varint_decode64(value, &mut offset), return length ignored
  if (dec64(vals + v0, v1 - v0, off) < 0) st = MTBLX_DIR_PANIC;
  // Reader::block
  if (st == MTBLX_DIR_OK && !(off < file_len)) st = MTBLX_DIR_PANIC;   // assert!(offset < len)
  uint64_t ll = 0;
  if (st == MTBLX_DIR_OK) {
    if (version == 0) {  // FormatV1: u32 LE length
      if (off + 4 > file_len) st = MTBLX_DIR_PANIC;
      else {
        ll = 4;
        MTBLX_CHK(file + off, 4);
        sz = (uint64_t)file[off] | ((uint64_t)file[off + 1] << 8) | ((uint64_t)file[off + 2] << 16) |
             ((uint64_t)file[off + 3] << 24);
      }
    } else {
      const int k = dec64(file + off, file_len - off, sz);
      if (k < 0) st = MTBLX_DIR_PANIC;
      else ll = (uint64_t)k;
    }
  }
  if (st == MTBLX_DIR_OK) {
    start = off + ll + 4;
    if (start > file_len || sz > file_len - start) st = MTBLX_DIR_PANIC;   // BytesView::slice assert
    else if (sz > 0xFFFFFFFFull) st = MTBLX_DIR_UNSUPPORTED;
  }
  MTBLX_CHK(blk_off + i, 8);
  MTBLX_CHK(blk_len + i, 4);
  MTBLX_CHK(dir_st + i, 4);
  blk_off[i] = (st == MTBLX_DIR_OK || st == MTBLX_DIR_UNSUPPORTED) ? start : 0;   // >= 4 GiB: start only
  blk_len[i] = st == MTBLX_DIR_OK ? (uint32_t)sz : 0u;
  dir_st[i] = st;
}


// ------------------------------------------------------------------------------------
// batched point lookups (f2): Reader::get (src/reader.rs:111-122) for many keys at once.
// One wave per query; the seek logic runs wave-uniform (every lane computes the same
// values), the lanes share the CRC-32C of each data block the lookup loads.
// Restated from the reference (and the oracle, oracle/mtbl_oracle.c):
//   BlockIter::seek          src/block.rs:154-194  (restart binary search + linear scan)
//   parse_next_key           src/block.rs:119-143  (truncate/extend, Vec capacity assert)
//   decode_entry             src/block.rs:216-238
//   ReaderIntoIter::new_from src/reader.rs:256-279, next (Get) :337-405
// Keys are never materialised: the scan tracks the length of the common prefix of the
// current key with the target and the sign of the first difference.
// ------------------------------------------------------------------------------------
constexpr uint64_t kU32 = 0xFFFFFFFFull;

struct Blk {
  const uint8_t* d;
  uint64_t L, R;
  uint32_t n;
  bool wide;   // u64 restart array (blocks >= 4 GiB)
};

struct It {
  uint64_t current, next, klen, kcap, c, voff, vlen;
  int cmp;            // sign of key[c] - target[c] when c < min(klen, tlen), else 0
  bool has_next;
  bool has_val;       // `val` is Some: an entry has been parsed (src/block.rs:70-71, :136)
};

enum { R_OK = 1, R_END = 0, R_PANIC = -1, R_LOOP = -2 };

__device__ __forceinline__ uint32_t rd32g(const uint8_t* p) {
  MTBLX_CHK(p, 4);
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// varint_decode32 on d[0..n), n >= 1
__device__ __forceinline__ uint32_t dec32g(const uint8_t* d, uint64_t n, uint32_t& v) {
  MTBLX_CHK(d, 1);
  const uint32_t l = length_packed(d, n < 5 ? n : 5);
  uint32_t val = d[0] & 0x7fu;
  if (l > 1) val |= (uint32_t)(d[1] & 0x7fu) << 7;
  if (l > 2) val |= (uint32_t)(d[2] & 0x7fu) << 14;
  if (l > 3) val |= (uint32_t)(d[3] & 0x7fu) << 21;
  if (l > 4) val |= (uint32_t)d[4] << 28;
  v = val;
  return l;
}

// Block::init (src/block.rs:16-49): 0 ok, 1 InvalidBlock, -1 panic.  A restart offset past
// u32::MAX means a u64 restart array (blocks >= 4 GiB, src/block.rs:25-42).
__device__ __forceinline__ int block_init(const uint8_t* d, uint64_t L, Blk& b) {
  if (L < 4) return 1;
  if (L < 8) return -1;
  const uint32_t n = rd32g(d + L - 4);
  uint64_t ro = L - (1ull + n) * 4ull;
  if (ro > kU32) {
    ro = L - (4ull + (uint64_t)n * 8ull);
    if (ro <= kU32) return 1;
  }
  if (ro > L - 4) return 1;
  b.d = d; b.L = L; b.R = ro; b.n = n; b.wide = ro > kU32;
  return 0;
}

// BlockIter::restart_point (src/block.rs:95-104): a u64 array keeps the 4-byte stride of the
// u32 one (the reference indexes `restarts + idx * 4` either way)
__device__ __forceinline__ uint64_t restart_point(const Blk& b, uint32_t i) {
  const uint8_t* p = b.d + b.R + 4ull * i;
  return b.wide ? ((uint64_t)rd32g(p) | ((uint64_t)rd32g(p + 4) << 32)) : (uint64_t)rd32g(p);
}

// decode_entry (src/block.rs:216-238): R_OK or R_PANIC
__device__ __forceinline__ int decode_entry(const Blk& b, uint64_t p, uint64_t limit, uint32_t& sh, uint32_t& ns,
                                            uint32_t& vl, uint64_t& pout) {
  if (limit - p < 3) return R_PANIC;
  if (p + 2 >= b.L) return R_PANIC;
  MTBLX_CHK(b.d + p, 3);
  uint32_t x = b.d[p], y = b.d[p + 1], z = b.d[p + 2];
  if ((x | y | z) < 128u) {
    p += 3;
  } else {
    if (p >= b.L) return R_PANIC;
    p += dec32g(b.d + p, b.L - p, x);
    if (p >= b.L) return R_PANIC;
    p += dec32g(b.d + p, b.L - p, y);
    if (p >= b.L) return R_PANIC;
    p += dec32g(b.d + p, b.L - p, z);
    if (!(p <= limit)) return R_PANIC;
  }
  const uint64_t sum = (uint64_t)y + z;
  if (sum > kU32 || (limit - p) < sum) return R_PANIC;
  sh = x; ns = y; vl = z; pout = p;
  return R_OK;
}

// the number of equal leading bytes of a[0..n) and b[0..n): 8-byte loads (never past n), the
// first difference by the lowest set byte of the XOR; then the last < 8 bytes one at a time
typedef uint64_t __attribute__((aligned(1))) u64u;
__device__ __forceinline__ uint64_t match_len(const uint8_t* a, const uint8_t* b, uint64_t n) {
  uint64_t c = 0;
  while (c + 8 <= n) {
    MTBLX_CHK(a + c, 8), MTBLX_CHK(b + c, 8);
    const uint64_t x = *reinterpret_cast<const u64u*>(a + c) ^ *reinterpret_cast<const u64u*>(b + c);
    if (x) return c + (uint64_t)(__builtin_ctzll(x) >> 3);
    c += 8;
  }
  while (c < n && (MTBLX_CHK(a + c, 1), MTBLX_CHK(b + c, 1), a[c] == b[c])) ++c;
  return c;
}

__device__ __forceinline__ int cmp_key(const It& it, uint64_t tlen) {   // Ord of key vs target
  if (it.cmp) return it.cmp;
  return it.klen < tlen ? -1 : (it.klen > tlen ? 1 : 0);
}

__device__ __forceinline__ void restart_at(const Blk& b, It& it, uint32_t i) {   // seek_to_restart_point
  it.klen = 0; it.c = 0; it.cmp = 0;
  it.has_next = true;
  it.next = restart_point(b, i);
}

// parse_next_key (src/block.rs:119-143) with the common-prefix tracking; R_OK / R_END /
// R_PANIC / R_LOOP (an entry that does not advance: the reference spins forever)
__device__ int parse_next_key(const Blk& b, It& it, const uint8_t* t, uint64_t tlen) {
  const uint64_t prev = it.current;
  it.current = it.has_next ? it.next : 0;
  if (it.current >= b.R) { it.current = b.R; return R_END; }
  uint32_t sh, ns, vl;
  uint64_t p;
  if (decode_entry(b, it.current, b.R, sh, ns, vl, p) != R_OK) return R_PANIC;
  if (!(it.kcap >= sh)) return R_PANIC;                     // Vec capacity assert (:132)
  const uint64_t m = sh < it.klen ? sh : it.klen;           // truncate (:134)
  if (p + ns > b.L) return R_PANIC;
  if (ns > 0 && it.kcap - m < ns) {                         // Vec growth (:135)
    uint64_t c = it.kcap * 2, req = m + ns;
    if (req > c) c = req;
    if (c < 8) c = 8;
    it.kcap = c;
  }
  if (m <= it.c) {            // the kept prefix matches the target: compare the suffix
    const uint64_t lim = ns < tlen - (tlen < m ? tlen : m) ? ns : tlen - (tlen < m ? tlen : m);
    const uint64_t j = m < tlen ? match_len(b.d + p, t + m, lim) : 0;
    const uint64_t c = m + j;
    it.cmp = (j < ns && c < tlen) ? (b.d[p + j] < t[c] ? -1 : 1) : 0;
    it.c = c;
  }                           // else: the first difference lies in the kept prefix
  it.klen = m + ns;
  it.has_next = true;
  it.next = p + ns + vl;
  it.voff = p + ns;
  it.vlen = vl;
  it.has_val = true;
  if (it.next == it.current && it.current == prev) return R_LOOP;
  return R_OK;
}

// BlockIter::seek (src/block.rs:154-194)
__device__ int seek(const Blk& b, It& it, const uint8_t* t, uint64_t tlen) {
  uint32_t left = 0, right = b.n - 1;
  while (left < right) {
    const uint32_t mid = (uint32_t)(((uint64_t)left + right + 1) / 2);
    uint32_t sh, ns, vl;
    uint64_t ko;
    if (decode_entry(b, restart_point(b, mid), b.R, sh, ns, vl, ko) != R_OK) return R_PANIC;
    if (sh != 0) return R_OK;                                 // "corruption": early return
    if (ko + ns > b.L) return R_PANIC;
    const uint64_t c = match_len(b.d + ko, t, ns < tlen ? ns : tlen);
    const int r = (c < ns && c < tlen) ? (b.d[ko + c] < t[c] ? -1 : 1) : (ns < tlen ? -1 : (ns > tlen ? 1 : 0));
    if (r < 0) left = mid;
    else right = mid - 1;
  }
  restart_at(b, it, left);
  for (uint64_t steps = 0;; ++steps) {
    const uint64_t before = it.current;
    const int r = parse_next_key(b, it, t, tlen);
    if (r != R_OK) return r == R_END ? R_OK : r;
    if (cmp_key(it, tlen) >= 0) return R_OK;
    if (it.next == it.current || (steps > 0 && it.current == before)) return R_LOOP;
  }
}

__device__ __forceinline__ bool valid(const Blk& b, const It& it) { return it.current < b.R; }

// BlockIter::init (src/block.rs:75-93)
__device__ __forceinline__ int iter_init(const Blk& b, It& it) {
  if (b.n == 0) return R_PANIC;
  it.current = b.R; it.has_next = false; it.next = 0; it.has_val = false;
  it.klen = 0; it.kcap = 0; it.c = 0; it.cmp = 0; it.voff = 0; it.vlen = 0;
  return R_OK;
}

// decompressed blocks of a compressed file (mtblx_get_decompressed), sorted by stored start
struct DecTab {
  const uint64_t* start;
  const uint64_t* doff;
  const uint64_t* dlen;
  const int32_t* st;
  uint32_t n;
  const uint8_t* dec;
};

struct FileCtx {
  const uint8_t* file;
  uint64_t len;
  uint32_t version;
  int verify;
  const uint32_t* T;   // crc byte table (LDS)
  int lane;
  DecTab tab;          // tab.dec == nullptr: the file is not compressed
};

// block_at_index + Reader::block (src/reader.rs:177-186, :139-174), in two halves around the
// checksum.  frame_at_index: the landed index entry's offset and the block's framing ->
// 0 = None (get() -> None), R_PANIC, 1 = framed: content [start, start + sz), stored checksum crc.
__device__ __forceinline__ int frame_at_index(const FileCtx& f, const Blk& ib, const It& ii, uint64_t& start,
                                              uint64_t& sz, uint32_t& crc) {
  if (!valid(ib, ii)) return 0;                                // get() -> None
  if (ii.voff + ii.vlen > ib.L) return R_PANIC;
  uint64_t off = 0;
  if (dec64(ib.d + ii.voff, ii.vlen, off) < 0) return R_PANIC;
  if (!(off < f.len)) return R_PANIC;
  uint64_t ll;
  if (f.version == 0) {
    if (off + 4 > f.len) return R_PANIC;
    ll = 4; sz = rd32g(f.file + off);
  } else {
    const int k = dec64(f.file + off, f.len - off, sz);
    if (k < 0) return R_PANIC;
    ll = (uint64_t)k;
  }
  start = off + ll + 4;
  if (start > f.len || sz > f.len - start) return R_PANIC;
  crc = rd32g(f.file + off + ll);
  return 1;
}
// after the checksum (when verified): decompression (the caller's table) and Block::init ->
// 1 = Some(block), R_PANIC, 2 = Err(InvalidBlock), 3 = a compressed block the caller's table does
// not hold (its stored content [mstart, + msz) passed framing and the checksum)
__device__ __forceinline__ int block_after_crc(const FileCtx& f, uint64_t start, uint64_t sz, Blk& out,
                                               uint64_t& mstart, uint64_t& msz) {
  const uint8_t* content = f.file + start;
  if (f.tab.dec) {   // decompress (src/reader.rs:166-170): the caller's decompressed copy
    uint32_t lo = 0, hi = f.tab.n;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) / 2;
      MTBLX_CHK(f.tab.start + mid, 8);
      if (f.tab.start[mid] < start) lo = mid + 1;
      else hi = mid;
    }
    if (lo == f.tab.n || f.tab.start[lo] != start) {   // not decompressed by the caller (yet)
      mstart = start;
      msz = sz;
      return 3;
    }
    if (f.tab.st[lo] != 0) return 2;   // the crate's decompress error: Err(Io)
    MTBLX_CHK(f.tab.doff + lo, 8);
    MTBLX_CHK(f.tab.dlen + lo, 8);
    content = f.tab.dec + f.tab.doff[lo];
    sz = f.tab.dlen[lo];
  }
  const int bi = block_init(content, sz, out);
  if (bi == 1) return 2;
  if (bi < 0) return R_PANIC;
  return 1;
}
// the whole of it, for a wave-uniform caller (the checksum shared by the wave's lanes)
__device__ int block_at_index(const FileCtx& f, const Blk& ib, const It& ii, Blk& out, uint64_t& mstart,
                              uint64_t& msz) {
  uint64_t start = 0, sz = 0;
  uint32_t crc = 0;
  const int fr = frame_at_index(f, ib, ii, start, sz, crc);
  if (fr != 1) return fr;
  if (f.verify && mtblx_crc::wave_crc32c(f.file + start, sz, f.T, f.lane) != crc) return R_PANIC;
  return block_after_crc(f, start, sz, out, mstart, msz);
}

__global__ void __launch_bounds__(256) k_get(const uint8_t* file, uint64_t file_len, uint32_t version, int verify,
                                             uint64_t idx_off, uint64_t idx_len, DecTab tab, const uint8_t* qkeys,
                                             const uint64_t* qend, uint32_t nq, int32_t* st, uint64_t* voff,
                                             uint64_t* vlen) {
  __shared__ uint32_t T[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) T[i] = mtblx_crc::kTab.byte[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (blockDim.x / 64);
  const FileCtx f{file, file_len, version, verify, T, lane, tab};
  const uint8_t* vbase = tab.dec ? tab.dec : file;   // values are offsets into the scanned bytes
  for (uint32_t q = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); q < nq; q += waves) {
    MTBLX_CHK(qend + q, 8);
    const uint64_t k0 = q ? qend[q - 1] : 0, k1 = qend[q];
    const uint8_t* t = qkeys + k0;
    const uint64_t tl = k1 - k0;
    int32_t res = MTBLX_GET_NONE;
    uint64_t ro = 0, rl = 0;
    Blk ib{};
    It ii{}, di{};
    Blk db{};
    do {
      const int ibi = block_init(file + idx_off, idx_len, ib);   // the Reader's index block
      if (ibi != 0) { res = ibi == 1 ? MTBLX_GET_ERR : MTBLX_GET_PANIC; break; }
      if (iter_init(ib, ii) != R_OK) { res = MTBLX_GET_PANIC; break; }
      int r = seek(ib, ii, t, tl);                                // new_from: index_iter.seek(key)
      if (r != R_OK) { res = r == R_LOOP ? MTBLX_GET_LOOP : MTBLX_GET_PANIC; break; }
      uint64_t ms = 0, ml = 0;
      int b = block_at_index(f, ib, ii, db, ms, ml);
      if (b == R_PANIC) { res = MTBLX_GET_PANIC; break; }
      if (b == 3) { res = MTBLX_GET_MISSING; ro = ms; rl = ml; break; }
      if (b == 2) { res = MTBLX_GET_ERR; break; }                  // Err at open (new_get)
      if (b == 0) break;                                           // no block: next() -> None
      if (iter_init(db, di) != R_OK) { res = MTBLX_GET_PANIC; break; }
      r = seek(db, di, t, tl);                                     // bi.seek(key)
      if (r != R_OK) { res = r == R_LOOP ? MTBLX_GET_LOOP : MTBLX_GET_PANIC; break; }
      // next() (first call, Get)
      if (valid(db, di)) {
        if (di.voff + di.vlen > db.L) { res = MTBLX_GET_PANIC; break; }
        if (cmp_key(di, tl) == 0) { res = MTBLX_GET_FOUND; ro = (uint64_t)(db.d - vbase) + di.voff; rl = di.vlen; }
        break;
      }
      // the seek ran past the end of the block: the next index entry's first record
      if (!valid(ib, ii)) break;
      r = parse_next_key(ib, ii, t, tl);
      if (r == R_PANIC) { res = MTBLX_GET_PANIC; break; }
      if (r == R_LOOP) { res = MTBLX_GET_LOOP; break; }
      if (!valid(ib, ii)) break;
      b = block_at_index(f, ib, ii, db, ms, ml);
      if (b == R_PANIC) { res = MTBLX_GET_PANIC; break; }
      if (b == 3) { res = MTBLX_GET_MISSING; ro = ms; rl = ml; break; }
      if (b == 2) {
        // next() returned Some(Err(InvalidBlock)).  Reader::get matches Some(_) and returns
        // Ok(ReaderIntoGet::new(iter.bi)) with iter.bi still the OLD block iterator (it is not
        // reassigned on Err, src/reader.rs:111-122, :376-379): its `val` is the last entry the
        // seek parsed -> Ok(Some(that value)), or Ok(None) if the seek parsed none (:195-203).
        // block_at_index left db untouched (Block::init failed before assigning it).
        if (di.has_val) { res = MTBLX_GET_FOUND; ro = (uint64_t)(db.d - vbase) + di.voff; rl = di.vlen; }
        break;
      }
      if (b == 0) break;
      if (iter_init(db, di) != R_OK) { res = MTBLX_GET_PANIC; break; }
      restart_at(db, di, 0);                                       // seek_to_first
      r = parse_next_key(db, di, t, tl);
      if (r == R_PANIC) { res = MTBLX_GET_PANIC; break; }
      if (!valid(db, di)) break;
      if (di.voff + di.vlen > db.L) { res = MTBLX_GET_PANIC; break; }
      if (cmp_key(di, tl) == 0) { res = MTBLX_GET_FOUND; ro = (uint64_t)(db.d - vbase) + di.voff; rl = di.vlen; }
    } while (false);
    MTBLX_CHK(st + q, 4);
    MTBLX_CHK(voff + q, 8);
    MTBLX_CHK(vlen + q, 8);
    if (lane == 0) { st[q] = res; voff[q] = ro; vlen[q] = rl; }
  }
}

// The same lookups, one LANE per query (round 5): the seeks run per lane -- 64 queries in flight
// per wave instead of one -- and only the checksums are shared: after each stage the wave
// computes, one block at a time, the CRC-32C of every block a lane landed on (its lanes
// cooperating), and each lane goes on with its own result.  The stages follow k_get's control
// flow exactly: A = index seek + framing of the landed block; B = its Block::init, the block
// seek, and when the seek runs past the block's end the next index entry's framing; C = that
// block's Block::init and its first record.
__device__ __forceinline__ void lanes_crc(const FileCtx& f, bool need, uint64_t start, uint64_t sz, uint32_t stored,
                                          bool& ok) {
  uint64_t m = __ballot(need);
  ok = true;
  while (m) {
    const int j = __builtin_ctzll(m);
    m &= m - 1;
    const uint64_t st = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(start >> 32), j) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)start, j);
    const uint64_t n = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(sz >> 32), j) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sz, j);
    const uint32_t c = mtblx_crc::wave_crc32c(f.file + st, n, f.T, f.lane);
    if (f.lane == j) ok = c == stored;
  }
}

__global__ void __launch_bounds__(256) k_get_lanes(const uint8_t* file, uint64_t file_len, uint32_t version,
                                                   int verify, uint64_t idx_off, uint64_t idx_len, DecTab tab,
                                                   const uint8_t* qkeys, const uint64_t* qend, uint32_t nq, int32_t* st,
                                                   uint64_t* voff, uint64_t* vlen) {
  __shared__ uint32_t T[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) T[i] = mtblx_crc::kTab.byte[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const FileCtx f{file, file_len, version, verify, T, lane, tab};
  const uint8_t* vbase = tab.dec ? tab.dec : file;   // values are offsets into the scanned bytes
  const uint64_t all = (uint64_t)gridDim.x * blockDim.x;
  // wave-uniform trip count: the whole wave runs every stage and every checksum pass
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < nq; base += all) {
    const uint64_t q = base + (uint64_t)lane;
    bool live = q < nq;
    int32_t res = MTBLX_GET_NONE;
    uint64_t ro = 0, rl = 0, tl = 0, start = 0, sz = 0, ms = 0, ml = 0;
    uint32_t crc = 0;
    const uint8_t* t = qkeys;
    Blk ib{}, db{};
    It ii{}, di{};
    bool need = false, ok = true;
    // ---- stage A ----
    if (live) {
      MTBLX_CHK(qend + q, 8);
      const uint64_t k0 = q ? qend[q - 1] : 0, k1 = qend[q];
      t = qkeys + k0;
      tl = k1 - k0;
      do {
        const int ibi = block_init(file + idx_off, idx_len, ib);   // the Reader's index block
        if (ibi != 0) { res = ibi == 1 ? MTBLX_GET_ERR : MTBLX_GET_PANIC; live = false; break; }
        if (iter_init(ib, ii) != R_OK) { res = MTBLX_GET_PANIC; live = false; break; }
        const int r = seek(ib, ii, t, tl);                          // new_from: index_iter.seek(key)
        if (r != R_OK) { res = r == R_LOOP ? MTBLX_GET_LOOP : MTBLX_GET_PANIC; live = false; break; }
        const int fr = frame_at_index(f, ib, ii, start, sz, crc);
        if (fr == R_PANIC) { res = MTBLX_GET_PANIC; live = false; break; }
        if (fr == 0) { live = false; break; }                       // no block: next() -> None
        need = verify != 0;
      } while (false);
    }
    lanes_crc(f, live && need, start, sz, crc, ok);
    // ---- stage B ----
    need = false;
    if (live) {
      do {
        if (!ok) { res = MTBLX_GET_PANIC; live = false; break; }   // Reader::block's assert_eq
        const int b = block_after_crc(f, start, sz, db, ms, ml);
        if (b == R_PANIC) { res = MTBLX_GET_PANIC; live = false; break; }
        if (b == 3) { res = MTBLX_GET_MISSING; ro = ms; rl = ml; live = false; break; }
        if (b == 2) { res = MTBLX_GET_ERR; live = false; break; }   // Err at open (new_get)
        if (iter_init(db, di) != R_OK) { res = MTBLX_GET_PANIC; live = false; break; }
        int r = seek(db, di, t, tl);                                  // bi.seek(key)
        if (r != R_OK) { res = r == R_LOOP ? MTBLX_GET_LOOP : MTBLX_GET_PANIC; live = false; break; }
        if (valid(db, di)) {                                          // next() (first call, Get)
          if (di.voff + di.vlen > db.L) res = MTBLX_GET_PANIC;
          else if (cmp_key(di, tl) == 0) { res = MTBLX_GET_FOUND; ro = (uint64_t)(db.d - vbase) + di.voff; rl = di.vlen; }
          live = false;
          break;
        }
        // the seek ran past the end of the block: the next index entry's first record
        if (!valid(ib, ii)) { live = false; break; }
        r = parse_next_key(ib, ii, t, tl);
        if (r == R_PANIC) { res = MTBLX_GET_PANIC; live = false; break; }
        if (r == R_LOOP) { res = MTBLX_GET_LOOP; live = false; break; }
        if (!valid(ib, ii)) { live = false; break; }
        const int fr = frame_at_index(f, ib, ii, start, sz, crc);
        if (fr == R_PANIC) { res = MTBLX_GET_PANIC; live = false; break; }
        if (fr == 0) { live = false; break; }
        need = verify != 0;
      } while (false);
    }
    lanes_crc(f, live && need, start, sz, crc, ok);
    // ---- stage C ----
    if (live) {
      do {
        if (!ok) { res = MTBLX_GET_PANIC; break; }
        const int b = block_after_crc(f, start, sz, db, ms, ml);
        if (b == R_PANIC) { res = MTBLX_GET_PANIC; break; }
        if (b == 3) { res = MTBLX_GET_MISSING; ro = ms; rl = ml; break; }
        if (b == 2) {
          // next() returned Some(Err(InvalidBlock)): Reader::get returns the OLD block
          // iterator's `val` (k_get above; src/reader.rs:111-122, :376-379, :195-203)
          if (di.has_val) { res = MTBLX_GET_FOUND; ro = (uint64_t)(db.d - vbase) + di.voff; rl = di.vlen; }
          break;
        }
        if (iter_init(db, di) != R_OK) { res = MTBLX_GET_PANIC; break; }
        restart_at(db, di, 0);                                       // seek_to_first
        const int r = parse_next_key(db, di, t, tl);
        if (r == R_PANIC) { res = MTBLX_GET_PANIC; break; }
        if (!valid(db, di)) break;
        if (di.voff + di.vlen > db.L) { res = MTBLX_GET_PANIC; break; }
        if (cmp_key(di, tl) == 0) { res = MTBLX_GET_FOUND; ro = (uint64_t)(db.d - vbase) + di.voff; rl = di.vlen; }
      } while (false);
    }
    if (q < nq) {
      MTBLX_CHK(st + q, 4), MTBLX_CHK(voff + q, 8), MTBLX_CHK(vlen + q, 8);
      st[q] = res;
      voff[q] = ro;
      vlen[q] = rl;
    }
  }
}

// ------------------------------------------------------------------------------------
// seek-based iteration (ReaderIntoIter::new_from / seek, src/reader.rs:256-335)
// ------------------------------------------------------------------------------------

// Reader::block (src/reader.rs:139-175) at a block_at_index offset: framing, checksum and
// Block::init.  MTBLX_SEEK_OK / _ERR / _PANIC / _UNSUPPORTED.
__device__ int frame_block(const FileCtx& f, uint64_t off, uint64_t& start, uint64_t& sz) {
  if (!(off < f.len)) return MTBLX_SEEK_PANIC;
  uint64_t ll;
  if (f.version == 0) {
    if (off + 4 > f.len) return MTBLX_SEEK_PANIC;
    ll = 4; sz = rd32g(f.file + off);
  } else {
    const int k = dec64(f.file + off, f.len - off, sz);
    if (k < 0) return MTBLX_SEEK_PANIC;
    ll = (uint64_t)k;
  }
  start = off + ll + 4;
  if (start > f.len || sz > f.len - start) return MTBLX_SEEK_PANIC;
  if (f.verify && mtblx_crc::wave_crc32c(f.file + start, sz, f.T, f.lane) != rd32g(f.file + off + ll))
    return MTBLX_SEEK_PANIC;
  Blk b;
  const int bi = block_init(f.file + start, sz, b);
  return bi == 1 ? MTBLX_SEEK_ERR : bi < 0 ? MTBLX_SEEK_PANIC : MTBLX_SEEK_OK;
}

__global__ void __launch_bounds__(256) k_index_seek(const uint8_t* file, uint64_t file_len, uint32_t version,
                                                    int verify, uint64_t idx_off, uint64_t idx_len,
                                                    const uint8_t* qkeys, const uint64_t* qend, uint32_t nq,
                                                    mtblx_index_seek* out) {
  __shared__ uint32_t T[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) T[i] = mtblx_crc::kTab.byte[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (blockDim.x / 64);
  const FileCtx f{file, file_len, version, verify, T, lane};
  for (uint32_t q = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); q < nq; q += waves) {
    MTBLX_CHK(qend + q, 8);
    const uint64_t k0 = q ? qend[q - 1] : 0;
    const uint8_t* t = qkeys + k0;
    const uint64_t tl = qend[q] - k0;
    mtblx_index_seek r{};
    r.block_status = MTBLX_SEEK_OK;
    Blk ib{};
    It ii{};
    do {
      const int ibi = block_init(file + idx_off, idx_len, ib);
      if (ibi != 0) { r.status = ibi == 1 ? MTBLX_SEEK_ERR : MTBLX_SEEK_PANIC; break; }
      if (iter_init(ib, ii) != R_OK) { r.status = MTBLX_SEEK_PANIC; break; }
      const int s = seek(ib, ii, t, tl);                          // index_iter.seek(key)
      if (s != R_OK) { r.status = s == R_LOOP ? MTBLX_SEEK_LOOP : MTBLX_SEEK_PANIC; break; }
      r.entry = ii.current;
      if (!valid(ib, ii)) break;                                   // get() -> None
      if (ii.voff + ii.vlen > ib.L) { r.status = MTBLX_SEEK_PANIC; break; }   // get()'s slice
      r.valid = 1;
      uint64_t off = 0;
      if (dec64(ib.d + ii.voff, ii.vlen, off) < 0) { r.status = MTBLX_SEEK_PANIC; break; }
      r.block_off = off;
      uint64_t start = 0, sz = 0;
      r.block_status = frame_block(f, off, start, sz);
      r.data_off = start;
      r.data_len = sz;
    } while (false);
    MTBLX_CHK(out + q, sizeof(mtblx_index_seek));
    if (lane == 0) out[q] = r;
  }
}

// BlockIter over one block with the key materialised in LDS (the emitting seek)
constexpr uint32_t kSeekStage = 65536;   // blocks up to this size are staged in LDS
constexpr uint32_t kSeekKey = 65536;     // longest key the emitting seek carries
enum { R_TOOLONG = -3 };

struct SIt {
  uint64_t current, next, klen, kcap, voff, vlen;
  bool has_next, has_val;
};

// Ord of K[0..kl) vs t[0..tl), the wave together
__device__ int wave_cmp(const uint8_t* K, uint64_t kl, const uint8_t* t, uint64_t tl, int lane) {
  const uint64_t m = kl < tl ? kl : tl;
  for (uint64_t c0 = 0; c0 < m; c0 += 64) {
    const uint64_t c = c0 + (uint64_t)lane;
    if (c < m) { MTBLX_CHK(K + c, 1); MTBLX_CHK(t + c, 1); }
    const bool diff = c < m && K[c] != t[c];
    const uint64_t bal = __ballot(diff);
    if (bal) {
      const uint64_t cc = c0 + (uint64_t)__builtin_ctzll(bal);
      return K[cc] < t[cc] ? -1 : 1;
    }
  }
  return kl < tl ? -1 : (kl > tl ? 1 : 0);
}

// parse_next_key (src/block.rs:119-143): R_OK / R_END / R_PANIC / R_TOOLONG (key past klim,
// the key buffer's size)
__device__ __forceinline__ int s_parse(const Blk& b, SIt& it, uint8_t* K, uint64_t klim, int lane) {
  it.current = it.has_next ? it.next : 0;
  if (it.current >= b.R) { it.current = b.R; return R_END; }
  uint32_t sh, ns, vl;
  uint64_t p;
  if (decode_entry(b, it.current, b.R, sh, ns, vl, p) != R_OK) return R_PANIC;
  if (!(it.kcap >= sh)) return R_PANIC;                       // Vec capacity assert (:132)
  const uint64_t m = sh < it.klen ? sh : it.klen;             // truncate (:134)
  if (p + ns > b.L) return R_PANIC;
  if (ns > 0 && it.kcap - m < ns) {                           // Vec growth (:135)
    uint64_t c = it.kcap * 2, req = m + ns;
    if (req > c) c = req;
    if (c < 8) c = 8;
    it.kcap = c;
  }
  if (m + ns > klim) return R_TOOLONG;
  for (uint32_t j = (uint32_t)lane; j < ns; j += 64) {
    MTBLX_CHK(K + m + j, 1);
    MTBLX_CHK(b.d + p + j, 1);
    K[m + j] = b.d[p + j];
  }
  __syncthreads();   // one-wave workgroup: orders the key writes (LDS or global) before other lanes read K
  it.klen = m + ns;
  it.has_next = true;
  it.next = p + ns + vl;
  it.voff = p + ns;
  it.vlen = vl;
  it.has_val = true;
  return R_OK;
}

// BlockIter::seek (src/block.rs:154-194) with the key materialised.  early: the binary search
// returned on a restart entry with shared != 0 -- the iterator is left as it was (the caller
// keeps its previous state; this matters for the live index iterator, src/reader.rs:303)
__device__ __forceinline__ int s_seek(const Blk& b, SIt& it, uint8_t* K, uint64_t klim, const uint8_t* t, uint64_t tl,
                                      int lane, bool& early) {
  uint32_t left = 0, right = b.n - 1;
  early = false;
  while (left < right) {
    const uint32_t mid = (uint32_t)(((uint64_t)left + right + 1) / 2);
    uint32_t sh, ns, vl;
    uint64_t ko;
    if (decode_entry(b, restart_point(b, mid), b.R, sh, ns, vl, ko) != R_OK) return R_PANIC;
    if (sh != 0) { early = true; return R_OK; }               // "corruption": early return
    if (ko + ns > b.L) return R_PANIC;
    if (wave_cmp(b.d + ko, ns, t, tl, lane) < 0) left = mid;
    else right = mid - 1;
  }
  it.klen = 0;                                                // seek_to_restart_point(left)
  it.has_next = true;
  it.next = restart_point(b, left);
  for (;;) {
    const int r = s_parse(b, it, K, klim, lane);
    if (r != R_OK) return r == R_END ? R_OK : r;
    if (wave_cmp(K, it.klen, t, tl, lane) >= 0) return R_OK;
    if (it.next == it.current) return R_LOOP;
  }
}

// GK: the key lives in the caller's buffer (kbuf + q * kbuf_cap) instead of LDS -- keys longer
// than 64 KiB (mtblx_block_seek_batch_kbuf).  DEFER: value bytes are not copied by the wave;
// record r's value source (content offset) goes to vsrc[q * rec_cap + r] and the caller moves
// the bytes with the whole grid (mtblx_block_seek_batch_ex + mtblx_copy_ranges: blocks >= 4 GiB
// hold values of GiBs, which one wave copies at a few GB/s)
template <bool GK, bool DEFER = false>
__global__ void __launch_bounds__(64) k_block_seek(const uint8_t* data, const uint8_t* qkeys, const uint64_t* qend,
                                                   uint32_t nq, mtblx_block_seek* qs, uint8_t* okeys,
                                                   uint64_t keys_cap, uint8_t* ovals, uint64_t vals_cap,
                                                   uint64_t* oke, uint64_t* ove, uint64_t* okcap, uint64_t rec_cap,
                                                   uint8_t* kbuf, uint64_t kbuf_cap, uint64_t* vsrc = nullptr) {
  __shared__ uint8_t stage[kSeekStage];
  __shared__ uint8_t Klds[GK ? 1 : kSeekKey];
  const int lane = threadIdx.x;
  const uint64_t klim = GK ? kbuf_cap : kSeekKey;
  for (uint32_t q = blockIdx.x; q < nq; q += gridDim.x) {
    uint8_t* K = GK ? kbuf + (uint64_t)q * kbuf_cap : Klds;
    MTBLX_CHK(qs + q, sizeof(mtblx_block_seek));
    MTBLX_CHK(qend + q, 8);
    mtblx_block_seek Q = qs[q];
    const uint64_t k0 = q ? qend[q - 1] : 0;
    const uint8_t* t = qkeys + k0;
    const uint64_t tl = qend[q] - k0;
    Q.status = MTBLX_SEEK_OK;
    Q.end = MTBLX_EMIT_END;
    Q.nrec = Q.key_bytes = Q.val_bytes = 0;
    Q.entry = 0;
    Q.early = 0;
    Q.stop_off = 0;
    const uint64_t L = Q.data_len;
    const uint8_t* src = data + Q.data_off;
    const uint8_t* d = src;
    Blk b{};
    SIt it{};
    do {
      __syncthreads();
      if (L <= kSeekStage) {
        for (uint64_t i = (uint64_t)lane; i < L; i += 64) {
          MTBLX_CHK(src + i, 1);
          stage[i] = src[i];
        }
        __syncthreads();
        d = stage;
      }
      const int bi = block_init(d, L, b);                          // Block::init
      if (bi != 0) { Q.status = bi == 1 ? MTBLX_SEEK_ERR : MTBLX_SEEK_PANIC; break; }
      if (b.n == 0) { Q.status = MTBLX_SEEK_PANIC; break; }        // BlockIter::init assert
      it.current = b.R;
      it.has_next = false;
      it.kcap = Q.kcap;
      int r;
      bool early = false;
      if (Q.first == 1) {                                          // seek_to_first
        it.klen = 0;
        it.has_next = true;
        it.next = restart_point(b, 0);
        r = s_parse(b, it, K, klim, lane);
        if (r == R_END) r = R_OK;
      } else if (Q.first == 2) {                                   // resume: next() from a held state
        if (tl > klim) {
          r = R_TOOLONG;
        } else {
          for (uint64_t j = (uint64_t)lane; j < tl; j += 64) {
            MTBLX_CHK(K + j, 1);
            MTBLX_CHK(t + j, 1);
            K[j] = t[j];
          }
          __syncthreads();
          it.klen = tl;
          it.has_next = true;
          it.next = Q.resume_off;
          r = s_parse(b, it, K, klim, lane);
          if (r == R_END) r = R_OK;
        }
      } else {
        r = s_seek(b, it, K, klim, t, tl, lane, early);
      }
      Q.early = early ? 1 : 0;
      if (r != R_OK) {
        Q.status = r == R_LOOP ? MTBLX_SEEK_LOOP : r == R_TOOLONG ? MTBLX_SEEK_UNSUPPORTED : MTBLX_SEEK_PANIC;
        break;
      }
      Q.entry = it.current;
      // the records: get(), then next() until get() is None (ReaderIntoIter::next within a block)
      bool ovf = false;
      uint8_t* kd = okeys + (uint64_t)q * keys_cap;
      uint8_t* vd = ovals + (uint64_t)q * vals_cap;
      for (;;) {
        if (Q.nrec >= Q.max_records) { Q.end = MTBLX_EMIT_MAX; break; }
        if (!(it.current < b.R)) break;                            // get() -> None
        if (it.voff + it.vlen > b.L) { Q.end = MTBLX_EMIT_PANIC; break; }   // get()'s slice
        const uint64_t kb = Q.key_bytes + it.klen, vb = Q.val_bytes + it.vlen;
        if (!ovf && (Q.nrec >= rec_cap || kb > keys_cap || vb > vals_cap)) ovf = true;
        if (!ovf) {
          for (uint64_t j = (uint64_t)lane; j < it.klen; j += 64) {
            MTBLX_CHK(kd + Q.key_bytes + j, 1);
            MTBLX_CHK(K + j, 1);
            kd[Q.key_bytes + j] = K[j];
          }
          uint64_t j0 = 0;
          if (DEFER) {
            j0 = it.vlen;   // the caller copies the value (vsrc)
            MTBLX_CHK(vsrc + (uint64_t)q * rec_cap + Q.nrec, 8);
            if (lane == 0) vsrc[(uint64_t)q * rec_cap + Q.nrec] = it.voff;
          } else if (it.vlen >= 4096) {   // big values (blocks >= 4 GiB hold values of GiBs): 16 B per lane
            typedef uint32_t v4u __attribute__((ext_vector_type(4), aligned(1)));
            const uint64_t nv = it.vlen / 16;
            const uint8_t* vs = d + it.voff;
            uint8_t* vo = vd + Q.val_bytes;
            // kU loads in flight per lane (one wave moves GiBs: latency-bound otherwise)
            constexpr uint32_t kU = 16;
            uint64_t c = (uint64_t)lane;
            for (; c + (kU - 1) * 64 < nv; c += kU * 64) {
              v4u x[kU];
#pragma unroll
              for (uint32_t u = 0; u < kU; ++u) {
                MTBLX_CHK(vs + 16 * (c + 64 * u), 16);
                x[u] = *reinterpret_cast<const v4u*>(vs + 16 * (c + 64 * u));
              }
#pragma unroll
              for (uint32_t u = 0; u < kU; ++u) {
                MTBLX_CHK(vo + 16 * (c + 64 * u), 16);
                *reinterpret_cast<v4u*>(vo + 16 * (c + 64 * u)) = x[u];
              }
            }
            for (; c < nv; c += 64) {
              MTBLX_CHK(vo + 16 * c, 16);
              MTBLX_CHK(vs + 16 * c, 16);
              *reinterpret_cast<v4u*>(vo + 16 * c) = *reinterpret_cast<const v4u*>(vs + 16 * c);
            }
            j0 = 16 * nv;
          }
          for (uint64_t j = j0 + (uint64_t)lane; j < it.vlen; j += 64) {
            MTBLX_CHK(vd + Q.val_bytes + j, 1);
            MTBLX_CHK(d + it.voff + j, 1);
            vd[Q.val_bytes + j] = d[it.voff + j];
          }
          MTBLX_CHK(oke + (uint64_t)q * rec_cap + Q.nrec, 8);
          MTBLX_CHK(ove + (uint64_t)q * rec_cap + Q.nrec, 8);
          if (okcap) MTBLX_CHK(okcap + (uint64_t)q * rec_cap + Q.nrec, 8);
          if (lane == 0) {
            oke[(uint64_t)q * rec_cap + Q.nrec] = kb;
            ove[(uint64_t)q * rec_cap + Q.nrec] = vb;
            if (okcap) okcap[(uint64_t)q * rec_cap + Q.nrec] = it.kcap;
          }
        }
        Q.nrec++;
        Q.key_bytes = kb;
        Q.val_bytes = vb;
        if (it.has_next && it.next == it.current) { Q.end = MTBLX_EMIT_LOOP; break; }
        r = s_parse(b, it, K, klim, lane);                         // BlockIter::next
        if (r == R_PANIC) { Q.end = MTBLX_EMIT_PANIC; break; }
        if (r == R_TOOLONG) { Q.status = MTBLX_SEEK_UNSUPPORTED; break; }
      }
      if (ovf && Q.status == MTBLX_SEEK_OK) Q.end = MTBLX_EMIT_OVERFLOW;
    } while (false);
    Q.kcap = it.kcap;
    Q.stop_off = it.current;
    Q.has_val = it.has_val ? 1 : 0;
    Q.last_voff = it.voff;
    Q.last_vlen = it.vlen;
    MTBLX_CHK(qs + q, sizeof(mtblx_block_seek));
    if (lane == 0) qs[q] = Q;
  }
}

// chain of entry offsets from restart 0 (seek_to_first + next), see mtblx_entry_offsets
__device__ __forceinline__ bool chain_step(const Blk& b, uint64_t cur, uint64_t& nxt, uint32_t& sh, uint32_t& ns) {
  uint32_t vl;
  uint64_t p;
  if (decode_entry(b, cur, b.R, sh, ns, vl, p) != R_OK) return false;
  if (p + ns > b.L) return false;
  nxt = p + ns + vl;
  return true;
}
__device__ __forceinline__ bool chain_step(const Blk& b, uint64_t cur, uint64_t& nxt) {
  uint32_t sh, ns;
  return chain_step(b, cur, nxt, sh, ns);
}

__global__ void __launch_bounds__(1024) k_entry_offsets(const uint8_t* blk, uint64_t L, uint64_t* offs, uint64_t cap,
                                                        uint64_t* count, uint64_t* scratch, uint32_t* regular_out) {
  __shared__ int irregular, keys_irregular;
  __shared__ uint64_t wsum[16];
  __shared__ uint64_t carry;
  Blk b{};
  const int tid = threadIdx.x;
  if (tid == 0) { irregular = 0; keys_irregular = 0; carry = 0; }
  __syncthreads();
  if (block_init(blk, L, b) != 0 || b.n == 0) {
    if (tid == 0) {
      *count = 0;
      if (regular_out) *regular_out = 0;
    }
    return;
  }
  const uint32_t n = b.n;
  // pass 1: count each restart interval's chain; it must land exactly on the next restart point.
  // Also: every restart entry has shared == 0 and every other entry shared <= the previous
  // key's length -- then a seek starting at any restart point rebuilds the scan's own keys and
  // the key-capacity assert (src/block.rs:132) can never fire (see mtblx.h)
  for (uint32_t r = tid; r < n; r += blockDim.x) {
    const uint64_t s0 = restart_point(b, r), e0 = (r + 1 < n) ? restart_point(b, r + 1) : b.R;
    uint64_t c = 0, cur = s0, klen = 0;
    bool ok = s0 < e0 || (r + 1 == n && s0 == b.R);
    bool kok = true;
    while (ok && cur < e0) {
      uint64_t nx;
      uint32_t sh, ns;
      // a zero-progress entry (unterminated varints, ns = vl = 0) makes the interval irregular:
      // the serial walk below stops on it (r05: this loop spun on it forever)
      if (!chain_step(b, cur, nx, sh, ns) || nx <= cur) { ok = false; break; }
      if (c == 0 ? sh != 0 : sh > klen) kok = false;
      klen = (sh < klen ? sh : klen) + ns;
      cur = nx;
      ++c;
    }
    if (!ok || cur != e0) irregular = 1;
    if (!kok) keys_irregular = 1;
    MTBLX_CHK(scratch + r, 8);
    scratch[r] = c;
  }
  __syncthreads();
  if (tid == 0 && regular_out) *regular_out = (irregular || keys_irregular) ? 0u : 1u;
  if (!irregular) {
    // exclusive scan of scratch[0..n) in chunks of blockDim.x
    for (uint32_t base = 0; base < n; base += blockDim.x) {
      const uint32_t r = base + tid;
      if (r < n) MTBLX_CHK(scratch + r, 8);
      const uint64_t v = r < n ? scratch[r] : 0;
      uint64_t x = v;
      for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if ((tid & 63) >= o) x += y;
      }
      if ((tid & 63) == 63) wsum[tid >> 6] = x;
      __syncthreads();
      uint64_t wp = 0;
      for (int w = 0; w < (tid >> 6); ++w) wp += wsum[w];
      const uint64_t c0 = carry;
      __syncthreads();
      if (r < n) scratch[r] = c0 + wp + x - v;
      if (tid == (int)blockDim.x - 1) carry = c0 + wp + x;
      __syncthreads();
    }
    for (uint32_t r = tid; r < n; r += blockDim.x) {
      const uint64_t e0 = (r + 1 < n) ? restart_point(b, r + 1) : b.R;
      uint64_t i = scratch[r], cur = restart_point(b, r);
      while (cur < e0) {
        if (i < cap) { MTBLX_CHK(offs + i, 8); offs[i] = cur; }
        uint64_t nx;
        chain_step(b, cur, nx);
        cur = nx;
        ++i;
      }
    }
    if (tid == 0) *count = carry;
    return;
  }
  // irregular block (corruption): the scan's own walk, serial
  if (tid != 0) return;
  uint64_t i = 0, cur = restart_point(b, 0);
  while (cur < b.R) {
    if (i < cap) { MTBLX_CHK(offs + i, 8); offs[i] = cur; }
    ++i;
    uint64_t nx;
    if (!chain_step(b, cur, nx) || nx <= cur) break;
    cur = nx;
  }
  *count = i;
}

__global__ void k_key_filter(const uint8_t* keys, const uint64_t* key_end, uint64_t n, int32_t type, const uint8_t* k,
                             uint64_t kl, unsigned long long* first_fail) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  MTBLX_CHK(key_end + i, 8);
  const uint64_t a = i ? key_end[i - 1] : 0, l = key_end[i] - a;
  const uint8_t* key = keys + a;
  const uint64_t m = l < kl ? l : kl;
  uint64_t c = 0;
  while (c < m && (MTBLX_CHK(key + c, 1), MTBLX_CHK(k + c, 1), key[c] == k[c])) ++c;
  const int cmp = (c < m) ? (key[c] < k[c] ? -1 : 1) : (l < kl ? -1 : (l > kl ? 1 : 0));
  bool fail = false;
  if (type == 1) fail = cmp != 0;
  else if (type == 2) fail = !(kl <= l && c == kl);
  else if (type == 3) fail = cmp > 0;
  if (fail) { MTBLX_CHK(first_fail, 8); atomicMin(first_fail, (unsigned long long)i); }
}

}  // namespace mtblx_rd

extern "C" int mtblx_block_dir(const uint8_t* file, uint64_t file_len, uint32_t version, const uint8_t* vals,
                               const uint32_t* val_end, uint64_t val_base, uint32_t nent, uint64_t* blk_off,
                               uint32_t* blk_len, int32_t* dir_st, void* stream) {
  if (nent == 0) return MTBLX_OK;
  if (!file || !vals || !val_end || !blk_off || !blk_len || !dir_st || version > 1) return MTBLX_E_INVAL;
  const uint32_t threads = 256;
  MTBLX_LAUNCH((MTBLX_R(file, file_len), vals, MTBLX_R(val_end, 4ull * nent), MTBLX_R(blk_off, 8ull * nent),
                MTBLX_R(blk_len, 4ull * nent), MTBLX_R(dir_st, 4ull * nent)),
               mtblx_rd::k_block_dir,
               dim3((nent + threads - 1) / threads), dim3(threads), 0, reinterpret_cast<hipStream_t>(stream), file, file_len, version, vals, val_end, val_base, nent,
                     blk_off, blk_len, dir_st);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

// k_get_lanes (one lane per query) unless MTBLX_GET_KERNEL=wave (k_get, one wave per query: A/B)
static void get_launch(const uint8_t* file, uint64_t file_len, uint32_t version, int verify, uint64_t index_off,
                       uint64_t index_len, mtblx_rd::DecTab tab, const uint8_t* keys, const uint64_t* key_end,
                       uint32_t nq, int32_t* status, uint64_t* val_off, uint64_t* val_len, hipStream_t s) {
  const int grid = mtblx_dev::cu_count() * 8;
  const char* ge = getenv("MTBLX_GET_KERNEL");   // A/B knob, read per call
  const int wave = ge && ge[0] == 'w' ? 1 : 0;
  const uint64_t per = wave ? 4u : 256u;   // queries per workgroup per pass
  const uint64_t need = (nq + per - 1) / per;
  const dim3 g((unsigned)(need < (uint64_t)grid ? need : (uint64_t)grid));
  const uint64_t ntab = tab.dec ? tab.n : 0;
  if (wave) {
    MTBLX_LAUNCH((MTBLX_R(file, file_len), MTBLX_R(tab.start, 8ull * ntab), MTBLX_R(tab.doff, 8ull * ntab),
                  MTBLX_R(tab.dlen, 8ull * ntab), MTBLX_R(tab.st, 4ull * ntab), tab.dec, keys, MTBLX_R(key_end, 8ull * nq),
                  MTBLX_R(status, 4ull * nq), MTBLX_R(val_off, 8ull * nq), MTBLX_R(val_len, 8ull * nq)),
                 mtblx_rd::k_get, g, dim3(256), 0, s, file, file_len, version, verify, index_off, index_len, tab, keys,
                 key_end, nq, status, val_off, val_len);
  } else {
    MTBLX_LAUNCH((MTBLX_R(file, file_len), MTBLX_R(tab.start, 8ull * ntab), MTBLX_R(tab.doff, 8ull * ntab),
                  MTBLX_R(tab.dlen, 8ull * ntab), MTBLX_R(tab.st, 4ull * ntab), tab.dec, keys, MTBLX_R(key_end, 8ull * nq),
                  MTBLX_R(status, 4ull * nq), MTBLX_R(val_off, 8ull * nq), MTBLX_R(val_len, 8ull * nq)),
                 mtblx_rd::k_get_lanes, g, dim3(256), 0, s, file, file_len, version, verify, index_off, index_len, tab,
                 keys, key_end, nq, status, val_off, val_len);
  }
}

extern "C" int mtblx_get(const uint8_t* file, uint64_t file_len, uint32_t version, int verify, uint64_t index_off,
                         uint64_t index_len, const uint8_t* keys, const uint64_t* key_end, uint32_t nq, int32_t* status,
                         uint64_t* val_off, uint64_t* val_len, void* stream) {
  if (nq == 0) return MTBLX_OK;
  if (!file || !keys || !key_end || !status || !val_off || !val_len || version > 1) return MTBLX_E_INVAL;
  get_launch(file, file_len, version, verify, index_off, index_len,
             mtblx_rd::DecTab{nullptr, nullptr, nullptr, nullptr, 0u, nullptr}, keys, key_end, nq, status, val_off,
             val_len, reinterpret_cast<hipStream_t>(stream));
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
extern "C" int mtblx_get_decompressed(const uint8_t* file, uint64_t file_len, uint32_t version, int verify,
                                      uint64_t index_off, uint64_t index_len, const uint64_t* tab_start,
                                      const uint64_t* tab_doff, const uint64_t* tab_dlen, const int32_t* tab_st,
                                      uint32_t ntab, const uint8_t* dec, const uint8_t* keys, const uint64_t* key_end,
                                      uint32_t nq, int32_t* status, uint64_t* val_off, uint64_t* val_len,
                                      void* stream) {
  if (nq == 0) return MTBLX_OK;
  if (!file || !keys || !key_end || !status || !val_off || !val_len || version > 1 || !dec) return MTBLX_E_INVAL;
  if (ntab && (!tab_start || !tab_doff || !tab_dlen || !tab_st)) return MTBLX_E_INVAL;
  get_launch(file, file_len, version, verify, index_off, index_len,
             mtblx_rd::DecTab{tab_start, tab_doff, tab_dlen, tab_st, ntab, dec}, keys, key_end, nq, status, val_off,
             val_len, reinterpret_cast<hipStream_t>(stream));
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

extern "C" int mtblx_index_seek_batch(const uint8_t* file, uint64_t file_len, uint32_t version, int verify,
                                      uint64_t index_off, uint64_t index_len, const uint8_t* keys,
                                      const uint64_t* key_end, uint32_t nq, mtblx_index_seek* out, void* stream) {
  if (nq == 0) return MTBLX_OK;
  if (!file || !keys || !key_end || !out || version > 1) return MTBLX_E_INVAL;
  const uint32_t need = (nq + 3u) / 4u;
  MTBLX_LAUNCH((MTBLX_R(file, file_len), keys, MTBLX_R(key_end, 8ull * nq), MTBLX_R(out, sizeof(*out) * nq)),
               mtblx_rd::k_index_seek, dim3(need < 2048u ? need : 2048u), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), file, file_len, version, verify, index_off, index_len,
                     keys, key_end, nq, out);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

extern "C" int mtblx_block_seek_batch(const uint8_t* data, const uint8_t* keys, const uint64_t* key_end, uint32_t nq,
                                      mtblx_block_seek* q, uint8_t* out_keys, uint64_t keys_cap, uint8_t* out_vals,
                                      uint64_t vals_cap, uint64_t* key_end_out, uint64_t* val_end_out,
                                      uint64_t* kcap_out, uint64_t rec_cap, void* stream) {
  if (nq == 0) return MTBLX_OK;
  if (!data || !keys || !key_end || !q || !out_keys || !out_vals || !key_end_out || !val_end_out) return MTBLX_E_INVAL;
  MTBLX_LAUNCH((data, keys, MTBLX_R(key_end, 8ull * nq), MTBLX_R(q, sizeof(*q) * nq), MTBLX_R(out_keys, keys_cap * nq),
                MTBLX_R(out_vals, vals_cap * nq), MTBLX_R(key_end_out, 8 * rec_cap * nq),
                MTBLX_R(val_end_out, 8 * rec_cap * nq), MTBLX_R(kcap_out, 8 * rec_cap * nq)),
               mtblx_rd::k_block_seek<false>, dim3(nq < 1024u ? nq : 1024u), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), data, keys, key_end, nq, q, out_keys, keys_cap, out_vals,
                     vals_cap, key_end_out, val_end_out, kcap_out, rec_cap, nullptr, 0);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

extern "C" int mtblx_block_seek_batch_kbuf(const uint8_t* data, const uint8_t* keys, const uint64_t* key_end,
                                           uint32_t nq, mtblx_block_seek* q, uint8_t* out_keys, uint64_t keys_cap,
                                           uint8_t* out_vals, uint64_t vals_cap, uint64_t* key_end_out,
                                           uint64_t* val_end_out, uint64_t* kcap_out, uint64_t rec_cap,
                                           uint8_t* key_buf, uint64_t key_buf_cap, void* stream) {
  if (nq == 0) return MTBLX_OK;
  if (!data || !keys || !key_end || !q || !out_keys || !out_vals || !key_end_out || !val_end_out || !key_buf ||
      key_buf_cap == 0)
    return MTBLX_E_INVAL;
  MTBLX_LAUNCH((data, keys, MTBLX_R(key_end, 8ull * nq), MTBLX_R(q, sizeof(*q) * nq), MTBLX_R(out_keys, keys_cap * nq),
                MTBLX_R(out_vals, vals_cap * nq), MTBLX_R(key_end_out, 8 * rec_cap * nq),
                MTBLX_R(val_end_out, 8 * rec_cap * nq), MTBLX_R(kcap_out, 8 * rec_cap * nq),
                MTBLX_R(key_buf, key_buf_cap * nq)),
               mtblx_rd::k_block_seek<true>, dim3(nq < 1024u ? nq : 1024u), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), data, keys, key_end, nq, q, out_keys, keys_cap, out_vals,
                     vals_cap, key_end_out, val_end_out, kcap_out, rec_cap, key_buf, key_buf_cap);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

extern "C" int mtblx_block_seek_batch_ex(const uint8_t* data, const uint8_t* keys, const uint64_t* key_end,
                                         uint32_t nq, mtblx_block_seek* q, uint8_t* out_keys, uint64_t keys_cap,
                                         uint8_t* out_vals, uint64_t vals_cap, uint64_t* key_end_out,
                                         uint64_t* val_end_out, uint64_t* kcap_out, uint64_t rec_cap, uint8_t* key_buf,
                                         uint64_t key_buf_cap, uint64_t* val_src_out, void* stream) {
  if (nq == 0) return MTBLX_OK;
  if (!data || !keys || !key_end || !q || !out_keys || !key_end_out || !val_end_out || !val_src_out ||
      (key_buf && key_buf_cap == 0))
    return MTBLX_E_INVAL;
  const dim3 g(nq < 1024u ? nq : 1024u);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (key_buf)
    MTBLX_LAUNCH((data, keys, MTBLX_R(key_end, 8ull * nq), MTBLX_R(q, sizeof(*q) * nq), MTBLX_R(out_keys, keys_cap * nq),
                  MTBLX_R(key_end_out, 8 * rec_cap * nq), MTBLX_R(val_end_out, 8 * rec_cap * nq),
                  MTBLX_R(kcap_out, 8 * rec_cap * nq), MTBLX_R(key_buf, key_buf_cap * nq),
                  MTBLX_R(val_src_out, 8 * rec_cap * nq)),
                 (mtblx_rd::k_block_seek<true, true>), g, dim3(64), 0, s, data, keys, key_end, nq, q, out_keys,
                 keys_cap, out_vals, vals_cap, key_end_out, val_end_out, kcap_out, rec_cap, key_buf, key_buf_cap,
                 val_src_out);
  else
    MTBLX_LAUNCH((data, keys, MTBLX_R(key_end, 8ull * nq), MTBLX_R(q, sizeof(*q) * nq), MTBLX_R(out_keys, keys_cap * nq),
                  MTBLX_R(key_end_out, 8 * rec_cap * nq), MTBLX_R(val_end_out, 8 * rec_cap * nq),
                  MTBLX_R(kcap_out, 8 * rec_cap * nq), MTBLX_R(val_src_out, 8 * rec_cap * nq)),
                 (mtblx_rd::k_block_seek<false, true>), g, dim3(64), 0, s, data, keys, key_end, nq, q, out_keys,
                 keys_cap, out_vals, vals_cap, key_end_out, val_end_out, kcap_out, rec_cap, nullptr, 0, val_src_out);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

extern "C" int mtblx_entry_offsets(const uint8_t* block, uint64_t len, uint64_t* offs, uint64_t cap, uint64_t* count,
                                   uint32_t* regular, void* stream) {
  if (!block || !count || (cap && !offs)) return MTBLX_E_INVAL;
  if (len > mtblx_rd::kU32) return MTBLX_E_INVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint64_t nr = len / 4 + 1;   // restart count bound: 4 bytes per restart point
  // the per-interval counts: a plain allocation freed once the launch has completed (once per
  // Reader; r05: no stream-ordered pool allocations next to the caller's caching allocator)
  uint64_t* scratch = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&scratch), nr * sizeof(uint64_t)) != hipSuccess) return MTBLX_E_HIP;
  // test knob (MTBLX_DEBUG_POISON, tests/conftest.py): fresh scratch filled with 0xFF, so a read
  // before a write is deterministic and far out of range
  if (getenv("MTBLX_DEBUG_POISON") && hipMemsetAsync(scratch, 0xFF, nr * sizeof(uint64_t), s) != hipSuccess) {
    (void)hipFree(scratch);
    return MTBLX_E_HIP;
  }
  MTBLX_LAUNCH((MTBLX_R(block, len), MTBLX_R(offs, 8 * cap), MTBLX_R(count, 8), MTBLX_R(scratch, 8 * nr),
                MTBLX_R(regular, 4)), mtblx_rd::k_entry_offsets, dim3(1), dim3(1024), 0, s, block, len, offs, cap, count, scratch,
                     regular);
  const bool ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
  (void)hipFree(scratch);
  return ok ? MTBLX_OK : MTBLX_E_HIP;
}

extern "C" int mtblx_key_filter(const uint8_t* keys, const uint64_t* key_end, uint64_t n, int32_t type,
                                const uint8_t* k, uint64_t klen, uint64_t* first_fail, void* stream) {
  if (n == 0) return MTBLX_OK;
  if (!keys || !key_end || !first_fail || (klen && !k) || type < 1 || type > 3) return MTBLX_E_INVAL;
  const uint64_t blocks = (n + 255) / 256;
  if (blocks > 0x7FFFFFFFull) return MTBLX_E_INVAL;
  MTBLX_LAUNCH((keys, MTBLX_R(key_end, 8 * n), MTBLX_R(k, klen), MTBLX_R(first_fail, 8)), mtblx_rd::k_key_filter, dim3((uint32_t)blocks), dim3(256), 0,
               reinterpret_cast<hipStream_t>(stream),
                     keys, key_end, n, type, k, klen, reinterpret_cast<unsigned long long*>(first_fail));
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
