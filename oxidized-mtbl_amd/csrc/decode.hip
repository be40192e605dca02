// decode.hip — MI355X (gfx950) kernel for mtbl data-block decode.
//
// Replaces the reference's per-record CPU scan of one block
//   Block::init            /root/reference/src/block.rs:16-49
//   BlockIter::init        src/block.rs:75-93
//   seek_to_first / next / get / parse_next_key / decode_entry   src/block.rs:119-238
//   varint_decode32        src/varint.rs:44-61
// with ONE single-pass launch over a batch of blocks, output laid out contiguously
// (include/mtblx.h).  See k_decode_tiles below and DESIGN.md "Kernels".
//
// Everything is integer/byte work: HBM-bandwidth bound (the fused verify's CRC is VALU slicing
// here; the separate-launch CRC, crc.hip, runs it on the matrix cores).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>

#include <algorithm>

#include "bounds.h"
#include "devinfo.h"
#include "crc_dev.h"
#include "crc_mfma.h"
#include "crc_mfma_dev.h"
#include "mtblx.h"

// Ablations (outputs incomplete by construction) and the spilling variant build only through the
// Makefile's diagnostic targets, which define MTBLX_DIAG; the product build rejects them.
#if (defined(MTBLX_ABL_NOKEY) || defined(MTBLX_ABL_NOVAL) || defined(MTBLX_ABL_NOVSTORE) || \
     defined(MTBLX_ABL_CRC) || defined(MTBLX_SPILL) || defined(MTBLX_CALL_PROBE)) && !defined(MTBLX_DIAG)
#error "ablation / spill knobs are diagnostic: build them through a Makefile diagnostic target (-DMTBLX_DIAG)"
#endif

namespace mtblx {

constexpr int kWave = 64;
constexpr uint64_t kU32Max = 0xFFFFFFFFull;
// block stage offsets: not staged in LDS (read from HBM)
constexpr uint32_t kNotStaged = 0xFFFFFFFFu;
// stage offset of a block whose window [blk_off, blk_off + blk_len) runs past data_len: the
// reference's slice of it panics (BytesView::slice, src/lib.rs:93-99) -> MTBLX_ST_CORRUPT, and
// nothing reads it
constexpr uint32_t kOutOfBounds = 0xFFFFFFFEu;

// ----------------------------------------------------------------------------------
// small helpers
// ----------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t byte_of(const uint4& w, uint32_t t) {
  uint32_t d = (t < 4) ? w.x : (t < 8) ? w.y : (t < 12) ? w.z : w.w;
  return (d >> (8 * (t & 3))) & 0xffu;
}

// LDS reads at arbitrary byte offsets.  gfx950 runs LDS in unaligned access mode, but a
// misaligned ds_read_b32 / ds_read_b128 issues at a fraction of the aligned rate (measured with
// scripts/lds_probe.hip: ~10x and ~7.5x less throughput; a ds_read_b128 needs 16-byte
// alignment for full rate), so both helpers read aligned dwords and join them with a funnel
// shift: +4% on PipeSmall and PipeLarge against one misaligned ds_read_b128 / ds_read_b32.
// `lds` is the 16-byte aligned base of a stage buffer; up to 4 bytes past the window are read.
__device__ __forceinline__ uint4 lds_win16(const uint8_t* lds, uint32_t a) {   // bytes [a, a + 16)
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds) + (a >> 2);
  MTBLX_LCHK(w, 20);
  const uint32_t sh = (a & 3u) * 8u;
  const uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3], x4 = w[4];
  return make_uint4(__builtin_amdgcn_alignbit(x1, x0, sh), __builtin_amdgcn_alignbit(x2, x1, sh),
                    __builtin_amdgcn_alignbit(x3, x2, sh), __builtin_amdgcn_alignbit(x4, x3, sh));
}

__device__ __forceinline__ uint32_t lds_rd32(const uint8_t* lds, uint32_t a) {   // bytes [a, a + 4)
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds) + (a >> 2);
  MTBLX_LCHK(w, 8);
  return __builtin_amdgcn_alignbit(w[1], w[0], (a & 3u) * 8u);
}

// byte mask selecting bytes [lo, hi) of a dword whose first byte is byte `base`
__device__ __forceinline__ uint32_t dmask(int lo, int hi, int base) {
  int l = lo - base, h = hi - base;
  l = l < 0 ? 0 : (l > 4 ? 4 : l);
  h = h < 0 ? 0 : (h > 4 ? 4 : h);
  if (h <= l) return 0u;
  uint64_t m = ((1ull << (8 * h)) - 1ull) ^ ((1ull << (8 * l)) - 1ull);
  return (uint32_t)m;
}

__device__ __forceinline__ void merge_bytes(uint4& out, const uint4& w, int lo, int hi) {
  uint32_t m;
  m = dmask(lo, hi, 0);  out.x = (out.x & ~m) | (w.x & m);
  m = dmask(lo, hi, 4);  out.y = (out.y & ~m) | (w.y & m);
  m = dmask(lo, hi, 8);  out.z = (out.z & ~m) | (w.z & m);
  m = dmask(lo, hi, 12); out.w = (out.w & ~m) | (w.w & m);
}

// Unaligned global stores (gfx950 runs with unaligned memory access enabled).
typedef uint32_t v4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t v2u __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint16_t __attribute__((aligned(1))) u16u;

// Output stores.  The decoded keys / values / ends are written once and never read back by
// this launch: non-temporal stores (MTBLX_NT_STORES) stream them out instead of leaving the
// XCD L2s full of dirty lines that the end-of-launch release must write back.
#ifndef MTBLX_NT_STORES
#define MTBLX_NT_STORES 2
#endif
// LDS-DMA of the block bytes with the non-temporal policy (aux = 2): the blocks are read once, so
// they stay out of the L2s the byte-granular key stores merge in (cfg2 +5 %, 64 KiB +4 %)
#ifndef MTBLX_DMA_AUX   // cache-policy bits of the LDS-DMA loads (2 = non-temporal)
#define MTBLX_DMA_AUX 2
#endif
#ifndef MTBLX_NT_LOADS
#define MTBLX_NT_LOADS 1
#endif
#ifndef MTBLX_WSEND_LIGHT
#define MTBLX_WSEND_LIGHT 1
#endif
#if MTBLX_NT_STORES
#define ost(p, ...) (MTBLX_CHK((p), sizeof(*(p))), __builtin_nontemporal_store((__VA_ARGS__), (p)))
#else
#define ost(p, ...) (MTBLX_CHK((p), sizeof(*(p))), (void)(*(p) = (__VA_ARGS__)))
#endif
// byte-granular stores (keys of any length, value tails): MTBLX_NT_STORES == 1 streams them
// too; == 2 keeps them in L2, where partial lines merge before they are written back
#if MTBLX_NT_STORES == 1
#define ostb(p, ...) __builtin_nontemporal_store((__VA_ARGS__), (p))
#else
#define ostb(p, ...) (void)(*(p) = (__VA_ARGS__))
#endif

// store the first m (0..16) bytes of w at p
__device__ __forceinline__ void store_bytes(uint8_t* p, uint4 w, uint32_t m) {
  MTBLX_CHK(p, m);
  if (m == 16) { ostb(reinterpret_cast<v4u*>(p), v4u{w.x, w.y, w.z, w.w}); return; }
  if (m & 8) { ostb(reinterpret_cast<v2u*>(p), v2u{w.x, w.y}); w = make_uint4(w.z, w.w, 0, 0); p += 8; }
  if (m & 4) { ostb(reinterpret_cast<u32u*>(p), w.x); w.x = w.y; p += 4; }
  if (m & 2) { ostb(reinterpret_cast<u16u*>(p), (uint16_t)w.x); w.x >>= 16; p += 2; }
  if (m & 1) { ostb(p, (uint8_t)w.x); }
}

// Inclusive scan over the 64 lanes with DPP (row_shr 1/2/4/8 inside each 16-lane row,
// then row_bcast:15 / row_bcast:31 across rows): 6 VALU ops, no LDS permutes.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int /*lane*/ = 0) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// sum over the 64 lanes, broadcast (uniform)
__device__ __forceinline__ uint32_t wave_sum32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(x), 63);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// varint_decode32 (src/varint.rs:44-61) over a register window; k = first byte,
// avail = bytes to the end of the block (>= 1).  Returns len (0 = unterminated).
__device__ __forceinline__ uint32_t dec32(const uint4& W, uint32_t k, uint32_t avail, uint32_t& val) {
  uint32_t win = avail < 5u ? avail : 5u;
  uint32_t len = 0;
  for (uint32_t t = 0; t < win; ++t) {
    if (!(byte_of(W, k + t) & 0x80u)) { len = t + 1; break; }
  }
  uint32_t v = byte_of(W, k) & 0x7fu;
  if (len > 1) v |= (byte_of(W, k + 1) & 0x7fu) << 7;
  if (len > 2) v |= (byte_of(W, k + 2) & 0x7fu) << 14;
  if (len > 3) v |= (byte_of(W, k + 3) & 0x7fu) << 21;
  if (len > 4) v |= byte_of(W, k + 4) << 28;  // unmasked (src/varint.rs:54)
  val = v;
  return len;
}

// ----------------------------------------------------------------------------------
// generic path: exact serial emulation of the reference on one block, lane 0 only,
// reading HBM directly.  Handles every quirk (DESIGN.md "Reference quirks").
// ----------------------------------------------------------------------------------
struct GenOut {
  uint32_t nrec;
  uint64_t kb, vb;
  int32_t st;
};

__device__ __forceinline__ uint32_t grd32(const uint8_t* p) {
  MTBLX_CHK(p, 4);
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// varint_decode32 on global bytes d[0..avail), avail >= 1
__device__ uint32_t gdec32(const uint8_t* d, uint64_t avail, uint32_t& val) {
  uint32_t win = avail < 5 ? (uint32_t)avail : 5u;
  MTBLX_CHK(d, win);
  uint32_t len = 0;
  for (uint32_t t = 0; t < win; ++t) {
    if (!(d[t] & 0x80u)) { len = t + 1; break; }
  }
  uint32_t v = d[0] & 0x7fu;
  if (len > 1) v |= (uint32_t)(d[1] & 0x7fu) << 7;
  if (len > 2) v |= (uint32_t)(d[2] & 0x7fu) << 14;
  if (len > 3) v |= (uint32_t)(d[3] & 0x7fu) << 21;
  if (len > 4) v |= (uint32_t)d[4] << 28;
  val = v;
  return len;
}

template <bool WRITE>
__device__ GenOut generic_block(const uint8_t* d, uint64_t L, uint8_t* keys, uint8_t* vals, uint32_t* key_end,
                                uint32_t* val_end) {
  GenOut o{0, 0, 0, MTBLX_ST_OK};
  // Block::init (src/block.rs:16-49), release-mode wrapping arithmetic
  if (L < 4) { o.st = MTBLX_ST_INVALID_BLOCK; return o; }
  if (L < 8) { o.st = MTBLX_ST_CORRUPT; return o; }
  uint32_t n = grd32(d + L - 4);
  uint64_t ro = L - (1ull + n) * 4ull;
  if (ro > kU32Max) {
    ro = L - (4ull + (uint64_t)n * 8ull);
    if (ro <= kU32Max) { o.st = MTBLX_ST_INVALID_BLOCK; return o; }
  }
  if (ro > L - 4) { o.st = MTBLX_ST_INVALID_BLOCK; return o; }
  if (ro > kU32Max) { o.st = MTBLX_ST_UNSUPPORTED; return o; }   // unreachable for u32 lengths
  if (n == 0) { o.st = MTBLX_ST_CORRUPT; return o; }              // BlockIter::init assert (:79)
  const uint64_t R = ro;
  uint64_t next = grd32(d + R);                                  // seek_to_first -> restart_point(0)
  uint64_t klen = 0, kcap = 0, kprev = 0;
  for (;;) {
    const uint64_t cur = next;
    if (cur >= R) break;                                         // parse_next_key -> invalid
    // decode_entry (:216-238)
    uint64_t p = cur;
    if (R - p < 3) { o.st = MTBLX_ST_CORRUPT; break; }
    MTBLX_CHK(d + p, 3);
    uint32_t sh = d[p], ns = d[p + 1], vl = d[p + 2];
    if ((sh | ns | vl) < 128u) {
      p += 3;
    } else {
      uint32_t k;
      k = gdec32(d + p, L - p, sh); p += k;
      if (p >= L) { o.st = MTBLX_ST_CORRUPT; break; }
      k = gdec32(d + p, L - p, ns); p += k;
      if (p >= L) { o.st = MTBLX_ST_CORRUPT; break; }
      k = gdec32(d + p, L - p, vl); p += k;
      if (p > R) { o.st = MTBLX_ST_CORRUPT; break; }
    }
    if ((uint64_t)ns + vl > kU32Max || (uint64_t)ns + vl > R - p) { o.st = MTBLX_ST_CORRUPT; break; }
    if (kcap < sh) { o.st = MTBLX_ST_CORRUPT; break; }           // assert capacity (:132)
    uint64_t m = sh < klen ? sh : klen;                          // truncate (:134)
    if (ns > 0 && kcap - m < ns) {                               // Vec growth (:135)
      uint64_t c = kcap * 2, req = m + ns;
      if (req > c) c = req;
      if (c < 8) c = 8;
      kcap = c;
    }
    const uint64_t newlen = m + ns;
    if (WRITE) {
      uint8_t* kd = keys + o.kb;
      const uint8_t* ks = keys + kprev;
      if (m) { MTBLX_CHK(ks, m); }
      if (newlen) { MTBLX_CHK(kd, newlen); }
      if (ns) { MTBLX_CHK(d + p, ns); }
      if (vl) { MTBLX_CHK(d + p + ns, vl); MTBLX_CHK(vals + o.vb, vl); }
      MTBLX_CHK(key_end + o.nrec, 4);
      MTBLX_CHK(val_end + o.nrec, 4);
      for (uint64_t i = 0; i < m; ++i) kd[i] = ks[i];
      for (uint64_t i = 0; i < ns; ++i) kd[m + i] = d[p + i];
      uint8_t* vd = vals + o.vb;
      for (uint64_t i = 0; i < vl; ++i) vd[i] = d[p + ns + i];
      key_end[o.nrec] = (uint32_t)(o.kb + newlen);
      val_end[o.nrec] = (uint32_t)(o.vb + vl);
    }
    kprev = o.kb;
    o.kb += newlen;
    o.vb += vl;
    o.nrec += 1;
    klen = newlen;
    next = p + ns + vl;
    if (next == cur) { o.st = MTBLX_ST_LOOP; break; }            // never terminates in the reference
  }
  // key / value END offsets are u32 relative to the block (include/mtblx.h): a block whose
  // rebuilt keys or values reach 4 GiB (shared prefixes re-expanded, e.g. a crafted 256 KiB
  // block) is not representable -> UNSUPPORTED, nothing written (the caller decodes it on the host)
  if (!WRITE && (o.kb > kU32Max || o.vb > kU32Max)) o = GenOut{0, 0, 0, MTBLX_ST_UNSUPPORTED};
  return o;
}

// blocks of a tile the exact path must not write: outside the data buffer, or UNSUPPORTED
__device__ __forceinline__ bool gen_writable(uint32_t bo, int32_t st) {
  return bo != kOutOfBounds && st != MTBLX_ST_UNSUPPORTED;
}

// ----------------------------------------------------------------------------------
// single-pass tiled decoder
// ----------------------------------------------------------------------------------
// A tile = up to `bpt` consecutive blocks of the batch, staged together in the LDS of
// one workgroup (256 threads).  Workgroups are persistent and take tiles t = blockIdx.x,
// + G, + 2G ... (G = gridDim.x, never more than the resident capacity).
// Per tile:
//   stage (from registers prefetched during the previous tile) -> prefetch the next tile
//   -> trailers -> walk 1 (one thread per restart interval across the tile, counts)
//   -> interval scan -> publish the tile aggregate -> issue the look-back loads
//   -> walk 2 (per-record metadata into LDS, hides the look-back latency)
//   -> finish the look-back -> per-block outputs -> copy (one thread per record)
//   -> irregular blocks (exact serial emulation).
//
// Look-back ("rolling"): prefix(t) = incl(t - G) + sum of the aggregates of tiles
// t-G+1 .. t-1.  incl(t - G) is this workgroup's own previous tile, so only the
// aggregates of the other G-1 tiles of the trailing window are read: one packed 8-byte
// agent-scope atomic per tile (the value IS the flag; no fences), <= 4 loads per thread,
// issued before walk 2 and consumed after it.

constexpr int kThreads = 256;
constexpr int kMaxLookbackLoads = 4;               // G - 1 <= 4 * 256
constexpr uint64_t kReady = 1ull << 63;
constexpr uint32_t kField = (1u << 21) - 1;        // 21-bit fields: nrec | vbytes | kbytes
constexpr int kPrefetch = 8;                       // uint4 per thread prefetched (32 KiB tiles)

template <int TB_, int MAXREC_, int MAXINT_, int MAXBLK_, bool PREFETCH_, int MINW_>
struct TileCfg {
  static constexpr int MINW = MINW_;     // workgroups per CU to keep resident (__launch_bounds__)
  static constexpr int TB = TB_;          // staging bytes
  static constexpr int MAXREC = MAXREC_;  // records with metadata per chunk
  static constexpr int MAXINT = MAXINT_;  // restart intervals per tile (<= kThreads)
  static constexpr int MAXBLK = MAXBLK_;  // blocks per tile (<= 64)
  static constexpr bool PREFETCH = PREFETCH_;
};

// per-record metadata, 16 bytes: one ds_write_b128 / ds_read_b128
struct Rec {
  uint32_t pos_sh;   // pos (block offset of the key suffix) | shared << 16
  uint32_t ns_vl;    // non_shared | value_length << 16
  uint32_t ks;       // tile-relative key start
  uint32_t vs_blk;   // tile-relative value start (< 2^24: bounded by the staging bytes) | block << 24
};

template <class C>
struct alignas(16) TileLds {
  uint8_t stage[C::TB];
  Rec rec[C::MAXREC];
  // per block of the tile
  uint32_t boff[C::MAXBLK];   // stage offset of block byte 0 (kNotStaged if not staged)
  uint32_t blen[C::MAXBLK];
  uint32_t bR[C::MAXBLK];     // restart offset
  uint32_t bn[C::MAXBLK];     // restart count (0 = irregular)
  uint32_t bint0[C::MAXBLK + 1];
  uint32_t bok[C::MAXBLK];    // 1 = regular fast path
  uint32_t bwr[C::MAXBLK];    // 1 = outputs of this block are written
  int32_t bst[C::MAXBLK];
  uint32_t bcnt[C::MAXBLK], bkb[C::MAXBLK], bvb[C::MAXBLK];   // block totals
  uint32_t brb[C::MAXBLK], bkbb[C::MAXBLK], bvbb[C::MAXBLK];  // tile-relative block bases
  uint32_t brf[C::MAXBLK];    // first metadata slot (regular records before the block)
  // per restart interval: counts after walk 1, exclusive bases after the scan
  uint32_t icnt[C::MAXINT + 1], ikb[C::MAXINT + 1], ivb[C::MAXINT + 1];
  uint8_t iblk[C::MAXINT];
  // tile scalars
  uint64_t tpre[3];           // global exclusive prefix of the tile (records, key bytes, value bytes)
  uint64_t tinc[3];           // inclusive prefix of this workgroup's previous tile
  uint32_t ttot[3];
  uint32_t nfastrec;
  uint32_t contig;            // 1 = tile staged as one contiguous byte range
  uint32_t wsum[4][3];
  uint64_t lbsum[4][3];
};

struct TileArgs {
  const uint8_t* data;
  uint64_t data_len;
  const uint64_t* blk_off;
  const uint32_t* blk_len;
  uint32_t nblk;
  uint32_t bpt;     // blocks per tile
  uint32_t slot;    // per-block staging slot bytes (fallback layout)
  uint32_t ntiles;
  uint32_t* nrec;
  uint64_t* rec_base;
  uint64_t* key_base;
  uint64_t* val_base;
  int32_t* status;
  uint32_t* key_end;
  uint32_t* val_end;
  uint64_t rec_cap;
  uint8_t* keys;
  uint64_t keys_cap;
  uint8_t* vals;
  uint64_t vals_cap;
  uint64_t* totals;
  uint64_t* lbw;    // workspace tile entries: kTileWords u64 per tile (lb_slot / lbx_slot)
  struct WsHdr* hdr;
  uint64_t* dbg;    // [16] phase stamps (diagnostic build only)
  int write;
  uint32_t* crc;     // VERIFY kernels: crc32c of every block's content (may be NULL)
  uint8_t* crc_bad;  // VERIFY kernels: 1 where the stored checksum differs (may be NULL)
  int crc_framed;    // the u32 before each content is its stored checksum (an mtbl file)
  // set at kernel start from the workspace header (ws_begin)
  uint32_t wscap;   // tile entries the workspace holds (from workspace_bytes)
  uint32_t par;     // launch parity: aggregates live in slot `par` of each tile entry
  uint32_t hw_other;
  unsigned long long inject;   // debug: bits ORed into totals[3] (MTBLX_DEBUG_FLAGS, mtblx_impl_run)
  uint32_t flags_direct;       // k_decode_pipe: flags go straight to totals[3] (pipe_zero_flags)
  uint64_t wait_ticks;         // WaitBound's limit (kWaitTicks; MTBLX_DEBUG_WAIT_MS shortens it)
  uint64_t dbg_delay0;         // debug: workgroup 0 starts this many ticks late (MTBLX_DEBUG_DELAY0_MS)
};

// Workspace header (byte 128 of the workspace).  The workspace carries state from call to
// call so no fill is needed per call: it must be zero-filled once after allocation.
//  - epoch: launch counter; parity = epoch & 1 selects the aggregate slot of this launch
//  - hw[p]: most tiles any launch of parity p used (slots to clear before they are reused)
//  - done: workgroups finished in this launch; the last one publishes totals[3], resets
//    the flags and done, bumps hw and epoch
struct WsHdr {
  uint32_t epoch;
  uint32_t done;
  uint32_t hw[2];
  unsigned long long flags;   // bit0 overflow, bit1 look-back timeout (-> totals[3])
  unsigned long long tflags[2];   // k_decode_pipe: flags of the launch of each parity (pipe_zero_flags)
};

// Blocks of tile t: [b0, b0 + nb) with b0 = floor(t nblk / ntiles), ntiles = ceil(nblk / bpt)
// (so nb <= bpt).  (Rounding ntiles up to a multiple of the grid, so that every workgroup runs
// the same number of smaller tiles, measured 2 % slower on cfg2: the busiest workgroups keep
// their tile count and every tile pays its fixed costs.)
// (a multiply, not floor(t * nblk / ntiles): two 64-bit divisions per call sat on the
// walker's critical path and on the CU's shared scalar unit -- measured 4 % of the launch)
__device__ __forceinline__ void tile_span(const TileArgs& a, uint32_t t, uint32_t& b0, uint32_t& nb) {
  b0 = t * a.bpt;
  nb = min(a.bpt, a.nblk - b0);
}

// workspace tile entry t: {packed aggregate of launch parity 0, of parity 1, exact key bytes,
// exact records | exact value bytes << 32}.  The exact words are written only when a field of
// the packed word saturates (pack_agg).
constexpr int kTileWords = 4;
__device__ __forceinline__ uint64_t* lb_slot(const TileArgs& a, uint64_t t) { return a.lbw + kTileWords * t + a.par; }
__device__ __forceinline__ uint64_t* lbx_slot(const TileArgs& a, uint64_t t) { return a.lbw + kTileWords * t + 2; }
__device__ __forceinline__ uint64_t* lbx2_slot(const TileArgs& a, uint64_t t) { return a.lbw + kTileWords * t + 3; }

// n records / bytes at `base` fit a buffer of `cap`, without wrap-around: a prefix built from a
// stale or corrupt look-back word (a side word is a full u64) must not pass by overflowing the
// sum and then address below the buffer (base + n wrapping to a small number)
__device__ __forceinline__ bool fits_at(uint64_t base, uint64_t n, uint64_t cap) { return base <= cap && n <= cap - base; }

// kernel prologue: pick the parity, clear the other parity's slots of every tile a previous
// launch of that parity used (the next launch uses them)
__device__ __forceinline__ void ws_begin(TileArgs& a) {
  const uint32_t ep = __hip_atomic_load(&a.hdr->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  a.par = ep & 1u;
  a.hw_other = __hip_atomic_load(&a.hdr->hw[a.par ^ 1u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.hw_other > a.wscap) a.hw_other = a.wscap;   // never write past the caller's workspace
  const uint32_t n = blockDim.x, tid = threadIdx.x;
  for (uint64_t t = (uint64_t)blockIdx.x * n + tid; t < a.hw_other; t += (uint64_t)gridDim.x * n)
    a.lbw[kTileWords * t + (a.par ^ 1u)] = 0;
  // the next launch's flag word (the previous launch of that parity has ended: stream order)
  if (blockIdx.x == 0 && tid == 0)
    __hip_atomic_store(&a.hdr->tflags[a.par ^ 1u], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// test knob (MTBLX_DEBUG_DELAY0_MS): workgroup 0 starts late, as if it were not resident.  Not in
// the fused-verify kernels: any extra code there pushes PipeLargeV past its 128 VGPRs.
__device__ __forceinline__ void ws_debug_delay(const TileArgs& a) {
  if (blockIdx.x == 0 && a.dbg_delay0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < a.dbg_delay0) __builtin_amdgcn_s_sleep(127);
  }
}

// A flag of this launch: k_decode_pipe (flags_direct) ORs it straight into totals[3], other
// kernels into the workspace header (ws_end publishes it).
__device__ __forceinline__ void ws_flag(const TileArgs& a, unsigned long long bit) {
  atomicOr(a.flags_direct ? reinterpret_cast<unsigned long long*>(a.totals + 3) : &a.hdr->flags, bit);
}

// A timeout (bit 1).  Tile 0's walker zeroes totals[3] at a time nobody waits for -- a
// workgroup whose look-back on A(0) gives up because workgroup 0 is late / not resident flags
// BEFORE the zeroing -- so k_decode_pipe also records the timeout in the launch's workspace word,
// which pipe_zero_flags re-reads after its zeroing store: store-buffering with s_waitcnt
// between the two accesses on each side (agent-scope atomics are performed at the device's
// coherence point), so either the re-read sees this timeout or this OR into totals[3] lands
// after the zeroing.  (Overflow flags, bit 0, are set after a look-back that waited on A(0).)
__device__ __forceinline__ void ws_timeout(const TileArgs& a) {
  if (a.flags_direct) {
    __hip_atomic_fetch_or(&a.hdr->tflags[a.par], 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  ws_flag(a, 2ull);
}

// Bounded waits.  A wait on another workgroup (look-back) or on another wave gives up after
// kWaitTicks of wall time (s_memrealtime, 100 MHz) and the launch reports a timeout (totals[3]
// bit 1) instead of hanging.  Generous on purpose: a predecessor tile can legitimately take
// long (a multi-MiB block on the exact serial path), and giving up is only for lost
// co-residency (tiles are assigned round-robin: t = g + k G; claiming them from a ticket
// instead removes that assumption but measured 25 % slower on cfg2 -- one hot atomic word and
// longer look-back waits -- DESIGN.md §4).  Call once per spin; the clock is read every 64.
constexpr uint64_t kWaitTicks = 20ull * 100000000ull;   // 20 s
struct WaitBound {
  uint64_t t0 = 0;
  uint32_t n = 0;
  __device__ __forceinline__ bool expired(uint64_t ticks) {
    if ((++n & 63u) != 0u) return false;
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (t0 == 0) t0 = t;
    return t - t0 > ticks;
  }
};

// kernel epilogue (every thread): the last workgroup to finish closes the launch
__device__ __forceinline__ void ws_end(const TileArgs& a) {
  __syncthreads();
  if (threadIdx.x == 0) {
#if MTBLX_WSEND_LIGHT
    // What the last workgroup reads from the others is only `flags`, which they update with
    // agent-scope atomics; the __syncthreads above waited (vmcnt) until this workgroup's were
    // performed.  No agent-scope release: on gfx950 it writes back the XCD's whole L2
    // (buffer_wbl2), i.e. every dirty output line, once per workgroup.
    const uint32_t old = __hip_atomic_fetch_add(&a.hdr->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t old = __hip_atomic_fetch_add(&a.hdr->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
#endif
    if (old == gridDim.x - 1) {
      const unsigned long long f = __hip_atomic_exchange(&a.hdr->flags, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      a.totals[3] = f | a.inject;
      __hip_atomic_fetch_max(&a.hdr->hw[a.par], a.ntiles, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_exchange(&a.hdr->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&a.hdr->epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}


// k_decode_pipe's launch bookkeeping needs no end-of-launch fan-in (a returning atomic that
// every workgroup waits on took up to ~15 us under the launch's own store traffic, measured):
//  - totals[3] is zeroed by the walker of tile 0 right before it publishes A(0), and every
//    flag is ORed straight into totals[3] (a.flags_direct).  Every look-back -- where
//    overflow flags are set -- waits, directly or through its workgroup's previous tile, on
//    A(0); so every OR lands after the zeroing.
//  - the workgroup owning the last tile bumps the epoch and the high-water mark at its own
//    end: that tile's look-back waited on the aggregate of the G-1 tiles before it, one from
//    every other workgroup (G <= ntiles), so all of them have passed ws_begin by then.
//    A flag set before the zeroing (a look-back on A(0) that timed out because workgroup 0 was
//    not resident) is re-read from the launch's workspace word right after it (ws_flag).
__device__ __forceinline__ void pipe_zero_flags(const TileArgs& a) {   // walker of tile 0, lane 0
  unsigned long long* tot = reinterpret_cast<unsigned long long*>(a.totals + 3);
  __hip_atomic_store(tot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the zeroing is performed before the re-read
  const unsigned long long early = __hip_atomic_load(&a.hdr->tflags[a.par], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (early) __hip_atomic_fetch_or(tot, early, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // performed before A(0) is published
}

__device__ __forceinline__ void pipe_close(const TileArgs& a) {   // last tile's workgroup, thread 0, at its end
  if (a.inject) __hip_atomic_fetch_or(a.totals + 3, a.inject, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_max(&a.hdr->hw[a.par], a.ntiles, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_add(&a.hdr->epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Contiguous range of tile t: [r0, r1) of the data buffer (r0 16-aligned), or r1 = 0 if the
// tile's blocks do not sit in one range that fits the staging buffer.
__device__ __forceinline__ void tile_range(const TileArgs& a, uint32_t t, uint32_t tb, uint64_t& r0, uint64_t& r1) {
  uint32_t b0, nb;
  tile_span(a, t, b0, nb);
  MTBLX_CHK(a.blk_off + b0, 8 * nb);
  MTBLX_CHK(a.blk_len + b0, 4 * nb);
  const uint64_t s = a.blk_off[b0];
  const uint64_t e = a.blk_off[b0 + nb - 1] + a.blk_len[b0 + nb - 1];
  const uint64_t base = reinterpret_cast<uintptr_t>(a.data);
  r0 = ((base + s) & ~15ull) - base;   // may be "negative" (wraps) if data is unaligned: clamp
  if (base + s < 16 || ((base + s) & ~15ull) < base) r0 = 0;
  r1 = (e > s && e - r0 + 48 <= tb) ? e : 0;
  for (uint32_t j = 1; r1 && j + 1 < nb; ++j)   // every block inside [s, e) (see pipe_dma)
    if (a.blk_off[b0 + j] < s || a.blk_off[b0 + j] + a.blk_len[b0 + j] > e) r1 = 0;
}

// prefetch chunk c (16 B) of a contiguous range into v (zero-filled outside the buffer)
__device__ __forceinline__ uint4 load_chunk(const TileArgs& a, uint64_t off) {
  if (off + 16 <= a.data_len) {
    MTBLX_CHK(a.data + off, 16);
    return *reinterpret_cast<const uint4*>(a.data + off);
  }
  uint32_t t[4] = {0, 0, 0, 0};
  for (int i = 0; i < 16; ++i)
    if (off + i < a.data_len) MTBLX_CHK(a.data + off + i, 1), t[i >> 2] |= (uint32_t)a.data[off + i] << (8 * (i & 3));
  return make_uint4(t[0], t[1], t[2], t[3]);
}

// Stage one block into a 16-byte aligned slot (fallback layout); returns the offset of
// block byte 0 within the slot.
__device__ __forceinline__ uint32_t stage_slot(const TileArgs& a, uint8_t* slot, uint64_t off, uint32_t L, int lane) {
  const uint64_t base = reinterpret_cast<uintptr_t>(a.data);
  const uint64_t a0 = ((base + off) & ~15ull) - base;
  const uint32_t delta = (uint32_t)(off - a0);
  const uint32_t nch = (delta + L + 15u) >> 4;
  for (uint32_t c = lane; c < nch; c += kWave) *reinterpret_cast<uint4*>(slot + 16 * c) = load_chunk(a, a0 + 16ull * c);
  return delta;
}

// Tight walk of restart interval [s, e) of a staged block (byte 0 at stage offset bo).
// Regular-path preconditions (DESIGN.md "regular blocks"): every entry decodes without a
// reference panic; varints are terminated; the first entry has shared == 0 and later
// ones shared <= previous key length (so Vec capacity never matters); fields fit 16
// bits; the walk lands exactly on e.  Under these the reference's linear chain
// (src/block.rs:119-143) visits exactly these entries and rebuilds exactly these keys.
template <bool WRITE>
__device__ __forceinline__ bool walk_interval(const uint8_t* stage, Rec* recs, uint32_t bo, uint32_t L, uint32_t R, uint32_t s,
                                              uint32_t e, uint32_t& cnt, uint32_t& kb, uint32_t& vb, uint32_t slot0,
                                              uint32_t kbase, uint32_t vbase, uint32_t blk, uint32_t rlo,
                                              uint32_t rhi) {
  cnt = kb = vb = 0;
  if (!(s < e && e <= R)) return false;
  uint32_t p = s, prevlen = 0;
  const uint32_t* st32 = reinterpret_cast<const uint32_t*>(stage);
  while (p < e) {
    const uint32_t ad = bo + p;
    uint32_t hw = (MTBLX_LCHK(st32 + (ad >> 2), 8), __builtin_amdgcn_alignbit(st32[(ad >> 2) + 1], st32[ad >> 2], (ad & 3u) * 8u));
    uint32_t sh = hw & 0xffu, ns = (hw >> 8) & 0xffu, vl = (hw >> 16) & 0xffu, h = 3;
    if (__builtin_expect((hw & 0x808080u) != 0u, 0)) {  // multi-byte varint header (slow path)
      if (R - p < 3u) return false;
      uint4 W = lds_win16(stage, ad);
      uint32_t l0 = dec32(W, 0, L - p, sh);
      if (l0 == 0) return false;
      uint32_t l1 = dec32(W, l0, L - p - l0, ns);
      if (l1 == 0) return false;
      uint32_t l2 = dec32(W, l0 + l1, L - p - l0 - l1, vl);
      if (l2 == 0) return false;
      h = l0 + l1 + l2;
      if (p + h > R) return false;                        // assert!(p <= limit)
      if ((sh | ns | vl) > 0xFFFFu) return false;
    }
    // R - p >= h + ns + vl covers decode_entry's `limit - p >= 3` and the slice assert
    if (R - p < h + ns + vl) return false;
    if (sh > prevlen) return false;                       // first entry: prevlen = 0 -> shared == 0
    const uint32_t klen = sh + ns;
    if (WRITE) {
      const uint32_t r = slot0 + cnt;
      if (r >= rlo && r < rhi) {
        Rec x;
        x.pos_sh = (p + h) | (sh << 16);
        x.ns_vl = ns | (vl << 16);
        x.ks = kbase + kb;
        x.vs_blk = (vbase + vb) | (blk << 24);
        recs[r - rlo] = x;
      }
    }
    cnt += 1;
    kb += klen;
    vb += vl;
    prevlen = klen;
    p += h + ns + vl;
  }
  return p == e && (prevlen <= 0xFFFFu);
}

// Tight walk for the common case: every header is three 1-byte varints.  All checks are
// accumulated into `bad` off the loop-carried chain (p -> LDS read -> p'); any multi-byte
// header, shared > previous length, or overrun ends it and the caller falls back to the
// exact walk_interval above.  Same preconditions, same results when it returns true.
template <bool WRITE>
__device__ __forceinline__ bool walk_fast(const uint8_t* stage, Rec* recs, uint32_t bo, uint32_t R, uint32_t s, uint32_t e,
                                          uint32_t& cnt, uint32_t& kb, uint32_t& vb, uint32_t slot0, uint32_t kbase,
                                          uint32_t vbase, uint32_t blk, uint32_t rlo, uint32_t rhi) {
  cnt = kb = vb = 0;
  if (!(s < e && e <= R)) return false;
  uint32_t p = s, prevlen = 0, bad = 0;
  const uint32_t* st32 = reinterpret_cast<const uint32_t*>(stage);
  do {
    const uint32_t ad = bo + p;
    const uint32_t hw = (MTBLX_LCHK(st32 + (ad >> 2), 8), __builtin_amdgcn_alignbit(st32[(ad >> 2) + 1], st32[ad >> 2], (ad & 3u) * 8u));
    const uint32_t sh = hw & 0xffu, ns = (hw >> 8) & 0xffu, vl = (hw >> 16) & 0xffu;
    const uint32_t np = p + 3u + ns + vl;
    bad |= (hw & 0x808080u) | (uint32_t)(sh > prevlen) | (uint32_t)(np > R);
    if (WRITE) {
      const uint32_t r = slot0 + cnt;
      if (r >= rlo && r < rhi) {
        Rec x;
        x.pos_sh = (p + 3u) | (sh << 16);
        x.ns_vl = ns | (vl << 16);
        x.ks = kbase + kb;
        x.vs_blk = (vbase + vb) | (blk << 24);
        recs[r - rlo] = x;
      }
    }
    const uint32_t klen = sh + ns;
    cnt += 1;
    kb += klen;
    vb += vl;
    prevlen = klen;
    p = np;
  } while (p < e && !bad);
  return !bad && p == e;
}

// exclusive scan of 3 u32 per thread over the workgroup; returns the workgroup totals
template <class C>
__device__ __forceinline__ void wg_excl_scan3(TileLds<C>& S, uint32_t& a, uint32_t& b, uint32_t& c, uint32_t tot[3]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t ia = wave_incl_scan(a, lane), ib = wave_incl_scan(b, lane), ic = wave_incl_scan(c, lane);
  if (lane == kWave - 1) { S.wsum[wv][0] = ia; S.wsum[wv][1] = ib; S.wsum[wv][2] = ic; }
  __syncthreads();
  uint32_t oa = 0, ob = 0, oc = 0;
  tot[0] = tot[1] = tot[2] = 0;
  for (int k = 0; k < kThreads / kWave; ++k) {
    if (k < wv) { oa += S.wsum[k][0]; ob += S.wsum[k][1]; oc += S.wsum[k][2]; }
    tot[0] += S.wsum[k][0]; tot[1] += S.wsum[k][1]; tot[2] += S.wsum[k][2];
  }
  a = oa + ia - a;
  b = ob + ib - b;
  c = oc + ic - c;
  __syncthreads();
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) v += __shfl_xor(v, d, kWave);
  return v;
}

// Publish the aggregate (records r, key bytes k, value bytes v) of tile t: one packed 8-byte
// agent-scope word, ready | r << 42 | v << 21 | k (21 bits each).  If any of the three does not
// fit its field, the exact values go to the tile's side words first (release-ordered) and the
// packed word carries the marker k == kField; lb_take then reads all three from the side words.
// (A tile can hold one block of up to 4 GiB: k_decode_tiles, or an unstaged block.)
__device__ __forceinline__ void lb_publish(const TileArgs& a, uint64_t t, uint32_t r, uint64_t k, uint32_t v) {
  uint64_t w;
  if (r >= kField || v >= kField || k >= kField) {
    __hip_atomic_store(lbx_slot(a, t), k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(lbx2_slot(a, t), (uint64_t)r | ((uint64_t)v << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the side words are performed before the flag word
    w = kReady | ((uint64_t)kField << 42) | ((uint64_t)kField << 21) | (uint64_t)kField;
  } else {
    w = kReady | ((uint64_t)r << 42) | ((uint64_t)v << 21) | k;
  }
  __hip_atomic_store(lb_slot(a, t), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Add the aggregate of tile i (its ready packed word w) to the running sums.
__device__ __forceinline__ void lb_take(const TileArgs& a, uint64_t i, uint64_t w, uint64_t& sr, uint64_t& sk,
                                        uint64_t& sv) {
  uint64_t r = (w >> 42) & kField, v = (w >> 21) & kField, k = w & kField;
  if (k == kField) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    k = __hip_atomic_load(lbx_slot(a, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t x = __hip_atomic_load(lbx2_slot(a, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    r = (uint32_t)x;
    v = x >> 32;
  }
  sr += r;
  sk += k;
  sv += v;
}

// wave-wide sum of per-lane look-back sums (32-bit adds unless some lane saw an exact word)
__device__ __forceinline__ uint64_t lb_wave_sum(uint64_t x) {
  return __ballot(x >= (1ull << 24)) == 0ull ? (uint64_t)wave_sum32((uint32_t)x) : wave_sum64(x);
}

template <class C>
__global__ void __launch_bounds__(kThreads, C::MINW) k_decode_tiles(TileArgs a) {
  __shared__ TileLds<C> S;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t G = gridDim.x;
  ws_begin(a);
#ifdef MTBLX_STAMPS
  // diagnostic build only: per-phase cycles of thread 0 (s_memtime), summed over tiles
  uint64_t tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tprev = __builtin_amdgcn_s_memtime(), ntl = 0;
#define STAMP(k) do { if (tid == 0) { const uint64_t _t = __builtin_amdgcn_s_memtime(); tacc[k] += _t - tprev; tprev = _t; } } while (0)
#else
#define STAMP(k) do { } while (0)
#endif
  if (tid == 0) { S.tinc[0] = S.tinc[1] = S.tinc[2] = 0; }

  // prefetch registers for the next tile's contiguous range
  uint4 pf[kPrefetch];
  uint64_t pr0 = 0, pr1 = 0;
  if (C::PREFETCH && blockIdx.x < a.ntiles) {
    tile_range(a, blockIdx.x, C::TB, pr0, pr1);
    if (pr1) {
#pragma unroll
      for (int k = 0; k < kPrefetch; ++k) {
        const uint64_t o = pr0 + 16ull * (tid + k * kThreads);
        pf[k] = (o < pr1) ? load_chunk(a, o) : make_uint4(0, 0, 0, 0);
      }
    }
  }

  for (uint32_t t = blockIdx.x; t < a.ntiles; t += G) {
    uint32_t b0, nb;
    tile_span(a, t, b0, nb);
#ifdef MTBLX_STAMPS
    ++ntl;
#endif
    STAMP(7);

    // ---- 1. stage ----
    uint64_t r0 = pr0, r1 = pr1;
    if (!C::PREFETCH) tile_range(a, t, C::TB, r0, r1);
    if (r1) {
      // contiguous layout: range byte x at stage offset 16 + x
      const uint32_t nch = (uint32_t)((r1 - r0 + 15) >> 4);
      if (C::PREFETCH) {
#pragma unroll
        for (int k = 0; k < kPrefetch; ++k) {
          const uint32_t c = tid + k * kThreads;
          if (c < nch) *reinterpret_cast<uint4*>(S.stage + 16 + 16 * c) = pf[k];
        }
        for (uint32_t c = tid + kPrefetch * kThreads; c < nch; c += kThreads)
          *reinterpret_cast<uint4*>(S.stage + 16 + 16 * c) = load_chunk(a, r0 + 16ull * c);
      } else {
        constexpr int U = 4;
        uint32_t c = tid;
        for (; c + (U - 1) * kThreads < nch; c += U * kThreads) {
          uint4 v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) v[u] = load_chunk(a, r0 + 16ull * (c + u * kThreads));
#pragma unroll
          for (int u = 0; u < U; ++u) *reinterpret_cast<uint4*>(S.stage + 16 + 16 * (c + u * kThreads)) = v[u];
        }
        for (; c < nch; c += kThreads) *reinterpret_cast<uint4*>(S.stage + 16 + 16 * c) = load_chunk(a, r0 + 16ull * c);
      }
      if (tid < (int)nb) {
        MTBLX_CHK(a.blk_off + b0 + tid, 8);
        MTBLX_CHK(a.blk_len + b0 + tid, 4);
        const uint64_t off = a.blk_off[b0 + tid];
        const uint32_t L = a.blk_len[b0 + tid];
        S.boff[tid] = off + L > a.data_len ? kOutOfBounds
                      : (off >= r0 && off + L <= r1) ? (uint32_t)(16 + off - r0) : kNotStaged;
        S.blen[tid] = L;
      }
    } else {
      // fallback: one 16-aligned slot per block, wave w stages blocks w, w+4, ...
      for (uint32_t j = wv; j < nb; j += kThreads / kWave) {
        MTBLX_CHK(a.blk_off + b0 + j, 8);
        MTBLX_CHK(a.blk_len + b0 + j, 4);
        const uint32_t L = a.blk_len[b0 + j];
        const uint64_t off = a.blk_off[b0 + j];
        const uint32_t so = 16u + j * a.slot;
        uint32_t bo = kNotStaged;
        if (off + L > a.data_len) bo = kOutOfBounds;
        else if (L + 15u <= a.slot && so + a.slot + 32u <= (uint32_t)C::TB) bo = so + stage_slot(a, S.stage + so, off, L, lane);
        if (lane == 0) { S.boff[j] = bo; S.blen[j] = L; }
      }
    }
    __syncthreads();
    STAMP(0);

    // ---- 1b. prefetch the next tile of this workgroup into registers ----
    if (C::PREFETCH) {
      pr1 = 0;
      if (t + G < a.ntiles) {
        tile_range(a, t + G, C::TB, pr0, pr1);
        if (pr1) {
#pragma unroll
          for (int k = 0; k < kPrefetch; ++k) {
            const uint64_t o = pr0 + 16ull * (tid + k * kThreads);
            pf[k] = (o < pr1) ? load_chunk(a, o) : make_uint4(0, 0, 0, 0);
          }
        }
      }
    }

    // ---- 2. trailers (Block::init, src/block.rs:16-49) + interval numbering (wave 0) ----
    if (wv == 0) {
      uint32_t n = 0, R = 0, ok = 0;
      if (lane < (int)nb) {
        const uint32_t j = lane, L = S.blen[j], bo = S.boff[j];
        if (bo < kOutOfBounds && L >= 8) {
          n = lds_rd32(S.stage, bo + L - 4);
          if (n != 0 && (uint64_t)(n + 1ull) * 4ull <= L) { R = L - 4u * (n + 1u); ok = 1; }
        }
        if (!ok) n = 0;
      }
      uint32_t incl = wave_incl_scan(n, lane);
      // blocks whose intervals overflow MAXINT become irregular
      if (ok && incl > (uint32_t)C::MAXINT) { ok = 0; }
      n = ok ? n : 0;
      incl = wave_incl_scan(n, lane);
      if (lane < (int)nb) {
        S.bn[lane] = n;
        S.bR[lane] = R;
        S.bok[lane] = ok;
        S.bwr[lane] = S.boff[lane] != kOutOfBounds;
        S.bst[lane] = MTBLX_ST_OK;
        S.bint0[lane] = incl - n;
      }
      if (lane == (int)nb - 1) S.bint0[nb] = incl;
    }
    __syncthreads();
    const uint32_t nint = S.bint0[nb];

    // ---- 3. walk 1: one thread per restart interval across the tile ----
    if (tid < (int)nint) {
      const uint32_t f = tid;
      uint32_t j = 0;
      while (S.bint0[j + 1] <= f) ++j;
      const uint32_t i = f - S.bint0[j], bo = S.boff[j], L = S.blen[j], R = S.bR[j], n = S.bn[j];
      const uint32_t s = lds_rd32(S.stage, bo + R + 4u * i);
      const uint32_t e = (i + 1 < n) ? lds_rd32(S.stage, bo + R + 4u * (i + 1)) : R;
      uint32_t cnt, kb, vb;
      bool ok = walk_fast<false>(S.stage, S.rec, bo, R, s, e, cnt, kb, vb, 0, 0, 0, 0, 0, 0);
      if (!ok) ok = walk_interval<false>(S.stage, S.rec, bo, L, R, s, e, cnt, kb, vb, 0, 0, 0, 0, 0, 0);
      ok = ok && cnt <= (uint32_t)C::MAXREC;
      S.icnt[f] = cnt;
      S.ikb[f] = kb;
      S.ivb[f] = vb;
      S.iblk[f] = (uint8_t)j;
      if (!ok) S.bok[j] = 0;
    }
    __syncthreads();
    STAMP(1);

    // ---- 4. irregular blocks: exact serial count (generic path, lane per block) ----
    if (tid < (int)nb && !S.bok[tid]) {
      const uint32_t j = tid, bo = S.boff[j], L = S.blen[j];
      const uint8_t* d = (bo != kNotStaged) ? (S.stage + bo) : (a.data + a.blk_off[b0 + j]);
      const GenOut o = bo == kOutOfBounds ? GenOut{0, 0, 0, MTBLX_ST_CORRUPT}
                                          : generic_block<false>(d, L, nullptr, nullptr, nullptr, nullptr);
      S.bcnt[j] = o.nrec;
      S.bkb[j] = (uint32_t)o.kb;
      S.bvb[j] = (uint32_t)o.vb;
      S.bst[j] = o.st;
      if (!gen_writable(bo, o.st)) S.bwr[j] = 0;
    }
    // interval scan (regular blocks only) -> exclusive bases
    {
      uint32_t xc = 0, xk = 0, xv = 0;
      const uint32_t f = tid;
      if (f < nint && S.bok[S.iblk[f]]) { xc = S.icnt[f]; xk = S.ikb[f]; xv = S.ivb[f]; }
      uint32_t tot[3];
      wg_excl_scan3(S, xc, xk, xv, tot);
      if (f < nint) { S.icnt[f] = xc; S.ikb[f] = xk; S.ivb[f] = xv; }
      if (tid == 0) { S.icnt[nint] = tot[0]; S.ikb[nint] = tot[1]; S.ivb[nint] = tot[2]; S.nfastrec = tot[0]; }
    }
    __syncthreads();
    // block totals + tile-relative block bases (wave 0, one lane per block)
    if (wv == 0) {
      uint32_t c = 0, k = 0, v = 0, rf = 0;
      if (lane < (int)nb) {
        const uint32_t j = lane;
        const uint32_t fa = S.bint0[j], fb = S.bint0[j + 1];
        rf = S.icnt[fa];
        if (S.bok[j]) {
          c = S.icnt[fb] - S.icnt[fa];
          k = S.ikb[fb] - S.ikb[fa];
          v = S.ivb[fb] - S.ivb[fa];
        } else {
          c = S.bcnt[j];
          k = S.bkb[j];
          v = S.bvb[j];
        }
      }
      const uint32_t ic = wave_incl_scan(c, lane), ik = wave_incl_scan(k, lane), iv = wave_incl_scan(v, lane);
      if (lane < (int)nb) {
        S.bcnt[lane] = c; S.bkb[lane] = k; S.bvb[lane] = v;
        S.brb[lane] = ic - c; S.bkbb[lane] = ik - k; S.bvbb[lane] = iv - v;
        S.brf[lane] = rf;
      }
      if (lane == (int)nb - 1) { S.ttot[0] = ic; S.ttot[1] = ik; S.ttot[2] = iv; }
    }
    __syncthreads();
    STAMP(2);

    // ---- 5. publish the tile aggregate, issue the look-back loads ----
    const uint32_t agg_r = S.ttot[0], agg_k = S.ttot[1], agg_v = S.ttot[2];
    if (tid == 0) lb_publish(a, t, agg_r, agg_k, agg_v);
    const uint32_t lo = (t >= G) ? t - G + 1 : 0;   // window of predecessors [lo, t)
    uint64_t lw[kMaxLookbackLoads];
#pragma unroll
    for (int m = 0; m < kMaxLookbackLoads; ++m) {
      const int64_t i = (int64_t)t - 1 - tid - (int64_t)m * kThreads;
      lw[m] = kReady;  // outside the window: contributes 0
      if (i >= (int64_t)lo) lw[m] = __hip_atomic_load(lb_slot(a, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    STAMP(3);

    // ---- 6. walk 2: per-record metadata (chunk 0) ----
    const uint32_t nfr = S.nfastrec;
    uint32_t fa = 0, fb = 0, rlo = 0, rhi = 0;
    auto plan_chunk = [&](uint32_t from) {
      fa = from;
      const uint32_t lim = S.icnt[fa] + (uint32_t)C::MAXREC;
      if (S.icnt[nint] <= lim) {
        fb = nint;
      } else {  // largest fb with icnt[fb] <= lim (walk 1 guarantees one interval fits)
        uint32_t l = fa + 1, h = nint;
        while (l < h) {
          const uint32_t m = (l + h + 1) / 2;
          if (S.icnt[m] <= lim) l = m; else h = m - 1;
        }
        fb = l;
      }
      rlo = S.icnt[fa];
      rhi = S.icnt[fb];
    };
    auto walk2 = [&]() {
      const uint32_t f = fa + tid;
      if (f < fb) {
        const uint32_t j = S.iblk[f];
        if (S.bok[j]) {
          const uint32_t fj = S.bint0[j];
          const uint32_t i = f - fj, bo = S.boff[j], L = S.blen[j], R = S.bR[j], n = S.bn[j];
          const uint32_t s = lds_rd32(S.stage, bo + R + 4u * i);
          const uint32_t e = (i + 1 < n) ? lds_rd32(S.stage, bo + R + 4u * (i + 1)) : R;
          const uint32_t kin = S.ikb[f] - S.ikb[fj], vin = S.ivb[f] - S.ivb[fj];
          uint32_t c, k, v;
          if (!walk_fast<true>(S.stage, S.rec, bo, R, s, e, c, k, v, S.icnt[f], S.bkbb[j] + kin, S.bvbb[j] + vin, j, rlo, rhi))
            walk_interval<true>(S.stage, S.rec, bo, L, R, s, e, c, k, v, S.icnt[f], S.bkbb[j] + kin, S.bvbb[j] + vin, j, rlo,
                                rhi);
        }
      }
    };
    if (a.write && nfr) {
      plan_chunk(0);
      walk2();
    }
    STAMP(4);

    // ---- 7. finish the look-back ----
    {
      uint64_t sr = 0, sk = 0, sv = 0;
      bool timeout = false;
#pragma unroll
      for (int m = 0; m < kMaxLookbackLoads; ++m) {
        const int64_t i = (int64_t)t - 1 - tid - (int64_t)m * kThreads;
        uint64_t w = lw[m];
        WaitBound wb;
        while (!(w & kReady)) {
          __builtin_amdgcn_s_sleep(2);
          w = __hip_atomic_load(lb_slot(a, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (wb.expired(a.wait_ticks)) { timeout = true; w = kReady; }
        }
        if (i >= (int64_t)lo) lb_take(a, (uint64_t)i, w, sr, sk, sv);
      }
      if (timeout) ws_timeout(a);
      // per-thread sums are < 2^23 (4 tiles x 21-bit fields) unless a tile published exact words
      sr = lb_wave_sum(sr);
      sv = lb_wave_sum(sv);
      sk = lb_wave_sum(sk);
      if (lane == 0) { S.lbsum[wv][0] = sr; S.lbsum[wv][1] = sk; S.lbsum[wv][2] = sv; }
      __syncthreads();
      if (tid == 0) {
        const uint64_t pre0 = S.tinc[0] + S.lbsum[0][0] + S.lbsum[1][0] + S.lbsum[2][0] + S.lbsum[3][0];
        const uint64_t pre1 = S.tinc[1] + S.lbsum[0][1] + S.lbsum[1][1] + S.lbsum[2][1] + S.lbsum[3][1];
        const uint64_t pre2 = S.tinc[2] + S.lbsum[0][2] + S.lbsum[1][2] + S.lbsum[2][2] + S.lbsum[3][2];
        S.tpre[0] = pre0; S.tpre[1] = pre1; S.tpre[2] = pre2;
        S.tinc[0] = pre0 + agg_r; S.tinc[1] = pre1 + agg_k; S.tinc[2] = pre2 + agg_v;
        if (t == a.ntiles - 1) {
          MTBLX_CHK(a.totals, 24);
          a.totals[0] = pre0 + agg_r;
          a.totals[1] = pre1 + agg_k;
          a.totals[2] = pre2 + agg_v;
        }
      }
      __syncthreads();
    }
    const uint64_t pr = S.tpre[0], pk = S.tpre[1], pv = S.tpre[2];
    STAMP(5);

    // ---- 8. per-block outputs + capacity check ----
    if (tid < (int)nb) {
      const uint32_t j = tid, b = b0 + j;
      const uint64_t rb = pr + S.brb[j], kb = pk + S.bkbb[j], vb = pv + S.bvbb[j];
      MTBLX_CHK(a.nrec + b, 4);
      MTBLX_CHK(a.rec_base + b, 8);
      MTBLX_CHK(a.key_base + b, 8);
      MTBLX_CHK(a.val_base + b, 8);
      MTBLX_CHK(a.status + b, 4);
      a.nrec[b] = S.bcnt[j];
      a.rec_base[b] = rb;
      a.key_base[b] = kb;
      a.val_base[b] = vb;
      int32_t st = S.bst[j];
      if (a.write && !(fits_at(rb, S.bcnt[j], a.rec_cap) && fits_at(kb, S.bkb[j], a.keys_cap) &&
                       fits_at(vb, S.bvb[j], a.vals_cap))) {
        st = MTBLX_ST_OVERFLOW;
        S.bwr[j] = 0;
        ws_flag(a, 1ull);
      }
      a.status[b] = st;
    }
    if (!a.write) { __syncthreads(); continue; }
    __syncthreads();

    // ---- 9. copy (one thread per record), chunk by chunk ----
    while (nfr) {
      for (uint32_t q = tid; q < rhi - rlo; q += kThreads) {
        const uint4 rr = *reinterpret_cast<const uint4*>(&S.rec[q]);
        const uint32_t j = rr.w >> 24;
        if (!S.bwr[j]) continue;
        const uint32_t bo = S.boff[j];
        const uint32_t pos = rr.x & 0xFFFFu, shr = rr.x >> 16, ns = rr.y & 0xFFFFu, vl = rr.y >> 16;
        const uint32_t ks = rr.z, vs = rr.w & 0xFFFFFFu;
        const uint32_t klen = shr + ns;
        // key_end / val_end: END offsets relative to the block's bases
        const uint64_t gr = pr + S.brb[j] + (q + rlo - S.brf[j]);
        MTBLX_CHK(a.key_end + gr, 4);
        MTBLX_CHK(a.val_end + gr, 4);
        a.key_end[gr] = ks + klen - S.bkbb[j];
        a.val_end[gr] = vs + vl - S.bvbb[j];
#ifndef MTBLX_ABL_NOVAL
        // value bytes: LDS window -> unaligned 16-byte stores
        const uint32_t vsrc = bo + pos + ns;
        uint8_t* vd = a.vals + pv + vs;
        for (uint32_t o = 0; o < vl; o += 16) {
          uint4 w4 = lds_win16(S.stage, vsrc + o);
          const uint32_t m = vl - o;
          store_bytes(vd + o, w4, m < 16 ? m : 16);
        }
#endif
#ifndef MTBLX_ABL_NOKEY
        // key bytes: each byte comes from the suffix of the latest record s <= q (same
        // interval) with shared_s <= byte index
        uint8_t* kd = a.keys + pk + ks;
        for (uint32_t j0 = 0; j0 < klen; j0 += 16) {
          const uint32_t jend = (j0 + 16 < klen) ? j0 + 16 : klen;
          uint4 outw = make_uint4(0, 0, 0, 0);
          uint32_t jj = j0;
          while (jj < jend) {
            uint32_t sidx = q, m = klen, shs = shr, ps = pos;
            while (shs > jj) {
              m = shs < m ? shs : m;
              --sidx;
              const uint32_t x = S.rec[sidx].pos_sh;
              shs = x >> 16;
              ps = x & 0xFFFFu;
            }
            const uint32_t seg = m < jend ? m : jend;
            const uint32_t src = bo + ps + (jj - shs);
            uint4 w4 = lds_win16(S.stage, src - (jj - j0));
            merge_bytes(outw, w4, (int)(jj - j0), (int)(seg - j0));
            jj = seg;
          }
          store_bytes(kd + j0, outw, jend - j0);
        }
#endif
      }
      __syncthreads();
      if (fb >= nint) break;
      plan_chunk(fb);
      walk2();
      __syncthreads();
    }
    STAMP(6);

    // ---- 10. irregular blocks: exact serial write (lane per block) ----
    if (tid < (int)nb && !S.bok[tid] && S.bwr[tid]) {
      const uint32_t j = tid, bo = S.boff[j], L = S.blen[j];
      const uint8_t* d = (bo != kNotStaged) ? (S.stage + bo) : (a.data + a.blk_off[b0 + j]);
      generic_block<true>(d, L, a.keys + pk + S.bkbb[j], a.vals + pv + S.bvbb[j], a.key_end + pr + S.brb[j],
                          a.val_end + pr + S.brb[j]);
    }
    __syncthreads();
  }
  ws_end(a);
#ifdef MTBLX_STAMPS
  if (tid == 0 && a.dbg) {
    for (int k = 0; k < 8; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg + k), (unsigned long long)tacc[k]);
    atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg + 8), (unsigned long long)ntl);
  }
#endif
}

// ----------------------------------------------------------------------------------
// software-pipelined decoder for small blocks (k_decode_pipe)
// ----------------------------------------------------------------------------------
// One 512-thread workgroup per CU, persistent, static round-robin over tiles
// (t = g + kG), three LDS tile buffers.  Iteration i (buffers rotate mod 3):
//   wave 0      : LDS-DMA (global_load_lds, no registers) of tile i+2; walk of tile i+1
//                 -- the minimal header chain: one lane per restart interval records
//                 the header offset of every entry in slot 16 f + k and counts; interval
//                 scan; block totals; publish the tile aggregate A; vmcnt(0) (retires
//                 the DMA of tile i+2 before the barrier, read one phase later)
//   wave 1      : look-back of tile i from aggregate words it loaded one iteration
//                 earlier; per-block outputs; then issues the loads for tile i+1
//   waves 2..7  : record pass + copy of tile i: one 16-lane DPP row per restart
//                 interval (entry k = lane k of the row).  Key prefixes are rebuilt
//                 in parallel by a row-wide Hillis-Steele scan of the associative
//                 "truncate-then-append" operator (src/block.rs:134-135), 16 key
//                 bytes per plane, any key length; values and keys go out with
//                 unaligned 16 B stores
//   s_waitcnt lgkmcnt(0); s_barrier (raw: global stores and the DMA in flight are not
//   drained at the barrier)
// Restart intervals of more than 16 entries (the reference default is 16,
// src/lib.rs:4), tiles of more than MAXINT intervals and anything irregular take the
// exact generic path for the affected blocks.
// diagnostic per-phase cycle stamps (MTBLX_STAMPS builds only; lane 0 of a wave)
struct Stamps {
#ifdef MTBLX_STAMPS
  uint64_t acc[15] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t prev = 0;
  __device__ __forceinline__ void init() { prev = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void hit(int k) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    acc[k] += t - prev;
    prev = t;
  }
#else
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void hit(int) {}
#endif
};

#ifdef MTBLX_STAMPS
// diagnostic timeline (s_memrealtime, 100 MHz) per workgroup of the last k_decode_pipe launch:
// [0] entry [1] preload done [2] first walk done (it = -1) [3] it = 0 done [4] loop end
// [5] after ws_end [6] tiles of this workgroup
__device__ uint64_t g_tl[1024][16];
#define TL(k) do { if (threadIdx.x == 0 && blockIdx.x < 1024) g_tl[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
// stamp by lane 0 of the calling wave (any wave)
#define TLW(k) do { if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) g_tl[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define TL(k) do { } while (0)
#define TLW(k) do { } while (0)
#endif

constexpr int kPipeThreads = 1024;
constexpr int kPipeLoadWave = 2;                                         // LDS-DMA loaders (issue no stores)
constexpr int kP2Spi = 16;                                               // slots per interval (= DPP row)
constexpr uint32_t kLargeDmaSplit = 24;   // PipeLarge, short copies: pieces staged before the walk ends (of ~64)

// Pipeline configurations.  TB = staging bytes of a tile buffer, NBUF = tile buffers in
// LDS (3: DMA / walk / copy of three tiles overlap; 2: DMA of the next tile overlaps the
// walk + copy of this one), MAXBLK blocks and MAXINT (<= 64: one walk lane each) restart
// intervals per tile.
// LOADW LDS-DMA loader waves (waves 2 .. 2 + LOADW - 1); the rest from 2 + LOADW copy.
template <int TB_, int NBUF_, int MAXBLK_, int MAXINT_, bool VERIFY_ = false, int LOADW_ = 2>
struct PipeCfg {
  static constexpr int TB = TB_, NBUF = NBUF_, MAXBLK = MAXBLK_, MAXINT = MAXINT_;
  static constexpr int SLOTS = MAXINT * kP2Spi;
  static constexpr bool VERIFY = VERIFY_;   // fused CRC-32C of every staged block (f1)
  static constexpr int LOADW = LOADW_;
  static constexpr int COPY0 = kPipeLoadWave + LOADW;             // first copy wave
  static constexpr int NCOPY = kPipeThreads / kWave - COPY0;      // copy waves
  static constexpr int ROWS = NCOPY * (kWave / 16);               // intervals per copy round
};
// (PipeLarge with four loaders and ten copy waves: +0.8 % on 16 B keys, -16 % on cfg3's long
// Zipf keys, whose copy is the longer half of the iteration)
// PipeSmall's staging bytes per tile buffer (three buffers in LDS).  49 664 fits twelve 4 KiB blocks
// (cfg2) or three 16 KiB blocks (cfg4's middle leg) per tile with their framing; 49 152 fitted
// eleven / two: cfg4 2302 -> 2544 GiB/s (16 KiB leg 2182 -> 2794), profiles/r06/small_tb/
#ifndef MTBLX_SMALL_TB
#define MTBLX_SMALL_TB 49664
#endif
using PipeSmall = PipeCfg<MTBLX_SMALL_TB, 3, 16, 56>;   // blocks up to ~48 KiB (cfg2 4 KiB, cfg4 16 KiB)
#ifndef MTBLX_LARGE_LOADW
#define MTBLX_LARGE_LOADW 2
#endif
using PipeLarge = PipeCfg<65664, 2, 2, 64, false, MTBLX_LARGE_LOADW>;    // blocks up to ~64 KiB (cfg3, cfg4 64 KiB)
using PipeSmallV = PipeCfg<49152, 3, 16, 56, true>;
using PipeLargeV = PipeCfg<65664, 2, 2, 64, true>;

template <class P>
struct alignas(16) PipeBuf {
  uint8_t stage[P::TB];
  uint16_t pos[P::SLOTS];     // header offset (block-relative) of entry k of interval f: slot 16 f + k
  uint32_t boff[P::MAXBLK], blen[P::MAXBLK];
  uint32_t bok[P::MAXBLK], bwr[P::MAXBLK];
  int32_t bst[P::MAXBLK];
  uint32_t bcnt[P::MAXBLK], bkb[P::MAXBLK], bvb[P::MAXBLK];
  uint32_t brb[P::MAXBLK], bkbb[P::MAXBLK], bvbb[P::MAXBLK];
  // per interval: tile-relative bases after the scan
  uint32_t icnt[P::MAXINT + 1], ikb[P::MAXINT + 1], ivb[P::MAXINT + 1];
  uint8_t iraw[P::MAXINT];    // entries of the interval (<= 16)
  uint8_t iblk[P::MAXINT];
  uint64_t tpre[3];
  uint32_t ttot[3];
  uint32_t nb, b0, nint;
};

template <class P>
struct alignas(16) PipeLds {
  PipeBuf<P> buf[P::NBUF];
  uint32_t ready;    // wave 1 sets after the prefix + per-block outputs of the tile to copy
  uint32_t pub;      // wave 0 sets after publishing the aggregate of the tile it walked
  uint32_t cdone;    // copy waves that finished their copy (monotonic)
  uint32_t staged;   // late-walk schedule: loader waves whose DMA of a tile has landed (monotonic)
  uint8_t cmk[kPipeThreads / kWave][kWave];   // per copy wave: first-chunk marks of the dense key-tail copy
  // VERIFY: slicing-by-4 CRC-32C tables, per-block XOR accumulators (by tile parity), and
  // the count of CRC waves done (monotonic; the last of a tile finalises it)
  uint32_t crcT[P::VERIFY ? 4 : 1][P::VERIFY ? 256 : 1];
  uint32_t cacc[2][P::VERIFY ? P::MAXBLK : 1];
  uint32_t cst[2][P::VERIFY ? P::MAXBLK : 1];   // stored checksums (copy wave 0), by tile parity
  uint32_t cfr[2][P::VERIFY ? P::MAXBLK : 1];   // ... present (framed batch, offset >= 4)
  uint32_t shK[P::VERIFY ? 64 : 1];              // window shifts x^(8 W l), lane l
  uint32_t shX[P::VERIFY ? 32 : 1];              // round shifts x^(8 W 64 r)
  uint32_t crcdone;
};

__device__ __forceinline__ void raw_barrier() {
  // LDS traffic complete, then the hardware barrier; outstanding global stores and
  // LDS-DMA stay in flight (a __syncthreads() would wait vmcnt(0) here)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int D>
__device__ __forceinline__ uint32_t row_shr_keep(uint32_t x) {  // lane k <- lane k-D of its row, else itself
  return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x110 + D, 0xf, 0xf, false);
}
template <int D>
__device__ __forceinline__ uint32_t row_shr_zero(uint32_t x) {  // lane k <- lane k-D of its row, else 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x110 + D, 0xf, 0xf, false);
}

// exclusive prefix sum inside each 16-lane row
__device__ __forceinline__ uint32_t row_excl_scan(uint32_t x) {
  uint32_t y = x;
  y += row_shr_zero<1>(y);
  y += row_shr_zero<2>(y);
  y += row_shr_zero<4>(y);
  y += row_shr_zero<8>(y);
  return y - x;
}

// dword i of the mask of bytes b >= t of a 16-byte plane
__device__ __forceinline__ uint32_t keep_mask(int t, int i) {
  int lo = t - 4 * i;
  lo = lo < 0 ? 0 : lo;
  return lo >= 4 ? 0u : (0xFFFFFFFFu << (8 * lo));
}

// One Hillis-Steele step of the key-prefix scan.  State of a run of entries = (m, W):
// m = smallest `shared` in the run, W = key bytes of the run's last entry at positions
// >= m (this plane).  compose(L, R) = (min(mL, mR), bytes >= mR from R, the rest from L):
// key.truncate(shared) + key.extend(suffix) applied entry after entry.
template <int D>
__device__ __forceinline__ void key_scan_step(uint32_t& m, uint4& W, uint32_t q0) {
  const uint32_t mL = row_shr_keep<D>(m);
  uint4 L;
  L.x = row_shr_keep<D>(W.x);
  L.y = row_shr_keep<D>(W.y);
  L.z = row_shr_keep<D>(W.z);
  L.w = row_shr_keep<D>(W.w);
  const int t = (int)m - (int)q0;
  uint32_t k;
  k = keep_mask(t, 0); W.x = (W.x & k) | (L.x & ~k);
  k = keep_mask(t, 1); W.y = (W.y & k) | (L.y & ~k);
  k = keep_mask(t, 2); W.z = (W.z & k) | (L.z & ~k);
  k = keep_mask(t, 3); W.w = (W.w & k) | (L.w & ~k);
  m = mL < m ? mL : m;
}

// Walk of restart interval [s, e) of a staged block.  The loop-carried chain is only
// p -> LDS header read -> p' (about a dozen VALU ops per entry); every validity check is
// folded into accumulators that are tested once at the end:
//  - any header byte >= 128 (multi-byte varint)      -> `orf`
//  - shared > previous key length (first: 0)          -> `badsh`
//  - an entry running past R (p is monotonic, so the walk then ends with p != e)
//  - more than 16 entries                             -> loop bound, p != e
// Reads past R stay inside the LDS allocation (at most 513 bytes past the last header)
// and are never used when the walk is rejected; the caller then runs the exact
// walk_careful_pos.  Preconditions as walk_interval (regular blocks).
__device__ __forceinline__ bool walk_pos(const uint8_t* stage, uint16_t* pos, uint32_t bo, uint32_t s, uint32_t e,
                                         uint32_t slot0, uint32_t& cnt, uint32_t& kb, uint32_t& vb) {
  cnt = kb = vb = 0;
  if (!(s < e)) return false;
  uint32_t p = s, prevlen = 0, orf = 0, badsh = 0, ssh = 0, svl = 0, c = 0;
  const uint32_t* st32 = reinterpret_cast<const uint32_t*>(stage);
  uint32_t ad = bo + p;
  MTBLX_LCHK(st32 + (ad >> 2), 8);
  uint32_t w0 = st32[ad >> 2], w1 = st32[(ad >> 2) + 1];
  do {
    const uint32_t hw = __builtin_amdgcn_alignbit(w1, w0, (ad & 3u) * 8u);
    const uint32_t sh = hw & 0xffu, ns = (hw >> 8) & 0xffu, vl = (hw >> 16) & 0xffu;
    const uint32_t np = p + 3u + ns + vl;
    ad = bo + np;
    MTBLX_LCHK(st32 + (ad >> 2), 8);
    w0 = st32[ad >> 2];
    w1 = st32[(ad >> 2) + 1];
    pos[slot0 + c] = (uint16_t)p;
    orf |= hw;
    badsh |= (uint32_t)(sh > prevlen);
    prevlen = sh + ns;
    ssh += sh;
    svl += vl;
    c += 1;
    p = np;
  } while (p < e && c < (uint32_t)kP2Spi);
  cnt = c;
  vb = svl;
  kb = ssh + (p - s) - 3u * c - svl;   // sum(shared + non_shared): p - s = sum(3 + ns + vl)
  return p == e && (orf & 0x808080u) == 0u && badsh == 0u;
}

// Walk of [s, e) that also accepts 2-byte varints (values < 16384: cfg3's long key suffixes).
// Same deferred-check structure as walk_pos; an 8-byte window per header; rejects (-> the
// exact walk_careful_pos) any varint of 3+ bytes, shared > previous key length, an overshoot
// or more than 16 entries.  Reads past R land inside the LDS allocation or return 0 and are
// never used when the walk is rejected (p is monotonic; the result requires p == e <= R).
#ifndef MTBLX_WALK2D   // 1: the instruction-lean walk below (+1.7 % on cfg3's decode, round 5); 0: round 4's
#define MTBLX_WALK2D 1
#endif
__device__ __forceinline__ bool walk_pos2(const uint8_t* stage, uint16_t* pos, uint32_t bo, uint32_t s, uint32_t e,
                                          uint32_t slot0, uint32_t& cnt, uint32_t& kb, uint32_t& vb, bool& all1) {
  cnt = kb = vb = 0;
  all1 = false;
  if (!(s < e)) return false;
#if MTBLX_WALK2D
  // fewer instructions per entry on the serial chain: each varint's start from its predecessor's
  // continuation bit as a 64-bit shift of the window, its value by mask-and-merge, and the checks
  // folded into accumulators -- bit 15 of y & (y << 8) (the first two bytes of a varint both
  // continue: 3+ bytes), the sign of prevlen - shared (shared > the previous key's length)
  {
    uint32_t p = s, prevlen = 0, chk = 0, dsh = 0, any2 = 0, kbs = 0, vbs = 0, c = 0;
    const uint32_t* st32 = reinterpret_cast<const uint32_t*>(stage);
    do {
      const uint32_t ad = bo + p, q = ad >> 2, sft = (ad & 3u) * 8u;
      MTBLX_LCHK(st32 + q, 12);
      const uint32_t w0 = st32[q], w1 = st32[q + 1], w2 = st32[q + 2];
      const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, sft), hi = __builtin_amdgcn_alignbit(w2, w1, sft);
      const uint64_t x = ((uint64_t)hi << 32) | lo;
      const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int)lo, 7, 1);   // 0 or ~0: 2-byte varint
      const uint32_t s1 = 8u + (m0 & 8u);                                     // bits to varint 1
      const uint32_t y1 = (uint32_t)(x >> s1);
      const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int)y1, 7, 1);
      const uint32_t s2 = s1 + 8u + (m1 & 8u);
      const uint32_t y2 = (uint32_t)(x >> s2);
      const uint32_t m2 = (uint32_t)__builtin_amdgcn_sbfe((int)y2, 7, 1);
      const uint32_t hl = (s2 >> 3) + 1u + (m2 & 1u);
      const uint32_t f0 = (lo & 0x7fu) | ((lo >> 1) & 0x3f80u & m0);
      const uint32_t f1 = (y1 & 0x7fu) | ((y1 >> 1) & 0x3f80u & m1);
      const uint32_t f2 = (y2 & 0x7fu) | ((y2 >> 1) & 0x3f80u & m2);
      chk |= (lo & (lo << 8)) | (y1 & (y1 << 8)) | (y2 & (y2 << 8));
      any2 |= m0 | m1 | m2;
      pos[slot0 + c] = (uint16_t)p;
      dsh |= prevlen - f0;
      prevlen = f0 + f1;
      kbs += prevlen;
      vbs += f2;
      c += 1;
      p += hl + f1 + f2;
    } while (p < e && c < (uint32_t)kP2Spi);
    cnt = c;
    vb = vbs;
    kb = kbs;
    all1 = any2 == 0u;   // every header 1-byte varints: walk_pos would have accepted it
    return p == e && (chk & 0x8000u) == 0u && (dsh >> 31) == 0u;
  }
#endif
  uint32_t p = s, prevlen = 0, bad = 0, ssh = 0, svl = 0, shl = 0, c = 0;
  const uint32_t* st32 = reinterpret_cast<const uint32_t*>(stage);
  do {
    const uint32_t ad = bo + p, q = ad >> 2, sft = (ad & 3u) * 8u;
    MTBLX_LCHK(st32 + q, 12);
    const uint32_t w0 = st32[q], w1 = st32[q + 1], w2 = st32[q + 2];
    uint64_t x = (uint64_t)__builtin_amdgcn_alignbit(w1, w0, sft) |
                 ((uint64_t)__builtin_amdgcn_alignbit(w2, w1, sft) << 32);
    uint32_t f[3], hl = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint32_t b0 = (uint32_t)x & 0xffu, b1 = (uint32_t)(x >> 8) & 0xffu, two = b0 >> 7;
      f[k] = (b0 & 0x7fu) | (two ? (b1 & 0x7fu) << 7 : 0u);
      bad |= two & (b1 >> 7);                    // a 3+ byte varint
      x >>= 8u * (1u + two);
      hl += 1u + two;
    }
    pos[slot0 + c] = (uint16_t)p;
    bad |= (uint32_t)(f[0] > prevlen);
    prevlen = f[0] + f[1];
    ssh += f[0];
    svl += f[2];
    shl += hl;
    c += 1;
    p += hl + f[1] + f[2];
  } while (p < e && c < (uint32_t)kP2Spi);
  cnt = c;
  vb = svl;
  kb = ssh + (p - s) - shl - svl;   // sum(shared + non_shared): p - s = sum(header + ns + vl)
  all1 = shl == 3u * c;             // every header 1-byte varints: walk_pos would have accepted it
  return p == e && bad == 0u;
}

// exact walk (multi-byte varint headers allowed) recording header offsets; same checks as
// walk_interval
__device__ __forceinline__ bool walk_careful_pos(const uint8_t* stage, uint16_t* pos, uint32_t bo, uint32_t L, uint32_t R,
                                                 uint32_t s, uint32_t e, uint32_t slot0, uint32_t& cnt, uint32_t& kb,
                                                 uint32_t& vb) {
  cnt = kb = vb = 0;
  if (!(s < e && e <= R)) return false;
  uint32_t p = s, prevlen = 0;
  while (p < e) {
    if (cnt >= (uint32_t)kP2Spi) return false;
    const uint32_t ad = bo + p;
    const uint32_t hw = lds_rd32(stage, ad);
    uint32_t sh = hw & 0xffu, ns = (hw >> 8) & 0xffu, vl = (hw >> 16) & 0xffu, h = 3;
    if ((hw & 0x808080u) != 0u) {
      if (R - p < 3u) return false;
      const uint4 W = lds_win16(stage, ad);
      const uint32_t l0 = dec32(W, 0, L - p, sh);
      if (l0 == 0) return false;
      const uint32_t l1 = dec32(W, l0, L - p - l0, ns);
      if (l1 == 0) return false;
      const uint32_t l2 = dec32(W, l0 + l1, L - p - l0 - l1, vl);
      if (l2 == 0) return false;
      h = l0 + l1 + l2;
      if (p + h > R) return false;
      if ((sh | ns | vl) > 0xFFFFu) return false;
    }
    if (R - p < h + ns + vl) return false;
    if (sh > prevlen) return false;
    pos[slot0 + cnt] = (uint16_t)p;
    const uint32_t klen = sh + ns;
    cnt += 1;
    kb += klen;
    vb += vl;
    prevlen = klen;
    p += h + ns + vl;
  }
  return p == e && (prevlen <= 0xFFFFu);
}

// wave 0: LDS-DMA of tile t into B (contiguous range, or one 16 B aligned slot per block).
// (off_l, len_l) = directory entry of block `lane` of the tile (lanes < nb).
template <class P>
// Pieces (1 KiB wave-instructions) m in [mlo, mhi) with m = part (mod LOADW) of the
// contiguous layout are issued; the per-block slot layout is issued whole when mlo == 0.
__device__ __forceinline__ void pipe_dma(PipeBuf<P>& B, const TileArgs& a, uint32_t t, uint64_t off_l, uint32_t len_l,
                                         int lane, uint32_t part, uint32_t mlo = 0, uint32_t mhi = 0xFFFFFFFFu) {
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) const void g_void;
  uint32_t b0, nb;
  tile_span(a, t, b0, nb);
  const uint64_t base = reinterpret_cast<uintptr_t>(a.data);
  const uint64_t s = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(off_l >> 32), 0) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)off_l, 0);
  const uint64_t end_l = off_l + len_l;
  const uint64_t e = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(end_l >> 32), (int)nb - 1) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)end_l, (int)nb - 1);
  uint64_t r0 = ((base + s) & ~15ull) - base;
  if (base + s < 16 || ((base + s) & ~15ull) < base) r0 = 0;
  // one contiguous range only if EVERY block of the tile lies inside [first start, last end):
  // the directory is the caller's (a corrupt index can point a block anywhere, before its
  // predecessor or into it); lanes >= nb repeat the last block
  const bool inside = off_l >= s && end_l <= e;
  const bool contig = e > s && e - r0 + 48 <= (uint64_t)P::TB && __ballot(!inside) == 0ull;
  if (contig) {
    // range byte x at stage offset 16 + x; wave-instruction m writes chunks [64m, 64m + 64)
    const uint32_t nch = (uint32_t)((e - r0 + 15) >> 4);
    // chunks [0, nfull) are 16-byte aligned and inside the buffer: whole pieces of them take a
    // lean loop (address add + DMA); the tail piece goes lane by lane
    const bool al = ((base + r0) & 15ull) == 0;
    const uint64_t room = a.data_len > r0 ? (a.data_len - r0) / 16u : 0u;
    const uint32_t nfull = al ? (uint32_t)min<uint64_t>(nch, room) : 0u;
    const uint32_t mfull = min(nfull / kWave, mhi);   // pieces made only of such chunks
    uint32_t m = part + ((mlo + P::LOADW - 1 - part) / P::LOADW) * P::LOADW;   // first piece >= mlo
    if (mlo <= part) m = part;
    const uint8_t* gp = a.data + r0 + 16ull * ((uint64_t)m * kWave + (uint32_t)lane);
    for (; m < mfull; m += P::LOADW, gp += 16 * kWave * P::LOADW)
      MTBLX_CHK(gp, 16), MTBLX_LCHK(B.stage + 16 + 1024 * m, 1024), __builtin_amdgcn_global_load_lds((g_void*)gp, (lds_void*)(B.stage + 16 + 1024 * m), 16, 0, MTBLX_NT_LOADS ? MTBLX_DMA_AUX : 0);
    for (; m * kWave < nch && m < mhi; m += P::LOADW) {
      const uint32_t c = m * kWave + lane;
      const uint64_t go = r0 + 16ull * c;
      if (c < nfull)
        MTBLX_CHK(a.data + go, 16), MTBLX_LCHK(B.stage + 16 + 1024 * m, 1024), __builtin_amdgcn_global_load_lds((g_void*)(a.data + go), (lds_void*)(B.stage + 16 + 1024 * m), 16, 0, MTBLX_NT_LOADS ? MTBLX_DMA_AUX : 0);
      else if (c < nch)
        *reinterpret_cast<uint4*>(B.stage + 16 + 16 * c) = load_chunk(a, go);
    }
    if (part == 0 && lane < (int)nb) {
      B.boff[lane] = off_l + len_l > a.data_len ? kOutOfBounds : (uint32_t)(16 + off_l - r0);
      B.blen[lane] = len_l;
    }
  } else if (mlo == 0) {
    // per-block slots of a.slot bytes (blocks not adjacent in the buffer)
    for (uint32_t j = 0; j < nb; ++j) {
      const uint64_t off = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(off_l >> 32), (int)j) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)off_l, (int)j);
      const uint32_t L = (uint32_t)__builtin_amdgcn_readlane((int)len_l, (int)j);
      const uint32_t so = 16u + j * a.slot;
      uint32_t bo = kNotStaged;
      if (off + L > a.data_len) {
        bo = kOutOfBounds;
      } else if (L + 15u <= a.slot && so + a.slot + 32u <= (uint32_t)P::TB) {
        uint64_t a0 = ((base + off) & ~15ull) - base;
        if (base + off < 16 || ((base + off) & ~15ull) < base) a0 = off;  // unaligned data base: not reached
        const uint32_t delta = (uint32_t)(off - a0);
        const uint32_t nch = (delta + L + 15u) >> 4;
        for (uint32_t m = part; m * kWave < nch; m += P::LOADW) {
          const uint32_t c = m * kWave + lane;
          const uint64_t go = a0 + 16ull * c;
          if (c < nch) {
            if (go + 16 <= a.data_len && ((base + go) & 15ull) == 0)
              MTBLX_CHK(a.data + go, 16), MTBLX_LCHK(B.stage + so + 1024 * m, 1024), __builtin_amdgcn_global_load_lds((g_void*)(a.data + go), (lds_void*)(B.stage + so + 1024 * m), 16, 0,
                                               MTBLX_NT_LOADS ? MTBLX_DMA_AUX : 0);
            else
              *reinterpret_cast<uint4*>(B.stage + so + 16 * c) = load_chunk(a, go);
          }
        }
        bo = so + delta;
      }
      if (part == 0 && lane == 0) { B.boff[j] = bo; B.blen[j] = L; }
    }
  }
  if (part == 0 && lane == 0) { B.nb = nb; B.b0 = b0; }
}

// wave 0: trailers, walk (header offsets into slots), irregular counts, interval scan,
// publish A(t), then the block / interval bases the copy and the look-back read.
// Cross-lane traffic uses readlane / DPP / bpermute (no LDS round trips before the walk).
template <class P>
// wmode (wave 0's, carried across its tiles): 1 = walk with walk_pos2 first.  A wave walks its
// intervals in lockstep, so one interval with a 2-byte varint (cfg3: 8 % of keys have a suffix
// of >= 128 bytes, ~3/4 of intervals one such entry) made every lane walk twice (walk_pos, then
// walk_pos2); the previous tile decides which walk goes first.
__device__ __forceinline__ void pipe_walk(PipeBuf<P>& B, const TileArgs& a, uint32_t t, int lane, Stamps& ST,
                                          uint32_t& wmode) {
  uint32_t b0, nb;
  tile_span(a, t, b0, nb);
  // trailers (Block::init, src/block.rs:16-49): lane = block
  uint32_t n = 0, R = 0, ok = 0, L = 0, bo = kNotStaged;
  if (lane < (int)nb) {
    L = B.blen[lane];
    bo = B.boff[lane];
    if (bo < kOutOfBounds && L >= 8) {
      n = lds_rd32(B.stage, bo + L - 4);
      if (n != 0 && (uint64_t)(n + 1ull) * 4ull <= L) { R = L - 4u * (n + 1u); ok = 1; }
    }
  }
  uint32_t incl = wave_incl_scan(ok ? n : 0u);
  if (ok && incl > (uint32_t)P::MAXINT) ok = 0;
  n = ok ? n : 0;
  incl = wave_incl_scan(n);                   // lane b: intervals of blocks 0..b
  const uint32_t bint0 = incl - n;
  const uint32_t nint = (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)nb - 1);
  // interval f = lane: its block j and that block's fields
  uint32_t j = 0;
  for (uint32_t b = 0; b + 1 < nb; ++b) j += ((uint32_t)__builtin_amdgcn_readlane((int)incl, (int)b) <= (uint32_t)lane);
  const int js = (int)j;
  const uint32_t jbo = (uint32_t)__shfl((int)bo, js, kWave), jR = (uint32_t)__shfl((int)R, js, kWave);
  const uint32_t jn = (uint32_t)__shfl((int)n, js, kWave), jb0 = (uint32_t)__shfl((int)bint0, js, kWave);
  const uint32_t jL = (uint32_t)__shfl((int)L, js, kWave);
  ST.hit(9);
  const bool fl = (uint32_t)lane < nint;
  uint32_t cnt = 0, kb = 0, vb = 0;
  bool wok = false, need2 = false;
  if (fl) {
    const uint32_t i = (uint32_t)lane - jb0;
    const uint32_t s = lds_rd32(B.stage, jbo + jR + 4u * i);
    const uint32_t e = (i + 1 < jn) ? lds_rd32(B.stage, jbo + jR + 4u * (i + 1)) : jR;
    ST.hit(10);
    const uint32_t slot0 = (uint32_t)lane * kP2Spi;
    bool all1 = true;
    // (PipeLarge only: the fused-verify kernels are at their VGPR cap, and PipeSmall's cfg2
    // headers are all 1-byte varints -- the extra code cost its launch 1 %)
    constexpr bool kAdaptive = P::NBUF == 2 && !P::VERIFY;
    if (!kAdaptive || wmode == 0u) {
      wok = e <= jR && walk_pos(B.stage, B.pos, jbo, s, e, slot0, cnt, kb, vb);
      if (!wok) {
        wok = e <= jR && walk_pos2(B.stage, B.pos, jbo, s, e, slot0, cnt, kb, vb, all1);
        all1 = false;   // walk_pos failed here
      }
    } else {
      wok = e <= jR && walk_pos2(B.stage, B.pos, jbo, s, e, slot0, cnt, kb, vb, all1);
      all1 = all1 || !wok;   // a rejected interval goes to the careful walk either way
    }
    need2 = !all1;
    if (!wok) wok = walk_careful_pos(B.stage, B.pos, jbo, jL, jR, s, e, slot0, cnt, kb, vb);
    B.iraw[lane] = (uint8_t)(cnt < 255u ? cnt : 255u);
    B.iblk[lane] = (uint8_t)j;
  }
  ST.hit(2);
  if constexpr (P::NBUF == 2 && !P::VERIFY) wmode = __ballot(need2) != 0ull ? 1u : 0u;
  // a block with a rejected interval is irregular
  const uint64_t failm = __ballot(fl && !wok);
  {
    const uint64_t hi = incl >= 64u ? ~0ull : ((1ull << incl) - 1ull);
    const uint64_t lo = (1ull << bint0) - 1ull;
    if (ok && (failm & hi & ~lo) != 0ull) ok = 0;
  }
  const bool jok = __shfl((int)ok, js, kWave) != 0;
  // irregular blocks: exact serial count (generic path, lane per block)
  uint32_t gc = 0, gk = 0, gv = 0;
  int32_t gst = MTBLX_ST_OK;
  if (lane < (int)nb && !ok) {
    if (bo == kNotStaged) MTBLX_CHK(a.blk_off + b0 + lane, 8);
    const uint8_t* d = (bo != kNotStaged) ? (B.stage + bo) : (a.data + a.blk_off[b0 + lane]);
    const GenOut o = bo == kOutOfBounds ? GenOut{0, 0, 0, MTBLX_ST_CORRUPT}
                                        : generic_block<false>(d, L, nullptr, nullptr, nullptr, nullptr);
    gc = o.nrec; gk = (uint32_t)o.kb; gv = (uint32_t)o.vb; gst = o.st;
  }
  const uint32_t gwr = ok || gen_writable(bo, gst);
  // interval scan over regular blocks (one interval per lane)
  const bool reg = fl && jok;
  const uint32_t c = reg ? cnt : 0u, k = reg ? kb : 0u, v = reg ? vb : 0u;
  const uint32_t ic = wave_incl_scan(c), ik = wave_incl_scan(k), iv = wave_incl_scan(v);
  // tile totals -> publish A(t) first (other workgroups' look-back waits on it)
  const uint32_t tr = (uint32_t)__builtin_amdgcn_readlane((int)ic, 63) + wave_sum32(gc);
  const uint32_t tk = (uint32_t)__builtin_amdgcn_readlane((int)ik, 63) + wave_sum32(gk);
  const uint32_t tv = (uint32_t)__builtin_amdgcn_readlane((int)iv, 63) + wave_sum32(gv);
  if (lane == 0) {
    if (t == 0) pipe_zero_flags(a);
    lb_publish(a, t, tr, tk, tv);
    B.ttot[0] = tr; B.ttot[1] = tk; B.ttot[2] = tv;
    B.nint = nint;
  }
  // block totals (regular: differences of the interval scan) and tile-relative block bases.
  if (nb == 1) {
    // one block per tile (64 KiB blocks): every cross-lane value is lane 0's or the last
    // interval's -- readlanes instead of permutes, no scans
    const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)incl, 0);
    const uint32_t tc = n0 ? (uint32_t)__builtin_amdgcn_readlane((int)ic, (int)n0 - 1) : 0u;
    const uint32_t tkk = n0 ? (uint32_t)__builtin_amdgcn_readlane((int)ik, (int)n0 - 1) : 0u;
    const uint32_t tvv = n0 ? (uint32_t)__builtin_amdgcn_readlane((int)iv, (int)n0 - 1) : 0u;
    if (lane == 0) {
      B.bok[0] = ok; B.bwr[0] = gwr; B.bst[0] = ok ? MTBLX_ST_OK : gst;
      B.bcnt[0] = ok ? tc : gc; B.bkb[0] = ok ? tkk : gk; B.bvb[0] = ok ? tvv : gv;
      B.brb[0] = 0; B.bkbb[0] = 0; B.bvbb[0] = 0;
    }
    if (fl) {
      B.icnt[lane] = ic - c;
      B.ikb[lane] = ik - k;
      B.ivb[lane] = iv - v;
    }
    return;
  }
  // Every lane executes the permutes (a disabled source lane reads as 0).
  const int ea_l = bint0 ? (int)bint0 - 1 : 0, eb_l = incl ? (int)incl - 1 : 0;
  const uint32_t ea0 = (uint32_t)__shfl((int)ic, ea_l, kWave), eb0 = (uint32_t)__shfl((int)ic, eb_l, kWave);
  const uint32_t ka0 = (uint32_t)__shfl((int)ik, ea_l, kWave), kb0 = (uint32_t)__shfl((int)ik, eb_l, kWave);
  const uint32_t va0 = (uint32_t)__shfl((int)iv, ea_l, kWave), vb0 = (uint32_t)__shfl((int)iv, eb_l, kWave);
  uint32_t bc = 0, bk = 0, bv = 0;
  if (lane < (int)nb) {
    if (ok) {
      bc = (incl ? eb0 : 0u) - (bint0 ? ea0 : 0u);
      bk = (incl ? kb0 : 0u) - (bint0 ? ka0 : 0u);
      bv = (incl ? vb0 : 0u) - (bint0 ? va0 : 0u);
    } else {
      bc = gc; bk = gk; bv = gv;
    }
  }
  const uint32_t jc = wave_incl_scan(bc), jk = wave_incl_scan(bk), jv = wave_incl_scan(bv);
  const uint32_t brb = jc - bc, bkbb = jk - bk, bvbb = jv - bv;
  if (lane < (int)nb) {
    B.bok[lane] = ok; B.bwr[lane] = gwr; B.bst[lane] = ok ? MTBLX_ST_OK : gst;
    B.bcnt[lane] = bc; B.bkb[lane] = bk; B.bvb[lane] = bv;
    B.brb[lane] = brb; B.bkbb[lane] = bkbb; B.bvbb[lane] = bvbb;
  }
  // tile-relative interval bases (record index, key byte, value byte)
  const uint32_t jea = (uint32_t)__shfl((int)(bint0 ? ea0 : 0u), js, kWave);
  const uint32_t jka = (uint32_t)__shfl((int)(bint0 ? ka0 : 0u), js, kWave);
  const uint32_t jva = (uint32_t)__shfl((int)(bint0 ? va0 : 0u), js, kWave);
  const uint32_t jrb = (uint32_t)__shfl((int)brb, js, kWave), jkb = (uint32_t)__shfl((int)bkbb, js, kWave),
                 jvb = (uint32_t)__shfl((int)bvbb, js, kWave);
  if (fl) {
    B.icnt[lane] = jrb + (ic - c) - jea;
    B.ikb[lane] = jkb + (ik - k) - jka;
    B.ivb[lane] = jvb + (iv - v) - jva;
  }
}

// wave 1: issue the look-back loads of tile t (aggregates of tiles t-G+1 .. t-1) one
// iteration before they are consumed; they complete behind the copy phase.
__device__ __forceinline__ void pipe_lookback_issue(const TileArgs& a, uint32_t t, uint32_t G,
                                                    uint64_t lbv[kMaxLookbackLoads], int lane) {
  const int64_t lo = (t >= G) ? (int64_t)t - G + 1 : 0;
#pragma unroll
  for (int m = 0; m < kMaxLookbackLoads; ++m) {
    const int64_t i = (int64_t)t - 1 - lane - (int64_t)m * kWave;
    lbv[m] = (i >= lo) ? __hip_atomic_load(lb_slot(a, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kReady;
  }
}

// wave 1: re-poll the words of tile t that were not ready when loaded, until all are or
// the copy waves have finished this iteration (the barrier must not wait for laggards;
// what is still missing is polled again when the tile is consumed).
__device__ __forceinline__ void pipe_lookback_poll(const TileArgs& a, uint32_t t, uint32_t G,
                                                   uint64_t lbv[kMaxLookbackLoads], int lane, const uint32_t* cdone,
                                                   uint32_t want) {
  const int64_t lo = (t >= G) ? (int64_t)t - G + 1 : 0;
  for (uint32_t spin = 0; spin < (1u << 22); ++spin) {
    bool pend = false;
#pragma unroll
    for (int m = 0; m < kMaxLookbackLoads; ++m) {
      const int64_t i = (int64_t)t - 1 - lane - (int64_t)m * kWave;
      pend |= (i >= lo) && !(lbv[m] & kReady);
    }
    if (__ballot(pend) == 0ull) return;
    if (__hip_atomic_load(cdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= want) return;
    __builtin_amdgcn_s_sleep(2);
#pragma unroll
    for (int m = 0; m < kMaxLookbackLoads; ++m) {
      const int64_t i = (int64_t)t - 1 - lane - (int64_t)m * kWave;
      if (i >= lo && !(lbv[m] & kReady)) lbv[m] = __hip_atomic_load(lb_slot(a, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// wave 1: finish the look-back of tile t (re-polling words that were not ready yet),
// per-block outputs.  tinc = inclusive prefix of this workgroup's previous tile.
template <class P>
__device__ __forceinline__ void pipe_lookback(PipeBuf<P>& B, const TileArgs& a, uint32_t t, uint32_t G, uint64_t tinc[3],
                                              uint64_t lbv[kMaxLookbackLoads], int lane, uint32_t* ready,
                                              uint32_t rv) {
  const uint32_t nb = B.nb, b0 = B.b0;
  const int64_t lo = (t >= G) ? (int64_t)t - G + 1 : 0;
  uint64_t sr = 0, sk = 0, sv = 0;
  bool timeout = false;
#pragma unroll
  for (int m = 0; m < kMaxLookbackLoads; ++m) {
    const int64_t i = (int64_t)t - 1 - lane - (int64_t)m * kWave;
    uint64_t w = lbv[m];
    WaitBound wb;
    while (!(w & kReady)) {
      __builtin_amdgcn_s_sleep(2);
      w = __hip_atomic_load(lb_slot(a, i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (wb.expired(a.wait_ticks)) { timeout = true; w = kReady; }
    }
    if (i < lo) continue;
    lb_take(a, (uint64_t)i, w, sr, sk, sv);
  }
  if (timeout) ws_timeout(a);
  sr = lb_wave_sum(sr);
  sv = lb_wave_sum(sv);
  sk = lb_wave_sum(sk);
  const uint64_t pr = tinc[0] + sr, pk = tinc[1] + sk, pv = tinc[2] + sv;
  tinc[0] = pr + B.ttot[0];
  tinc[1] = pk + B.ttot[1];
  tinc[2] = pv + B.ttot[2];
  if (lane == 0) {
    B.tpre[0] = pr; B.tpre[1] = pk; B.tpre[2] = pv;
    if (t == a.ntiles - 1) MTBLX_CHK(a.totals, 24);
    if (t == a.ntiles - 1) { a.totals[0] = tinc[0]; a.totals[1] = tinc[1]; a.totals[2] = tinc[2]; }
  }
  // the copy waves need only tpre, and bwr where a block overflows the caller's buffers: when
  // the whole tile fits, release them before the per-block outputs are written
  const bool fits = !a.write || (fits_at(pr, B.ttot[0], a.rec_cap) && fits_at(pk, B.ttot[1], a.keys_cap) &&
                                 fits_at(pv, B.ttot[2], a.vals_cap));
  if (fits) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(ready, rv, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (lane < (int)nb) {
    const uint32_t j = lane, b = b0 + j;
    const uint64_t rb = pr + B.brb[j], kb = pk + B.bkbb[j], vb = pv + B.bvbb[j];
    MTBLX_CHK(a.nrec + b, 4);
    MTBLX_CHK(a.rec_base + b, 8);
    MTBLX_CHK(a.key_base + b, 8);
    MTBLX_CHK(a.val_base + b, 8);
    MTBLX_CHK(a.status + b, 4);
    a.nrec[b] = B.bcnt[j];
    a.rec_base[b] = rb;
    a.key_base[b] = kb;
    a.val_base[b] = vb;
    int32_t st = B.bst[j];
    if (a.write && !(fits_at(rb, B.bcnt[j], a.rec_cap) && fits_at(kb, B.bkb[j], a.keys_cap) &&
                     fits_at(vb, B.bvb[j], a.vals_cap))) {
      st = MTBLX_ST_OVERFLOW;
      B.bwr[j] = 0;
      ws_flag(a, 1ull);
    }
    a.status[b] = st;
  }
  if (!fits) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(ready, rv, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// Copy waves: record pass + copy of one tile.  Copy wave cw owns 16-lane rows
// 4 cw .. 4 cw + 3 of each round; row = restart interval, lane k of the row = entry k.
// Each round is split into a prepare part (LDS + DPP only: headers, row scans, first key
// plane) and an emit part (global stores); the first round is prepared before the
// look-back of the tile is ready, overlapping the wait.
struct CopyRow {
  uint32_t f, j, k, bo, sh, ns, vl, klen, ks, vs, sp, m0;
  uint4 W0;          // key bytes [0, 16) of the entry (valid for live entries)
  bool fv, live;
};

template <class P>
__device__ __forceinline__ CopyRow copy_prepare(const PipeBuf<P>& B, uint32_t fb, int lane) {
  CopyRow r;
  const uint32_t nint = B.nint;
  r.k = lane & 15;
  r.f = fb + (lane >> 4);
  r.fv = r.f < nint;
  r.j = r.fv ? B.iblk[r.f] : 0u;
  r.live = r.fv && r.k < B.iraw[r.f] && B.bok[r.j];
  r.bo = B.boff[r.j];
  const uint32_t p = r.live ? B.pos[r.f * kP2Spi + r.k] : 0u;
  uint32_t sh = 0, ns = 0, vl = 0, h = 3;
  if (r.live) {  // decode_entry (src/block.rs:216-238) at a header the walk validated
    const uint32_t hw = lds_rd32(B.stage, r.bo + p);
    sh = hw & 0xffu; ns = (hw >> 8) & 0xffu; vl = (hw >> 16) & 0xffu;
    if ((hw & 0x808080u) != 0u) {
      const uint4 W = lds_win16(B.stage, r.bo + p);
      const uint32_t l0 = dec32(W, 0, 16, sh);
      const uint32_t l1 = dec32(W, l0, 16, ns);
      const uint32_t l2 = dec32(W, l0 + l1, 16, vl);
      h = l0 + l1 + l2;
    }
  }
  r.sh = sh; r.ns = ns; r.vl = vl;
  r.klen = sh + ns;
  const uint32_t kx = row_excl_scan(r.klen), vx = row_excl_scan(vl);
  r.ks = (r.fv ? B.ikb[r.f] : 0u) + kx;
  r.vs = (r.fv ? B.ivb[r.f] : 0u) + vx;
  r.sp = r.bo + p + h;   // stage offset of the key suffix
#ifndef MTBLX_ABL_NOKEY
  // first key plane (bytes 0..15): row scan of the truncate-then-append operator
  const bool own = r.live && sh < 16u && r.klen > 0u;
  uint4 W = own ? lds_win16(B.stage, r.sp - sh) : make_uint4(0, 0, 0, 0);
  uint32_t m = sh;
  key_scan_step<1>(m, W, 0);
  key_scan_step<2>(m, W, 0);
  key_scan_step<4>(m, W, 0);
  key_scan_step<8>(m, W, 0);
  r.W0 = W;
  r.m0 = m;
#endif
  return r;
}

// Key bytes at positions >= 16 when no live entry of the wave inherits one there: each such
// byte is the entry's own suffix (key.truncate(shared) + key.extend(suffix), src/block.rs:134-135),
// so the wave's key tails form one dense list of 16-byte chunks and pass c0 gives chunk c0 + l
// to lane l.  The chunk's entry is the last one whose first chunk is <= it: entries mark their
// first chunk in the wave's LDS row (by lane id; 0 = no mark, lane 0 never starts past chunk 0)
// and a prefix max over the row, seeded with the entry holding chunk c0 (a ballot), fills the rest.  That is
// ceil(sum of chunks / 64) passes instead of one per 16-byte plane of the wave's longest key
// (cfg3's Zipf keys: ~2 instead of ~15).  src / dst = stage offset / key-region offset of the
// entry's byte 16.
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
  uint32_t y;
  y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false); x = x > y ? x : y;  // row_shr:1
  y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false); x = x > y ? x : y;  // row_shr:2
  y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false); x = x > y ? x : y;  // row_shr:4
  y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false); x = x > y ? x : y;  // row_shr:8
  y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false); x = x > y ? x : y;  // row_bcast:15
  y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false); x = x > y ? x : y;  // row_bcast:31
  return x;
}

__device__ __forceinline__ void key_tails_dense(uint8_t* kb, const uint8_t* stage, uint8_t* mk, bool tl, uint32_t klen,
                                                uint32_t src, uint32_t dst, int lane) {
  const uint32_t nc = tl ? (klen - 1u) >> 4 : 0u;   // ceil((klen - 16) / 16)
  const uint32_t ci = wave_incl_scan(nc);
  const uint32_t cx = ci - nc;
  const uint32_t C = (uint32_t)__builtin_amdgcn_readlane((int)ci, 63);
  const uint32_t tail = klen - 16u;
  for (uint32_t c0 = 0; c0 < C; c0 += kWave) {   // wave-uniform
    const uint32_t seed = (uint32_t)__builtin_popcountll(__ballot(ci <= c0));   // entry holding chunk c0
    mk[lane] = 0;
    if (nc != 0u && cx > c0 && cx < c0 + kWave) mk[cx - c0] = (uint8_t)lane;   // lane > 0 here
    wave_sync();   // DS instructions of one wave run in order: the read sees both writes
    uint32_t own = mk[lane];
    own = wave_incl_max(own > seed ? own : seed);
    wave_sync();   // the row is rewritten next pass after every lane has read it
    const int o = (int)own;
    const uint32_t ocx = (uint32_t)__shfl((int)cx, o, kWave), osrc = (uint32_t)__shfl((int)src, o, kWave);
    const uint32_t odst = (uint32_t)__shfl((int)dst, o, kWave), otl = (uint32_t)__shfl((int)tail, o, kWave);
    const uint32_t c = c0 + (uint32_t)lane;
    if (c < C) {
      const uint32_t q = 16u * (c - ocx), n = otl - q;
      store_bytes(kb + odst + q, lds_win16(stage, osrc + q), n < 16u ? n : 16u);
    }
  }
}

template <class P>
__device__ __forceinline__ void copy_emit(const PipeBuf<P>& B, const TileArgs& a, const CopyRow& r, int lane, uint8_t* mk) {
  const uint64_t pr = B.tpre[0], pk = B.tpre[1], pv = B.tpre[2];
  const bool live = r.live && B.bwr[r.j];   // bwr may have been cleared by the look-back (overflow)
  if (live) {
    const uint64_t gr = pr + B.icnt[r.f] + r.k;
    ost(a.key_end + gr, r.ks + r.klen - B.bkbb[r.j]);
    ost(a.val_end + gr, r.vs + r.vl - B.bvbb[r.j]);
  }
#ifndef MTBLX_ABL_NOVAL
  // values.  Fast path (wave-uniform): every live entry of this round has the same value
  // length U, a multiple of 16 -> lane k of a row writes 16 B chunks k, k+16, ... of the
  // interval's contiguous value range (coalesced stores).  Otherwise one entry per lane.
  const uint64_t lv = __ballot(live);
  if (lv != 0ull) {
    const int l0 = __builtin_ctzll(lv);
    const uint32_t U = (uint32_t)__builtin_amdgcn_readlane((int)r.vl, l0);
    const bool uni = (U % 16u) == 0u && U != 0u && __ballot(live && r.vl != U) == 0ull;
    const uint32_t vsrc = r.sp + r.ns;   // stage offset of the entry's value
    if (uni) {
      const uint32_t cpr = U >> 4;                                  // chunks per entry
      const bool pow2 = (cpr & (cpr - 1u)) == 0u;
      const uint32_t cprs = (uint32_t)__builtin_ctz(cpr);
      const uint32_t nrow = (r.fv && B.bok[r.j] && B.bwr[r.j]) ? (uint32_t)B.iraw[r.f] : 0u;
      const uint32_t nch = nrow * cpr;
      uint8_t* vd0 = a.vals + pv + (r.fv ? B.ivb[r.f] : 0u);
      const int rowbase = lane & ~15;
      // 4 chunks per lane per pass: the 4 permutes and LDS reads are in flight together
      // before the stores (one latency chain per pass instead of per chunk)
      for (uint32_t c0 = r.k; __ballot(c0 < nch) != 0ull; c0 += 64) {   // wave-uniform trip count
        uint4 w4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t c = c0 + 16u * (uint32_t)u;
          const bool act = c < nch;
          const uint32_t e = act ? (pow2 ? c >> cprs : c / cpr) : 0u;
          const uint32_t src = (uint32_t)__shfl((int)vsrc, rowbase + (int)e, kWave);
          w4[u] = act ? lds_win16(B.stage, src + 16u * (c - e * cpr)) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t c = c0 + 16u * (uint32_t)u;
#ifdef MTBLX_ABL_NOVSTORE   // diagnostic: the value reads without the value stores
          if (c < nch) asm volatile("" ::"v"(w4[u].x), "v"(w4[u].y), "v"(w4[u].z), "v"(w4[u].w));
#else
          if (c < nch) ost(reinterpret_cast<v4u*>(vd0 + 16u * c), v4u{w4[u].x, w4[u].y, w4[u].z, w4[u].w});
#endif
        }
      }
    } else if (live) {
      uint8_t* vd = a.vals + pv + r.vs;
      for (uint32_t o = 0; o < r.vl; o += 16) {
        const uint32_t mlen = r.vl - o;
        store_bytes(vd + o, lds_win16(B.stage, vsrc + o), mlen < 16 ? mlen : 16);
      }
    }
  }
#endif
#ifndef MTBLX_ABL_NOKEY
  uint8_t* kd = a.keys + pk + r.ks;
  if (live && r.klen > 0u) store_bytes(kd, r.W0, r.klen < 16u ? r.klen : 16u);
  const bool tl = live && r.klen > 16u;
  if (__ballot(tl) == 0ull) return;
  // (not in the fused-verify kernels: at their 128-VGPR cap it pushes PipeLargeV into scratch)
  if (!P::VERIFY && __ballot(tl && r.sh > 16u) == 0ull) {
    key_tails_dense(a.keys + pk, B.stage, mk, tl, r.klen, r.sp - r.sh + 16u, r.ks + 16u, lane);
    return;
  }
  for (uint32_t q0 = 16; __ballot(live && r.klen > q0) != 0ull; q0 += 16) {   // further planes (keys > 16 B)
    if (__ballot(live && r.sh > q0 && q0 < r.klen) == 0ull) {
      // no live entry inherits a byte of this plane from an earlier key: every byte is the
      // entry's own suffix (typical for long keys with short shared prefixes), copy it directly
      if (live && q0 < r.klen) {
        const uint32_t n = r.klen - q0;
        store_bytes(kd + q0, lds_win16(B.stage, r.sp - r.sh + q0), n < 16 ? n : 16);
      }
      continue;
    }
    const bool own = live && r.sh < q0 + 16u && q0 < r.klen;
    uint4 W = own ? lds_win16(B.stage, r.sp - r.sh + q0) : make_uint4(0, 0, 0, 0);
    uint32_t m = r.sh;
    key_scan_step<1>(m, W, q0);
    key_scan_step<2>(m, W, q0);
    key_scan_step<4>(m, W, q0);
    key_scan_step<8>(m, W, q0);
    if (live && q0 < r.klen) {
      const uint32_t n = r.klen - q0;
      store_bytes(kd + q0, W, n < 16 ? n : 16);
    }
  }
#endif
}

// Wait for a workgroup-local LDS counter.  Bounded: giving up means this launch's outputs are
// not trustworthy (look-back / hand-off timeout, totals[3] bit 1), never a hang.  A hand-off
// inside a workgroup waits one look-back bound plus a margin (handoff_ticks), so a look-back that
// gives up (and still releases its copy waves, microseconds later) never cascades into a hand-off
// that gives up with the LDS state unwritten; with the default 20 s bound a stuck launch reports
// after ~21 s (the earlier 4x multiple made that 80 s).
constexpr uint64_t kHandoffMargin = 100000000ull;   // 1 s of s_memrealtime (100 MHz)
__device__ __forceinline__ uint64_t handoff_ticks(const TileArgs& a) { return a.wait_ticks + kHandoffMargin; }
__device__ __forceinline__ void wait_flag(const TileArgs& a, const uint32_t* flag, uint32_t want) {
  WaitBound wb;
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < want) {
    __builtin_amdgcn_s_sleep(1);
    if (wb.expired(handoff_ticks(a))) { ws_timeout(a); break; }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <class P>
__device__ __forceinline__ void pipe_copy(const PipeBuf<P>& B, const TileArgs& a, int cw, int lane, const uint32_t* ready,
                                          uint32_t want, Stamps& ST, uint8_t* mk, uint32_t rows = P::ROWS) {
  const uint32_t nint = B.nint, nb = B.nb;
  uint32_t fb = (uint32_t)cw * (kWave / 16);
  if (fb < nint) {
    const CopyRow r = copy_prepare(B, fb, lane);
    ST.hit(14);
    wait_flag(a, ready, want);
    ST.hit(0);
    if (a.write) copy_emit(B, a, r, lane, mk);
    for (fb += rows; fb < nint; fb += rows) {   // wave-uniform
      const CopyRow r2 = copy_prepare(B, fb, lane);
      if (a.write) copy_emit(B, a, r2, lane, mk);
    }
  } else {
    wait_flag(a, ready, want);
    ST.hit(0);
  }
  // irregular blocks: exact serial write (thread per block)
  const int ct = cw * kWave + lane;
  if (a.write && ct < (int)nb && !B.bok[ct] && B.bwr[ct]) {
    const uint64_t pr = B.tpre[0], pk = B.tpre[1], pv = B.tpre[2];
    const uint32_t j = ct, bo = B.boff[j], L = B.blen[j];
    const uint8_t* d = (bo != kNotStaged) ? (B.stage + bo) : (a.data + a.blk_off[B.b0 + j]);
    generic_block<true>(d, L, a.keys + pk + B.bkbb[j], a.vals + pv + B.bvbb[j], a.key_end + pr + B.brb[j],
                        a.val_end + pr + B.brb[j]);
  }
}

// ---------------------------------------------------------------------------------
// fused CRC-32C verify (VERIFY kernels): the checksum Reader::block asserts
// before it decodes a block (src/reader.rs:159-164, crate crc32c 0.4), computed from the tile
// already staged in LDS by the COPY waves once their copy is done (they have the issue slots;
// round 2 ran it on the look-back and loader waves, which sit on the pipeline's critical path:
// 0.59 ms vs 0.148 for the decode alone, and ablating the CRC loop gave back 0.41 ms of it).
//   * a block's windows are 72 bytes counted from its END (window k = block bytes
//     [L - 72 (k + 1), L - 72 k)); bytes before the block start read as zero (leading zeros
//     leave a zero-init CRC unchanged) and the 0xFFFFFFFF init is folded into bytes 0..3;
//   * lane l takes windows k = l + 64 r: raw CRC by slicing-by-4 over 18 words (LDS tables),
//     shifted into place by x^(576 k) = K_l * X^r with K_l = x^(576 l) and X^r = x^(576 64 r)
//     held in registers from the kernel start (a GF(2) multiply each, none for r = 0);
//   * the wave XOR-reduces; copy wave w takes blocks w, w + NC, ... (or, with fewer blocks than
//     copy waves, one of g = NC / nb waves per block takes rounds r = s (mod g)); partials go
//     into a per-block LDS accumulator; the last copy wave to finish a tile finalises it.
// Copy wave 0 loads the stored checksums (the u32 before each content) at the start of its
// share, so their latency hides behind the window work.
// ---------------------------------------------------------------------------------
template <class P>
__device__ __forceinline__ uint32_t crc_word4(const PipeLds<P>& S, uint32_t c, uint32_t w) {
  c ^= w;   // slicing-by-4 (the LDS budget of PipeSmallV leaves room for 4 tables, not 8)
  return S.crcT[3][c & 0xffu] ^ S.crcT[2][(c >> 8) & 0xffu] ^ S.crcT[1][(c >> 16) & 0xffu] ^ S.crcT[0][c >> 24];
}

// Always inlined: under register pressure the compiler outlined a call of the round-2 CRC
// routine (PipeLargeV's look-back wave) and the out-of-line call is what faulted (DESIGN.md §4,
// "the spill fault"); MTBLX_CRC_NOINLINE (diagnostic builds only) forces the call.
#ifdef MTBLX_CRC_NOINLINE
#define MTBLX_PIPE_CRC_INLINE __attribute__((noinline))
#else
#define MTBLX_PIPE_CRC_INLINE __forceinline__
#endif
// MTBLX_ABL_CRC (diagnostic ablation builds only; results are wrong by construction):
// bit 0 skips the window loop, bit 1 the stored-checksum reads, bit 2 the whole CRC
#ifndef MTBLX_ABL_CRC
#define MTBLX_ABL_CRC 0
#endif
#ifndef MTBLX_CRC_WIN
#define MTBLX_CRC_WIN 72     // window bytes (36: 0.375 ms, 72: 0.340 on cfg2 -- LDS lookups, not chains, bound it)
#endif
#ifndef MTBLX_CRC_INFLIGHT
#define MTBLX_CRC_INFLIGHT 1 // window rounds in flight per lane (2: 0.416 ms at 72 B windows)
#endif
#ifndef MTBLX_CRC_UNROLL
#define MTBLX_CRC_UNROLL 9   // window steps unrolled
#endif
#ifndef MTBLX_CRC_EARLY
#define MTBLX_CRC_EARLY 0    // 1: before the copy (the tile is staged; the copy waits on the look-back)
#endif
constexpr uint32_t kCrcWinB = MTBLX_CRC_WIN;
constexpr uint32_t kCrcRounds = (65664u + 64u * kCrcWinB - 1u) / (64u * kCrcWinB);   // rounds of the largest block

// raw CRC (init 0) of the window whose first byte is at stage address A (block position p0);
// positions < 0 are zero, the init is folded into positions 0..3
template <class P>
__device__ __forceinline__ uint32_t lds_window_raw(const PipeLds<P>& S, const uint32_t* st32, int32_t A, int32_t p0) {
  const int32_t q = A >> 2;                       // floor
  if (q + (int32_t)kCrcWinB / 4 >= 0) MTBLX_LCHK(st32 + (q > 0 ? q : 0), 4 * (q + (int32_t)kCrcWinB / 4 + 1 - (q > 0 ? q : 0)));
  const uint32_t sft = (uint32_t)(A & 3) * 8u;
  uint32_t d0 = q >= 0 ? st32[q] : 0u;
  uint32_t c = 0;
#pragma unroll MTBLX_CRC_UNROLL
  for (int m = 0; m < (int)kCrcWinB / 4; ++m) {
    const int32_t qa = q + m + 1;
    const uint32_t d1 = qa >= 0 ? st32[qa] : 0u;
    uint32_t w = __builtin_amdgcn_alignbit(d1, d0, sft);
    d0 = d1;
    const int32_t pos = p0 + 4 * m;               // block position of the word's first byte
    if (pos < 4) {
      const uint32_t keep = pos <= -4 ? 0u : (pos < 0 ? 0xFFFFFFFFu << (8u * (uint32_t)(-pos)) : 0xFFFFFFFFu);
      const uint32_t fold = pos < 0 ? keep : 0xFFFFFFFFu >> (8u * (uint32_t)pos);
      w = (w & keep) ^ fold;
    }
    c = crc_word4(S, c, w);
  }
  return c;
}

// the finalisation of tile B's checksums: crc[] / crc_bad[] of its blocks (lanes < nb)
template <class P>
__device__ __forceinline__ void pipe_crc_final(const PipeBuf<P>& B, const TileArgs& a, PipeLds<P>& S, int lane,
                                               uint32_t par) {
  const uint32_t nb = B.nb, b0 = B.b0;
  uint32_t crc = 0, L = 0, o = kNotStaged;
  if (lane < (int)nb) {
    L = B.blen[lane];
    o = B.boff[lane];
    if (o < kOutOfBounds && L >= 4u) {
      crc = S.cacc[par][lane] ^ 0xFFFFFFFFu;
    } else if (o < kOutOfBounds) {   // < 4 bytes: byte-wise with the init
      uint32_t x = 0xFFFFFFFFu;
      MTBLX_LCHK(B.stage + o, L);
      for (uint32_t t = 0; t < L; ++t) x = S.crcT[0][(x ^ B.stage[o + t]) & 0xffu] ^ (x >> 8);
      crc = x ^ 0xFFFFFFFFu;
    }
    S.cacc[par][lane] = 0;
  }
  // blocks that were not staged (larger than a slot): from HBM, the wave together
  for (uint32_t j = 0; j < nb; ++j) {
    if (B.boff[j] != kNotStaged) continue;
    MTBLX_CHK(a.blk_off + b0 + j, 8);
    const uint64_t off = a.blk_off[b0 + j];
    const uint32_t x = mtblx_crc::wave_crc32c(a.data + off, B.blen[j], &S.crcT[0][0], lane);
    if (lane == (int)j) crc = x;
  }
  if (lane < (int)nb) {
    const uint32_t b = b0 + lane;
    if (a.crc) MTBLX_CHK(a.crc + b, 4);
    if (a.crc_bad) MTBLX_CHK(a.crc_bad + b, 1);
    if (a.crc) a.crc[b] = crc;
    if (a.crc_bad) {
      uint8_t bad = 0;
      if (o == kOutOfBounds) bad = 1;   // the reference's slice of the block panics before its checksum
      else if (a.crc_framed && S.cfr[par][lane]) bad = S.cst[par][lane] != crc;
      a.crc_bad[b] = bad;
    }
  }
}

// The fused checksum on the matrix cores (MTBLX_FUSED_MFMA=1, the A/B variant; the default, 0, is
// the VALU slicing path below, which measured faster -- DESIGN §0.4 item 6): the staged blocks' CRC-32C
// by the method of k_crc32c_mfma (crc_mfma.h) read straight from the tile's LDS stage.  Work unit
// = (block j, super-window sw: 8 steps of 1 KiB counted from the block's 16-byte aligned end in
// the stage); copy wave cw takes units cw, cw + NC, ... of the tile after its copy.  Per step a
// lane reads its aligned 16-byte chunk (ds_read_b128), masks the bytes before the block start
// and folds the init into bytes 0..3 (head_chunk), masks the pad after the block end
// (tail_chunk), then 8 fp4 + 2 f16 MFMAs (mfma_step); per unit the column parities, the column
// and super-window shifts and the pad removal x^(-8t) (nibble tables), XORed into the block's
// accumulator.  Round 4's VALU window loop (slicing-by-4, MTBLX_FUSED_MFMA=0) is the product.
#ifndef MTBLX_FUSED_MFMA
#define MTBLX_FUSED_MFMA 0
#endif
constexpr int kDecSup = (65664 + mtblx_crc::kMStep * mtblx_crc::kMSup - 1) / (mtblx_crc::kMStep * mtblx_crc::kMSup) + 1;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunneeded-internal-declaration"   // read only by the A/B path
static __constant__ mtblx_crc::MfmaTabs kDecMfma = mtblx_crc::MfmaTabs();
static __constant__ mtblx_crc::SwTabs<kDecSup> kDecSw = mtblx_crc::SwTabs<kDecSup>();
#pragma clang diagnostic pop

template <class P>
__device__ __forceinline__ void pipe_crc_mfma(const PipeBuf<P>& B, PipeLds<P>& S, uint32_t cw, int lane, uint32_t par) {
  using namespace mtblx_crc;
  constexpr uint32_t NC = (uint32_t)P::NCOPY;
  const uint32_t nb = B.nb;
  const int g = lane >> 4, n = lane & 15;
  const int32_t kx16 = 16 * (60 - 4 * n + g);   // the lane's chunk of a step
  uint32_t u = 0;   // running unit number over the tile's blocks
  for (uint32_t j = 0; j < nb; ++j) {
    const uint32_t L = B.blen[j], bo = B.boff[j];
    if (bo >= kOutOfBounds || L < 4u) continue;   // pipe_crc_final: from HBM / byte-wise
    const uint32_t t = (16u - ((bo + L) & 15u)) & 15u, Lp = L + t;
    const uint32_t steps = (Lp + kMStep - 1) / kMStep, nsup = (steps + kMSup - 1) / kMSup;
    // this wave's units of block j: sw with (u + sw) % NC == cw
    uint32_t sw = (cw + NC - u % NC) % NC;
    u += nsup;
    for (; sw < nsup; sw += NC) {
      v4f c2a = {0.f, 0.f, 0.f, 0.f}, c2b = c2a;
#pragma unroll 1
      for (int tt = kMSup - 1; tt >= 0; --tt) {   // from the super-window's start
        const uint32_t s = sw * kMSup + (uint32_t)tt;
        if (s < steps) {
          const int32_t pos = (int32_t)Lp - (int32_t)(kMStep * (s + 1)) + kx16;   // block position, 16-aligned in LDS
          v4u x = {0u, 0u, 0u, 0u};
          if (pos > -16) {
            MTBLX_LCHK(B.stage + (int32_t)bo + pos, 16);
            const uint4 w = *reinterpret_cast<const uint4*>(B.stage + (int32_t)bo + pos);
            x = v4u{w.x, w.y, w.z, w.w};
            if (pos < 4) x = head_chunk(x, pos);
          }
          if (s == 0 && t != 0 && lane == 48) x = tail_chunk(x, t);   // lane (g 3, n 0): the step's last chunk
          // the stage-1 operands are read per step (L1 / L2 hits): held in registers through the
          // tile loop they pushed the fused-verify kernels past 128 VGPRs into scratch
          const v4i* pa = reinterpret_cast<const v4i*>(&kDecMfma.a[0][0][0][0]) + lane;
          const v4i a2lo = reinterpret_cast<const v4i*>(&kDecMfma.a2[tt][0][0][0])[lane];
          const v4i a2hi = reinterpret_cast<const v4i*>(&kDecMfma.a2[tt][1][0][0])[lane];
          mfma_step_ld(pa, x, a2lo, a2hi, c2a, c2b);
        }
      }
      uint32_t c = kDecMfma.col[n][g][par_nib(c2a)] ^ kDecMfma.col[n][4 + g][par_nib(c2b)];
      c = row_xor(c);
      uint32_t C = (uint32_t)__builtin_amdgcn_readlane((int)c, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)c, 16) ^
                   (uint32_t)__builtin_amdgcn_readlane((int)c, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)c, 48);
      const uint32_t jl = (uint32_t)lane & 15u;
      if (sw) {   // x^(8·8192·sw)
        const uint32_t v = jl < 8u ? kDecSw.t[sw][jl][(C >> (4 * jl)) & 15u] : 0u;
        C = (uint32_t)__builtin_amdgcn_readlane((int)row_xor(v), 0);
      }
      if (t) {    // x^(-8t): the pad removed (linear: per unit, before the XOR of the units)
        const uint32_t v = jl < 8u ? kDecMfma.inv[t][jl][(C >> (4 * jl)) & 15u] : 0u;
        C = (uint32_t)__builtin_amdgcn_readlane((int)row_xor(v), 0);
      }
      if (lane == 0) __hip_atomic_fetch_xor(&S.cacc[par][j], C, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

// copy wave cw (of NC) after its copy of tile B: its share of the windows, then the count; the
// last of the NC waves finalises the tile
template <class P>
__device__ MTBLX_PIPE_CRC_INLINE void pipe_crc_copy(const PipeBuf<P>& B, const TileArgs& a, PipeLds<P>& S, uint32_t cw,
                                                    int lane, uint32_t par) {
  if constexpr ((MTBLX_ABL_CRC & 4) != 0) return;
#ifdef MTBLX_CALL_PROBE   // diagnostic (the outlined-call fault): the callee's arguments
  if (lane == 0 && cw == 0 && blockIdx.x < 2)
    printf("probe wg %u par %u B %p a %p data %p len %lu blk_off %p nblk %u crc %p bad %p "
           "framed %d nb %u b0 %u boff0 %u blen0 %u S %p crcT %p\n",
           blockIdx.x, par, (const void*)&B, (const void*)&a, (const void*)a.data, (unsigned long)a.data_len,
           (const void*)a.blk_off, a.nblk, (void*)a.crc, (void*)a.crc_bad, a.crc_framed, B.nb, B.b0, B.boff[0],
           B.blen[0], (void*)&S, (void*)&S.crcT[0][0]);
#if MTBLX_CALL_PROBE == 1
  return;   // arguments only: the body (and the fault) skipped
#endif
#endif
  constexpr uint32_t NC = (uint32_t)P::NCOPY;
  constexpr int kIn = MTBLX_CRC_INFLIGHT;
  const uint32_t nb = B.nb;
  // copy wave 0: the stored checksums (framed batches), loaded now, written to LDS at the end
  uint32_t stored = 0, framed = 0;
  if (cw == 0 && lane < (int)nb && a.crc_framed && (MTBLX_ABL_CRC & 2) == 0) {
    MTBLX_CHK(a.blk_off + B.b0 + lane, 8);
    const uint64_t off = a.blk_off[B.b0 + lane];
    // a window past the buffer (a corrupt directory) is never read: pipe_crc_final reports it as
    // bad without its stored checksum (r05: this read was unguarded)
    if (off >= 4 && off <= a.data_len) {
      const uint8_t* d = a.data + off;
      MTBLX_CHK(d - 4, 4);
      stored = (uint32_t)d[-4] | ((uint32_t)d[-3] << 8) | ((uint32_t)d[-2] << 16) | ((uint32_t)d[-1] << 24);
      framed = 1;
    }
  }
  const uint32_t* st32 = reinterpret_cast<const uint32_t*>(B.stage);
  const uint32_t g = nb >= NC ? 1u : NC / nb;           // waves per block
  const uint32_t jstep = nb >= NC ? NC : nb;            // (nb < NC: one block per wave, then done)
  if constexpr ((MTBLX_ABL_CRC & 1) == 0 && MTBLX_FUSED_MFMA) pipe_crc_mfma(B, S, cw, lane, par);
  if constexpr ((MTBLX_ABL_CRC & 1) == 0 && !MTBLX_FUSED_MFMA)
  for (uint32_t j = nb >= NC ? cw : cw / g; j < nb; j += jstep) {
    const uint32_t s = nb >= NC ? 0u : cw % g;
    const uint32_t L = B.blen[j], bo = B.boff[j];
    if (bo >= kOutOfBounds || L < 4u) continue;         // finalisation: from HBM / byte-wise
    const uint32_t nwin = (L + kCrcWinB - 1) / kCrcWinB, nr = (nwin + 63u) / 64u;
    uint32_t acc = 0;
    if constexpr (kIn == 1) {
      for (uint32_t r = s; r < nr; r += g) {
        const uint32_t k = (uint32_t)lane + 64u * r;
        uint32_t c = 0;
        if (k < nwin) {
          const int32_t p0 = (int32_t)L - (int32_t)(kCrcWinB * (k + 1u));
          c = lds_window_raw(S, st32, (int32_t)bo + p0, p0);
        }
        acc ^= r ? mtblx_crc::dmultmodp(S.shX[r], c) : c;
      }
    } else
    for (uint32_t r0 = s; r0 < nr; r0 += g * kIn) {
      // rounds r0, r0 + g, ... (kIn of them) side by side: independent chains
      uint32_t c[kIn], d0[kIn];
      int32_t Aw[kIn], p0[kIn];
#pragma unroll
      for (int i = 0; i < kIn; ++i) {
        const uint32_t k = (uint32_t)lane + 64u * (r0 + (uint32_t)i * g);
        const bool on = r0 + (uint32_t)i * g < nr && k < nwin;
        p0[i] = on ? (int32_t)L - (int32_t)(kCrcWinB * (k + 1u)) : (1 << 20);   // off: never masked, dropped
        Aw[i] = on ? (int32_t)bo + p0[i] : 0;
        d0[i] = Aw[i] >= 0 ? st32[Aw[i] >> 2] : 0u;
        c[i] = 0;
      }
#pragma unroll MTBLX_CRC_UNROLL
      for (int m = 0; m < (int)kCrcWinB / 4; ++m) {
#pragma unroll
        for (int i = 0; i < kIn; ++i) {
          const int32_t qa = (Aw[i] >> 2) + m + 1;
          const uint32_t d1 = qa >= 0 ? st32[qa] : 0u;
          uint32_t w = __builtin_amdgcn_alignbit(d1, d0[i], (uint32_t)(Aw[i] & 3) * 8u);
          d0[i] = d1;
          const int32_t pos = p0[i] + 4 * m;           // block position of the word's first byte
          if (pos < 4) {
            const uint32_t keep = pos <= -4 ? 0u : (pos < 0 ? 0xFFFFFFFFu << (8u * (uint32_t)(-pos)) : 0xFFFFFFFFu);
            const uint32_t fold = pos < 0 ? keep : 0xFFFFFFFFu >> (8u * (uint32_t)pos);
            w = (w & keep) ^ fold;
          }
          c[i] = crc_word4(S, c[i], w);
        }
      }
#pragma unroll
      for (int i = 0; i < kIn; ++i) {
        const uint32_t r = r0 + (uint32_t)i * g;
        if (r >= nr || p0[i] == (1 << 20)) continue;
        acc ^= r ? mtblx_crc::dmultmodp(S.shX[r], c[i]) : c[i];
      }
    }
    acc = mtblx_crc::dmultmodp(S.shK[lane], acc);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o, kWave);
    if (lane == 0) __hip_atomic_fetch_xor(&S.cacc[par][j], acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  if (cw == 0 && lane < (int)nb) {
    S.cst[par][lane] = stored;
    S.cfr[par][lane] = framed;
  }
  uint32_t old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(&S.crcdone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
  if (old % NC != NC - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  pipe_crc_final(B, a, S, lane, par);
}

#ifdef MTBLX_LARGE_SERIAL
constexpr bool kLargeSerial = true;   // A/B: the round-2 two-buffer schedule for PipeLarge
#else
constexpr bool kLargeSerial = false;
#endif
// Two-buffer schedule (PipeLarge): 1 = late walk (the DMA of tile it+1 into the free buffer at
// the start of iteration it, beside the prepare + copy of tile it; the walker walks tile it+1 once
// it has landed); 0 = walk of tile it+1 beside the copy of tile it, DMA of tile it+2 after it.
#ifndef MTBLX_LARGE_LATE
#define MTBLX_LARGE_LATE 1
#endif
#ifndef MTBLX_PHASE_DELAY     // A/B: PipeLarge workgroups of one half start this many cycles late
#define MTBLX_PHASE_DELAY 0
#endif
#ifndef MTBLX_PHASE_SEL       // ... the half: 0 = odd workgroups, 1 = (g >> 3) odd (half of each XCD)
#define MTBLX_PHASE_SEL 0
#endif
#ifndef MTBLX_LATE_LOADCOPY   // late walk: the loaders copy rows of tile it after their DMA
#define MTBLX_LATE_LOADCOPY 0
#endif

// MTBLX_SPILL (diagnostic build only, `make spill`): keep kSpillPad extra VGPRs live across the
// whole pipeline kernel, which pushes it past its 128 VGPRs into scratch -- checks that a
// spilling build is still correct (tests/test_spill_gpu.py)
#ifdef MTBLX_SPILL
constexpr int kSpillPad = MTBLX_SPILL;
#else
constexpr int kSpillPad = 0;
#endif
template <class P>
__global__ void __launch_bounds__(kPipeThreads, 1) k_decode_pipe(TileArgs a) {
  uint32_t spill_pad[kSpillPad > 0 ? kSpillPad : 1];
  if constexpr (kSpillPad > 0) {
#pragma unroll
    for (int i = 0; i < kSpillPad; ++i) spill_pad[i] = a.blk_len[((uint32_t)threadIdx.x + 7u * i) % a.nblk];   // loads: not rematerialisable
  }
  __shared__ PipeLds<P> S;
  // Two buffers, serial: tile it is walked, looked back and copied in iteration it while the
  // loaders stage tile it+1 (PipeLargeV: its fused CRC reads the tile being copied).  Otherwise
  // the three-stage schedule: walk it+1 | look-back + copy it | DMA it+2 -- with two buffers
  // the DMA of tile it+2 goes into tile it's buffer once the copy waves have left it.
  constexpr bool serial2 = P::NBUF == 2 && (P::VERIFY || kLargeSerial);
  // Two buffers, three stages: the loaders have nothing to do until the copy waves leave tile
  // it's buffer, so they copy too (as copy waves NCOPY ..): 56 rows per pass, so a 64 KiB block
  // (~53 restart intervals) takes one pass instead of 48 + 5.
  constexpr bool kLate = P::NBUF == 2 && !serial2 && MTBLX_LARGE_LATE;
  constexpr bool kLoadCopy = P::NBUF == 2 && !serial2 && (!kLate || MTBLX_LATE_LOADCOPY);
  constexpr uint32_t kCopyW = P::NCOPY + (kLoadCopy ? P::LOADW : 0);   // waves that copy a tile
  constexpr uint32_t kRows = kCopyW * (kWave / 16);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t g = blockIdx.x, G = gridDim.x;
  const uint32_t nloc = (a.ntiles > g) ? (a.ntiles - g + G - 1) / G : 0;  // tiles of this workgroup
  Stamps ST;
  ST.init();
  TL(0);
  ws_begin(a);
  if constexpr (!P::VERIFY) ws_debug_delay(a);
  a.flags_direct = 1;
  if (tid == 0) { S.ready = 0; S.pub = 0; S.cdone = 0; S.crcdone = 0; S.staged = 0; }
  if constexpr (P::VERIFY) {
    for (int i = tid; i < 4 * 256; i += kPipeThreads) S.crcT[i >> 8][i & 255] = mtblx_crc::kTab.slice[i >> 8][i & 255];
    for (int i = tid; i < 2 * P::MAXBLK; i += kPipeThreads) S.cacc[i / P::MAXBLK][i % P::MAXBLK] = 0;
    // the copy waves' window / round shift constants (read after the barrier before the loop)
    if (tid < 64) S.shK[tid] = mtblx_crc::xpow8((uint64_t)kCrcWinB * (uint32_t)tid);
    else if (tid < 64 + (int)kCrcRounds) S.shX[tid - 64] = mtblx_crc::xpow8((uint64_t)kCrcWinB * 64u * (uint32_t)(tid - 64));
  }

  uint64_t tinc[3] = {0, 0, 0};           // wave 1
  uint64_t lbv[kMaxLookbackLoads];        // wave 1: look-back words of the next tile to copy
  uint64_t ioff = 0;                      // wave 0: directory entry (lane < nb) of the next tile to stage
  uint32_t ilen = 0;
  auto load_info = [&](uint32_t kk) {
    if (kk >= nloc) return;
    uint32_t b0, nb;
    tile_span(a, g + kk * G, b0, nb);
    const uint32_t j = (uint32_t)lane < nb ? (uint32_t)lane : nb - 1;
    MTBLX_CHK(a.blk_off + b0 + j, 8);
    MTBLX_CHK(a.blk_len + b0 + j, 4);
    ioff = a.blk_off[b0 + j];
    ilen = a.blk_len[b0 + j];
  };
  // loaders split every tile's DMA pieces (even / odd 1 KiB pieces)
  const bool loader = wv >= kPipeLoadWave && wv < kPipeLoadWave + P::LOADW;
  const uint32_t part = (uint32_t)(wv - kPipeLoadWave);
  if (loader) {
    load_info(0);
    if constexpr (!kLate) {
      if (nloc > 0) pipe_dma(S.buf[0], a, g, ioff, ilen, lane, part);
      load_info(1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (wv == 1) {
    if (!serial2 && nloc > 0) pipe_lookback_issue(a, g, G, lbv, lane);
  }
  __syncthreads();
  TL(1);
#if MTBLX_PHASE_DELAY > 0
  // A/B (diagnostic builds): start half of the workgroups MTBLX_PHASE_DELAY shader cycles late so
  // that the two halves' DMA + store phases (HBM-bound) do not coincide
  if constexpr (P::NBUF == 2) {
    const bool late_half = MTBLX_PHASE_SEL == 0 ? (g & 1u) != 0u : ((g >> 3) & 1u) != 0u;
    if (late_half) {
      const uint64_t t0 = __builtin_amdgcn_s_memtime();
      while (__builtin_amdgcn_s_memtime() - t0 < (uint64_t)MTBLX_PHASE_DELAY) __builtin_amdgcn_s_sleep(8);
    }
  }
#endif
  if (wv == 0) __builtin_amdgcn_s_setprio(2);  // the walk is a serial latency chain
  uint64_t ntl = 0;
  uint32_t wmode = 0;   // wave 0: which interval walk goes first (pipe_walk)

  if constexpr (serial2) {
    for (uint32_t it = 0; it < nloc; ++it) {
      PipeBuf<P>& C = S.buf[it & 1u];
      const uint32_t tc = g + it * G;
      if (wv == 0) {
        pipe_walk(C, a, tc, lane, ST, wmode);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&S.pub, it + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        ST.hit(3);
      } else if (loader) {
        if (it + 1 < nloc) {
          // DMA landing in LDS slows the walker's tail (LDS writes and fences queue behind it)
          // by ~3.5k cycles per 64 KiB tile, but beside the copy it slows a key-heavy copy
          // (cfg3's long keys read many 16-byte key planes).  So: when the previous tile's key
          // bytes were under a third of its value bytes (the copy is short), stage only the
          // first kLargeDmaSplit pieces beside the walk's chain and the rest after the walk.
          // (the other buffer still holds that tile's totals: the DMA writes only its stage)
          PipeBuf<P>& N = S.buf[(it + 1) & 1u];
          const bool late = it >= 1 && 3ull * N.ttot[1] <= (uint64_t)N.ttot[2];
          pipe_dma(N, a, tc + G, ioff, ilen, lane, part, 0, late ? kLargeDmaSplit : 0xFFFFFFFFu);
          if (late) {
            wait_flag(a, &S.pub, it + 1);
            pipe_dma(N, a, tc + G, ioff, ilen, lane, part, kLargeDmaSplit);
          }
          load_info(it + 2);
        }
        ST.hit(4);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // retire the DMA of tile it+1 (read next phase)
        ST.hit(6);
      } else if (wv == 1) {
        wait_flag(a, &S.pub, it + 1);
        pipe_lookback_issue(a, tc, G, lbv, lane);
        pipe_lookback(C, a, tc, G, tinc, lbv, lane, &S.ready, it + 1);
        ST.hit(1);
      } else {
        wait_flag(a, &S.pub, it + 1);
        if constexpr (P::VERIFY && MTBLX_CRC_EARLY) pipe_crc_copy(C, a, S, (uint32_t)(wv - P::COPY0), lane, it & 1u);
        pipe_copy(C, a, wv - P::COPY0, lane, &S.ready, it + 1, ST, S.cmk[wv]);
        if constexpr (P::VERIFY && !MTBLX_CRC_EARLY) pipe_crc_copy(C, a, S, (uint32_t)(wv - P::COPY0), lane, it & 1u);
        ST.hit(7);
      }
      raw_barrier();
      if (wv == 0) { ST.hit(8); ++ntl; }
      else if (wv == P::COPY0) ST.hit(5);
      else if (loader) ST.hit(12);
      else ST.hit(1);
    }
  } else if constexpr (kLate) {
    // iteration it: the loaders stage tile it+1 into the buffer tile it-1 left, then (optionally)
    // copy rows of tile it; the walker walks tile it+1 once both loaders' DMA has landed; the
    // look-back and copy waves finish tile it meanwhile.  The DMA (HBM reads) now overlaps the
    // copy's prepare and stores instead of following them.
    for (int it = -1; it < (int)nloc; ++it) {
      const uint32_t k1 = (uint32_t)(it + 1);
      if (wv == 0) {
        if (k1 < nloc) {
          wait_flag(a, &S.staged, (k1 + 1) * (uint32_t)P::LOADW);
          ST.hit(8);   // stamps: the DMA-landing wait counts with the barrier, "trailers" is the trailers alone
          pipe_walk(S.buf[k1 & 1u], a, g + k1 * G, lane, ST, wmode);
          if (lane == 0) __hip_atomic_store(&S.pub, k1 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        ST.hit(3);
      } else if (loader) {
        if (k1 < nloc) {
          pipe_dma(S.buf[k1 & 1u], a, g + k1 * G, ioff, ilen, lane, part);
          load_info(k1 + 1);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of tile it+1 has landed
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) __hip_atomic_fetch_add(&S.staged, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        ST.hit(4);
        if constexpr (kLoadCopy) {
          if (it >= 0) {
            pipe_copy(S.buf[(uint32_t)it & 1u], a, P::NCOPY + (int)part, lane, &S.ready, (uint32_t)it + 1, ST, S.cmk[wv], kRows);
            if (lane == 0) __hip_atomic_fetch_add(&S.cdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
        ST.hit(6);
      } else if (it >= 0) {
        PipeBuf<P>& C = S.buf[(uint32_t)it & 1u];
        const uint32_t tc = g + (uint32_t)it * G;
        if (wv == 1) {
          pipe_lookback(C, a, tc, G, tinc, lbv, lane, &S.ready, (uint32_t)it + 1);
          if (it + 1 == (int)nloc) TLW(8);
          else if (it + 2 == (int)nloc) TLW(11);
          ST.hit(1);
          if (k1 < nloc) {
            WaitBound wb;
            while (__hip_atomic_load(&S.pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < k1 + 1) {
              __builtin_amdgcn_s_sleep(1);
              if (wb.expired(handoff_ticks(a))) { ws_timeout(a); break; }
            }
            pipe_lookback_issue(a, tc + G, G, lbv, lane);
            pipe_lookback_poll(a, tc + G, G, lbv, lane, &S.cdone, (uint32_t)(it + 1) * kCopyW);
          }
          ST.hit(1);
        } else {
          pipe_copy(C, a, wv - P::COPY0, lane, &S.ready, (uint32_t)it + 1, ST, S.cmk[wv], kRows);
          if (wv == P::COPY0 && it + 1 == (int)nloc) TLW(9);
          if (wv == P::COPY0 + P::NCOPY - 1 && it + 1 == (int)nloc) TLW(10);
          if (lane == 0) __hip_atomic_fetch_add(&S.cdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          ST.hit(7);
        }
      }
      raw_barrier();
      if (it == -1) TL(2);
      else if (it == 0) TL(3);
      else if (it + 2 == (int)nloc) TL(7);
      if (wv == 0) { ST.hit(8); ++ntl; }
      else if (wv >= P::COPY0) ST.hit(5);
      else if (loader) ST.hit(12);
      else ST.hit(11);
    }
  } else
  for (int it = -1; it < (int)nloc; ++it) {
    const uint32_t k1 = (uint32_t)(it + 1), k2 = (uint32_t)(it + 2);
    if (wv == 0) {
      // walk first: the aggregate A(tile it+1) is published as early as possible
      if (k1 < nloc) {
        pipe_walk(S.buf[k1 % P::NBUF], a, g + k1 * G, lane, ST, wmode);
        if (lane == 0) __hip_atomic_store(&S.pub, k1 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      ST.hit(3);
    } else if (loader) {
      if constexpr (kLoadCopy) {
        if (it >= 0) {
          pipe_copy(S.buf[(uint32_t)it % P::NBUF], a, P::NCOPY + (int)part, lane, &S.ready, (uint32_t)it + 1, ST, S.cmk[wv], kRows);
          if (lane == 0) __hip_atomic_fetch_add(&S.cdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      if (k2 < nloc) {
        if constexpr (P::NBUF == 2) {
          // tile it+2 goes into tile it's buffer: wait until every copy wave has left it
          if (it >= 0) wait_flag(a, &S.cdone, (uint32_t)(it + 1) * kCopyW);
        }
        pipe_dma(S.buf[k2 % P::NBUF], a, g + k2 * G, ioff, ilen, lane, part);
        load_info(k2 + 1);
      }
      ST.hit(4);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // retire the DMA of tile it+2 (read next phase)
      ST.hit(6);
    } else if (it >= 0) {
      PipeBuf<P>& C = S.buf[(uint32_t)it % P::NBUF];
      const uint32_t tc = g + (uint32_t)it * G;
      if (wv == 1) {
        pipe_lookback(C, a, tc, G, tinc, lbv, lane, &S.ready, (uint32_t)it + 1);
        if (it + 1 == (int)nloc) TLW(8);         // look-back of the last tile done
        else if (it + 2 == (int)nloc) TLW(11);   // ... of the second-to-last
        ST.hit(1);
        if (k1 < nloc) {
          // the other workgroups publish A(tile it+1's predecessors) about when this
          // workgroup's wave 0 publishes A(tile it+1): issue the look-back loads after that
          WaitBound wb;
          while (__hip_atomic_load(&S.pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < k1 + 1) {
            __builtin_amdgcn_s_sleep(1);
            if (wb.expired(handoff_ticks(a))) { ws_timeout(a); break; }
          }
          pipe_lookback_issue(a, tc + G, G, lbv, lane);
          pipe_lookback_poll(a, tc + G, G, lbv, lane, &S.cdone, (uint32_t)(it + 1) * kCopyW);
        }
        ST.hit(1);
      } else {
        if constexpr (P::VERIFY && MTBLX_CRC_EARLY) pipe_crc_copy(C, a, S, (uint32_t)(wv - P::COPY0), lane, (uint32_t)it & 1u);
        pipe_copy(C, a, wv - P::COPY0, lane, &S.ready, (uint32_t)it + 1, ST, S.cmk[wv], kRows);
        if (wv == P::COPY0 && it + 1 == (int)nloc) TLW(9);   // first copy wave: last tile's stores issued
        if (wv == P::COPY0 + P::NCOPY - 1 && it + 1 == (int)nloc) TLW(10);
        if (lane == 0) __hip_atomic_fetch_add(&S.cdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if constexpr (P::VERIFY && !MTBLX_CRC_EARLY) pipe_crc_copy(C, a, S, (uint32_t)(wv - P::COPY0), lane, (uint32_t)it & 1u);
        ST.hit(7);
      }
    }
    raw_barrier();
    if (it == -1) TL(2);
    else if (it == 0) TL(3);
    else if (it + 2 == (int)nloc) TL(7);   // end of the second-to-last iteration
    if (wv == 0) { ST.hit(8); ++ntl; }
    else if (wv >= P::COPY0) ST.hit(5);
    else if (loader) ST.hit(12);
    else ST.hit(11);
  }
  TL(4);
  // retire this wave's outstanding global stores before the workgroup ends
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (wv >= P::COPY0) TLW(12 + (wv & 1));   // copy waves' drains (two of them)
  TLW(14 + (wv == 1));                       // wave 0 / wave 1 drains (the slots race; diagnostic)
  if (g == (a.ntiles - 1) % G && tid == 0) pipe_close(a);
  if constexpr (kSpillPad > 0) {
#pragma unroll
    for (int i = 0; i < kSpillPad; ++i) asm volatile("" ::"v"(spill_pad[i]));
  }
  TL(5);
#ifdef MTBLX_STAMPS
  if (tid == 0 && blockIdx.x < 1024) g_tl[blockIdx.x][6] = nloc;
#endif
#ifdef MTBLX_STAMPS
  // wave 0: [2] trailers + walk loop, [3] scans + publish, [8] barrier.  wave 1: [1]
  // look-back (+ barrier).  first loader: [4] DMA issue, [6] DMA wait + barrier.  first copy
  // wave: [0] wait ready, [7] copy, [5] barrier.  Summed over workgroups (lane 0); [15] tiles.
  // copy waves: [13] the smallest barrier wait among them (the last to arrive), [14] the
  // longest prepare of the first round (before the wait for the look-back), per workgroup
  __shared__ unsigned long long cmin, cmax;
  if (tid == 0) { cmin = ~0ull; cmax = 0; }
  __syncthreads();
  if (lane == 0 && wv >= P::COPY0) {
    atomicMin(&cmin, (unsigned long long)ST.acc[5]);
    atomicMax(&cmax, (unsigned long long)ST.acc[14]);
  }
  __syncthreads();
  if (tid == 0 && a.dbg) {
    atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg + 13), cmin);
    atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg + 14), cmax);
  }
  if (lane == 0 && a.dbg && (wv <= kPipeLoadWave || wv == P::COPY0)) {
    for (int k = 0; k < 13; ++k) {
      const bool mine = (wv == 0) ? (k == 2 || k == 3 || k == 8 || k == 9 || k == 10) : (wv == 1) ? (k == 1 || k == 11) : loader ? (k == 4 || k == 6 || k == 12) : (k == 0 || k == 5 || k == 7);
      if (mine) atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg + k), (unsigned long long)ST.acc[k]);
    }
    if (wv == 0) atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg + 15), (unsigned long long)ntl);
  }
#else
  (void)ntl;
#endif
}

using CfgSmall = TileCfg<32768, 640, 256, 64, true, 3>;
using CfgLarge = TileCfg<67584, 1024, 256, 16, false, 1>;

}  // namespace mtblx

// ----------------------------------------------------------------------------------
// launch glue (called from mtblx_api.cpp)
// ----------------------------------------------------------------------------------
using namespace mtblx;

namespace {
struct Plan {
  uint32_t bpt, slot, ntiles;
  int kind;   // 0 = k_decode_pipe<PipeSmall>, 1 = k_decode_pipe<PipeLarge>, 2 = k_decode_tiles<CfgLarge>
};

// tile shape for staging bytes TB: contiguous staging needs blocks + framing (<= 14 B each)
// + 16 B alignment + a 32 B tail; the fallback layout uses one 16 B aligned slot per block
static bool fit_plan(uint32_t max_len, uint32_t tb, uint32_t maxblk, Plan& p) {
  const uint32_t slot = ((max_len + 30u) / 16u) * 16u;
  const uint32_t per = max_len + 16u;
  const uint32_t usable = tb - 48;
  if (max_len == 0 || slot > usable) return false;
  p.slot = slot;
  p.bpt = std::max<uint32_t>(1, std::min<uint32_t>(usable / std::max(per, slot), maxblk));
  return true;
}

// (the fused-verify kernels may stage fewer bytes than their plain twins: the tile shape follows
// the kernel that will run)
Plan make_plan(uint32_t nblk, uint32_t max_len, bool verify) {
  Plan p{};
  if (fit_plan(max_len, verify ? PipeSmallV::TB : PipeSmall::TB, PipeSmall::MAXBLK, p)) {
    p.kind = 0;
  } else if (fit_plan(max_len, verify ? PipeLargeV::TB : PipeLarge::TB, PipeLarge::MAXBLK, p)) {
    p.kind = 1;
  } else {
    const uint32_t usable = CfgLarge::TB - 48;
    const uint32_t slot = ((max_len + 30u) / 16u) * 16u, per = max_len + 16u;
    p.kind = 2;
    p.slot = (max_len != 0 && slot <= usable) ? slot : usable;
    p.bpt = std::max<uint32_t>(1, std::min<uint32_t>(usable / std::max(per, p.slot), CfgLarge::MAXBLK));
  }
  p.ntiles = (nblk + p.bpt - 1) / p.bpt;
  return p;
}



// One workgroup per CU: every workgroup of a launch is resident, which the look-back between
// workgroups needs.  MTBLX_PIPE_CUS caps it (diagnostic: several processes sharing one GPU, e.g.
// bench.py --share-gpu, each keep their launches co-resident on their share of the CUs).
int pipe_grid(uint32_t ntiles) {
  static mtblx_dev::Cache cache;
  const int g = cache.get([] {
    int ncu = mtblx_dev::cu_count();
    const char* cap = getenv("MTBLX_PIPE_CUS");
    if (cap && atoi(cap) > 0) ncu = std::min(ncu, atoi(cap));
    return std::max(1, std::min(ncu, kMaxLookbackLoads * kWave + 1));
  });
  return (int)std::min<uint32_t>(ntiles, (uint32_t)g);
}

template <class C>
int resident_grid(uint32_t ntiles) {
  static mtblx_dev::Cache cache;
  const int g = cache.get([] {
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_decode_tiles<C>, kThreads, 0) != hipSuccess || occ < 1)
      occ = 1;
    int lds_lim = (int)((160u * 1024u) / sizeof(TileLds<C>));
    if (lds_lim < 1) lds_lim = 1;
    const int c = std::max(1, mtblx_dev::cu_count() * std::min(occ, lds_lim));
    return std::min(c, kMaxLookbackLoads * kThreads + 1);  // look-back window = G - 1
  });
  return (int)std::min<uint32_t>(ntiles, (uint32_t)g);
}
}  // namespace

// workspace: [0, 128) diagnostic stamps | [128, 256) WsHdr | 3 u64 per tile (tiles <= nblk).
// Zero-filled once by the caller; every launch leaves it ready for the next (ws_end).
#ifdef MTBLX_STAMPS
extern "C" int mtblx_dbg_timeline(uint64_t* out, uint32_t nwg) {   // diagnostic build only
  if (nwg > 1024) nwg = 1024;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mtblx::g_tl), (size_t)nwg * 16 * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" size_t mtblx_impl_ws_bytes(uint32_t nblk) { return 256u + (size_t)nblk * 8u * kTileWords + 64u; }

extern "C" int mtblx_crc32c_blocks(const mtblx_block_batch* in, uint32_t* crc, uint8_t* bad, int framed,
                                   void* stream);

// MTBLX_DEBUG_FLAGS (test knob): bits ORed into totals[3] at the end of every decode launch,
// e.g. 2 = report a look-back timeout, to check that every reader surface rejects such a launch.
static unsigned long long debug_flags() {
  const char* e = getenv("MTBLX_DEBUG_FLAGS");
  return e ? strtoull(e, nullptr, 0) : 0ull;
}
// MTBLX_DEBUG_WAIT_MS / MTBLX_DEBUG_DELAY0_MS (test knobs): the bounded waits give up after
// that many ms instead of 20 s; workgroup 0 starts (and publishes A(0)) that many ms late
// (tests/test_robust_gpu.py: a look-back timeout that happens before tile 0 starts survives)
static uint64_t debug_ms(const char* name, uint64_t dflt) {
  const char* e = getenv(name);
  return e ? strtoull(e, nullptr, 0) * 100000ull : dflt;   // s_memrealtime: 100 MHz
}

extern "C" int mtblx_impl_run(const mtblx_block_batch* in, const mtblx_decoded* out, void* ws, size_t ws_bytes,
                              int write, hipStream_t s, int verify, uint32_t* crc, uint8_t* crc_bad, int framed) {
  const uint32_t nblk = in->nblk;
  const uint64_t cap64 = ws_bytes > 320u ? (ws_bytes - 320u) / (8u * kTileWords) : 0u;
  const uint32_t wscap = cap64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cap64;
  const Plan p = make_plan(nblk, in->max_blk_len, verify != 0);
  uint64_t* dbg = reinterpret_cast<uint64_t*>(ws);
  WsHdr* hdr = reinterpret_cast<WsHdr*>(reinterpret_cast<uint8_t*>(ws) + 128);
  uint64_t* lbw = dbg + 32;
  TileArgs a{in->data,     in->data_len,  in->blk_off,  in->blk_len,   nblk,         p.bpt,         p.slot,
             p.ntiles,     out->nrec,     out->rec_base, out->key_base, out->val_base, out->status, out->key_end,
             out->val_end, out->rec_cap,  out->keys,    out->keys_cap, out->vals,    out->vals_cap, out->totals,
             lbw,          hdr,           dbg,          write ? 1 : 0, crc,         crc_bad,       framed ? 1 : 0,
             wscap,        0,             0,            debug_flags()};
  a.wait_ticks = debug_ms("MTBLX_DEBUG_WAIT_MS", kWaitTicks);
  a.dbg_delay0 = debug_ms("MTBLX_DEBUG_DELAY0_MS", 0);
#define MTBLX_DECODE_PTRS                                                                                        \
  (MTBLX_R(in->data, in->data_len), MTBLX_R(in->blk_off, 8ull * nblk), MTBLX_R(in->blk_len, 4ull * nblk),         \
   MTBLX_R(out->nrec, 4ull * nblk), MTBLX_R(out->rec_base, 8ull * nblk), MTBLX_R(out->key_base, 8ull * nblk),      \
   MTBLX_R(out->val_base, 8ull * nblk), MTBLX_R(out->status, 4ull * nblk), MTBLX_R(out->key_end, 4 * out->rec_cap), \
   MTBLX_R(out->val_end, 4 * out->rec_cap), MTBLX_R(out->keys, out->keys_cap), MTBLX_R(out->vals, out->vals_cap),   \
   MTBLX_R(out->totals, 32), MTBLX_R(ws, ws_bytes), MTBLX_R(crc, 4ull * nblk), MTBLX_R(crc_bad, nblk))
  if (p.kind == 0) {
    if (verify)
      MTBLX_LAUNCH(MTBLX_DECODE_PTRS, k_decode_pipe<PipeSmallV>, dim3(pipe_grid(p.ntiles)), dim3(kPipeThreads), 0, s, a);
    else
      MTBLX_LAUNCH(MTBLX_DECODE_PTRS, k_decode_pipe<PipeSmall>, dim3(pipe_grid(p.ntiles)), dim3(kPipeThreads), 0, s, a);
  } else if (p.kind == 1) {
    if (verify)
      MTBLX_LAUNCH(MTBLX_DECODE_PTRS, k_decode_pipe<PipeLargeV>, dim3(pipe_grid(p.ntiles)), dim3(kPipeThreads), 0, s, a);
    else
      MTBLX_LAUNCH(MTBLX_DECODE_PTRS, k_decode_pipe<PipeLarge>, dim3(pipe_grid(p.ntiles)), dim3(kPipeThreads), 0, s, a);
  } else {
    MTBLX_LAUNCH(MTBLX_DECODE_PTRS, k_decode_tiles<CfgLarge>, dim3(resident_grid<CfgLarge>(p.ntiles)), dim3(kThreads), 0, s, a);
    // blocks above ~64 KiB: the checksum is a separate launch (k_crc32c_blocks)
    if (verify && hipGetLastError() == hipSuccess) return mtblx_crc32c_blocks(in, crc, crc_bad, framed, s);
  }
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
