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
// Everything is integer/byte work: HBM-bandwidth bound, no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "mtblx.h"

namespace mtblx {

constexpr int kWave = 64;
constexpr uint64_t kU32Max = 0xFFFFFFFFull;

// ----------------------------------------------------------------------------------
// small helpers
// ----------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t byte_of(const uint4& w, uint32_t t) {
  uint32_t d = (t < 4) ? w.x : (t < 8) ? w.y : (t < 12) ? w.z : w.w;
  return (d >> (8 * (t & 3))) & 0xffu;
}

// 16 bytes starting at byte offset `a` of an LDS byte array whose base is 16B aligned.
// Five aligned dword reads + v_alignbyte (no unaligned LDS access).
__device__ __forceinline__ uint4 lds_win16(const uint8_t* lds, uint32_t a) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (a & ~3u));
  uint32_t s = (a & 3u) * 8u;
  uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
  uint4 r;
  r.x = __builtin_amdgcn_alignbit(w1, w0, s);
  r.y = __builtin_amdgcn_alignbit(w2, w1, s);
  r.z = __builtin_amdgcn_alignbit(w3, w2, s);
  r.w = __builtin_amdgcn_alignbit(w4, w3, s);
  return r;
}

__device__ __forceinline__ uint32_t lds_rd32(const uint8_t* lds, uint32_t a) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (a & ~3u));
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

// store the first m (0..16) bytes of w at p
__device__ __forceinline__ void store_bytes(uint8_t* p, uint4 w, uint32_t m) {
  if (m == 16) { *reinterpret_cast<v4u*>(p) = v4u{w.x, w.y, w.z, w.w}; return; }
  if (m & 8) { *reinterpret_cast<v2u*>(p) = v2u{w.x, w.y}; w = make_uint4(w.z, w.w, 0, 0); p += 8; }
  if (m & 4) { *reinterpret_cast<u32u*>(p) = w.x; w.x = w.y; p += 4; }
  if (m & 2) { *reinterpret_cast<u16u*>(p) = (uint16_t)w.x; w.x >>= 16; p += 2; }
  if (m & 1) { *p = (uint8_t)w.x; }
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    uint32_t t = __shfl_up(v, d, kWave);
    if (lane >= d) v += t;
  }
  return v;
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
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// varint_decode32 on global bytes d[0..avail), avail >= 1
__device__ uint32_t gdec32(const uint8_t* d, uint64_t avail, uint32_t& val) {
  uint32_t win = avail < 5 ? (uint32_t)avail : 5u;
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
  return o;
}

// ----------------------------------------------------------------------------------
// single-pass tiled decoder
// ----------------------------------------------------------------------------------
// A tile = up to `bpt` consecutive blocks of the batch, staged together in the LDS of
// one workgroup (256 threads).  Workgroups are persistent and take tiles t = blockIdx.x,
// + gridDim.x, ... (static round-robin; the grid never exceeds the resident capacity).
// Per tile:
//   stage -> parse trailers -> walk (one thread per restart interval, across all blocks
//   of the tile) -> tile-local scans -> publish the tile aggregate -> decoupled
//   look-back for the tile's global (record, key byte, value byte) prefix -> per-block
//   outputs -> second walk writes per-record metadata -> every thread copies records.
// Blocks that are not "regular" (see walk_interval) run the exact serial emulation.

constexpr uint32_t kNotStaged = 0xFFFFFFFFu;
constexpr uint64_t kFlagA = 1ull << 62;   // look-back word holds the tile aggregate
constexpr uint64_t kFlagP = 2ull << 62;   // look-back word holds the inclusive prefix
constexpr uint64_t kValMask = (1ull << 62) - 1;
constexpr int kThreads = 256;

template <int TB_, int MAXREC_, int MAXINT_, int MAXBLK_>
struct TileCfg {
  static constexpr int TB = TB_;          // staging bytes
  static constexpr int MAXREC = MAXREC_;  // records with metadata per tile
  static constexpr int MAXINT = MAXINT_;  // restart intervals per tile
  static constexpr int MAXBLK = MAXBLK_;  // blocks per tile
};

template <class C>
struct alignas(16) TileLds {
  uint8_t stage[C::TB];
  // per block of the tile
  uint32_t boff[C::MAXBLK];   // stage offset of block byte 0 (kNotStaged if not staged)
  uint32_t blen[C::MAXBLK];
  uint32_t bR[C::MAXBLK];     // restart offset
  uint32_t bn[C::MAXBLK];     // restart count
  uint32_t bint0[C::MAXBLK + 1];
  uint32_t bok[C::MAXBLK];    // 1 = regular fast path
  uint32_t bwr[C::MAXBLK];    // 1 = outputs of this block are written
  int32_t bst[C::MAXBLK];
  uint32_t bcnt[C::MAXBLK], bkb[C::MAXBLK], bvb[C::MAXBLK];   // block totals
  uint32_t brb[C::MAXBLK], bkbb[C::MAXBLK], bvbb[C::MAXBLK];  // tile-relative block bases
  // per restart interval: counts after walk 1, exclusive tile-relative bases after the scan
  uint32_t icnt[C::MAXINT + 1], ikb[C::MAXINT + 1], ivb[C::MAXINT + 1];
  uint8_t iblk[C::MAXINT];
  // per record (fast blocks), tile-relative index
  uint16_t rpos[C::MAXREC];   // block offset of the key suffix
  uint16_t rsh[C::MAXREC];
  uint16_t rns[C::MAXREC];
  uint16_t rvl[C::MAXREC];
  uint32_t rks[C::MAXREC];    // tile-relative key start
  uint32_t rvs[C::MAXREC];    // tile-relative value start
  uint8_t rblk[C::MAXREC];
  // tile scalars
  uint64_t tpre[3];           // global exclusive prefix of the tile (records, key bytes, value bytes)
  uint32_t ttot[3];           // tile totals
  uint32_t nfastrec;
  uint32_t wsum[4][3];        // per-wave scan totals
  uint32_t lbfirst[4][3];     // look-back: first P lane per wave
  uint64_t lbsum[4][3];       // look-back: per-wave partial sums
};

// Stage one block into a 16-byte aligned slot; returns the offset of block byte 0 within
// the slot (the block's global misalignment).  Reads stay inside [lo, hi).
__device__ __forceinline__ uint32_t stage_slot(uint8_t* slot, const uint8_t* gptr, uint32_t L, uintptr_t lo,
                                               uintptr_t hi, int lane) {
  uintptr_t ga = reinterpret_cast<uintptr_t>(gptr);
  uintptr_t a0 = ga & ~uintptr_t(15);
  uint32_t delta = (uint32_t)(ga - a0);
  uint32_t nch = (delta + L + 15u) >> 4;
  uint32_t c = lane;
  // main body: 4 independent 16-byte loads in flight per lane
  for (; c + 3 * kWave < nch; c += 4 * kWave) {
    uintptr_t a = a0 + 16u * c;
    if (a >= lo && a + 16 * (3 * kWave) + 16 <= hi) {
      uint4 v0 = *reinterpret_cast<const uint4*>(a);
      uint4 v1 = *reinterpret_cast<const uint4*>(a + 16 * kWave);
      uint4 v2 = *reinterpret_cast<const uint4*>(a + 32 * kWave);
      uint4 v3 = *reinterpret_cast<const uint4*>(a + 48 * kWave);
      *reinterpret_cast<uint4*>(slot + 16 * c) = v0;
      *reinterpret_cast<uint4*>(slot + 16 * (c + kWave)) = v1;
      *reinterpret_cast<uint4*>(slot + 16 * (c + 2 * kWave)) = v2;
      *reinterpret_cast<uint4*>(slot + 16 * (c + 3 * kWave)) = v3;
    } else {
      break;
    }
  }
  for (; c < nch; c += kWave) {
    uintptr_t a = a0 + 16u * c;
    uint4 v;
    if (a >= lo && a + 16 <= hi) {
      v = *reinterpret_cast<const uint4*>(a);
    } else {
      uint32_t t[4] = {0, 0, 0, 0};
      for (int i = 0; i < 16; ++i)
        if (a + i >= lo && a + i < hi) t[i >> 2] |= (uint32_t)(*reinterpret_cast<const uint8_t*>(a + i)) << (8 * (i & 3));
      v = make_uint4(t[0], t[1], t[2], t[3]);
    }
    *reinterpret_cast<uint4*>(slot + 16 * c) = v;
  }
  return delta;
}

// One restart interval [s, e) of a staged block (block byte 0 at stage offset bo).
// Regular-path preconditions (DESIGN.md "fast path"): every entry decodes without a
// reference panic; varints are terminated; the interval's first entry has shared == 0;
// later entries have shared <= previous key length (so Vec capacity never matters);
// field values fit 16 bits; the walk lands exactly on e.  Under these the reference's
// linear chain (src/block.rs:119-143) visits exactly these entries and rebuilds exactly
// these keys.  Returns false if they do not hold.
template <bool WRITE, class C>
__device__ __forceinline__ bool walk_interval(TileLds<C>& S, uint32_t bo, uint32_t L, uint32_t R, uint32_t s,
                                              uint32_t e, uint32_t& cnt, uint32_t& kb, uint32_t& vb, uint32_t rbase,
                                              uint32_t kbase, uint32_t vbase, uint32_t blk, uint32_t rlo,
                                              uint32_t rhi, uint32_t* key_end, uint32_t* val_end,
                                              uint32_t kend0, uint32_t vend0) {
  cnt = kb = vb = 0;
  if (!(s < e && e <= R)) return false;
  uint32_t p = s, prevlen = 0;
  bool first = true;
  while (p < e) {
    if (R - p < 3u) return false;                         // decode_entry Err -> panic
    const uint32_t* w = reinterpret_cast<const uint32_t*>(S.stage + ((bo + p) & ~3u));
    uint32_t sft = ((bo + p) & 3u) * 8u;
    uint32_t hw = __builtin_amdgcn_alignbit(w[1], w[0], sft);
    uint32_t sh = hw & 0xffu, ns = (hw >> 8) & 0xffu, vl = (hw >> 16) & 0xffu, h = 3;
    if ((hw & 0x808080u) != 0u) {                         // slow header path
      uint4 W = lds_win16(S.stage, bo + p);
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
    if (ns + vl > R - p - h) return false;                // no overflow: both < 2^16
    if (first ? (sh != 0) : (sh > prevlen)) return false;
    const uint32_t klen = sh + ns;
    if (klen > 0xFFFFu) return false;
    if (WRITE) {
      const uint32_t r = rbase + cnt;
      if (r >= rlo && r < rhi) {
        const uint32_t q = r - rlo;
        S.rpos[q] = (uint16_t)(p + h);
        S.rsh[q] = (uint16_t)sh;
        S.rns[q] = (uint16_t)ns;
        S.rvl[q] = (uint16_t)vl;
        S.rks[q] = kbase + kb;
        S.rvs[q] = vbase + vb;
        S.rblk[q] = (uint8_t)blk;
      }
      if (key_end) {
        key_end[cnt] = kend0 + kb + klen;
        val_end[cnt] = vend0 + vb + vl;
      }
    }
    cnt += 1;
    kb += klen;
    vb += vl;
    prevlen = klen;
    first = false;
    p += h + ns + vl;
  }
  return p == e;
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

struct TileArgs {
  const uint8_t* data;
  uint64_t data_len;
  const uint64_t* blk_off;
  const uint32_t* blk_len;
  uint32_t nblk;
  uint32_t bpt;     // blocks per tile
  uint32_t slot;    // staging slot bytes per block (multiple of 16)
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
  uint64_t* lb;     // [ntiles * 3] look-back words, zeroed before launch
  uint64_t* dbg;    // [16] phase stamps (diagnostic build only)
  int write;
};

// Decoupled look-back over a workgroup-wide window: publish the tile aggregate (flag A),
// then read predecessors back in windows of 256 tiles (one per thread) until every
// quantity meets an inclusive prefix (flag P); publish our own P.  A 256-wide window
// lets the inclusive-prefix front advance 256 tiles per round trip, so the tiles of a
// persistent round do not serialise on each other.  Look-back words are single 8-byte
// agent-scope atomics: the value IS the flag, no fence needed (MI355X_MICROARCH.md,
// hand-off granules).  Spins are bounded: on timeout bit1 of totals[3] is set.
template <class C>
__device__ void tile_lookback(TileLds<C>& S, uint64_t* lb, uint32_t t, uint64_t* totals) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t agg[3] = {S.ttot[0], S.ttot[1], S.ttot[2]};
  if (t == 0) {
    if (tid < 3) __hip_atomic_store(&lb[tid], kFlagP | agg[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) { S.tpre[0] = S.tpre[1] = S.tpre[2] = 0; }
    return;
  }
  if (tid < 3)
    __hip_atomic_store(&lb[3ull * t + tid], kFlagA | agg[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t acc[3] = {0, 0, 0};
  bool done[3] = {false, false, false};
  int64_t base = (int64_t)t - 1;
  bool timeout = false;
  while (!(done[0] && done[1] && done[2])) {
    const int64_t p = base - tid;
    uint64_t w[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      w[q] = kFlagP;  // before tile 0: inclusive prefix 0
      if (done[q]) continue;
      if (p >= 0) {
        uint32_t spins = 0;
        for (;;) {
          w[q] = __hip_atomic_load(&lb[3ull * p + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (w[q] >> 62) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > (1u << 22)) { timeout = true; w[q] = kFlagP; break; }
        }
      }
      const uint64_t pm = __ballot((w[q] >> 62) == 2u);
      if (lane == 0) S.lbfirst[wv][q] = pm ? (uint32_t)__builtin_ctzll(pm) : 64u;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (done[q]) continue;
      uint32_t gfirst = kThreads;
      for (int k = 0; k < kThreads / kWave; ++k)
        if (S.lbfirst[k][q] < 64u) { gfirst = k * kWave + S.lbfirst[k][q]; break; }
      uint64_t v = w[q] & kValMask;
      if ((uint32_t)tid > gfirst) v = 0;
      const uint64_t ws = wave_sum64(v);
      if (lane == 0) S.lbsum[wv][q] = ws;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (done[q]) continue;
      for (int k = 0; k < kThreads / kWave; ++k) acc[q] += S.lbsum[k][q];
      for (int k = 0; k < kThreads / kWave; ++k)
        if (S.lbfirst[k][q] < 64u) done[q] = true;
    }
    __syncthreads();
    base -= kThreads;
  }
  if (tid < 3)
    __hip_atomic_store(&lb[3ull * t + tid], kFlagP | (acc[tid] + agg[tid]), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (timeout) atomicOr(reinterpret_cast<unsigned long long*>(totals + 3), 2ull);
  if (tid == 0) { S.tpre[0] = acc[0]; S.tpre[1] = acc[1]; S.tpre[2] = acc[2]; }
}

template <class C>
__global__ void __launch_bounds__(kThreads) k_decode_tiles(TileArgs a) {
  __shared__ TileLds<C> S;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(a.data), hi = lo + a.data_len;
#ifdef MTBLX_STAMPS
  // diagnostic build only: per-phase cycles of thread 0 (s_memtime), summed over tiles
  uint64_t tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tprev = __builtin_amdgcn_s_memtime(), ntl = 0;
#define STAMP(k) do { if (tid == 0) { const uint64_t _t = __builtin_amdgcn_s_memtime(); tacc[k] += _t - tprev; tprev = _t; } } while (0)
#else
#define STAMP(k) do { } while (0)
#endif

  for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const uint32_t b0 = t * a.bpt;
    const uint32_t nb = min(a.bpt, a.nblk - b0);
#ifdef MTBLX_STAMPS
    ++ntl;
#endif
    STAMP(7);

    // ---- 1. stage: wave w stages blocks w, w+4, ... ----
    for (uint32_t j = wv; j < nb; j += kThreads / kWave) {
      const uint32_t L = a.blk_len[b0 + j];
      const uint8_t* g = a.data + a.blk_off[b0 + j];
      const uint32_t so = 16u + j * a.slot;
      uint32_t bo = kNotStaged;
      if (L + 15u <= a.slot && so + a.slot + 32u <= (uint32_t)C::TB) bo = so + stage_slot(S.stage + so, g, L, lo, hi, lane);
      if (lane == 0) { S.boff[j] = bo; S.blen[j] = L; }
    }
    __syncthreads();
    STAMP(0);

    // ---- 2. trailers (Block::init, src/block.rs:16-49) ----
    if (tid < (int)nb) {
      const uint32_t j = tid, L = S.blen[j], bo = S.boff[j];
      uint32_t n = 0, R = 0, ok = 0;
      if (bo != kNotStaged && L >= 8) {
        n = lds_rd32(S.stage, bo + L - 4);
        if (n != 0 && (uint64_t)(n + 1ull) * 4ull <= L) { R = L - 4u * (n + 1u); ok = 1; }
      }
      S.bn[j] = ok ? n : 0;
      S.bR[j] = R;
      S.bok[j] = ok;
      S.bwr[j] = 1;
      S.bst[j] = MTBLX_ST_OK;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t f = 0;
      for (uint32_t j = 0; j < nb; ++j) {
        S.bint0[j] = f;
        if (S.bok[j] && f + S.bn[j] <= (uint32_t)C::MAXINT) f += S.bn[j];
        else S.bok[j] = 0;
      }
      S.bint0[nb] = f;
    }
    __syncthreads();
    const uint32_t nint = S.bint0[nb];

    // ---- 3. walk 1: one thread per restart interval across the tile ----
    for (uint32_t f = tid; f < nint; f += kThreads) {
      uint32_t j = 0;
      while (S.bint0[j + 1] <= f) ++j;
      const uint32_t i = f - S.bint0[j], bo = S.boff[j], L = S.blen[j], R = S.bR[j], n = S.bn[j];
      const uint32_t s = lds_rd32(S.stage, bo + R + 4u * i);
      const uint32_t e = (i + 1 < n) ? lds_rd32(S.stage, bo + R + 4u * (i + 1)) : R;
      uint32_t cnt, kb, vb;
      const bool ok = walk_interval<false, C>(S, bo, L, R, s, e, cnt, kb, vb, 0, 0, 0, 0, 0, 0, nullptr, nullptr, 0, 0) &&
                      cnt <= (uint32_t)C::MAXREC;
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
      GenOut o = generic_block<false>(d, L, nullptr, nullptr, nullptr, nullptr);
      S.bcnt[j] = o.nrec;
      S.bkb[j] = (uint32_t)o.kb;
      S.bvb[j] = (uint32_t)o.vb;
      S.bst[j] = o.st;
    }
    // scan of interval counts (regular blocks only) -> tile-relative interval bases
    // (MAXINT <= 256: one interval per thread)
    {
      uint32_t xc = 0, xk = 0, xv = 0;
      const uint32_t f = tid;
      if (f < nint && S.bok[S.iblk[f]]) { xc = S.icnt[f]; xk = S.ikb[f]; xv = S.ivb[f]; }
      uint32_t tot[3];
      wg_excl_scan3(S, xc, xk, xv, tot);
      if (f < nint) { S.icnt[f] = xc; S.ikb[f] = xk; S.ivb[f] = xv; }
      if (tid == 0) { S.icnt[nint] = tot[0]; S.ikb[nint] = tot[1]; S.ivb[nint] = tot[2]; }
    }
    __syncthreads();
    // block totals + tile-relative block bases (serial over <= MAXBLK blocks)
    if (tid == 0) {
      uint32_t rr = 0, rk = 0, rv = 0, fastrec = 0;
      for (uint32_t j = 0; j < nb; ++j) {
        if (S.bok[j]) {
          const uint32_t fa = S.bint0[j], fb = S.bint0[j + 1];
          S.bcnt[j] = S.icnt[fb] - S.icnt[fa];
          S.bkb[j] = S.ikb[fb] - S.ikb[fa];
          S.bvb[j] = S.ivb[fb] - S.ivb[fa];
          fastrec += S.bcnt[j];
        }
        S.brb[j] = rr; S.bkbb[j] = rk; S.bvbb[j] = rv;
        rr += S.bcnt[j]; rk += S.bkb[j]; rv += S.bvb[j];
      }
      S.ttot[0] = rr; S.ttot[1] = rk; S.ttot[2] = rv;
      S.nfastrec = fastrec;
    }
    __syncthreads();

    // ---- 5. publish aggregate + decoupled look-back (whole workgroup) ----
    STAMP(2);
    tile_lookback<C>(S, a.lb, t, a.totals);
    __syncthreads();
    if (tid == 0 && t == a.ntiles - 1) {
      a.totals[0] = S.tpre[0] + S.ttot[0];
      a.totals[1] = S.tpre[1] + S.ttot[1];
      a.totals[2] = S.tpre[2] + S.ttot[2];
    }
    STAMP(3);
    const uint64_t pr = S.tpre[0], pk = S.tpre[1], pv = S.tpre[2];

    // ---- 6. per-block outputs + capacity check ----
    if (tid < (int)nb) {
      const uint32_t j = tid, b = b0 + j;
      const uint64_t rb = pr + S.brb[j], kb = pk + S.bkbb[j], vb = pv + S.bvbb[j];
      a.nrec[b] = S.bcnt[j];
      a.rec_base[b] = rb;
      a.key_base[b] = kb;
      a.val_base[b] = vb;
      int32_t st = S.bst[j];
      if (a.write && (rb + S.bcnt[j] > a.rec_cap || kb + S.bkb[j] > a.keys_cap || vb + S.bvb[j] > a.vals_cap)) {
        st = MTBLX_ST_OVERFLOW;
        S.bwr[j] = 0;
        atomicOr(reinterpret_cast<unsigned long long*>(a.totals + 3), 1ull);
      }
      a.status[b] = st;
    }
    if (!a.write) { __syncthreads(); continue; }
    __syncthreads();

    STAMP(4);
    // ---- 7. walk 2 (metadata) + copy, in chunks of whole intervals of <= MAXREC records ----
    // icnt[f] = regular records before interval f (irregular blocks contribute 0), so
    // icnt is the metadata slot numbering and is monotone: chunks are found by search.
    for (uint32_t fa = 0; fa < nint;) {
      uint32_t fb;
      {
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
      }
      const uint32_t rlo = S.icnt[fa], rhi = S.icnt[fb];
      for (uint32_t f = fa + tid; f < fb; f += kThreads) {
        const uint32_t j = S.iblk[f];
        if (!S.bok[j]) continue;
        const uint32_t fj = S.bint0[j];
        const uint32_t i = f - fj, bo = S.boff[j], L = S.blen[j], R = S.bR[j], n = S.bn[j];
        const uint32_t s = lds_rd32(S.stage, bo + R + 4u * i);
        const uint32_t e = (i + 1 < n) ? lds_rd32(S.stage, bo + R + 4u * (i + 1)) : R;
        const uint32_t kin = S.ikb[f] - S.ikb[fj], vin = S.ivb[f] - S.ivb[fj];  // bytes before f in block
        const uint32_t rin = S.icnt[f] - S.icnt[fj];                             // records before f in block
        uint32_t* ke = S.bwr[j] ? a.key_end + pr + S.brb[j] + rin : nullptr;
        uint32_t* ve = S.bwr[j] ? a.val_end + pr + S.brb[j] + rin : nullptr;
        uint32_t c, k, v;
        walk_interval<true, C>(S, bo, L, R, s, e, c, k, v, S.icnt[f], S.bkbb[j] + kin, S.bvbb[j] + vin, j, rlo, rhi,
                               ke, ve, kin, vin);
      }
      __syncthreads();
      STAMP(5);
      // copy: one thread per record
      for (uint32_t q = tid; q < rhi - rlo; q += kThreads) {
        const uint32_t j = S.rblk[q];
        if (!S.bwr[j]) continue;
        const uint32_t bo = S.boff[j];
        const uint32_t vl = S.rvl[q];
        const uint32_t vsrc = bo + S.rpos[q] + S.rns[q];
        uint8_t* vd = a.vals + pv + S.rvs[q];
        for (uint32_t o = 0; o < vl; o += 16) {
          uint4 wv4 = lds_win16(S.stage, vsrc + o);
          const uint32_t m = vl - o;
          store_bytes(vd + o, wv4, m < 16 ? m : 16);
        }
        const uint32_t shr = S.rsh[q];
        const uint32_t klen = shr + S.rns[q];
        uint8_t* kd = a.keys + pk + S.rks[q];
        for (uint32_t j0 = 0; j0 < klen; j0 += 16) {
          const uint32_t jend = (j0 + 16 < klen) ? j0 + 16 : klen;
          uint4 outw = make_uint4(0, 0, 0, 0);
          uint32_t jj = j0;
          while (jj < jend) {
            // source of key byte jj: the latest record s <= q with shared_s <= jj (same interval;
            // the interval's first record has shared 0 and lies in this chunk)
            uint32_t sidx = q, m = klen, shs = shr;
            while (shs > jj) {
              m = shs < m ? shs : m;
              --sidx;
              shs = S.rsh[sidx];
            }
            const uint32_t seg = m < jend ? m : jend;
            const uint32_t src = bo + S.rpos[sidx] + (jj - shs);
            uint4 w4 = lds_win16(S.stage, src - (jj - j0));
            merge_bytes(outw, w4, (int)(jj - j0), (int)(seg - j0));
            jj = seg;
          }
          store_bytes(kd + j0, outw, jend - j0);
        }
      }
      __syncthreads();
      STAMP(6);
      fa = fb;
    }

    // ---- 8. irregular blocks: exact serial write (lane per block) ----
    if (tid < (int)nb && !S.bok[tid] && S.bwr[tid]) {
      const uint32_t j = tid, bo = S.boff[j], L = S.blen[j];
      const uint8_t* d = (bo != kNotStaged) ? (S.stage + bo) : (a.data + a.blk_off[b0 + j]);
      generic_block<true>(d, L, a.keys + pk + S.bkbb[j], a.vals + pv + S.bvbb[j], a.key_end + pr + S.brb[j],
                          a.val_end + pr + S.brb[j]);
    }
    __syncthreads();
  }
#ifdef MTBLX_STAMPS
  if (tid == 0 && a.dbg) {
    for (int k = 0; k < 8; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg + k), (unsigned long long)tacc[k]);
    atomicAdd(reinterpret_cast<unsigned long long*>(a.dbg + 8), (unsigned long long)ntl);
  }
#endif
}

using CfgSmall = TileCfg<32768, 512, 128, 16>;
using CfgLarge = TileCfg<67584, 1024, 256, 4>;

}  // namespace mtblx

// ----------------------------------------------------------------------------------
// launch glue (called from mtblx_api.cpp)
// ----------------------------------------------------------------------------------
using namespace mtblx;

namespace {
struct Plan {
  uint32_t bpt, slot, ntiles;
  bool large;
};

Plan make_plan(uint32_t nblk, uint32_t max_len) {
  Plan p{};
  const uint32_t slot = ((max_len + 15u + 15u) / 16u) * 16u;
  uint32_t usable = CfgSmall::TB - 48;
  if (max_len != 0 && slot <= usable) {
    p.large = false;
    p.slot = slot;
    p.bpt = std::min<uint32_t>(usable / slot, CfgSmall::MAXBLK);
  } else {
    usable = CfgLarge::TB - 48;
    p.large = true;
    p.slot = (max_len != 0 && slot <= usable) ? slot : usable;
    p.bpt = std::max<uint32_t>(1, std::min<uint32_t>(usable / p.slot, CfgLarge::MAXBLK));
  }
  p.ntiles = (nblk + p.bpt - 1) / p.bpt;
  return p;
}

template <class C>
int resident_grid(uint32_t ntiles) {
  static int cached = 0;
  if (!cached) {
    int dev = 0, ncu = 0, occ = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_decode_tiles<C>, kThreads, 0) != hipSuccess || occ < 1)
      occ = 1;
    int lds_lim = (int)((160u * 1024u) / sizeof(TileLds<C>));
    if (lds_lim < 1) lds_lim = 1;
    cached = std::max(1, ncu * std::min(occ, lds_lim));
  }
  return (int)std::min<uint32_t>(ntiles, (uint32_t)cached);
}
}  // namespace

// workspace: [0, 256) diagnostic stamps | look-back words (worst case one block per tile)
extern "C" size_t mtblx_impl_ws_bytes(uint32_t nblk) { return 256u + (size_t)nblk * 24u + 64u; }

extern "C" int mtblx_impl_run(const mtblx_block_batch* in, const mtblx_decoded* out, void* ws, int write,
                              hipStream_t s) {
  const uint32_t nblk = in->nblk;
  const Plan p = make_plan(nblk, in->max_blk_len);
  uint64_t* dbg = reinterpret_cast<uint64_t*>(ws);
  uint64_t* lb = dbg + 32;
  if (hipMemsetAsync(ws, 0, 256u + (size_t)p.ntiles * 24u, s) != hipSuccess) return MTBLX_E_HIP;
  if (hipMemsetAsync(out->totals, 0, 32, s) != hipSuccess) return MTBLX_E_HIP;
  TileArgs a{in->data,     in->data_len,  in->blk_off,  in->blk_len,   nblk,         p.bpt,         p.slot,
             p.ntiles,     out->nrec,     out->rec_base, out->key_base, out->val_base, out->status, out->key_end,
             out->val_end, out->rec_cap,  out->keys,    out->keys_cap, out->vals,    out->vals_cap, out->totals,
             lb,           dbg,           write ? 1 : 0};
  if (p.large) {
    hipLaunchKernelGGL(k_decode_tiles<CfgLarge>, dim3(resident_grid<CfgLarge>(p.ntiles)), dim3(kThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL(k_decode_tiles<CfgSmall>, dim3(resident_grid<CfgSmall>(p.ntiles)), dim3(kThreads), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
