// decode.hip — MI355X (gfx950) kernels for mtbl data-block decode.
//
// Replaces the reference's per-record CPU scan of one block
//   Block::init            /root/reference/src/block.rs:16-49
//   BlockIter::init        src/block.rs:75-93
//   seek_to_first / next / get / parse_next_key / decode_entry   src/block.rs:119-238
//   varint_decode32        src/varint.rs:44-61
// with a batched device decode of many blocks, laid out contiguously (include/mtblx.h).
//
// Kernel pipeline (two-pass form; DESIGN.md "Kernels"):
//   k_count   one wave per block: stage block HBM->LDS, walk the restart intervals in
//             parallel (one lane per interval), validate the "regular" fast path, count
//             records / key bytes / value bytes.  Irregular blocks run the exact serial
//             emulation (generic path) in lane 0 instead.
//   k_scan_*  exclusive prefix sums over blocks -> rec_base / key_base / val_base.
//   k_decode  one wave per block: stage, walk twice (counts, then per-record metadata
//             into LDS), then every lane copies whole records: value bytes LDS->HBM,
//             key bytes resolved through the shared-prefix chain straight from the
//             staged suffix bytes (no per-key serial rebuild).
//
// Everything is integer/byte work: HBM-bandwidth bound, no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

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
// per-wave LDS state of the fast path
// ----------------------------------------------------------------------------------
template <int STAGE>
struct alignas(16) WaveLds {
  static constexpr int kMaxRec = STAGE / 16;   // avg record >= 16 B, else generic path
  static constexpr int kMaxInt = 256;          // restart intervals handled by the fast path
  uint8_t stage[STAGE + 64];                   // 16 B front pad; block byte i at boff + i
  uint16_t rpos[kMaxRec];                      // block offset of the key suffix
  uint16_t rsh[kMaxRec];                       // shared
  uint16_t rns[kMaxRec];                       // non_shared
  uint16_t rvl[kMaxRec];                       // value_length
  uint16_t rks[kMaxRec];                       // key start, relative to the block's key base
  uint16_t rvs[kMaxRec];                       // value start, relative to the block's value base
  uint16_t ibr[kMaxInt];                       // per-interval record base
  uint16_t ibk[kMaxInt];                       // per-interval key-byte base
  uint16_t ibv[kMaxInt];                       // per-interval value-byte base
};

// Stage block [gbase, gbase+L) into lds.stage; returns boff (stage offset of byte 0).
// data_lo/data_hi bound the readable device range.
__device__ __forceinline__ uint32_t stage_block(uint8_t* stage, const uint8_t* gptr, uint32_t L,
                                                const uint8_t* data_lo, const uint8_t* data_hi, int lane) {
  uintptr_t ga = reinterpret_cast<uintptr_t>(gptr);
  uintptr_t a0 = ga & ~uintptr_t(15);
  uint32_t delta = (uint32_t)(ga - a0);
  uint32_t nch = (delta + L + 15u) >> 4;
  uintptr_t lo = reinterpret_cast<uintptr_t>(data_lo), hi = reinterpret_cast<uintptr_t>(data_hi);
  for (uint32_t c = lane; c < nch; c += kWave) {
    uintptr_t a = a0 + 16u * c;
    uint4 v;
    if (a >= lo && a + 16 <= hi) {
      v = *reinterpret_cast<const uint4*>(a);
    } else {
      uint8_t t[16];
      for (int i = 0; i < 16; ++i) t[i] = (a + i >= lo && a + i < hi) ? *reinterpret_cast<const uint8_t*>(a + i) : 0;
      v = make_uint4((uint32_t)t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24,
                     (uint32_t)t[4] | (uint32_t)t[5] << 8 | (uint32_t)t[6] << 16 | (uint32_t)t[7] << 24,
                     (uint32_t)t[8] | (uint32_t)t[9] << 8 | (uint32_t)t[10] << 16 | (uint32_t)t[11] << 24,
                     (uint32_t)t[12] | (uint32_t)t[13] << 8 | (uint32_t)t[14] << 16 | (uint32_t)t[15] << 24);
    }
    *reinterpret_cast<uint4*>(stage + 16 + 16 * c) = v;
  }
  return 16u + delta;
}

// One restart interval [s, e) of a staged block.  Fast-path preconditions:
// every entry decodes without a reference panic, the interval's first entry has
// shared == 0, later entries have shared <= previous key length, the walk lands exactly
// on e.  Under these the reference's linear chain (src/block.rs:119-143) visits exactly
// these entries and rebuilds exactly these keys.  Returns false if not satisfied.
template <bool PASS2, int STAGE>
__device__ __forceinline__ bool walk_interval(WaveLds<STAGE>& S, uint32_t boff, uint32_t L, uint32_t R,
                                              uint32_t s, uint32_t e, uint32_t& cnt, uint32_t& kb, uint32_t& vb,
                                              uint32_t rbase, uint32_t kbase, uint32_t vbase, uint32_t* key_end,
                                              uint32_t* val_end) {
  cnt = kb = vb = 0;
  if (!(s < e && e <= R)) return false;
  uint32_t p = s, prevlen = 0;
  bool first = true;
  while (p < e) {
    if (R - p < 3u) return false;                         // decode_entry Err -> panic
    uint4 W = lds_win16(S.stage, boff + p);
    uint32_t sh = W.x & 0xffu, ns = (W.x >> 8) & 0xffu, vl = (W.x >> 16) & 0xffu, h = 3;
    if ((sh | ns | vl) >= 128u) {                         // slow header path
      uint32_t l0 = dec32(W, 0, L - p, sh);
      if (l0 == 0) return false;
      uint32_t l1 = dec32(W, l0, L - p - l0, ns);
      if (l1 == 0) return false;
      uint32_t l2 = dec32(W, l0 + l1, L - p - l0 - l1, vl);
      if (l2 == 0) return false;
      h = l0 + l1 + l2;
      if (p + h > R) return false;                        // assert!(p <= limit)
    }
    if ((uint64_t)ns + vl > (uint64_t)(R - p - h)) return false;
    if (first ? (sh != 0) : (sh > prevlen)) return false;
    uint32_t klen = sh + ns;
    if (klen > 0xFFFFu) return false;
    if (PASS2) {
      uint32_t r = rbase + cnt;
      S.rpos[r] = (uint16_t)(p + h);
      S.rsh[r] = (uint16_t)sh;
      S.rns[r] = (uint16_t)ns;
      S.rvl[r] = (uint16_t)vl;
      S.rks[r] = (uint16_t)(kbase + kb);
      S.rvs[r] = (uint16_t)(vbase + vb);
      key_end[r] = kbase + kb + klen;
      val_end[r] = vbase + vb + vl;
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
// fast-path block analysis shared by count and decode
// ----------------------------------------------------------------------------------
struct FastInfo {
  bool ok;
  uint32_t nrec, kb, vb;
  uint32_t L, R, n, boff;
};

// Walk pass 1 over all intervals of a staged block; fills S.ib* with exclusive bases.
template <int STAGE>
__device__ FastInfo fast_analyze(WaveLds<STAGE>& S, uint32_t boff, uint32_t L, int lane) {
  FastInfo fi{false, 0, 0, 0, L, 0, 0, boff};
  if (L < 8 || L > (uint32_t)STAGE) return fi;
  uint32_t n = lds_rd32(S.stage, boff + L - 4);
  if (n == 0 || (uint64_t)(n + 1ull) * 4ull > L) return fi;
  if (n > (uint32_t)WaveLds<STAGE>::kMaxInt) return fi;
  uint32_t R = L - 4u * (n + 1u);
  fi.R = R;
  fi.n = n;
  bool ok = true;
  uint32_t rb = 0, kbt = 0, vbt = 0;
  for (uint32_t c0 = 0; c0 < n; c0 += kWave) {
    uint32_t i = c0 + lane;
    uint32_t cnt = 0, kb = 0, vb = 0;
    bool lok = true;
    if (i < n) {
      uint32_t s = lds_rd32(S.stage, boff + R + 4u * i);
      uint32_t e = (i + 1 < n) ? lds_rd32(S.stage, boff + R + 4u * (i + 1)) : R;
      lok = walk_interval<false>(S, boff, L, R, s, e, cnt, kb, vb, 0, 0, 0, nullptr, nullptr);
    }
    ok = ok && (__ballot(!lok) == 0ull);
    uint32_t ic = wave_incl_scan(cnt, lane);
    uint32_t ik = wave_incl_scan(kb, lane);
    uint32_t iv = wave_incl_scan(vb, lane);
    if (i < n) {
      S.ibr[i] = (uint16_t)(rb + ic - cnt);
      S.ibk[i] = (uint16_t)(kbt + ik - kb);
      S.ibv[i] = (uint16_t)(vbt + iv - vb);
    }
    rb += __shfl(ic, kWave - 1, kWave);
    kbt += __shfl(ik, kWave - 1, kWave);
    vbt += __shfl(iv, kWave - 1, kWave);
    if (rb > (uint32_t)WaveLds<STAGE>::kMaxRec || kbt > 0xFFFFu) ok = false;
  }
  fi.ok = ok;
  fi.nrec = rb;
  fi.kb = kbt;
  fi.vb = vbt;
  return fi;
}

// ----------------------------------------------------------------------------------
// kernels
// ----------------------------------------------------------------------------------
struct CountArgs {
  const uint8_t* data;
  uint64_t data_len;
  const uint64_t* blk_off;
  const uint32_t* blk_len;
  uint32_t nblk;
  uint32_t* nrec;
  uint64_t* kb;
  uint64_t* vb;
  int32_t* status;
};

template <int STAGE, int WPG>
__global__ void __launch_bounds__(WPG * 64) k_count(CountArgs a) {
  __shared__ WaveLds<STAGE> lds[WPG];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x * WPG + w;
  if (b >= a.nblk) return;
  WaveLds<STAGE>& S = lds[w];
  const uint32_t L = a.blk_len[b];
  const uint8_t* g = a.data + a.blk_off[b];
  FastInfo fi{false, 0, 0, 0, L, 0, 0, 0};
  if (L >= 8 && L <= (uint32_t)STAGE) {
    uint32_t boff = stage_block(S.stage, g, L, a.data, a.data + a.data_len, lane);
    wave_sync();
    fi = fast_analyze<STAGE>(S, boff, L, lane);
  }
  if (fi.ok) {
    if (lane == 0) {
      a.nrec[b] = fi.nrec;
      a.kb[b] = fi.kb;
      a.vb[b] = fi.vb;
      a.status[b] = MTBLX_ST_OK;
    }
  } else if (lane == 0) {
    GenOut o = generic_block<false>(g, L, nullptr, nullptr, nullptr, nullptr);
    a.nrec[b] = o.nrec;
    a.kb[b] = o.kb;
    a.vb[b] = o.vb;
    a.status[b] = o.st;
  }
}

struct DecodeArgs {
  const uint8_t* data;
  uint64_t data_len;
  const uint64_t* blk_off;
  const uint32_t* blk_len;
  uint32_t nblk;
  const uint32_t* nrec;
  const uint64_t* kbytes;
  const uint64_t* vbytes;
  const uint64_t* rec_base;
  const uint64_t* key_base;
  const uint64_t* val_base;
  int32_t* status;
  uint32_t* key_end;
  uint32_t* val_end;
  uint64_t rec_cap;
  uint8_t* keys;
  uint64_t keys_cap;
  uint8_t* vals;
  uint64_t vals_cap;
  uint64_t* totals;
};

template <int STAGE, int WPG>
__global__ void __launch_bounds__(WPG * 64) k_decode(DecodeArgs a) {
  __shared__ WaveLds<STAGE> lds[WPG];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const uint32_t b = blockIdx.x * WPG + w;
  if (b >= a.nblk) return;
  WaveLds<STAGE>& S = lds[w];
  const uint32_t L = a.blk_len[b];
  const uint8_t* g = a.data + a.blk_off[b];
  const uint64_t rb = a.rec_base[b], kb0 = a.key_base[b], vb0 = a.val_base[b];
  const uint32_t nr = a.nrec[b];
  if (rb + nr > a.rec_cap || kb0 + a.kbytes[b] > a.keys_cap || vb0 + a.vbytes[b] > a.vals_cap) {
    if (lane == 0) {
      a.status[b] = MTBLX_ST_OVERFLOW;
      atomicOr(reinterpret_cast<unsigned long long*>(a.totals + 3), 1ull);
    }
    return;
  }
  uint32_t* key_end = a.key_end + rb;
  uint32_t* val_end = a.val_end + rb;
  uint8_t* keys = a.keys + kb0;
  uint8_t* vals = a.vals + vb0;

  FastInfo fi{false, 0, 0, 0, L, 0, 0, 0};
  uint32_t boff = 0;
  if (L >= 8 && L <= (uint32_t)STAGE) {
    boff = stage_block(S.stage, g, L, a.data, a.data + a.data_len, lane);
    wave_sync();
    fi = fast_analyze<STAGE>(S, boff, L, lane);
  }
  if (!fi.ok) {
    if (lane == 0) generic_block<true>(g, L, keys, vals, key_end, val_end);
    return;
  }
  // pass 2: per-record metadata into LDS, key_end/val_end to HBM
  const uint32_t R = fi.R, n = fi.n;
  for (uint32_t i = lane; i < n; i += kWave) {
    uint32_t s = lds_rd32(S.stage, boff + R + 4u * i);
    uint32_t e = (i + 1 < n) ? lds_rd32(S.stage, boff + R + 4u * (i + 1)) : R;
    uint32_t c, k, v;
    walk_interval<true>(S, boff, L, R, s, e, c, k, v, S.ibr[i], S.ibk[i], S.ibv[i], key_end, val_end);
  }
  wave_sync();
  // copy: one lane per record
  for (uint32_t r = lane; r < fi.nrec; r += kWave) {
    const uint32_t vl = S.rvl[r];
    const uint32_t vsrc = boff + S.rpos[r] + S.rns[r];
    uint8_t* vd = vals + S.rvs[r];
    for (uint32_t o = 0; o < vl; o += 16) {
      uint4 wv = lds_win16(S.stage, vsrc + o);
      uint32_t m = vl - o;
      store_bytes(vd + o, wv, m < 16 ? m : 16);
    }
    const uint32_t shr = S.rsh[r];
    const uint32_t klen = shr + S.rns[r];
    uint8_t* kd = keys + S.rks[r];
    for (uint32_t j0 = 0; j0 < klen; j0 += 16) {
      const uint32_t jend = (j0 + 16 < klen) ? j0 + 16 : klen;
      uint4 outw = make_uint4(0, 0, 0, 0);
      uint32_t j = j0;
      while (j < jend) {
        // source of key byte j: the latest record s <= r with shared_s <= j
        uint32_t s = r, m = klen, shs = shr;
        while (shs > j) {
          m = shs < m ? shs : m;
          --s;
          shs = S.rsh[s];
        }
        const uint32_t seg = m < jend ? m : jend;
        const uint32_t src = boff + S.rpos[s] + (j - shs);
        uint4 wv = lds_win16(S.stage, src - (j - j0));
        merge_bytes(outw, wv, (int)(j - j0), (int)(seg - j0));
        j = seg;
      }
      store_bytes(kd + j0, outw, jend - j0);
    }
  }
}

// ----------------------------------------------------------------------------------
// scan over blocks: (nrec, key bytes, value bytes) -> exclusive bases + totals
// ----------------------------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

struct Trip {
  uint64_t r, k, v;
};
__device__ __forceinline__ Trip tadd(Trip a, Trip b) { return Trip{a.r + b.r, a.k + b.k, a.v + b.v}; }

__device__ Trip block_excl_scan(Trip x, Trip* sh, Trip& total) {
  // Hillis-Steele over 256 threads in LDS (scan kernels are a tiny share of the time)
  const int t = threadIdx.x;
  sh[t] = x;
  __syncthreads();
  for (int d = 1; d < kScanThreads; d <<= 1) {
    Trip y = (t >= d) ? sh[t - d] : Trip{0, 0, 0};
    __syncthreads();
    if (t >= d) sh[t] = tadd(sh[t], y);
    __syncthreads();
  }
  total = sh[kScanThreads - 1];
  Trip incl = sh[t];
  __syncthreads();
  return Trip{incl.r - x.r, incl.k - x.k, incl.v - x.v};
}

__global__ void __launch_bounds__(kScanThreads) k_scan_partial(const uint32_t* nrec, const uint64_t* kb,
                                                                const uint64_t* vb, uint32_t nblk, Trip* part) {
  __shared__ Trip sh[kScanThreads];
  Trip acc{0, 0, 0};
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  for (int i = 0; i < kScanItems; ++i) {
    uint64_t b = base + (uint64_t)i * kScanThreads + threadIdx.x;
    if (b < nblk) acc = tadd(acc, Trip{nrec[b], kb[b], vb[b]});
  }
  Trip tot;
  block_excl_scan(acc, sh, tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(kScanThreads) k_scan_top(Trip* part, uint32_t nparts, uint64_t* totals) {
  __shared__ Trip sh[kScanThreads];
  Trip carry{0, 0, 0};
  for (uint32_t c0 = 0; c0 < nparts; c0 += kScanThreads) {
    uint32_t i = c0 + threadIdx.x;
    Trip x = (i < nparts) ? part[i] : Trip{0, 0, 0};
    Trip tot;
    Trip ex = block_excl_scan(x, sh, tot);
    if (i < nparts) part[i] = tadd(carry, ex);
    carry = tadd(carry, tot);
  }
  if (threadIdx.x == 0) {
    totals[0] = carry.r;
    totals[1] = carry.k;
    totals[2] = carry.v;
    totals[3] = 0;
  }
}

__global__ void __launch_bounds__(kScanThreads) k_scan_final(const uint32_t* nrec, const uint64_t* kb,
                                                              const uint64_t* vb, uint32_t nblk, const Trip* part,
                                                              uint64_t* rec_base, uint64_t* key_base,
                                                              uint64_t* val_base) {
  __shared__ Trip sh[kScanThreads];
  // thread t owns items base + t*kScanItems .. +kScanItems (contiguous)
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  Trip loc[kScanItems];
  Trip acc{0, 0, 0};
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    uint64_t b = base + i;
    loc[i] = (b < nblk) ? Trip{nrec[b], kb[b], vb[b]} : Trip{0, 0, 0};
    acc = tadd(acc, loc[i]);
  }
  Trip tot;
  Trip ex = tadd(part[blockIdx.x], block_excl_scan(acc, sh, tot));
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    uint64_t b = base + i;
    if (b < nblk) {
      rec_base[b] = ex.r;
      key_base[b] = ex.k;
      val_base[b] = ex.v;
    }
    ex = tadd(ex, loc[i]);
  }
}

}  // namespace mtblx

// ----------------------------------------------------------------------------------
// launch glue (called from mtblx_api.cpp)
// ----------------------------------------------------------------------------------
using namespace mtblx;

extern "C" size_t mtblx_impl_scan_parts(uint32_t nblk) { return (nblk + kScanTile - 1) / kScanTile; }

template <int STAGE, int WPG>
static hipError_t launch_count(const CountArgs& c, hipStream_t s) {
  dim3 grid((c.nblk + WPG - 1) / WPG);
  hipLaunchKernelGGL((k_count<STAGE, WPG>), grid, dim3(WPG * 64), 0, s, c);
  return hipGetLastError();
}
template <int STAGE, int WPG>
static hipError_t launch_decode(const DecodeArgs& d, hipStream_t s) {
  dim3 grid((d.nblk + WPG - 1) / WPG);
  hipLaunchKernelGGL((k_decode<STAGE, WPG>), grid, dim3(WPG * 64), 0, s, d);
  return hipGetLastError();
}

// ws layout: kb[nblk] u64 | vb[nblk] u64 | parts[nparts] Trip
extern "C" int mtblx_impl_run(const mtblx_block_batch* in, const mtblx_decoded* out, void* ws, int write,
                              hipStream_t s) {
  const uint32_t nblk = in->nblk;
  uint64_t* kb = reinterpret_cast<uint64_t*>(ws);
  uint64_t* vb = kb + nblk;
  Trip* parts = reinterpret_cast<Trip*>(vb + nblk);
  const uint32_t nparts = (uint32_t)mtblx_impl_scan_parts(nblk);
  const uint32_t mx = in->max_blk_len ? in->max_blk_len : 0xFFFFFFFFu;

  CountArgs c{in->data, in->data_len, in->blk_off, in->blk_len, nblk, out->nrec, kb, vb, out->status};
  hipError_t e = hipSuccess;
  if (write == 2) goto decode;  // counts + bases already in out/ws (mtblx_decode_counted)
  if (mx <= 4096) e = launch_count<4096, 4>(c, s);
  else e = launch_count<8192, 2>(c, s);
  if (e != hipSuccess) return MTBLX_E_HIP;

  hipLaunchKernelGGL(k_scan_partial, dim3(nparts), dim3(kScanThreads), 0, s, (const uint32_t*)out->nrec,
                     (const uint64_t*)kb, (const uint64_t*)vb, nblk, parts);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanThreads), 0, s, parts, nparts, out->totals);
  hipLaunchKernelGGL(k_scan_final, dim3(nparts), dim3(kScanThreads), 0, s, (const uint32_t*)out->nrec,
                     (const uint64_t*)kb, (const uint64_t*)vb, nblk, (const Trip*)parts, out->rec_base, out->key_base,
                     out->val_base);
  if (hipGetLastError() != hipSuccess) return MTBLX_E_HIP;
  if (!write) return MTBLX_OK;
decode:
  DecodeArgs d{in->data,      in->data_len,   in->blk_off, in->blk_len,  nblk,          out->nrec,     kb,
               vb,            out->rec_base,  out->key_base, out->val_base, out->status, out->key_end, out->val_end,
               out->rec_cap,  out->keys,      out->keys_cap, out->vals,    out->vals_cap, out->totals};
  if (mx <= 4096) e = launch_decode<4096, 4>(d, s);
  else e = launch_decode<8192, 2>(d, s);
  return e == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
