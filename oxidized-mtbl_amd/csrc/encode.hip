// encode.hip — MI355X (gfx950) encode side of the block codec (BASELINE cfg3 round trip).
//
//   Writer::insert flush rule  /root/reference/src/writer.rs:125-130   -> k_plan (block cut)
//   BlockBuilder::current_size_estimate   src/block_builder.rs:40-47
//   BlockBuilder::add / finish            src/block_builder.rs:49-104  -> k_encode
//   write_block framing + crc32c          src/writer.rs:203-237        -> k_encode (framed)
//   varint_encode32 / varint_encode64     src/varint.rs:12-42, :63-76
//   Writer::insert order check            src/writer.rs:119-123        -> k_plan flags
//
// k_plan: one wave per shard (an independent Writer over a contiguous record range); the
// flush rule is a serial chain over records, so the wave advances 64 records per step:
// every lane sizes its record at the position it would take in the current block, DPP/shfl
// scans give the size estimate before each record, a ballot finds the first record that
// flushes, and the wave restarts from it (a new block).  Two passes: count, then write.
// k_encode: one workgroup per block, in ticket order.  Phase A sums the entry sizes (the
// block length is known before a byte is written) and publishes the framed size for a
// decoupled look-back across blocks; phase B assembles the block in LDS (entries, restart
// array, count); then the look-back resolves the block's file offset, the CRC-32C of the
// content is computed from LDS and the block streams out with 16-byte stores.  Blocks larger
// than the LDS buffer are assembled in place in HBM after the look-back.
// Integer/byte work, HBM bound; the block CRC-32C runs on the matrix cores (crc_mfma_dev.h).
// Round 3 variants, measured on cfg3 (2 x 200 000 blocks, profiles/r03/late, product 914-916
// GiB/s) and removed: persistent workgroups (2 per CU) claiming the next block's ticket at the
// block's start 900-901 / at the look-back 905-908 (the block loop raised scratch 48 -> 96-104
// bytes per lane); the block CRC with slicing-by-8 tables (16 dependent steps per 128 bytes
// instead of 32; 4 KiB more LDS) 882.  Earlier ones: profiles/r03/encode_gather.txt.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <vector>

#include "crc_dev.h"
#include "bounds.h"
#include "crc_mfma_dev.h"
#include "mtblx.h"

namespace mtblx_enc {

constexpr int kWave = 64;
#ifndef MTBLX_ENC_THREADS
#define MTBLX_ENC_THREADS 512
#endif
constexpr int kThreads = MTBLX_ENC_THREADS;   // one workgroup per block, 2 per CU (LDS)
constexpr int kWaves = kThreads / kWave;
#ifndef MTBLX_ENC_LDS_BLOCK
#define MTBLX_ENC_LDS_BLOCK (65536 + 1024)
#endif
#ifndef MTBLX_ENC_WPE   // waves per SIMD the register budget is sized for
#define MTBLX_ENC_WPE (kThreads / 128)
#endif
constexpr uint32_t kLdsBlock = MTBLX_ENC_LDS_BLOCK;   // contents up to this many bytes are assembled in LDS
constexpr uint32_t kShCache = 2048;            // entries whose `shared` phase A keeps for phase B
constexpr uint64_t kIncl = 1ull << 63, kAgg = 1ull << 62, kVal = kAgg - 1;

typedef uint64_t __attribute__((aligned(1))) u64u;
typedef uint32_t v4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t v4a __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t vlen32(uint64_t v) {
  return v < (1ull << 7) ? 1u : v < (1ull << 14) ? 2u : v < (1ull << 21) ? 3u : v < (1ull << 28) ? 4u : 5u;
}
__device__ __forceinline__ uint32_t vlen64(uint64_t v) {
  uint32_t n = 1;
  while (v >= 128) { v >>= 7; ++n; }
  return n;
}
struct Recs {
  const uint8_t* keys;
  const uint64_t* key_end;
  const uint8_t* vals;
  const uint64_t* val_end;
};

__device__ __forceinline__ void rec_of(const Recs& R, uint64_t r, uint64_t& k0, uint64_t& kl, uint64_t& v0,
                                       uint64_t& vl) {
  k0 = r ? R.key_end[r - 1] : 0;
  kl = R.key_end[r] - k0;
  v0 = r ? R.val_end[r - 1] : 0;
  vl = R.val_end[r] - v0;
}

// common prefix length of a[0..al) and b[0..bl); cmp = sign of a <=> b (lexicographic, Ord for [u8])
__device__ __forceinline__ uint64_t lcp_cmp(const uint8_t* a, uint64_t al, const uint8_t* b, uint64_t bl, int& cmp) {
  const uint64_t m = al < bl ? al : bl;
  uint64_t i = 0;
  while (i + 8 <= m) {
    const uint64_t x = *reinterpret_cast<const u64u*>(a + i), y = *reinterpret_cast<const u64u*>(b + i);
    if (x != y) {
      i += (uint64_t)(__builtin_ctzll(x ^ y) >> 3);
      cmp = a[i] < b[i] ? -1 : 1;
      return i;
    }
    i += 8;
  }
  while (i < m && a[i] == b[i]) ++i;
  cmp = (i < m) ? (a[i] < b[i] ? -1 : 1) : (al < bl ? -1 : (al > bl ? 1 : 0));
  return i;
}

// restart bookkeeping of BlockBuilder::add (src/block_builder.rs:50-62) for entry p of a block:
// counter < interval -> shared = LCP(last_key, key) (0 for the first entry: last_key is
// empty); else push a restart and shared = 0.  With interval == 0 the first add pushes a
// restart and the second add fails `assert!(counter <= interval)`.
__device__ __forceinline__ bool pushes_restart(uint64_t p, uint32_t iv) {
  return iv == 0 ? p == 0 : (p > 0 && p % iv == 0);
}
__device__ __forceinline__ bool shares(uint64_t p, uint32_t iv) { return p > 0 && !pushes_restart(p, iv); }

__device__ __forceinline__ uint64_t entry_bytes(uint64_t sh, uint64_t kl, uint64_t vl) {
  return vlen32(sh) + vlen32(kl - sh) + vlen32(vl) + (kl - sh) + vl;
}

template <typename T>
__device__ __forceinline__ T wave_incl_scan(T x, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const T y = __shfl_up(x, d, kWave);
    if (lane >= d) x += y;
  }
  return x;
}

// ---------------------------------------------------------------------------------
// k_plan: Writer::insert's flush rule per shard
// ---------------------------------------------------------------------------------
struct PlanArgs {
  Recs R;
  const uint64_t* shard_rec;   // [nshard + 1]
  uint32_t nshard;
  uint32_t interval;
  uint64_t block_size;
  uint64_t* shard_nblk;        // pass 0 output
  const uint64_t* shard_blk0;  // pass 1 input
  uint64_t* blk_rec;           // pass 1 output
  uint32_t* flags;             // MTBLX_PLAN_*
  int write;
};

__global__ void __launch_bounds__(kWave) k_plan(PlanArgs a) {
  const uint32_t s = blockIdx.x;
  const int lane = threadIdx.x;
  if (s >= a.nshard) return;
  const uint64_t rb = a.shard_rec[s], re = a.shard_rec[s + 1];
  const uint64_t out0 = a.write ? a.shard_blk0[s] : 0;
  uint64_t nb = 0, bstart = rb, buf = 0, nrest = 1, r0 = rb;
  uint32_t fl = 0;
  if (rb < re) {
    nb = 1;
    if (a.write && lane == 0) a.blk_rec[out0] = rb;
  }
  while (r0 < re) {
    const uint64_t r = r0 + (uint64_t)lane;
    const bool v = r < re;
    uint64_t k0 = 0, kl = 0, v0 = 0, vl = 0, sz = 0, push = 0;
    if (v) {
      rec_of(a.R, r, k0, kl, v0, vl);
      if (kl > 0xFFFFFFFFull || vl > 0xFFFFFFFFull) fl |= MTBLX_PLAN_TOO_LONG;
      const uint64_t p = r - bstart;
      uint64_t sh = 0;
      if (r > rb) {   // Writer::insert: key must be > the previous key (src/writer.rs:119-123)
        uint64_t pk0, pkl, pv0, pvl;
        rec_of(a.R, r - 1, pk0, pkl, pv0, pvl);
        int c = 0;
        const uint64_t l = lcp_cmp(a.R.keys + pk0, pkl, a.R.keys + k0, kl, c);
        if (c >= 0) fl |= MTBLX_PLAN_OUT_OF_ORDER;
        if (shares(p, a.interval)) sh = l;
      }
      if (a.interval == 0 && p > 0) fl |= MTBLX_PLAN_PANIC;
      push = pushes_restart(p, a.interval) ? 1 : 0;
      sz = entry_bytes(sh, kl, vl);
    }
    const uint64_t isz = wave_incl_scan<uint64_t>(sz, lane);
    const uint64_t ipu = wave_incl_scan<uint64_t>(push, lane);
    // current_size_estimate before record r (src/block_builder.rs:40-47) + 15 + |k| + |v|
    const uint64_t bb = buf + isz - sz, nr = nrest + ipu - push;
    const uint64_t est = bb + nr * (bb > 0xFFFFFFFFull ? 8u : 4u) + 4u;
    const bool flush = v && r > bstart && est + 15 + kl + vl >= a.block_size;
    const uint64_t fm = __ballot(flush);
    if (fm) {
      const int f = __builtin_ctzll(fm);
      bstart = r0 + (uint64_t)f;
      r0 = bstart;
      buf = 0;
      nrest = 1;
      if (a.write && lane == 0) a.blk_rec[out0 + nb] = bstart;
      ++nb;
    } else {
      const int last = (int)(re - r0 < (uint64_t)kWave ? re - r0 : (uint64_t)kWave) - 1;
      buf += __shfl(isz, last, kWave);
      nrest += __shfl(ipu, last, kWave);
      r0 += kWave;
    }
  }
  // wave-uniform: OR of the lanes' flags
  uint32_t f = fl;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) f |= (uint32_t)__shfl_xor((int)f, d, kWave);
  if (lane == 0) {
    if (!a.write) a.shard_nblk[s] = nb;
    if (f) atomicOr(a.flags, f);
  }
}

// ---------------------------------------------------------------------------------
// k_encode: BlockBuilder per block + Writer framing, decoupled look-back for offsets
// ---------------------------------------------------------------------------------
struct X8Tab {
  uint32_t p[64];   // x^(8 t) mod P, t < 64 (reflected, x^0 = bit 31)
  constexpr X8Tab() : p() {
    uint32_t x = 0x80000000u;
    for (int t = 0; t < 64; ++t) {
      p[t] = x;
      for (int k = 0; k < 8; ++k) x = (x & 1u) ? (x >> 1) ^ mtblx_crc::kPoly : x >> 1;
    }
  }
};
static __constant__ X8Tab kX8 = X8Tab();

// The block CRC on the matrix cores (crc_mfma.h): the operands of k_crc32c_mfma, plus the shift of
// super-window S (8 KiB steps counted from the block's aligned end) x^(8·8192·S) as nibble tables,
// S <= 8 for blocks assembled in LDS (kLdsBlock bytes)
#ifndef MTBLX_ENC_CRC_MFMA
#define MTBLX_ENC_CRC_MFMA 1
#endif
#if defined(MTBLX_ENC_ABL) && !defined(MTBLX_DIAG)
#error "MTBLX_ENC_ABL is a timing ablation (wrong output): build it through a diagnostic target"
#endif
#ifndef MTBLX_ENC_CONTIG   // each thread owns contiguous entries (phase B without per-round scans)
#define MTBLX_ENC_CONTIG 1
#endif
#ifndef MTBLX_ENC_LAZY_T   // slicing-by-4 tables built only by blocks that use them
#define MTBLX_ENC_LAZY_T 1
#endif
#ifndef MTBLX_ENC_TW   // planned mode: stores before the block CRC, stage-2 operand per wave (see k_encode)
#define MTBLX_ENC_TW 1
#endif
#ifndef MTBLX_ENC_CRC_UNROLL
#define MTBLX_ENC_CRC_UNROLL 4
#endif
constexpr int kEncSup = (kLdsBlock + mtblx_crc::kMStep * mtblx_crc::kMSup - 1) / (mtblx_crc::kMStep * mtblx_crc::kMSup);
using EncSw = mtblx_crc::SwTabs<kEncSup>;
static __constant__ mtblx_crc::MfmaTabs kEncMfma = mtblx_crc::MfmaTabs();
static __constant__ EncSw kEncSw = EncSw();

struct EncArgs {
  Recs R;
  const uint64_t* blk_rec;   // [nblk + 1]
  uint32_t nblk;
  uint32_t interval;
  int framed;
  uint8_t* out;
  uint64_t out_cap;
  uint64_t* blk_off;
  uint32_t* blk_len;
  int32_t* status;
  uint64_t* totals;          // [2]: bytes written, flags
  uint32_t* ticket;
  uint64_t* lbw;             // [nblk] look-back words
  // planned mode (mtblx_encode_blocks_planned): the block cut's kept sums, local to record plo
  const uint64_t* PA;        // inclusive prefix of the entry sizes with sharing
  const uint64_t* Q;         // inclusive prefix of the restart savings along residue classes mod interval
  const uint32_t* SH;        // shared-prefix length with the previous record
  uint64_t plo, pm;          // the plan's first record and record count
  const uint64_t* fincl;     // [nblk] inclusive prefix of the framed block sizes (the file offsets)
};

// planned mode: the byte offset of entry i (0 <= i <= n) in a block whose first record is local
// record j0 (src/block_builder.rs:49-83: entries before i, restart entries without sharing)
__device__ __forceinline__ uint64_t planned_off(const EncArgs& a, uint64_t j0, uint64_t i, uint32_t iv) {
  if (i == 0) return 0;
  const uint64_t last = j0 + (uint64_t)iv * ((i - 1) / iv);
  MTBLX_CHK(a.PA + j0 + i - 1, 8), MTBLX_CHK(a.Q + last, 8);
  return a.PA[j0 + i - 1] - (j0 ? a.PA[j0 - 1] : 0) + a.Q[last] - (j0 >= iv ? a.Q[j0 - iv] : 0);
}

struct alignas(16) EncLds {
  uint8_t ob[kLdsBlock];
  uint32_t T[4][256];        // slicing-by-4 CRC-32C tables
  uint16_t shc[kShCache];    // phase A's `shared` of the first entries (0xFFFF: recompute)
  uint64_t red[kWaves];
  uint32_t redf[kWaves];
  uint64_t sh_u64[4];
  uint32_t sh_u32[4];
};

// block-wide exclusive scan of a u64 (all threads); returns the exclusive prefix, total in `tot`
__device__ __forceinline__ uint64_t wg_excl_scan(EncLds& S, uint64_t x, uint64_t& tot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_scan<uint64_t>(x, lane);
  if (lane == kWave - 1) S.red[w] = inc;
  __syncthreads();
  uint64_t before = 0;
  tot = 0;
#pragma unroll
  for (int k = 0; k < kWaves; ++k) {
    const uint64_t v = S.red[k];
    if (k < w) before += v;
    tot += v;
  }
  __syncthreads();
  return before + inc - x;
}

#ifndef MTBLX_ENC_CARRY   // the next entry's offsets carried from this one (A/B: 0 = reload both ends)
#define MTBLX_ENC_CARRY 1
#endif
#ifndef MTBLX_ENC_TAILV   // tails of 1..15 bytes as 8/4/2/1-byte pieces (0: byte stores, the A/B base)
#define MTBLX_ENC_TAILV 1
#endif
#ifndef MTBLX_ENC_NT_STORES
#define MTBLX_ENC_NT_STORES 1
#endif

// the last t (1..15) bytes of the 16-byte window w, stored at d
__device__ __forceinline__ void store_tail(uint8_t* d, const v4u& w, uint32_t t) {
#if MTBLX_ENC_TAILV
  // the window shifted right by r = 16 - t bytes (funnel shifts), then stored as pieces of 8,
  // 4, 2 and 1 bytes (the bits of t) instead of t byte stores: a wave paid for its longest tail
  const uint32_t r = 16u - t, dq = r >> 2, bs = r & 3u;
  const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
  uint32_t o[4];
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    const uint32_t lo = dq + i < 4 ? (dq + i == 0 ? ws[0] : dq + i == 1 ? ws[1] : dq + i == 2 ? ws[2] : ws[3]) : 0u;
    const uint32_t hi = dq + i + 1 < 4 ? (dq + i + 1 == 1 ? ws[1] : dq + i + 1 == 2 ? ws[2] : ws[3]) : 0u;
    o[i] = __builtin_amdgcn_alignbyte(hi, lo, bs);
  }
  typedef uint64_t __attribute__((aligned(1))) u64t;
  typedef uint32_t __attribute__((aligned(1))) u32t;
  typedef uint16_t __attribute__((aligned(1))) u16t;
  uint32_t off = 0;
  if (t & 8u) {
    *reinterpret_cast<u64t*>(d) = (uint64_t)o[0] | ((uint64_t)o[1] << 32);
    off = 8;
  }
  if (t & 4u) {
    *reinterpret_cast<u32t*>(d + off) = off ? o[2] : o[0];
    off += 4;
  }
  const auto word = [&](uint32_t q) { return q == 0 ? o[0] : q == 1 ? o[1] : q == 2 ? o[2] : o[3]; };
  if (t & 2u) {
    *reinterpret_cast<u16t*>(d + off) = (uint16_t)(word(off >> 2) >> (8 * (off & 3u)));
    off += 2;
  }
  if (t & 1u) d[off] = (uint8_t)(word(off >> 2) >> (8 * (off & 3u)));
#else
  for (uint32_t k = 0; k < t; ++k) {
    const uint32_t q = 16 - t + k;
    const uint32_t v = q < 4 ? w.x : q < 8 ? w.y : q < 12 ? w.z : w.w;
    d[k] = (uint8_t)(v >> (8 * (q & 3)));
  }
#endif
}

// copy n bytes from global src to dst (LDS or global, generic pointer).  Four 16-byte loads
// are in flight before their stores (the loads are the latency: a serial load -> store chain
// per 16 bytes was most of the encode time); stores are unaligned 16-byte stores (gfx950 runs
// in unaligned access mode).  A tail of 1..15 bytes is read as the 16-byte window ending at n
// when the record is at least 16 bytes long (never before `base`, the blob's start), else
// byte by byte.
__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, uint64_t n, const uint8_t* base) {
  // chunks of 16 bytes: [0, nfull); tail bytes [16 nfull, n)
  const uint64_t nfull = n / 16;
  for (uint64_t c = 0; c < nfull; c += 4) {
    v4u w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (c + u < nfull) w[u] = *reinterpret_cast<const v4u*>(src + 16 * (c + u));
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (c + u < nfull) *reinterpret_cast<v4u*>(dst + 16 * (c + u)) = w[u];
  }
  const uint32_t t = (uint32_t)(n % 16);
  if (t == 0) return;
  const uint64_t to = 16 * nfull;
  if (src + n >= base + 16) {   // the 16-byte window ending at n holds the tail in its last t bytes
    store_tail(dst + to, *reinterpret_cast<const v4u*>(src + n - 16), t);
  } else {
    for (uint64_t k = to; k < n; ++k) dst[k] = src[k];
  }
}

// n bytes from src to dst as 16-byte chunks at offsets min(16 c, n - 16): the last, partial chunk
// is the 16-byte window ending at n, rewriting bytes of the chunk before it with the same values,
// so a field of n >= 16 bytes takes ceil(n / 16) whole loads and stores, issued four at a time --
// one round trip for up to 64 bytes, no tail pieces.  A field of 1..15 bytes is the window ending
// at n shifted down; with `fwd` (this thread rewrites the bytes after the field later: the key
// suffix before its value) it goes out as one 16-byte store, else as 8/4/2/1-byte pieces.
#ifndef MTBLX_ENC_OVER
#define MTBLX_ENC_OVER 0
#endif
__device__ __forceinline__ void copy_over(uint8_t* dst, const uint8_t* src, uint32_t n, const uint8_t* base, bool fwd) {
  if (n >= 16u) {
    const uint32_t m = (n + 15u) >> 4;
    for (uint32_t c = 0; c < m; c += 4) {
      v4u w[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t o = 16u * (c + u) < n - 16u ? 16u * (c + u) : n - 16u;
        if (c + u < m) w[u] = *reinterpret_cast<const v4u*>(src + o);
      }
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t o = 16u * (c + u) < n - 16u ? 16u * (c + u) : n - 16u;
        if (c + u < m) *reinterpret_cast<v4u*>(dst + o) = w[u];
      }
    }
    return;
  }
  if (n == 0u) return;
  if (src + n >= base + 16) {
    const v4u w = *reinterpret_cast<const v4u*>(src + n - 16);
    if (fwd) {   // bytes n..15 of the store are rewritten by this thread afterwards
      const uint32_t r = 16u - n, dq = r >> 2, bs = r & 3u;
      const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
      uint32_t o[4];
#pragma unroll
      for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t lo = dq + i < 4 ? (dq + i == 0 ? ws[0] : dq + i == 1 ? ws[1] : dq + i == 2 ? ws[2] : ws[3]) : 0u;
        const uint32_t hi = dq + i + 1 < 4 ? (dq + i + 1 == 1 ? ws[1] : dq + i + 1 == 2 ? ws[2] : ws[3]) : 0u;
        o[i] = __builtin_amdgcn_alignbyte(hi, lo, bs);
      }
      *reinterpret_cast<v4u*>(dst) = v4u{o[0], o[1], o[2], o[3]};
    } else {
      store_tail(dst, w, n);
    }
  } else {
    for (uint32_t k = 0; k < n; ++k) dst[k] = src[k];
  }
}

// an entry's key suffix (kn bytes at ks) and value (vn bytes at vs), back to back at dst: when
// both are at most 64 bytes (cfg3's common case) every load of both -- whole chunks and the two
// tail windows -- is issued before the first store, one memory round trip instead of the 2-4 of
// two copy_bytes calls (each waits for its chunks, then for its tail window)
#ifndef MTBLX_ENC_EARLY   // planned mode: first entry's fields loaded beside phase A's sums
#define MTBLX_ENC_EARLY 0
#endif
#ifndef MTBLX_ENC_KV
#define MTBLX_ENC_KV 0
#endif
__device__ __forceinline__ void copy_kv(uint8_t* dst, const uint8_t* ks, uint64_t kn, const uint8_t* kbase,
                                        const uint8_t* vs, uint64_t vn, const uint8_t* vbase) {
  if (!MTBLX_ENC_KV || kn > 64 || vn > 64) {
    copy_bytes(dst, ks, kn, kbase);
    copy_bytes(dst + kn, vs, vn, vbase);
    return;
  }
  const uint32_t nk = (uint32_t)kn / 16u, tk = (uint32_t)kn % 16u, nv = (uint32_t)vn / 16u, tv = (uint32_t)vn % 16u;
  const bool wk = tk && ks + kn >= kbase + 16, wv = tv && vs + vn >= vbase + 16;
  v4u K[4], V[4], KT = {0u, 0u, 0u, 0u}, VT = {0u, 0u, 0u, 0u};
#pragma unroll
  for (uint32_t u = 0; u < 4; ++u)
    if (u < nk) K[u] = *reinterpret_cast<const v4u*>(ks + 16 * u);
  if (wk) KT = *reinterpret_cast<const v4u*>(ks + kn - 16);
#pragma unroll
  for (uint32_t u = 0; u < 4; ++u)
    if (u < nv) V[u] = *reinterpret_cast<const v4u*>(vs + 16 * u);
  if (wv) VT = *reinterpret_cast<const v4u*>(vs + vn - 16);
#pragma unroll
  for (uint32_t u = 0; u < 4; ++u)
    if (u < nk) *reinterpret_cast<v4u*>(dst + 16 * u) = K[u];
  if (wk) store_tail(dst + 16 * nk, KT, tk);
  else for (uint32_t k = 16 * nk; k < (uint32_t)kn; ++k) dst[k] = ks[k];
  uint8_t* dv = dst + kn;
#pragma unroll
  for (uint32_t u = 0; u < 4; ++u)
    if (u < nv) *reinterpret_cast<v4u*>(dv + 16 * u) = V[u];
  if (wv) store_tail(dv + 16 * nv, VT, tv);
  else for (uint32_t k = 16 * nv; k < (uint32_t)vn; ++k) dv[k] = vs[k];
}

__device__ __forceinline__ void put32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

// CRC-32C of d[0..L) by the workgroup (crate crc32c 0.4).  Thread t takes the contiguous span
// [t S, (t+1) S) (S a multiple of 16: aligned 16 B reads of the LDS buffer), computes its raw
// CRC with slicing-by-4, and shifts it by the bytes after the span, x^(8 m) = x^(512 (m / 64))
// * x^(8 (m % 64)); the spans are XOR-combined.  The 0xFFFFFFFF init is folded into the first
// 4 bytes; the final complement is the xorout.
__device__ __forceinline__ uint32_t crc_word(const EncLds& S, uint32_t c, uint32_t w) {
  c ^= w;
  return S.T[3][c & 0xffu] ^ S.T[2][(c >> 8) & 0xffu] ^ S.T[1][(c >> 16) & 0xffu] ^ S.T[0][c >> 24];
}

__device__ __forceinline__ uint32_t wg_crc32c(EncLds& S, const uint8_t* d, uint64_t L) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t acc = 0;
  if (L >= 4) {
    const uint64_t per = (L + kThreads - 1) / kThreads;
    const uint64_t span = ((per + 15) / 16) * 16;
    const uint64_t a0 = (uint64_t)tid * span;
    const uint64_t a1 = a0 + span < L ? a0 + span : L;
    if (a0 < a1) {
      uint32_t c = 0;
      uint64_t o = a0;
      for (; o + 16 <= a1; o += 16) {
        const v4u x = *reinterpret_cast<const v4u*>(d + o);
        c = crc_word(S, c, o == 0 ? x.x ^ 0xFFFFFFFFu : x.x);
        c = crc_word(S, c, x.y);
        c = crc_word(S, c, x.z);
        c = crc_word(S, c, x.w);
      }
      for (; o < a1; ++o) {   // tail bytes (byte loads: never past the content)
        uint32_t byte = d[o];
        if (o < 4) byte ^= 0xFFu;
        c = S.T[0][(c ^ byte) & 0xFFu] ^ (c >> 8);
      }
      const uint64_t m = L - a1;
      if (m) c = mtblx_crc::dmultmodp(mtblx_crc::dmultmodp(mtblx_crc::xpow512(m / 64), kX8.p[m % 64]), c);
      acc = c;
    }
  } else if (tid == 0) {
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < L; ++i) c = S.T[0][(c ^ d[i]) & 0xFFu] ^ (c >> 8);
    acc = c ^ 0xFFFFFFFFu ^ 0xFFFFFFFFu;   // complemented again below
  }
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, s, kWave);
  if (lane == 0) S.redf[w] = acc;
  __syncthreads();
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < kWaves; ++k) r ^= S.redf[k];
  __syncthreads();
  return r ^ 0xFFFFFFFFu;
}

// CRC-32C of the block assembled at S.ob[0..L) (4 <= L <= kLdsBlock; the caller zeroes the pad
// S.ob[L .. L + t), t = the bytes to a 16-byte boundary) on the matrix cores: windows counted from
// the padded end as k_crc32c_mfma (crc.hip, crc_mfma.h); wave w takes the super-windows w,
// w + kWaves, ... (8 steps of 1 KiB each, straight from LDS: every step's chunks are 16-byte
// aligned, so the block start needs no partial masks) and shifts their raw CRC by x^(8·8192·S)
// (crc_mfma_part, no barrier: wave 0 runs the look-back first); after a barrier the waves'
// parts are XOR-combined and the pad is removed by x^(-8t) (crc_mfma_final).  The operands come
// from constant memory.
__device__ __forceinline__ void crc_mfma_part(EncLds& S, uint32_t L) {
  using namespace mtblx_crc;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, n = lane & 15;
  const uint32_t t = (16u - (L & 15u)) & 15u, Lp = L + t;
  const uint32_t steps = (Lp + kMStep - 1) / kMStep, nsup = (steps + kMSup - 1) / kMSup;
  const int32_t kx16 = 16 * (60 - 4 * n + g);   // the lane's chunk of a step
  uint32_t C = 0;
  if ((uint32_t)w < nsup) {
    v4i A[kMKs][2];
#pragma unroll
    for (int k = 0; k < kMKs; ++k) {
      A[k][0] = reinterpret_cast<const v4i*>(&kEncMfma.a[k][0][0][0])[lane];
      A[k][1] = reinterpret_cast<const v4i*>(&kEncMfma.a[k][1][0][0])[lane];
    }
    for (uint32_t sw = (uint32_t)w; sw < nsup; sw += kWaves) {
      v4f c2a = {0.f, 0.f, 0.f, 0.f}, c2b = c2a;
#pragma unroll MTBLX_ENC_CRC_UNROLL
      for (int tt = kMSup - 1; tt >= 0; --tt) {   // from the super-window's start
        const uint32_t s = sw * kMSup + (uint32_t)tt;
        if (s < steps) {
          const int32_t pos = (int32_t)Lp - (int32_t)(kMStep * (s + 1)) + kx16;   // a multiple of 16
          v4a x = {0u, 0u, 0u, 0u};
          if (pos >= 0) x = *reinterpret_cast<const v4a*>(S.ob + pos);
          if (pos == 0) x.x ^= 0xFFFFFFFFu;   // the init, folded into bytes 0..3
#if defined(MTBLX_ENC_ABL) && MTBLX_ENC_ABL == 4   // timing ablation only: no stage-2 operand loads
          const v4i a2lo = A[tt & 3][0], a2hi = A[tt & 3][1];
#else
          const v4i a2lo = reinterpret_cast<const v4i*>(&kEncMfma.a2[tt][0][0][0])[lane];
          const v4i a2hi = reinterpret_cast<const v4i*>(&kEncMfma.a2[tt][1][0][0])[lane];
#endif
          mfma_step(A, v4u{x.x, x.y, x.z, x.w}, a2lo, a2hi, c2a, c2b);
        }
      }
      // the column's parities (CRC bits 4g + i, 16 + 4g + i), column shift, XOR over the columns
      uint32_t c = kEncMfma.col[n][g][par_nib(c2a)] ^ kEncMfma.col[n][4 + g][par_nib(c2b)];
      c = row_xor(c);
      uint32_t Cs = (uint32_t)__builtin_amdgcn_readlane((int)c, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)c, 16) ^
                    (uint32_t)__builtin_amdgcn_readlane((int)c, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)c, 48);
      if (sw) {   // x^(8·8192·sw): nibble j looked up by lane j (j < 8) of each row
        const uint32_t j = (uint32_t)lane & 15u;
        const uint32_t v = j < 8u ? kEncSw.t[sw][j][(Cs >> (4 * j)) & 15u] : 0u;
        Cs = (uint32_t)__builtin_amdgcn_readlane((int)row_xor(v), 0);
      }
      C ^= Cs;
    }
  }
  if (lane == 0) S.redf[w] = C;
}
// after a barrier that follows every wave's crc_mfma_part
__device__ __forceinline__ uint32_t crc_mfma_final(const EncLds& S, uint32_t L) {
  const int lane = threadIdx.x & 63;
  const uint32_t t = (16u - (L & 15u)) & 15u;
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < kWaves; ++k) r ^= S.redf[k];
  if (t) {   // x^(-8t): the pad after the block's end removed
    const uint32_t j = (uint32_t)lane & 15u;
    const uint32_t v = j < 8u ? kEncMfma.inv[t][j][(r >> (4 * j)) & 15u] : 0u;
    r = (uint32_t)__builtin_amdgcn_readlane((int)mtblx_crc::row_xor(v), 0);
  }
  return r ^ 0xFFFFFFFFu;
}

// entry i of the block starting at record r0: fields and encoded size
struct Ent {
  uint64_t k0, kl, v0, vl, sh;
};
// share: the entry shares a prefix with its predecessor (shares(i, interval), tracked by the
// callers as a running restart phase: a 64-bit modulo per entry was ~100 vector instructions)
__device__ __forceinline__ Ent entry_of(const Recs& R, uint64_t r0, uint64_t i, bool share,
                                        const uint16_t* shc = nullptr, const uint32_t* SH = nullptr) {
  Ent e;
  rec_of(R, r0 + i, e.k0, e.kl, e.v0, e.vl);
  e.sh = 0;
  if (SH) {   // planned: the block cut kept every record's shared-prefix length
    if (share) {
      MTBLX_CHK(SH + i, 4);
      e.sh = SH[i];
    }
  } else if (shc && i < kShCache && shc[i] != 0xFFFFu) {
    e.sh = shc[i];
  } else if (share) {
    uint64_t pk0, pkl, pv0, pvl;
    rec_of(R, r0 + i - 1, pk0, pkl, pv0, pvl);
    int c;
    e.sh = lcp_cmp(R.keys + pk0, pkl, R.keys + e.k0, e.kl, c);
  }
  return e;
}

// entry i + 1 after entry p = entry i: its key and value start where p's end (the END offsets
// are cumulative), so only record r0 + i + 1's two END offsets are loaded, and its shared prefix
// (when not cached) is the LCP with p's key
__device__ __forceinline__ Ent entry_after(const Recs& R, uint64_t r0, uint64_t i1, const Ent& p, bool share,
                                           const uint16_t* shc = nullptr, const uint32_t* SH = nullptr) {
  Ent e;
  const uint64_t r = r0 + i1;
  MTBLX_CHK(R.key_end + r, 8), MTBLX_CHK(R.val_end + r, 8);
  e.k0 = p.k0 + p.kl;
  e.kl = R.key_end[r] - e.k0;
  e.v0 = p.v0 + p.vl;
  e.vl = R.val_end[r] - e.v0;
  e.sh = 0;
  if (SH) {
    if (share) {
      MTBLX_CHK(SH + i1, 4);
      e.sh = SH[i1];
    }
  } else if (shc && i1 < kShCache && shc[i1] != 0xFFFFu) {
    e.sh = shc[i1];
  } else if (share) {
    int c;
    e.sh = lcp_cmp(R.keys + p.k0, p.kl, R.keys + e.k0, e.kl, c);
  }
  return e;
}

// varint32 bytes of v packed little-endian in a register (<= 5 bytes), *len = their count
// (src/varint.rs:12-42)
__device__ __forceinline__ uint64_t vpack(uint64_t v, uint32_t& len) {
  uint64_t w = 0;
  uint32_t i = 0;
  while (v >= 128) {
    w |= ((v & 127u) | 128u) << (8 * i);
    v >>= 7;
    ++i;
  }
  len = i + 1;
  return w | (v << (8 * i));
}

// write entry e at dst (header varints, key suffix, value): src/block_builder.rs:69-77.  The
// header bytes are computed in registers (byte k of varint32(v): 7 bits of v, continuation bit
// unless last): a byte array here was dynamically indexed, i.e. lived in scratch.
__device__ __forceinline__ void put_varint(uint8_t* p, uint32_t v, uint32_t len) {
#pragma unroll
  for (uint32_t k = 0; k < 5; ++k)
    if (k < len) p[k] = (uint8_t)(((v >> (7 * k)) & 0x7fu) | (k + 1 < len ? 0x80u : 0u));
}
// varint32(v) (len = vlen32(v) bytes) as a little-endian word, branch-free: the 7-bit groups
// spread to bytes, the continuation bit on all but the last
__device__ __forceinline__ uint64_t vbytes32(uint32_t v, uint32_t len) {
  const uint64_t g = (uint64_t)(v & 0x7fu) | ((uint64_t)(v & 0x3f80u) << 1) | ((uint64_t)(v & 0x1fc000u) << 2) |
                     ((uint64_t)(v & 0xfe00000u) << 3) | ((uint64_t)(v >> 28) << 32);
  return g | (0x0000008080808080ull & ((1ull << (8 * (len - 1u))) - 1ull));
}
#ifndef MTBLX_ENC_HDR   // the three header varints as one 8-byte store when they fit (1) or byte by byte (0)
#define MTBLX_ENC_HDR 1
#endif
__device__ __forceinline__ void put_entry(uint8_t* dst, const Recs& R, const Ent& e) {
  const uint32_t sh = (uint32_t)e.sh, ks = (uint32_t)(e.kl - e.sh), vl = (uint32_t)e.vl;   // < 4 GiB (k_plan)
  const uint32_t l0 = vlen32(sh), l1 = vlen32(ks), l2 = vlen32(vl);
  const uint32_t n = l0 + l1 + l2;
  if (MTBLX_ENC_HDR && n <= 8u && (uint64_t)n + ks + vl >= 8u) {
    // one unaligned 8-byte store: its bytes n..7 are the key suffix / value's, rewritten below by
    // this thread (in program order) -- no conditional byte stores
    *reinterpret_cast<u64u*>(dst) = vbytes32(sh, l0) | (vbytes32(ks, l1) << (8 * l0)) | (vbytes32(vl, l2) << (8 * (l0 + l1)));
  } else {
    put_varint(dst, sh, l0);
    put_varint(dst + l0, ks, l1);
    put_varint(dst + l0 + l1, vl, l2);
  }
#if MTBLX_ENC_OVER
  copy_over(dst + n, R.keys + e.k0 + e.sh, ks, R.keys, (uint64_t)ks + vl >= 16u);
  copy_over(dst + n + ks, R.vals + e.v0, vl, R.vals, false);
#else
  copy_kv(dst + n, R.keys + e.k0 + e.sh, e.kl - e.sh, R.keys, R.vals + e.v0, e.vl, R.vals);
#endif
}
__device__ __forceinline__ uint64_t lookback(const EncArgs& a, uint32_t b, int lane, bool& timeout) {
  uint64_t excl = 0;
  int64_t j = (int64_t)b - 1;
  while (j >= 0) {
    const int64_t idx = j - lane;
    uint64_t w = idx >= 0 ? __hip_atomic_load(a.lbw + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kIncl;
    // bounded by wall time (s_memrealtime, 100 MHz; 20 s): tickets are claimed by running
    // workgroups, so this only gives up if the chip stalls -- never on a slow predecessor
    uint64_t t0 = 0;
    uint32_t spins = 0;
    while (__ballot(!(w & (kIncl | kAgg))) != 0ull) {
      __builtin_amdgcn_s_sleep(1);
      if (!(w & (kIncl | kAgg))) w = __hip_atomic_load(a.lbw + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((++spins & 63u) == 0u) {
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        if (t0 == 0) t0 = t;
        if (t - t0 > 2000000000ull) { timeout = true; w |= kIncl; }
      }
    }
    const uint64_t im = __ballot((w & kIncl) != 0ull);
    const int first = im ? __builtin_ctzll(im) : kWave;
    uint64_t v = (lane <= first) ? (w & kVal) : 0ull;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kWave);
    excl += v;
    if (im) break;
    j -= kWave;
  }
  return excl;
}

// diagnostic per-phase cycle stamps (MTBLX_ENC_STAMPS builds only): thread 0 of each workgroup
// adds s_memtime deltas into u64 slots 2.. of the workspace header, slot 15 counts blocks
#ifdef MTBLX_ENC_STAMPS
#define ESTAMP(k) do { __syncthreads(); if (threadIdx.x == 0) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    atomicAdd(reinterpret_cast<unsigned long long*>(a.ticket) + (k), (unsigned long long)(t_ - tprev)); tprev = t_; } } while (0)
#else
#define ESTAMP(k) do { } while (0)
#endif

#ifndef MTBLX_ENC_RAWB   // TW path: LDS-only barriers (1) or __syncthreads (0: also waits for the block's stores)
#define MTBLX_ENC_RAWB 0
#endif
__device__ __forceinline__ void tw_barrier() {
#if MTBLX_ENC_RAWB
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
  __syncthreads();
#endif
}

template <bool PL>   // PL: planned mode (sizes and offsets from the block cut's sums; no look-back)
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(MTBLX_ENC_WPE))) k_encode(EncArgs a) {   // 2 per CU
  __shared__ EncLds S;
#ifdef MTBLX_ENC_STAMPS
  uint64_t tprev = __builtin_amdgcn_s_memtime();
#endif
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // slicing-by-4 tables from the byte table: only the blocks whose CRC is not on the matrix cores
  // need them (built there; four dependent constant-memory loads were ~5k cycles of every block)
  auto build_tables = [&]() {
    for (int i = tid; i < 256; i += kThreads) {
      uint32_t t = mtblx_crc::kTab.byte[i];
      S.T[0][i] = t;
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        t = (t >> 8) ^ mtblx_crc::kTab.byte[t & 0xffu];
        S.T[k][i] = t;
      }
    }
  };
#if !MTBLX_ENC_LAZY_T
  build_tables();
#endif
  uint32_t b = blockIdx.x;
  if constexpr (!PL) {   // ticket order: every earlier block is running or done (the look-back)
    if (tid == 0) S.sh_u32[0] = atomicAdd(a.ticket, 1u);
    __syncthreads();
    b = S.sh_u32[0];
  }
  if (b >= a.nblk) return;
#if MTBLX_ENC_TW
  // planned mode: the file offset and the Horner table of the block CRC (below) loaded now, so
  // their latency overlaps the assembly
  uint64_t tw_fin = 0;
  uint32_t tw_swk = 0;
  if constexpr (PL) {
    if (tid == 0) {
      MTBLX_CHK(a.fincl + b, 8);
      tw_fin = a.fincl[b];
    }
    if (tid < 128) tw_swk = (&kEncMfma.swk[0][0])[tid];
  }
#endif
  const uint64_t r0 = a.blk_rec[b], n = a.blk_rec[b + 1] - r0;
  const uint32_t iv = a.interval;
  ESTAMP(2);   // tables + ticket

  // ---- phase A: the content length (entries + restart array + count) ----
  uint64_t part = 0;
  // planned mode: the block's record range must lie in the plan
  const bool pl_ok = !PL || (r0 >= a.plo && r0 + n <= a.plo + a.pm);
  const uint64_t j0 = PL ? r0 - a.plo : 0;
#if MTBLX_ENC_CONTIG
  // thread t owns the contiguous entries [i0, i1) (balanced: floor(n / threads) or one more
  // each): the scan of its byte total is the offset of its first entry, so phase B runs through
  // them with a running offset -- no per-round scans (two barriers each) and no round-wide wait
  // for the longest entry (Zipf keys).  (Phase A reading coalesced, entry i on thread i mod
  // threads, and handing the sizes over in LDS measured slower: 1043 vs 1069 GiB/s.)
  const uint64_t i0 = n * (uint64_t)tid / kThreads, i1 = n * (uint64_t)(tid + 1) / kThreads;
  // the restart phase of entry i0 (i0 mod interval), then advanced per entry
  const uint32_t ph0 = iv ? (uint32_t)(i0 % iv) : 0u;
  uint32_t ph = ph0;
  // planned mode: the first entry's fields are loaded now, beside the sums' loads (phase A), not
  // after them
  Ent en0{};
  (void)en0;
  if constexpr (PL && MTBLX_ENC_EARLY) {
    if (pl_ok && i0 < i1) en0 = entry_of(a.R, r0, i0, iv ? (i0 > 0 && ph0 != 0) : (i0 > 0), nullptr, a.SH + j0);
  }
  Ent pe{};   // the previous entry (MTBLX_ENC_CARRY)
  (void)pe;
  for (uint64_t i = i0; i < i1 && !PL; ++i) {
    const bool share = iv ? (i > 0 && ph != 0) : (i > 0);
    if (iv && ++ph == iv) ph = 0;
#if MTBLX_ENC_CARRY
    const Ent e = i == i0 ? entry_of(a.R, r0, i, share) : entry_after(a.R, r0, i, pe, share);
    pe = e;
#else
    const Ent e = entry_of(a.R, r0, i, share);
#endif
#else
  static_assert(!PL, "planned mode needs MTBLX_ENC_CONTIG");
  for (uint64_t i = tid; i < n; i += kThreads) {
    const bool share = shares(i, iv);
    const Ent e = entry_of(a.R, r0, i, share);
#endif
    part += entry_bytes(e.sh, e.kl, e.vl);
    if (i < kShCache)
      S.shc[i] = e.sh < 0xFFFFu ? (uint16_t)e.sh : (uint16_t)0xFFFFu;
  }
  uint64_t entries = 0, tbase = 0;
  if constexpr (PL) {   // the sums give every offset: no size pass, no scan
    if (pl_ok) {
      entries = planned_off(a, j0, n, iv);
#if MTBLX_ENC_CONTIG
      tbase = planned_off(a, j0, i0, iv);
#endif
    }
  } else {
    tbase = wg_excl_scan(S, part, entries);
  }
  (void)tbase;
  // restarts: [0] + one push per restart entry (src/block_builder.rs:21, :60)
  const uint64_t nrest = n == 0 ? 1 : (iv == 0 ? 2 : 1 + (n - 1) / iv);
  int32_t st = MTBLX_ST_OK;
  if (!pl_ok) st = MTBLX_ST_UNSUPPORTED;                   // planned mode: records outside the plan
  if (iv == 0 && n > 1) st = MTBLX_ST_CORRUPT;            // assert!(counter <= interval) (:50)
  if (entries > 0xFFFFFFFFull) st = MTBLX_ST_UNSUPPORTED;  // u64 restart arrays: blocks >= 4 GiB
  const uint64_t L = entries + 4 * nrest + 4;
  // a planned block outside the plan was counted 0 by k_enc_fsize: F = 0 keeps totals[0] the scan's total
  const uint64_t F = !pl_ok ? 0 : (a.framed ? vlen64(L) + 4 + L : L);
  if (!PL && tid == 0) {   // publish this block's framed size as early as possible
    __hip_atomic_store(a.lbw + b, (b == 0 ? kIncl : kAgg) | F, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const bool in_lds = L <= kLdsBlock && st == MTBLX_ST_OK;
  ESTAMP(3);   // phase A: sizes, scan, publish

  // ---- phase B (LDS path): assemble the block ----
  const uint64_t R = entries;   // restart array offset
  auto assemble = [&](uint8_t* dst, auto lds_tag) {
    constexpr bool lds = decltype(lds_tag)::value;
#if MTBLX_ENC_CONTIG
    uint64_t eo = tbase;
    Ent en{};   // the next entry's fields are loaded before this entry's bytes move
    const uint32_t* SHb = PL ? a.SH + j0 : nullptr;
    // restart phase of the entry and the number of restarts before it (multiples of the interval)
    uint32_t rp = ph0;
    uint64_t ri = iv ? (i0 + iv - 1) / iv : 0;
    const auto share_at = [&](uint64_t i, uint32_t p) { return iv ? (i > 0 && p != 0) : (i > 0); };
    if (i0 < i1) en = (PL && MTBLX_ENC_EARLY) ? en0 : entry_of(a.R, r0, i0, share_at(i0, rp), S.shc, SHb);
    for (uint64_t i = i0; i < i1; ++i) {
      const Ent e = en;
      const uint32_t rp1 = iv ? (rp + 1 == iv ? 0u : rp + 1) : 0u;
#if MTBLX_ENC_CARRY
      if (i + 1 < i1) en = entry_after(a.R, r0, i + 1, e, share_at(i + 1, rp1), S.shc, SHb);
#else
      if (i + 1 < i1) en = entry_of(a.R, r0, i + 1, share_at(i + 1, rp1), S.shc, SHb);
#endif
      const uint64_t sz = entry_bytes(e.sh, e.kl, e.vl);
      {
#else
    uint64_t carry = 0;
    for (uint64_t base = 0; base < n; base += kThreads) {
      const uint64_t i = base + tid;
      Ent e{};
      uint64_t sz = 0;
      if (i < n) {
        e = entry_of(a.R, r0, i, shares(i, iv), S.shc);
        sz = entry_bytes(e.sh, e.kl, e.vl);
      }
      uint64_t tot = 0;
      const uint64_t eo = carry + wg_excl_scan(S, sz, tot);
      if (i < n) {
#endif
#if defined(MTBLX_ENC_ABL) && MTBLX_ENC_ABL == 1   // timing ablation only (wrong output): no global loads in the copy
        {
          const uint32_t l0 = vlen32(e.sh), l1 = vlen32(e.kl - e.sh), l2 = vlen32(e.vl);
          copy_bytes(dst + eo + l0 + l1 + l2, dst + eo, e.kl - e.sh + e.vl, dst);
        }
#elif defined(MTBLX_ENC_ABL) && MTBLX_ENC_ABL == 2   // timing ablation only: no entry bytes at all
#else
        put_entry(dst + eo, a.R, e);
#endif
#if MTBLX_ENC_CONTIG
        if (iv > 0 && rp == 0) put32(dst + R + 4 * ri++, (uint32_t)eo);
        rp = rp1;
#else
        if (iv > 0 && i % iv == 0) put32(dst + R + 4 * (i / iv), (uint32_t)eo);
#endif
      }
#if MTBLX_ENC_CONTIG
      eo += sz;
#else
      carry += tot;
#endif
    }
    if (tid == 0) {
      if (n == 0 || iv == 0) put32(dst + R, 0u);      // restarts[0] = 0 (entry 0 writes it otherwise)
      if (iv == 0 && n > 0) put32(dst + R + 4, 0u);   // the push of entry 0 (buf.len() == 0)
      put32(dst + L - 4, (uint32_t)nrest);            // restart count
      if constexpr (lds)                              // the CRC's pad to a 16-byte boundary
        for (uint64_t z = L; z & 15u; ++z) S.ob[z] = 0;
    }
  };
  if (in_lds) assemble(S.ob, std::true_type{});
  ESTAMP(4);   // assembly in LDS

#if MTBLX_ENC_TW && !defined(MTBLX_ENC_ABL)
  // Planned mode with the block CRC on the matrix cores (cfg3's path).  The file offset is known
  // (the scan of the framed sizes), so the block streams out right after the assembly and the
  // CRC runs beside its stores; only the 4-byte checksum of the frame waits for it.  The CRC's
  // operands are loaded -- and waited for -- BEFORE the stores: a vector-memory wait counts loads
  // and stores in issue order (round 5 issued the stores first and lost 5 % to exactly that).
  // Wave w takes step position t = w of every super-window (steps s = 8 S + w counted from the
  // padded end), so it needs one stage-2 operand (a2[w]) instead of one per step; the integer
  // parity is linear, so each step's stage-2 parities are Horner-combined over S with
  // x^(8·8192) (a 512-byte nibble table in LDS) and the waves' partial column words XOR-combined.
  if constexpr (PL) {
    static_assert(kWaves == mtblx_crc::kMSup, "one wave per step position of a super-window");
    if (MTBLX_ENC_CRC_MFMA && a.framed && in_lds && L >= 256 && st == MTBLX_ST_OK) {   // uniform
      using namespace mtblx_crc;
      const int g = lane >> 4, nn = lane & 15;
      v4i A[kMKs][2];
#pragma unroll
      for (int k = 0; k < kMKs; ++k) {
        A[k][0] = reinterpret_cast<const v4i*>(&kEncMfma.a[k][0][0][0])[lane];
        A[k][1] = reinterpret_cast<const v4i*>(&kEncMfma.a[k][1][0][0])[lane];
      }
      const v4i a2lo = reinterpret_cast<const v4i*>(&kEncMfma.a2[w][0][0][0])[lane];
      const v4i a2hi = reinterpret_cast<const v4i*>(&kEncMfma.a2[w][1][0][0])[lane];
      uint32_t(*hk)[16] = reinterpret_cast<uint32_t(*)[16]>(&S.T[0][0]);   // x^(8·8192): swk
      if (tid < 128) (&hk[0][0])[tid] = tw_swk;
      if (tid == 0) S.sh_u64[0] = tw_fin - F;
      tw_barrier();   // the block (and its zero pad), the table, the offset
#pragma unroll
      for (int k = 0; k < kMKs; ++k) asm volatile("" ::"v"(A[k][0]), "v"(A[k][1]));
      asm volatile("" ::"v"(a2lo), "v"(a2hi));   // the operands' wait is here, before the stores
      const uint64_t pre = S.sh_u64[0];
      const uint64_t coff = pre + vlen64(L) + 4;
      const bool fits = pre + F <= a.out_cap;
      if (fits) {   // stream the block out: aligned 16 B LDS reads, unaligned 16 B stores
        uint8_t* dst = a.out + coff;
        const uint64_t nch = L / 16;
        for (uint64_t c = tid; c < nch; c += kThreads) {
          const v4a x = *reinterpret_cast<const v4a*>(S.ob + 16 * c);
#if MTBLX_ENC_NT_STORES
          __builtin_nontemporal_store(v4u{x.x, x.y, x.z, x.w}, reinterpret_cast<v4u*>(dst + 16 * c));
#else
          *reinterpret_cast<v4u*>(dst + 16 * c) = v4u{x.x, x.y, x.z, x.w};
#endif
        }
        for (uint64_t o = 16 * nch + tid; o < L; o += kThreads) dst[o] = S.ob[o];
      }
      // this wave's steps, from the block start (Horner over the super-windows)
      uint32_t acc = 0;
      const uint32_t t = (16u - (uint32_t)(L & 15u)) & 15u, Lp = (uint32_t)L + t;
      const uint32_t steps = (Lp + kMStep - 1) / kMStep, nsup = (steps + kMSup - 1) / kMSup;
      const int32_t kx16 = 16 * (60 - 4 * nn + g);   // the lane's chunk of a step
      if (fits) {
        for (int sw = (int)nsup - 1; sw >= 0; --sw) {
          const uint32_t sp = (uint32_t)sw * kMSup + (uint32_t)w;
          uint32_t dv = 0;
          if (sp < steps) {   // wave-uniform
            const int32_t pos = (int32_t)Lp - (int32_t)(kMStep * (sp + 1)) + kx16;   // a multiple of 16
            v4a x = {0u, 0u, 0u, 0u};
            if (pos >= 0) x = *reinterpret_cast<const v4a*>(S.ob + pos);
            if (pos == 0) x.x ^= 0xFFFFFFFFu;   // the init, folded into bytes 0..3
            v4f c2a = {0.f, 0.f, 0.f, 0.f}, c2b = c2a;
            mfma_step(A, v4u{x.x, x.y, x.z, x.w}, a2lo, a2hi, c2a, c2b);
            dv = (par_nib(c2a) << (4 * g)) | (par_nib(c2b) << (16 + 4 * g));
          }
          acc = mul_nib(acc, hk) ^ dv;
        }
      }
      uint32_t* part = reinterpret_cast<uint32_t*>(S.shc);   // planned mode never reads shc
      part[w * kWave + lane] = acc;
      tw_barrier();   // the parts (LDS); the block's stores stay in flight
      ESTAMP(6);   // stores issued + CRC
      if (w == 0 && fits) {   // column shift x^(8·64·n), XOR over the columns, pad removal x^(-8t)
        uint32_t pw = 0;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) pw ^= part[k * kWave + lane];
        uint32_t c = row_xor(mul_nib(pw, kEncMfma.col[nn]));
        uint32_t C = (uint32_t)__builtin_amdgcn_readlane((int)c, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)c, 16) ^
                     (uint32_t)__builtin_amdgcn_readlane((int)c, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)c, 48);
        if (t) {
          const uint32_t j = (uint32_t)lane & 15u;
          const uint32_t v = j < 8u ? kEncMfma.inv[t][j][(C >> (4 * j)) & 15u] : 0u;
          C = (uint32_t)__builtin_amdgcn_readlane((int)row_xor(v), 0);
        }
        if (tid == 0) {   // varint64(L) | crc32c (write_block, src/writer.rs:203-237)
          uint32_t hl;
          const uint64_t hw = vpack(L, hl);
#pragma unroll
          for (uint32_t k = 0; k < 5; ++k)
            if (k < hl) a.out[pre + k] = (uint8_t)(hw >> (8 * k));
          put32(a.out + pre + hl, C ^ 0xFFFFFFFFu);
        }
      }
      ESTAMP(7);
#ifdef MTBLX_ENC_STAMPS
      if (tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(a.ticket) + 15, 1ull);
#endif
      if (tid == 0) {
        const int32_t st2 = fits ? MTBLX_ST_OK : MTBLX_ST_OVERFLOW;
        a.blk_off[b] = fits ? coff : 0;
        a.blk_len[b] = fits ? (uint32_t)L : 0u;
        a.status[b] = st2;
        if (!fits) atomicOr(reinterpret_cast<unsigned long long*>(a.totals + 1), 1ull);
        if (b == a.nblk - 1) a.totals[0] = pre + F;
      }
      return;
    }
  }
#endif

  // ---- look-back: this block's offset in the output (wave 0), beside the block CRC (all waves,
  // wave 0 after its look-back) ----
#if defined(MTBLX_ENC_ABL) && MTBLX_ENC_ABL == 3   // timing ablation only (wrong checksums): no block CRC
  const bool crc_mfma = false;
#else
  const bool crc_mfma = MTBLX_ENC_CRC_MFMA && a.framed && in_lds && L >= 4;
#endif
  if (crc_mfma) {
    __syncthreads();   // the assembled block (entries, restarts, count, pad) before its CRC
    if (w != 0 || PL) crc_mfma_part(S, (uint32_t)L);
  }
  if constexpr (PL) {   // the file offset: the scan of the framed sizes
    if (tid == 0) S.sh_u64[0] = a.fincl[b] - F;
  } else if (w == 0) {
    bool to = false;
    const uint64_t excl = b == 0 ? 0 : lookback(a, b, lane, to);
    if (lane == 0) {
      if (b != 0) __hip_atomic_store(a.lbw + b, kIncl | (excl + F), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      S.sh_u64[0] = excl;
      if (to) atomicOr(reinterpret_cast<unsigned long long*>(a.totals + 1), 2ull);
    }
    if (crc_mfma) crc_mfma_part(S, (uint32_t)L);
  }
  __syncthreads();
  ESTAMP(5);   // look-back
  const uint64_t pre = S.sh_u64[0];
  const uint64_t coff = pre + (a.framed ? vlen64(L) + 4 : 0);
  if (st == MTBLX_ST_OK && pre + F > a.out_cap) st = MTBLX_ST_OVERFLOW;
  if (st == MTBLX_ST_OK) {
    uint8_t* dst = a.out + coff;
    const uint8_t* src = S.ob;
    if (!in_lds) {   // large block: assemble in place in HBM
      assemble(dst, std::false_type{});
      __threadfence_block();
      __syncthreads();
      src = dst;
    }
    if (a.framed) {
#if MTBLX_ENC_LAZY_T && !(defined(MTBLX_ENC_ABL) && MTBLX_ENC_ABL == 3)
      if (!crc_mfma) {   // uniform over the workgroup
        build_tables();
        __syncthreads();
      }
#endif
#if defined(MTBLX_ENC_ABL) && MTBLX_ENC_ABL == 3
      const uint32_t crc = 0u;
      (void)src;
#else
      const uint32_t crc = crc_mfma ? crc_mfma_final(S, (uint32_t)L) : wg_crc32c(S, src, L);
#endif
      ESTAMP(6);   // CRC-32C
      if (tid == 0) {
        uint32_t hl;   // varint64(L) | crc32c (write_block, src/writer.rs:203-237)
        const uint64_t hw = vpack(L, hl);   // L < 2^35: 5 bytes at most
#pragma unroll
        for (uint32_t k = 0; k < 5; ++k)
          if (k < hl) a.out[pre + k] = (uint8_t)(hw >> (8 * k));
        put32(a.out + pre + hl, crc);
      }
    }
    if (in_lds) {   // stream the block out: aligned 16 B LDS reads, unaligned 16 B stores
      const uint64_t nch = L / 16;
      for (uint64_t c = tid; c < nch; c += kThreads) {
        const v4a x = *reinterpret_cast<const v4a*>(S.ob + 16 * c);
#if MTBLX_ENC_NT_STORES   // the framed file bytes are written once: stream them out
        __builtin_nontemporal_store(v4u{x.x, x.y, x.z, x.w}, reinterpret_cast<v4u*>(dst + 16 * c));
#else
        *reinterpret_cast<v4u*>(dst + 16 * c) = v4u{x.x, x.y, x.z, x.w};
#endif
      }
      for (uint64_t o = 16 * nch + tid; o < L; o += kThreads) dst[o] = S.ob[o];
    }
  }
  ESTAMP(7);   // stream out
#ifdef MTBLX_ENC_STAMPS
  if (tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(a.ticket) + 15, 1ull);
#endif
  if (tid == 0) {
    a.blk_off[b] = st == MTBLX_ST_OK ? coff : 0;
    a.blk_len[b] = st == MTBLX_ST_OK ? (uint32_t)L : 0u;
    a.status[b] = st;
    if (st != MTBLX_ST_OK) atomicOr(reinterpret_cast<unsigned long long*>(a.totals + 1), 1ull);
    if (b == a.nblk - 1) a.totals[0] = pre + F;
  }
}

}  // namespace mtblx_enc

using namespace mtblx_enc;

namespace mtblx_plan {   // plan.hip
uint64_t sscan_words(uint64_t m, uint64_t w);
int sscan(uint64_t* X, uint64_t m, uint64_t w, uint64_t* S, hipStream_t s);
}

namespace mtblx_enc {
// planned mode: every block's framed size from the kept sums (the same formula k_encode applies)
__global__ void __launch_bounds__(256) k_enc_fsize(EncArgs a, uint64_t* F) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= a.nblk) return;
  MTBLX_CHK(a.blk_rec + b, 16);
  const uint64_t r0 = a.blk_rec[b], n = a.blk_rec[b + 1] - r0;
  const uint32_t iv = a.interval;
  uint64_t f = 0;
  if (r0 >= a.plo && r0 + n <= a.plo + a.pm) {
    const uint64_t entries = planned_off(a, r0 - a.plo, n, iv);
    const uint64_t nrest = n == 0 ? 1 : 1 + (n - 1) / iv;
    const uint64_t L = entries + 4 * nrest + 4;
    f = a.framed ? vlen64(L) + 4 + L : L;
  }
  MTBLX_CHK(F + b, 8);
  F[b] = f;
}
}  // namespace mtblx_enc

extern "C" size_t mtblx_encode_workspace_bytes(uint32_t nblk) {
  // look-back words (mtblx_encode_blocks) or the framed sizes + their scan (..._planned)
  const uint64_t lb = 256u + 8ull * (uint64_t)nblk;
  const uint64_t pl = 256u + 8ull * (uint64_t)nblk + 8ull * mtblx_plan::sscan_words(nblk, 1) + 256u;
  return lb > pl ? lb : pl;
}

// the round-1..4 block cut: one wave per shard walking the Writer's chain (plan.hip dispatches here
// for MTBLX_PLAN=serial, record ranges of 2^32 or more, and workspaces too small for the parallel
// cut).  Scratch from the caller's workspace: [nshard] counts | [nshard] firsts | flags.
extern "C" int mtblx_encode_plan_serial(const mtblx_records* rec, const uint64_t* shard_rec, uint32_t nshard,
                                        uint64_t block_size, uint32_t restart_interval, uint64_t* blk_rec, uint64_t blk_cap,
                                        uint64_t* nblk_out, uint32_t* flags_out, void* workspace, size_t ws_bytes,
                                        void* stream) {
  if (!rec || !shard_rec || !nblk_out || nshard == 0) return MTBLX_E_INVAL;
  if (!workspace || ws_bytes < 16ull * nshard + 16 || (reinterpret_cast<uintptr_t>(workspace) & 7u)) return MTBLX_E_INVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (block_size < 1024) block_size = 1024;   // WriterBuilder::block_size clamp (src/writer.rs:43-46)
  uint64_t* d = static_cast<uint64_t*>(workspace);
  uint32_t* dflags = reinterpret_cast<uint32_t*>(d + 2 * nshard);
  int rc = MTBLX_OK;
  std::vector<uint64_t> cnt(nshard), first(nshard);
  uint32_t fl = 0;
  PlanArgs a{{rec->keys, rec->key_end, rec->vals, rec->val_end}, shard_rec, nshard, restart_interval, block_size,
             d, d + nshard, blk_rec, dflags, 0};
  if (hipMemsetAsync(dflags, 0, 16, s) != hipSuccess) rc = MTBLX_E_HIP;
  if (rc == MTBLX_OK) {
    MTBLX_LAUNCH((rec->keys, rec->key_end, rec->vals, rec->val_end, shard_rec, d, blk_rec), k_plan, dim3(nshard), dim3(kWave), 0, s, a);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(cnt.data(), d, 8ull * nshard, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(&fl, dflags, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
      rc = MTBLX_E_HIP;
  }
  uint64_t total = 0;
  for (uint32_t i = 0; i < nshard; ++i) {
    first[i] = total;
    total += cnt[i];
  }
  *nblk_out = total;
  if (flags_out) *flags_out = fl;
  if (rc == MTBLX_OK && blk_rec && total + 1 <= blk_cap) {
    a.write = 1;
    if (hipMemcpyAsync(d + nshard, first.data(), 8ull * nshard, hipMemcpyHostToDevice, s) != hipSuccess) rc = MTBLX_E_HIP;
    if (rc == MTBLX_OK) {
      MTBLX_LAUNCH((rec->keys, rec->key_end, rec->vals, rec->val_end, shard_rec, d, blk_rec), k_plan, dim3(nshard), dim3(kWave), 0, s, a);
      // blk_rec[total] = the end of the last shard
      if (hipGetLastError() != hipSuccess ||
          hipMemcpyAsync(blk_rec + total, shard_rec + nshard, 8, hipMemcpyDeviceToDevice, s) != hipSuccess)
        rc = MTBLX_E_HIP;
    }
  } else if (rc == MTBLX_OK && blk_rec) {
    rc = MTBLX_E_INVAL;   // blk_cap too small: *nblk_out says how many are needed
  }
  if (hipStreamSynchronize(s) != hipSuccess) rc = MTBLX_E_HIP;
  if (rc == MTBLX_OK && (fl & (MTBLX_PLAN_OUT_OF_ORDER | MTBLX_PLAN_PANIC | MTBLX_PLAN_TOO_LONG))) rc = MTBLX_E_FORMAT;
  return rc;
}

extern "C" int mtblx_encode_blocks(const mtblx_records* rec, const uint64_t* blk_rec, uint32_t nblk,
                                   uint32_t restart_interval, int framed, uint8_t* out, uint64_t out_cap,
                                   uint64_t* blk_off, uint32_t* blk_len, int32_t* status, uint64_t* totals,
                                   void* workspace, size_t ws_bytes, void* stream) {
  if (!rec || !blk_rec || !totals) return MTBLX_E_INVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(totals, 0, 16, s) != hipSuccess) return MTBLX_E_HIP;
  if (nblk == 0) return MTBLX_OK;
  if (!out || !blk_off || !blk_len || !status || !workspace || ws_bytes < mtblx_encode_workspace_bytes(nblk) ||
      (reinterpret_cast<uintptr_t>(workspace) & 7u))
    return MTBLX_E_INVAL;
  // the look-back words and the ticket are polled: zero them every call
  if (hipMemsetAsync(workspace, 0, mtblx_encode_workspace_bytes(nblk), s) != hipSuccess) return MTBLX_E_HIP;
  uint8_t* ws = reinterpret_cast<uint8_t*>(workspace);
  EncArgs a{{rec->keys, rec->key_end, rec->vals, rec->val_end},
            blk_rec,
            nblk,
            restart_interval,
            framed ? 1 : 0,
            out,
            out_cap,
            blk_off,
            blk_len,
            status,
            totals,
            reinterpret_cast<uint32_t*>(ws),
            reinterpret_cast<uint64_t*>(ws + 256)};
  MTBLX_LAUNCH((rec->keys, rec->key_end, rec->vals, rec->val_end, blk_rec, out, blk_off, blk_len, status, totals, workspace), k_encode<false>, dim3(nblk), dim3(kThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

extern "C" int mtblx_encode_blocks_planned(const mtblx_records* rec, const uint64_t* blk_rec, uint32_t nblk,
                                           uint32_t restart_interval, int framed, uint8_t* out, uint64_t out_cap,
                                           uint64_t* blk_off, uint32_t* blk_len, int32_t* status, uint64_t* totals,
                                           void* workspace, size_t ws_bytes, const void* plan, void* stream) {
  if (!rec || !blk_rec || !totals || !plan) return MTBLX_E_INVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint64_t h[4] = {0, 0, 0, 0};   // magic, first record, records, interval (plan.hip KeepHdr)
  if (hipMemcpyAsync(h, plan, sizeof(h), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return MTBLX_E_HIP;
  if (h[0] != 0x4e414c5058544d31ull || h[3] != restart_interval || restart_interval == 0) return MTBLX_E_INVAL;
  if (hipMemsetAsync(totals, 0, 16, s) != hipSuccess) return MTBLX_E_HIP;
  if (nblk == 0) return MTBLX_OK;
  if (!out || !blk_off || !blk_len || !status || !workspace || ws_bytes < mtblx_encode_workspace_bytes(nblk) ||
      (reinterpret_cast<uintptr_t>(workspace) & 7u))
    return MTBLX_E_INVAL;
  const uint64_t m = h[2];
  const uint8_t* kp = static_cast<const uint8_t*>(plan) + 256;
  const uint64_t* PA = reinterpret_cast<const uint64_t*>(kp);
  const uint64_t* Q = PA + (m + 1);
  const uint32_t* SH = reinterpret_cast<const uint32_t*>(Q + (m + 1));
  uint64_t* F = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(workspace) + 256);
  uint64_t* scr = F + nblk;
  EncArgs a{{rec->keys, rec->key_end, rec->vals, rec->val_end},
            blk_rec, nblk, restart_interval, framed ? 1 : 0, out, out_cap, blk_off, blk_len, status, totals,
            nullptr, nullptr, PA, Q, SH, h[1], m, F};
#ifdef MTBLX_ENC_STAMPS   // diagnostic build: the stamps go to the workspace's first 256 bytes (no ticket here)
  if (hipMemsetAsync(workspace, 0, 256, s) != hipSuccess) return MTBLX_E_HIP;
  a.ticket = reinterpret_cast<uint32_t*>(workspace);
#endif
  MTBLX_LAUNCH((MTBLX_R(blk_rec, 8ull * (nblk + 1)), MTBLX_R(PA, 8 * m), MTBLX_R(Q, 8 * m), MTBLX_R(F, 8ull * nblk)),
               k_enc_fsize, dim3((nblk + 255) / 256), dim3(256), 0, s, a, F);
  if (hipGetLastError() != hipSuccess) return MTBLX_E_HIP;
  const int rc = mtblx_plan::sscan(F, nblk, 1, scr, s);
  if (rc != MTBLX_OK) return rc;
  MTBLX_LAUNCH((rec->keys, rec->key_end, rec->vals, rec->val_end, MTBLX_R(blk_rec, 8ull * (nblk + 1)), out, blk_off, blk_len,
                status, totals, MTBLX_R(PA, 8 * m), MTBLX_R(Q, 8 * m), MTBLX_R(SH, 4 * m), MTBLX_R(F, 8ull * nblk)),
               k_encode<true>, dim3(nblk), dim3(kThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
