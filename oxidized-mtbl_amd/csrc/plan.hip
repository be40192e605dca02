// plan.hip — MI355X (gfx950) Writer block cut for every record at once.
//
//   Writer::insert flush rule              /root/reference/src/writer.rs:125-130
//   BlockBuilder::current_size_estimate    src/block_builder.rs:40-47
//   BlockBuilder::add restart bookkeeping  src/block_builder.rs:49-62
//   Writer::flush (no-op on an empty block) src/writer.rs:183-200
//   Writer::insert order check             src/writer.rs:119-123
//
// The Writer decides where a block ends one record at a time: record k starts a new block when
// current_size_estimate() + 15 + |key_k| + |val_k| >= block_size, where the estimate counts the
// entries since the block's first record j (entry p shares a prefix with its predecessor unless
// p % interval == 0) plus 4 bytes per restart and 4 for the count.  That is a serial chain over
// records, and the round-1..4 kernel (`k_plan`, now `mtblx_encode_plan_serial` in encode.hip) ran
// it with one wave per shard: a dependent chain of global loads per 64 records, 36 ms for one
// cfg3 chunk of 6.5 M records on 64 waves.
//
// Here the chain is cut differently.  For EVERY record j the end of the block that would start
// at j, next(j), is computed independently: the estimate of entries [j, k) is O(1) from two
// prefix sums -- A = entry sizes with sharing, and Q = the sizes sharing saves, summed along each
// residue class mod the interval (the restart entries of a block starting at j are j, j + iv,
// j + 2 iv, ...) -- so an exponential search finds the first k where est + max(15 + |k| + |v|)
// can reach the block size, and a scan over 64-record chunks (skipped whole when est at the
// chunk's end plus the chunk's largest 15 + |k| + |v| stays below it) finds the flushing record.
// The blocks a Writer actually cuts are the chain j0 = shard start, next(j0), next(next(j0)),
// ...: pointer doubling builds JL = next^8 and JH = next^(2^lvHi) (lvHi per call, so that the
// largest shard needs at most ~128 JH hops); one thread per shard walks JH (k_plan_top), one per
// JH waypoint walks JL (2^(lvHi-3) hops, k_plan_mid), one per 8-block waypoint walks next (8
// hops) and writes the block starts (k_plan_emit).  Every step is a parallel pass over the
// records, so the cut of any number of shards -- one Writer over all records included -- takes a
// fixed handful of launches.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "bounds.h"
#include "mtblx.h"

extern "C" int mtblx_encode_plan_serial(const mtblx_records* rec, const uint64_t* shard_rec, uint32_t nshard,
                                        uint64_t block_size, uint32_t restart_interval, uint64_t* blk_rec,
                                        uint64_t blk_cap, uint64_t* nblk_out, uint32_t* flags_out, void* workspace,
                                        size_t ws_bytes, void* stream);

namespace mtblx_plan {

constexpr int kT = 256;
constexpr int kWave = 64;
// levels kept: next, JL = next^(2^kLvLo), JH = next^(2^lvHi) with lvHi chosen per call so that
// one thread per shard walks at most ~128 JH hops (the estimated blocks of the largest shard)
constexpr int kLvLo = 3;
constexpr uint32_t kLow = 1u << kLvLo;        // blocks per JL hop = hops of the emitting walk
constexpr uint32_t kTileRows = 64;  // rows per tile of the strided scan

typedef uint64_t __attribute__((aligned(1))) u64u;

struct Recs {
  const uint8_t* keys;
  const uint64_t* key_end;
  const uint8_t* vals;
  const uint64_t* val_end;
};

__device__ __forceinline__ uint64_t vlen32(uint64_t v) {
  return v < (1ull << 7) ? 1u : v < (1ull << 14) ? 2u : v < (1ull << 21) ? 3u : v < (1ull << 28) ? 4u : 5u;
}
// one BlockBuilder entry: varint32 shared | non_shared | value_length, key suffix, value (:69-77)
__device__ __forceinline__ uint64_t entry_bytes(uint64_t sh, uint64_t kl, uint64_t vl) {
  return vlen32(sh) + vlen32(kl - sh) + vlen32(vl) + (kl - sh) + vl;
}

// the shard holding local record j: the last s with sb[s] <= j (empty shards never match)
__device__ __forceinline__ uint32_t shard_of(const uint64_t* sb, uint32_t nsh, uint64_t j) {
  uint32_t lo = 0, hi = nsh;   // sb[lo] <= j < sb[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    MTBLX_CHK(sb + mid, 8);
    if (sb[mid] <= j) lo = mid; else hi = mid;
  }
  return lo;
}

struct RecArgs {
  Recs R;
  uint64_t lo, m;
  const uint64_t* sb;   // [nsh + 1] local shard starts
  uint32_t nsh;
  uint64_t* A;          // [m] entry size with sharing
  uint64_t* D;          // [m] size the sharing saves (restart entries pay it back)
  uint64_t* G;          // [m] 15 + |key| + |value|: the flush test's record term
  uint64_t* GM;         // [ceil(m / 64)] max G per 64-record chunk
  uint32_t* flags;
  uint32_t* SH;         // nullable: [m] the shared-prefix length with the previous record (kept for the encode)
};

// per record: sizes, the order check (key > predecessor within the shard) and the length limit
__global__ void __launch_bounds__(kT) k_plan_rec(RecArgs a) {
  const int lane = threadIdx.x & (kWave - 1);
  uint32_t fl = 0;
  for (uint64_t base = (uint64_t)blockIdx.x * kT; base < a.m; base += (uint64_t)gridDim.x * kT) {
    const uint64_t j = base + threadIdx.x;
    uint64_t g = 0;
    if (j < a.m) {
      const uint64_t i = a.lo + j;
      MTBLX_CHK(a.R.key_end + i, 8), MTBLX_CHK(a.R.val_end + i, 8);
      const uint64_t k0 = i ? a.R.key_end[i - 1] : 0, k1 = a.R.key_end[i];
      const uint64_t v0 = i ? a.R.val_end[i - 1] : 0, v1 = a.R.val_end[i];
      const uint64_t kl = k1 - k0, vl = v1 - v0;
      if (kl > 0xFFFFFFFFull || vl > 0xFFFFFFFFull) fl |= MTBLX_PLAN_TOO_LONG;
      const uint32_t s = shard_of(a.sb, a.nsh, j);
      uint64_t sh = 0;
      // the shared prefix with the predecessor (also across a shard start: a block of another cut
      // that spans it shares there, mtblx_encode_blocks_planned; the Writer's own cut starts a
      // block at every shard start, where the restart entry pays D back); the order check only
      // inside a Writer (src/writer.rs:119-123)
      if (i > 0) {
        const uint64_t p0 = i > 1 ? a.R.key_end[i - 2] : 0, pl = k0 - p0;
        const uint8_t* x = a.R.keys + p0;
        const uint8_t* y = a.R.keys + k0;
        const uint64_t mm = pl < kl ? pl : kl;
        uint64_t c = 0;
        int cmp = 0;
        bool done = false;
        while (c + 8 <= mm) {
          MTBLX_CHK(x + c, 8), MTBLX_CHK(y + c, 8);
          const uint64_t u = *reinterpret_cast<const u64u*>(x + c), w = *reinterpret_cast<const u64u*>(y + c);
          if (u != w) {
            c += (uint64_t)(__builtin_ctzll(u ^ w) >> 3);
            cmp = x[c] < y[c] ? -1 : 1;
            done = true;
            break;
          }
          c += 8;
        }
        if (!done) {
          while (c < mm && (MTBLX_CHK(x + c, 1), MTBLX_CHK(y + c, 1), x[c] == y[c])) ++c;
          cmp = c < mm ? (x[c] < y[c] ? -1 : 1) : (pl < kl ? -1 : (pl > kl ? 1 : 0));
        }
        if (cmp >= 0 && j != a.sb[s]) fl |= MTBLX_PLAN_OUT_OF_ORDER;
        sh = c;
      }
      const uint64_t A = entry_bytes(sh, kl, vl), Z = entry_bytes(0, kl, vl);
      g = 15 + kl + vl;
      MTBLX_CHK(a.A + j, 8), MTBLX_CHK(a.D + j, 8), MTBLX_CHK(a.G + j, 8);
      a.A[j] = A;
      a.D[j] = Z - A;
      a.G[j] = g;
      if (a.SH) {
        MTBLX_CHK(a.SH + j, 4);
        a.SH[j] = (uint32_t)(sh < 0xFFFFFFFFull ? sh : 0xFFFFFFFFull);
      }
    }
    // the chunk's largest record term (a wave = one aligned 64-record chunk)
    uint64_t mx = g;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const uint64_t o = __shfl_xor(mx, d, kWave);
      mx = o > mx ? o : mx;
    }
    if (lane == 0 && base + threadIdx.x < a.m) {
      MTBLX_CHK(a.GM + (base + threadIdx.x) / 64, 8);
      a.GM[(base + threadIdx.x) / 64] = mx;
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) fl |= (uint32_t)__shfl_xor((int)fl, d, kWave);
  if (lane == 0 && fl) atomicOr(a.flags, fl);
}

// max over GM: a grid-stride slice per workgroup, one atomic each (a same-address atomic per
// wave serialises ~100 k of them; one workgroup alone reads 8 MB too slowly)
__global__ void __launch_bounds__(1024) k_plan_gmax(const uint64_t* GM, uint64_t n, uint64_t* out) {
  __shared__ uint64_t part[1024 / kWave];
  uint64_t mx = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 1024) {
    MTBLX_CHK(GM + i, 8);
    mx = GM[i] > mx ? GM[i] : mx;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t o = __shfl_xor(mx, d, kWave);
    mx = o > mx ? o : mx;
  }
  if ((threadIdx.x & (kWave - 1)) == 0) part[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 1024 / kWave; ++k) mx = part[k] > mx ? part[k] : mx;
    MTBLX_CHK(out, 8);
    atomicMax(reinterpret_cast<unsigned long long*>(out), (unsigned long long)mx);
  }
}

// ---- strided inclusive scan in place: X[j] += X[j - w] + X[j - 2w] + ... (the columns of a
// row-major [rows][w] matrix scanned downwards; w = 1 is the plain prefix sum).  Tiles of
// kTileRows rows: the tile sums S[t][column] (up) are themselves a strided scan problem with
// stride min(w, m), solved recursively; the rescan (down) starts each tile from the previous
// tile's inclusive sum.  One column of at most kTileRows rows: a thread each (small). ----
__global__ void __launch_bounds__(kT) k_sscan_up(const uint64_t* X, uint64_t m, uint64_t w, uint64_t wc,
                                                 uint64_t nt, uint64_t* S) {
  const uint64_t it = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (it >= nt * wc) return;
  const uint64_t t = it / wc, r = it % wc;
  uint64_t s = 0;
  for (uint64_t q = t * kTileRows; q < (t + 1) * kTileRows; ++q) {
    const uint64_t j = q * w + r;
    if (j >= m) break;
    MTBLX_CHK(X + j, 8);
    s += X[j];
  }
  MTBLX_CHK(S + t * wc + r, 8);
  S[t * wc + r] = s;
}

__global__ void __launch_bounds__(kT) k_sscan_down(uint64_t* X, uint64_t m, uint64_t w, uint64_t wc, uint64_t nt,
                                                   const uint64_t* S) {
  const uint64_t it = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (it >= nt * wc) return;
  const uint64_t t = it / wc, r = it % wc;
  uint64_t run = 0;
  if (t) {
    MTBLX_CHK(S + (t - 1) * wc + r, 8);
    run = S[(t - 1) * wc + r];
  }
  for (uint64_t q = t * kTileRows; q < (t + 1) * kTileRows; ++q) {
    const uint64_t j = q * w + r;
    if (j >= m) break;
    MTBLX_CHK(X + j, 8);
    run += X[j];
    X[j] = run;
  }
}

// n / d for 32-bit n and a divisor fixed per launch (Granlund-Montgomery: multiply-high + shift);
// a 64-bit division per probe was most of k_plan_next's vector instructions
struct FastDiv {
  uint32_t d, m, s;
  static FastDiv make(uint32_t d) {
    FastDiv f{d, 0, 0};
    if (d > 1) {
      uint32_t l = 0;
      while ((1ull << l) < d) ++l;
      f.m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
      f.s = l - 1;
    }
    return f;
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    if (d == 1) return n;
    const uint32_t t = __umulhi(m, n);
    return (t + ((n - t) >> 1)) >> s;
  }
};

struct NextArgs {
  uint64_t m;
  uint32_t iv;
  uint64_t B;
  const uint64_t* PA;   // inclusive prefix of A
  const uint64_t* Q;    // inclusive prefix of D along residue classes mod iv (iv == 0: D itself)
  const uint64_t* G;
  const uint64_t* GM;
  const uint64_t* gmax;
  const uint64_t* sb;   // [nsh + 1] local shard starts
  uint32_t nsh;
  uint32_t* next;       // [m] local index of the record that starts the next block (or the shard end)
  uint8_t* pan;         // [m] iv == 0: a second entry would be added (assert, src/block_builder.rs:50)
  FastDiv div;          // by iv
};

// current_size_estimate() of a block holding entries [j, k) (src/block_builder.rs:40-47)
__device__ __forceinline__ uint64_t est(const NextArgs& a, uint64_t j, uint64_t base_a, uint64_t base_q, uint64_t k) {
  const uint64_t q = a.div.div((uint32_t)(k - 1 - j));   // < 2^32: the plan has fewer records
  const uint64_t nr = 1 + q;
  const uint64_t last = j + q * (uint64_t)a.iv;
  MTBLX_CHK(a.PA + k - 1, 8), MTBLX_CHK(a.Q + last, 8);
  const uint64_t buf = a.PA[k - 1] - base_a + a.Q[last] - base_q;
  return buf + nr * (buf > 0xFFFFFFFFull ? 8u : 4u) + 4u;
}

#ifndef MTBLX_PLAN_BATCH   // the direct probes as one batch of four loads (1: 14.5-14.7 ms) or one by one (0: 14.8)
#define MTBLX_PLAN_BATCH 1
#endif
#ifndef MTBLX_PLAN_LIN   // records probed one by one after ka before the 64-record chunk skip (0: 16.0 ms, 4: 14.9 ms per 3 cfg3 chunks)
#define MTBLX_PLAN_LIN 4
#endif
// next(j) for a start j of a shard ending at e (j + 1 < e, interval >= 1).  The first k with
// est(k) + gmax >= B (est grows with k) is bracketed by a gallop from `guess` (first step d) and
// bisected -- ka, returned for the next start's guess; from there the flushing record is found
// chunk by chunk (a 64-record chunk is skipped while est at its last record + its largest record
// term stays below the block size).
__device__ __forceinline__ uint64_t find_next(const NextArgs& a, uint64_t j, uint64_t e, uint64_t guess, uint64_t d,
                                              uint64_t gm, uint64_t& ka) {
  const uint64_t base_a = j ? a.PA[j - 1] : 0;
  const uint64_t base_q = j >= a.iv ? a.Q[j - a.iv] : 0;
  const uint64_t e1 = e - 1;
  const uint64_t k0 = guess < j + 1 ? j + 1 : (guess > e1 ? e1 : guess);
  uint64_t lo = j, hi = 0;   // lo: a k known false (j: none yet); hi: a k known true (0: none)
  if (est(a, j, base_a, base_q, k0) + gm >= a.B) {
    hi = k0;
    while (hi > j + 1) {   // downwards: a false k below hi
      const uint64_t k = hi - j - 1 > d ? hi - d : j + 1;
      if (est(a, j, base_a, base_q, k) + gm < a.B) { lo = k; break; }
      hi = k;
      d <<= 1;
    }
  } else {
    lo = k0;
    while (lo < e1) {   // upwards: a true k above lo
      const uint64_t k = e1 - lo > d ? lo + d : e1;
      if (est(a, j, base_a, base_q, k) + gm >= a.B) { hi = k; break; }
      lo = k;
      d <<= 1;
    }
  }
  if (!hi) {
    ka = e;
    return e;
  }
  while (hi - lo > 1) {
    const uint64_t mid = lo + ((hi - lo) >> 1);
    if (est(a, j, base_a, base_q, mid) + gm >= a.B) hi = mid; else lo = mid;
  }
  ka = hi;
  uint64_t k = hi;
  // the flushing record is usually within a few records of ka (gm bounds every record's term
  // from above): probe those directly before skipping by 64-record chunks
#if MTBLX_PLAN_BATCH
  {   // the four probes' loads issued together (one round trip), then tested in order
    uint64_t ev[4], gv[4];
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
      const uint64_t kc = k + u <= e1 ? k + u : k;   // k <= e1 here
      MTBLX_CHK(a.G + kc, 8);
      gv[u] = a.G[kc];
      ev[u] = est(a, j, base_a, base_q, kc);
    }
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u)
      if (k + u <= e1 && ev[u] + gv[u] >= a.B) return k + u;
    k = k + 4 <= e1 + 1 ? k + 4 : e1 + 1;
  }
#else
  for (uint32_t t = 0; t < MTBLX_PLAN_LIN && k <= e1; ++t, ++k) {
    MTBLX_CHK(a.G + k, 8);
    if (est(a, j, base_a, base_q, k) + a.G[k] >= a.B) return k;
  }
#endif
  while (k <= e1) {
    const uint64_t cl = std::min<uint64_t>((k | 63u), e1);
    MTBLX_CHK(a.GM + (k >> 6), 8);
    if (est(a, j, base_a, base_q, cl) + a.GM[k >> 6] < a.B) { k = cl + 1; continue; }
    for (; k <= cl; ++k) {
      MTBLX_CHK(a.G + k, 8);
      if (est(a, j, base_a, base_q, k) + a.G[k] >= a.B) return k;
    }
  }
  return e;
}

// kSweep starts per thread, kT apart (neighbouring threads take neighbouring starts: their probes
// coalesce): the first from a probe at the typical block length, each next one from the previous
// one's threshold + kT, which moves by about as much as the start did -- a few probes instead of
// a full search
#ifndef MTBLX_PLAN_SWEEP   // starts per thread in k_plan_next
#define MTBLX_PLAN_SWEEP 8
#endif
constexpr uint32_t kSweep = MTBLX_PLAN_SWEEP;
#ifndef MTBLX_PLAN_D0   // first gallop step from the previous start's threshold + kT (1: 16.3 ms, 8: 15.5 ms per 3 cfg3 chunks)
#define MTBLX_PLAN_D0 8
#endif
__global__ void __launch_bounds__(kT) k_plan_next(NextArgs a) {
  // the shard starts in LDS when they fit (the shard search is on every thread's chain)
  constexpr uint32_t kLsb = 1024;
  __shared__ uint64_t lsb[kLsb];
  const bool in_lds = a.nsh + 1 <= kLsb;
  if (in_lds) {
    for (uint32_t i = threadIdx.x; i <= a.nsh; i += kT) {
      MTBLX_CHK(a.sb + i, 8);
      lsb[i] = a.sb[i];
    }
    __syncthreads();
  }
  const uint64_t* sbp = in_lds ? lsb : a.sb;
  const uint64_t gm = *a.gmax;
  // typical records per block: block size / mean entry size (a heuristic: only where to probe first)
  const double tot = (double)a.PA[a.m - 1];
  const double hd = tot > 0.0 ? (double)a.B * (double)a.m / tot : 1.0;
  const uint64_t hint = hd < 1.0 ? 1u : hd > 1e12 ? (uint64_t)1e12 : (uint64_t)hd;
  uint64_t pe = 0, pka = 0;   // the previous start's shard end and threshold (pe == 0: none)
  for (uint32_t q = 0; q < kSweep; ++q) {
    const uint64_t j = ((uint64_t)blockIdx.x * kSweep + q) * kT + threadIdx.x;
    if (j >= a.m) break;
    const uint64_t e = j < pe ? pe : sbp[shard_of(sbp, a.nsh, j) + 1];
    uint64_t nx = e;
    if (a.pan) {
      MTBLX_CHK(a.pan + j, 1);
      a.pan[j] = 0;
    }
    if (j + 1 < e) {
      if (a.iv == 0) {   // the first add pushes a second restart (restarts = [0, 0]); a second add panics
        MTBLX_CHK(a.Q + j, 8), MTBLX_CHK(a.G + j + 1, 8), MTBLX_CHK(a.pan + j, 1);
        const uint64_t z = a.PA[j] - (j ? a.PA[j - 1] : 0) + a.Q[j];
        const uint64_t es = z + 2 * (z > 0xFFFFFFFFull ? 8u : 4u) + 4u;
        a.pan[j] = es + a.G[j + 1] >= a.B ? 0 : 1;
        nx = j + 1;
      } else if (e == pe && pka < pe) {   // the same shard: from the previous threshold
        nx = find_next(a, j, e, pka + kT, MTBLX_PLAN_D0, gm, pka);
      } else {
        nx = find_next(a, j, e, j + hint, hint / 16 + 1, gm, pka);
      }
    }
    pe = e;
    MTBLX_CHK(a.next + j, 4);
    a.next[j] = (uint32_t)nx;
  }
}

// the shard ends (local), one bit each: bit x set <=> x ends a shard (x <= m)
__global__ void __launch_bounds__(kT) k_plan_bounds(const uint64_t* sb, uint32_t nsh, uint32_t* bnd) {
  const uint32_t s = blockIdx.x * kT + threadIdx.x;
  if (s >= nsh) return;
  const uint64_t x = sb[s + 1];
  MTBLX_CHK(bnd + (x >> 5), 4);
  atomicOr(bnd + (x >> 5), 1u << (x & 31));
}

// one doubling step: dst = src o src, saturated at the shard end.  next(j) lies in (j, shard
// end], and the only shard end in that range is j's own, so "src[j] is a shard end" is one bit.
__global__ void __launch_bounds__(kT) k_plan_jump(const uint32_t* src, uint32_t* dst, const uint32_t* bnd, uint64_t m) {
  const uint64_t j = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (j >= m) return;
  MTBLX_CHK(src + j, 4), MTBLX_CHK(dst + j, 4);
  const uint32_t x = src[j];
  const uint32_t xs = x < m ? x : (uint32_t)(m - 1);   // loaded beside the bit (x == m is a shard end)
  MTBLX_CHK(bnd + (x >> 5), 4), MTBLX_CHK(src + xs, 4);
  const uint32_t b = bnd[x >> 5], y = src[xs];
  dst[j] = ((b >> (x & 31)) & 1u) ? x : y;
}

struct WalkArgs {
  const uint64_t* sb;      // [nsh + 1]
  uint32_t nsh;
  const uint64_t* base12;  // [nsh + 1] slot bases of each shard's next^512 waypoints
  uint32_t* n12;           // [nsh]
  uint32_t* W12;           // [slots]
  uint32_t* n6;            // [slots]
  const uint64_t* base6;   // [nsh + 1] W6 bases: shard s holds ceil(r_s / 8) next^8 waypoints at most
  uint32_t* W6;            // [base6[nsh]]
  const uint32_t* J0;
  const uint32_t* J6;
  const uint32_t* J12;
  uint64_t* nb;            // [nsh] blocks per shard
  const uint64_t* bb;      // [nsh] first block index of each shard
  uint64_t* blk_rec;       // nullable
  uint64_t lo;
  const uint8_t* pan;      // nullable (iv != 0)
  uint32_t* flags;
  uint64_t slots;
  uint32_t mid, top;       // JL hops per JH hop; blocks per JH hop
};

// one thread per shard: its next^512 waypoints
__global__ void __launch_bounds__(kT) k_plan_top(WalkArgs a) {
  const uint32_t s = blockIdx.x * kT + threadIdx.x;
  if (s >= a.nsh) return;
  const uint64_t b = a.sb[s], e = a.sb[s + 1];
  uint32_t c = 0;
  if (b < e) {
    uint64_t cur = b;
    while (true) {
      MTBLX_CHK(a.W12 + a.base12[s] + c, 4), MTBLX_CHK(a.J12 + cur, 4);
      a.W12[a.base12[s] + c] = (uint32_t)cur;
      ++c;
      const uint64_t nx = a.J12[cur];
      if (nx >= e || a.base12[s] + c >= a.base12[s + 1]) break;
      cur = nx;
    }
  }
  a.n12[s] = c;
}

// one thread per next^(2^lvHi) waypoint slot: its (up to) `mid` next^8 waypoints.  Waypoint q of
// shard s writes W6[base6[s] + q * mid + c]: every slot before the shard's last one is full (a JH
// hop is `mid` JL hops), so index q * mid + c counts JL waypoints from the shard start, i.e. block
// starts / 8 < ceil(r_s / 8) -- the shard's W6 range is sized by its own records (not by `top`)
__global__ void __launch_bounds__(kT) k_plan_mid(WalkArgs a) {
  const uint64_t u = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (u >= a.slots) return;
  uint32_t s = 0, hi = a.nsh;   // the shard whose slot range holds u: last s with base12[s] <= u
  while (hi - s > 1) {
    const uint32_t mid = (s + hi) >> 1;
    if (a.base12[mid] <= u) s = mid; else hi = mid;
  }
  uint32_t c = 0;
  if (u - a.base12[s] < a.n12[s]) {
    const uint64_t e = a.sb[s + 1];
    const uint64_t w0 = a.base6[s] + (u - a.base12[s]) * a.mid, w1 = a.base6[s + 1];
    uint64_t cur = a.W12[u];
    for (c = 0; c < a.mid && w0 + c < w1;) {
      MTBLX_CHK(a.W6 + w0 + c, 4), MTBLX_CHK(a.J6 + cur, 4);
      a.W6[w0 + c] = (uint32_t)cur;
      ++c;
      const uint64_t nx = a.J6[cur];
      if (nx >= e) break;
      cur = nx;
    }
  }
  MTBLX_CHK(a.n6 + u, 4);
  a.n6[u] = c;
}

// one thread per shard: its block count = full next^512 and next^8 steps + the last walk
__global__ void __launch_bounds__(kT) k_plan_count(WalkArgs a) {
  const uint32_t s = blockIdx.x * kT + threadIdx.x;
  if (s >= a.nsh) return;
  uint64_t n = 0;
  if (a.n12[s]) {
    const uint64_t u = a.base12[s] + a.n12[s] - 1;
    const uint32_t c6 = a.n6[u];
    const uint64_t e = a.sb[s + 1];
    uint64_t cur = a.W6[a.base6[s] + (uint64_t)(a.n12[s] - 1) * a.mid + c6 - 1], c = 0;
    while (true) {
      ++c;
      const uint64_t nx = a.J0[cur];
      if (nx >= e || c == kLow) break;
      cur = nx;
    }
    n = (uint64_t)(a.n12[s] - 1) * a.top + (uint64_t)(c6 - 1) * kLow + c;
  }
  a.nb[s] = n;
}

// one thread per next^8 waypoint slot of W6: its (up to) 8 blocks -> blk_rec; the restart-interval-0
// panic of any block holding two records
__global__ void __launch_bounds__(kT) k_plan_emit(WalkArgs a) {
  const uint64_t v = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (v >= a.base6[a.nsh]) return;
  uint32_t s = 0, hi = a.nsh;   // the shard whose W6 range holds v: last s with base6[s] <= v
  while (hi - s > 1) {
    const uint32_t mid = (s + hi) >> 1;
    if (a.base6[mid] <= v) s = mid; else hi = mid;
  }
  const uint64_t q = (v - a.base6[s]) / a.mid, w = (v - a.base6[s]) % a.mid;
  if (q >= a.n12[s]) return;
  const uint64_t u = a.base12[s] + q;
  MTBLX_CHK(a.n6 + u, 4);
  if (w >= a.n6[u]) return;
  const uint64_t e = a.sb[s + 1];
  uint64_t cur = a.W6[v];
  uint64_t out = a.bb ? a.bb[s] + q * a.top + w * kLow : 0;
  bool panic = false;
  for (uint32_t c = 0; c < kLow; ++c) {
    if (a.blk_rec) {
      MTBLX_CHK(a.blk_rec + out + c, 8);
      a.blk_rec[out + c] = a.lo + cur;
    }
    if (a.pan) panic |= a.pan[cur] != 0;
    MTBLX_CHK(a.J0 + cur, 4);
    const uint64_t nx = a.J0[cur];
    if (nx >= e) break;
    cur = nx;
  }
  if (panic) atomicOr(a.flags, MTBLX_PLAN_PANIC);
}

inline unsigned grid_of(uint64_t n, uint64_t per = kT) { return (unsigned)std::max<uint64_t>(1, (n + per - 1) / per); }

// Strides dividing 64 (1, 2, 4, ..., 64: the usual restart intervals and the plain prefix sum):
// a wave owns a tile of 4096 contiguous elements, rows of 64 lanes read coalesced; lane l's
// elements are all of class l mod w, so a row's class sums are a stride-w shuffle scan and a
// lane carries its class's running total down the rows.  Tile sums S[t][class] again form a
// stride-w problem (recursion, 4096x smaller each level).
constexpr uint64_t kWT = 4096;   // elements per wave tile
__global__ void __launch_bounds__(kT) k_wscan_up(const uint64_t* X, uint64_t m, uint32_t w, uint64_t nt, uint64_t* S) {
  const uint64_t t = ((uint64_t)blockIdx.x * kT + threadIdx.x) / kWave;
  const uint32_t l = threadIdx.x & (kWave - 1);
  if (t >= nt) return;
  uint64_t sum = 0;
  for (uint64_t q = 0; q < kWT / kWave; ++q) {
    const uint64_t e = t * kWT + q * kWave + l;
    if (e < m) {
      MTBLX_CHK(X + e, 8);
      sum += X[e];
    }
  }
  for (uint32_t d = w; d < (uint32_t)kWave; d <<= 1) sum += __shfl_xor(sum, d, kWave);
  if (l < w) {
    MTBLX_CHK(S + t * w + l, 8);
    S[t * w + l] = sum;
  }
}

__global__ void __launch_bounds__(kT) k_wscan_down(uint64_t* X, uint64_t m, uint32_t w, uint64_t nt, const uint64_t* S) {
  const uint64_t t = ((uint64_t)blockIdx.x * kT + threadIdx.x) / kWave;
  const uint32_t l = threadIdx.x & (kWave - 1);
  if (t >= nt) return;
  uint64_t carry = 0;
  if (t) {
    MTBLX_CHK(S + (t - 1) * w + (l % w), 8);
    carry = S[(t - 1) * w + (l % w)];
  }
  for (uint64_t q = 0; q < kWT / kWave; ++q) {
    const uint64_t e = t * kWT + q * kWave + l;
    if (t * kWT + q * kWave >= m) break;   // wave-uniform
    uint64_t x = 0;
    if (e < m) {
      MTBLX_CHK(X + e, 8);
      x = X[e];
    }
    for (uint32_t d = w; d < (uint32_t)kWave; d <<= 1) {
      const uint64_t y = __shfl_up(x, d, kWave);
      if (l >= d) x += y;
    }
    if (e < m) X[e] = carry + x;
    carry += __shfl(x, kWave - w + (l % w), kWave);
  }
}

inline bool wave_stride(uint64_t w) { return w <= (uint64_t)kWave && (kWave % w) == 0; }

// words of scratch the strided scan of m elements with stride w needs (all recursion levels)
uint64_t sscan_words(uint64_t m, uint64_t w) {
  uint64_t tot = 0;
  while (m) {
    if (wave_stride(w)) {
      if (m <= kWT) break;
      const uint64_t nt = (m + kWT - 1) / kWT;
      tot += nt * w;
      m = nt * w;
      continue;
    }
    const uint64_t wc = std::min<uint64_t>(w, m), rows = (m + w - 1) / w;
    if (rows <= kTileRows) break;
    const uint64_t nt = (rows + kTileRows - 1) / kTileRows;
    tot += nt * wc;
    m = nt * wc;
    w = wc;
  }
  return tot;
}

// strided inclusive scan of X[0..m) with stride w (S: sscan_words(m, w) words of scratch)
int sscan(uint64_t* X, uint64_t m, uint64_t w, uint64_t* S, hipStream_t s) {
  if (m == 0) return MTBLX_OK;
  if (wave_stride(w)) {
    const uint64_t nt = (m + kWT - 1) / kWT;
    const unsigned g = grid_of(nt * kWave);
    if (nt == 1) {
      MTBLX_LAUNCH((MTBLX_R(X, 8 * m)), k_wscan_down, dim3(g), dim3(kT), 0, s, X, m, (uint32_t)w, nt,
                   (const uint64_t*)nullptr);
      return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
    }
    MTBLX_LAUNCH((MTBLX_R(X, 8 * m), MTBLX_R(S, 8 * nt * w)), k_wscan_up, dim3(g), dim3(kT), 0, s, X, m, (uint32_t)w, nt, S);
    const int rc = sscan(S, nt * w, w, S + nt * w, s);
    if (rc != MTBLX_OK) return rc;
    MTBLX_LAUNCH((MTBLX_R(X, 8 * m), MTBLX_R(S, 8 * nt * w)), k_wscan_down, dim3(g), dim3(kT), 0, s, X, m, (uint32_t)w, nt,
                 S);
    return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
  }
  const uint64_t wc = std::min<uint64_t>(w, m), rows = (m + w - 1) / w;
  const uint64_t nt = (rows + kTileRows - 1) / kTileRows;
  if (nt == 1) {   // every column in one tile: its thread scans it
    MTBLX_LAUNCH((MTBLX_R(X, 8 * m)), k_sscan_down, dim3(grid_of(wc)), dim3(kT), 0, s, X, m, w, wc, nt,
                 (const uint64_t*)nullptr);
    return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
  }
  MTBLX_LAUNCH((MTBLX_R(X, 8 * m), MTBLX_R(S, 8 * nt * wc)), k_sscan_up, dim3(grid_of(nt * wc)), dim3(kT), 0, s, X, m, w,
               wc, nt, S);
  const int rc = sscan(S, nt * wc, wc, S + nt * wc, s);
  if (rc != MTBLX_OK) return rc;
  MTBLX_LAUNCH((MTBLX_R(X, 8 * m), MTBLX_R(S, 8 * nt * wc)), k_sscan_down, dim3(grid_of(nt * wc)), dim3(kT), 0, s, X, m,
               w, wc, nt, S);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

}  // namespace mtblx_plan

using namespace mtblx_plan;

// the kept plan (mtblx_encode_plan_keep): header, then PA [m] u64, Q [m] u64, SH [m] u32
struct KeepHdr {
  uint64_t magic, lo, m, iv;
};
constexpr uint64_t kKeepMagic = 0x4e414c5058544d31ull;   // "1MTXPLAN"
inline size_t keep_bytes(uint64_t n) { return 256 + 16 * (n + 1) + 4 * (n + 1) + 256; }

// The parallel cut's scratch, carved from the caller's workspace (the library keeps none of its
// own).  Sized by bounds that hold whatever the record sizes: the next^(2^lvHi) waypoint slots,
// sum over shards of ceil(r_s / top) <= m / 16 + nshard (top >= 16), and the next^8 waypoints,
// sum of ceil(r_s / 8) <= m / 8 + nshard -- so the size depends on (records, shards, interval) only.
struct PlanLayout {
  size_t oA, oD, oG, oGM, oS, oSB, oB12, oB6, oNB, oBB, oMX, oFL, oE, oJ0, oT1, oT2, oJ6, oJ12, oN12, oW12, oN6, oW6,
      oPAN, bytes;
};
static PlanLayout plan_layout(uint64_t m, uint32_t nshard, uint32_t iv, bool keep) {
  PlanLayout L{};
  const uint64_t m1 = std::max<uint64_t>(m, 1), nchunk = std::max<uint64_t>((m + 63) / 64, 1);
  const uint64_t scan_words = std::max<uint64_t>(std::max(sscan_words(m, 1), iv ? sscan_words(m, iv) : 0), 1);
  const uint64_t slots = m / 16 + nshard + 1, w6 = m / 8 + nshard + 1;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
  // 8-byte arrays first (A and D live in the kept plan in keep mode)
  L.oA = keep ? 0 : take(8 * m1);
  L.oD = keep ? 0 : take(8 * m1);
  L.oG = take(8 * m1);
  L.oGM = take(8 * nchunk);
  L.oS = take(8 * scan_words);
  L.oSB = take(8ull * (nshard + 1));
  L.oB12 = take(8ull * (nshard + 1));
  L.oB6 = take(8ull * (nshard + 1));
  L.oNB = take(8ull * nshard);
  L.oBB = take(8ull * nshard);
  L.oMX = take(8);
  L.oFL = take(4);
  L.oE = take(4 * ((m1 + 32) / 32 + 1));
  L.oJ0 = take(4 * m1);
  L.oT1 = take(4 * m1);
  L.oT2 = take(4 * m1);
  L.oJ6 = take(4 * m1);
  L.oJ12 = take(4 * m1);
  L.oN12 = take(4ull * nshard);
  L.oW12 = take(4 * slots);
  L.oN6 = take(4 * slots);
  L.oW6 = take(4 * w6);
  L.oPAN = take(iv == 0 ? m1 : 1);
  L.bytes = off;
  return L;
}
inline size_t serial_ws_bytes(uint32_t nshard) { return 16ull * nshard + 256; }

extern "C" size_t mtblx_plan_workspace_bytes(uint64_t nrec, uint32_t nshard, uint32_t restart_interval, int keep) {
  return plan_layout(nrec, nshard ? nshard : 1u, restart_interval, keep != 0).bytes;
}
extern "C" size_t mtblx_plan_serial_workspace_bytes(uint32_t nshard) { return serial_ws_bytes(nshard ? nshard : 1u); }
// ABI v2 compatibility: the cut used to cache its scratch in the library; it holds none now
extern "C" void mtblx_plan_release(void) {}

static int plan_impl(const mtblx_records* rec, const uint64_t* shard_rec, uint32_t nshard, uint64_t block_size,
                     uint32_t restart_interval, uint64_t* blk_rec, uint64_t blk_cap, uint64_t* nblk_out,
                     uint32_t* flags_out, void* keep, size_t keep_cap, void* workspace, size_t ws_bytes,
                     void* stream) {
  if (!rec || !shard_rec || !nblk_out || nshard == 0) return MTBLX_E_INVAL;
  if (!workspace || (reinterpret_cast<uintptr_t>(workspace) & 255u)) return MTBLX_E_INVAL;
  static const int serial = [] {
    const char* e = getenv("MTBLX_PLAN");
    return e && !strcmp(e, "serial") ? 1 : 0;
  }();
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  std::vector<uint64_t> sh(nshard + 1);
  if (hipMemcpyAsync(sh.data(), shard_rec, 8ull * (nshard + 1), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return MTBLX_E_HIP;
  const uint64_t lo = sh[0], hi = sh[nshard];
  uint64_t kv[4] = {0, 0, 0, 0};   // key END before lo, at hi - 1; value END likewise
  if (hi > lo && hi <= rec->n) {
    bool okc = true;
    if (lo) okc = okc && hipMemcpyAsync(&kv[0], rec->key_end + lo - 1, 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipMemcpyAsync(&kv[2], rec->val_end + lo - 1, 8, hipMemcpyDeviceToHost, s) == hipSuccess;
    okc = okc && hipMemcpyAsync(&kv[1], rec->key_end + hi - 1, 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
          hipMemcpyAsync(&kv[3], rec->val_end + hi - 1, 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
          hipStreamSynchronize(s) == hipSuccess;
    if (!okc) return MTBLX_E_HIP;
  }
  for (uint32_t i = 0; i < nshard; ++i)
    if (sh[i + 1] < sh[i]) return MTBLX_E_INVAL;
  if (hi > rec->n) return MTBLX_E_INVAL;
  const uint64_t m = hi - lo;
  // keep mode: the kept sums are the encode's, and the 32-bit next / waypoint arrays and FastDiv
  // need m < 2^32 - 16 -- no serial fallback here (the caller cuts without keep instead)
  if (keep && (keep_cap < keep_bytes(m) || (reinterpret_cast<uintptr_t>(keep) & 255u) || restart_interval == 0 ||
               m >= 0xFFFFFFF0ull))
    return MTBLX_E_INVAL;
  const uint32_t iv = restart_interval;
  const PlanLayout Ly = plan_layout(m, nshard, iv, keep != nullptr);
  if (keep && ws_bytes < Ly.bytes) return MTBLX_E_INVAL;
  // a workspace too small for the parallel cut (or MTBLX_PLAN=serial, or >= 2^32 - 16 records):
  // the serial walk, whose scratch is 16 B per shard (mtblx_plan_serial_workspace_bytes)
  if (!keep && (serial || m >= 0xFFFFFFF0ull || ws_bytes < Ly.bytes))
    return mtblx_encode_plan_serial(rec, shard_rec, nshard, block_size, restart_interval, blk_rec, blk_cap, nblk_out,
                                    flags_out, workspace, ws_bytes, stream);
  if (block_size < 1024) block_size = 1024;   // WriterBuilder::block_size clamp (src/writer.rs:43-46)
  // slot bases of the next^(2^lvHi) waypoints (a shard of r records has at most ceil(r / top)) and
  // of the next^8 waypoints (at most ceil(r / 8))
  std::vector<uint64_t> sb(nshard + 1), base12(nshard + 1), base6(nshard + 1);
  base12[0] = base6[0] = 0;
  uint64_t maxr = 0;
  for (uint32_t i = 0; i <= nshard; ++i) sb[i] = sh[i] - lo;
  for (uint32_t i = 0; i < nshard; ++i) maxr = std::max<uint64_t>(maxr, sb[i + 1] - sb[i]);
  // the largest shard's blocks, estimated from the mean record size (keys + values + 3 header
  // bytes): JH hops so that its walk takes ~128 of them (more if the estimate is low)
  int lvHi = kLvLo + 1;
  if (m) {
    const double per = (double)(kv[1] - kv[0] + kv[3] - kv[2]) / (double)m + 4.0;
    const double blocks = std::min<double>((double)maxr, (double)maxr * per / (double)block_size + 1.0);
    while (lvHi < 20 && blocks / (double)(1u << lvHi) > 128.0) ++lvHi;
  }
  const uint32_t top = 1u << lvHi, mid = top / kLow;
  for (uint32_t i = 0; i < nshard; ++i) {
    base12[i + 1] = base12[i] + (sb[i + 1] - sb[i] + top - 1) / top;
    base6[i + 1] = base6[i] + (sb[i + 1] - sb[i] + kLow - 1) / kLow;
  }
  const uint64_t slots = base12[nshard], w6 = base6[nshard];
  const uint64_t nchunk = (m + 63) / 64;
  [[maybe_unused]] const uint64_t m1 = std::max<uint64_t>(m, 1);   // the bounds build's range sizes
  uint8_t* ws = static_cast<uint8_t*>(workspace);
  auto p64 = [&](size_t o) { return reinterpret_cast<uint64_t*>(ws + o); };
  auto p32 = [&](size_t o) { return reinterpret_cast<uint32_t*>(ws + o); };
  uint64_t *A = keep ? reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(keep) + 256) : p64(Ly.oA),
           *D = keep ? A + (m + 1) : p64(Ly.oD), *G = p64(Ly.oG), *GM = p64(Ly.oGM), *S = p64(Ly.oS), *dsb = p64(Ly.oSB), *db12 = p64(Ly.oB12),
           *dnb = p64(Ly.oNB), *dbb = p64(Ly.oBB), *mx = p64(Ly.oMX), *db6 = p64(Ly.oB6);
  uint32_t *fl = p32(Ly.oFL), *bnd = p32(Ly.oE), *J0 = p32(Ly.oJ0), *T1 = p32(Ly.oT1), *T2 = p32(Ly.oT2), *J6 = p32(Ly.oJ6),
           *J12 = p32(Ly.oJ12), *n12 = p32(Ly.oN12), *W12 = p32(Ly.oW12), *n6 = p32(Ly.oN6), *W6 = p32(Ly.oW6);
  uint8_t* pan = iv == 0 ? ws + Ly.oPAN : nullptr;
  int rc = MTBLX_OK;
  uint32_t flags = 0;
  uint64_t total = 0;
  std::vector<uint64_t> nb(nshard), bb(nshard);
  auto ok = [&](hipError_t e) { if (e != hipSuccess && rc == MTBLX_OK) rc = MTBLX_E_HIP; return rc == MTBLX_OK; };
  do {
    if (!ok(hipMemcpyAsync(dsb, sb.data(), 8ull * (nshard + 1), hipMemcpyHostToDevice, s))) break;
    if (!ok(hipMemcpyAsync(db12, base12.data(), 8ull * (nshard + 1), hipMemcpyHostToDevice, s))) break;
    if (!ok(hipMemcpyAsync(db6, base6.data(), 8ull * (nshard + 1), hipMemcpyHostToDevice, s))) break;
    if (!ok(hipMemsetAsync(ws + Ly.oFL, 0, 4, s))) break;   // flags
    if (m) {
      uint32_t* SH = keep ? reinterpret_cast<uint32_t*>(D + (m + 1)) : nullptr;
      RecArgs ra{{rec->keys, rec->key_end, rec->vals, rec->val_end}, lo, m, dsb, nshard, A, D, G, GM, fl, SH};
      MTBLX_LAUNCH((MTBLX_R(rec->key_end, 8 * hi), MTBLX_R(rec->val_end, 8 * hi), rec->keys, MTBLX_R(dsb, 8 * (nshard + 1)),
                    MTBLX_R(A, 8 * m), MTBLX_R(D, 8 * m), MTBLX_R(G, 8 * m), MTBLX_R(GM, 8 * nchunk), MTBLX_R(fl, 4),
                    SH ? MTBLX_R(SH, 4 * m) : MTBLX_R(nullptr, 0)),
                   k_plan_rec, dim3((unsigned)std::min<uint64_t>(grid_of(m), 8192)), dim3(kT), 0, s, ra);
      if (!ok(hipMemsetAsync(mx, 0, 8, s))) break;
      MTBLX_LAUNCH((MTBLX_R(GM, 8 * nchunk), MTBLX_R(mx, 8)), k_plan_gmax,
                   dim3((unsigned)std::min<uint64_t>(256, (nchunk + 1023) / 1024)), dim3(1024), 0, s, GM, nchunk, mx);
      const uint64_t nbw = (m + 32) / 32 + 1;
      if (!ok(hipMemsetAsync(bnd, 0, 4 * nbw, s))) break;
      MTBLX_LAUNCH((MTBLX_R(dsb, 8 * (nshard + 1)), MTBLX_R(bnd, 4 * nbw)), k_plan_bounds, dim3(grid_of(nshard)), dim3(kT), 0,
                   s, dsb, nshard, bnd);
      if (!ok(hipGetLastError())) break;
      if ((rc = sscan(A, m, 1, S, s)) != MTBLX_OK) break;
      if (iv && (rc = sscan(D, m, iv, S, s)) != MTBLX_OK) break;
      NextArgs na{m, iv, block_size, A, D, G, GM, mx, dsb, nshard, J0, pan, FastDiv::make(iv ? iv : 1)};
      MTBLX_LAUNCH((MTBLX_R(A, 8 * m), MTBLX_R(D, 8 * m), MTBLX_R(G, 8 * m), MTBLX_R(GM, 8 * nchunk), MTBLX_R(mx, 8),
                    MTBLX_R(dsb, 8 * (nshard + 1)), MTBLX_R(J0, 4 * m), pan ? MTBLX_R(pan, m) : MTBLX_R(nullptr, 0)),
                   k_plan_next, dim3(grid_of(m, (uint64_t)kT * kSweep)), dim3(kT), 0, s, na);
      // next^8 and next^512 by doubling
      const uint32_t* src = J0;
      for (int t = 1; t <= lvHi; ++t) {
        uint32_t* dst = t == kLvLo ? J6 : t == lvHi ? J12 : (t & 1) ? T1 : T2;
        MTBLX_LAUNCH((MTBLX_R(src, 4 * m), MTBLX_R(dst, 4 * m), MTBLX_R(bnd, 4 * ((m + 32) / 32 + 1))), k_plan_jump,
                     dim3(grid_of(m)), dim3(kT), 0, s, src, dst, bnd, m);
        src = dst;
      }
      if (!ok(hipGetLastError())) break;
    }
    WalkArgs wa{dsb, nshard, db12, n12, W12, n6, db6, W6, J0, J6, J12, dnb, nullptr, nullptr, lo, pan, fl, slots, mid, top};
    MTBLX_LAUNCH((MTBLX_R(dsb, 8 * (nshard + 1)), MTBLX_R(db12, 8 * (nshard + 1)), MTBLX_R(n12, 4 * nshard),
                  MTBLX_R(W12, 4 * std::max<uint64_t>(slots, 1)), MTBLX_R(J12, 4 * m1)),
                 k_plan_top, dim3(grid_of(nshard)), dim3(kT), 0, s, wa);
    if (slots) {
      MTBLX_LAUNCH((MTBLX_R(dsb, 8 * (nshard + 1)), MTBLX_R(db12, 8 * (nshard + 1)), MTBLX_R(n12, 4 * nshard),
                    MTBLX_R(W12, 4 * slots), MTBLX_R(n6, 4 * slots), MTBLX_R(db6, 8 * (nshard + 1)), MTBLX_R(W6, 4 * w6), MTBLX_R(J6, 4 * m1)),
                   k_plan_mid, dim3(grid_of(slots)), dim3(kT), 0, s, wa);
    }
    MTBLX_LAUNCH((MTBLX_R(dsb, 8 * (nshard + 1)), MTBLX_R(db12, 8 * (nshard + 1)), MTBLX_R(n12, 4 * nshard),
                  MTBLX_R(n6, 4 * std::max<uint64_t>(slots, 1)), MTBLX_R(db6, 8 * (nshard + 1)), MTBLX_R(W6, 4 * std::max<uint64_t>(w6, 1)),
                  MTBLX_R(J0, 4 * m1), MTBLX_R(dnb, 8 * nshard)),
                 k_plan_count, dim3(grid_of(nshard)), dim3(kT), 0, s, wa);
    if (!ok(hipGetLastError())) break;
    if (!ok(hipMemcpyAsync(nb.data(), dnb, 8ull * nshard, hipMemcpyDeviceToHost, s))) break;
    if (!ok(hipStreamSynchronize(s))) break;
    for (uint32_t i = 0; i < nshard; ++i) {
      bb[i] = total;
      total += nb[i];
    }
    const bool write = blk_rec && total + 1 <= blk_cap;
    if (blk_rec && !write) rc = MTBLX_E_INVAL;   // blk_cap too small: *nblk_out says how many are needed
    if (!ok(hipMemcpyAsync(dbb, bb.data(), 8ull * nshard, hipMemcpyHostToDevice, s))) break;
    wa.bb = dbb;
    wa.blk_rec = write ? blk_rec : nullptr;
    if (slots) {
      MTBLX_LAUNCH((MTBLX_R(db12, 8 * (nshard + 1)), MTBLX_R(dsb, 8 * (nshard + 1)), MTBLX_R(n12, 4 * nshard),
                    MTBLX_R(n6, 4 * slots), MTBLX_R(db6, 8 * (nshard + 1)), MTBLX_R(W6, 4 * w6), MTBLX_R(J0, 4 * m1), MTBLX_R(dbb, 8 * nshard),
                    MTBLX_R(blk_rec, 8 * (write ? total : 0)), pan ? MTBLX_R(pan, m1) : MTBLX_R(nullptr, 0), MTBLX_R(fl, 4)),
                   k_plan_emit, dim3(grid_of(w6)), dim3(kT), 0, s, wa);
    }
    if (!ok(hipGetLastError())) break;
    // blk_rec[total] = the end of the last shard
    if (write && !ok(hipMemcpyAsync(blk_rec + total, shard_rec + nshard, 8, hipMemcpyDeviceToDevice, s))) break;
    if (!ok(hipMemcpyAsync(&flags, fl, 4, hipMemcpyDeviceToHost, s))) break;
    ok(hipStreamSynchronize(s));
  } while (false);
  if (rc == MTBLX_OK && keep) {
    const KeepHdr h{kKeepMagic, lo, m, restart_interval};
    if (hipMemcpyAsync(keep, &h, sizeof(h), hipMemcpyHostToDevice, s) != hipSuccess) rc = MTBLX_E_HIP;
  }
  if (hipStreamSynchronize(s) != hipSuccess && rc == MTBLX_OK) rc = MTBLX_E_HIP;
  *nblk_out = total;
  if (flags_out) *flags_out = flags;
  if (rc == MTBLX_OK && (flags & (MTBLX_PLAN_OUT_OF_ORDER | MTBLX_PLAN_PANIC | MTBLX_PLAN_TOO_LONG))) rc = MTBLX_E_FORMAT;
  return rc;
}

extern "C" int mtblx_encode_plan(const mtblx_records* rec, const uint64_t* shard_rec, uint32_t nshard,
                                 uint64_t block_size, uint32_t restart_interval, uint64_t* blk_rec, uint64_t blk_cap,
                                 uint64_t* nblk_out, uint32_t* flags_out, void* workspace, size_t ws_bytes,
                                 void* stream) {
  return plan_impl(rec, shard_rec, nshard, block_size, restart_interval, blk_rec, blk_cap, nblk_out, flags_out, nullptr,
                   0, workspace, ws_bytes, stream);
}

extern "C" size_t mtblx_plan_keep_bytes(uint64_t nrec) { return keep_bytes(nrec); }

extern "C" int mtblx_encode_plan_keep(const mtblx_records* rec, const uint64_t* shard_rec, uint32_t nshard,
                                      uint64_t block_size, uint32_t restart_interval, uint64_t* blk_rec, uint64_t blk_cap,
                                      uint64_t* nblk_out, uint32_t* flags_out, void* plan, size_t plan_bytes,
                                      void* workspace, size_t ws_bytes, void* stream) {
  if (!plan) return MTBLX_E_INVAL;
  return plan_impl(rec, shard_rec, nshard, block_size, restart_interval, blk_rec, blk_cap, nblk_out, flags_out, plan,
                   plan_bytes, workspace, ws_bytes, stream);
}
