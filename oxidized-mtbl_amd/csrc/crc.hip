// crc.hip — MI355X (gfx950) CRC-32C of block contents: the checksum Reader::block verifies
// before it decodes a block (/root/reference/src/reader.rs:159-164, crate crc32c 0.4:
// CRC-32C Castagnoli, reflected polynomial 0x82F63B78, init/xorout 0xFFFFFFFF).
//
// One wave per block: 72-byte windows counted from the block's END, one per lane; each window's
// raw CRC (slicing-by-8) is shifted into place with a GF(2) multiply by x^(576 k) mod P:
//   crc_raw(A || B) = multmodp(x^(8|B|), crc_raw(A)) ^ crc_raw(B)
// through nibble tables of the constants x^(576 k) (crc_dev.h MulTabs: 8 lookups instead of a
// 32-step bitwise multiply, which was ~190 of ~510 vector instructions per 4 KiB block)
// and the wave XOR-reduces; see k_crc32c_blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "crc_dev.h"
#include "mtblx.h"

namespace mtblx_crc {

constexpr int kCrcThreads = 1024;   // 16 waves per workgroup, 2 workgroups per CU (LDS: 48 KiB each)

// Slicing-by-8 tables: T8[k][i] = CRC of byte i followed by k zero bytes.
struct Slice8 {
  uint32_t t[8][256];
};

// raw CRC (init 0) of the kCrcWin-byte window ending at block position hi: bytes before the
// block start (positions < 0) count as zeros, which leave a zero-init CRC unchanged; the
// 0xFFFFFFFF init is folded into block bytes 0..3.  18 words -> 9 slicing-by-8 steps.
constexpr int kWords = kCrcWin / 4;
// block bytes are read once: non-temporal loads (MTBLX_CRC_NT_LOADS) keep them out of the L2s
#ifndef MTBLX_CRC_NT_LOADS
#define MTBLX_CRC_NT_LOADS 0
#endif
typedef uint32_t v2u __attribute__((ext_vector_type(2), aligned(1)));
__device__ __forceinline__ v4u crc_ld16(const uint8_t* p) {
#if MTBLX_CRC_NT_LOADS
  return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
#else
  return *reinterpret_cast<const v4u*>(p);
#endif
}
__device__ __forceinline__ v2u crc_ld8(const uint8_t* p) {
#if MTBLX_CRC_NT_LOADS
  return __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
#else
  return *reinterpret_cast<const v2u*>(p);
#endif
}
__device__ __forceinline__ uint32_t window_crc(const uint8_t* d, int64_t hi, const uint32_t (*T)[256], bool safe) {
  const int64_t lo = hi - kCrcWin;
  uint32_t w[kWords];
  if (safe) {   // d + lo is readable (inside the buffer) even where lo < 0
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const v4u x = crc_ld16(d + lo + 16 * q);
      w[4 * q] = x.x; w[4 * q + 1] = x.y; w[4 * q + 2] = x.z; w[4 * q + 3] = x.w;
    }
    const v2u y = crc_ld8(d + lo + 64);
    w[16] = y.x; w[17] = y.y;
  } else {      // the window starts before the buffer: byte loads of the in-block part only
#pragma unroll
    for (int m = 0; m < kWords; ++m) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int64_t p = lo + 4 * m + b;
        v |= (p >= 0 ? (uint32_t)d[p] : 0u) << (8 * b);
      }
      w[m] = v;
    }
  }
  if (lo < 4) {
#pragma unroll
    for (int m = 0; m < kWords; ++m) {
      const int64_t pos = lo + 4 * m;   // block position of the word's first byte
      if (pos < 4) {
        const uint32_t keep = pos <= -4 ? 0u : (pos < 0 ? 0xFFFFFFFFu << (8 * (uint32_t)(-pos)) : 0xFFFFFFFFu);
        const uint32_t fold = pos < 0 ? keep : 0xFFFFFFFFu >> (8 * (uint32_t)pos);
        w[m] = (w[m] & keep) ^ fold;
      }
    }
  }
  uint32_t c = 0;
#pragma unroll
  for (int m = 0; m < kWords; m += 2) {
    const uint32_t x = c ^ w[m], y = w[m + 1];
    c = T[7][x & 0xFFu] ^ T[6][(x >> 8) & 0xFFu] ^ T[5][(x >> 16) & 0xFFu] ^ T[4][x >> 24] ^
        T[3][y & 0xFFu] ^ T[2][(y >> 8) & 0xFFu] ^ T[1][(y >> 16) & 0xFFu] ^ T[0][y >> 24];
  }
  return c;
}

// One wave per block: lane j takes the kCrcWin-byte windows j, j + 64, ... counted from the
// block's END (window k = block bytes [L - W (k + 1), L - W k)), each a raw CRC shifted into
// place by x^(8 W k) (nibble tables in LDS), XOR-reduced over the wave.
__global__ void __launch_bounds__(kCrcThreads) k_crc32c_blocks(const uint8_t* data, uint64_t data_len,
                                                               const uint64_t* blk_off, const uint32_t* blk_len,
                                                               uint32_t nblk, uint32_t* crc_out, uint8_t* bad,
                                                               int framed) {
  __shared__ Slice8 S;
  __shared__ MulLds M;   // window shifts x^(576 k) as nibble tables
  for (int i = threadIdx.x; i < 4 * 256; i += kCrcThreads) S.t[i >> 8][i & 255] = kTab.slice[i >> 8][i & 255];
  {
    const uint4* src = reinterpret_cast<const uint4*>(&kMul);
    uint4* dst = reinterpret_cast<uint4*>(&M);
    for (int i = threadIdx.x; i < (int)(sizeof(MulLds) / 16); i += kCrcThreads) dst[i] = src[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 4 * 256; i += kCrcThreads) {   // tables 4..7 from table 3
    uint32_t t = S.t[3][i & 255];
    for (int k = 0; k <= (i >> 8); ++k) t = (t >> 8) ^ S.t[0][t & 0xFFu];
    S.t[4 + (i >> 8)][i & 255] = t;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (kCrcThreads / kWave);
  for (uint32_t b = blockIdx.x * (kCrcThreads / kWave) + (threadIdx.x >> 6); b < nblk; b += waves) {
    const uint64_t off = blk_off[b];
    const uint64_t L = blk_len[b];
    const uint8_t* d = data + off;
    // a window past the buffer: the reference's slice panics before the checksum (bad = 1)
    const bool oob = off + L > data_len;
    uint32_t acc = 0;
    if (!oob && L >= (uint64_t)kCrcWin) {
      for (uint64_t k = lane; k * kCrcWin < L; k += kWave) {
        const int64_t hi = (int64_t)(L - k * kCrcWin);
        const bool safe = (int64_t)off + hi - kCrcWin >= 0;
        const uint32_t c = window_crc(d, hi, S.t, safe);
        if (k < 64) acc ^= mul_nib(c, M.a[k]);
        else if (k < 1024) acc ^= mul_nib(mul_nib(c, M.a[k & 63]), M.b[k >> 6]);
        else acc ^= dmultmodp(xpow8(k * kCrcWin), c);
      }
#pragma unroll
      for (int sh = 32; sh >= 1; sh >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, sh, kWave);
      acc ^= 0xFFFFFFFFu;
    } else if (!oob) {
      acc = wave_crc32c(d, L, S.t[0], lane);   // < kCrcWin bytes (wave_crc32c: byte-wise under 64)
    }
    if (lane == 0) {
      if (crc_out) crc_out[b] = acc;
      if (bad && oob) {
        bad[b] = 1;
      } else if (bad) {
        uint32_t stored = 0;
        if (framed && off >= 4)
          stored = (uint32_t)d[-4] | ((uint32_t)d[-3] << 8) | ((uint32_t)d[-2] << 16) | ((uint32_t)d[-1] << 24);
        bad[b] = (framed && off >= 4) ? (uint8_t)(stored != acc) : (uint8_t)0;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Round 3: the block's first window (k = lane) is loaded one block AHEAD (the loads of block
// b + waves are in flight while block b is computed), and S72 computes a window's raw CRC
// without a serial chain: byte i of the 72-byte window is followed by 71 - i bytes, so
//   crc_raw(window) = XOR_i T72[71 - i][byte_i],   T72[d][x] = crc_raw(x followed by d zeros)
// -- 72 independent lookups instead of 9 dependent slicing-by-8 steps.  T72 (72 KiB) and the
// shift tables (40 KiB) fill 112 KiB of LDS: one 1024-thread workgroup per CU, as the VGPRs
// allowed before.
struct Slice72 {
  uint32_t t[kCrcWin][256];
  constexpr Slice72() : t() {
    for (uint32_t x = 0; x < 256; ++x) {
      uint32_t c = x;
      for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : c >> 1;
      t[0][x] = c;
    }
    for (int d = 1; d < kCrcWin; ++d)
      for (uint32_t x = 0; x < 256; ++x) t[d][x] = (t[d - 1][x] >> 8) ^ t[0][t[d - 1][x] & 0xFFu];
  }
};
static __constant__ Slice72 kS72 = Slice72();
struct Slice72Lds {
  uint32_t t[kCrcWin][256];
};

// the 18 words of the window [hi - kCrcWin, hi) of block d (bytes before the block as zeros,
// the 0xFFFFFFFF init folded into bytes 0..3)
__device__ __forceinline__ void window_words(const uint8_t* d, int64_t hi, bool safe, uint32_t (&w)[kWords]) {
  const int64_t lo = hi - kCrcWin;
  if (safe) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const v4u x = crc_ld16(d + lo + 16 * q);
      w[4 * q] = x.x; w[4 * q + 1] = x.y; w[4 * q + 2] = x.z; w[4 * q + 3] = x.w;
    }
    const v2u y = crc_ld8(d + lo + 64);
    w[16] = y.x; w[17] = y.y;
  } else {
#pragma unroll
    for (int m = 0; m < kWords; ++m) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int64_t p = lo + 4 * m + b;
        v |= (p >= 0 ? (uint32_t)d[p] : 0u) << (8 * b);
      }
      w[m] = v;
    }
  }
}

__device__ __forceinline__ void window_fold(int64_t lo, uint32_t (&w)[kWords]) {
  if (lo < 4) {
#pragma unroll
    for (int m = 0; m < kWords; ++m) {
      const int64_t pos = lo + 4 * m;
      if (pos < 4) {
        const uint32_t keep = pos <= -4 ? 0u : (pos < 0 ? 0xFFFFFFFFu << (8 * (uint32_t)(-pos)) : 0xFFFFFFFFu);
        const uint32_t fold = pos < 0 ? keep : 0xFFFFFFFFu >> (8 * (uint32_t)pos);
        w[m] = (w[m] & keep) ^ fold;
      }
    }
  }
}

template <bool S72>
__device__ __forceinline__ uint32_t window_raw(const uint32_t (&w)[kWords], const uint32_t (*T)[256]) {
  uint32_t c = 0;
  if constexpr (S72) {
#pragma unroll
    for (int m = 0; m < kWords; ++m) {
      const uint32_t x = w[m];
      const int d = kCrcWin - 1 - 4 * m;
      c ^= T[d][x & 0xFFu] ^ T[d - 1][(x >> 8) & 0xFFu] ^ T[d - 2][(x >> 16) & 0xFFu] ^ T[d - 3][x >> 24];
    }
  } else {
#pragma unroll
    for (int m = 0; m < kWords; m += 2) {
      const uint32_t x = c ^ w[m], y = w[m + 1];
      c = T[7][x & 0xFFu] ^ T[6][(x >> 8) & 0xFFu] ^ T[5][(x >> 16) & 0xFFu] ^ T[4][x >> 24] ^
          T[3][y & 0xFFu] ^ T[2][(y >> 8) & 0xFFu] ^ T[1][(y >> 16) & 0xFFu] ^ T[0][y >> 24];
    }
  }
  return c;
}

template <bool S72>
struct CrcLds {
  uint32_t t[S72 ? kCrcWin : 8][256];
  MulLds m;
};

template <bool S72>
__global__ void __launch_bounds__(kCrcThreads) k_crc32c_blocks_pf(const uint8_t* data, uint64_t data_len,
                                                                  const uint64_t* blk_off, const uint32_t* blk_len,
                                                                  uint32_t nblk, uint32_t* crc_out, uint8_t* bad,
                                                                  int framed) {
  __shared__ CrcLds<S72> S;
  {
    const uint4* src = S72 ? reinterpret_cast<const uint4*>(&kS72) : reinterpret_cast<const uint4*>(&kTab.slice[0][0]);
    uint4* dst = reinterpret_cast<uint4*>(&S.t[0][0]);
    const int n16 = S72 ? (int)(sizeof(Slice72Lds) / 16) : 4 * 256 / 4;
    for (int i = threadIdx.x; i < n16; i += kCrcThreads) dst[i] = src[i];
    const uint4* ms = reinterpret_cast<const uint4*>(&kMul);
    uint4* md = reinterpret_cast<uint4*>(&S.m);
    for (int i = threadIdx.x; i < (int)(sizeof(MulLds) / 16); i += kCrcThreads) md[i] = ms[i];
  }
  if constexpr (!S72) {
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * 256; i += kCrcThreads) {   // tables 4..7 from table 3
      uint32_t t = S.t[3][i & 255];
      for (int k = 0; k <= (i >> 8); ++k) t = (t >> 8) ^ S.t[0][t & 0xFFu];
      S.t[4 + (i >> 8)][i & 255] = t;
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t waves = gridDim.x * (kCrcThreads / kWave);
  uint32_t b = blockIdx.x * (kCrcThreads / kWave) + (threadIdx.x >> 6);
  // the first window (k = lane) of block b, loaded one block ahead
  uint32_t w[kWords];
  auto issue = [&](uint32_t bb) {
    if (bb >= nblk) return;
    const uint64_t off = blk_off[bb], L = blk_len[bb];
    if (off + L > data_len || L < (uint64_t)kCrcWin || (uint64_t)lane * kCrcWin >= L) return;
    const int64_t hi = (int64_t)(L - (uint64_t)lane * kCrcWin);
    window_words(data + off, hi, (int64_t)off + hi - kCrcWin >= 0, w);
  };
  issue(b);
  for (; b < nblk; b += waves) {
    const uint64_t off = blk_off[b];
    const uint64_t L = blk_len[b];
    const uint8_t* d = data + off;
    const bool oob = off + L > data_len;   // the reference's slice panics before the checksum
    uint32_t cw[kWords];
#pragma unroll
    for (int m = 0; m < kWords; ++m) cw[m] = w[m];
    issue(b + waves);
    uint32_t acc = 0;
    if (!oob && L >= (uint64_t)kCrcWin) {
      if ((uint64_t)lane * kCrcWin < L) {
        const int64_t hi = (int64_t)(L - (uint64_t)lane * kCrcWin);
        window_fold(hi - kCrcWin, cw);
        acc = mul_nib(window_raw<S72>(cw, S.t), S.m.a[lane]);
      }
      for (uint64_t k = lane + kWave; k * kCrcWin < L; k += kWave) {   // blocks > 4.5 KiB
        const int64_t hi = (int64_t)(L - k * kCrcWin);
        uint32_t xw[kWords];
        window_words(d, hi, (int64_t)off + hi - kCrcWin >= 0, xw);
        window_fold(hi - kCrcWin, xw);
        const uint32_t c = window_raw<S72>(xw, S.t);
        if (k < 1024) acc ^= mul_nib(mul_nib(c, S.m.a[k & 63]), S.m.b[k >> 6]);
        else acc ^= dmultmodp(xpow8(k * kCrcWin), c);
      }
#pragma unroll
      for (int sh = 32; sh >= 1; sh >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, sh, kWave);
      acc ^= 0xFFFFFFFFu;
    } else if (!oob) {
      acc = wave_crc32c(d, L, S.t[0], lane);   // < kCrcWin bytes
    }
    if (lane == 0) {
      if (crc_out) crc_out[b] = acc;
      if (bad && oob) {
        bad[b] = 1;
      } else if (bad) {
        uint32_t stored = 0;
        if (framed && off >= 4)
          stored = (uint32_t)d[-4] | ((uint32_t)d[-3] << 8) | ((uint32_t)d[-2] << 16) | ((uint32_t)d[-1] << 24);
        bad[b] = (framed && off >= 4) ? (uint8_t)(stored != acc) : (uint8_t)0;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Round 3: lane-private slicing-by-4 tables.  ds_read_b32 is serviced in two groups of 32 lanes
// over 32 banks (MI355X_MICROARCH.md, LDS): a random byte index into a shared 1 KiB table puts
// ~3.5 distinct addresses on the busiest bank of a group, so every lookup of the kernels above
// costs ~7 LDS cycles instead of 2, and at one lookup per input byte that bounds them near
// 0.1 ms on cfg2.  Here table j holds 32 copies, entry v of copy c at word (j 256 + v) 32 + c,
// and lane l reads copy l mod 32: one bank per lane of a group, conflict-free.  4 tables x
// 256 x 32 x 4 B = 128 KiB: one 1024-thread workgroup per CU, persistent (one table build per
// CU).  Windows as k_crc32c_blocks (72 B from the block end, lane = window), loaded one block
// ahead together with the stored checksum; window shifts x^(576 k) by GF(2) multiplies with
// per-lane constants (x^(576 lane) in a register, x^(576 64 r) from a small LDS table).
constexpr int kLpThreads = 1024;
constexpr int kLpRounds = 64;   // window rounds with an LDS shift constant (blocks up to 288 KiB)
struct LpLds {
  uint32_t t[4][256][32];
  uint32_t x[kLpRounds];
};

__device__ __forceinline__ uint32_t lp_word4(const uint32_t* T, uint32_t c, uint32_t w) {
  c ^= w;   // T = &S.t[0][0][lane & 31]; entry (j, v) at T[(j * 256 + v) * 32]
  return T[(3 * 256 + (c & 0xffu)) * 32] ^ T[(2 * 256 + ((c >> 8) & 0xffu)) * 32] ^
         T[(1 * 256 + ((c >> 16) & 0xffu)) * 32] ^ T[(c >> 24) * 32];
}

__global__ void __launch_bounds__(kLpThreads, 1) k_crc32c_lp(const uint8_t* data, uint64_t data_len,
                                                             const uint64_t* blk_off, const uint32_t* blk_len,
                                                             uint32_t nblk, uint32_t* crc_out, uint8_t* bad,
                                                             int framed) {
  __shared__ LpLds S;
  for (int i = threadIdx.x; i < 4 * 256 * 32; i += kLpThreads) S.t[i >> 13][(i >> 5) & 255][i & 31] = kTab.slice[i >> 13][(i >> 5) & 255];
  if (threadIdx.x < kLpRounds) S.x[threadIdx.x] = xpow8((uint64_t)kCrcWin * kWave * threadIdx.x);
  const int lane = threadIdx.x & 63;
  const uint32_t K = xpow8((uint64_t)kCrcWin * (uint32_t)lane);   // x^(576 lane)
  __syncthreads();
  const uint32_t* T = &S.t[0][0][lane & 31];
  const uint32_t waves = gridDim.x * (kLpThreads / kWave);
  uint32_t b = blockIdx.x * (kLpThreads / kWave) + (threadIdx.x >> 6);
  // block bb's first window (k = lane) and (lane 0) its stored checksum, loaded one block ahead
  uint32_t w[kWords];
  uint32_t nstored = 0;
  auto issue = [&](uint32_t bb) {
    if (bb >= nblk) return;
    const uint64_t off = blk_off[bb], L = blk_len[bb];
    if (off + L > data_len) return;
    if (lane == 0 && framed && off >= 4) {
      const uint8_t* d = data + off;
      nstored = (uint32_t)d[-4] | ((uint32_t)d[-3] << 8) | ((uint32_t)d[-2] << 16) | ((uint32_t)d[-1] << 24);
    }
    if (L < (uint64_t)kCrcWin || (uint64_t)lane * kCrcWin >= L) return;
    const int64_t hi = (int64_t)(L - (uint64_t)lane * kCrcWin);
    window_words(data + off, hi, (int64_t)off + hi - kCrcWin >= 0, w);
  };
  issue(b);
  for (; b < nblk; b += waves) {
    const uint64_t off = blk_off[b];
    const uint64_t L = blk_len[b];
    const uint8_t* d = data + off;
    const bool oob = off + L > data_len;   // the reference's slice panics before the checksum
    uint32_t cw[kWords];
#pragma unroll
    for (int m = 0; m < kWords; ++m) cw[m] = w[m];
    const uint32_t stored = nstored;
    issue(b + waves);
    uint32_t acc = 0;
    if (!oob && L >= (uint64_t)kCrcWin) {
      if ((uint64_t)lane * kCrcWin < L) {
        const int64_t hi = (int64_t)(L - (uint64_t)lane * kCrcWin);
        window_fold(hi - kCrcWin, cw);
        uint32_t c = 0;
#pragma unroll
        for (int m = 0; m < kWords; ++m) c = lp_word4(T, c, cw[m]);
        acc = c;
      }
      for (uint64_t r = 1; (uint64_t)lane * kCrcWin + r * kWave * kCrcWin < L; ++r) {   // blocks > 4.5 KiB
        const uint64_t k = (uint64_t)lane + r * kWave;
        const int64_t hi = (int64_t)(L - k * kCrcWin);
        uint32_t xw[kWords];
        window_words(d, hi, (int64_t)off + hi - kCrcWin >= 0, xw);
        window_fold(hi - kCrcWin, xw);
        uint32_t c = 0;
#pragma unroll
        for (int m = 0; m < kWords; ++m) c = lp_word4(T, c, xw[m]);
        acc ^= dmultmodp(r < (uint64_t)kLpRounds ? S.x[r] : xpow8(r * kWave * kCrcWin), c);
      }
      acc = dmultmodp(K, acc);
#pragma unroll
      for (int sh = 32; sh >= 1; sh >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, sh, kWave);
      acc ^= 0xFFFFFFFFu;
    } else if (!oob) {
      acc = wave_crc32c(d, L, kTab.byte, lane);   // < kCrcWin bytes (byte table from L1/L2)
    }
    if (lane == 0) {
      if (crc_out) crc_out[b] = acc;
      if (bad) bad[b] = oob ? (uint8_t)1 : (framed && off >= 4) ? (uint8_t)(stored != acc) : (uint8_t)0;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Round 3, kernel 5: lane-private tables for the window shifts too.  Kernel 3 (lane-private
// slicing tables, window shift by a 32-step GF(2) multiply) lost the LDS bank conflicts
// (SQ_LDS_BANK_CONFLICT 33 M -> 0) but doubled the vector instructions (33 M -> 69 M).  Here
// the shift x^(576 lane) of each lane's first-round window is a nibble-table multiply whose 128
// words live lane-interleaved (entry e of lane l at word e 64 + l: one bank per lane of a
// 32-lane group), filling the 32 KiB the slicing tables leave: 160 KiB in all.
struct Lp5Lds {
  uint32_t t[4][256][32];
  uint32_t m[8 * 16][64];
};

__global__ void __launch_bounds__(kLpThreads, 1) k_crc32c_lp5(const uint8_t* data, uint64_t data_len,
                                                              const uint64_t* blk_off, const uint32_t* blk_len,
                                                              uint32_t nblk, uint32_t* crc_out, uint8_t* bad,
                                                              int framed) {
  __shared__ Lp5Lds S;
  for (int i = threadIdx.x; i < 4 * 256 * 32; i += kLpThreads) S.t[i >> 13][(i >> 5) & 255][i & 31] = kTab.slice[i >> 13][(i >> 5) & 255];
  for (int i = threadIdx.x; i < 8 * 16 * 64; i += kLpThreads) S.m[i >> 6][i & 63] = kMul.a[i & 63][(i >> 10) & 7][(i >> 6) & 15];
  const int lane = threadIdx.x & 63;
  __syncthreads();
  const uint32_t* T = &S.t[0][0][lane & 31];
  const uint32_t* Mm = &S.m[0][lane];
  const uint32_t waves = gridDim.x * (kLpThreads / kWave);
  uint32_t b = blockIdx.x * (kLpThreads / kWave) + (threadIdx.x >> 6);
  uint32_t w[kWords];
  uint32_t nstored = 0;
  auto issue = [&](uint32_t bb) {
    if (bb >= nblk) return;
    const uint64_t off = blk_off[bb], L = blk_len[bb];
    if (off + L > data_len) return;
    if (lane == 0 && framed && off >= 4) {
      const uint8_t* d = data + off;
      nstored = (uint32_t)d[-4] | ((uint32_t)d[-3] << 8) | ((uint32_t)d[-2] << 16) | ((uint32_t)d[-1] << 24);
    }
    if (L < (uint64_t)kCrcWin || (uint64_t)lane * kCrcWin >= L) return;
    const int64_t hi = (int64_t)(L - (uint64_t)lane * kCrcWin);
    window_words(data + off, hi, (int64_t)off + hi - kCrcWin >= 0, w);
  };
  issue(b);
  for (; b < nblk; b += waves) {
    const uint64_t off = blk_off[b];
    const uint64_t L = blk_len[b];
    const uint8_t* d = data + off;
    const bool oob = off + L > data_len;
    uint32_t cw[kWords];
#pragma unroll
    for (int m = 0; m < kWords; ++m) cw[m] = w[m];
    const uint32_t stored = nstored;
    issue(b + waves);
    uint32_t acc = 0;
    if (!oob && L >= (uint64_t)kCrcWin) {
      uint32_t c = 0;
      if ((uint64_t)lane * kCrcWin < L) {
        const int64_t hi = (int64_t)(L - (uint64_t)lane * kCrcWin);
        window_fold(hi - kCrcWin, cw);
#pragma unroll
        for (int m = 0; m < kWords; ++m) c = lp_word4(T, c, cw[m]);
      }
      for (uint64_t r = 1; (uint64_t)lane * kCrcWin + r * kWave * kCrcWin < L; ++r) {   // blocks > 4.5 KiB
        const uint64_t k = (uint64_t)lane + r * kWave;
        const int64_t hi = (int64_t)(L - k * kCrcWin);
        uint32_t xw[kWords];
        window_words(d, hi, (int64_t)off + hi - kCrcWin >= 0, xw);
        window_fold(hi - kCrcWin, xw);
        uint32_t x = 0;
#pragma unroll
        for (int m = 0; m < kWords; ++m) x = lp_word4(T, x, xw[m]);
        c ^= r < 16 ? mul_nib(x, kMul.b[r]) : dmultmodp(xpow8(r * kWave * kCrcWin), x);
      }
      // c * x^(576 lane): the lane's nibble tables
#pragma unroll
      for (int j = 0; j < 8; ++j) acc ^= Mm[(j * 16 + ((c >> (4 * j)) & 15u)) * 64];
#pragma unroll
      for (int sh = 32; sh >= 1; sh >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, sh, kWave);
      acc ^= 0xFFFFFFFFu;
    } else if (!oob) {
      acc = wave_crc32c(d, L, kTab.byte, lane);
    }
    if (lane == 0) {
      if (crc_out) crc_out[b] = acc;
      if (bad) bad[b] = oob ? (uint8_t)1 : (framed && off >= 4) ? (uint8_t)(stored != acc) : (uint8_t)0;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Round 3, kernel 6: coalesced rows.  The counters of the window kernels (profiles/r03/crcprof)
// put the texture data path at 80 % busy (TD_TD_BUSY) with one cache access per lane per load
// (TCP_TOTAL_CACHE_ACCESSES ~ 64 per load instruction): lanes 72 bytes apart make every 16-byte
// load a scatter.  Here a wave reads its block in rows of 1 KiB counted from the block's END
// (row r = bytes [L - 1024 (r + 1), L - 1024 r)), lane l the 16 bytes at 16 l of the row: each
// load instruction covers 1 KiB contiguous.  A lane's raw CRC of its 16 bytes (4 slicing-by-4
// steps, lane-private tables) is shifted by x^(128 (63 - l)) (lane-private nibble tables), the
// wave XOR-reduces the row (DPP) and the rows are joined with Horner's rule on the scalar unit:
// S = S * x^8192 + R_r from the top row down.  Bytes before the block start are zero, the
// 0xFFFFFFFF init is folded into bytes 0..3 (as the window kernels).  160 KiB of LDS: one
// persistent 1024-thread workgroup per CU.
constexpr uint32_t kRowB = 1024;
constexpr int kRowGroup = 4;   // rows loaded together per lane (16 B each)

__device__ __forceinline__ uint32_t dpp_xor_reduce(uint32_t x) {   // -> the wave's XOR (uniform)
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);   // row_half_mirror
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);   // row_mirror
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)x, 16) ^
         (uint32_t)__builtin_amdgcn_readlane((int)x, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
}

// GF(2) multiply of uniform values (scalar unit)
__device__ __forceinline__ uint32_t smultmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & (0x80000000u >> i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

__global__ void __launch_bounds__(kLpThreads, 1) k_crc32c_rows(const uint8_t* data, uint64_t data_len,
                                                               const uint64_t* blk_off, const uint32_t* blk_len,
                                                               uint32_t nblk, uint32_t* crc_out, uint8_t* bad,
                                                               int framed) {
  __shared__ Lp5Lds S;
  for (int i = threadIdx.x; i < 4 * 256 * 32; i += kLpThreads) S.t[i >> 13][(i >> 5) & 255][i & 31] = kTab.slice[i >> 13][(i >> 5) & 255];
  {
    // lane l's nibble tables of K_l = x^(128 (63 - l)): entry (j, v) = K_l * (v << 4 j)
    const int l = threadIdx.x & 63;
    const uint32_t Kl = xpow8(16u * (63u - (uint32_t)l));
    for (int e = threadIdx.x >> 6; e < 128; e += kLpThreads / kWave)
      S.m[e][l] = dmultmodp(Kl, (uint32_t)(e & 15) << (4 * (e >> 4)));
  }
  const uint32_t X = (uint32_t)__builtin_amdgcn_readfirstlane((int)xpow8(kRowB));   // x^8192
  const int lane = threadIdx.x & 63;
  __syncthreads();
  const uint32_t* T = &S.t[0][0][lane & 31];
  const uint32_t* Mm = &S.m[0][lane];
  const uint32_t waves = gridDim.x * (kLpThreads / kWave);
  for (uint32_t b = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (kLpThreads / kWave) + (threadIdx.x >> 6)));
       b < nblk; b += waves) {
    const uint64_t off = blk_off[b];
    const uint64_t L = blk_len[b];
    const uint8_t* d = data + off;
    const bool oob = off + L > data_len;   // the reference's slice panics before the checksum
    uint32_t crc = 0;
    if (!oob && L >= 4) {
      const int64_t nrow = (int64_t)((L + kRowB - 1) / kRowB);
      uint32_t Sx = 0;
      for (int64_t r0 = nrow - 1; r0 >= 0; r0 -= kRowGroup) {
        v4u q[kRowGroup];
#pragma unroll
        for (int g = 0; g < kRowGroup; ++g) {   // rows r0, r0 - 1, ...: loads first
          const int64_t r = r0 - g;
          const int64_t pos = (int64_t)L - (int64_t)kRowB * (r + 1) + 16 * lane;   // block position of the quad
          q[g] = v4u{0u, 0u, 0u, 0u};
          if (r >= 0 && pos > -16) {
            if ((int64_t)off + pos >= 0) {
              q[g] = crc_ld16(d + pos);
            } else {   // the block starts at the buffer start: its in-block bytes only
              uint32_t wv[4] = {0u, 0u, 0u, 0u};
              for (int i = 0; i < 16; ++i)
                if (pos + i >= 0) wv[i >> 2] |= (uint32_t)d[pos + i] << (8 * (i & 3));
              q[g] = v4u{wv[0], wv[1], wv[2], wv[3]};
            }
          }
        }
#pragma unroll
        for (int g = 0; g < kRowGroup; ++g) {
          const int64_t r = r0 - g;
          if (r < 0) break;
          const int64_t pos = (int64_t)L - (int64_t)kRowB * (r + 1) + 16 * lane;
          uint32_t w[4] = {q[g].x, q[g].y, q[g].z, q[g].w};
          if (pos < 4) {   // bytes before the block: zero; the init into bytes 0..3
#pragma unroll
            for (int m = 0; m < 4; ++m) {
              const int64_t pm = pos + 4 * m;
              if (pm < 4) {
                const uint32_t keep = pm <= -4 ? 0u : (pm < 0 ? 0xFFFFFFFFu << (8 * (uint32_t)(-pm)) : 0xFFFFFFFFu);
                const uint32_t fold = pm < 0 ? keep : 0xFFFFFFFFu >> (8 * (uint32_t)pm);
                w[m] = (w[m] & keep) ^ fold;
              }
            }
          }
          uint32_t c = 0;
#pragma unroll
          for (int m = 0; m < 4; ++m) c = lp_word4(T, c, w[m]);
          uint32_t v = 0;   // c * x^(128 (63 - lane))
#pragma unroll
          for (int j = 0; j < 8; ++j) v ^= Mm[(j * 16 + ((c >> (4 * j)) & 15u)) * 64];
          const uint32_t Rr = dpp_xor_reduce(v);
          Sx = smultmodp(Sx, X) ^ Rr;
        }
      }
      crc = Sx ^ 0xFFFFFFFFu;
    } else if (!oob) {
      crc = wave_crc32c(d, L, kTab.byte, lane);   // < 4 bytes
    }
    if (lane == 0) {
      if (crc_out) crc_out[b] = crc;
      if (bad) {
        uint8_t x = 0;
        if (oob) {
          x = 1;
        } else if (framed && off >= 4) {
          const uint32_t stored = (uint32_t)d[-4] | ((uint32_t)d[-3] << 8) | ((uint32_t)d[-2] << 16) | ((uint32_t)d[-1] << 24);
          x = stored != crc;
        }
        bad[b] = x;
      }
    }
  }
}

}  // namespace mtblx_crc

// MTBLX_CRC_KERNEL (A/B knob, read once): 0 = the round-2 kernel, 1 = prefetch + slicing-by-8,
// 2 = prefetch + slicing-by-72 (measured 0.125 / 0.135 / 0.137 ms on cfg2: the round-2 kernel stays)
static int crc_kernel_choice() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("MTBLX_CRC_KERNEL");
    v = e ? atoi(e) : 0;
  }
  return v;
}

extern "C" int mtblx_crc32c_blocks(const mtblx_block_batch* in, uint32_t* crc, uint8_t* bad, int framed,
                                   void* stream) {
  if (!in || (!crc && !bad && in->nblk)) return MTBLX_E_INVAL;
  if (in->nblk == 0) return MTBLX_OK;
  if (!in->data || !in->blk_off || !in->blk_len) return MTBLX_E_INVAL;
  static int grid = 0;
  if (!grid) {
    int dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    grid = (ncu > 0 ? ncu : 256) * 2;   // 32 waves per CU
  }
  const uint32_t need = (in->nblk + 15u) / 16u;
  const int kc = crc_kernel_choice();
  const dim3 g(need < (uint32_t)grid ? need : (uint32_t)grid), t(mtblx_crc::kCrcThreads);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (kc == 6) {   // one workgroup per CU (160 KiB of LDS), persistent
    const uint32_t g1 = need < (uint32_t)(grid / 2) ? need : (uint32_t)(grid / 2);
    hipLaunchKernelGGL(mtblx_crc::k_crc32c_rows, dim3(g1), dim3(mtblx_crc::kLpThreads), 0, s, in->data, in->data_len,
                       in->blk_off, in->blk_len, in->nblk, crc, bad, framed);
  } else if (kc == 5) {   // one workgroup per CU (160 KiB of LDS), persistent
    const uint32_t g1 = need < (uint32_t)(grid / 2) ? need : (uint32_t)(grid / 2);
    hipLaunchKernelGGL(mtblx_crc::k_crc32c_lp5, dim3(g1), dim3(mtblx_crc::kLpThreads), 0, s, in->data, in->data_len,
                       in->blk_off, in->blk_len, in->nblk, crc, bad, framed);
  } else if (kc == 3) {   // one workgroup per CU (128 KiB of LDS each), persistent
    const uint32_t g1 = need < (uint32_t)(grid / 2) ? need : (uint32_t)(grid / 2);
    hipLaunchKernelGGL(mtblx_crc::k_crc32c_lp, dim3(g1), dim3(mtblx_crc::kLpThreads), 0, s, in->data, in->data_len,
                       in->blk_off, in->blk_len, in->nblk, crc, bad, framed);
  } else if (kc == 2)
    hipLaunchKernelGGL(mtblx_crc::k_crc32c_blocks_pf<true>, g, t, 0, s, in->data, in->data_len, in->blk_off,
                       in->blk_len, in->nblk, crc, bad, framed);
  else if (kc == 1)
    hipLaunchKernelGGL(mtblx_crc::k_crc32c_blocks_pf<false>, g, t, 0, s, in->data, in->data_len, in->blk_off,
                       in->blk_len, in->nblk, crc, bad, framed);
  else
    hipLaunchKernelGGL(mtblx_crc::k_crc32c_blocks, g, t, 0, s, in->data, in->data_len, in->blk_off, in->blk_len,
                       in->nblk, crc, bad, framed);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
