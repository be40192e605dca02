// crc_dev.h — CRC-32C device helpers shared by crc.hip (block verify) and reader.hip (get).
// See crc.hip for the method.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bounds.h"

namespace mtblx_crc {

typedef uint32_t v4u __attribute__((ext_vector_type(4), aligned(1)));

constexpr uint32_t kPoly = 0x82F63B78u;
constexpr int kChunk = 64;
constexpr int kWave = 64;
constexpr int kThreads = 256;

constexpr uint32_t multmodp(uint32_t a, uint32_t b) {  // a * b mod P, reflected (x^0 = bit 31)
  uint32_t p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & (0x80000000u >> i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

struct Tables {
  uint32_t byte[256];   // byte-wise table
  uint32_t slice[4][256];   // slicing-by-4: slice[k][i] = CRC of byte i followed by k zero bytes
  uint32_t xb[64];      // x^(8 * r)              r < 64
  uint32_t x0[512];     // x^(512 * m)            m < 512
  uint32_t x1[512];     // x^(512 * 512 * m)
  uint32_t x2[512];     // x^(512 * 512 * 512 * m)
  static constexpr uint32_t x8_1() {   // x^8
    uint32_t v = 0x80000000u;
    for (int k = 0; k < 8; ++k) v = (v & 1u) ? (v >> 1) ^ kPoly : v >> 1;
    return v;
  }
  constexpr Tables() : byte(), slice(), xb(), x0(), x1(), x2() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : c >> 1;
      byte[i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t t = byte[i];
      slice[0][i] = t;
      for (int k = 1; k < 4; ++k) {
        t = (t >> 8) ^ byte[t & 0xFFu];
        slice[k][i] = t;
      }
    }
    // x^8 = one byte of shift; x^(512) = 64 bytes
    uint32_t x8 = 0x80000000u;                                   // x^0
    for (int k = 0; k < 8; ++k) x8 = (x8 & 1u) ? (x8 >> 1) ^ kPoly : x8 >> 1;   // x^8
    xb[0] = 0x80000000u;
    for (int r = 1; r < 64; ++r) xb[r] = multmodp(x8_1(), xb[r - 1]);
    uint32_t x512 = 0x80000000u;
    for (int k = 0; k < kChunk; ++k) x512 = multmodp(x8, x512);
    x0[0] = 0x80000000u;
    for (int m = 1; m < 512; ++m) x0[m] = multmodp(x512, x0[m - 1]);
    const uint32_t s1 = multmodp(x512, x0[511]);                  // x^(512 * 512)
    x1[0] = 0x80000000u;
    for (int m = 1; m < 512; ++m) x1[m] = multmodp(s1, x1[m - 1]);
    const uint32_t s2 = multmodp(s1, x1[511]);                    // x^(512 * 512^2)
    x2[0] = 0x80000000u;
    for (int m = 1; m < 512; ++m) x2[m] = multmodp(s2, x2[m - 1]);
  }
};

static __constant__ Tables kTab = Tables();

// Block CRC windows (crc.hip): 72 bytes, so 64 lanes cover 4608 bytes in one pass -- the
// Writer's 4 KiB blocks run a little over 4096 bytes, which 64-byte windows would split into a
// full pass plus one for 1-2 lanes.
constexpr int kCrcWin = 72;

// Multiplication by the constants x^(8 kCrcWin k) through nibble tables: multmodp(c, K) is
// linear in c, so it is the XOR over c's eight nibbles of a[k][j][nibble j] =
// multmodp(nibble << 4j, K).  a: K = x^(576 k), k < 64 (the windows of a block up to 4.5 KiB);
// b: K = x^(576 * 64 m), m < 16 (with a, every window of a block up to 72 KiB).  Built from
// K·x^i, i < 32 (bit 31 - i of c is x^i).
struct MulTabs {
  uint32_t a[64][8][16];
  uint32_t b[16][8][16];
  static constexpr uint32_t mulx(uint32_t v) { return (v & 1u) ? (v >> 1) ^ kPoly : v >> 1; }
  static constexpr void fill(uint32_t (&t)[8][16], uint32_t K) {
    uint32_t base[32] = {};
    base[0] = K;
    for (int i = 1; i < 32; ++i) base[i] = mulx(base[i - 1]);
    for (int j = 0; j < 8; ++j)
      for (uint32_t v = 0; v < 16; ++v) {
        uint32_t p = 0;
        for (int u = 0; u < 4; ++u)
          if ((v >> u) & 1u) p ^= base[31 - 4 * j - u];
        t[j][v] = p;
      }
  }
  constexpr MulTabs() : a(), b() {
    uint32_t xw = 0x80000000u;   // x^0 -> x^(8 kCrcWin): single-bit shifts
    for (int i = 0; i < 8 * kCrcWin; ++i) xw = mulx(xw);
    uint32_t K = 0x80000000u;
    for (int k = 0; k < 64; ++k) {
      fill(a[k], K);
      K = multmodp(xw, K);
    }
    // K = x^(8 kCrcWin 64) now
    const uint32_t xw64 = K;
    uint32_t M = 0x80000000u;
    for (int m = 0; m < 16; ++m) {
      fill(b[m], M);
      M = multmodp(xw64, M);
    }
  }
};

static __constant__ MulTabs kMul = MulTabs();
struct MulLds {   // the same layout, trivially constructible (an LDS copy of kMul)
  uint32_t a[64][8][16];
  uint32_t b[16][8][16];
};
static_assert(sizeof(MulLds) == sizeof(MulTabs), "MulLds mirrors MulTabs");

// c * K through one [8][16] nibble table (LDS)
__device__ __forceinline__ uint32_t mul_nib(uint32_t c, const uint32_t (*T)[16]) {
  uint32_t p = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) p ^= T[j][(c >> (4 * j)) & 15u];
  return p;
}

__device__ __forceinline__ uint32_t dmultmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    p ^= ((a << i) & 0x80000000u) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? kPoly : 0u);
  }
  return p;
}

__device__ __forceinline__ uint32_t xpow512(uint64_t m) {  // x^(512 m) mod P
  uint32_t r = kTab.x0[m & 511];
  if (m >> 9) r = dmultmodp(kTab.x1[(m >> 9) & 511], r);
  if (m >> 18) r = dmultmodp(kTab.x2[(m >> 18) & 511], r);
  return r;
}

__device__ __forceinline__ uint32_t xpow8(uint64_t n) {  // x^(8 n) mod P: n bytes of shift
  const uint32_t r = kTab.xb[n & 63];
  return (n >> 6) ? dmultmodp(xpow512(n >> 6), r) : r;
}

// CRC-32C of d[0..L) by one wave (all 64 lanes call it with the same arguments; the result
// is returned to every lane).  T = the byte table in LDS.
__device__ __forceinline__ uint32_t wave_crc32c(const uint8_t* d, uint64_t L, const uint32_t* T, int lane) {
  uint32_t acc = 0;
  if (L >= (uint64_t)kChunk) {
    for (uint64_t j = lane; j * kChunk < L; j += kWave) {
      // chunk [lo, hi); the 64-byte window [lo, lo + 64) is always inside the block
      const uint64_t hi = L - j * kChunk, lo = hi > (uint64_t)kChunk ? hi - kChunk : 0;
      const uint32_t n = (uint32_t)(hi - lo);
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        MTBLX_CHK(d + lo + 16 * q, 16);
        const v4u x = *reinterpret_cast<const v4u*>(d + lo + 16 * q);
        w[4 * q] = x.x; w[4 * q + 1] = x.y; w[4 * q + 2] = x.z; w[4 * q + 3] = x.w;
      }
      // the 0xFFFFFFFF init, folded into the block's first 4 bytes (they may straddle the
      // leftmost two chunks when the leftmost one is shorter than 4 bytes)
      if (lo < 4) w[0] ^= 0xFFFFFFFFu >> (8 * lo);
      uint32_t c = 0;
#pragma unroll
      for (int k = 0; k < kChunk; ++k) {
        const uint32_t byte = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const uint32_t nc = T[(c ^ byte) & 0xFFu] ^ (c >> 8);
        c = ((uint32_t)k < n) ? nc : c;
      }
      acc ^= dmultmodp(xpow512(j), c);
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, s, kWave);
    return acc ^ 0xFFFFFFFFu;
  }
  uint32_t c = 0xFFFFFFFFu;   // short block: every lane serially (same result everywhere)
  for (uint64_t i = 0; i < L; ++i) {
    MTBLX_CHK(d + i, 1);
    c = T[(c ^ d[i]) & 0xFFu] ^ (c >> 8);
  }
  return c ^ 0xFFFFFFFFu;
}

}  // namespace mtblx_crc
