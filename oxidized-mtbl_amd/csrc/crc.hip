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
  if (kc == 2)
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
