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

#ifndef MTBLX_CRC_THREADS
#define MTBLX_CRC_THREADS 1024
#endif
constexpr int kCrcThreads = MTBLX_CRC_THREADS;   // 16 waves per workgroup (LDS: 48 KiB each)

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

// Round 3 variants, measured on the cfg2 batch (scripts/crc_ab.py, HIP events, two alternations,
// profiles/r03/crc_ab.txt) and removed -- all slower than k_crc32c_blocks (0.124-0.126 ms):
//   1 / 2  the first window loaded one block ahead; slicing-by-8 / slicing-by-72 (72
//          independent lookups per window, no serial chain)                   0.135 / 0.137 ms
//   3      lane-private slicing-by-4 tables (128 KiB, conflict-free), 32-step GF(2) shifts 0.157
//   5      3 + lane-interleaved nibble tables for the window shift (160 KiB)            0.130
//   6      coalesced 1 KiB rows (lane = 16 bytes), Horner across rows on the SALU         0.176
//   7      lane-private NIBBLE tables (16-entry: 32 KiB per workgroup, two per CU)        0.155
// Removing the bank conflicts (3, 5, 7) or the scattered window loads (6) did not pay: the
// kernel is not bound by either alone, and every variant added vector instructions per byte.

}  // namespace mtblx_crc

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
// 98 VGPRs: one 1024-thread workgroup is resident per CU, so a grid of one workgroup per CU runs
// in a single round; 2 per CU measured 0.1256-0.1261 ms against 0.1232 (profiles/r03/final2)
#ifndef MTBLX_CRC_WG_PER_CU
#define MTBLX_CRC_WG_PER_CU 1
#endif
    grid = (ncu > 0 ? ncu : 256) * MTBLX_CRC_WG_PER_CU;
  }
  const uint32_t wpg = mtblx_crc::kCrcThreads / mtblx_crc::kWave;   // waves (blocks in flight) per workgroup
  const uint32_t need = (in->nblk + wpg - 1u) / wpg;
  const dim3 g(need < (uint32_t)grid ? need : (uint32_t)grid), t(mtblx_crc::kCrcThreads);
  hipLaunchKernelGGL(mtblx_crc::k_crc32c_blocks, g, t, 0, reinterpret_cast<hipStream_t>(stream), in->data, in->data_len,
                     in->blk_off, in->blk_len, in->nblk, crc, bad, framed);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
