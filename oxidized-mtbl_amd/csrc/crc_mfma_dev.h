// crc_mfma_dev.h — device side of the matrix-core CRC-32C (crc_mfma.h has the method, the operand
// layout and the constant tables): the per-step MFMA chain shared by k_crc32c_mfma (crc.hip, block
// bytes through an LDS-DMA ring) and k_encode (encode.hip, the block assembled in LDS).
#pragma once
#include <stdint.h>

#include "crc_dev.h"
#include "crc_mfma.h"

namespace mtblx_crc {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));

__device__ __forceinline__ v4f mfma_fp4(v4i a, v4i b, v4f c) {
  const v8i a8 = {a.x, a.y, a.z, a.w, 0, 0, 0, 0};
  const v8i b8 = {b.x, b.y, b.z, b.w, 0, 0, 0, 0};
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, c, 4, 4, 0, 0, 0, 0);
}
__device__ __forceinline__ v4f mfma_f16(v4i a, v4i b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, a), __builtin_bit_cast(v8h, b), c, 0, 0, 0);
}
// two stage-1 sums as f16 (integers below 2048: exact)
__device__ __forceinline__ int pk16(float a, float b) { return __builtin_bit_cast(int, __builtin_amdgcn_cvt_pkrtz(a, b)); }

// the parities of four exact integer-valued sums (0 <= v < 2^19) as a nibble: v + 1.5·2^(23-k)
// keeps v · 2^k in the low mantissa bits, so bit k of the sum's bits is v's parity
__device__ __forceinline__ uint32_t bfi(uint32_t mask, uint32_t a, uint32_t b) { return (mask & a) | (~mask & b); }
__device__ __forceinline__ uint32_t par_nib(v4f v) {
  uint32_t x = __float_as_uint(v.x + 12582912.0f) & 1u;
  x = bfi(2u, __float_as_uint(v.y + 6291456.0f), x);
  x = bfi(4u, __float_as_uint(v.z + 3145728.0f), x);
  return bfi(8u, __float_as_uint(v.w + 1572864.0f), x);
}

// XOR over the 16 lanes of each DPP row, in every lane of the row (row_ror 8, 4, 2, 1)
__device__ __forceinline__ uint32_t row_xor(uint32_t x) {
  x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xf, 0xf, false);
  x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x124, 0xf, 0xf, false);
  x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x122, 0xf, 0xf, false);
  x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x121, 0xf, 0xf, false);
  return x;
}

// one step (16 windows of 64 bytes, one 16-byte chunk x per lane: lane (g, n) holds bytes
// [16 g, 16 g + 16) of window n) accumulated into the stage-2 sums of its super-window step t:
// the fp4 bit planes, stage 1 (8 MFMAs over A = MfmaTabs::a), the unreduced sums as f16 and stage 2
// (2 MFMAs over a2lo / a2hi = MfmaTabs::a2[t])
__device__ __forceinline__ void mfma_step(const v4i (&A)[kMKs][2], v4u x, v4i a2lo, v4i a2hi, v4f& c2a, v4f& c2b) {
  const uint32_t w[kMKs] = {x.x, x.y, x.z, x.w};
  v4f c1a = {0.f, 0.f, 0.f, 0.f}, c1b = c1a;
#pragma unroll
  for (int k = 0; k < kMKs; ++k) {
    const uint32_t v = w[k];
    const v4i b = {(int)(v & 0x11111111u), (int)(v & 0x22222222u), (int)(v & 0x44444444u),
                   (int)((v >> 1) & 0x44444444u)};
    c1a = mfma_fp4(A[k][0], b, c1a);
    c1b = mfma_fp4(A[k][1], b, c1b);
  }
  const v4i b2 = {pk16(c1a.x, c1a.y), pk16(c1a.z, c1a.w), pk16(c1b.x, c1b.y), pk16(c1b.z, c1b.w)};
  c2a = mfma_f16(a2lo, b2, c2a);
  c2b = mfma_f16(a2hi, b2, c2b);
}

// mfma_step with the stage-1 operand A read from memory (pa: lane's entry of MfmaTabs::a, as v4i,
// k-step k half h at pa[(2 k + h) 64]) instead of registers: 8 VGPRs live instead of 32
__device__ __forceinline__ void mfma_step_ld(const v4i* pa, v4u x, v4i a2lo, v4i a2hi, v4f& c2a, v4f& c2b) {
  const uint32_t w[kMKs] = {x.x, x.y, x.z, x.w};
  v4f c1a = {0.f, 0.f, 0.f, 0.f}, c1b = c1a;
#pragma unroll
  for (int k = 0; k < kMKs; ++k) {
    const uint32_t v = w[k];
    const v4i b = {(int)(v & 0x11111111u), (int)(v & 0x22222222u), (int)(v & 0x44444444u),
                   (int)((v >> 1) & 0x44444444u)};
    c1a = mfma_fp4(pa[(2 * k) * 64], b, c1a);
    c1b = mfma_fp4(pa[(2 * k + 1) * 64], b, c1b);
  }
  const v4i b2 = {pk16(c1a.x, c1a.y), pk16(c1a.z, c1a.w), pk16(c1b.x, c1b.y), pk16(c1b.z, c1b.w)};
  c2a = mfma_f16(a2lo, b2, c2a);
  c2b = mfma_f16(a2hi, b2, c2b);
}

// The block's first bytes: a step's chunks lie at block positions a = sb + 16 k, 16-byte aligned
// in memory while the block is not.  A chunk wholly before the block is zeroed (its DMA read
// the block's first aligned chunk instead); the chunk holding byte 0 keeps bytes >= 0 only; the
// 0xFFFFFFFF init is folded into bytes 0..3 (one or two chunks, one or two steps).
__device__ __forceinline__ uint32_t head_dword(uint32_t w, int pos) {
  if (pos >= 4) return w;
  const uint32_t keep = pos <= -4 ? 0u : (pos < 0 ? 0xFFFFFFFFu << (8 * (uint32_t)(-pos)) : 0xFFFFFFFFu);
  const uint32_t fold = pos < 0 ? keep : 0xFFFFFFFFu >> (8 * (uint32_t)pos);
  return (w & keep) ^ fold;
}
__device__ __forceinline__ v4u head_chunk(v4u x, int a) {
  if (a <= -16) return v4u{0u, 0u, 0u, 0u};
  if (a >= 4) return x;
  return v4u{head_dword(x.x, a), head_dword(x.y, a + 4), head_dword(x.z, a + 8), head_dword(x.w, a + 12)};
}
// head_chunk without branches (k_crc32c_mfma's head steps): dword d of the chunk starts at block
// position pos = a + 4 d; with S = 32 + 8 pos, the kept bytes (positions >= 0) are the low word of
// 0xFFFFFFFF'00000000 >> clamp(S, 0, 32) and the init bytes (positions 0..3) the low word of the same
// value >> clamp(S, 0, 64) mod 64 -- two 64-bit shifts and a bitop per dword, no divergent exec
__device__ __forceinline__ v4u head_chunk_fast(v4u x, int a) {
  constexpr uint64_t V = 0xFFFFFFFF00000000ull;
  const int S0 = 32 + 8 * a;
  uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int S = S0 + 32 * d;
    const int c = S < 0 ? 0 : S;
    const uint32_t keep = (uint32_t)(V >> (c < 32 ? c : 32));
    const uint32_t fold = (uint32_t)(V >> ((c < 64 ? c : 64) & 63));
    w[d] = (w[d] & keep) ^ fold;
  }
  return v4u{w[0], w[1], w[2], w[3]};
}
// the pad after the block's end: t < 16 zero bytes in the last chunk of the block's last step
__device__ __forceinline__ v4u tail_chunk(v4u y, uint32_t t) {
  const uint32_t k = 16u - t;   // bytes kept
  const auto m = [&](uint32_t d) {
    return k >= 4 * d + 4 ? 0xFFFFFFFFu : (k <= 4 * d ? 0u : 0xFFFFFFFFu >> (8 * (4 * d + 4 - k)));
  };
  return v4u{y.x & m(0), y.y & m(1), y.z & m(2), y.w & m(3)};
}

}  // namespace mtblx_crc
