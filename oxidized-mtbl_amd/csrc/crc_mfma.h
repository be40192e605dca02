// crc_mfma.h — constant operands of the matrix-core CRC-32C (crc.hip k_crc32c_mfma).
//
// CRC-32C without init/xorout ("raw") is linear over GF(2): the raw CRC of a 64-byte window is
// M_w · bits, M_w a constant 32 x 512 bit matrix.  With every bit as an fp4 (e2m1) operand
// element the product is one fp4 GEMM whose f32 sums carry the GF(2) result in their parity.
// A wave reads one block at a time, a STEP = 16 consecutive windows (1 KiB) per MFMA column set:
// column n of step s holds window w = 16 s + n, counted from the block's END.
//   stage 1  C1 = M_w · window bits            16x16x128 fp4 MFMA, K = 512 over 4 k-steps,
//            (rows = CRC bits, columns = the     two row halves per k-step
//             step's 16 windows)
//   stage 2  per column, the steps t of a super-window (kMSup = 8 steps = 8 KiB) shifted by
//            x^(8·1024·t) and summed: S_t · C1_t, one 16x16x32 f16 MFMA pair per step on the
//            UNREDUCED integer sums (exact in f16 below 2048; their parity is linear, so the
//            GF(2) shift applied to the integers keeps the parity of the shifted result)
//   stage 3  per column, Horner over the super-windows from the block's start: acc = acc ·
//            x^(8·8192) + parity(C2_S) (nibble table swk), then the column shift x^(8·64·n)
//            (nibble tables col) and an XOR over the 16 columns: the raw CRC of the block padded
//            with t < 16 zero bytes to a 16-byte aligned end, times x^(-8t) (nibble tables inv):
//            the block's raw CRC
// The reference's checksum is crate crc32c 0.4 over each block's stored bytes
// (/root/reference/src/reader.rs:159-164); polynomial and tables as crc_dev.h.
//
// Operand layout.  Lane l of a 16x16x128 MFMA holds 32 K-elements of row (A) / column (B) l & 15;
// A's lane l and B's lane l hold the same K indices in the same slots (slot s = nibble s & 7 of
// dword s >> 3), whatever K order the hardware uses.  So a B slot is bound to a data bit by how the
// kernel fills it, and A's slot in the same lane group carries M_w's entry for that bit:
//   B: lane (g = l >> 4, n = l & 15), k-step t: raw dword w = window dword D = 4g + t of window
//      n (the lane holds window bytes [16g, 16g + 16)); the four operand dwords are the bit planes
//      w & 0x11111111, w & 0x22222222, w & 0x44444444, (w >> 1) & 0x44444444: slot (q, i) is bit
//      4i + q of w, as an e2m1 value 0.5 / 1 / 2 / 2 (q = 0 / 1 / 2 / 3).
//   A: the matching entry times 2 / 1 / 0.5 / 0.5, so every product of two set bits is exactly 1.
// The stage-2 f16 MFMA (8 halves per lane, again the same K in the same slot of A and B): B lane
// (g, n) slot j = the stage-1 sum of CRC row rho(g, j) = (j < 4 ? 4g + j : 16 + 4g + j - 4) of
// window n -- exactly the lane's C1 registers in order, packed by v_cvt_pkrtz; A lane (g, r) slot
// j = bit r (row half 0) or 16 + r (half 1) of S_t(e_rho) as 1.0 / 0.0.
// C/D (dtype-independent on gfx950): lane l, register i = row 4 (l >> 4) + i, column l & 15.
#pragma once
#include <stdint.h>

#include "crc_dev.h"

namespace mtblx_crc {

constexpr int kMWin = 64;             // stage-1 window: bytes of one column per 4 k-steps
constexpr int kMKs = kMWin / 16;       // k-steps per window (one raw dword of the lane each)
constexpr int kMStep = 16 * kMWin;     // a step: 16 consecutive windows of one block, 1 KiB
constexpr int kMSup = 8;               // steps per super-window (stage 2): 8 KiB
constexpr uint32_t kFp4Half = 0x1u, kFp4One = 0x2u, kFp4Two = 0x4u;   // e2m1 codes of 0.5, 1, 2
constexpr uint32_t kF16One = 0x3C00u;                                 // f16 1.0

struct MfmaTabs {
  uint32_t a[kMKs][2][64][4];   // stage-1 A operand: [k-step][row half][lane][dword]
  uint32_t a2[kMSup][2][64][4];   // stage-2 f16 A operand: [step][row half][lane][dword]
  uint32_t swk[8][16];            // nibble tables of x^(8·1024·kMSup): one super-window (stage 3)
  uint32_t col[16][8][16];    // nibble tables of x^(8·64·n): the column shift, n < 16
  uint32_t inv[16][8][16];    // nibble tables of x^(-8 t), t < 16: t zero bytes appended, removed
  uint32_t max_row;           // largest popcount of an M_w row (the stage-1 sums stay below it)

  static constexpr uint32_t zbyte(uint32_t c) {   // c · x^8: one zero byte appended
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : c >> 1;
    return c;
  }
  static constexpr uint32_t unx(uint32_t c) {   // c · x^-1: one step of the reflected CRC undone
    return (c & 0x80000000u) ? (((c ^ kPoly) << 1) | 1u) : (c << 1);
  }
  constexpr MfmaTabs() : a(), a2(), swk(), col(), inv(), max_row(0) {
    // column of M_w for window byte p, bit b: raw CRC of a kMWin-byte message holding only that bit
    uint32_t mcol[kMWin][8] = {};
    for (int b = 0; b < 8; ++b) {
      uint32_t c = zbyte(1u << b);
      for (int p = kMWin - 1; p >= 0; --p) {
        mcol[p][b] = c;
        c = zbyte(c);
      }
    }
    for (int r = 0; r < 32; ++r) {
      uint32_t pc = 0;
      for (int p = 0; p < kMWin; ++p)
        for (int b = 0; b < 8; ++b) pc += (mcol[p][b] >> r) & 1u;
      if (pc > max_row) max_row = pc;
    }
    const uint32_t code[4] = {kFp4Two, kFp4One, kFp4Half, kFp4Half};
    for (int t = 0; t < kMKs; ++t)
      for (int h = 0; h < 2; ++h)
        for (int l = 0; l < 64; ++l) {
          const int g = l >> 4, r = 16 * h + (l & 15);
          const int D = 4 * g + t;
          for (int s = 0; s < 32; ++s) {
            const int q = s >> 3, i = s & 7, beta = 4 * i + q;
            const int byte = 4 * D + beta / 8, bit = beta % 8;
            if ((mcol[byte][bit] >> r) & 1u) a[t][h][l][q] |= code[q] << (4 * i);
          }
        }
    // column shifts x^(8·kMWin·n)
    uint32_t xw = 0x80000000u;
    for (int i = 0; i < 8 * kMWin; ++i) xw = (xw & 1u) ? (xw >> 1) ^ kPoly : xw >> 1;
    uint32_t C = 0x80000000u;
    for (int n = 0; n < 16; ++n) {
      MulTabs::fill(col[n], C);
      C = multmodp(xw, C);
    }
    // S_t(e_r) = x^(8·kMStep·t) · x^(31 - r) (bit r of a reflected CRC word is x^(31 - r))
    const uint32_t xs = C;   // x^(8·kMStep)
    uint32_t S[kMSup][32] = {};
    uint32_t K = 0x80000000u;
    for (int t = 0; t < kMSup; ++t) {
      uint32_t v = K;   // K · x^i for i = 0..31
      for (int i = 0; i < 32; ++i) {
        S[t][31 - i] = v;
        v = (v & 1u) ? (v >> 1) ^ kPoly : v >> 1;
      }
      K = multmodp(xs, K);
    }
    // stage-2 A (f16): lane (g, r), half h, slot j -> dword j >> 1, half j & 1
    for (int t = 0; t < kMSup; ++t)
      for (int h = 0; h < 2; ++h)
        for (int l = 0; l < 64; ++l) {
          const int g = l >> 4, ro = 16 * h + (l & 15);
          for (int j = 0; j < 8; ++j) {
            const int rho = j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4);
            if ((S[t][rho] >> ro) & 1u) a2[t][h][l][j >> 1] |= kF16One << (16 * (j & 1));
          }
        }
    uint32_t U = 0x80000000u;   // x^(-8 t)
    for (int t = 0; t < 16; ++t) {
      MulTabs::fill(inv[t], U);
      for (int k = 0; k < 8; ++k) U = unx(U);
    }
    MulTabs::fill(swk, K);   // K = x^(8·1024·kMSup) now
  }
};

// nibble tables of the super-window shifts x^(8·8192·S), S < N (a super-window's raw CRC moved to
// its place in a block of N super-windows at most): encode.hip (blocks assembled in LDS) and the
// fused verify of decode.hip (blocks staged in LDS)
template <int N>
struct SwTabs {
  uint32_t t[N][8][16];
  constexpr SwTabs() : t() {
    static_assert(kMStep * kMSup == 8192, "8 KiB super-windows");
    uint32_t K = 0x80000000u;   // x^8, squared 13 times: x^(8·8192)
    for (int k = 0; k < 8; ++k) K = (K & 1u) ? (K >> 1) ^ kPoly : K >> 1;
    for (int q = 0; q < 13; ++q) K = multmodp(K, K);
    uint32_t P = 0x80000000u;
    for (int S = 0; S < N; ++S) {
      MulTabs::fill(t[S], P);
      P = multmodp(K, P);
    }
  }
};

}  // namespace mtblx_crc
