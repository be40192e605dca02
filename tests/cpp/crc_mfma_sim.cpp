// Host-side model of k_crc32c_mfma (oxidized-mtbl_amd/csrc/crc.hip) over the constant operands of
// csrc/crc_mfma.h: every MFMA is evaluated as the sum over its lane groups and operand slots
// (A's slot and B's slot in one lane group hold the same K index -- the property the kernel
// relies on), with the operands filled exactly as the kernel fills them: the fp4 bit planes of
// the window dwords (stage 1), the f16 pairs of the unreduced stage-1 sums (stage 2), the parity,
// the Horner step over super-windows, the column shift, the pad removal.  Checked against a
// bytewise CRC-32C (crate crc32c 0.4's function: Castagnoli, reflected, init / xorout ~0) on
// every length 0..2100 at all 16 alignments and on long blocks (several super-windows).
// Prints "ok <n>" or the first mismatch; exit status 0 / 1.  Test only (tests/test_crc_mfma_sim.py).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "crc_mfma.h"

using namespace mtblx_crc;

static uint32_t crc_ref(const uint8_t* d, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= d[i];
    for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kPoly : c >> 1;
  }
  return c ^ 0xFFFFFFFFu;
}

static double e2m1(uint32_t c) {   // fp4 code -> value
  static const double v[8] = {0, 0.5, 1, 1.5, 2, 3, 4, 6};
  return (c & 8u) ? -v[c & 7u] : v[c & 7u];
}

static uint32_t mul_tab(uint32_t c, const uint32_t (&T)[8][16]) {
  uint32_t p = 0;
  for (int j = 0; j < 8; ++j) p ^= T[j][(c >> (4 * j)) & 15u];
  return p;
}

// the kernel on one block: `blk` = the L content bytes, `o` = the block's start address mod 16
static uint32_t model(const MfmaTabs& T, const uint8_t* blk, uint32_t L, uint32_t o) {
  const uint32_t t = (16u - ((o + L) & 15u)) & 15u;
  const int64_t Lp = (int64_t)L + t;
  const uint32_t steps = (uint32_t)((Lp + kMStep - 1) / kMStep);
  const int64_t sb0 = Lp - (int64_t)kMStep * steps;
  // the bytes the lanes see, by block position p in [sb0, Lp): zero outside [0, L), init folded
  std::vector<uint8_t> P((size_t)kMStep * steps, 0);
  for (int64_t p = 0; p < L; ++p) P[(size_t)(p - sb0)] = blk[p];
  for (int i = 0; i < 4; ++i) P[(size_t)(i - sb0)] ^= 0xFFu;
  uint32_t acc[16] = {};
  bool first_sw = true;
  double c2[32][16] = {};
  for (int64_t s = steps - 1; s >= 0; --s) {
    const uint8_t* st = &P[(size_t)(Lp - kMStep * (s + 1) - sb0)];
    // stage 1: C1[r][n] over lane groups g, k-steps k, slots (q, i)
    double c1[32][16] = {};
    for (int n = 0; n < 16; ++n)
      for (int g = 0; g < 4; ++g) {
        const uint8_t* ch = st + 16 * (60 - 4 * n + g);   // chunk kx of the lane (g, n)
        for (int k = 0; k < kMKs; ++k) {
          uint32_t w;
          memcpy(&w, ch + 4 * k, 4);
          const uint32_t b[4] = {w & 0x11111111u, w & 0x22222222u, w & 0x44444444u, (w >> 1) & 0x44444444u};
          for (int r = 0; r < 32; ++r) {
            const uint32_t* a = T.a[k][r >> 4][16 * g + (r & 15)];
            for (int q = 0; q < 4; ++q)
              for (int i = 0; i < 8; ++i) c1[r][n] += e2m1((a[q] >> (4 * i)) & 15u) * e2m1((b[q] >> (4 * i)) & 15u);
          }
        }
      }
    // stage 2 (f16): B lane (g, n) slot j = C1[rho(g, j)][n]; A lane (g, r) slot j
    const int tt = (int)(s & (kMSup - 1));
    for (int n = 0; n < 16; ++n)
      for (int ro = 0; ro < 32; ++ro)
        for (int g = 0; g < 4; ++g)
          for (int j = 0; j < 8; ++j) {
            const int rho = j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4);
            const uint32_t h16 = (T.a2[tt][ro >> 4][16 * g + (ro & 15)][j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
            if (h16 != 0 && h16 != kF16One) return 0xDEADu;
            if (c1[rho][n] >= 2048) return 0xBEEFu;   // f16 exactness bound
            if (h16) c2[ro][n] += c1[rho][n];
          }
    if (tt != 0) continue;
    for (int n = 0; n < 16; ++n) {
      uint32_t dv = 0;
      for (int r = 0; r < 32; ++r) dv |= ((uint32_t)(int64_t)c2[r][n] & 1u) << r;
      acc[n] = first_sw ? dv : mul_tab(acc[n], T.swk) ^ dv;
      for (int r = 0; r < 32; ++r) c2[r][n] = 0;
    }
    first_sw = false;
  }
  uint32_t C = 0;
  for (int n = 0; n < 16; ++n) C ^= mul_tab(acc[n], T.col[n]);
  if (t) C = mul_tab(C, T.inv[t]);
  return C ^ 0xFFFFFFFFu;
}

int main() {
  static MfmaTabs T;   // the constexpr constructor, run on the host
  std::mt19937_64 rng(7);
  std::vector<uint8_t> buf(70000);
  for (auto& b : buf) b = (uint8_t)rng();
  int n = 0;
  auto check = [&](uint32_t L, uint32_t o) {
    const uint8_t* d = buf.data() + 3 + (rng() % 1000);
    const uint32_t got = model(T, d, L, o), exp = crc_ref(d, L);
    ++n;
    if (got != exp) {
      printf("mismatch L=%u o=%u got %08x exp %08x\n", L, o, got, exp);
      exit(1);
    }
  };
  for (uint32_t L = 4; L <= 2100; L += (L < 80 ? 1 : 37))
    for (uint32_t o = 0; o < 16; o += (L < 80 ? 1 : 5)) check(L, o);
  for (uint32_t L : {8191u, 8192u, 8193u, 9000u, 16384u, 16400u, 24577u, 40000u, 65536u})
    for (uint32_t o : {0u, 7u, 15u}) check(L, o);
  printf("ok %d\n", n);
  return 0;
}
