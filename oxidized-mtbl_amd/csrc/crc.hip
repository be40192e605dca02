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

#include "bounds.h"
#include "devinfo.h"
#include "crc_dev.h"
#include "crc_mfma.h"
#include "crc_mfma_dev.h"
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
  MTBLX_CHK(p, 16);
#if MTBLX_CRC_NT_LOADS
  return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
#else
  return *reinterpret_cast<const v4u*>(p);
#endif
}
__device__ __forceinline__ v2u crc_ld8(const uint8_t* p) {
  MTBLX_CHK(p, 8);
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
        if (p >= 0) MTBLX_CHK(d + p, 1);
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
    MTBLX_CHK(blk_off + b, 8);
    MTBLX_CHK(blk_len + b, 4);
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
      if (crc_out) MTBLX_CHK(crc_out + b, 4);
      if (bad) MTBLX_CHK(bad + b, 1);
      if (bad && !oob && framed && off >= 4) MTBLX_CHK(d - 4, 4);
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

// ---------------------------------------------------------------------------------------------
// k_crc32c_mfma: the same checksum on the matrix cores (crc_mfma.h has the method and the
// operand layout).  Persistent, one kMWaves-wave workgroup per CU: wave w takes the blocks w,
// w + W, w + 2W, ... (interleaved: concurrent waves read neighbouring blocks, which spreads the
// reads over the HBM channels), their offsets / lengths 64 at a time in lane registers.  A wave
// reads each block from its start to its end, a STEP of 16 consecutive 64-byte windows (1 KiB,
// one LDS-DMA wave-instruction) at a time; windows are counted from the block's 16-byte aligned
// END, so one set of shift matrices serves every block length; bytes before the block start are
// zero and the 0xFFFFFFFF init is folded into bytes 0..3.  Lane (g = lane >> 4, n = lane & 15)
// feeds 16 bytes of window n.  The steps reach the lanes through a per-wave LDS ring of kRing
// slots filled kRing - 1 steps ahead across block boundaries, so the wait for a step is one
// constant s_waitcnt.  Per step: 5 vector instructions per loaded dword (the fp4 bit planes),
// 8 fp4 MFMAs, 4 conversions and 2 f16 MFMAs; per super-window (8 KiB) a parity extraction and
// a Horner step; per block the column shifts, a 64-lane XOR and the pad removal.
// ---------------------------------------------------------------------------------------------
static __constant__ MfmaTabs kMfma = MfmaTabs();
static_assert(MfmaTabs().max_row < 1024, "stage-1 sums stay below 2^10: exact in f16 and in the stage-2 sums");

// MTBLX_CRC_ABL (diagnostic, wrong checksums by construction): 1 = the ring without stage 1/2,
// 2 = stage 1/2 on whatever the ring holds, no block reads
#if defined(MTBLX_CRC_ABL) && !defined(MTBLX_DIAG)
#error "MTBLX_CRC_ABL is an ablation: build it only through a diagnostic target (-DMTBLX_DIAG)"
#endif
#ifndef MTBLX_CRC_ABL
#define MTBLX_CRC_ABL 0
#endif
#ifndef MTBLX_CRC_MWAVES
#define MTBLX_CRC_MWAVES 16
#endif
#ifndef MTBLX_CRC_RING
#define MTBLX_CRC_RING 8
#endif
#ifndef MTBLX_CRC_PAIR   // two steps per loop iteration (in-wave ILP, A/B: measured slower); 0 = one
#define MTBLX_CRC_PAIR 0
#endif
#ifndef MTBLX_CRC_STEADY   // steady-state steps wait with the constant vmcnt(kRing - 1) (0: the variable wait)
#define MTBLX_CRC_STEADY 1
#endif
#ifndef MTBLX_CRC_HEAD2   // head steps: branch-free masks (head_chunk_fast); 0 = head_chunk
#define MTBLX_CRC_HEAD2 1
#endif
#ifndef MTBLX_CRC_DMA_AUX
#define MTBLX_CRC_DMA_AUX 2   // non-temporal: the block bytes are read once
#endif
constexpr int kMWaves = MTBLX_CRC_MWAVES;      // waves per workgroup, one workgroup per CU
constexpr int kMThreads = kMWaves * kWave;
constexpr int kRing = MTBLX_CRC_RING;          // steps per wave ring (1 KiB each)
static_assert((kRing & (kRing - 1)) == 0, "ring offsets wrap by a mask");
constexpr int kMTabLds = kMSup * 2 * 64 * 16 + 2 * 16 * 8 * 16 * 4;   // 32 KiB
static_assert(kMTabLds + kMWaves * kRing * kMStep <= 160 * 1024, "LDS: tables + rings");

typedef __attribute__((address_space(3))) void lds_void;

struct RingSlot {   // one step: its 64 16-byte chunks, lowest address first
  v4u c[kMStep / 16];
};
static_assert(kMStep / 16 == kWave, "one LDS-DMA wave-instruction per step");

// s_waitcnt vmcnt(k): a step has landed once at most the k DMA instructions of the k steps
// issued after it are outstanding (the counter retires in issue order).  The steady state waits
// vmcnt(kRing - 1) inline; this is the drain at the end of the wave's blocks.
__device__ __forceinline__ void wait_ring(uint32_t k) {
  switch (k) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
  }
}
__device__ __forceinline__ void wait_vm(uint32_t k) {   // vmcnt(k), k <= 7
  switch (k) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
  }
}
__device__ __forceinline__ void wait_steady() {
  static_assert(kRing >= 2 && kRing <= 8, "wait_ring covers up to 7 steps ahead");
  switch (kRing - 1) {
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
  }
}

// the lane's chunk of a landed slot (LDS address ax), and the step's two stage-2 operands (aa,
// aa + 1 KiB; issued first, so their latency overlaps).  Inline asm: the compiler treats a read
// of the ring it can see as aliasing every LDS-DMA in flight and waits vmcnt(0) before it, which
// would drain the ring; wait_ring / wait_steady has already waited for exactly this slot's DMA.
__device__ __forceinline__ v4u ring_read(uint32_t ax, uint32_t aa, v4i& lo, v4i& hi) {
  v4u x;
  asm volatile(
      "ds_read_b128 %1, %4\n\t"
      "ds_read_b128 %2, %4 offset:1024\n\t"
      "ds_read_b128 %0, %3\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(x), "=&v"(lo), "=&v"(hi)
      : "v"(ax), "v"(aa)
      : "memory");
  return x;
}

// two landed slots (steps s and s - 1 of one super-window) and their stage-2 operands, one wait
__device__ __forceinline__ void ring_read2(uint32_t ax, uint32_t ay, uint32_t aa, uint32_t ab, v4u& x, v4u& y,
                                           v4i& lo, v4i& hi, v4i& lo2, v4i& hi2) {
  asm volatile(
      "ds_read_b128 %2, %8\n\t"
      "ds_read_b128 %3, %8 offset:1024\n\t"
      "ds_read_b128 %4, %9\n\t"
      "ds_read_b128 %5, %9 offset:1024\n\t"
      "ds_read_b128 %0, %6\n\t"
      "ds_read_b128 %1, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(x), "=&v"(y), "=&v"(lo), "=&v"(hi), "=&v"(lo2), "=&v"(hi2)
      : "v"(ax), "v"(ay), "v"(aa), "v"(ab)
      : "memory");
}

// serial CRC-32C of a short block (< 4 bytes), one lane
__device__ __forceinline__ uint32_t crc_tiny(const uint8_t* d, uint64_t L) {
  uint32_t c = 0xFFFFFFFFu;
  for (uint64_t i = 0; i < L; ++i) {
    MTBLX_CHK(d + i, 1);
    c = kTab.byte[(c ^ d[i]) & 0xFFu] ^ (c >> 8);
  }
  return c ^ 0xFFFFFFFFu;
}

__device__ __forceinline__ void crc_store(const uint8_t* d, uint64_t off, bool oob, uint32_t c, uint32_t b,
                                          uint32_t* crc_out, uint8_t* bad, int framed) {
  if (crc_out) MTBLX_CHK(crc_out + b, 4);
  if (bad) MTBLX_CHK(bad + b, 1);
  if (bad && !oob && framed && off >= 4) MTBLX_CHK(d - 4, 4);
  if (crc_out) crc_out[b] = oob ? 0u : c;
  if (bad) {
    if (oob) {
      bad[b] = 1;   // the window runs past the buffer: the reference's slice panics
    } else {
      uint32_t stored = 0;
      if (framed && off >= 4)
        stored = (uint32_t)d[-4] | ((uint32_t)d[-3] << 8) | ((uint32_t)d[-2] << 16) | ((uint32_t)d[-1] << 24);
      bad[b] = (framed && off >= 4) ? (uint8_t)(stored != c) : (uint8_t)0;
    }
  }
}

// a block of the stream (wave-uniform values, read from the lane that holds the block)
struct MBlk {
  const uint8_t* p;   // the block's first byte
  uint32_t steps;     // ceil(Lp / 1 KiB), Lp = content length + t: padded to a 16-byte aligned end
  uint32_t t;         // pad bytes, < 16
  int32_t sb0;        // block position of the first step's chunk 0: Lp - 1 KiB · steps, in (-1024, 0]
  int32_t a0;         // block position of the 16-byte aligned chunk holding byte 0 (in [-15, 0])
};
__device__ __forceinline__ MBlk mblk_lane(const uint8_t* data, uint64_t off, uint32_t pk, int32_t sb0, int j) {
  MBlk m;
  m.p = data + ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)off, j) |
                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(off >> 32), j) << 32));
  const uint32_t q = (uint32_t)__builtin_amdgcn_readlane((int)pk, j);
  m.steps = q & 0x7FFFFFu;
  m.t = (q >> 23) & 15u;
  m.a0 = -(int32_t)(q >> 27);
  m.sb0 = __builtin_amdgcn_readlane(sb0, j);
  return m;
}

__global__ void __launch_bounds__(kMThreads, 1) k_crc32c_mfma(const uint8_t* __restrict__ data, uint64_t data_len,
                                                             const uint64_t* __restrict__ blk_off,
                                                             const uint32_t* __restrict__ blk_len, uint32_t nblk,
                                                             uint32_t* __restrict__ crc_out, uint8_t* __restrict__ bad,
                                                             int framed) {
  __shared__ v4i sA2[kMSup * 2 * 64];          // 16 KiB: stage-2 operands
  __shared__ uint32_t sCol[16][8][16];         // 8 KiB: column shifts
  __shared__ uint32_t sInv[16][8][16];         // 8 KiB: pad removal, t = 1..15; [0]: one super-window
  __shared__ RingSlot sRing[kMWaves][kRing];   // 128 KiB at 16 waves x 8 steps
  const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  {
    const v4i* a2 = reinterpret_cast<const v4i*>(&kMfma.a2[0][0][0][0]);
    for (int i = threadIdx.x; i < kMSup * 2 * 64; i += kMThreads) sA2[i] = a2[i];
    // sInv[0] (t = 0: no pad, never looked up) holds the Horner step's table instead
    for (int i = threadIdx.x; i < 16 * 8 * 16; i += kMThreads) {
      (&sCol[0][0][0])[i] = (&kMfma.col[0][0][0])[i];
      (&sInv[0][0][0])[i] = i < 8 * 16 ? (&kMfma.swk[0][0])[i] : (&kMfma.inv[0][0][0])[i];
    }
  }
  v4i A[kMKs][2];
#pragma unroll
  for (int t = 0; t < kMKs; ++t) {
    A[t][0] = reinterpret_cast<const v4i*>(&kMfma.a[t][0][0][0])[lane];
    A[t][1] = reinterpret_cast<const v4i*>(&kMfma.a[t][1][0][0])[lane];
  }
  // use A here, so the wait for its loads is placed before the loop: left to its first use
  // inside the loop, the wait would be a vmcnt(0) in every iteration, draining the ring
#pragma unroll
  for (int t = 0; t < kMKs; ++t) asm volatile("" ::"v"(A[t][0]), "v"(A[t][1]));
  __syncthreads();
  const uint64_t base = (uint64_t)(uintptr_t)data;
  const uint32_t W = gridDim.x * kMWaves;
  const uint32_t w0 = blockIdx.x * kMWaves + wv;
  const uint32_t kx = 60u - 4u * (uint32_t)n + (uint32_t)g;   // the lane's chunk of a step
  // LDS addresses: the wave's ring (slot k at + 1 KiB k), the lane's chunk in slot 0, and the
  // lane's stage-2 operand of step 0, half 0 (step t, half h: + 2 KiB t + 1 KiB h)
  const uint32_t ring_base = (uint32_t)(uintptr_t)(const lds_void*)&sRing[wv][0];
  const uint32_t ring_lane = ring_base + 16u * kx;
  const uint32_t a2_lane = (uint32_t)(uintptr_t)(const lds_void*)&sA2[lane];
  const int32_t lane16 = 16 * lane;
  constexpr uint32_t kRingMask = (uint32_t)(kRing * kMStep) - 1u;

  // the wave's blocks w0 + k W, 64 at a time: lane j holds block k = 64 m + j of window m
  for (uint64_t kb = 0; w0 + kb * W < nblk; kb += kWave) {
    const uint64_t bi = w0 + (kb + (uint64_t)lane) * W;
    const bool valid = bi < nblk;
    uint64_t off = 0, L = 0;
    if (valid) {
      MTBLX_CHK(blk_off + bi, 8);
      MTBLX_CHK(blk_len + bi, 4);
      off = blk_off[bi];
      L = blk_len[bi];
    }
    const bool oob = valid && off + L > data_len;
    // the MFMA path: whole 16-byte aligned chunks around the block inside the buffer, L >= 4
    const bool elig = valid && !oob && L >= 4 && ((base + off) & ~15ull) >= base &&
                      ((base + off + L + 15u) & ~15ull) <= base + data_len;
    const uint64_t em = __ballot(elig);
    uint32_t res = 0;   // lane j: the checksum of block j of the window
    // the lane's block parameters, packed for the cursors' readlanes: steps (23 bits), t, -a0
    const uint32_t bt = (uint32_t)((16u - ((base + off + L) & 15u)) & 15u);
    const uint64_t Lp = L + bt;
    const uint32_t bsteps = (uint32_t)((Lp + kMStep - 1) / kMStep);
    const uint32_t pk = bsteps | (bt << 23) | ((uint32_t)((base + off) & 15u) << 27);
    const int32_t bsb0 = (int32_t)(uint32_t)(Lp - (uint64_t)kMStep * bsteps);

    // issue cursor: the next step to load is at ip (block I, irem steps left, ihd: its first)
    uint64_t irest = em;
    uint32_t irem = 0, ioff = 0, pend = 0;
    const uint8_t* ip = data;
    MBlk I{};
    bool ilive = false, ihd = false;
    auto inext = [&]() {
      ilive = irest != 0;
      if (ilive) {
        I = mblk_lane(data, off, pk, bsb0, __builtin_ctzll(irest));
        irest &= irest - 1;
        irem = I.steps;
        ip = I.p + I.sb0;   // before the block start: the first step's leading lanes are redirected
        ihd = true;
      }
    };
    auto issue = [&]() {
      const uint8_t* p = ip + lane16;
      if (ihd) {   // the block's first step: chunks wholly before the block (zeroed on read)
        asm volatile("");   // a branch, not a select in every step
        if (I.sb0 + lane16 + 16 <= 0) p = I.p + I.a0;
        ihd = false;
      }
      MTBLX_CHK(p, 16);
#if MTBLX_CRC_ABL != 2
      __builtin_amdgcn_global_load_lds(p, (lds_void*)(uintptr_t)(ring_base + ioff), 16, 0, MTBLX_CRC_DMA_AUX);
#else
      (void)p;
#endif
      ioff = (ioff + (uint32_t)kMStep) & kRingMask;
      ip += kMStep;
      if (--irem == 0) inext();
    };
    inext();
    while (ilive && pend < (uint32_t)(kRing - 1)) {
      issue();
      ++pend;
    }

    uint64_t crest = em;
    uint32_t coff = 0;
    v4f c2a = {0.f, 0.f, 0.f, 0.f}, c2b = c2a;   // zero between super-windows
    while (crest) {
      const int cj = __builtin_ctzll(crest);
      crest &= crest - 1;
      const MBlk Cb = mblk_lane(data, off, pk, bsb0, cj);
      uint32_t s = Cb.steps - 1;   // the step's window numbering: steps from the block's end
      int32_t sbc = Cb.sb0;        // block position of the step's chunk 0, while < 4
      uint32_t acc = 0, lo = 0, hi = 0;
      bool first_sw = true;
      for (;;) {
        // two steps of one super-window per iteration when the block has them (MTBLX_CRC_PAIR):
        // their stage-1 chains are independent, so the wave keeps two in flight -- the per-wave
        // step is latency-bound (LDS read -> bit planes -> 8 dependent-pair MFMAs -> f16 stage 2)
        const bool pair = MTBLX_CRC_PAIR && s >= 1u && (s & (uint32_t)(kMSup - 1)) != 0u;
        bool steady = false;
        if (ilive) {   // steady state: kRing - 1 steps stay in flight behind this one
          issue();
          ++pend;
          steady = MTBLX_CRC_STEADY && !pair;   // pend == kRing here: the wait is a constant
        }
        // (the variable wait is a switch: ~25 scalar instructions and 8 branches per step)
        if (steady) wait_steady();
        else wait_vm(pend - (pair ? 2u : 1u));
        const uint32_t t = s & (uint32_t)(kMSup - 1);
        v4i a2lo, a2hi, b2lo, b2hi;
        v4u x, y;
        if (pair) {
          ring_read2(ring_lane + coff, ring_lane + ((coff + (uint32_t)kMStep) & kRingMask), a2_lane + t * 2048u,
                     a2_lane + (t - 1u) * 2048u, x, y, a2lo, a2hi, b2lo, b2hi);
          coff = (coff + 2u * (uint32_t)kMStep) & kRingMask;
          pend -= 2;
          if (ilive) {   // into the slot just read
            issue();
            ++pend;
          }
        } else {
          x = ring_read(ring_lane + coff, a2_lane + t * 2048u, a2lo, a2hi);
          coff = (coff + (uint32_t)kMStep) & kRingMask;
          pend -= 1;
        }
        if (sbc < 4) {   // the block's first bytes (sbc > -1024)
          x = MTBLX_CRC_HEAD2 ? head_chunk_fast(x, sbc + 16 * (int)kx) : head_chunk(x, sbc + 16 * (int)kx);
          sbc += kMStep;
        }
        if (pair && sbc < 4) {
          y = head_chunk(y, sbc + 16 * (int)kx);
          sbc += kMStep;
        }
        const uint32_t sl = pair ? s - 1u : s;   // the iteration's last step
        if (sl == 0) {   // the pad after the block's end: lane (g 3, n 0) holds chunk 63
          asm volatile("");   // a branch, not a select in every step
          if (Cb.t != 0 && lane == 48) {
            if (pair) y = tail_chunk(y, Cb.t);
            else x = tail_chunk(x, Cb.t);
          }
        }
#if MTBLX_CRC_ABL == 1
        acc ^= x.x ^ x.y ^ x.z ^ x.w;
        lo = acc & 15u;
        (void)a2lo;
        (void)a2hi;
        (void)y;
#else
        mfma_step(A, x, a2lo, a2hi, c2a, c2b);
        if (pair) mfma_step(A, y, b2lo, b2hi, c2a, c2b);
        if ((sl & (uint32_t)(kMSup - 1)) == 0u) {
          // super-window done: the parities of the column's raw CRC bits 4g + i (lo) and
          // 16 + 4g + i (hi); with more than one super-window, Horner-combined as a full word with
          // the super-windows before it (nearer the block start)
          asm volatile("");
          lo = par_nib(c2a);
          hi = par_nib(c2b);
          c2a = v4f{0.f, 0.f, 0.f, 0.f};
          c2b = c2a;
          if (Cb.steps > (uint32_t)kMSup) {
            const uint32_t dv = (lo << (4 * g)) | (hi << (16 + 4 * g));
            acc = first_sw ? dv : mul_nib(acc, sInv[0]) ^ dv;
            first_sw = false;
          }
        }
#endif
        if (sl == 0) break;
        s = sl - 1u;
      }
      // block done: column shift, XOR over all 64 lanes, pad removal.  With one super-window the
      // lane holds only its own 8 bits of the column -- nibbles g and 4 + g -- so the column
      // shift takes 2 lookups; after a Horner step it is a full word.
      uint32_t c = Cb.steps <= (uint32_t)kMSup ? sCol[n][g][lo] ^ sCol[n][4 + g][hi] : mul_nib(acc, sCol[n]);
      c = row_xor(c);                                          // over the 16 columns of a row
      uint32_t C = (uint32_t)__builtin_amdgcn_readlane((int)c, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)c, 16) ^
                   (uint32_t)__builtin_amdgcn_readlane((int)c, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)c, 48);
      if (Cb.t) {   // x^(-8t): nibble j looked up by lane j (j < 8) of each row
        const uint32_t j = (uint32_t)lane & 15u;
        const uint32_t v = j < 8u ? sInv[Cb.t][j][(C >> (4 * j)) & 15u] : 0u;
        C = (uint32_t)__builtin_amdgcn_readlane((int)row_xor(v), 0);
      }
      if (lane == cj) res = C ^ 0xFFFFFFFFu;
    }
    // blocks the MFMA path does not take: < 4 bytes, windows past the buffer, unaligned chunks
    // outside it (a block at the very start / end of an unaligned buffer)
    uint64_t todo = __ballot(valid && !elig && !oob);
    while (todo) {
      const int src = __builtin_ctzll(todo);
      todo &= todo - 1;
      const uint64_t bo = (uint64_t)__shfl((long long)off, src, kWave);
      const uint64_t bl = (uint64_t)__shfl((long long)L, src, kWave);
      uint32_t c = 0;
      if (bl >= 4) c = wave_crc32c(data + bo, bl, kTab.byte, lane);
      else if (lane == 0) c = crc_tiny(data + bo, bl);
      c = (uint32_t)__shfl((int)c, 0, kWave);
      if (lane == src) res = c;
    }
    if (valid) crc_store(data + off, off, oob, res, (uint32_t)bi, crc_out, bad, framed);
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
  // the matrix-core kernel unless MTBLX_CRC_KERNEL=lanes (the VALU table kernel, kept for A/B):
  // 0.102 vs 0.120 ms on cfg2 (profiles/r04/crc_mfma)
  const char* kv = getenv("MTBLX_CRC_KERNEL");
  if (!kv || kv[0] != 'l') {
    const int mgrid = mtblx_dev::cu_count();   // persistent: one 16-wave workgroup (160 KiB LDS) per CU
    const uint32_t need = (in->nblk + mtblx_crc::kMWaves - 1u) / mtblx_crc::kMWaves;
    const dim3 g(need < (uint32_t)mgrid ? need : (uint32_t)mgrid), t(mtblx_crc::kMThreads);
    MTBLX_LAUNCH((MTBLX_R(in->data, in->data_len), MTBLX_R(in->blk_off, 8ull * in->nblk),
                  MTBLX_R(in->blk_len, 4ull * in->nblk), MTBLX_R(crc, 4ull * in->nblk), MTBLX_R(bad, in->nblk)),
                 mtblx_crc::k_crc32c_mfma, g, t, 0,
                 reinterpret_cast<hipStream_t>(stream), in->data,
                       in->data_len, in->blk_off, in->blk_len, in->nblk, crc, bad, framed);
    return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
  }
// 98 VGPRs: one 1024-thread workgroup is resident per CU, so a grid of one workgroup per CU runs
// in a single round; 2 per CU measured 0.1256-0.1261 ms against 0.1232 (profiles/r03/final2)
#ifndef MTBLX_CRC_WG_PER_CU
#define MTBLX_CRC_WG_PER_CU 1
#endif
  const int grid = mtblx_dev::cu_count() * MTBLX_CRC_WG_PER_CU;
  const uint32_t wpg = mtblx_crc::kCrcThreads / mtblx_crc::kWave;   // waves (blocks in flight) per workgroup
  const uint32_t need = (in->nblk + wpg - 1u) / wpg;
  const dim3 g(need < (uint32_t)grid ? need : (uint32_t)grid), t(mtblx_crc::kCrcThreads);
  MTBLX_LAUNCH((MTBLX_R(in->data, in->data_len), MTBLX_R(in->blk_off, 8ull * in->nblk),
                MTBLX_R(in->blk_len, 4ull * in->nblk), MTBLX_R(crc, 4ull * in->nblk), MTBLX_R(bad, in->nblk)),
               mtblx_crc::k_crc32c_blocks, g, t, 0,
               reinterpret_cast<hipStream_t>(stream), in->data, in->data_len,
                     in->blk_off, in->blk_len, in->nblk, crc, bad, framed);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
