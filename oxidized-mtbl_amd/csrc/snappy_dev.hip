// snappy_dev.hip — snappy raw decompression of mtbl data blocks on the device (SURVEY.md
// §8(f) f4).
//
// Reference path it replaces: Reader::block decompresses every data block after its checksum
// (/root/reference/src/reader.rs:166-170) via decompress -> snappy_decompress
// (src/compression.rs:57-68, :116-119: snap::raw::Decoder::decompress_vec, crate snap 1.x,
// which is not in /root/reference).  Decompression is format-defined (snappy
// format_description.txt), so the checks below are the host codec's (csrc/snappy_host.cpp)
// and the oracle's (oracle/mtbl_oracle.c oracle_snappy_decompress):
//   preamble  varint32 uncompressed length (unterminated in 5 bytes or > u32: corrupt)
//   literal   tag&3 == 0: len-1 = tag>>2 (< 60) or the next 1..4 LE bytes; the bytes follow
//   copy-1    tag&3 == 1: len = 4 + ((tag>>2)&7), offset = (tag>>5)<<8 | next byte
//   copy-2/4  tag&3 == 2/3: len = 1 + (tag>>2), offset = next 2/4 LE bytes
//   a copy's offset is 1 .. bytes produced so far; nothing may run past the input or the
//   stated length; the output must be exactly the stated length.
//
// Three kernels, chosen per call in mtblx_snappy_decompress_dev (blocks are independent):
//  - k_snappy_quads: outputs <= 4.5 KiB, four blocks per wave, one LDS buffer per block;
//  - k_snappy_lanes: in batches of >= 49 152 blocks, the blocks expanding > 2x, one LANE per
//    block, output streamed to HBM through a per-lane LDS ring and writer waves;
//  - k_snappy_blocks / k_snappy_deferred: larger outputs and what the quads leave, one wave per
//    block, as below.
// One-wave-per-block design:
//  - the block's stored bytes are staged through an LDS window (coalesced 16-byte loads);
//    the output is assembled in LDS (Small: <= 4.5 KiB out, 16 waves per CU; Large: <= 65 KiB
//    out, 2 waves per CU) and streamed to HBM with 16-byte stores; larger outputs are
//    assembled in place in HBM;
//  - the tag stream is a serial chain, parsed with wave-uniform (scalar) arithmetic from LDS;
//    parsed elements are parked one per lane (up to 64);
//  - a RUN is a sequence of elements whose copy sources all lie before the run's first output
//    byte: its bytes are independent, so the wave writes them all at once (lane = output byte,
//    element found by a 6-step binary search over the parked starts).  A copy that reads bytes
//    of the current run (short offsets, overlapping copies) closes the run first.  A run of
//    long elements (>= 64 bytes on average) is instead copied element by element, 4 bytes per
//    lane with aligned dword stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <utility>

#include "bounds.h"
#include "devinfo.h"
#include "mtblx.h"

// timing ablations (wrong output by construction): diagnostic targets only (-DMTBLX_DIAG)
#if (defined(MTBLX_SNAP_ABL_NOSTORE) || defined(MTBLX_LANE_ABL_NOFAR)) && !defined(MTBLX_DIAG)
#error "snappy ablation knobs are diagnostic: build them through a Makefile diagnostic target (-DMTBLX_DIAG)"
#endif
#include "mtblx_host.h"

namespace mtblx_snap {

constexpr int kWave = 64;
// No stream of n bytes decodes to more than 64/3 * n bytes (a 3-byte copy-2 yields at most 64),
// so a longer preamble length can never be met: snap fails on it (Err(Io)) after allocating;
// here it is CORRUPT up front, which also bounds the layout a corrupt preamble can ask for.
constexpr uint64_t kMaxExpand = 22;

template <int W_, int OUT_, int WAVES_>
struct Cfg {
  static constexpr int W = W_, OUT = OUT_, WAVES = WAVES_;
};
using Small = Cfg<4608, 4608, 4>;   // 4 x 9.25 KiB per workgroup, 4 workgroups per CU
using Large = Cfg<8192, 66560, 1>;  // 73 KiB per workgroup, 2 workgroups per CU

template <class C>
struct alignas(16) WaveLds {
  uint8_t win[C::W + 16];   // stored bytes of the block at positions [wstart, wstart + W); 16 B slack
  uint8_t out[C::OUT + 16];
};

__device__ __forceinline__ void lds_fence() { __asm__ volatile("" ::: "memory"); }

#ifdef MTBLX_SNAP_STAMPS
// diagnostic build only: per-phase shader cycles summed over waves (lane 0) --
// [0] total per block [1] inside flush [2] output store [3] elements [4] flushes [5] blocks
// [6] restages [7] 64-byte run steps
__device__ unsigned long long g_snap_dbg[8];
#define SNAP_T() __builtin_amdgcn_s_memtime()
#define SNAP_ADD(k, v) do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_snap_dbg[k], (unsigned long long)(v)); } while (0)
#else
#define SNAP_T() 0ull
#define SNAP_ADD(k, v) do { } while (0)
#endif

__device__ __forceinline__ uint32_t ufl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// A window: the block's stored bytes at block positions [wstart, wstart + W) (wstart = p0
// rounded down to a 16-byte address; bytes outside the block read as 0), loaded as 16-byte
// chunks, up to NCH per lane, all loads in flight before the first LDS store.
template <class C>
struct Window {
  static constexpr int NCH = (C::W / 16 + kWave - 1) / kWave;
  int32_t wstart;
  uint32_t whi, nch;   // block positions [max(wstart, 0), whi) are valid; nch chunks
  uint4 v[NCH];

  __device__ __forceinline__ void load(const uint8_t* s, uint32_t n, uint32_t p0, int lane) {
    const uint32_t r = (uint32_t)(((uintptr_t)s + p0) & 15u);
    wstart = (int32_t)p0 - (int32_t)r;
    const int32_t e = wstart + C::W;
    whi = (e > (int32_t)n) ? n : (uint32_t)e;
    nch = (uint32_t)((int32_t)whi - wstart + 15) / 16u;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const uint32_t c = (uint32_t)lane + (uint32_t)k * kWave;
      const int32_t bp = wstart + 16 * (int32_t)c;
      if (c < nch && bp >= 0 && bp + 16 <= (int32_t)n) {
        v[k] = *reinterpret_cast<const uint4*>(s + bp);
      } else if (c < nch) {
        uint32_t w[4] = {0, 0, 0, 0};
        for (int t = 0; t < 16; ++t) {
          const int32_t q = bp + t;
          if (q >= 0 && q < (int32_t)n) w[t >> 2] |= (uint32_t)s[q] << (8 * (t & 3));
        }
        v[k] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  }
  __device__ __forceinline__ void store(uint8_t* win, int lane) const {
    lds_fence();
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const uint32_t c = (uint32_t)lane + (uint32_t)k * kWave;
      if (c < nch) *reinterpret_cast<uint4*>(win + 16 * c) = v[k];
    }
    lds_fence();
  }
};

// pf: the first window of this block, loaded while the previous block ran; it is stored here
// and refilled with the first window of the wave's next block (s2, n2) right away.
template <class C>
__device__ __forceinline__ void snap_block(WaveLds<C>& S, Window<C>& pf, const uint8_t* __restrict__ s, uint32_t n,
                                           const uint8_t* s2, uint32_t n2, uint8_t* __restrict__ dg, uint32_t cap,
                                           int lane, int32_t* st_out, uint32_t* dec_len) {
  const uint64_t t_blk = SNAP_T();
  uint64_t t_fl = 0, n_el = 0, n_fl = 0, n_rs = 0, n_st = 0;
  (void)t_blk; (void)t_fl; (void)n_el; (void)n_fl; (void)n_rs; (void)n_st;   // debug counters only
  // ---- LDS window over the stored bytes ----
  int32_t wstart = pf.wstart;   // block position of window byte 0 (16-byte aligned in memory; may be < 0)
  uint32_t whi = pf.whi;        // window holds block positions [max(wstart, 0), whi)
  pf.store(S.win, lane);
  pf.load(s2, n2, 0, lane);
  auto restage = [&](uint32_t p0) {
    ++n_rs;
    Window<C> w;
    w.load(s, n, p0, lane);
    w.store(S.win, lane);
    wstart = w.wstart;
    whi = w.whi;
  };
  const uint32_t* w32 = reinterpret_cast<const uint32_t*>(S.win);
  // 8 bytes at block position p (p in the window), wave-uniform.  The words are moved to SGPRs
  // and shifted with 64-bit scalar shifts, so the whole tag parse that follows stays on the
  // scalar unit (a v_alignbit here put it on the VALU: ~100 vector instructions per element).
  auto hdr8 = [&](uint32_t p, uint32_t& lo, uint32_t& hi) {
    const uint32_t wi = (uint32_t)((int32_t)p - wstart), q = wi >> 2, sh = (wi & 3u) * 8u;
    const uint32_t a = ufl(w32[q]), b = ufl(w32[q + 1]), c = ufl(w32[q + 2]);
    const uint64_t ab = ((uint64_t)b << 32 | a) >> sh, bc = ((uint64_t)c << 32 | b) >> sh;
    lo = ufl((uint32_t)ab);
    hi = ufl((uint32_t)bc);
  };

  // ---- preamble: varint32 uncompressed length ----
  uint32_t lo, hi;
  hdr8(0, lo, hi);
  uint64_t want = 0;
  uint32_t pos = 0;
  bool term = false;
  for (uint32_t i = 0; i < 5 && i < n; ++i) {
    const uint32_t byte = (i < 4 ? lo >> (8 * i) : hi) & 0xffu;
    want |= (uint64_t)(byte & 0x7fu) << (7 * i);
    if (!(byte & 0x80u)) {
      term = true;
      pos = i + 1;
      break;
    }
  }
  int32_t st = MTBLX_SNAPPY_OK;
  if (!term || want > 0xFFFFFFFFull || want > kMaxExpand * (uint64_t)n) st = MTBLX_SNAPPY_CORRUPT;
  else if (want > cap) st = MTBLX_SNAPPY_TOO_SMALL;
  const uint32_t W = ufl((uint32_t)want);
  const bool glob = W > (uint32_t)C::OUT;   // assemble in place in HBM

  // ---- element runs ----
  uint32_t e_d = 0xFFFFFFFFu, e_len = 0, e_x = 0;   // lane k: parked element k (start, len | lit<<31, x)
  uint32_t ne = 0, D = 0, d = 0;                    // parked count, run start, output position
  // every byte of the run [D, d), 64 at a time (lane = output byte).  k0 = the element holding
  // the first byte of the step (uniform, carried); the m elements starting inside the step are
  // found with one ballot, and each lane binary-searches only those (none for long elements).
  auto run_bytes = [&](auto* out) {
    const uint32_t T = d - D;
    uint32_t k0 = 0;
    for (uint32_t base = 0; base < T; base += kWave) {
      ++n_st;
      const uint32_t B = D + base;
      const uint32_t i = min(base + (uint32_t)lane, T - 1u), p = D + i;
      const uint32_t m = (uint32_t)__popcll(__ballot(e_d > B && e_d <= B + (kWave - 1)));   // lanes >= ne: ~0
      uint32_t k = k0, ed, el, ex;
      if (m == 0) {
        ed = (uint32_t)__builtin_amdgcn_readlane((int)e_d, (int)k0);
        el = (uint32_t)__builtin_amdgcn_readlane((int)e_len, (int)k0);
        ex = (uint32_t)__builtin_amdgcn_readlane((int)e_x, (int)k0);
      } else {
        for (uint32_t stp = 1u << (31 - __builtin_clz(m)); stp; stp >>= 1) {
          const uint32_t kk = k + stp;
          // the shuffle runs on every lane: a bpermute from a lane masked off by a branch reads garbage
          const uint32_t v = (uint32_t)__shfl((int)e_d, (int)min(kk, 63u), kWave);
          if (kk <= k0 + m && v <= p) k = kk;
        }
        ed = (uint32_t)__shfl((int)e_d, (int)k, kWave);
        el = (uint32_t)__shfl((int)e_len, (int)k, kWave);
        ex = (uint32_t)__shfl((int)e_x, (int)k, kWave);
      }
      k0 += (uint32_t)__popcll(__ballot(e_d > B && e_d <= B + kWave));
      const uint32_t r = p - ed;
      uint8_t v;
      if (el >> 31) {
        v = S.win[ex + r];
      } else {
        const uint32_t rr = ex >= (el & 0x7FFFFFFFu) ? r : r % ex;   // overlapping copy: period `off`
        v = out[ed - ex + rr];
      }
      if (base + (uint32_t)lane < T) out[p] = v;
    }
  };
  auto flush = [&]() {
    if (ne == 0) return;
    const uint64_t t0 = SNAP_T();
    ++n_fl;
    const uint32_t T = d - D;
    lds_fence();
    if (glob) {
      run_bytes(dg);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // this run's HBM bytes before the next run's reads
    } else if (T >= (uint32_t)kWave * ne) {
      // long elements (>= 64 bytes on average): one at a time, 4 bytes per lane with aligned
      // dword stores (literals, and copies that do not overlap themselves); self-overlapping
      // copies byte by byte (their pattern repeats every `off` bytes)
      const uint32_t* o32r = reinterpret_cast<const uint32_t*>(S.out);
      for (uint32_t k = 0; k < ne; ++k) {
        const uint32_t ed = (uint32_t)__builtin_amdgcn_readlane((int)e_d, (int)k);
        const uint32_t el = (uint32_t)__builtin_amdgcn_readlane((int)e_len, (int)k);
        const uint32_t ex = (uint32_t)__builtin_amdgcn_readlane((int)e_x, (int)k);
        const uint32_t len = el & 0x7FFFFFFFu;
        const bool lit = (el >> 31) != 0;
        if (!lit && ex < len) {
          for (uint32_t j = (uint32_t)lane; j < len; j += kWave) S.out[ed + j] = S.out[ed - ex + j % ex];
          continue;
        }
        const uint8_t* src = lit ? S.win : S.out;
        const uint32_t* src32 = lit ? w32 : o32r;
        const uint32_t s0 = lit ? ex : ed - ex;
        const uint32_t h = min((4u - (ed & 3u)) & 3u, len);
        if ((uint32_t)lane < h) S.out[ed + lane] = src[s0 + lane];
        const uint32_t nd = (len - h) / 4u, sp0 = s0 + h, sh = (sp0 & 3u) * 8u;
        uint32_t* o32 = reinterpret_cast<uint32_t*>(S.out + ed + h);
        for (uint32_t j = (uint32_t)lane; j < nd; j += kWave) {
          const uint32_t q = (sp0 >> 2) + j;
          o32[j] = __builtin_amdgcn_alignbit(src32[q + 1], src32[q], sh);
        }
        const uint32_t t0 = h + 4u * nd;
        if ((uint32_t)lane < len - t0) S.out[ed + t0 + lane] = src[s0 + t0 + lane];
      }
    } else {
      run_bytes(S.out);
    }
    lds_fence();
    ne = 0;
    D = d;
    e_d = 0xFFFFFFFFu;
    t_fl += SNAP_T() - t0;
  };
  auto park = [&](uint32_t len, uint32_t lit, uint32_t x) {
    ++n_el;
    if ((uint32_t)lane == ne) {
      e_d = d;
      e_len = len | (lit << 31);
      e_x = x;
    }
    ++ne;
    d += len;
    if (ne == (uint32_t)kWave) flush();
  };

  n = ufl(n);
  while (st == MTBLX_SNAPPY_OK && pos < n) {
    // the parse state is wave-uniform: pin it to SGPRs so the tag decode runs on the scalar
    // unit (left to divergence analysis, it lived in VGPRs: ~100 VALU ops per element)
    pos = ufl(pos);
    d = ufl(d);
    D = ufl(D);
    ne = ufl(ne);
    wstart = (int32_t)ufl((uint32_t)wstart);
    whi = ufl(whi);
    const uint32_t need = min(pos + 5u, n);
    if (need > whi) {
      flush();
      restage(pos);
    }
    hdr8(pos, lo, hi);
    const uint32_t tag = lo & 0xffu, kind = tag & 3u;
    const uint32_t avail = n - pos - 1u;   // stored bytes after the tag
    if (kind == 0) {
      uint64_t len = (tag >> 2) + 1u;
      uint32_t hl = 1;
      if (len > 60) {
        const uint32_t nb = (uint32_t)len - 60u;
        if (avail < nb) { st = MTBLX_SNAPPY_CORRUPT; break; }
        const uint64_t raw = ((uint64_t)hi << 32 | lo) >> 8;
        len = (raw & ((1ull << (8 * nb)) - 1ull)) + 1ull;
        hl += nb;
      }
      const uint32_t src = pos + hl;
      if ((uint64_t)(n - src) < len || (uint64_t)(W - d) < len) { st = MTBLX_SNAPPY_CORRUPT; break; }
      const uint32_t L = (uint32_t)len;
      if (src + L > whi) {   // literal bytes not in the window
        flush();
        if (L <= (uint32_t)C::W - 32u) {
          restage(src);
        } else {   // longer than a window: piece by piece, each a one-literal run
          for (uint32_t o = 0; o < L; o += (uint32_t)C::W - 32u) {
            const uint32_t piece = min((uint32_t)C::W - 32u, L - o);
            restage(src + o);
            park(piece, 1u, (uint32_t)((int32_t)(src + o) - wstart));
            flush();
          }
          pos = src + L;
          continue;
        }
      }
      park(L, 1u, (uint32_t)((int32_t)src - wstart));
      pos = src + L;
      continue;
    }
    uint32_t len, off, hl;
    if (kind == 1) {
      if (avail < 1) { st = MTBLX_SNAPPY_CORRUPT; break; }
      len = 4u + ((tag >> 2) & 7u);
      off = ((tag >> 5) << 8) | ((lo >> 8) & 0xffu);
      hl = 2;
    } else if (kind == 2) {
      if (avail < 2) { st = MTBLX_SNAPPY_CORRUPT; break; }
      len = 1u + (tag >> 2);
      off = (lo >> 8) & 0xffffu;
      hl = 3;
    } else {
      if (avail < 4) { st = MTBLX_SNAPPY_CORRUPT; break; }
      len = 1u + (tag >> 2);
      off = (lo >> 8) | (hi << 24);
      hl = 5;
    }
    if (off == 0 || off > d || W - d < len) { st = MTBLX_SNAPPY_CORRUPT; break; }
    // its source must be written before the step that reads it: before the run (the first
    // bytes of the pattern for an overlapping copy), or -- LDS output, 64-byte steps in order
    // -- at least one step back (off >= 64)
    if (d - off + min(len, off) > D && (glob || off < (uint32_t)kWave)) flush();
    park(len, 0u, off);
    pos += hl;
  }
  if (st == MTBLX_SNAPPY_OK) {
    flush();
    if (d != W) st = MTBLX_SNAPPY_CORRUPT;
  }
  // ---- LDS output -> HBM ----
  [[maybe_unused]] const uint64_t t_out = SNAP_T();
  if (st == MTBLX_SNAPPY_OK && !glob) {
    lds_fence();
    if (((uintptr_t)dg & 15u) == 0) {
      const uint32_t n16 = W / 16u;
      for (uint32_t j = (uint32_t)lane; j < n16; j += kWave)
        reinterpret_cast<uint4*>(dg)[j] = reinterpret_cast<const uint4*>(S.out)[j];
      if ((uint32_t)lane < W - 16u * n16) dg[16u * n16 + lane] = S.out[16u * n16 + lane];
    } else {
      for (uint32_t j = (uint32_t)lane; j < W; j += kWave) dg[j] = S.out[j];
    }
  }
  if (lane == 0) {
    st_out[0] = st;
    if (dec_len) dec_len[0] = st == MTBLX_SNAPPY_OK ? W : 0u;
  }
  lds_fence();
  SNAP_ADD(0, SNAP_T() - t_blk);
  SNAP_ADD(1, t_fl);
  SNAP_ADD(2, SNAP_T() - t_out);
  SNAP_ADD(3, n_el);
  SNAP_ADD(4, n_fl);
  SNAP_ADD(5, 1);
  SNAP_ADD(6, n_rs);
  SNAP_ADD(7, n_st);
}

template <class C>
__global__ void __launch_bounds__(C::WAVES * kWave) k_snappy_blocks(const uint8_t* src, const uint64_t* src_off,
                                                                     const uint32_t* src_len, uint32_t nblk, uint8_t* dst,
                                                                     const uint64_t* dst_off, const uint32_t* dst_len,
                                                                     int32_t* status, uint32_t* dec_len) {
  __shared__ WaveLds<C> S[C::WAVES];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * C::WAVES;
  uint32_t b = blockIdx.x * C::WAVES + wv;
  if (b >= nblk) return;
  const uint8_t* s = src + src_off[b];
  uint32_t n = src_len[b];
  if (n) MTBLX_CHK(s, n);
  Window<C> pf;
  pf.load(s, n, 0, lane);
  for (; b < nblk; b += nw) {
    const uint32_t b2 = b + nw;
    const uint8_t* s2 = b2 < nblk ? src + src_off[b2] : s;
    const uint32_t n2 = b2 < nblk ? src_len[b2] : 0u;
    if (n2) MTBLX_CHK(s2, n2);
    if (dst_len[b]) MTBLX_CHK(dst + dst_off[b], dst_len[b]);
    snap_block<C>(S[wv], pf, s, n, s2, n2, dst + dst_off[b], dst_len[b], lane, status + b,
                  dec_len ? dec_len + b : nullptr);
    s = s2;
    n = n2;
  }
}

// ---- Small outputs (<= 4.5 KiB): four blocks per wave, one LDS buffer per block ----
//
// One wave per block leaves the tag chain to the CU's one scalar unit, shared by all 16 waves
// (~70 scalar instructions per element: profiles/r02/snappy).  Here a wave decodes FOUR blocks
// at once, one per 16-lane group: the parse state is group-uniform and lives in VGPRs, so one
// vector instruction advances four chains, and the 16 lanes of a group then write the element
// (4 bytes per lane, 64 per step) -- element by element, so an overlapping copy reads only
// bytes written before it (its period pattern), and no parking or run flushes are needed.
// The four blocks of a wave start and end together (a "quad").
//
// The loop is latency-bound, so throughput is blocks in flight per CU, and LDS sets that: each
// block has ONE buffer, its output growing from offset 0 and its stored bytes staged
// right-aligned at the end.  An element is written only if its bytes end before the first
// stored byte not yet consumed (checked per element; a stream ordinary compressors write never
// trips it, the output only catches up with the input at the end); a block that would is left
// to the one-wave-per-block kernel (status kDefer, k_snappy_deferred), as is a block whose
// stored bytes or output do not fit.  4.6 KiB per block: 8 waves per CU, twice the blocks of
// separate window + output buffers.
namespace quad {
constexpr int G = 16, NG = kWave / G;
constexpr int OUT = 4608;
constexpr int BUF = 4672;               // output [0, W) and the stored bytes right-aligned below BUF
constexpr int NCH = BUF / 16;           // 16-byte chunks of a buffer
constexpr int NPL = (NCH + G - 1) / G;  // chunks per lane
constexpr int WG_PER_CU = 8;
constexpr int32_t kDefer = 0x7fffffff;  // internal status: the block goes to k_snappy_deferred
constexpr int32_t kLanes = 0x7ffffffe;  // internal status: a compressible block, left to k_snappy_lanes

struct alignas(16) Blk {
  uint8_t b[BUF + 16];   // 16 B slack: 8-byte header reads and 4-byte writes past the end
};

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint32_t v2u __attribute__((ext_vector_type(2), aligned(1)));

struct Meta {
  const uint8_t* s;
  uint8_t* dg;
  uint32_t n, cap;
};

__device__ __forceinline__ Meta load_meta(uint32_t b, uint32_t nblk, const uint8_t* src, const uint64_t* src_off,
                                          const uint32_t* src_len, uint8_t* dst, const uint64_t* dst_off,
                                          const uint32_t* dst_len) {
  Meta m{src, dst, 0u, 0u};
  if (b < nblk) {
    m.s = src + src_off[b];
    m.n = src_len[b];
    m.dg = dst + dst_off[b];
    m.cap = dst_len[b];
    if (m.n) MTBLX_CHK(m.s, m.n);
    if (m.cap) MTBLX_CHK(m.dg, m.cap);
  }
  return m;
}

// j mod off for j < 2^20, off >= 1: float quotient (rcp within an ulp), one correction each way
__device__ __forceinline__ uint32_t umod(uint32_t j, uint32_t off, float rcp) {
  const int32_t q = (int32_t)((float)j * rcp);
  int32_t r = (int32_t)j - q * (int32_t)off;
  r = r < 0 ? r + (int32_t)off : r;
  r = r >= (int32_t)off ? r - (int32_t)off : r;
  return (uint32_t)r;
}

__global__ void __launch_bounds__(kWave) k_snappy_quads(const uint8_t* src, const uint64_t* src_off,
                                                        const uint32_t* src_len, uint32_t nblk, uint8_t* dst,
                                                        const uint64_t* dst_off, const uint32_t* dst_len,
                                                        uint32_t max_out, int32_t* status, uint32_t* dec_len,
                                                        uint32_t lanes_x) {
  __shared__ Blk S[NG];
  const int lane = threadIdx.x, g = lane >> 4, l = lane & 15;
  uint8_t* base = S[g].b;
  const uint32_t nquad = (nblk + NG - 1) / NG, qstride = gridDim.x;
  uint32_t q = blockIdx.x;
  if (q >= nquad) return;
  auto blk_of = [&](uint32_t qq) { return qq * NG + (uint32_t)g; };
  auto meta = [&](uint32_t qq) {
    return load_meta(qq < nquad ? blk_of(qq) : nblk, nblk, src, src_off, src_len, dst, dst_off, dst_len);
  };
  Meta cur = meta(q), m1 = meta(q + qstride);   // offsets of the next quad are loaded a quad ahead

  for (;;) {
    const uint32_t b = blk_of(q);
    const bool on = b < nblk;
    const uint8_t* s = cur.s;
    const uint32_t n = cur.n;
    // stored bytes: stream position p <-> buffer offset p + sh (16-byte chunks from the aligned
    // address at or below position 0, placed so the last one ends at or below BUF)
    const int32_t wb = -(int32_t)((uintptr_t)s & 15u);
    const uint32_t span = n + (uint32_t)(-wb);            // bytes from the aligned start
    const bool fits = on && span <= (uint32_t)BUF;
    const uint32_t nch = fits ? (span + 15u) / 16u : 0u;
    const uint32_t ib = (uint32_t)BUF - 16u * nch;        // buffer offset of chunk 0
    const uint32_t sh = ib - (uint32_t)wb;                // stream position p at buffer offset p + sh
    {
      uint4 v[NPL];
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const int32_t c = l + G * k, bp = wb + 16 * c;
        v[k] = make_uint4(0, 0, 0, 0);
        if ((uint32_t)c < nch && bp >= 0 && bp + 16 <= (int32_t)n) v[k] = *reinterpret_cast<const uint4*>(s + bp);
      }
      // the partial head / tail chunks, one byte per lane
      const int32_t ph = wb + l;
      const uint32_t hb = (fits && ph >= 0 && ph < (int32_t)n) ? s[ph] : 0u;
      const uint32_t ct = nch ? nch - 1u : 0u;
      const int32_t pt = wb + 16 * (int32_t)ct + l;
      const uint32_t tb = (fits && pt >= 0 && pt < (int32_t)n) ? s[pt] : 0u;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const uint32_t c = (uint32_t)(l + G * k);
        if (c < nch) *reinterpret_cast<uint4*>(base + ib + 16 * c) = v[k];
      }
      if (nch) {
        base[ib + l] = (uint8_t)hb;
        base[ib + 16 * ct + l] = (uint8_t)tb;
      }
    }
    const uint32_t qn = q + qstride;
    Meta m2 = meta(qn + qstride);
    auto hdr8 = [&](uint32_t p, uint32_t& lo, uint32_t& hi) {   // stream bytes [p, p + 8), p < n
      const v2u x = *reinterpret_cast<const v2u*>(base + p + sh);
      lo = x.x;
      hi = x.y;
    };
    // ---- preamble ----
    uint32_t lo = 0, hi = 0, pos = 0, W = 0, d = 0;
    int32_t st = MTBLX_SNAPPY_OK;
    if (on) {
      if (fits && n) hdr8(0, lo, hi);
      uint64_t want = 0;
      bool term = false;
      for (uint32_t i = 0; i < 5 && i < n; ++i) {
        const uint32_t byte = (i < 4 ? lo >> (8 * i) : hi) & 0xffu;
        want |= (uint64_t)(byte & 0x7fu) << (7 * i);
        if (!(byte & 0x80u)) {
          term = true;
          pos = i + 1;
          break;
        }
      }
      if (!fits) st = kDefer;
      else if (!term || want > 0xFFFFFFFFull || want > kMaxExpand * (uint64_t)n) st = MTBLX_SNAPPY_CORRUPT;
      else if (want > cur.cap) st = MTBLX_SNAPPY_TOO_SMALL;
      else if (lanes_x && want > (uint64_t)lanes_x * n) st = kLanes;   // expands > lanes_x times
      else if (want > min(max_out, (uint32_t)OUT)) st = kDefer;
      W = (uint32_t)want;
    }
    // ---- elements: decode one per group, then the groups write them together ----
    // Software-pipelined: the next element's 8 header bytes are read before this element's
    // bytes are written, so the two LDS round trips overlap; the decode is select-based (all
    // three tag kinds computed, one picked) so the four groups do not split into branches.
    bool work = on && st == MTBLX_SNAPPY_OK && pos < n;
    if (work) hdr8(pos, lo, hi);
    while (__ballot(work)) {
      const uint32_t tag = lo & 0xffu, kind = tag & 3u, t2 = tag >> 2, avail = n - pos - 1u;
      const uint32_t raw = (lo >> 8) | (hi << 24);   // the 4 bytes after the tag
      // literal: len-1 = t2 (< 60) or the next nb = t2 - 59 bytes
      const bool lg = t2 >= 60u;
      const uint32_t nb = t2 - 59u;
      const uint32_t ext = raw & (nb >= 4u ? 0xFFFFFFFFu : (1u << (8u * (nb & 3u))) - 1u);
      const uint32_t llit = lg ? ext + 1u : t2 + 1u, hlit = lg ? 1u + nb : 1u;
      const bool lbad = lg && (avail < nb || ext == 0xFFFFFFFFu);
      // copies: copy-1 (1 extra byte), copy-2 (2), copy-4 (4)
      const uint32_t lc = kind == 1u ? 4u + (t2 & 7u) : t2 + 1u;
      const uint32_t off = kind == 1u ? ((tag >> 5) << 8) | ((lo >> 8) & 0xffu) : kind == 2u ? raw & 0xffffu : raw;
      const uint32_t need = kind == 1u ? 1u : kind == 2u ? 2u : 4u;
      const bool lit = kind == 0u;
      const uint32_t L0 = lit ? llit : lc, hl = lit ? hlit : need + 1u, sp = pos + hl;
      bool bad = lit ? (lbad || n - sp < L0) : (avail < need || off == 0u || off > d);
      bad = bad || W - d < L0;
      const uint32_t np = lit ? sp + L0 : sp;                   // the next unread stream byte
      const bool over = !bad && d + L0 + 3u > np + sh;          // the writes would reach it
      const uint32_t so = lit ? sp + sh : d - off;               // buffer offset of the source
      const uint32_t P = (!lit && off < L0) ? off : 0xFFFFFFFFu; // overlapping copy: period off
      const float rcp = __builtin_amdgcn_rcpf((float)(P & 0xffffu));
      uint32_t L = 0;
      if (work) {
        if (bad) {
          st = MTBLX_SNAPPY_CORRUPT;
        } else if (over) {
          st = kDefer;
        } else {
          L = L0;
          pos = np;
        }
      }
      const bool go = work && !bad && !over;
      work = go && pos < n;
      if (work) hdr8(pos, lo, hi);   // next element's header, in flight during the writes below
      // write the element: lane l covers bytes [4 l, 4 l + 4) of each 64-byte step (bytes past
      // L land in the next element's space and are overwritten before anything reads them).
      // The dword accesses are misaligned: gfx950 runs those well below the aligned rate, but
      // this loop moves few bytes per cycle and is latency-bound -- aligned reads + a funnel
      // shift and aligned writes with a bytewise lead measured slower (77 -> 59 GB/s).
      for (uint32_t s0 = 0; __ballot(s0 < L); s0 += 4u * G) {
        const uint32_t j = s0 + 4u * (uint32_t)l;
        if (j < L) {
          uint32_t v;
          uint32_t r = P == 0xFFFFFFFFu ? j : umod(j, P, rcp);
          if (r + 4u <= P) {
            v = *reinterpret_cast<const u32u*>(base + so + r);
          } else {
            v = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              v |= (uint32_t)base[so + r] << (8 * t);
              r = r + 1u == P ? 0u : r + 1u;
            }
          }
          *reinterpret_cast<u32u*>(base + d + j) = v;
        }
      }
      d += L;
    }
    if (on && st == MTBLX_SNAPPY_OK && d != W) st = MTBLX_SNAPPY_CORRUPT;

    // ---- output to HBM, statuses ----
    if (on && st == MTBLX_SNAPPY_OK) {
      if (((uintptr_t)cur.dg & 15u) == 0) {
        const uint32_t n16 = W / 16u;
        for (uint32_t c = (uint32_t)l; c < n16; c += G)
          reinterpret_cast<uint4*>(cur.dg)[c] = *reinterpret_cast<const uint4*>(base + 16 * c);
        const uint32_t tb = 16u * n16 + (uint32_t)l;
        if (tb < W) cur.dg[tb] = base[tb];
      } else {
#pragma unroll 1
        for (uint32_t j = (uint32_t)l; j < W; j += G) cur.dg[j] = base[j];
      }
    }
    if (on && l == 0) {
      status[b] = st;
      if (dec_len && st != kDefer && st != kLanes) dec_len[b] = st == MTBLX_SNAPPY_OK ? W : 0u;
    }
    if (qn >= nquad) break;   // wave-uniform
    q = qn;
    cur = m1;
    m1 = m2;
  }
}

// The blocks k_snappy_quads left (status kDefer): one wave per block, the one-wave kernel's
// code (Large config: outputs up to 65 KiB in LDS, larger in place in HBM).  A wave checks 64
// statuses per load and decodes the deferred ones among them.
__global__ void __launch_bounds__(kWave) k_snappy_deferred(const uint8_t* src, const uint64_t* src_off,
                                                           const uint32_t* src_len, uint32_t nblk, uint8_t* dst,
                                                           const uint64_t* dst_off, const uint32_t* dst_len,
                                                           int32_t* status, uint32_t* dec_len) {
  __shared__ WaveLds<Large> SL;
  const int lane = threadIdx.x;
  for (uint32_t b0 = blockIdx.x * kWave; b0 < nblk; b0 += gridDim.x * kWave) {
    const uint32_t bl = b0 + (uint32_t)lane;
    uint64_t m = __ballot(bl < nblk && status[bl] == kDefer);
    while (m) {
      const uint32_t b = b0 + (uint32_t)__builtin_ctzll(m);
      m &= m - 1ull;
      const uint8_t* s = src + src_off[b];
      const uint32_t n = src_len[b];
      if (n) MTBLX_CHK(s, n);
      if (dst_len[b]) MTBLX_CHK(dst + dst_off[b], dst_len[b]);
      Window<Large> pf;
      pf.load(s, n, 0, lane);
      snap_block<Large>(SL, pf, s, n, s, 0u, dst + dst_off[b], dst_len[b], lane, status + b,
                        dec_len ? dec_len + b : nullptr);
    }
  }
}
}  // namespace quad

// ---- Compressible blocks (round 3): one LANE per block, the output streamed to HBM ----
//
// The quad kernel is bound by blocks in flight per CU (LDS holds each block's whole output) and
// by ~1000 cycles of dependent latency per element: on compressible streams (~13 B per element)
// that is 172 GB/s over 100 000 blocks.  Here every lane decodes its own block, so one vector
// instruction advances 64 blocks and every block of the batch is in flight at once:
//  - the element header and short literals come from a 48-byte register window of the stored
//    bytes (two 16-byte chunks in use, the third loaded 16 bytes ahead);
//  - the loop emits one chunk (<= 16 bytes) per iteration into a 256-byte per-lane ring in LDS
//    (64 words, word k of lane t at ring[k][t]: one bank per lane), from which copies with
//    offsets up to kRingOff read their source;
//  - writer waves store the ring to the block's HBM slot (see below), and copies from further
//    back read HBM once those stores are complete;
//  - an overlapping copy (off < 16, off < L) starts with the off-byte period built by two byte
//    permutes per word from a per-offset selector table; its chunk j >= 16 then reads the 16
//    bytes at j - off2, off2 = off * ceil(16 / off) in [16, 16 + off): bytes already written, or
//    the period's bytes before the element, which equal it.
// All state is 32-bit (a block and its output are < 4 GiB).  Checks and statuses are the quad
// kernel's (the oracle's): CORRUPT / TOO_SMALL / OK.  DESIGN.md §4 has the measurements.
namespace lanes {
typedef uint32_t v4u __attribute__((ext_vector_type(4), aligned(1)));
#ifndef MTBLX_LANE_THREADS   // decoding lanes per workgroup (as many writer lanes again); 128: 1.045-1.049 ms vs 1.073-1.074 at 256, 1.091 at 64 (round 6)
#define MTBLX_LANE_THREADS 128
#endif
#ifndef MTBLX_LANE_RING_ALL5   // ring_put writes all five words (no per-word branch)
#define MTBLX_LANE_RING_ALL5 1
#endif
#ifndef MTBLX_LANE_RING_WORDS   // per-lane ring, 4-byte words (a power of two)
#define MTBLX_LANE_RING_WORDS 64
#endif
constexpr int kThreads = MTBLX_LANE_THREADS;
constexpr int kRingWords = MTBLX_LANE_RING_WORDS;
constexpr uint32_t kRingBytes = 4u * kRingWords;
constexpr uint32_t kRingOff = kRingBytes - 16u;   // copies reaching back at most this far read the ring

struct Q4 {
  uint32_t w[4];
};
__device__ __forceinline__ Q4 q4(const v4u x) { return Q4{{x.x, x.y, x.z, x.w}}; }
__device__ __forceinline__ uint32_t alignb(uint32_t hi, uint32_t lo, uint32_t r) {   // ((hi:lo) >> 8r), r < 4
  return __builtin_amdgcn_alignbyte(hi, lo, r);
}
// stored bytes [p, p + 16) of s[0, n) (zero past n): one unaligned load inside, bytes at the end
// Past the end (p + 16 > n) the 16 bytes ENDING at n are loaded -- in bounds whenever n >= 16 --
// and shifted down by r = p + 16 - n bytes: one load and a funnel shift instead of 16 byte
// loads (a wave has some lane near its stream's end in most iterations).
__device__ __forceinline__ Q4 ld16(const uint8_t* s, uint32_t n, uint32_t p) {
  if ((uint64_t)p + 16u <= n) return MTBLX_CHK(s + p, 16), q4(*reinterpret_cast<const v4u*>(s + p));
  Q4 q{{0u, 0u, 0u, 0u}};
  if (n >= 16u) {
    MTBLX_CHK(s + n - 16u, 16);
    const Q4 x = q4(*reinterpret_cast<const v4u*>(s + n - 16u));
    const uint32_t r = p >= n ? 16u : p + 16u - n, rq = r >> 2, rb = r & 3u;   // r in [1, 16]
    uint32_t y[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {   // y[i] = x.w[i + rq] (0 past the end)
      uint32_t v = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if ((uint32_t)(i + 0) + rq == (uint32_t)j) v = x.w[j];
      y[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) q.w[i] = alignb(y[i + 1], y[i], rb);
    return q;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {   // a stream under 16 bytes: clamped loads, no branches
    const uint32_t pk = p + (uint32_t)k < n ? p + (uint32_t)k : 0u;
    const uint32_t v = n ? (uint32_t)s[pk] : 0u;
    q.w[k >> 2] |= ((uint64_t)p + k < n ? v : 0u) << (8 * (k & 3));
  }
  return q;
}
// 16 bytes to dg[o, o + 16), or only dg[o, end) when the slot (cap bytes) ends before o + 16
__device__ __forceinline__ void st16(uint8_t* dg, uint32_t o, const Q4& v, uint32_t end, uint32_t cap) {
#ifdef MTBLX_SNAP_ABL_NOSTORE   // timing ablation only (wrong output): no HBM stores
  return;
#endif
  if ((uint64_t)o + 16u <= cap) {
    MTBLX_CHK(dg + o, 16);
    *reinterpret_cast<v4u*>(dg + o) = v4u{v.w[0], v.w[1], v.w[2], v.w[3]};
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if ((uint64_t)o + k < end) dg[o + k] = (uint8_t)(v.w[k >> 2] >> (8 * (k & 3)));
  }
}
// ring: append cnt (1..16) bytes of v at output position d (the output's last partial word is
// `carry`, merged into the first word written)
__device__ __forceinline__ void ring_put(uint32_t (*R)[kThreads], int t, uint32_t& carry, uint32_t d, const Q4& v,
                                         uint32_t cnt) {
  const uint32_t r = d & 3u, q = d >> 2;
  uint32_t w[5];
  w[0] = (carry & ((1u << (8 * r)) - 1u)) | (v.w[0] << (8 * r));
  w[1] = r ? alignb(v.w[1], v.w[0], 4u - r) : v.w[1];
  w[2] = r ? alignb(v.w[2], v.w[1], 4u - r) : v.w[2];
  w[3] = r ? alignb(v.w[3], v.w[2], 4u - r) : v.w[3];
  w[4] = r ? v.w[3] >> (32u - 8u * r) : 0u;
  const uint32_t e = r + cnt, nw = (e + 3u) >> 2;
#if MTBLX_LANE_RING_ALL5
  // all five words, unconditionally: the words past the chunk hold bytes at or past the new
  // position, which no reader uses before a later put rewrites them (the carry lives in a
  // register), and room() has already waited for the writer to take up to position + 20
  (void)nw;
#pragma unroll
  for (int k = 0; k < 5; ++k) R[(q + k) & (kRingWords - 1)][t] = w[k];
#else
#pragma unroll
  for (int k = 0; k < 5; ++k)
    if ((uint32_t)k < nw) R[(q + k) & (kRingWords - 1)][t] = w[k];
#endif
  const uint32_t c = e >> 2;
  carry = c == 0u ? w[0] : c == 1u ? w[1] : c == 2u ? w[2] : c == 3u ? w[3] : w[4];
}
// ring: output bytes [x, x + 16) (x >= d - 255; bytes at or past d are whatever the ring holds)
__device__ __forceinline__ Q4 ring_get(const uint32_t (*R)[kThreads], int t, uint32_t x) {
  const uint32_t r = x & 3u, q = x >> 2;
  uint32_t w[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) w[k] = R[(q + k) & (kRingWords - 1)][t];
  return Q4{{alignb(w[1], w[0], r), alignb(w[2], w[1], r), alignb(w[3], w[2], r), alignb(w[4], w[3], r)}};
}

// v3: the HBM stores move to WRITER waves.  A vector-memory wait is in issue order over loads and
// stores alike, so every header / literal load a decoding lane waited for also waited for all the
// 16-byte stores it had issued before (an ablation without stores ran 1.63 -> 1.04 ms).  Here the
// workgroup is kThreads decoding lanes + kThreads writer lanes (128 + 128 since round 6), lane
// t + kThreads writing lane t's block: the
// decoder appends to its LDS ring and publishes its position (dpos); the writer copies whole
// 16-byte chunks [fpos, dpos) from the ring to HBM and publishes fpos (issued) and fvis (stores
// completed).  The decoder never overwrites ring words the writer has not taken (it waits on
// fpos), and a copy whose source is beyond the ring (off > kRingOff) waits for fvis to cover its
// whole lines and reads HBM with a cached load (far16).  LDS operations of one wave execute in order, so a position read
// from dpos / fpos covers every ring write / read issued before it.  Short literals come from the
// register window (48 bytes: two in use, the third loaded 16 bytes ahead).
constexpr uint32_t kRun = 0xFFFFFFFFu;   // dend while the decoder runs
constexpr uint32_t kGone = 0xFFFFFFFEu;  // dend after the writer gave up (it won the CAS from kRun)
#ifndef MTBLX_SNAP_WSLEEP
#define MTBLX_SNAP_WSLEEP 8   // writer's idle sleep, x 64 cycles
#endif
constexpr uint64_t kSpinTicks = 2ull * 100000000ull;   // 2 s of s_memrealtime: only a bug waits that long

struct LaneSync {
  uint32_t dpos[kThreads], fpos[kThreads], fvis[kThreads], dend[kThreads];
};

__device__ __forceinline__ uint32_t vld(const uint32_t* p) { return *reinterpret_cast<const volatile uint32_t*>(p); }
__device__ __forceinline__ void vst(uint32_t* p, uint32_t v) { *reinterpret_cast<volatile uint32_t*>(p) = v; }

// 16 bytes at window byte k (k + 16 <= 32) of the window words w[0..7]
__device__ __forceinline__ Q4 win16(const uint32_t (&w)[8], uint32_t k) {
  const uint32_t q = k >> 2, r = k & 3u;
  uint32_t x[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (q + i == (uint32_t)j) v = w[j];
    x[i] = v;
  }
  return Q4{{alignb(x[1], x[0], r), alignb(x[2], x[1], r), alignb(x[3], x[2], r), alignb(x[4], x[3], r)}};
}

__global__ void __launch_bounds__(2 * kThreads) k_snappy_lanes(const uint8_t* src, const uint64_t* src_off,
                                                               const uint32_t* src_len, uint32_t nblk, uint8_t* dst,
                                                               const uint64_t* dst_off, const uint32_t* dst_len,
                                                               int32_t* status, uint32_t* dec_len, int only_marked) {
  __shared__ uint32_t ring[kRingWords][kThreads];
  __shared__ LaneSync Y;
  // period selectors: for offset o < 16 and output word i, byte j = source byte (4 i + j) mod o:
  // psel[o][i] = {v_perm selector over source bytes 0..7, over bytes 8..15, mask of the latter}
  __shared__ uint32_t psel[16][4][3];
  const int tid = threadIdx.x, t = tid & (kThreads - 1);
  const bool writer = tid >= kThreads;
  const uint32_t b = blockIdx.x * kThreads + (uint32_t)t;
  if (tid < 64) {
    const uint32_t o = (uint32_t)tid >> 2, i = (uint32_t)tid & 3u;
    uint32_t lo = 0, hi = 0, mk = 0;
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t m = o ? (4u * i + j) % o : 0u;
      if (m < 8u) lo |= m << (8 * j);
      else {
        hi |= (m - 8u) << (8 * j);
        mk |= 0xFFu << (8 * j);
      }
    }
    psel[o][i][0] = lo;
    psel[o][i][1] = hi;
    psel[o][i][2] = mk;
  }
  if (!writer) {   // the lane's block, decided once (the decoder rewrites status[b] at its end)
    const bool act = b < nblk && (!only_marked || status[b] == quad::kLanes);
    Y.dpos[t] = 0;
    Y.fpos[t] = 0;
    Y.fvis[t] = 0;
    Y.dend[t] = act ? kRun : 0u;
  }
  __syncthreads();
  if (b >= nblk) return;
  uint8_t* dg = b < nblk ? dst + dst_off[b] : dst;

  if (writer) {   // ---- writer lane: ring -> HBM ----
    uint32_t f = 0;
    uint64_t t0 = 0;
    uint32_t spins = 0;
    for (;;) {
      const uint32_t de = vld(&Y.dend[t]);
      const uint32_t dp = de != kRun ? de : vld(&Y.dpos[t]);
      bool moved = false;
      while (f + 16u <= dp) {
        const uint32_t q = f >> 2;
        const v4u x = v4u{ring[q & (kRingWords - 1)][t], ring[(q + 1) & (kRingWords - 1)][t],
                          ring[(q + 2) & (kRingWords - 1)][t], ring[(q + 3) & (kRingWords - 1)][t]};
        *reinterpret_cast<v4u*>(dg + f) = x;
        f += 16u;
        moved = true;
      }
      if (de != kRun) {   // the decoder is done: the last partial chunk, byte by byte
        for (uint32_t p = f; p < de; ++p)
          dg[p] = (uint8_t)(ring[(p >> 2) & (kRingWords - 1)][t] >> (8 * (p & 3u)));
        break;
      }
      if (moved) {
        vst(&Y.fpos[t], f);
        __builtin_amdgcn_s_waitcnt(0);   // stores performed (vmcnt / lgkmcnt 0): far copies may read them
        vst(&Y.fvis[t], f);
        t0 = 0;
      } else {
        // idle: sleep (64 x MTBLX_SNAP_WSLEEP cycles) -- 2, 8 and 20 measured within 1 %: the
        // decoding lanes, not the writers' issue slots, bound the kernel
        __builtin_amdgcn_s_sleep(MTBLX_SNAP_WSLEEP);
        if ((++spins & 15u) == 0u) {
          const uint64_t now = __builtin_amdgcn_s_memrealtime();
          if (t0 == 0) t0 = now;
          // 2 s without a chunk or the end from ITS decoder (which publishes dend as soon as its
          // own block is done, not when the wave is): leave, and say so -- the decoder then
          // reports MTBLX_SNAPPY_TIMEOUT instead of OK for a block whose bytes were not all stored.
          // One CAS on dend decides between giving up and the decoder's end (a plain
          // flag could be set after the decoder had already published OK, truncating silently):
          // if the decoder published first, the loop goes on and stores the block's tail.
          if (now - t0 > kSpinTicks) {
            if (atomicCAS(&Y.dend[t], kRun, kGone) == kRun) break;
            t0 = 0;
          }
        }
      }
    }
    return;
  }

  // ---- decoder lane ----
  if (vld(&Y.dend[t]) == 0u) return;
  const uint8_t* s = src + src_off[b];
  const uint32_t n = src_len[b];
  const uint32_t cap = dst_len[b];
  if (n) MTBLX_CHK(s, n);
  if (cap) MTBLX_CHK(dg, cap);
  uint64_t want = 0;
  uint32_t pos = 0;
  bool term = false;
  for (uint32_t i = 0; i < 5 && i < n; ++i) {   // preamble
    const uint32_t byte = s[i];
    want |= (uint64_t)(byte & 0x7fu) << (7 * i);
    if (!(byte & 0x80u)) {
      term = true;
      pos = i + 1;
      break;
    }
  }
  int32_t st = MTBLX_SNAPPY_OK;
  if (!term || want > 0xFFFFFFFFull || want > kMaxExpand * (uint64_t)n) st = MTBLX_SNAPPY_CORRUPT;
  else if (want > cap) st = MTBLX_SNAPPY_TOO_SMALL;
  const uint32_t W = st == MTBLX_SNAPPY_OK ? (uint32_t)want : 0u;
  uint32_t d = 0, carry = 0;
  bool hang = false;
  // wait until the writer has taken the ring words an append at x overwrites
  // (fseen: the writer's position last read -- it only grows, so most chunks need no LDS read)
  uint32_t fseen = 0;
  auto room = [&](uint32_t x) {
    const uint32_t need = 4u * (x >> 2) + 20u;
    if (need <= fseen + kRingBytes) return;
    fseen = vld(&Y.fpos[t]);
    if (need <= fseen + kRingBytes) return;
    uint64_t t0 = 0;
    uint32_t spins = 0;
    while ((fseen = vld(&Y.fpos[t])) + kRingBytes < need) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 63u) == 0u) {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (t0 == 0) t0 = now;
        if (now - t0 > kSpinTicks) { hang = true; return; }
      }
    }
  };
  // output bytes [x, x + 16) from HBM once the writer's stores cover [x, lim): device-coherent loads
#ifndef MTBLX_LANE_FAR_CACHED
#define MTBLX_LANE_FAR_CACHED 1
#endif
  // (Round 3: a far copy's next chunk -- and a long literal's from HBM -- loaded one iteration
  // ahead measured 346-348 GB/s against 354-355 (profiles/r03/late/snap_pf); not kept.)
  auto far16 = [&](uint32_t x) {
#if MTBLX_LANE_FAR_CACHED
    // Wait until the writer's completed stores cover every 128-byte line the 16 bytes touch, then
    // read them with an ordinary (cacheable) load: a line this CU caches was complete when it
    // was loaded, so no copy of it can be stale.  (Lines shared with a neighbouring block's slot
    // hold that block's LAST bytes, which are never a copy source: sources lie >= 224 bytes
    // before the decoding position.)  Device-coherent dword loads here cost a trip to the L2
    // per dword in ~80 % of the wave's iterations.
    const uintptr_t base = reinterpret_cast<uintptr_t>(dg);
    const uint32_t lim = (uint32_t)((((base + x + 15u) | 127u) + 1u) - base);
#else
    const uint32_t lim = x + 16u;
#endif
    uint64_t t0 = 0;
    uint32_t spins = 0;
    while (vld(&Y.fvis[t]) < lim && !hang) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 63u) == 0u) {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (t0 == 0) t0 = now;
        if (now - t0 > kSpinTicks) hang = true;
      }
    }
    // the load below must not move above the spin: a volatile read orders only other volatile
    // accesses, so a compiler barrier pins it (the hardware issues it after the last spin read
    // returned: it depends on the branch).  The 128-byte bound assumes L1 lines of at most 128
    // bytes (gfx950's vector L1 line is 128 bytes).
    __asm__ volatile("" ::: "memory");
#if MTBLX_LANE_FAR_CACHED
    return q4(*reinterpret_cast<const v4u*>(dg + x));
#else
    const uint8_t* p = dg + x;
    const uint32_t* a = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)3);
    const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3u);
    uint32_t w[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) w[k] = __hip_atomic_load(a + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return Q4{{alignb(w[1], w[0], r), alignb(w[2], w[1], r), alignb(w[3], w[2], r), alignb(w[4], w[3], r)}};
#endif
  };
  // The loop emits ONE chunk (up to 16 bytes) per iteration: the next chunk of the current
  // element, or -- once it is done -- the first chunk of the next one.  An element-per-iteration
  // loop with an inner loop over its chunks made every lane of a wave pay for the wave's longest
  // element in every iteration (~520 vector + ~490 scalar instructions per element, SQ counters).
  // the window: stored bytes [wp, wp + 48) in c0 c1 c2 (c2 loaded 16 bytes ahead)
  uint32_t wp = pos;
  Q4 c0 = ld16(s, n, wp), c1 = ld16(s, n, wp + 16u), c2 = ld16(s, n, wp + 32u);
  uint32_t rem = 0;    // bytes of the current element still to emit
  bool elit = false;   // the current element is a literal: next bytes at stream position es
  uint32_t es = 0;     // literal: stream position; copy: source distance (d - source)
  bool fin = st != MTBLX_SNAPPY_OK || pos >= n;
#ifdef MTBLX_SNAP_STAMPS
  // diagnostic: per wave iteration, whether any lane took each path:
  // [0] iterations [1] decode [2] literal from the window [3] literal from HBM [4] ring copy
  // [5] far copy [6] overlapping copy [7] full window reload
  uint32_t dbg_path = 0;
#define LANE_PATH(k) (dbg_path |= 1u << (k))
#else
#define LANE_PATH(k) ((void)0)
#endif
  // the lane's end (status + dend for its writer), as soon as the LANE is done: the wave keeps
  // looping for its other lanes, possibly for long, and the writer must not wait for them
  bool published = false;
  auto publish = [&]() {
    if (hang) st = MTBLX_SNAPPY_TIMEOUT;   // an internal wait gave up: not CORRUPT
    if (st == MTBLX_SNAPPY_OK && d != W) st = MTBLX_SNAPPY_CORRUPT;
    // the writer's give-up and this end race for dend: whoever moves it off kRun decides
    if (atomicCAS(&Y.dend[t], kRun, st == MTBLX_SNAPPY_OK ? d : 0u) != kRun) st = MTBLX_SNAPPY_TIMEOUT;
    published = true;
  };
  while (__ballot(!fin)) {
#ifdef MTBLX_SNAP_STAMPS
    dbg_path = 0;
#endif
    if (fin) {
      if (!published) publish();
#ifdef MTBLX_SNAP_STAMPS
      goto lane_stamp;
#else
      continue;
#endif
    }
    {
    bool first = false, ov = false;
    uint32_t off = 0;
    if (rem == 0u) {   // ---- decode the next element ----
      if (pos - wp >= 16u) {
        if (pos - wp < 32u) {   // advance 16 bytes, load the next 16 two steps ahead
          c0 = c1;
          c1 = c2;
          wp += 16u;
          c2 = ld16(s, n, wp + 32u);
        } else {                // a long literal jumped past the window
          LANE_PATH(7);
          wp = pos;
          c0 = ld16(s, n, wp);
          c1 = ld16(s, n, wp + 16u);
          c2 = ld16(s, n, wp + 32u);
        }
      }
      const uint32_t k = pos - wp, kq = k >> 2, kr = k & 3u;   // tag + 4 bytes at window byte k < 16
      uint32_t a = c0.w[0], bb = c0.w[1], c = c0.w[2];
      if (kq == 1u) { a = c0.w[1]; bb = c0.w[2]; c = c0.w[3]; }
      if (kq == 2u) { a = c0.w[2]; bb = c0.w[3]; c = c1.w[0]; }
      if (kq == 3u) { a = c0.w[3]; bb = c1.w[0]; c = c1.w[1]; }
      const uint32_t lo = alignb(bb, a, kr), hi = alignb(c, bb, kr);
      const uint32_t tag = lo & 0xffu, kind = tag & 3u, t2 = tag >> 2;
      const uint32_t avail = n - pos - 1u;
      const uint32_t raw = alignb(hi, lo, 1u);   // the 4 bytes after the tag
      const bool lg = t2 >= 60u;
      const uint32_t nb = t2 - 59u;
      const uint32_t ext = raw & (nb >= 4u ? 0xFFFFFFFFu : (1u << (8u * (nb & 3u))) - 1u);
      const uint32_t lc = kind == 1u ? 4u + (t2 & 7u) : t2 + 1u;
      off = kind == 1u ? ((tag >> 5) << 8) | ((lo >> 8) & 0xffu) : kind == 2u ? raw & 0xffffu : raw;
      const uint32_t need = kind == 1u ? 1u : kind == 2u ? 2u : 4u;
      elit = kind == 0u;
      const uint32_t L = elit ? (lg ? ext + 1u : t2 + 1u) : lc;   // ext + 1 wraps only when ext == ~0: bad
      const uint32_t sp = pos + (elit ? (lg ? 1u + nb : 1u) : need + 1u);
      bool bad = elit ? ((lg && (avail < nb || ext == 0xFFFFFFFFu)) || n - sp < L) : (avail < need || off == 0u || off > d);
      bad = bad || W - d < L;
      if (bad) {
        st = MTBLX_SNAPPY_CORRUPT;
        fin = true;
        continue;
      }
      rem = L;
      first = true;
      LANE_PATH(1);
      ov = !elit && off < 16u && off < L;   // overlapping short copy: the period
      es = elit ? sp : off;
      pos = elit ? sp + L : sp;
    }
    // ---- one chunk ----
    const uint32_t cnt = rem < 16u ? rem : 16u;
    Q4 v;
    if (elit) {
      const uint32_t lk = es - wp;   // the literal's window byte (es >= wp while it is in the window)
      if (es >= wp && lk + cnt <= 32u) {   // inside c0 c1 (c2 may still be in flight: not read)
        const bool h = lk >= 16u;
        const uint32_t w8[8] = {h ? c1.w[0] : c0.w[0], h ? c1.w[1] : c0.w[1], h ? c1.w[2] : c0.w[2],
                                h ? c1.w[3] : c0.w[3], h ? 0u : c1.w[0],    h ? 0u : c1.w[1],
                                h ? 0u : c1.w[2],      h ? 0u : c1.w[3]};
        v = win16(w8, lk & 15u);   // bytes past the literal are not used
        LANE_PATH(2);
      } else {
        v = ld16(s, n, es);
        LANE_PATH(3);
      }
      es += 16u;
    } else if (es <= kRingOff) {
      v = ring_get(ring, t, d - es);
      LANE_PATH(4);
    } else {
#ifdef MTBLX_LANE_ABL_NOFAR   // timing ablation only (wrong output): far copies read the ring
      v = ring_get(ring, t, d - 16u);
#else
      v = far16(d - es);
#endif
      LANE_PATH(5);
    }
    if (first && ov) {
      LANE_PATH(6);   // the period of an overlapping copy; later chunks read it back at off2
      const uint32_t o = off;
      Q4 pp;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t pl = __builtin_amdgcn_perm(v.w[1], v.w[0], psel[o][i][0]);
        const uint32_t ph = __builtin_amdgcn_perm(v.w[3], v.w[2], psel[o][i][1]);
        const uint32_t mk = psel[o][i][2];
        pp.w[i] = (pl & ~mk) | (ph & mk);
      }
      v = pp;
      // chunk j >= 16 reads [d + j - off2, +16), off2 = off * ceil(16 / off) in [16, 16 + off):
      // bytes written by earlier chunks, or the period's bytes before the element, which equal it
      es = off * ((16u + off - 1u) / off);
    }
    room(d);
    ring_put(ring, t, carry, d, v, cnt);
    d += cnt;
    rem -= cnt;
    // no fence: a workgroup release would also wait for the window's loads in flight; LDS
    // operations of a wave execute in order, so the ring writes land before this one
    __asm__ volatile("" ::: "memory");
    vst(&Y.dpos[t], d);
    if (hang || (rem == 0u && pos >= n)) fin = true;
    }
#ifdef MTBLX_SNAP_STAMPS
  lane_stamp:
    {
      uint32_t any = dbg_path;   // OR over the wave's lanes
#pragma unroll
      for (int sh = 32; sh >= 1; sh >>= 1) any |= (uint32_t)__shfl_xor((int)any, sh, 64);
      if ((threadIdx.x & 63) == 0) {
        atomicAdd(&g_snap_dbg[0], 1ull);
        for (int k = 1; k < 8; ++k)
          if (any & (1u << k)) atomicAdd(&g_snap_dbg[k], 1ull);
      }
    }
#endif
  }
  if (!published) publish();
  status[b] = st;
  if (dec_len) dec_len[b] = st == MTBLX_SNAPPY_OK ? W : 0u;
}
}  // namespace lanes

// ---- Compressible blocks (round 4): two passes, PARSE then EXECUTE ----
//
// k_snappy_lanes runs the tag parse and the byte moves in one per-lane chain (~390 vector and
// ~390 scalar instructions per 16-byte chunk, divergent element kinds); k_snappy_quads runs them
// in one per-group chain (~1000 cycles of dependent latency per element).  Here:
//  - k_snappy_parse: one LANE per block walks the tag stream only (positions, no data): every
//    element becomes an 8-byte entry {output offset | length << 16, source | literal << 16}
//    (source = the literal's stream position, or the copy's offset) with the quad kernel's checks
//    (corrupt streams, the shared-buffer overrun) -- written into the block's OWN output slot
//    after an 8-byte header {entries, output length} (a compressible block's table is smaller than
//    its output; a block whose table does not fit is left to the one-wave kernel);
//  - k_snappy_exec: four blocks per wave as k_snappy_quads (the stored bytes staged in LDS, the
//    output assembled beside them), but each element comes from the table: 16 entries per group
//    load at once, so an element costs its byte moves (one LDS read -> write round trip) and no
//    header decode; the table is read before the output overwrites it.
namespace two {
using lanes::Q4;
using lanes::ld16;
using lanes::alignb;
constexpr int32_t kTable = 0x7ffffffd;   // internal status: the block's element table is in its slot
constexpr int kParseThreads = 256;
template <typename F, int... Ks>
__device__ __forceinline__ void each_k(F&& f, std::integer_sequence<int, Ks...>) {   // f(K) for K in Ks, unrolled
  (f(std::integral_constant<int, Ks>{}), ...);
}

// 8 stream bytes at window byte k < 16 of the window words (c0, c1)
__device__ __forceinline__ void hdr8w(const Q4& c0, const Q4& c1, uint32_t k, uint32_t& lo, uint32_t& hi) {
  const uint32_t q = k >> 2, r = k & 3u;
  const uint32_t x0 = q == 0u ? c0.w[0] : q == 1u ? c0.w[1] : q == 2u ? c0.w[2] : c0.w[3];
  const uint32_t x1 = q == 0u ? c0.w[1] : q == 1u ? c0.w[2] : q == 2u ? c0.w[3] : c1.w[0];
  const uint32_t x2 = q == 0u ? c0.w[2] : q == 1u ? c0.w[3] : q == 2u ? c1.w[0] : c1.w[1];
  lo = alignb(x1, x0, r);
  hi = alignb(x2, x1, r);
}

__global__ void __launch_bounds__(kParseThreads) k_snappy_parse(const uint8_t* src, const uint64_t* src_off,
                                                                const uint32_t* src_len, uint32_t nblk, uint8_t* dst,
                                                                const uint64_t* dst_off, const uint32_t* dst_len,
                                                                uint32_t max_out, int32_t* status, uint32_t* dec_len) {
  const uint32_t b = blockIdx.x * kParseThreads + threadIdx.x;
  if (b >= nblk || status[b] != quad::kLanes) return;   // the blocks k_snappy_quads marked
  const uint8_t* s = src + src_off[b];
  const uint32_t n = src_len[b], cap = dst_len[b];
  uint8_t* dg = dst + dst_off[b];
  if (n) MTBLX_CHK(s, n);
  if (cap) MTBLX_CHK(dg, cap);
  // the quad kernel already read the preamble: it is valid and fits the slot (else not marked)
  uint64_t want = 0;
  uint32_t pos = 0;
  for (uint32_t i = 0; i < 5 && i < n; ++i) {
    const uint32_t byte = s[i];
    want |= (uint64_t)(byte & 0x7fu) << (7 * i);
    if (!(byte & 0x80u)) {
      pos = i + 1;
      break;
    }
  }
  const uint32_t W = (uint32_t)want;
  // the exec kernel's LDS layout (as k_snappy_quads): stream position p at buffer offset p + sh
  const int32_t wb = -(int32_t)((uintptr_t)s & 15u);
  const uint32_t span = n + (uint32_t)(-wb);
  int32_t st = kTable;
  if (span > (uint32_t)quad::BUF || W > min(max_out, (uint32_t)quad::OUT) || cap < 8u) st = quad::kDefer;
  const uint32_t nch = (span + 15u) / 16u, ib = (uint32_t)quad::BUF - 16u * nch, sh = ib - (uint32_t)wb;
  const uint32_t tcap = cap >= 8u ? (cap - 8u) / 8u : 0u;   // entries the slot holds after the header
  uint32_t d = 0, ne = 0;
  uint32_t wp = pos;
  Q4 c0 = ld16(s, n, wp), c1 = ld16(s, n, wp + 16u), c2 = ld16(s, n, wp + 32u);
  bool work = st == kTable && pos < n;
  while (work) {
    uint32_t lo, hi;
    hdr8w(c0, c1, pos - wp, lo, hi);
    const uint32_t tag = lo & 0xffu, kind = tag & 3u, t2 = tag >> 2, avail = n - pos - 1u;
    const uint32_t raw = (lo >> 8) | (hi << 24);
    const bool lg = t2 >= 60u;
    const uint32_t nb = t2 - 59u;
    const uint32_t ext = raw & (nb >= 4u ? 0xFFFFFFFFu : (1u << (8u * (nb & 3u))) - 1u);
    const uint32_t llit = lg ? ext + 1u : t2 + 1u, hlit = lg ? 1u + nb : 1u;
    const bool lbad = lg && (avail < nb || ext == 0xFFFFFFFFu);
    const uint32_t lc = kind == 1u ? 4u + (t2 & 7u) : t2 + 1u;
    const uint32_t off = kind == 1u ? ((tag >> 5) << 8) | ((lo >> 8) & 0xffu) : kind == 2u ? raw & 0xffffu : raw;
    const uint32_t need = kind == 1u ? 1u : kind == 2u ? 2u : 4u;
    const bool lit = kind == 0u;
    const uint32_t L0 = lit ? llit : lc, hl = lit ? hlit : need + 1u, sp = pos + hl;
    bool bad = lit ? (lbad || n - sp < L0) : (avail < need || off == 0u || off > d);
    bad = bad || W - d < L0;
    const uint32_t np = lit ? sp + L0 : sp;
    if (bad) {
      st = MTBLX_SNAPPY_CORRUPT;
      break;
    }
    if (d + L0 + 3u > np + sh || ne >= tcap) {   // the exec kernel's writes would reach unread bytes / table full
      st = quad::kDefer;
      break;
    }
    const uint32_t e0 = d | (L0 << 16), e1 = (lit ? sp : off) | (lit ? 0x10000u : 0u);
    *reinterpret_cast<uint2*>(dg + 8u + 8u * ne) = make_uint2(e0, e1);
    ++ne;
    d += L0;
    pos = np;
    work = pos < n;
    // keep pos - wp < 16: shift the window (the next chunk loaded 32 bytes ahead), or reload it
    // after a long literal
    if (work) {
      if (pos - wp >= 48u) {
        wp = pos;
        c0 = ld16(s, n, wp);
        c1 = ld16(s, n, wp + 16u);
        c2 = ld16(s, n, wp + 32u);
      } else {
        while (pos - wp >= 16u) {
          c0 = c1;
          c1 = c2;
          c2 = ld16(s, n, wp + 48u);
          wp += 16u;
        }
      }
    }
  }
  if (st == kTable && d != W) st = MTBLX_SNAPPY_CORRUPT;
  if (st == kTable) *reinterpret_cast<uint2*>(dg) = make_uint2(ne, W);
  status[b] = st;   // kTable (to k_snappy_exec), kDefer (to k_snappy_deferred) or CORRUPT (final)
  if (st == MTBLX_SNAPPY_CORRUPT && dec_len) dec_len[b] = 0u;
}

__global__ void __launch_bounds__(kWave) k_snappy_exec(const uint8_t* src, const uint64_t* src_off,
                                                       const uint32_t* src_len, uint32_t nblk, uint8_t* dst,
                                                       const uint64_t* dst_off, int32_t* status, uint32_t* dec_len) {
  using namespace quad;
  __shared__ Blk S[NG];
  const int lane = threadIdx.x, g = lane >> 4, l = lane & 15;
  uint8_t* base = S[g].b;
  const uint32_t nquad = (nblk + NG - 1) / NG;
  for (uint32_t q = blockIdx.x; q < nquad; q += gridDim.x) {
    const uint32_t b = q * NG + (uint32_t)g;
    const bool on = b < nblk && status[b] == kTable;
    if (__ballot(on) == 0ull) continue;
    const uint8_t* s = on ? src + src_off[b] : src;
    const uint32_t n = on ? src_len[b] : 0u;
    uint8_t* dg = on ? dst + dst_off[b] : dst;
    if (n) MTBLX_CHK(s, n);
    const int32_t wb = -(int32_t)((uintptr_t)s & 15u);
    const uint32_t span = n + (uint32_t)(-wb);
    const uint32_t nch = on ? (span + 15u) / 16u : 0u;
    const uint32_t ib = (uint32_t)BUF - 16u * nch, sh = ib - (uint32_t)wb;
    {   // stage the stored bytes right-aligned (as k_snappy_quads)
      uint4 v[NPL];
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const int32_t c = l + G * k, bp = wb + 16 * c;
        v[k] = make_uint4(0, 0, 0, 0);
        if ((uint32_t)c < nch && bp >= 0 && bp + 16 <= (int32_t)n) v[k] = *reinterpret_cast<const uint4*>(s + bp);
      }
      const int32_t ph = wb + l;
      const uint32_t hb = (on && ph >= 0 && ph < (int32_t)n) ? s[ph] : 0u;
      const uint32_t ct = nch ? nch - 1u : 0u;
      const int32_t pt = wb + 16 * (int32_t)ct + l;
      const uint32_t tb = (on && pt >= 0 && pt < (int32_t)n) ? s[pt] : 0u;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const uint32_t c = (uint32_t)(l + G * k);
        if (c < nch) *reinterpret_cast<uint4*>(base + ib + 16 * c) = v[k];
      }
      if (nch) {
        base[ib + l] = (uint8_t)hb;
        base[ib + 16 * ct + l] = (uint8_t)tb;
      }
    }
    uint2 hd = make_uint2(0u, 0u);
    if (on) hd = *reinterpret_cast<const uint2*>(dg);
    const uint32_t ne = hd.x, W = hd.y;
    const uint2* tab = reinterpret_cast<const uint2*>(dg + 8);
    // entries 16 at a time: lane l holds entry e0 + l; the next batch is loaded a batch ahead
    uint2 cur = make_uint2(0u, 0u), nxt = make_uint2(0u, 0u);
    if ((uint32_t)l < ne) cur = tab[l];
    if ((uint32_t)l + 16u < ne) nxt = tab[16 + l];
    // element K of the batch: broadcast from lane K of each group's row by DPP row_newbcast (a
    // VALU modifier; a __shfl here is two LDS round trips per element)
    auto elem = [&](auto kc, const uint2 bat, uint32_t e0) {
      constexpr int K = decltype(kc)::value;
      const uint32_t x0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)bat.x, 0x150 + K, 0xf, 0xf, false);
      const uint32_t x1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)bat.y, 0x150 + K, 0xf, 0xf, false);
      const bool act = e0 + (uint32_t)K < ne;
      if (__ballot(act) == 0ull) return;
      const uint32_t d = x0 & 0xffffu, L = act ? x0 >> 16 : 0u, v = x1 & 0xffffu;
      const bool lit = (x1 >> 16) != 0u;
      const uint32_t so = lit ? v + sh : d - v;
      const uint32_t P = (!lit && v < L) ? v : 0xFFFFFFFFu;   // overlapping copy: period v
      const float rcp = __builtin_amdgcn_rcpf((float)(P & 0xffffu));
      for (uint32_t s0 = 0; __ballot(s0 < L); s0 += 4u * G) {
        const uint32_t j = s0 + 4u * (uint32_t)l;
        if (j < L) {
          uint32_t w;
          uint32_t r = P == 0xFFFFFFFFu ? j : umod(j, P, rcp);
          if (r + 4u <= P) {
            w = *reinterpret_cast<const u32u*>(base + so + r);
          } else {
            w = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              w |= (uint32_t)base[so + r] << (8 * t);
              r = r + 1u == P ? 0u : r + 1u;
            }
          }
          *reinterpret_cast<u32u*>(base + d + j) = w;
        }
      }
    };
    for (uint32_t e0 = 0; __ballot(e0 < ne); e0 += 16u) {
      const uint2 bat = cur;
      cur = nxt;
      if (e0 + 32u + (uint32_t)l < ne) nxt = tab[e0 + 32u + l];
      each_k([&](auto kc) { elem(kc, bat, e0); }, std::make_integer_sequence<int, 16>{});
    }
    // output to HBM (the table in the slot is read: every load above has returned), statuses
    if (on) {
      if (((uintptr_t)dg & 15u) == 0) {
        const uint32_t n16 = W / 16u;
        for (uint32_t c = (uint32_t)l; c < n16; c += G)
          reinterpret_cast<uint4*>(dg)[c] = *reinterpret_cast<const uint4*>(base + 16 * c);
        const uint32_t tb = 16u * n16 + (uint32_t)l;
        if (tb < W) dg[tb] = base[tb];
      } else {
#pragma unroll 1
        for (uint32_t j = (uint32_t)l; j < W; j += G) dg[j] = base[j];
      }
      if (l == 0) {
        status[b] = MTBLX_SNAPPY_OK;
        if (dec_len) dec_len[b] = W;
      }
    }
  }
}
}  // namespace two

// ---- Compressible blocks (round 6): one WAVE per block, the element chain found in parallel ----
//
// k_snappy_lanes pays the whole tag chain of a block serially on one lane (~300 vector and ~250
// scalar instructions per 16-byte chunk, 65 % of wave time waiting, SQ counters in
// profiles/r06/snappy).  Its copies do not need that order: on the bench's compressible stream a
// block's 316 elements (199 copies) form a dependency DAG only ~25 levels deep (a copy depends on
// the elements that wrote its source bytes).  Here a wave takes one block, everything in LDS:
//  1. parse: J(p) = p + size of the element whose tag is at stream position p, for EVERY p; the
//     element starts are the positions reachable from the preamble end, marked by pointer doubling
//     (mark J_k(p) for marked p, J_(k+1) = J_k o J_k; ceil(log2(n + 2)) rounds) -- position n ends
//     the chain, n + 1 is an overshoot (a header or literal past the end: corrupt);
//  2. the starts compacted in stream order, every element decoded at once, output offsets by a
//     wave prefix sum; the checks of the serial decoder per element (header bytes present,
//     literal inside the stream, copy offset in 1 .. bytes before it, output not past the stated
//     length) and the total, so CORRUPT exactly where the serial decode is;
//  3. literals written at once; then copies in ROUNDS: a copy runs once every byte it reads is
//     written (a bitmap of written output bytes), ~25 rounds instead of 199 steps;
//  4. the output to HBM with 16-byte stores.
// Blocks whose stream or output exceed the LDS buffers, or with more than 512 elements, are left
// to k_snappy_deferred (status kDefer).
namespace wavep {
constexpr int IN = 2304;                        // stored bytes (compressible: W > 2n, W <= OUT)
constexpr int OUT = 4608;                       // output bytes
constexpr int K = 8;                            // elements per lane
constexpr int MAXE = K * kWave;                 // 512
constexpr int NP = IN + 2;                      // chain positions: stream, n (end), n + 1 (overshoot)
[[maybe_unused]] constexpr int PPL = (NP + kWave - 1) / kWave;   // positions per lane (contiguous)
#ifndef MTBLX_WAVEP_WG_PER_CU
#define MTBLX_WAVEP_WG_PER_CU 12
#endif

struct alignas(16) Lds {
  uint8_t in[IN + 32];          // the stored stream; slack: 8-byte header reads past its end
  uint8_t out[OUT + 64];        // the output; during the parse J_k as u16 per position
  uint16_t jb[NP + 2];          // element starts after the parse (epos)
  uint32_t mark[NP / 32 + 2];   // reachable chain positions
  uint32_t rdy[OUT / 32 + 4];   // output bytes written
  uint32_t psel[16][4][3];      // period selectors of short overlapping copies (as k_snappy_lanes)
};

typedef uint32_t v4w __attribute__((ext_vector_type(4)));
typedef uint32_t v4g __attribute__((ext_vector_type(4), aligned(1)));   // unaligned global loads

// 16 bytes of LDS at any byte address a (5 aligned dwords joined)
__device__ __forceinline__ v4w lds16(const uint8_t* base, uint32_t a) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(base + (a & ~3u));
  const uint32_t r = a & 3u;
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
  return v4w{__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r),
             __builtin_amdgcn_alignbyte(w3, w2, r), __builtin_amdgcn_alignbyte(w4, w3, r)};
}
__device__ __forceinline__ uint32_t wsel(const v4w& v, uint32_t i) {   // dword i (0..4, 4 = 0)
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : i == 3 ? v.w : 0u;
}
// bytes [0, cnt) of v (cnt <= 16) to LDS address a, exactly: bytes up to the first dword boundary,
// whole dwords, trailing bytes (no read-modify-write: neighbouring bytes may belong to other lanes)
__device__ __forceinline__ void lds_put(uint8_t* base, uint32_t a, const v4w& v, uint32_t cnt) {
  const uint32_t h = (4u - (a & 3u)) & 3u;   // head bytes
  const uint32_t hb = h < cnt ? h : cnt;
  for (uint32_t i = 0; i < hb; ++i) base[a + i] = (uint8_t)(wsel(v, i >> 2) >> (8 * (i & 3u)));
  // dword k of the rest starts at byte hb + 4k of v
  const uint32_t nw = (cnt - hb) >> 2, sh = hb & 3u, q = hb >> 2;
  uint32_t* wd = reinterpret_cast<uint32_t*>(base + a + hb);
  for (uint32_t k = 0; k < nw; ++k)
    wd[k] = __builtin_amdgcn_alignbyte(wsel(v, q + k + 1), wsel(v, q + k), sh);
  for (uint32_t i = hb + 4 * nw; i < cnt; ++i) base[a + i] = (uint8_t)(wsel(v, i >> 2) >> (8 * (i & 3u)));
}
// output bytes [a, b) written: bits in rdy
__device__ __forceinline__ void set_rdy(uint32_t* rdy, uint32_t a, uint32_t b) {
  for (uint32_t w = a >> 5; a < b && w <= (b - 1) >> 5; ++w) {
    const uint32_t lo = w == (a >> 5) ? (a & 31u) : 0u, hi = w == ((b - 1) >> 5) ? ((b - 1) & 31u) : 31u;
    const uint32_t m = (hi == 31u ? 0xFFFFFFFFu : ((1u << (hi + 1u)) - 1u)) & ~((1u << lo) - 1u);
    atomicOr(rdy + w, m);
  }
}
__device__ __forceinline__ bool all_rdy(const uint32_t* rdy, uint32_t a, uint32_t b) {   // [a, b), b - a <= 64
  bool ok = true;
  for (uint32_t w = a >> 5; a < b && w <= (b - 1) >> 5; ++w) {
    const uint32_t lo = w == (a >> 5) ? (a & 31u) : 0u, hi = w == ((b - 1) >> 5) ? ((b - 1) & 31u) : 31u;
    const uint32_t m = (hi == 31u ? 0xFFFFFFFFu : ((1u << (hi + 1u)) - 1u)) & ~((1u << lo) - 1u);
    ok = ok && (rdy[w] & m) == m;
  }
  return ok;
}
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, int lane, uint32_t& total) {
  uint32_t v = x;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)v, d, kWave);
    if (lane >= d) v += y;
  }
  total = (uint32_t)__shfl((int)v, kWave - 1, kWave);
  return v - x;
}

constexpr uint32_t kRounds = 10;   // pointer-doubling rounds: chains of up to 2^10 elements (more: kDefer)
// J(p): the position after the element whose tag is at p (n + 1: past the stream's end)
__device__ __forceinline__ uint32_t jnext(const uint8_t* in, uint32_t p, uint32_t pos0, uint32_t n) {
  if (p < pos0 || p >= n) return p;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(in + (p & ~3u));
  const uint32_t lo = __builtin_amdgcn_alignbyte(w[1], w[0], p & 3u), hi = __builtin_amdgcn_alignbyte(w[2], w[1], p & 3u);
  const uint32_t tag = lo & 0xffu, kind = tag & 3u, t2 = tag >> 2;
  const uint32_t raw = __builtin_amdgcn_alignbyte(hi, lo, 1u);
  uint64_t sz;
  if (kind == 0u) {
    const uint32_t nb = t2 >= 60u ? t2 - 59u : 0u;
    const uint32_t ext = raw & (nb >= 4u ? 0xFFFFFFFFu : (1u << (8u * nb)) - 1u);
    sz = t2 >= 60u ? 2ull + nb + (uint64_t)ext : 2ull + t2;
  } else {
    sz = kind == 1u ? 2u : kind == 2u ? 3u : 5u;
  }
  return (uint64_t)p + sz > (uint64_t)n ? n + 1u : p + (uint32_t)sz;
}

__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(3))) k_snappy_waves(const uint8_t* src, const uint64_t* src_off,
                                                        const uint32_t* src_len, uint32_t nblk, uint8_t* dst,
                                                        const uint64_t* dst_off, const uint32_t* dst_len,
                                                        int32_t* status, uint32_t* dec_len, int only_marked) {
  __shared__ Lds S;
  const int lane = threadIdx.x;
  {   // period selectors: offset o < 16, output dword i, byte j = source byte (4 i + j) mod o
    const uint32_t o = (uint32_t)lane >> 2, i = (uint32_t)lane & 3u;
    uint32_t lo = 0, hi = 0, mk = 0;
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t m = o ? (4u * i + j) % o : 0u;
      if (m < 8u) lo |= m << (8 * j);
      else {
        hi |= (m - 8u) << (8 * j);
        mk |= 0xFFu << (8 * j);
      }
    }
    S.psel[o][i][0] = lo;
    S.psel[o][i][1] = hi;
    S.psel[o][i][2] = mk;
  }
  uint16_t* J = reinterpret_cast<uint16_t*>(S.out);
  uint64_t wdbg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    MTBLX_CHK(status + b, 4);
    if (only_marked && status[b] != quad::kLanes) continue;   // uniform
    const uint8_t* s = src + src_off[b];
    const uint32_t n = src_len[b];
    uint8_t* dg = dst + dst_off[b];
    const uint32_t cap = dst_len[b];
    if (n) MTBLX_CHK(s, n);
    if (cap) MTBLX_CHK(dg, cap);
    // ---- preamble (the quad kernel's checks) ----
    uint64_t want = 0;
    uint32_t pos0 = 0;
    bool term = false;
    for (uint32_t i = 0; i < 5 && i < n; ++i) {
      const uint32_t byte = s[i];
      want |= (uint64_t)(byte & 0x7fu) << (7 * i);
      if (!(byte & 0x80u)) {
        term = true;
        pos0 = i + 1;
        break;
      }
    }
    int32_t st = MTBLX_SNAPPY_OK;
    if (!term || want > 0xFFFFFFFFull || want > kMaxExpand * (uint64_t)n) st = MTBLX_SNAPPY_CORRUPT;
    else if (want > cap) st = MTBLX_SNAPPY_TOO_SMALL;
    else if (n > (uint32_t)IN || want > (uint64_t)OUT) st = quad::kDefer;
    const uint32_t W = (uint32_t)want;
    uint64_t tw = SNAP_T();   // diagnostic stamps (snapstamps build): per-phase cycles, summed per wave
    auto stamp = [&](int k) { const uint64_t t = SNAP_T(); wdbg[k] += t - tw; tw = t; };
    wdbg[5] += 1;
    if (st == MTBLX_SNAPPY_OK) {
      // ---- the stream into LDS (16-byte chunks; zeros past n) ----
      for (uint32_t c = (uint32_t)lane; 16u * c < n + 16u; c += kWave) {
        const uint32_t p = 16u * c;
        v4w v = {0u, 0u, 0u, 0u};
        if (p + 16u <= n) {
          MTBLX_CHK(s + p, 16);
          v = *reinterpret_cast<const v4g*>(s + p);
        } else if (p < n) {
          uint32_t w[4] = {0u, 0u, 0u, 0u};
          for (uint32_t t = 0; p + t < n; ++t) w[t >> 2] |= (uint32_t)s[p + t] << (8 * (t & 3u));
          v = v4w{w[0], w[1], w[2], w[3]};
        }
        *reinterpret_cast<v4w*>(S.in + p) = v;
      }
      stamp(0);
      // ---- 1. the chain: J(p) for every position (lane + 64 i), reachability by doubling ----
      const uint32_t np = n + 2u;
      uint16_t* A = J;        // J_k
      uint16_t* B = S.jb;     // J_(k+1)
      for (uint32_t p = (uint32_t)lane; p < np; p += kWave) A[p] = (uint16_t)jnext(S.in, p, pos0, n);
      for (uint32_t w = (uint32_t)lane; w < np / 32u + 2u; w += kWave) S.mark[w] = 0u;
      if (lane == 0) atomicOr(&S.mark[pos0 >> 5], 1u << (pos0 & 31u));
      for (uint32_t r = 0; r < kRounds; ++r) {
#pragma unroll 4
        for (uint32_t p = (uint32_t)lane; p < np; p += kWave) {
          const uint32_t j = A[p];
          if ((S.mark[p >> 5] >> (p & 31u)) & 1u) atomicOr(&S.mark[j >> 5], 1u << (j & 31u));
          B[p] = A[j];
        }
        uint16_t* t = A;
        A = B;
        B = t;
      }
      const bool ends = (S.mark[n >> 5] >> (n & 31u)) & 1u, over = (S.mark[(n + 1u) >> 5] >> ((n + 1u) & 31u)) & 1u;
      if (over) st = MTBLX_SNAPPY_CORRUPT;
      else if (!ends) st = quad::kDefer;   // a chain of more than 2^kRounds elements
      stamp(1);
      // ---- 2. element records in stream order (row i = positions 64 i .. 64 i + 63) ----
      uint32_t* erec = reinterpret_cast<uint32_t*>(S.jb);   // [e] = d | L << 16, [MAXE + e] = x | lit << 31
      uint32_t m = 0, dsum = 0;
      bool bad = false;
      for (uint32_t row = 0; st == MTBLX_SNAPPY_OK && 64u * row < n; ++row) {
        const uint32_t p = 64u * row + (uint32_t)lane;
        const bool isel = p >= pos0 && p < n && ((S.mark[p >> 5] >> (p & 31u)) & 1u);
        uint32_t L = 0, x = 0;
        bool lit = false, eb = false;
        if (isel) {
          const uint32_t* w = reinterpret_cast<const uint32_t*>(S.in + (p & ~3u));
          const uint32_t lo = __builtin_amdgcn_alignbyte(w[1], w[0], p & 3u), hi = __builtin_amdgcn_alignbyte(w[2], w[1], p & 3u);
          const uint32_t tag = lo & 0xffu, kind = tag & 3u, t2 = tag >> 2, avail = n - p - 1u;
          const uint32_t raw = __builtin_amdgcn_alignbyte(hi, lo, 1u);
          lit = kind == 0u;
          if (lit) {
            const bool lg = t2 >= 60u;
            const uint32_t nb = lg ? t2 - 59u : 0u;
            const uint32_t ext = raw & (nb >= 4u ? 0xFFFFFFFFu : (1u << (8u * nb)) - 1u);
            const uint32_t sp = p + 1u + nb;
            L = lg ? ext + 1u : t2 + 1u;
            eb = (lg && (avail < nb || ext == 0xFFFFFFFFu)) || sp > n || n - sp < L;
            x = sp;
          } else {
            const uint32_t need = kind == 1u ? 1u : kind == 2u ? 2u : 4u;
            L = kind == 1u ? 4u + (t2 & 7u) : t2 + 1u;
            x = kind == 1u ? ((tag >> 5) << 8) | ((lo >> 8) & 0xffu) : kind == 2u ? raw & 0xffffu : raw;
            eb = avail < need || x == 0u;
          }
        }
        const uint64_t mk = __ballot(isel);
        const uint32_t e = m + (uint32_t)__builtin_popcountll(mk & ((1ull << lane) - 1ull));
        const uint32_t Lc = L > 0xFFFFu ? 0xFFFFu : L;   // a bad element's length: only the sum must not wrap
        uint32_t tot = 0;
        const uint32_t d = dsum + wave_excl_scan(isel ? Lc : 0u, lane, tot);
        if (isel) {
          eb = eb || (!lit && x > d) || d > W || W - d < L;
          bad = bad || eb;
          if (e < (uint32_t)MAXE) {
            erec[e] = d | (Lc << 16);
            erec[MAXE + e] = (x & 0xFFFFu) | (lit ? 0x80000000u : 0u);
          }
        }
        m += (uint32_t)__builtin_popcountll(mk);
        dsum += tot;
      }
      if (st == MTBLX_SNAPPY_OK) {
        if (__ballot(bad) != 0ull || dsum != W) st = MTBLX_SNAPPY_CORRUPT;
        else if (m > (uint32_t)MAXE) st = quad::kDefer;
      }
      if (st == MTBLX_SNAPPY_OK) {
        stamp(2);
        // ---- 3. literals, then copies in rounds (element e on lane e mod 64) ----
        for (uint32_t w = (uint32_t)lane; w < W / 32u + 2u; w += kWave) S.rdy[w] = 0u;
        uint32_t pend = 0;   // bit k: element lane + 64 k is a copy not yet written
        for (uint32_t k = 0, e = (uint32_t)lane; e < m; ++k, e += kWave) {
          const uint32_t r0 = erec[e], r1 = erec[MAXE + e];
          const uint32_t d = r0 & 0xFFFFu, L = r0 >> 16;
          if (r1 & 0x80000000u) {
            const uint32_t sp = r1 & 0xFFFFu;
            for (uint32_t c = 0; c < L; c += 16u) lds_put(S.out, d + c, lds16(S.in, sp + c), L - c < 16u ? L - c : 16u);
            set_rdy(S.rdy, d, d + L);
          } else {
            pend |= 1u << k;
          }
        }
        stamp(3);
        for (uint32_t guard = 0; __ballot(pend != 0u) != 0ull && guard <= (uint32_t)MAXE; ++guard) {
          wdbg[6] += 1;
          uint32_t go = 0;
          for (uint32_t q = pend; q; q &= q - 1u) {
            const uint32_t k = (uint32_t)__builtin_ctz(q), e = (uint32_t)lane + (uint32_t)kWave * k;
            const uint32_t r0 = erec[e], off = erec[MAXE + e] & 0xFFFFu;
            const uint32_t d = r0 & 0xFFFFu, L = r0 >> 16;
            if (all_rdy(S.rdy, d - off, d - off + (L < off ? L : off))) go |= 1u << k;
          }
          for (uint32_t q = go; q; q &= q - 1u) {
            const uint32_t k = (uint32_t)__builtin_ctz(q), e = (uint32_t)lane + (uint32_t)kWave * k;
            const uint32_t r0 = erec[e], off = erec[MAXE + e] & 0xFFFFu;
            const uint32_t d = r0 & 0xFFFFu, L = r0 >> 16;
            if (off < 16u && off < L) {   // the period: chunk 0 by byte permutes, later chunks at off2
              const v4w qv = lds16(S.out, d - off);
              uint32_t pw[4];
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const uint32_t pl = __builtin_amdgcn_perm(qv.y, qv.x, S.psel[off][i][0]);
                const uint32_t ph = __builtin_amdgcn_perm(qv.w, qv.z, S.psel[off][i][1]);
                const uint32_t mk = S.psel[off][i][2];
                pw[i] = (pl & ~mk) | (ph & mk);
              }
              lds_put(S.out, d, v4w{pw[0], pw[1], pw[2], pw[3]}, L < 16u ? L : 16u);
              const uint32_t off2 = off * ((16u + off - 1u) / off);
              for (uint32_t c = 16u; c < L; c += 16u) lds_put(S.out, d + c, lds16(S.out, d + c - off2), L - c < 16u ? L - c : 16u);
            } else {
              for (uint32_t c = 0; c < L; c += 16u) lds_put(S.out, d + c, lds16(S.out, d - off + c), L - c < 16u ? L - c : 16u);
            }
            set_rdy(S.rdy, d, d + L);
          }
          pend &= ~go;
        }
        if (__ballot(pend != 0u) != 0ull) st = MTBLX_SNAPPY_CORRUPT;   // unreachable: a round without progress
        stamp(4);
      }
    }
    // ---- 4. output, statuses ----
    if (st == MTBLX_SNAPPY_OK) {
      const uint32_t n16 = W / 16u;
      if (((uintptr_t)dg & 15u) == 0) {
        for (uint32_t c = (uint32_t)lane; c < n16; c += kWave) {
          MTBLX_CHK(dg + 16u * c, 16);
          *reinterpret_cast<v4w*>(dg + 16u * c) = *reinterpret_cast<const v4w*>(S.out + 16u * c);
        }
        for (uint32_t j = 16u * n16 + (uint32_t)lane; j < W; j += kWave) dg[j] = S.out[j];
      } else {
        for (uint32_t j = (uint32_t)lane; j < W; j += kWave) dg[j] = S.out[j];
      }
    }
    if (lane == 0) {
      status[b] = st;
      if (dec_len && st != quad::kDefer) dec_len[b] = st == MTBLX_SNAPPY_OK ? W : 0u;
    }
    stamp(7);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) SNAP_ADD(k, wdbg[k]);
  (void)wdbg;
}
}  // namespace wavep


// ---- directory: preamble lengths, 16-byte aligned exclusive prefix ----
constexpr int kDirThreads = 256, kDirPer = 8, kDirSpan = kDirThreads * kDirPer;

__device__ __forceinline__ uint32_t preamble(const uint8_t* s, uint32_t n, bool& ok) {
  uint64_t v = 0;
  for (uint32_t i = 0; i < 5 && i < n; ++i) {
    const uint32_t byte = s[i];
    v |= (uint64_t)(byte & 0x7fu) << (7 * i);
    if (!(byte & 0x80u)) {
      ok = v <= 0xFFFFFFFFull && v <= kMaxExpand * (uint64_t)n;
      return ok ? (uint32_t)v : 0u;
    }
  }
  ok = false;
  return 0;
}

__device__ __forceinline__ uint64_t pad16(uint32_t x) { return ((uint64_t)x + 15u) & ~15ull; }

// per-thread sums -> workgroup exclusive scan (in `sh`), returns the thread's exclusive base
__device__ uint64_t wg_excl_scan(uint64_t v, uint64_t* sh, uint64_t& total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < kDirThreads; o <<= 1) {
    const uint64_t a = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += a;
    __syncthreads();
  }
  total = sh[kDirThreads - 1];
  const uint64_t r = sh[t] - v;
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(kDirThreads) k_snap_len(const uint8_t* src, const uint64_t* src_off,
                                                          const uint32_t* src_len, uint32_t nblk, uint32_t* dst_len,
                                                          int32_t* status, uint64_t* wsum, uint64_t* totals) {
  __shared__ uint64_t sh[kDirThreads];
  const uint32_t b0 = blockIdx.x * kDirSpan + threadIdx.x * kDirPer;
  uint64_t sum = 0;
  uint32_t mx = 0, bad = 0;
  for (int j = 0; j < kDirPer; ++j) {
    const uint32_t b = b0 + j;
    if (b >= nblk) break;
    bool ok = false;
    if (src_len[b]) MTBLX_CHK(src + src_off[b], src_len[b] < 5u ? src_len[b] : 5u);
    const uint32_t u = preamble(src + src_off[b], src_len[b], ok);
    dst_len[b] = u;
    status[b] = ok ? MTBLX_SNAPPY_OK : MTBLX_SNAPPY_CORRUPT;
    sum += pad16(u);
    mx = max(mx, u);
    bad += ok ? 0u : 1u;
  }
  uint64_t tot = 0;
  (void)wg_excl_scan(sum, sh, tot);
  if (threadIdx.x == 0) wsum[blockIdx.x] = tot;
  if (mx) atomicMax(reinterpret_cast<unsigned long long*>(totals + 1), (unsigned long long)mx);
  if (bad) atomicAdd(reinterpret_cast<unsigned long long*>(totals + 2), (unsigned long long)bad);
}

__global__ void __launch_bounds__(kDirThreads) k_snap_scan(uint64_t* wsum, uint32_t nwg, uint64_t* totals) {
  __shared__ uint64_t sh[kDirThreads];
  uint64_t carry = 0;
  for (uint32_t c = 0; c < nwg; c += kDirThreads) {
    const uint32_t i = c + threadIdx.x;
    const uint64_t v = i < nwg ? wsum[i] : 0;
    uint64_t tot = 0;
    const uint64_t e = wg_excl_scan(v, sh, tot);
    if (i < nwg) wsum[i] = carry + e;
    carry += tot;
  }
  if (threadIdx.x == 0) totals[0] = carry;
}

__global__ void __launch_bounds__(kDirThreads) k_snap_off(const uint32_t* dst_len, uint32_t nblk, const uint64_t* wsum,
                                                          uint64_t* dst_off) {
  __shared__ uint64_t sh[kDirThreads];
  const uint32_t b0 = blockIdx.x * kDirSpan + threadIdx.x * kDirPer;
  uint64_t sum = 0;
  uint32_t u[kDirPer];
  for (int j = 0; j < kDirPer; ++j) {
    u[j] = b0 + j < nblk ? dst_len[b0 + j] : 0u;
    sum += pad16(u[j]);
  }
  uint64_t tot = 0;
  uint64_t base = wg_excl_scan(sum, sh, tot) + wsum[blockIdx.x];
  for (int j = 0; j < kDirPer; ++j) {
    if (b0 + j >= nblk) break;
    dst_off[b0 + j] = base;
    base += pad16(u[j]);
  }
}

int grid_for(int per_cu, uint32_t units) {
  const uint32_t g = (uint32_t)(mtblx_dev::cu_count() * per_cu);
  return (int)(units < g ? (units ? units : 1u) : g);
}

}  // namespace mtblx_snap

using namespace mtblx_snap;

extern "C" size_t mtblx_snappy_workspace_bytes(uint32_t nblk) {
  return 8u * ((size_t)(nblk + kDirSpan - 1) / kDirSpan + 1);
}

extern "C" int mtblx_snappy_dir(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len, uint32_t nblk,
                                uint64_t* dst_off, uint32_t* dst_len, int32_t* status, uint64_t* totals,
                                void* workspace, size_t workspace_bytes, void* stream) {
  if (!totals || (nblk && (!src || !src_off || !src_len || !dst_off || !dst_len || !status || !workspace)))
    return MTBLX_E_INVAL;
  if (workspace_bytes < mtblx_snappy_workspace_bytes(nblk)) return MTBLX_E_INVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (hipMemsetAsync(totals, 0, 3 * sizeof(uint64_t), s) != hipSuccess) return MTBLX_E_HIP;
  if (nblk == 0) return MTBLX_OK;
  const uint32_t nwg = (nblk + kDirSpan - 1) / kDirSpan;
  uint64_t* wsum = reinterpret_cast<uint64_t*>(workspace);
  MTBLX_LAUNCH((src, src_off, src_len, dst_len, status, wsum, totals), k_snap_len, dim3(nwg), dim3(kDirThreads), 0, s, src, src_off, src_len, nblk, dst_len, status,
                     wsum, totals);
  MTBLX_LAUNCH((wsum, totals), k_snap_scan, dim3(1), dim3(kDirThreads), 0, s, wsum, nwg, totals);
  MTBLX_LAUNCH((dst_len, wsum, dst_off), k_snap_off, dim3(nwg), dim3(kDirThreads), 0, s, dst_len, nblk, wsum, dst_off);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

extern "C" int mtblx_snappy_decompress_dev(const uint8_t* src, const uint64_t* src_off, const uint32_t* src_len,
                                           uint32_t nblk, uint8_t* dst, const uint64_t* dst_off,
                                           const uint32_t* dst_len, uint32_t max_dst_len, int32_t* status,
                                           uint32_t* dec_len, void* stream) {
  if (nblk == 0) return MTBLX_OK;
  if (!src || !src_off || !src_len || !dst || !dst_off || !dst_len || !status) return MTBLX_E_INVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  constexpr uint32_t kLanesMinBlocks = 49152;
  // MTBLX_SNAPPY_KERNEL (read per call; tests switch it): "auto" (default: in batches of
  // >= kLanesMinBlocks, blocks expanding > 2x go to k_snappy_lanes, the rest to the quad /
  // one-wave kernels), "lanes" (every block), "quads"
  const char* e = getenv("MTBLX_SNAPPY_KERNEL");
  const int mode = (e && !strcmp(e, "lanes")) ? 2 : (e && !strcmp(e, "quads")) ? 1 : (e && !strcmp(e, "two")) ? 3
                   : (e && !strcmp(e, "waves")) ? 4 : 0;
  // the compressible blocks k_snappy_quads marks: two passes (parse, execute) or one lane each
#ifndef MTBLX_SNAPPY_TWO_DEFAULT
#define MTBLX_SNAPPY_TWO_DEFAULT 0
#endif
  const bool two_pass = mode == 3 || (mode == 0 && MTBLX_SNAPPY_TWO_DEFAULT);
  const dim3 glanes((nblk + lanes::kThreads - 1) / lanes::kThreads), tlanes(2 * lanes::kThreads);
  if (mode == 2) {
    MTBLX_LAUNCH((src, MTBLX_R(src_off, 8ull * nblk), MTBLX_R(src_len, 4ull * nblk), dst, MTBLX_R(dst_off, 8ull * nblk), MTBLX_R(dst_len, 4ull * nblk), MTBLX_R(status, 4ull * nblk), MTBLX_R(dec_len, 4ull * nblk)), lanes::k_snappy_lanes, glanes, tlanes, 0, s, src, src_off, src_len, nblk, dst, dst_off, dst_len,
                       status, dec_len, 0);
  } else if (max_dst_len != 0 && max_dst_len <= (uint32_t)quad::OUT) {
    // k_snappy_lanes costs about one block's serial decode however many blocks run (all are in
    // flight), the quads ~0.19 ms per round of 8 192 blocks: the lanes win from ~50 000 blocks
    // (25 000 compressible blocks: quads 0.66 ms, lanes ~1.0 ms; 100 000: 2.33 vs 1.24 ms)
    const uint32_t lanes_x = ((mode == 0 && nblk >= kLanesMinBlocks) || mode == 3 || mode == 4) ? 2u : 0u;
    MTBLX_LAUNCH((src, MTBLX_R(src_off, 8ull * nblk), MTBLX_R(src_len, 4ull * nblk), dst, MTBLX_R(dst_off, 8ull * nblk), MTBLX_R(dst_len, 4ull * nblk), MTBLX_R(status, 4ull * nblk), MTBLX_R(dec_len, 4ull * nblk)), quad::k_snappy_quads, dim3(grid_for(quad::WG_PER_CU, (nblk + quad::NG - 1) / quad::NG)),
                       dim3(kWave), 0, s, src, src_off, src_len, nblk, dst, dst_off, dst_len, max_dst_len, status,
                       dec_len, lanes_x);
    if (lanes_x && two_pass) {
      MTBLX_LAUNCH((src, MTBLX_R(src_off, 8ull * nblk), MTBLX_R(src_len, 4ull * nblk), dst, MTBLX_R(dst_off, 8ull * nblk), MTBLX_R(dst_len, 4ull * nblk), MTBLX_R(status, 4ull * nblk), MTBLX_R(dec_len, 4ull * nblk)), two::k_snappy_parse, dim3((nblk + two::kParseThreads - 1) / two::kParseThreads),
                         dim3(two::kParseThreads), 0, s, src, src_off, src_len, nblk, dst, dst_off, dst_len, max_dst_len,
                         status, dec_len);
      MTBLX_LAUNCH((src, MTBLX_R(src_off, 8ull * nblk), MTBLX_R(src_len, 4ull * nblk), dst, MTBLX_R(dst_off, 8ull * nblk), MTBLX_R(status, 4ull * nblk), MTBLX_R(dec_len, 4ull * nblk)), two::k_snappy_exec, dim3(grid_for(quad::WG_PER_CU, (nblk + quad::NG - 1) / quad::NG)),
                         dim3(kWave), 0, s, src, src_off, src_len, nblk, dst, dst_off, status, dec_len);
    } else if (lanes_x && mode == 4) {   // the wave-per-block kernel (round 6); its oversize blocks -> deferred
      MTBLX_LAUNCH((src, MTBLX_R(src_off, 8ull * nblk), MTBLX_R(src_len, 4ull * nblk), dst, MTBLX_R(dst_off, 8ull * nblk), MTBLX_R(dst_len, 4ull * nblk), MTBLX_R(status, 4ull * nblk), MTBLX_R(dec_len, 4ull * nblk)), wavep::k_snappy_waves, dim3(grid_for(MTBLX_WAVEP_WG_PER_CU, nblk)), dim3(kWave), 0, s,
                         src, src_off, src_len, nblk, dst, dst_off, dst_len, status, dec_len, 1);
    } else if (lanes_x) {
      MTBLX_LAUNCH((src, MTBLX_R(src_off, 8ull * nblk), MTBLX_R(src_len, 4ull * nblk), dst, MTBLX_R(dst_off, 8ull * nblk), MTBLX_R(dst_len, 4ull * nblk), MTBLX_R(status, 4ull * nblk), MTBLX_R(dec_len, 4ull * nblk)), lanes::k_snappy_lanes, glanes, tlanes, 0, s, src, src_off, src_len, nblk, dst, dst_off,
                         dst_len, status, dec_len, 1);
    }
    MTBLX_LAUNCH((src, MTBLX_R(src_off, 8ull * nblk), MTBLX_R(src_len, 4ull * nblk), dst, MTBLX_R(dst_off, 8ull * nblk), MTBLX_R(dst_len, 4ull * nblk), MTBLX_R(status, 4ull * nblk), MTBLX_R(dec_len, 4ull * nblk)), quad::k_snappy_deferred, dim3(grid_for(2, (nblk + kWave - 1) / kWave)), dim3(kWave), 0, s,
                       src, src_off, src_len, nblk, dst, dst_off, dst_len, status, dec_len);
  } else {
    MTBLX_LAUNCH((src, MTBLX_R(src_off, 8ull * nblk), MTBLX_R(src_len, 4ull * nblk), dst, MTBLX_R(dst_off, 8ull * nblk), MTBLX_R(dst_len, 4ull * nblk), MTBLX_R(status, 4ull * nblk), MTBLX_R(dec_len, 4ull * nblk)), k_snappy_blocks<Large>, dim3(grid_for(2, nblk)), dim3(Large::WAVES * kWave), 0, s, src,
                       src_off, src_len, nblk, dst, dst_off, dst_len, status, dec_len);
  }
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

#ifdef MTBLX_SNAP_STAMPS
extern "C" int mtblx_snap_debug(uint64_t* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(mtblx_snap::g_snap_dbg), 8 * sizeof(uint64_t)) != hipSuccess) return -1;
  if (reset) {
    static const uint64_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(mtblx_snap::g_snap_dbg), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif
