// copy.hip — gfx950 device copy at the HBM ceiling: the box's own reference for bench.py's
// roofline (what a plain streaming kernel moving the same bytes reaches on this MI355X).
// Not on the decode path.  16 bytes per lane per access, U accesses in flight per lane, a
// grid of 8 workgroups per CU striding over the buffer; variant bits select non-temporal
// stores / loads so bench.py can take the best of a small sweep.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtblx.h"
#include "bounds.h"
#include "devinfo.h"

namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int U, bool NTS, bool NTL>
__global__ void __launch_bounds__(256) k_stream_copy(const v4u* __restrict__ src, v4u* __restrict__ dst,
                                                     uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u * U;
  for (uint64_t i = (uint64_t)blockIdx.x * 256u * U + threadIdx.x; i < n16; i += stride) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = i + 256u * (uint64_t)u;
      if (j < n16) v[u] = NTL ? __builtin_nontemporal_load(src + j) : src[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = i + 256u * (uint64_t)u;
      if (j < n16) {
        if (NTS) __builtin_nontemporal_store(v[u], dst + j);
        else dst[j] = v[u];
      }
    }
  }
}

template <int U>
void launch(int variant, dim3 g, hipStream_t s, const v4u* src, v4u* dst, uint64_t n16) {
  switch (variant & (MTBLX_COPY_NT_STORES | MTBLX_COPY_NT_LOADS)) {
    case 0: MTBLX_LAUNCH((src, dst), (k_stream_copy<U, false, false>), g, dim3(256), 0, s, src, dst, n16); break;
    case MTBLX_COPY_NT_STORES: MTBLX_LAUNCH((src, dst), (k_stream_copy<U, true, false>), g, dim3(256), 0, s, src, dst, n16); break;
    case MTBLX_COPY_NT_LOADS: MTBLX_LAUNCH((src, dst), (k_stream_copy<U, false, true>), g, dim3(256), 0, s, src, dst, n16); break;
    default: MTBLX_LAUNCH((src, dst), (k_stream_copy<U, true, true>), g, dim3(256), 0, s, src, dst, n16); break;
  }
}

// n byte ranges src + src_off[i] -> dst + dst_off[i], len[i] bytes, by the whole grid: the
// ranges' 16-byte destination chunks are numbered across all ranges (exclusive prefix in
// chunk_base, host-computed) and every thread takes chunks grid-stride, U in flight: an unaligned
// 16-byte load and store per whole chunk, bytes at each range's ragged ends.  For the values of
// blocks >= 4 GiB (mtblx_block_seek_batch_ex).
typedef uint32_t v4uu __attribute__((ext_vector_type(4), aligned(1)));
__global__ void __launch_bounds__(256) k_copy_ranges(const uint8_t* __restrict__ src, const uint64_t* src_off,
                                                     uint8_t* __restrict__ dst, const uint64_t* dst_off,
                                                     const uint64_t* len, const uint64_t* chunk_base, uint32_t n,
                                                     uint64_t nchunks) {
  constexpr int U = 4;
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  uint64_t c = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  for (; c < nchunks; c += stride * U) {
    v4uu v[U];
    uint8_t* dp[U];
    uint32_t m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t cc = c + stride * (uint64_t)u;
      m[u] = 0;
      if (cc >= nchunks) continue;
      uint32_t lo = 0, hi = n;   // the range holding chunk cc: last i with chunk_base[i] <= cc
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (chunk_base[mid] <= cc) lo = mid; else hi = mid;
      }
      const uint64_t k = 16 * (cc - chunk_base[lo]), L = len[lo];
      const uint8_t* sp = src + src_off[lo] + k;
      dp[u] = dst + dst_off[lo] + k;
      m[u] = L - k < 16 ? (uint32_t)(L - k) : 16u;
      MTBLX_CHK(sp, m[u]);
      if (m[u] == 16) {
        v[u] = *reinterpret_cast<const v4uu*>(sp);
      } else {
        uint32_t t[4] = {0, 0, 0, 0};
        for (uint32_t b = 0; b < m[u]; ++b) t[b >> 2] |= (uint32_t)sp[b] << (8 * (b & 3));
        v[u] = v4uu{t[0], t[1], t[2], t[3]};
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (m[u] == 0) continue;
      MTBLX_CHK(dp[u], m[u]);
      if (m[u] == 16) {
        *reinterpret_cast<v4uu*>(dp[u]) = v[u];
      } else {
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        for (uint32_t b = 0; b < m[u]; ++b) dp[u][b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
      }
    }
  }
}

}  // namespace

extern "C" int mtblx_copy_ranges(const uint8_t* src, const uint64_t* src_off, uint8_t* dst, const uint64_t* dst_off,
                                 const uint64_t* len, const uint64_t* chunk_base, uint32_t n, uint64_t nchunks,
                                 void* stream) {
  if (n == 0 || nchunks == 0) return MTBLX_OK;
  if (!src || !src_off || !dst || !dst_off || !len || !chunk_base) return MTBLX_E_INVAL;
  const int ncu = mtblx_dev::cu_count();
  const uint64_t want = (nchunks + 4 * 256 - 1) / (4 * 256);
  const dim3 g((unsigned)(want < (uint64_t)ncu * 8u ? want : (uint64_t)ncu * 8u));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  MTBLX_LAUNCH((src, MTBLX_R(src_off, 8ull * n), dst, MTBLX_R(dst_off, 8ull * n), MTBLX_R(len, 8ull * n),
                MTBLX_R(chunk_base, 8ull * n)),
               k_copy_ranges, g, dim3(256), 0, s, src, src_off, dst, dst_off, len, chunk_base, n, nchunks);
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}

extern "C" int mtblx_stream_copy(void* dst, const void* src, uint64_t bytes, int variant, void* stream) {
  if (!dst || !src || (bytes & 15u) || ((uintptr_t)dst & 15u) || ((uintptr_t)src & 15u)) return MTBLX_E_INVAL;
  if (bytes == 0) return MTBLX_OK;
  const int ncu = mtblx_dev::cu_count();
  const uint64_t n16 = bytes / 16u;
  const dim3 g((unsigned)ncu * 8u);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const v4u* sp = static_cast<const v4u*>(src);
  v4u* dp = static_cast<v4u*>(dst);
  switch (variant & 3) {
    case 0: launch<1>(variant, g, s, sp, dp, n16); break;
    case 1: launch<2>(variant, g, s, sp, dp, n16); break;
    case 2: launch<4>(variant, g, s, sp, dp, n16); break;
    default: launch<8>(variant, g, s, sp, dp, n16); break;
  }
  return hipGetLastError() == hipSuccess ? MTBLX_OK : MTBLX_E_HIP;
}
