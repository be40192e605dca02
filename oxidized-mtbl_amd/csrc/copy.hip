// copy.hip — gfx950 device copy at the HBM ceiling: the box's own reference for bench.py's
// roofline (what a plain streaming kernel moving the same bytes reaches on this MI355X).
// Not on the decode path.  16 bytes per lane per access, U accesses in flight per lane, a
// grid of 8 workgroups per CU striding over the buffer; variant bits select non-temporal
// stores / loads so bench.py can take the best of a small sweep.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtblx.h"
#include "bounds.h"

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

}  // namespace

extern "C" int mtblx_stream_copy(void* dst, const void* src, uint64_t bytes, int variant, void* stream) {
  if (!dst || !src || (bytes & 15u) || ((uintptr_t)dst & 15u) || ((uintptr_t)src & 15u)) return MTBLX_E_INVAL;
  if (bytes == 0) return MTBLX_OK;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
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
