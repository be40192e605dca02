// Diagnostic: latency and throughput of aligned vs unaligned LDS reads/writes on gfx950.
//   hipcc --offload-arch=gfx950 -O3 scripts/lds_probe.hip -o build/lds_probe && ./build/lds_probe
// Latency: one wave, a dependent chain of reads (the next address comes from the loaded value).
// Throughput: 16 waves per workgroup, independent reads of consecutive per-lane addresses.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint32_t v2u __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t v4u __attribute__((ext_vector_type(4), aligned(1)));

constexpr int kBytes = 32768;

template <int W>
__device__ __forceinline__ uint32_t rd(const uint8_t* p) {
  if constexpr (W == 4) return *reinterpret_cast<const u32u*>(p);
  else if constexpr (W == 8) { v2u x = *reinterpret_cast<const v2u*>(p); return x.x ^ x.y; }
  else { v4u x = *reinterpret_cast<const v4u*>(p); return x.x ^ x.y ^ x.z ^ x.w; }
}

template <int W>
__global__ void k_lat(uint32_t mis, uint32_t mask, int iters, uint64_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t L[kBytes + 64];
  for (int i = threadIdx.x; i < (kBytes + 64) / 4; i += blockDim.x) reinterpret_cast<uint32_t*>(L)[i] = 0;
  __syncthreads();
  uint32_t a = (threadIdx.x * 64u) % kBytes + mis;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    const uint32_t v = rd<W>(L + a);
    a = ((a + 256u + (v & mask)) % kBytes) | mis;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if (a == 0xFFFFFFFFu) out[1] = a;
}

template <int W>
__global__ void k_thr(uint32_t mis, int iters, uint64_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t L[kBytes + 64];
  for (int i = threadIdx.x; i < (kBytes + 64) / 4; i += blockDim.x) reinterpret_cast<uint32_t*>(L)[i] = i;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    const uint32_t a = ((uint32_t)(wv * 1024 + i * 64) * W / 4u + (uint32_t)lane * W) % kBytes + mis;
    acc += rd<W>(L + a);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if (acc == 0x12345u) out[1] = acc;
}

__global__ void k_wr(uint32_t mis, int iters, uint64_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t L[kBytes + 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    const uint32_t a = ((uint32_t)(wv * 1024 + i * 256) + (uint32_t)lane * 4u) % kBytes + mis;
    *reinterpret_cast<u32u*>(L + a) = (uint32_t)i;
  }
  __syncthreads();
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if (L[lane] == 0xEE) out[1] = 1;
}

int main() {
  uint64_t* d;
  hipMalloc(&d, 16);
  uint64_t h[2];
  const int it = 4096;
  auto run = [&](const char* what, auto launch) {
    launch();
    hipDeviceSynchronize();
    launch();
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("%-34s %8.1f memtime ticks per iteration\n", what, (double)h[0] / it);
  };
  for (uint32_t mis : {0u, 1u, 2u, 3u}) {
    char b[64];
    snprintf(b, sizeof b, "latency b32 mis=%u", mis);
    run(b, [&] { k_lat<4><<<1, 64>>>(mis, 0, it, d); });
    snprintf(b, sizeof b, "latency b64 mis=%u", mis);
    run(b, [&] { k_lat<8><<<1, 64>>>(mis, 0, it, d); });
    snprintf(b, sizeof b, "latency b128 mis=%u", mis);
    run(b, [&] { k_lat<16><<<1, 64>>>(mis, 0, it, d); });
  }
  for (uint32_t mis : {0u, 1u, 4u}) {
    char b[64];
    snprintf(b, sizeof b, "thr 16 waves b32 mis=%u", mis);
    run(b, [&] { k_thr<4><<<1, 1024>>>(mis, it, d); });
    snprintf(b, sizeof b, "thr 16 waves b128 mis=%u", mis);
    run(b, [&] { k_thr<16><<<1, 1024>>>(mis, it, d); });
    snprintf(b, sizeof b, "thr 16 waves write b32 mis=%u", mis);
    run(b, [&] { k_wr<<<1, 1024>>>(mis, it, d); });
  }
  printf("(s_memtime ticks at 100 MHz on gfx9: multiply by core clock / 100 MHz for cycles)\n");
  return 0;
}
