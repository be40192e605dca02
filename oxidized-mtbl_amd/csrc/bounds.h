// bounds.h — the bounds-checked diagnostic build (-DMTBLX_BOUNDS, Makefile target `bounds`,
// build/libmtblx_bounds.so; never the product or the measured build).
//
// What it checks: every global access a kernel makes through MTBLX_CHK(p, n) must fall inside
// one of the ranges its launch was handed: the caller-declared extent of an argument where the
// entry point knows it (Rng{ptr, bytes}: data_len, capacities, nblk / nq sized arrays), else the
// device allocation that contains the pointer (the hipMalloc / caching-allocator segment, found
// with hipMemGetAddressRange).  An access outside every range breaks the entry point's contract;
// outside every allocation it is exactly the kind that can fault the GPU
// (hipErrorIllegalAddress) when the next page is unmapped, and that silently reads or corrupts
// another buffer when it is not.  The first violation of a launch is recorded in a device word (source line, address,
// size); the host side of every launch (MTBLX_LAUNCH) then synchronizes the stream and prints it
// with the kernel's name, so a fault or a violation is reported by the launch that caused it,
// not by whatever API call comes next.  mtblx_bounds_report() (mtblx_api.cpp) returns the
// number of violations seen by the process; tests/conftest.py fails the test that caused one
// when MTBLX_BOUNDS_CHECK is set.
//
// In the product build MTBLX_CHK is empty and MTBLX_LAUNCH is hipLaunchKernelGGL.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef MTBLX_BOUNDS
#include <stdio.h>
#include <stdlib.h>

#include <initializer_list>
#include <mutex>

extern "C" void mtblx_bounds_note(const char* kernel, uint64_t line, uint64_t addr, uint64_t nbytes, int fault);

// The table and the first-violation record are one per translation unit: launches from several
// host threads (the concurrent-cut test) would overwrite each other's table between a set_ranges
// and its launch, so the diagnostic build serializes set_ranges + launch + after process-wide
// (an inline function with external linkage: one mutex for the whole library).
inline std::mutex& mtblx_bounds_launch_lock() {
  static std::mutex m;
  return m;
}

namespace {   // one copy per translation unit: its kernels read their own table
namespace mtblx_bounds {
constexpr int kMaxRanges = 24;
struct Tab {
  uint64_t lo[kMaxRanges], hi[kMaxRanges];
  uint32_t n;
};
__device__ Tab g_tab;
// first violation of the current launch: {line, address, bytes, count}
__device__ unsigned long long g_first[4];

// no call and no printf in the kernels (a call changes how the pipe kernels address LDS,
// DESIGN.md §4): the host prints the record after the launch
__device__ __forceinline__ void violation(uint32_t line, uint64_t a, uint64_t n) {
  const unsigned long long c = atomicAdd(&g_first[3], 1ull);
  if (c == 0) {
    g_first[0] = line;
    g_first[1] = a;
    g_first[2] = n;
  }
}

__device__ __forceinline__ void check(const void* p, uint64_t n, uint32_t line) {
  // LDS and scratch are not checked here (a generic pointer may point into either)
  if (__builtin_amdgcn_is_shared((const __attribute__((address_space(0))) void*)p) ||
      __builtin_amdgcn_is_private((const __attribute__((address_space(0))) void*)p))
    return;
  const uint64_t a = (uint64_t)(uintptr_t)p;
  const uint32_t m = g_tab.n;
  for (uint32_t i = 0; i < m; ++i)
    if (a >= g_tab.lo[i] && a + n <= g_tab.hi[i]) return;
  violation(line, a, n);
}

// an LDS access [p, p + n) of a pointer known to point into LDS: inside the kernel's static LDS
// allocation (an access past it reads 0 / is dropped through ds_*, faults through flat_*).
// Recorded with bit 31 of the line set.
__device__ __forceinline__ void lcheck(const void* p, uint32_t n, uint32_t line) {
  const uint32_t off = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
  if ((uint64_t)off + n > (uint64_t)__builtin_amdgcn_groupstaticsize()) violation(line | 0x80000000u, off, n);
}

// one range of a launch: [p, p + n), or (n == 0) the allocation holding p
struct Rng {
  const void* p;
  uint64_t n;
  Rng(const void* q) : p(q), n(0) {}
  Rng(const void* q, uint64_t m) : p(q), n(m) {}
};

// host: the launch's ranges -> the table; the whole device is synchronized first, so no kernel of
// this translation unit still reads the previous table.  MTBLX_BOUNDS_SELFTEST=1
// (tests/test_bounds_gpu.py): the launch's FIRST range is left out of the table, so the checker
// must report that launch's accesses to it.
inline void set_ranges(hipStream_t s, std::initializer_list<Rng> rs) {
  (void)hipDeviceSynchronize();
  Tab t{};
  const char* st = getenv("MTBLX_BOUNDS_SELFTEST");
  bool skip = st && st[0] == '1';
  for (const Rng& r : rs) {
    if (skip) { skip = false; continue; }
    if (!r.p || t.n >= (uint32_t)kMaxRanges) continue;
    if (r.n) {
      t.lo[t.n] = (uint64_t)(uintptr_t)r.p;
      t.hi[t.n] = (uint64_t)(uintptr_t)r.p + r.n;
      ++t.n;
      continue;
    }
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, const_cast<void*>(r.p)) != hipSuccess || !base) {
      (void)hipGetLastError();
      continue;
    }
    t.lo[t.n] = (uint64_t)(uintptr_t)base;
    t.hi[t.n] = (uint64_t)(uintptr_t)base + size;
    ++t.n;
  }
  const unsigned long long z[4] = {0, 0, 0, 0};
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_tab), &t, sizeof(t), 0, hipMemcpyHostToDevice, s);
  (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_first), z, sizeof(z), 0, hipMemcpyHostToDevice, s);
  (void)hipStreamSynchronize(s);
}

inline void after(const char* name, hipStream_t s) {
  const hipError_t e = hipStreamSynchronize(s);
  unsigned long long f[4] = {0, 0, 0, 0};
  if (e == hipSuccess) (void)hipMemcpyFromSymbol(f, HIP_SYMBOL(g_first), sizeof(f), 0, hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    fprintf(stderr, "MTBLX_BOUNDS: launch of %s failed: %s\n", name, hipGetErrorString(e));
    mtblx_bounds_note(name, 0, 0, 0, 1);
  } else if (f[3]) {
    fprintf(stderr, "MTBLX_BOUNDS: %s: %llu accesses outside the %s, first at line %llu: 0x%llx +%llu\n", name,
            f[3], (f[0] & 0x80000000ull) ? "kernel's LDS allocation" : "argument allocations", f[0] & 0x7FFFFFFFull,
            f[1], f[2]);
    mtblx_bounds_note(name, f[0], f[1], f[2], 0);
  }
  fflush(stderr);
}
}  // namespace mtblx_bounds
}  // namespace

#define MTBLX_CHK(p, n) mtblx_bounds::check((const void*)(p), (uint64_t)(n), __LINE__)
#define MTBLX_LCHK(p, n) mtblx_bounds::lcheck((const void*)(p), (uint32_t)(n), __LINE__)
// MTBLX_LAUNCH((range, range, ...), kernel, grid, block, shmem, stream, args...): a range is a
// pointer (its allocation) or MTBLX_R(ptr, bytes) (the caller-declared extent)
#define MTBLX_PTRS(...) {__VA_ARGS__}
#define MTBLX_R(p, n) mtblx_bounds::Rng((const void*)(p), (uint64_t)(n))
#define MTBLX_LAUNCH(ptrs, kern, g, b, sh, s, ...)                                        \
  do {                                                                                    \
    std::lock_guard<std::mutex> bounds_lock_(mtblx_bounds_launch_lock());                   \
    mtblx_bounds::set_ranges((s), std::initializer_list<mtblx_bounds::Rng> MTBLX_PTRS ptrs); \
    hipLaunchKernelGGL(kern, g, b, sh, s, __VA_ARGS__);                              \
    mtblx_bounds::after(#kern, (s));                                                 \
  } while (0)
#else
#define MTBLX_CHK(p, n) ((void)0)
#define MTBLX_LCHK(p, n) ((void)0)
#define MTBLX_R(p, n) (p)
#define MTBLX_LAUNCH(ptrs, kern, g, b, sh, s, ...) hipLaunchKernelGGL(kern, g, b, sh, s, __VA_ARGS__)
#endif
