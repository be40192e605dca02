// devinfo.h — immutable device properties the launch sizes need, cached per device.
//
// The library keeps no mutable state between calls (include/mtblx.h); the one process-wide data
// is this cache of what the hardware is (compute units, occupancy of a kernel), filled on first
// use per device.  Relaxed atomics: concurrent first calls from several host threads store the
// same value, and a device's entry never changes afterwards.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>

namespace mtblx_dev {

constexpr int kMaxDevices = 64;

// compute units of the current device (256 on MI355X; 256 if the query fails)
inline int cu_count() {
  static std::atomic<int> cache[kMaxDevices];
  int dev = 0;
  (void)hipGetDevice(&dev);
  int v = (dev >= 0 && dev < kMaxDevices) ? cache[dev].load(std::memory_order_relaxed) : 0;
  if (v <= 0) {
    (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
    if (v <= 0) v = 256;
    if (dev >= 0 && dev < kMaxDevices) cache[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}

// a per-device cached value computed by f() (e.g. an occupancy query): one Cache object per use
struct Cache {
  std::atomic<int> v[kMaxDevices] = {};
  template <class F>
  int get(F f) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= kMaxDevices) return f();
    int x = v[dev].load(std::memory_order_relaxed);
    if (x <= 0) {
      x = f();
      v[dev].store(x, std::memory_order_relaxed);
    }
    return x;
  }
};

}  // namespace mtblx_dev
