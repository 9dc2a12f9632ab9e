// Host-side launch helpers shared by the kernel launchers: per-device, thread-safe caches.
//
// The ABI is re-entrant (include/raman_mi355x.h): launches may come from several threads and for
// streams of different devices.  hipFuncSetAttribute(MaxDynamicSharedMemorySize) and the CU count
// are per device, so both caches are keyed by the device that owns the launch stream and guarded
// by one mutex (taken once per (kernel, device) pair on the slow path; lock-free afterwards).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <mutex>

namespace rdn {

constexpr int MAX_DEVICES = 64;

// device that executes work enqueued on `s` (the current device for the null stream)
inline int stream_device(hipStream_t s) {
  int dev = 0;
  if (s) {
    hipDevice_t d;
    if (hipStreamGetDevice(s, &d) == hipSuccess) return (int)d;
  }
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  return dev;
}

// One flag per (kernel slot, device).  `slot` is a small per-launcher index (< 64) naming the
// kernel function; callers own disjoint slot ranges (see the launchers).
inline std::mutex& attr_mutex() {
  static std::mutex m;
  return m;
}
constexpr int ATTR_SLOTS = 128;
inline std::atomic<bool>* attr_flags() {
  static std::atomic<bool> f[ATTR_SLOTS * MAX_DEVICES];
  return f;
}

// Allow `bytes` of dynamic LDS for kernel `fn` on device `dev` (once per pair).
inline hipError_t ensure_dynamic_lds(const void* fn, int slot, int bytes, int dev) {
  if (slot < 0 || slot >= ATTR_SLOTS || dev < 0 || dev >= MAX_DEVICES) return hipErrorInvalidValue;
  std::atomic<bool>& flag = attr_flags()[dev * ATTR_SLOTS + slot];
  if (flag.load(std::memory_order_acquire)) return hipSuccess;
  std::lock_guard<std::mutex> lock(attr_mutex());
  if (flag.load(std::memory_order_relaxed)) return hipSuccess;
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e != hipSuccess) return e;
  if (cur != dev && (e = hipSetDevice(dev)) != hipSuccess) return e;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (cur != dev) {
    const hipError_t e2 = hipSetDevice(cur);
    if (e == hipSuccess) e = e2;
  }
  if (e == hipSuccess) flag.store(true, std::memory_order_release);
  return e;
}

// Copy `bytes` (<= 16) of status words from the device to `out` behind the work on `s` and wait for
// it: through a 16-byte pinned buffer of the calling thread (a copy into pageable memory takes the
// runtime's staging path, ≈ 20 µs more per call of the batch-1 loop).  The buffer is allocated on
// the thread's first read and kept (16 B per thread that ever read a status word); stack memory if
// the allocation fails.
inline hipError_t read_words(void* out, const void* dev_words, size_t bytes, hipStream_t s) {
  thread_local void* pinned = nullptr;
  thread_local bool tried = false;
  if (!tried) {
    tried = true;
    if (hipHostMalloc(&pinned, 16, hipHostMallocPortable) != hipSuccess) {
      pinned = nullptr;
      (void)hipGetLastError();
    }
  }
  if (bytes > 16) return hipErrorInvalidValue;
  void* dst = pinned ? pinned : out;
  hipError_t e = hipMemcpyAsync(dst, dev_words, bytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess && pinned) memcpy(out, pinned, bytes);
  return e;
}

// Compute units of device `dev` (0 if the query fails), cached per device.
inline int device_cus(int dev) {
  static std::atomic<int> cus[MAX_DEVICES];
  if (dev < 0 || dev >= MAX_DEVICES) return 0;
  int v = cus[dev].load(std::memory_order_relaxed);
  if (v > 0) return v;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  cus[dev].store(v, std::memory_order_relaxed);
  return v;
}

}  // namespace rdn
