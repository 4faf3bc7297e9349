// Dynamic-LDS limit for kernels that stage more than the default 64 KB.
// hipFuncAttributeMaxDynamicSharedMemorySize is a per-device attribute of a kernel, so it is raised once
// per (device, kernel) pair, under a lock (a process may drive several GPUs from several threads).
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <set>
#include <utility>

namespace dgppo {

inline void allow_lds(const void* fn, int bytes = 160 * 1024) {
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(mu);
  if (done.insert({dev, fn}).second) (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

}  // namespace dgppo
