// Content-addressed, never-freed device copies of small launch tables.
//
// The grouped kernels (gradient gather, KL dot / apply, factor SYRK / EMA)
// used to take their job tables as ~1-4 KB by-value kernel arguments.  When
// such a launch is captured into a hipGraph and the graph is replayed
// back-to-back, the kernels read corrupted tables on ROCm 7.2 (garbage
// gathered gradients, a NaN / inf KL scale; scripts/probes/debug_replay_nan.py,
// profiles/README.md), while kernels that read their tables from device memory
// (the preconditioning GEMMs) replay correctly.  So every table now lives in
// device memory: a table seen before costs nothing (the same device copy is
// returned, so a captured graph and eager launches share an immutable table);
// a new table is copied stream-ordered from a pinned host copy that the cache
// owns forever (inside a capture the copy becomes a graph memcpy node).
#pragma once
#include "common.h"

#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace kfac_devtable {

struct Cache {
  std::mutex mu;
  std::unordered_map<std::string, const void*> map;
  char* dev = nullptr;      // current device arena
  char* host = nullptr;     // matching pinned host arena
  size_t used = 0, cap = 0;
};

inline Cache& cache() {
  static Cache c;
  return c;
}

// Device pointer to an immutable copy of `bytes` bytes at `host`.
// Returns nullptr (and sets *err) on failure.
inline const void* get(const void* host, size_t bytes, hipStream_t stream, int* err) {
  Cache& c = cache();
  std::lock_guard<std::mutex> lk(c.mu);
  std::string key((const char*)host, bytes);
  auto it = c.map.find(key);
  if (it != c.map.end()) return it->second;
  const size_t need = (bytes + 255) / 256 * 256;
  if (c.used + need > c.cap) {
    // a new arena (allocation is not capturable: the first use of a table
    // happens in an eager warm-up run in practice)
    const size_t cap = need > (size_t)(4 << 20) ? need : (size_t)(4 << 20);
    char* d = nullptr;
    char* h = nullptr;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
      *err = -20;   // would allocate inside a capture
      return nullptr;
    }
    if (hipMalloc(&d, cap) != hipSuccess || hipHostMalloc(&h, cap, 0) != hipSuccess) {
      (void)hipGetLastError();
      *err = -21;
      return nullptr;
    }
    c.dev = d; c.host = h; c.used = 0; c.cap = cap;
  }
  char* d = c.dev + c.used;
  char* h = c.host + c.used;
  c.used += need;
  memcpy(h, host, bytes);
  const hipError_t e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) {
    *err = (int)e;
    return nullptr;
  }
  c.map.emplace(std::move(key), (const void*)d);
  return d;
}

}  // namespace kfac_devtable
