// pt_graph.h — replay the whole T-step launch sequence of a forward / backward
// as one hipGraph.
//
// A call's launch sequence is fully determined by its arguments (descriptor,
// device pointers, flags), so the first call with a given argument set is
// captured on a private stream (capture records, it does not execute), the
// graph is instantiated, and it and every later call with the same arguments
// are a single hipGraphLaunch on the caller's stream.  Under PyTorch's caching
// allocator the per-step buffers come back at the same addresses, so a
// training loop hits the cache from its second step on.  Kernels that read
// the parameters (the weight-fragment preparation) are part of the graph, so
// parameter updates between replays are seen.
//
// The cache is process-wide and mutex-guarded (graph execs are not bound to a
// host thread); entries are per device, least-recently-used beyond CAP.
// PT_CELL_GRAPH=0 in the environment disables it (direct launches).
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

namespace ptg {

inline bool graphs_enabled() {
  static const bool on = [] {
    const char* e = getenv("PT_CELL_GRAPH");
    return !(e && e[0] == '0');
  }();
  return on;
}

class GraphCache {
 public:
  static constexpr size_t CAP = 16;

  // body(stream) issues the launch sequence on `stream` and returns 0 or an
  // error code (returned unchanged).  hip_err receives HIP failures of the
  // capture / instantiate / launch steps.
  template <class Body>
  int run(const void* key, size_t nkey, hipStream_t st, int hip_err, Body&& body) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hip_err;
    hipGraphExec_t exec = lookup(key, nkey, dev);
    if (!exec) {
      hipStream_t cs;
      if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return hip_err;
      if (hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipStreamDestroy(cs);
        return hip_err;
      }
      const int rc = body(cs);
      hipGraph_t g = nullptr;
      const hipError_t ec = hipStreamEndCapture(cs, &g);
      (void)hipStreamDestroy(cs);
      if (rc != 0 || ec != hipSuccess || !g) {
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        return rc != 0 ? rc : hip_err;
      }
      const hipError_t ei = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (ei != hipSuccess) return hip_err;
      exec = insert(key, nkey, dev, exec);     // another thread may have won the race
    }
    return hipGraphLaunch(exec, st) == hipSuccess ? 0 : hip_err;
  }

 private:
  struct Entry {
    std::vector<char> key;
    int dev;
    hipGraphExec_t exec;
    uint64_t used;
  };
  std::mutex mu_;
  std::vector<Entry> e_;
  uint64_t tick_ = 0;

  hipGraphExec_t lookup(const void* key, size_t n, int dev) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& x : e_)
      if (x.dev == dev && x.key.size() == n && memcmp(x.key.data(), key, n) == 0) {
        x.used = ++tick_;
        return x.exec;
      }
    return nullptr;
  }
  // Returns the exec to launch: `exec`, or the entry another thread inserted
  // for the same key meanwhile (then `exec` is destroyed: it never launched).
  hipGraphExec_t insert(const void* key, size_t n, int dev, hipGraphExec_t exec) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& x : e_)
      if (x.dev == dev && x.key.size() == n && memcmp(x.key.data(), key, n) == 0) {
        (void)hipGraphExecDestroy(exec);
        x.used = ++tick_;
        return x.exec;
      }
    if (e_.size() >= CAP) {
      size_t lru = 0;
      for (size_t i = 1; i < e_.size(); ++i)
        if (e_[i].used < e_[lru].used) lru = i;
      // a replay of the evicted graph may still be queued: drain the device
      // first (rare: only past CAP distinct argument sets)
      (void)hipDeviceSynchronize();
      (void)hipGraphExecDestroy(e_[lru].exec);
      e_.erase(e_.begin() + lru);
    }
    Entry x;
    x.key.assign((const char*)key, (const char*)key + n);
    x.dev = dev;
    x.exec = exec;
    x.used = ++tick_;
    e_.push_back(std::move(x));
    return exec;
  }
};

// Key builder: appends the raw bytes of each argument.
struct Key {
  std::vector<char> b;
  template <class T> Key& add(const T& v) {
    const char* p = (const char*)&v;
    b.insert(b.end(), p, p + sizeof(T));
    return *this;
  }
};

}  // namespace ptg
