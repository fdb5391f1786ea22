// Split-K arrival counter pool (see launch.h splitk_counters).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <mutex>

#include "launch.h"

namespace tfsk {

namespace {
constexpr int kPoolInts = 1 << 22;   // 16 MB per device
// Used by the split-K fixup (TFSERVE_SPLITK_FIXUP=1, opt-in) and by the
// control words of captured flow launches (flow.hip, kernels/flow.h).
// [0, kCapInts): permanent slices for launches captured into HIP graphs (a
// graph node keeps its counters for the graph's lifetime; slices are never
// returned, so repeated captures -- tuning candidates, reloads, more buckets
// or lanes -- use the 3.75M ints up, after which launches fall back to the
// reduce launch, logged once); [kCapInts, kPoolInts): a ring for eager
// launches (autotuning, warm-up), reused cyclically.  A maximal take (32K
// ints) wraps the 256K-int ring after 8 launches; reuse is still safe because
// eager launches are stream-ordered and counters return to zero when a
// tile's last slice arrives, before the next launch on the stream starts.
constexpr int kCapInts = 15 << 18;
struct Pool {
  int* base = nullptr;
  int used = 0;
  int ring = kCapInts;
};
std::mutex g_mu;
std::map<int, Pool> g_pools;

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}
}  // namespace

void splitk_counters_prepare(hipStream_t s) {
  if (capturing(s)) return;     // allocation + memset only outside a capture
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  std::lock_guard<std::mutex> g(g_mu);
  Pool& p = g_pools[dev];
  if (p.base != nullptr) return;
  void* ptr = nullptr;
  if (hipMalloc(&ptr, size_t(kPoolInts) * sizeof(int)) != hipSuccess) return;
  if (hipMemset(ptr, 0, size_t(kPoolInts) * sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    hipFree(ptr);
    return;
  }
  p.base = static_cast<int*>(ptr);
}

int* splitk_counters(int n, hipStream_t s) {
  if (n <= 0) return nullptr;
  const bool cap = capturing(s);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_pools.find(dev);
  if (it == g_pools.end() || it->second.base == nullptr) return nullptr;
  Pool& p = it->second;
  const int take = (n + 63) / 64 * 64;
  if (!cap) {
    if (take > (kPoolInts - kCapInts) / 8) return nullptr;
    if (p.ring + take > kPoolInts) p.ring = kCapInts;
    int* r = p.base + p.ring;
    p.ring += take;
    return r;
  }
  if (p.used + take > kCapInts) {
    static bool warned = false;
    if (!warned) {
      warned = true;
      fprintf(stderr, "[tfserve] split-K counter pool for captured graphs is used up; "
                      "further captures reduce split-K in a separate launch\n");
    }
    return nullptr;
  }
  int* r = p.base + p.used;
  p.used += take;
  return r;
}

}  // namespace tfsk
