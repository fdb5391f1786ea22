// Split-K arrival counter pool (see launch.h splitk_counters).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <map>
#include <mutex>
#include <vector>

#include "launch.h"

namespace tfsk {

namespace {
constexpr int kPoolInts = 1 << 22;   // 16 MB per device
// Used by the split-K fixup (bindings.cpp split_fixup_mode: small launches by default).
// [0, kCapInts): slices for launches captured into HIP graphs (a graph node
// keeps its counters for the graph's lifetime).  A capture made under an
// owner token (splitk_counters_set_owner, set by the Python runtime around
// each graph capture) returns its slices to a free list when the runtime
// releases the token as the graph is destroyed -- tuning candidates and
// reload cycles no longer use the range up; slices taken without an owner
// stay taken.  A release only quarantines the slices (pending, stamped):
// splitk_counters_reclaim zeroes the old-enough ones and frees them then, so
// neither a replay still queued behind the dropped graph nor a counter left
// non-zero by an abandoned lane can hand a later capture a live counter.
// [kCapInts, kPoolInts): a ring for eager launches (autotuning,
// warm-up), reused cyclically.  A maximal take (32K ints) wraps the 256K-int
// ring after 8 launches; reuse is still safe because eager launches are
// stream-ordered and counters return to zero when a tile's last slice
// arrives, before the next launch on the stream starts (which is also why a
// released slice is zero again: every replay of its graph completed).
constexpr int kCapInts = 15 << 18;
struct Range {
  int off, len;
};
using Clock = std::chrono::steady_clock;
struct Pending {
  Range r;
  Clock::time_point at;
};
struct Pool {
  int* base = nullptr;
  int used = 0;
  int ring = kCapInts;
  std::vector<Range> free_list;                     // zeroed released slices, reusable
  std::vector<Pending> pending;                     // released, not yet zeroed (quarantine)
  std::map<int64_t, std::vector<Range>> owned;      // owner token -> its captured slices
};
std::mutex g_mu;
std::map<int, Pool> g_pools;
thread_local int64_t g_owner = 0;

// first fit from the free list (splitting the range), else -1
int take_free(Pool& p, int take) {
  for (size_t i = 0; i < p.free_list.size(); ++i) {
    Range& r = p.free_list[i];
    if (r.len < take) continue;
    const int off = r.off;
    r.off += take;
    r.len -= take;
    if (r.len == 0) p.free_list.erase(p.free_list.begin() + long(i));
    return off;
  }
  return -1;
}

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
  int off = take_free(p, take);
  if (off < 0) {
    if (p.used + take > kCapInts) {
      static bool warned = false;
      if (!warned) {
        warned = true;
        fprintf(stderr, "[tfserve] split-K counter pool for captured graphs is used up; "
                        "further captures reduce split-K in a separate launch\n");
      }
      return nullptr;
    }
    off = p.used;
    p.used += take;
  }
  if (g_owner != 0) p.owned[g_owner].push_back(Range{off, take});
  return p.base + off;
}

void splitk_counters_set_owner(int64_t owner) { g_owner = owner; }

int64_t splitk_counters_release(int64_t owner) {
  // no HIP call here: this runs from a Python finalizer on whatever thread
  // dropped the graph (possibly one that is capturing)
  std::lock_guard<std::mutex> g(g_mu);
  int64_t n = 0;
  const auto now = Clock::now();
  for (auto& kv : g_pools) {
    Pool& p = kv.second;
    auto it = p.owned.find(owner);
    if (it == p.owned.end()) continue;
    for (const Range& r : it->second) {
      p.pending.push_back(Pending{r, now});
      n += r.len;
    }
    p.owned.erase(it);
  }
  return n;
}

int64_t splitk_counters_pending() {
  std::lock_guard<std::mutex> g(g_mu);
  int64_t n = 0;
  for (auto& kv : g_pools)
    for (const Pending& q : kv.second.pending) n += q.r.len;
  return n;
}

int64_t splitk_counters_reclaim(double min_age_s) {
  std::lock_guard<std::mutex> g(g_mu);
  int64_t n = 0;
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return 0;
  const auto now = Clock::now();
  for (auto& kv : g_pools) {
    Pool& p = kv.second;
    if (p.pending.empty() || p.base == nullptr) continue;
    std::vector<Range> ready;
    std::vector<Pending> keep;
    for (const Pending& q : p.pending) {
      if (std::chrono::duration<double>(now - q.at).count() >= min_age_s) ready.push_back(q.r);
      else keep.push_back(q);
    }
    if (ready.empty()) continue;
    // zero them on a private non-blocking stream of that device and wait for
    // that memset only (no device-wide synchronize: the lanes keep replaying)
    if (hipSetDevice(kv.first) != hipSuccess) continue;
    hipStream_t zs = nullptr;
    bool ok = hipStreamCreateWithFlags(&zs, hipStreamNonBlocking) == hipSuccess;
    for (const Range& r : ready)
      ok = ok && hipMemsetAsync(p.base + r.off, 0, size_t(r.len) * sizeof(int), zs) == hipSuccess;
    ok = ok && hipStreamSynchronize(zs) == hipSuccess;
    if (zs != nullptr) hipStreamDestroy(zs);
    if (!ok) continue;                               // stay quarantined; retried next time
    p.pending.swap(keep);
    for (const Range& r : ready) {
      p.free_list.push_back(r);
      n += r.len;
    }
    // coalesce adjacent ranges (keeps first-fit effective over many cycles)
    std::sort(p.free_list.begin(), p.free_list.end(), [](const Range& a, const Range& b) { return a.off < b.off; });
    std::vector<Range> merged;
    for (const Range& r : p.free_list) {
      if (!merged.empty() && merged.back().off + merged.back().len == r.off) merged.back().len += r.len;
      else merged.push_back(r);
    }
    // a free range that ends at the bump pointer gives the space back to it
    if (!merged.empty() && merged.back().off + merged.back().len == p.used) {
      p.used = merged.back().off;
      merged.pop_back();
    }
    p.free_list.swap(merged);
  }
  hipSetDevice(cur);
  return n;
}

int64_t splitk_counters_captured_in_use() {
  std::lock_guard<std::mutex> g(g_mu);
  int64_t n = 0;
  for (auto& kv : g_pools) {
    n += kv.second.used;
    for (const Range& r : kv.second.free_list) n -= r.len;
    for (const Pending& q : kv.second.pending) n -= q.r.len;
  }
  return n;
}

}  // namespace tfsk
