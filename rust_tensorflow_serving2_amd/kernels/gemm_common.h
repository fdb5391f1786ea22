// Device helpers shared by the pipelined MFMA GEMM kernels (cgemm.hip,
// halo.hip) and the host-side per-device LDS attribute cache.
#pragma once
#include <mutex>
#include <set>
#include <tuple>

#include "common.h"
#include "launch.h"

namespace tfsk {

// hipFuncAttributeMaxDynamicSharedMemorySize is per (kernel, device): a
// process that drives several GPUs must set it on each.  Thread-safe; a set
// lookup under a mutex per launch (host side only, never inside a graph replay).
inline hipError_t ensure_dyn_lds(const void* fn, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  static std::mutex mu;
  static std::set<std::tuple<const void*, int, int>> done;
  std::lock_guard<std::mutex> g(mu);
  const auto key = std::make_tuple(fn, dev, bytes);
  if (done.count(key)) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.insert(key);
  return e;
}

namespace gemm {

constexpr int KT = 64;                    // k-tile depth (bf16) = 128 B per LDS row
constexpr uint32_t kOOB = 0x80000000u;    // voffset beyond any buffer: the DMA returns zeros

// a / d for 0 <= a < 2^24, d >= 1 via the float reciprocal `inv` = 1/d (one
// multiply + a +-1 fix-up, ~8 VALU instead of the ~35 of an integer division).
__device__ __forceinline__ int fdiv(int a, int d, float inv) {
  int q = int(float(a) * inv);
  const int r = a - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt at their maxima; gfx9 encoding).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Barrier without a vmcnt(0) drain: waits for this wave's own LDS reads
// (lgkmcnt(0)) and then meets the other waves.  The lgkmcnt wait matters: the
// compiler may leave the previous step's ds_reads in flight (their MFMAs sunk
// below the barrier), and the DMA issued right after the barrier refills that
// very ring slot -- found as run-to-run differences of chain.hip's output.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---- epilogue over the fp32 tile staged in LDS (8-column row chunks, NT threads)
// NTE = the threads that take part: a multiple of the chunks per row, so a
// thread's column is fixed (all NT unless BN / 8 does not divide NT, e.g. the
// 96-wide tiles); EXACT = every (thread, iteration) maps inside the tile.
template <int BM, int BN, int NT>
struct Epi {
  static constexpr int CPR = BN / 8;
  static constexpr int NTE = (NT / CPR) * CPR;
  static constexpr int ITERS = (BM * CPR + NTE - 1) / NTE;
  static constexpr bool EXACT = NTE == NT && (BM * CPR) % NT == 0;
  static constexpr int PRE = ITERS <= 8 ? ITERS : 0;
  static_assert(NTE > 0, "epilogue chunk mapping");
};

// chunk `it` of thread `tid`: row-major 8-column chunks, NTE apart (a thread's
// column is fixed); false when the chunk lies outside the tile
template <int BM, int BN, int NT>
__device__ __forceinline__ bool epi_rowcol(int tid, int it, int& row, int& col) {
  using E = Epi<BM, BN, NT>;
  const int c = tid + it * E::NTE;
  row = c / E::CPR;
  col = (c - row * E::CPR) * 8;
  return E::EXACT || (tid < E::NTE && row < BM);
}

// 16 B at byte offset `voff` of a buffer resource as float4 (an offset past the
// buffer's records -- kOOB, or any offset of a 0-record resource -- reads zeros)
__device__ __forceinline__ float4 buffer_f4(__amdgpu_buffer_rsrc_t rs, uint32_t voff) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// Workgroup phase trace (profiling only, p.trace == nullptr in production):
// stamp k of this workgroup = the steady wall clock (100 MHz), written by
// thread 0 with a vector store; stamp 0 also records the XCC / SE / CU id.
__device__ __forceinline__ void trace_stamp(const IGemmArgs& p, int k) {
  if (p.trace != nullptr && threadIdx.x == 0) {
    const long wgi = long(blockIdx.y) * gridDim.x + blockIdx.x;
    if (wgi < p.trace_cap) {
      long long* d = p.trace + wgi * 8;
      d[k] = wall_clock64();
      if (k == 0) d[7] = __smid();
    }
  }
}

// This thread's 8 bias values (its epilogue column is fixed), loaded before the
// K loop so the latency of the load hides under it.  Branch-free buffer loads:
// a guarded `if (ok) b = *p` became a conditional block whose register moves
// waited (vmcnt(0)) for the load -- and for every residual prefetch issued
// before it -- ahead of the first operand DMA, i.e. one full memory round trip
// per workgroup before its K loop could start (seen in the gfx950 ISA).
template <int BM, int BN, int NT>
__device__ __forceinline__ void prefetch_bias(const IGemmArgs& p, int n0, int tid, float4& b0, float4& b1) {
  int row0, col0;
  epi_rowcol<BM, BN, NT>(tid, 0, row0, col0);   // col0 < BN for every thread
  const int n = n0 + col0;
  const bool use = p.bias && p.splits <= 1 && p.N % 8 == 0;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.bias), 0, use ? p.N * 4 : 0, 0x00020000);
  const uint32_t voff = n + 8 <= p.N ? uint32_t(n) * 4u : kOOB;
  b0 = buffer_f4(rs, voff);
  b1 = buffer_f4(rs, voff + 16u);
}

// Split-K without a reduce launch: every slice stores its fp32 slab with
// agent-scope (write-through) stores, waits for them to complete, and counts
// its arrival; the slice whose arrival completes tile `t` gets true (the others
// false), re-zeroes the counter for the next launch and reads the slabs back
// with agent-scope loads.  No __threadfence: on gfx950 its release writes back
// the whole L2 and its acquire invalidates it, which made the fixed-up layers
// slower than a separate reduce launch (MI355X_MICROARCH.md 'handoff-flag':
// write-through payload + drained vmcnt + flag).
// The split-K workspace (splits slabs of M x N fp32) as a buffer resource.
// Slab stores and the last slice's slab loads are 16-B buffer accesses with
// the sc1 cache policy (aux 16): agent-coherent, i.e. written through / read
// past the XCD's own L2, which other XCDs' workgroups do not see -- the same
// encoding `__hip_atomic_store/load(..., __HIP_MEMORY_SCOPE_AGENT)` gets, but
// 16 B per lane instead of one dword (8x fewer instructions; the per-dword
// form made a split tile's fixup epilogue 3-7 us, profiles/round4/s9).
constexpr int kCpolAgent = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t splitk_rsrc(const IGemmArgs& p) {
  const long bytes = long(p.splits) * p.M * p.N * 4;
  return __builtin_amdgcn_make_buffer_rsrc(p.ws, 0, int(bytes < 0x7fffffffL ? bytes : 0x7fffffffL), 0x00020000);
}

// 8 fp32 partials of this slice (blockIdx.y) at (m, n), agent-coherent.
__device__ __forceinline__ void splitk_store8(const IGemmArgs& p, __amdgpu_buffer_rsrc_t rs, int m, int n,
                                              const float4 a, const float4 b) {
  const uint32_t voff = (uint32_t(m) * uint32_t(p.N) + uint32_t(n)) * 4u;
  const uint32_t soff = uint32_t(blockIdx.y) * uint32_t(p.M) * uint32_t(p.N) * 4u;
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), rs, voff, soff, kCpolAgent);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, b), rs, voff + 16u, soff, kCpolAgent);
}

__device__ __forceinline__ bool splitk_arrive(const IGemmArgs& p, int t) {
  __shared__ int s_last;
  __builtin_amdgcn_s_waitcnt(0);          // this thread's slab stores have completed
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(p.counters + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == p.splits - 1;
    if (s_last) __hip_atomic_store(p.counters + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return s_last;
}

// Sum of the `splits` slabs for 8 columns at (m, n): agent-coherent loads,
// four slices per round all in flight at once (slices past `splits` read
// past the descriptor's records: zeros).  A rolled one-slice-per-trip loop
// paid a full memory-side round trip per slice: the last arriver's epilogue
// took ~5 us at 4 slices (profiles/round4/s10).
__device__ __forceinline__ void splitk_sum8(const IGemmArgs& p, __amdgpu_buffer_rsrc_t rs, int m, int n,
                                            float4& lo, float4& hi) {
  constexpr int NS = 4;
  const uint32_t voff = (uint32_t(m) * uint32_t(p.N) + uint32_t(n)) * 4u;
  const uint32_t slab = uint32_t(p.M) * uint32_t(p.N) * 4u;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < p.splits; s0 += NS) {
    u32x4 a[NS], b[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const uint32_t soff = uint32_t(min(s0 + j, p.splits)) * slab;
      a[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, kCpolAgent);
      b[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16u, soff, kCpolAgent);
    }
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const float4 x = __builtin_bit_cast(float4, a[j]), y = __builtin_bit_cast(float4, b[j]);
      v[0] += x.x; v[1] += x.y; v[2] += x.z; v[3] += x.w;
      v[4] += y.x; v[5] += y.y; v[6] += y.z; v[7] += y.w;
    }
  }
  lo = make_float4(v[0], v[1], v[2], v[3]);
  hi = make_float4(v[4], v[5], v[6], v[7]);
}

// Two floats -> packed bf16 pair (round-to-nearest-even; a plain __bf16 cast
// compiles to one v_cvt_pk_bf16_f32 on gfx950 and keeps NaNs NaN).
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const __bf16 lo = static_cast<__bf16>(a), hi = static_cast<__bf16>(b);
  return uint32_t(__builtin_bit_cast(uint16_t, lo)) | (uint32_t(__builtin_bit_cast(uint16_t, hi)) << 16);
}

// 8 values -> one 16-B bf16 (or 2 x 16-B f32) store at row m, column n of `out`
// (nullptr: nothing stored)
__device__ __forceinline__ void store_chunk(const IGemmArgs& p, void* out, int m, int n, const float (&v)[8]) {
  if (!out) return;
  if (p.out_f32) {
    float* o = static_cast<float*>(out) + size_t(m) * p.ldc + n;
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(out) + size_t(m) * p.ldc + n) =
        make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                   pack_bf16x2(v[6], v[7]));
  }
}

// The post-activation output: out2 = act2(v * scale2 + shift2) (per channel;
// scale2 / shift2 are L2-resident and read per chunk rather than prefetched,
// so kernels without a second output pay no registers for it).
__device__ __forceinline__ void post_chunk(const IGemmArgs& p, int m, int n, const float (&v)[8]) {
  const float4 s0 = *reinterpret_cast<const float4*>(p.scale2 + n);
  const float4 s1 = *reinterpret_cast<const float4*>(p.scale2 + n + 4);
  const float4 t0 = *reinterpret_cast<const float4*>(p.shift2 + n);
  const float4 t1 = *reinterpret_cast<const float4*>(p.shift2 + n + 4);
  const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float sh[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
  float w[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = v[e] * sc[e] + sh[e];
    w[e] = p.act2 == kActRelu ? fmaxf(x, 0.f) : x;
  }
  store_chunk(p, p.out2, m, n, w);
}

// One 8-column chunk: alpha * acc + bias (+ residual) -> act -> 16-B bf16 (or
// 2 x 16-B f32) store (+ the post-activation output).  The launchers
// guarantee N, ldc, ldr % 8 == 0.
template <int ACT>
__device__ __forceinline__ void epi_chunk(const IGemmArgs& p, const float* src, int m, int n, const float (&bv)[8],
                                          const uint4 rr) {
  const float4 lo = *reinterpret_cast<const float4*>(src);
  const float4 hi = *reinterpret_cast<const float4*>(src + 4);
  float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  const uint32_t w[4] = {rr.x, rr.y, rr.z, rr.w};
  const float alpha = p.alpha;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = act_fn<ACT>(v[2 * e] * alpha + bv[2 * e] + __uint_as_float(w[e] << 16));
    v[2 * e + 1] = act_fn<ACT>(v[2 * e + 1] * alpha + bv[2 * e + 1] + __uint_as_float(w[e] & 0xffff0000u));
  }
  store_chunk(p, p.out, m, n, v);
  if (p.out2) post_chunk(p, m, n, v);
}

// ---- deferred LayerNorm (IGemmArgs::st_out / a_st / r_st)
// (mean, rstd) of row m from its `parts` (sum, sum of squares) partials.
// One-pass variance in fp32 over bf16 values: E[x^2] - mean^2 loses
// ~eps_f32 * E[x^2] / var relative, i.e. nothing while |mean| is within a few
// standard deviations (LayerNorm inputs: residual streams).
__device__ __forceinline__ float2 ln_row_stats(const float* st, int parts, int m, float inv_len, float eps) {
  const float2* s = reinterpret_cast<const float2*>(st) + size_t(m) * parts;
  float a = 0.f, b = 0.f;
#pragma unroll 4
  for (int j = 0; j < parts; ++j) {
    const float2 v = s[j];
    a += v.x;
    b += v.y;
  }
  const float mean = a * inv_len;
  return make_float2(mean, rsqrtf(fmaxf(b * inv_len - mean * mean, 0.f) + eps));
}

// 8 consecutive fp32 values at p (16-B aligned) into registers
__device__ __forceinline__ void load8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

}  // namespace gemm
}  // namespace tfsk
