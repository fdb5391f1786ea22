// Persistent dataflow executor (flow.h): a whole chain of conv / GEMM layers
// in ONE launch, for the small-batch buckets whose forward is a latency chain.
//
// Per task (one 32 x 64 output tile of one layer, or one K-slice of it):
//   1. ticket: one agent-scope atomicAdd on ctrl[0] (tasks are numbered in
//      program order, so every task a workgroup waits on is already held by
//      a running workgroup -- deadlock-free at any residency, beside the
//      other lanes' kernels too);
//   2. weights first: the first S-1 k-tiles of the task's weight slice go
//      into the LDS ring by direct-to-LDS DMA (buffer_load ... lds) BEFORE
//      the dependency wait -- weights are constants, so the prefetch overlaps
//      the producers' tail ("prefetch-credit", MI355X_MICROARCH.md);
//   3. dependency wait: lane 0 polls the producer layers' tile counters
//      (relaxed agent loads + s_sleep, bounded by a 0.5 s wall-clock timeout
//      that sets a sticky error flag instead of hanging), then ONE agent
//      acquire, vmcnt(0), and a workgroup barrier (the guide's consumer
//      recipe);
//   4. the activation operand (dense rows, im2col taps of an NHWC tensor with
//      padding / stride, or the dual [h | strided x] source of a projecting
//      bottleneck) streams through the rest of the ring, MFMA 16x16x32 bf16;
//   5. epilogue (bias, residual, ReLU) -> bf16 written with agent-scope
//      (write-through) stores, drained (vmcnt 0), then one lane adds 1 to the
//      counter of the tile's 32-row block (a consumer waits only on the
//      producer row blocks it reads: same rows, strided samples or the
//      im2col window): the 'sc1 payload + drained vmcnt + counter'
//      hand-off, no L2 write-back fence.  A K-sliced tile stores an fp32
//      slab instead; the slice that completes the tile's arrival counter sums
//      the slabs and runs the epilogue (cgemm's in-kernel fixup).
// The last workgroup to leave re-zeroes the ticket, the exit count and the
// exit count and advances the epoch the row-block counters are compared
// against, so a captured HIP graph can replay the launch as is.
#include <climits>
#include <cstdlib>

#include "gemm_common.h"
#include "flow.h"

namespace tfsk {

namespace {

using namespace gemm;

constexpr int BM = kFlowTileM, BN = kFlowTileN;
constexpr int NW = 4, NT = 64 * NW, S = 4;         // 4 waves (2 x 2 of 16 x 32), 4-slot ring
constexpr int WGM = 2, WGN = 2, WM = BM / WGM, WN = BN / WGN;
constexpr int TN = WN / 16;
constexpr int APW = BM / (8 * NW), BPW = BN / (8 * NW), PPW = APW + BPW;   // 1-KB DMA pieces per wave per slot
constexpr int A_ST = BM * KT, B_ST = BN * KT;                             // elements per ring slot
constexpr int LDS_MAIN = S * (A_ST + B_ST) * 2;                           // 48 KB
constexpr int CS_LD = BN + 4;
constexpr int LDS_EPI = BM * CS_LD * 4;
constexpr int LDS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
static_assert(APW == 1 && BPW == 2 && WM == 16 && TN == 2, "flow tile mapping");
static_assert(BM * (BN / 8) == NT, "one 8-column epilogue chunk per thread");
constexpr uint64_t kOffMask = (uint64_t(1) << kFlowRefShift) - 1;
constexpr uint64_t kWaitTicks = 50000000ull;   // 0.5 s of the 100-MHz wall clock

// (integer arithmetic: `nullptr + off` for the absolute kind would be UB, and
// the compiler used that to fold null checks of the decoded bias away)
__device__ __forceinline__ char* ref_ptr(int64_t r, char* arena, const char* entry, char* out) {
  const uint64_t kind = uint64_t(r) >> kFlowRefShift, off = uint64_t(r) & kOffMask;
  const uint64_t base = kind == 0 ? reinterpret_cast<uint64_t>(arena)
                        : kind == 1 ? reinterpret_cast<uint64_t>(entry)
                        : kind == 2 ? reinterpret_cast<uint64_t>(out) : 0ull;
  return reinterpret_cast<char*>(base + off);
}

// lane 0 only: wait until the wrapping counter *p has reached `target`
// (false on timeout)
__device__ __forceinline__ bool wait_count(int* p, uint32_t target, bool spin) {
  auto reached = [&] {
    return int(uint32_t(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) - target) >= 0;
  };
  if (reached()) return true;
  const uint64_t t0 = wall_clock64();
  for (;;) {
    if (!spin) __builtin_amdgcn_s_sleep(2);
    if (reached()) return true;
    if (wall_clock64() - t0 > kWaitTicks) return false;
  }
}

// Producer row blocks [lo, hi] holding the rows a consumer tile (output rows
// m0..m1 of step P) reads: rel 0 = the same rows (dense / dual h / residual),
// 1 = the strided 1x1 samples of P's [H][W] input (dual x), 2 = the im2col
// window (whole input rows ho*SH - PT .. + KH - 1, clamped).
__device__ __forceinline__ void dep_rows(const FlowStep& P, int rel, int m0, int m1, int& lo, int& hi) {
  if (rel == 0) {
    lo = m0 / BM;
    hi = m1 / BM;
    return;
  }
  const int hw = P.Ho * P.Wo;
  const int n0 = m0 / hw, r0 = m0 - n0 * hw, ho0 = r0 / P.Wo, wo0 = r0 - ho0 * P.Wo;
  const int n1 = m1 / hw, r1 = m1 - n1 * hw, ho1 = r1 / P.Wo, wo1 = r1 - ho1 * P.Wo;
  int a, b;
  if (rel == 1) {
    a = (n0 * P.H + ho0 * P.SH) * P.W + wo0 * P.SW;
    b = (n1 * P.H + ho1 * P.SH) * P.W + wo1 * P.SW;
  } else {
    const int h0 = max(0, ho0 * P.SH - P.PT), h1 = min(P.H - 1, ho1 * P.SH - P.PT + P.KH - 1);
    a = (n0 * P.H + h0) * P.W;
    b = (n1 * P.H + h1) * P.W + P.W - 1;
  }
  lo = a / BM;
  hi = b / BM;
}

__device__ __forceinline__ void store8_sc1(uint16_t* dst, const float (&v)[8]) {
  const uint32_t w[4] = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                         pack_bf16x2(v[6], v[7])};
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
  for (int e = 0; e < 4; ++e) __hip_atomic_store(d + e, w[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(NT) void flow_kernel(const char* __restrict__ table, int nsteps, int ntasks, char* arena,
                                                  const char* entry, char* outp, int* ctrl, int dbg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_task, s_last;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int prow = lane >> 3;
  const uint32_t kc = uint32_t(((lane & 7) ^ prow) * 8);
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t ra0 = uint32_t(((wm * WM + fr) * KT + ((fq ^ (fr & 7)) * 8)) * 2);
  const uint32_t ra1 = uint32_t(((wm * WM + fr) * KT + (((4 + fq) ^ (fr & 7)) * 8)) * 2);
  const uint32_t rb0 = uint32_t(((wn * WN + fr) * KT + ((fq ^ (fr & 7)) * 8)) * 2);
  const uint32_t rb1 = uint32_t(((wn * WN + fr) * KT + (((4 + fq) ^ (fr & 7)) * 8)) * 2);
  const int erow = tid >> 3, ecol = (tid & 7) * 8;     // this thread's epilogue chunk

  const int* starts = reinterpret_cast<const int*>(table);
  const FlowStep* steps = reinterpret_cast<const FlowStep*>(table + kFlowMaxSteps * 4);
  const int my_start = lane < nsteps ? starts[lane] : INT_MAX;
  const uint32_t epoch = uint32_t(__hip_atomic_load(ctrl + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));

  for (;;) {
    if (tid == 0) s_task = __hip_atomic_fetch_add(ctrl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds_barrier();
    const int t = __builtin_amdgcn_readfirstlane(s_task);
    if (t >= ntasks) break;
    const int si = __builtin_amdgcn_readfirstlane(int(__popcll(__ballot(my_start <= t))) - 1);
    const FlowStep& P = steps[si];

    // ---- task -> (tile, K slice)
    const int local = t - starts[si];
    const int splits = P.splits;
    const int split = local % splits, tile = local / splits;
    const int bm = tile / P.ntn, bn = tile - bm * P.ntn;
    const int m0 = bm * BM, n0 = bn * BN;
    const int M = P.M, N = P.N, mode = P.mode;
    const int kt0 = split * P.ktps;
    const int nk = min(P.K / KT - kt0, P.ktps);

    const char* A = ref_ptr(P.a, arena, entry, outp);
    const char* A2 = ref_ptr(P.a2, arena, entry, outp);
    const uint16_t* Wt = reinterpret_cast<const uint16_t*>(ref_ptr(P.w, arena, entry, outp));
    const float* bias = reinterpret_cast<const float*>(ref_ptr(P.bias, arena, entry, outp));
    const uint16_t* R = reinterpret_cast<const uint16_t*>(ref_ptr(P.res, arena, entry, outp));
    uint16_t* O = reinterpret_cast<uint16_t*>(ref_ptr(P.out, arena, entry, outp));
    float* ws = reinterpret_cast<float*>(ref_ptr(P.ws, arena, entry, outp));

    // ---- buffer descriptors (im2col: rebased by the top/left padding so every
    // in-image offset is non-negative; invalid taps read kOOB -> zeros)
    const char* abase = A;
    uint32_t arec = uint32_t(P.a_bytes);
    if (mode == kFlowIm2col) {
      const uint32_t shift = uint32_t((P.PT * P.W + P.PL) * P.C) * 2u;
      abase -= shift;
      arec += shift;
    }
    const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(abase), 0, int(arec), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsA2 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(mode == kFlowDual ? A2 : A), 0, mode == kFlowDual ? P.a2_bytes : P.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(Wt), 0, P.b_bytes, 0x00020000);

    // ---- this thread's 8 bias values (issued before every DMA: the ring's
    // vmcnt accounting only counts younger operations)
    float4 bias0, bias1;
    {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bias), 0, bias ? N * 4 : 0, 0x00020000);
      const int n = n0 + ecol;
      const uint32_t voff = n + 8 <= N ? uint32_t(n) * 4u : kOOB;
      bias0 = buffer_f4(rs, voff);
      bias1 = buffer_f4(rs, voff + 16u);
    }

    // ---- per-lane DMA offsets
    uint32_t a_off = kOOB, a_msk = 0, a_off2 = kOOB;
    {
      const int m = m0 + wid * 8 + prow;
      const bool ok = m < M;
      if (mode == kFlowDense) {
        a_off = ok ? (uint32_t(m) * uint32_t(P.lda) + kc) * 2u : kOOB;
      } else {
        const int mm = ok ? m : 0;
        const int hw = P.Ho * P.Wo;
        const int n = mm / hw, r = mm - n * hw;
        const int ho = r / P.Wo, wo = r - ho * P.Wo;
        if (mode == kFlowDual) {
          a_off = ok ? (uint32_t(m) * uint32_t(P.lda) + kc) * 2u : kOOB;
          a_off2 = ok ? (uint32_t((n * P.H + ho * P.SH) * P.W + wo * P.SW) * uint32_t(P.C) + kc) * 2u : kOOB;
        } else {
          const int hb = ho * P.SH, wb = wo * P.SW;
          a_off = (uint32_t((n * P.H + hb) * P.W + wb) * uint32_t(P.C) + kc) * 2u;
          const int hi0 = hb - P.PT, wi0 = wb - P.PL;
          uint32_t wbits = 0;
          for (int kw = 0; kw < P.KW; ++kw) wbits |= uint32_t((unsigned)(wi0 + kw) < (unsigned)P.W) << kw;
          uint32_t msk = 0;
          for (int kh = 0; kh < P.KH; ++kh)
            if ((unsigned)(hi0 + kh) < (unsigned)P.H) msk |= wbits << (kh * P.KW);
          a_msk = ok ? msk : 0u;
        }
      }
    }
    uint32_t b_off[BPW];
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      const int n = n0 + (wid * BPW + j) * 8 + prow;
      b_off[j] = n < N ? (uint32_t(n) * uint32_t(P.ldb) + kc) * 2u : kOOB;
    }

    // ---- producers: weight k-tiles and activation k-tiles walk separately
    // (the weights of the first S-1 tiles are issued before the dependency wait)
    int kb = kt0 * KT;
    auto issueB = [&](int slot) {
      const uint32_t soff = uint32_t(kb) * 2u;
#pragma unroll
      for (int j = 0; j < BPW; ++j) {
        const uint32_t v = b_off[j];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsB, (lds_ptr_t)(smem + (S * A_ST + slot * B_ST + (wid * BPW + j) * 512) * 2), 16, v, soff, 0, 0);
      }
      kb += KT;
    };
    int w_k = kt0 * KT, w_ci = 0, w_tap = 0, w_kh = 0, w_kw = 0;
    if (mode == kFlowIm2col) {
      w_tap = w_k / P.C;
      w_ci = w_k - w_tap * P.C;
      w_kh = w_tap / P.KW;
      w_kw = w_tap - w_kh * P.KW;
    }
    auto issueA = [&](int slot) {
      const lds_ptr_t dst = (lds_ptr_t)(smem + (slot * A_ST + wid * 512) * 2);
      if (mode == kFlowDual && w_k >= P.K1) {
        const uint32_t v = a_off2;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA2, dst, 16, v, uint32_t(w_k - P.K1) * 2u, 0, 0);
      } else if (mode == kFlowIm2col) {
        const uint32_t v = ((a_msk >> w_tap) & 1u) ? a_off : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, dst, 16, v, uint32_t((w_kh * P.W + w_kw) * P.C + w_ci) * 2u,
                                                 0, 0);
      } else {
        const uint32_t v = a_off;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, dst, 16, v, uint32_t(w_k) * 2u, 0, 0);
      }
      w_k += KT;
      if (mode == kFlowIm2col) {
        w_ci += KT;
        if (w_ci == P.C) {
          w_ci = 0;
          ++w_tap;
          if (++w_kw == P.KW) {
            w_kw = 0;
            ++w_kh;
          }
        }
      }
    };

#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (s < nk) issueB(s);

    // ---- dependency wait (lane 0), then acquire: the guide's consumer recipe
    if (tid == 0 && !(dbg & 2)) {
      bool ok = true;
      const int deps[3] = {P.dep_a, P.dep_a2, P.dep_res};
      const int rels[3] = {mode == kFlowIm2col ? 2 : 0, 1, 0};
      const int m1 = min(m0 + BM, M) - 1;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        if (deps[d] < 0) continue;
        const FlowStep& Q = steps[deps[d]];
        int lo, hi;
        dep_rows(P, rels[d], m0, m1, lo, hi);
        hi = min(hi, Q.ntm - 1);
        const uint32_t target = (epoch + 1u) * uint32_t(Q.ntn);
        for (int b = lo; b <= hi; ++b) ok = wait_count(ctrl + Q.rctr + b * kFlowRowStride, target, dbg & 4) && ok;
      }
      if (!ok) __hip_atomic_store(ctrl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!(dbg & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();

#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (s < nk) issueA(s);

    f32x4 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](int slot) {
      const char* sa = smem + slot * A_ST * 2;
      const char* sb = smem + (S * A_ST + slot * B_ST) * 2;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(sa + (kk ? ra1 : ra0));
        bf16x8 bfr[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sb + (kk ? rb1 : rb0) + j * 16 * KT * 2);
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[j], 0, 0, 0);
      }
    };

    // ---- main loop, unrolled by the ring depth.  Issue order: B(0..S-2),
    // A(0..S-2), then A+B of one slot per step; before tile t only the ops
    // issued after tile t's own may stay in flight: (S-2-t)*APW + t*PPW in the
    // first round (t <= S-2), (S-2)*PPW afterwards.
    for (int kt = 0; kt < nk; kt += S) {
#pragma unroll
      for (int u = 0; u < S; ++u) {
        const int t2 = kt + u;
        if (t2 < nk) {
          if (t2 + S - 2 >= nk) {
            wait_vmcnt<0>();
          } else if (kt == 0 && u == 0) {
            wait_vmcnt<(S - 2) * APW>();
          } else if (kt == 0 && u == 1) {
            wait_vmcnt<(S - 3) * APW + PPW>();
          } else {
            wait_vmcnt<(S - 2) * PPW>();
          }
          lds_barrier();
          if (t2 + S - 1 < nk) {
            issueA((u + S - 1) % S);
            issueB((u + S - 1) % S);
          }
          compute(u);
        }
      }
    }
    wait_vmcnt<0>();
    __syncthreads();

    // ---- epilogue: the fp32 tile through LDS, one 8-column chunk per thread
    float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(wm * WM + fq * 4 + r) * CS_LD + wn * WN + j * 16 + fr] = acc[j][r];
    __syncthreads();
    const int m = m0 + erow, n = n0 + ecol;
    const bool in = m < M && n + 8 <= N;
    float v[8];
    load8(Cs + erow * CS_LD + ecol, v);
    bool finish = true;
    if (splits > 1) {
      // this slice's raw partial (write-through), then the tile's arrival count
      float* slab = ws + (size_t(split) * M + m) * N + n;
      if (in) splitk_store8(slab, make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]));
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (tid == 0) {
        int* c = ctrl + P.ctr + tile;
        const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == splits - 1;
        if (s_last) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      finish = s_last != 0;
      if (finish && in) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.f;
        const float* src = ws + size_t(m) * N + n;
        for (int q = 0; q < splits; ++q)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            v[e] += __hip_atomic_load(src + size_t(q) * M * N + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (finish) {
      if (in) {
        const float bv[8] = {bias0.x, bias0.y, bias0.z, bias0.w, bias1.x, bias1.y, bias1.z, bias1.w};
        float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (R) {
          const uint4 rr = *reinterpret_cast<const uint4*>(R + size_t(m) * N + n);
          const uint32_t w[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            rv[2 * e] = __uint_as_float(w[e] << 16);
            rv[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
          }
        }
        const int act = P.act;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e] + bv[e] + rv[e], act);
        store8_sc1(O + size_t(m) * N + n, v);
      }
      // every wave's write-through stores have completed; one lane counts the tile
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(ctrl + P.rctr + bm * kFlowRowStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();   // LDS (Cs, s_task) is rewritten by the next task
  }

  // ---- the last workgroup out re-zeroes the ticket and the exit count and
  // advances the epoch (every workgroup read it when it started)
  if (tid == 0) {
    const int done = __hip_atomic_fetch_add(ctrl + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == int(gridDim.x) - 1) {
      __hip_atomic_store(ctrl + 0, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctrl + 3, int(epoch + 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctrl + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

// timing ablations (TFSERVE_FLOW_DBG, results are wrong with them): bit 0 skips
// the acquire fence, bit 1 the dependency waits; bit 2 polls without s_sleep
int dbg_flags() {
  static const int v = [] {
    const char* e = getenv("TFSERVE_FLOW_DBG");
    return e ? atoi(e) : 0;
  }();
  return v;
}

hipError_t flow_launch(const void* table, int nsteps, int ntasks, void* arena, const void* entry, void* out,
                       int* ctrl, int grid, hipStream_t stream) {
  if (nsteps <= 0 || nsteps > kFlowMaxSteps || ntasks <= 0 || grid <= 0 || ctrl == nullptr)
    return hipErrorInvalidValue;
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&flow_kernel), LDS);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(flow_kernel, dim3(grid), dim3(NT), LDS, stream, static_cast<const char*>(table), nsteps, ntasks,
                     static_cast<char*>(arena), static_cast<const char*>(entry), static_cast<char*>(out), ctrl, dbg_flags());
  return hipGetLastError();
}

}  // namespace tfsk
