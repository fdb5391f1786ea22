// Implicit-GEMM convolution / GEMM for MI355X (gfx950), bf16 in, fp32 MFMA accumulate.
//
// C[M][N] = epilogue( A[M][K] * B[N][K]^T )
//   A: NHWC activations gathered on the fly (im2col never materialised), a dense
//      row-major matrix, or (stem) the fp32 request tensor itself — the ingest
//      fp32->bf16 cast is fused into the stem conv's operand load.
//   B: weights [Cout][K] bf16 (BN scale folded in at load time).
//   epilogue: *alpha + bias[n] (+ residual[m][n]) -> act -> bf16/f32 store.
//
// CDNA4 mapping:
//   * 256-thread workgroups = 4 wave64s in a 2x2 grid; each wave owns a
//     (BM/2)x(BN/2) sub-tile built from v_mfma_f32_16x16x32_bf16 tiles.
//   * BK = 64: each tile row is 128 B; 16-B chunks are XOR-swizzled by
//     (row & 7) so the ds_read_b128 fragment reads of a 16-lane group hit 16
//     distinct 16-B bank slots (conflict-free; see MI355X LDS banking).
//   * register-staged double-buffered LDS: the global loads of k-tile t+1 are
//     issued before the MFMAs of tile t and written to the other LDS buffer
//     after them -> one barrier per k-tile.
//   * bijective XCD-aware block remap + GROUP_M tile ordering so tiles that
//     share operand panels run on the same XCD (shared 4 MB L2).
//   * epilogue staged through LDS as fp32 so bias/residual/activation work on
//     coalesced 16-B row chunks (residual read once, output written once).
#include "common.h"
#include "gemm_common.h"
#include "launch.h"

namespace tfsk {

namespace {

constexpr int BK = 64;
constexpr int kThreads = 256;
constexpr int kGroupM = 8;

template <int BM, int BN, int AMODE, int NSTAGE, int WAVES_M = 2, int BKT = 64>
struct IGemm {
  // 4 waves in a WAVES_M x (4 / WAVES_M) grid, each owning a WM x WN sub-tile
  static constexpr int WAVES_N = 4 / WAVES_M;
  static constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  static constexpr int TM = WM / 16, TN = WN / 16;
  // direct-to-LDS modes may use deeper k-tiles (BK = 128 / 256): fewer barriers
  // and DMA round trips per MFMA; register-staged modes keep BK = 64
  static constexpr bool GL_ = (AMODE == kADense || AMODE == kAIm2col);
  static constexpr int BK = GL_ ? BKT : 64;
  static constexpr int CPR = BK / 8;                    // 16-B chunks per LDS row
  static constexpr int RPI = 64 / CPR;                  // rows per wave DMA instruction (1 KB)
  static constexpr int SWZ = CPR >= 16 ? 15 : 7;        // XOR swizzle mask (conflict-free b128 reads)
  static constexpr int A_CHUNKS = BM * BK / 8 / kThreads;
  static constexpr int B_CHUNKS = BN * BK / 8 / kThreads;
  // direct-to-LDS operand modes run a STAGES-deep DMA ring (S-1 k-tiles in
  // flight while one is consumed): per k-tile a 64x64 tile does only ~128
  // MFMA cycles per SIMD, far below one memory round trip, so two buffers
  // leave the loop latency-bound.  Register-staged modes keep 2 buffers.
  static constexpr bool GL = (AMODE == kADense || AMODE == kAIm2col);
  static constexpr int STAGES = GL ? NSTAGE : 2;
  static constexpr int PER_STAGE = A_CHUNKS + B_CHUNKS;   // DMA instructions per stage per wave
  static constexpr int LDS_MAIN = STAGES * (BM + BN) * BK * 2;
  static constexpr int CS_LD = BN + 4;
  static constexpr int LDS_EPI = BM * CS_LD * 4;
  static constexpr int LDS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
};


// s_waitcnt vmcnt(N) only (expcnt/lgkmcnt left at their maxima; gfx9 encoding:
// vmcnt[3:0] + vmcnt[5:4] at bits 15:14, expcnt 6:4, lgkmcnt 11:8).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Workgroup barrier WITHOUT the vmcnt(0) drain that __syncthreads' fence
// implies (that drain would empty the DMA ring every k-tile).  The "memory"
// clobber keeps the compiler from moving LDS accesses across it; LDS reads
// feeding MFMAs have already been waited on by then.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_barrier" ::: "memory"); }

// Epilogue over the fp32 tile staged in LDS: coalesced 8-column row chunks,
// alpha * acc + bias (+ residual) -> activation -> bf16 / f32 store.
// Chunk `it` of this thread: row-major 8-column chunks, kThreads apart; since
// kThreads is a multiple of the chunks per row, a thread's column never changes.
template <int BM, int BN>
struct EpiMap {
  static constexpr int CPR = BN / 8;
  static constexpr int ITERS = BM * CPR / kThreads;
  static_assert(kThreads % CPR == 0 && (BM * CPR) % kThreads == 0, "epilogue chunk mapping");
  static constexpr int PRE = ITERS <= 8 ? ITERS : 0;   // residual chunks prefetched into registers
};

template <int BM, int BN>
__device__ __forceinline__ void epi_rowcol(int tid, int it, int& row, int& col) {
  constexpr int CPR = BN / 8;
  const int c = tid + it * kThreads;
  row = c / CPR;
  col = (c - row * CPR) * 8;
}

// Issue the residual loads of this thread's epilogue chunks early (before the
// K loop) so their latency hides under the operand DMA and the MFMAs.
template <int BM, int BN>
__device__ __forceinline__ void prefetch_residual(const IGemmArgs& p, int m0, int n0, int tid,
                                                  uint4 (&rpre)[EpiMap<BM, BN>::PRE > 0 ? EpiMap<BM, BN>::PRE : 1]) {
  constexpr int PRE = EpiMap<BM, BN>::PRE;
  if (PRE == 0 || !p.residual || p.splits > 1 || (p.N % 8) || (p.ldr % 8)) return;
#pragma unroll
  for (int it = 0; it < PRE; ++it) {
    int row, col;
    epi_rowcol<BM, BN>(tid, it, row, col);
    const int m = m0 + row, n = n0 + col;
    rpre[it] = (m < p.M && n + 8 <= p.N) ? *reinterpret_cast<const uint4*>(p.residual + size_t(m) * p.ldr + n)
                                          : make_uint4(0, 0, 0, 0);
  }
}

template <int BM, int BN, int CS_LD, int ACT>
__device__ __forceinline__ void epilogue_rows(const IGemmArgs& p, const float* Cs, int m0, int n0, int tid,
                                              const uint4 (&rpre)[EpiMap<BM, BN>::PRE > 0 ? EpiMap<BM, BN>::PRE : 1]) {
  using EM = EpiMap<BM, BN>;
  const int M = p.M, N = p.N;
  const float alpha = p.alpha;
  const bool vec_ok = (N % 8 == 0) && (p.ldc % 8 == 0) && (!p.residual || p.ldr % 8 == 0);
  // bias: fixed column per thread -> loaded once
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  {
    int row0, col0;
    epi_rowcol<BM, BN>(tid, 0, row0, col0);
    const int n = n0 + col0;
    if (p.bias && vec_ok && n + 8 <= N) {
      const float4 b0 = *reinterpret_cast<const float4*>(p.bias + n);
      const float4 b1 = *reinterpret_cast<const float4*>(p.bias + n + 4);
      bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
      bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
    }
  }
  // cheap activations: fully unrolled, residual from prefetched registers;
  // GELU / tanh: rolled (the transcendental expansion is emitted once, not
  // ITERS x 8 times — it used to make this kernel tens of thousands of
  // instructions, far beyond the instruction cache)
  auto chunk = [&](int it, bool use_pre) {
    int row, col;
    epi_rowcol<BM, BN>(tid, it, row, col);
    const int m = m0 + row, n = n0 + col;
    if (m >= M || n >= N) return;
    const float4 lo = *reinterpret_cast<const float4*>(Cs + row * CS_LD + col);
    const float4 hi = *reinterpret_cast<const float4*>(Cs + row * CS_LD + col + 4);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    if (vec_ok && n + 8 <= N) {
      float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (p.residual) {
        const uint4 rr = (EM::PRE > 0 && use_pre) ? rpre[EM::PRE > 0 ? it : 0]
                                     : *reinterpret_cast<const uint4*>(p.residual + size_t(m) * p.ldr + n);
        const uint32_t w[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          rv[2 * e] = bf16_to_f32(uint16_t(w[e] & 0xffff));
          rv[2 * e + 1] = bf16_to_f32(uint16_t(w[e] >> 16));
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = act_fn<ACT>(v[e] * alpha + bv[e] + rv[e]);
      if (p.out_f32) {
        float* o = static_cast<float*>(p.out) + size_t(m) * p.ldc + n;
        *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        uint16_t b[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) b[e] = f32_to_bf16(v[e]);
        *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p.out) + size_t(m) * p.ldc + n) =
            make_uint4(b[0] | (uint32_t(b[1]) << 16), b[2] | (uint32_t(b[3]) << 16),
                       b[4] | (uint32_t(b[5]) << 16), b[6] | (uint32_t(b[7]) << 16));
      }
    } else {
      for (int e = 0; e < 8 && n + e < N; ++e) {
        float x = v[e] * alpha;
        if (p.bias) x += p.bias[n + e];
        if (p.residual) x += bf16_to_f32(p.residual[size_t(m) * p.ldr + n + e]);
        x = act_fn<ACT>(x);
        if (p.out_f32) static_cast<float*>(p.out)[size_t(m) * p.ldc + n + e] = x;
        else static_cast<uint16_t*>(p.out)[size_t(m) * p.ldc + n + e] = f32_to_bf16(x);
      }
    }
  };
  if constexpr (ACT == 0 || ACT == kActRelu) {
#pragma unroll
    for (int it = 0; it < EM::ITERS; ++it) chunk(it, true);
  } else {
#pragma unroll 1
    for (int it = 0; it < EM::ITERS; ++it) chunk(it, false);
  }
}

template <int BM, int BN, int AMODE, int NSTAGE, int WAVES_M, int BKT>
__global__ __launch_bounds__(kThreads, 2) void igemm_kernel(IGemmArgs p) {
  using G = IGemm<BM, BN, AMODE, NSTAGE, WAVES_M, BKT>;
  constexpr int BK = G::BK;
  auto swz = [](int row, int ch) { return ch ^ (row & G::SWZ); };
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int S = G::STAGES;
  uint16_t* As = reinterpret_cast<uint16_t*>(smem);
  uint16_t* Bs = As + S * BM * BK;

  const int M = p.M, N = p.N, K = p.K;
  const int nbm = (M + BM - 1) / BM, nbn = (N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = kGroupM * nbn;
  const int group = wg / per_group;
  const int first_m = group * kGroupM;
  const int gsz = min(nbm - first_m, kGroupM);
  const int bm = first_m + (wg % per_group) % gsz;
  const int bn = (wg % per_group) / gsz;
  const int m0 = bm * BM, n0 = bn * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / G::WAVES_N, wn = wid % G::WAVES_N;
  const int chunk = tid & 7;
  const int row_base = tid >> 3;   // 0..31
  // Direct-to-LDS staging (dense / im2col operands): each wave instruction
  // DMAs 64 lanes x 16 B = 8 rows x 128 B into a lane-linear LDS image, so
  // lane l fills row (l>>3) at 16-B slot (l&7); the XOR swizzle is applied to
  // the *source* chunk instead (logical chunk = slot ^ (row & 7)).
  constexpr bool GL = G::GL;
  // DMA lane -> (row within the 1-KB instruction block, 16-B slot); the slot
  // holds logical chunk slot ^ (row & SWZ) (the swizzle applied at the source)
  const int gl_row = lane / G::CPR, gl_slot = lane % G::CPR;
  auto gl_chunk_of = [&](int i) { return gl_slot ^ ((i * G::RPI + gl_row) & G::SWZ); };

  // ---- per-thread A row descriptors
  int a_off[G::A_CHUNKS];     // element offset of the row's base (dense: m*lda; im2col: image base)
  int a_hi[G::A_CHUNKS], a_wi[G::A_CHUNKS];
  bool a_ok[G::A_CHUNKS];
#pragma unroll
  for (int i = 0; i < G::A_CHUNKS; ++i) {
    const int rloc = GL ? wid * (BM / 4) + i * G::RPI + gl_row : row_base + 32 * i;
    const int m = m0 + rloc;
    a_ok[i] = m < M;
    const int mm = a_ok[i] ? m : 0;
    if (AMODE == kADense) {
      a_off[i] = mm * p.lda;
      a_hi[i] = a_wi[i] = 0;
    } else {
      const int hw = p.Ho * p.Wo;
      const int n = mm / hw, r = mm - n * hw;
      const int ho = r / p.Wo, wo = r - ho * p.Wo;
      a_off[i] = n * p.H * p.W * p.C;
      a_hi[i] = ho * p.SH - p.PT;
      a_wi[i] = wo * p.SW - p.PL;
    }
  }

  uint4 ra[G::A_CHUNKS], rb[G::B_CHUNKS];
  const uint16_t* __restrict__ Bg = p.b;

  auto gload = [&](int kt) {
    const int k0 = kt * BK;
    if (AMODE == kADense) {
      const uint16_t* __restrict__ Ag = static_cast<const uint16_t*>(p.a);
      const int k = k0 + chunk * 8;
#pragma unroll
      for (int i = 0; i < G::A_CHUNKS; ++i) {
        if (a_ok[i] && k < K) ra[i] = *reinterpret_cast<const uint4*>(Ag + a_off[i] + k);
        else ra[i] = make_uint4(0, 0, 0, 0);
      }
    } else if (AMODE == kAIm2col) {
      const uint16_t* __restrict__ Ag = static_cast<const uint16_t*>(p.a);
      // C % 8 == 0, so a 16-B chunk never straddles two filter taps
      const int k = k0 + chunk * 8;
      const int tap = k / p.C;
      const int ci = k - tap * p.C;
      const int kh = tap / p.KW, kw = tap - kh * p.KW;
      const bool kok = k < K;
#pragma unroll
      for (int i = 0; i < G::A_CHUNKS; ++i) {
        const int hi = a_hi[i] + kh, wi = a_wi[i] + kw;
        const bool ok = kok && a_ok[i] && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
        if (ok) ra[i] = *reinterpret_cast<const uint4*>(Ag + a_off[i] + (hi * p.W + wi) * p.C + ci);
        else ra[i] = make_uint4(0, 0, 0, 0);
      }
    } else if (AMODE == kAC4) {
      const uint16_t* __restrict__ Ag = static_cast<const uint16_t*>(p.a);
      const int k = k0 + chunk * 8;
      const int kh = k >> 5, kw = (k & 31) >> 2;   // kw even: taps kw, kw+1
      const bool kok = kh < p.KH;
      const bool t1ok = kw + 1 < p.KW;
#pragma unroll
      for (int i = 0; i < G::A_CHUNKS; ++i) {
        const int hi = a_hi[i] + kh, wi = a_wi[i] + kw;
        const bool rok = kok && a_ok[i] && (unsigned)hi < (unsigned)p.H;
        const uint16_t* rowp = Ag + a_off[i] + hi * p.W * 4;
        uint2 t0 = make_uint2(0, 0), t1 = make_uint2(0, 0);
        if (rok && kw < p.KW && (unsigned)wi < (unsigned)p.W) t0 = *reinterpret_cast<const uint2*>(rowp + wi * 4);
        if (rok && t1ok && (unsigned)(wi + 1) < (unsigned)p.W)
          t1 = *reinterpret_cast<const uint2*>(rowp + (wi + 1) * 4);
        ra[i] = make_uint4(t0.x, t0.y, t1.x, t1.y);
      }
    } else if (AMODE == kAStem7x7x3) {
      // k = kh*21 + j, j = kw*3 + c: for a fixed kh the 21 operands of one output
      // pixel are 21 *contiguous* floats of input row hi (cols wi0..wi0+6, 3 ch),
      // so only kh needs a (constant) division and one bounds test per element.
      const float* __restrict__ Ag = static_cast<const float*>(p.a);
      const int W3 = p.W * 3;
#pragma unroll
      for (int i = 0; i < G::A_CHUNKS; ++i) {
        uint16_t v[8];
        const float* rowp = Ag + a_off[i] + a_wi[i] * 3;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = k0 + chunk * 8 + e;
          const int kh = k / 21, j = k - kh * 21;
          const int hi = a_hi[i] + kh, wi = a_wi[i] + j / 3;
          float x = 0.f;
          if (a_ok[i] && k < 147 && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
            x = rowp[hi * W3 + j];
          v[e] = f32_to_bf16(x);
        }
        ra[i] = make_uint4(v[0] | (uint32_t(v[1]) << 16), v[2] | (uint32_t(v[3]) << 16),
                           v[4] | (uint32_t(v[5]) << 16), v[6] | (uint32_t(v[7]) << 16));
      }
    } else {  // kAStemF32: fp32 NHWC, tiny C, element gather + cast
      const float* __restrict__ Ag = static_cast<const float*>(p.a);
#pragma unroll
      for (int i = 0; i < G::A_CHUNKS; ++i) {
        uint16_t v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int k = k0 + chunk * 8 + e;
          float x = 0.f;
          if (a_ok[i] && k < K) {
            const int tap = k / p.C, c = k - tap * p.C;
            const int kh = tap / p.KW, kw = tap - kh * p.KW;
            const int hi = a_hi[i] + kh, wi = a_wi[i] + kw;
            if ((unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
              x = Ag[a_off[i] + (hi * p.W + wi) * p.C + c];
          }
          v[e] = f32_to_bf16(x);
        }
        ra[i] = make_uint4(v[0] | (uint32_t(v[1]) << 16), v[2] | (uint32_t(v[3]) << 16),
                           v[4] | (uint32_t(v[5]) << 16), v[6] | (uint32_t(v[7]) << 16));
      }
    }
    {
      const int k = k0 + chunk * 8;
#pragma unroll
      for (int i = 0; i < G::B_CHUNKS; ++i) {
        const int n = n0 + row_base + 32 * i;
        if (n < N && k < p.ldb) rb[i] = *reinterpret_cast<const uint4*>(Bg + size_t(n) * p.ldb + k);
        else rb[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };

  // buffer descriptors: out-of-range offsets read as 0 (conv padding, M/N/K tails)
  constexpr uint32_t kOOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.a), 0, int(p.a_bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(p.b), 0, int(p.b_bytes), 0x00020000);
  typedef __attribute__((address_space(3))) void* lds_ptr_t;

  // Per-lane byte offsets precomputed once: every k-tile then costs one add per
  // 16-B chunk (out-of-range rows keep a kOOB base, which stays out of range
  // after adding k offsets).  K tails are checked only in the last k-tile.
  uint32_t b_base[G::B_CHUNKS];
  int b_kofs[G::B_CHUNKS];        // this lane's k offset within a k-tile (elements)
#pragma unroll
  for (int i = 0; i < G::B_CHUNKS; ++i) {
    const int n = n0 + wid * (BN / 4) + i * G::RPI + gl_row;
    b_kofs[i] = gl_chunk_of(i) * 8;
    b_base[i] = n < N ? (uint32_t(n) * uint32_t(p.ldb) + uint32_t(b_kofs[i])) * 2u : kOOB;
  }
  uint32_t a_base[G::A_CHUNKS];   // dense: row base; im2col: pixel base (tap 0, channel chunk)
  int a_kofs[G::A_CHUNKS];
#pragma unroll
  for (int i = 0; i < G::A_CHUNKS; ++i) {
    a_kofs[i] = gl_chunk_of(i) * 8;
    if (AMODE == kADense)
      a_base[i] = a_ok[i] ? uint32_t(a_off[i] + a_kofs[i]) * 2u : kOOB;
    else if (AMODE == kAIm2col)
      a_base[i] = uint32_t(a_off[i] + (a_hi[i] * p.W + a_wi[i]) * p.C + a_kofs[i]) * 2u;
    else
      a_base[i] = 0;
  }
  // im2col with C % 64 == 0: one k-tile = one tap's 64-channel slice.  The
  // tap walk (channel offset, kw, kh) advances incrementally in scalar regs.
  const bool c_tiles = (AMODE == kAIm2col) && (p.C % BK == 0);
  int t_ci = 0, t_kw = 0, t_kh = 0;
  auto tap_seek = [&](int kt) {       // (only for the first stage / split-K start)
    const int kc0 = kt * BK;
    const int tap = kc0 / p.C;
    t_ci = kc0 - tap * p.C;
    t_kh = tap / p.KW;
    t_kw = tap - t_kh * p.KW;
  };

  auto gstage = [&](int buf, int kt, bool live) {
    const int kc0 = kt * BK;                 // wave-uniform
    uint16_t* as = As + buf * BM * BK;
    uint16_t* bs = Bs + buf * BN * BK;
    if (AMODE == kADense) {
      const bool tail = kc0 + BK > K;
#pragma unroll
      for (int i = 0; i < G::A_CHUNKS; ++i) {
        uint32_t off = a_base[i] + uint32_t(kc0) * 2u;
        if (!live || (tail && kc0 + a_kofs[i] >= K)) off = kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_ptr_t)(as + (wid * (BM / 4) + i * G::RPI) * BK), 16,
                                                 off, 0, 0, 0);
      }
    } else if (c_tiles) {
      const int tap_off = (t_kh * p.W + t_kw) * p.C + t_ci;
      const bool kok = live && kc0 < K;
#pragma unroll
      for (int i = 0; i < G::A_CHUNKS; ++i) {
        const bool ok = kok && a_ok[i] && (unsigned)(a_hi[i] + t_kh) < (unsigned)p.H &&
                        (unsigned)(a_wi[i] + t_kw) < (unsigned)p.W;
        const uint32_t off = ok ? a_base[i] + uint32_t(tap_off) * 2u : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_ptr_t)(as + (wid * (BM / 4) + i * G::RPI) * BK), 16,
                                                 off, 0, 0, 0);
      }
      // advance to the next k-tile's tap slice
      t_ci += BK;
      if (t_ci == p.C) {
        t_ci = 0;
        if (++t_kw == p.KW) {
          t_kw = 0;
          ++t_kh;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < G::A_CHUNKS; ++i) {
        const int kc = kc0 + a_kofs[i];
        const int tap = kc / p.C;
        const int ci = kc - tap * p.C;
        const int kh = tap / p.KW, kw = tap - kh * p.KW;
        const int hi = a_hi[i] + kh, wi = a_wi[i] + kw;
        const bool ok = live && kc < K && a_ok[i] && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W;
        const uint32_t off = ok ? uint32_t(a_off[i] + (hi * p.W + wi) * p.C + ci) * 2u : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_ptr_t)(as + (wid * (BM / 4) + i * G::RPI) * BK), 16,
                                                 off, 0, 0, 0);
      }
    }
    const bool btail = kc0 + BK > p.ldb;
#pragma unroll
    for (int i = 0; i < G::B_CHUNKS; ++i) {
      uint32_t off = b_base[i] + uint32_t(kc0) * 2u;
      if (!live || (btail && kc0 + b_kofs[i] >= p.ldb)) off = kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_ptr_t)(bs + (wid * (BN / 4) + i * G::RPI) * BK), 16, off,
                                               0, 0, 0);
    }
  };

  auto sstore = [&](int buf) {
    uint16_t* as = As + buf * BM * BK;
    uint16_t* bs = Bs + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < G::A_CHUNKS; ++i) {
      const int row = row_base + 32 * i;
      *reinterpret_cast<uint4*>(as + row * BK + swz(row, chunk) * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < G::B_CHUNKS; ++i) {
      const int row = row_base + 32 * i;
      *reinterpret_cast<uint4*>(bs + row * BK + swz(row, chunk) * 8) = rb[i];
    }
  };

  f32x4 acc[G::TM][G::TN];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 rpre[EpiMap<BM, BN>::PRE > 0 ? EpiMap<BM, BN>::PRE : 1];
  prefetch_residual<BM, BN>(p, m0, n0, tid, rpre);

  const int nk_all = (K + BK - 1) / BK;
  const int kt0 = p.splits > 1 ? blockIdx.y * p.kt_per_split : 0;
  const int nk = p.splits > 1 ? min(nk_all, kt0 + p.kt_per_split) - kt0 : nk_all;
  const int fr = lane & 15, fq = lane >> 4;

  auto mfma_tile = [&](const uint16_t* as, const uint16_t* bs) {
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int ch = kk * 4 + fq;
      bf16x8 af[G::TM], bfr[G::TN];
#pragma unroll
      for (int i = 0; i < G::TM; ++i) {
        const int row = wm * G::WM + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(as + row * BK + swz(row, ch) * 8);
      }
#pragma unroll
      for (int j = 0; j < G::TN; ++j) {
        const int row = wn * G::WN + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(bs + row * BK + swz(row, ch) * 8);
      }
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  if (GL) {
    if (c_tiles) tap_seek(kt0);
    // prologue: S-1 k-tiles in flight
#pragma unroll
    for (int st = 0; st < S - 1; ++st) gstage(st, kt0 + st, st < nk);
    for (int kt = 0; kt < nk; ++kt) {
      // this wave's DMA of tile kt has landed once <= S-2 stages remain
      // outstanding; the barrier publishes every wave's DMA and guarantees all
      // waves are done reading tile kt-1, whose buffer the next DMA reuses
      wait_vmcnt<(S - 2) * G::PER_STAGE>();
      lds_barrier();
      const int nxt = kt + S - 1;
      gstage(nxt % S, kt0 + nxt, nxt < nk);
      const int cur = kt % S;
      mfma_tile(As + cur * BM * BK, Bs + cur * BN * BK);
    }
    wait_vmcnt<0>();
    __syncthreads();
  } else {
    gload(kt0);
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) gload(kt0 + kt + 1);
      mfma_tile(As + cur * BM * BK, Bs + cur * BN * BK);
      if (kt + 1 < nk) sstore(cur ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue: stage fp32 tile in LDS, then coalesced 8-wide row chunks
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * G::WM + i * 16 + fq * 4 + r) * G::CS_LD + wn * G::WN + j * 16 + fr] = acc[i][j][r];
  __syncthreads();

  const float alpha = p.alpha;
  constexpr int CPR = BN / 8;   // chunks per row
  if (p.splits > 1) {
    // raw partial slab of this K split; splitk_reduce applies the epilogue
    float* ws = p.ws + size_t(blockIdx.y) * M * N;
    const bool v4 = (N % 4 == 0);
    for (int c = tid; c < BM * CPR; c += kThreads) {
      const int row = c / CPR, col = (c - row * CPR) * 8;
      const int m = m0 + row, n = n0 + col;
      if (m >= M || n >= N) continue;
      const float* src = Cs + row * G::CS_LD + col;
      float* dst = ws + size_t(m) * N + n;
      if (v4 && n + 8 <= N) {
        float4 a = *reinterpret_cast<const float4*>(src);
        float4 b = *reinterpret_cast<const float4*>(src + 4);
        a.x *= alpha; a.y *= alpha; a.z *= alpha; a.w *= alpha;
        b.x *= alpha; b.y *= alpha; b.z *= alpha; b.w *= alpha;
        *reinterpret_cast<float4*>(dst) = a;
        *reinterpret_cast<float4*>(dst + 4) = b;
      } else {
        for (int e = 0; e < 8 && n + e < N; ++e) dst[e] = src[e] * alpha;
      }
    }
    return;
  }
  switch (p.act) {
    case kActRelu: epilogue_rows<BM, BN, G::CS_LD, kActRelu>(p, Cs, m0, n0, tid, rpre); break;
    case kActGeluTanh: epilogue_rows<BM, BN, G::CS_LD, kActGeluTanh>(p, Cs, m0, n0, tid, rpre); break;
    case kActGeluErf: epilogue_rows<BM, BN, G::CS_LD, kActGeluErf>(p, Cs, m0, n0, tid, rpre); break;
    case kActTanh: epilogue_rows<BM, BN, G::CS_LD, kActTanh>(p, Cs, m0, n0, tid, rpre); break;
    default: epilogue_rows<BM, BN, G::CS_LD, 0>(p, Cs, m0, n0, tid, rpre); break;
  }
}

template <int BM, int BN, int AMODE, int NSTAGE, int WAVES_M = 2, int BKT = 64>
hipError_t launch_cfg(const IGemmArgs& a0, hipStream_t s) {
  using G = IGemm<BM, BN, AMODE, NSTAGE, WAVES_M, BKT>;
  IGemmArgs a = a0;
  if (a.splits > 1) {   // split ranges in units of this config's k-tile
    const int nk = (a.K + G::BK - 1) / G::BK;
    a.kt_per_split = (nk + a.splits - 1) / a.splits;
  }
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (tiles == 0) return hipSuccess;
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&igemm_kernel<BM, BN, AMODE, NSTAGE, WAVES_M, BKT>),
                                G::LDS);
  if (e != hipSuccess) return e;
  const int splits = a.splits > 1 ? a.splits : 1;
  hipLaunchKernelGGL((igemm_kernel<BM, BN, AMODE, NSTAGE, WAVES_M, BKT>), dim3(tiles, splits), dim3(kThreads), G::LDS, s, a);
  return hipGetLastError();
}

// Sum the split-K slabs (fixed order -> deterministic) + epilogue; 8 columns per thread.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(IGemmArgs p) {
  const int M = p.M, N = p.N;
  const int cpr = (N + 7) / 8;
  const long total = long(M) * cpr;
  const size_t slab = size_t(M) * N;
  for (long c = blockIdx.x * long(blockDim.x) + threadIdx.x; c < total; c += long(gridDim.x) * blockDim.x) {
    const int m = int(c / cpr), n = int(c - long(m) * cpr) * 8;
    const int ne = min(8, N - n);
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < p.splits; ++s) {
      const float* src = p.ws + s * slab + size_t(m) * N + n;
      if (ne == 8 && (N % 4 == 0)) {
        const float4 a = *reinterpret_cast<const float4*>(src);
        const float4 b = *reinterpret_cast<const float4*>(src + 4);
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
      } else {
        for (int e = 0; e < ne; ++e) v[e] += src[e];
      }
    }
    for (int e = 0; e < ne; ++e) {
      float x = v[e];
      if (p.bias) x += p.bias[n + e];
      if (p.residual) x += bf16_to_f32(p.residual[size_t(m) * p.ldr + n + e]);
      x = apply_act(x, p.act);
      if (p.out) {
        if (p.out_f32) static_cast<float*>(p.out)[size_t(m) * p.ldc + n + e] = x;
        else static_cast<uint16_t*>(p.out)[size_t(m) * p.ldc + n + e] = f32_to_bf16(x);
      }
      if (p.out2) {   // post-activation output (ResNet v2 pre-activation of the next block)
        float y = x * p.scale2[n + e] + p.shift2[n + e];
        if (p.act2 == kActRelu) y = fmaxf(y, 0.f);
        if (p.out_f32) static_cast<float*>(p.out2)[size_t(m) * p.ldc + n + e] = y;
        else static_cast<uint16_t*>(p.out2)[size_t(m) * p.ldc + n + e] = f32_to_bf16(y);
      }
    }
  }
}

// Tile configs: (BM, BN, DMA ring depth).  Deeper rings hide more memory
// latency per workgroup but cost LDS, i.e. resident workgroups per CU (160 KB
// LDS): the tuner picks per layer (K=64 1x1 convs want occupancy, long-K
// small-grid layers want depth).  Register-staged operand modes ignore the
// depth (always 2).
constexpr int kCfgBM[kNumIGemmConfigs] = {128, 128, 64, 64, 128, 64, 128, 64, 64, 256, 128, 256, 64, 64, 64, 128, 128};
constexpr int kCfgBN[kNumIGemmConfigs] = {128, 64, 128, 64, 128, 64, 64, 128, 256, 64, 256, 128, 64, 64, 128, 64, 128};
constexpr int kCfgST[kNumIGemmConfigs] = {2, 2, 2, 2, 3, 4, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2};
constexpr int kCfgBK[kNumIGemmConfigs] = {64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 128, 256, 128, 128, 128};
// register-staged operand modes only instantiate configs 0-3
constexpr int kCfgBase[kNumIGemmConfigs] = {0, 1, 2, 3, 0, 3, 1, 2, 2, 1, 0, 0, 3, 3, 2, 1, 0};

template <int AMODE>
hipError_t launch_mode(const IGemmArgs& a, int cfg, hipStream_t s) {
  constexpr bool GL = (AMODE == kADense || AMODE == kAIm2col);
  if (!GL) cfg = kCfgBase[cfg];
  switch (cfg) {
    case 0: return launch_cfg<128, 128, AMODE, 2>(a, s);
    case 1: return launch_cfg<128, 64, AMODE, 2>(a, s);
    case 2: return launch_cfg<64, 128, AMODE, 2>(a, s);
    case 3: return launch_cfg<64, 64, AMODE, 2>(a, s);
    default: break;
  }
  if constexpr (GL) {
    switch (cfg) {
      case 4: return launch_cfg<128, 128, AMODE, 3>(a, s);
      case 5: return launch_cfg<64, 64, AMODE, 4>(a, s);
      case 6: return launch_cfg<128, 64, AMODE, 3>(a, s);
      case 7: return launch_cfg<64, 128, AMODE, 3>(a, s);
      // wide tiles (one wave row / column): 4x the outputs per workgroup setup
      case 8: return launch_cfg<64, 256, AMODE, 2, 1>(a, s);
      case 9: return launch_cfg<256, 64, AMODE, 2, 4>(a, s);
      case 10: return launch_cfg<128, 256, AMODE, 2, 2>(a, s);
      case 11: return launch_cfg<256, 128, AMODE, 2, 4>(a, s);
      // deep k-tiles: 2-4x the MFMA work per barrier / DMA round trip
      case 12: return launch_cfg<64, 64, AMODE, 2, 2, 128>(a, s);
      case 13: return launch_cfg<64, 64, AMODE, 2, 2, 256>(a, s);
      case 14: return launch_cfg<64, 128, AMODE, 2, 2, 128>(a, s);
      case 15: return launch_cfg<128, 64, AMODE, 2, 2, 128>(a, s);
      case 16: return launch_cfg<128, 128, AMODE, 2, 2, 128>(a, s);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace

int igemm_config_bm(int cfg) { return kCfgBM[cfg]; }
int igemm_config_bn(int cfg) { return kCfgBN[cfg]; }
int igemm_config_stages(int cfg) { return kCfgST[cfg]; }
int igemm_config_bk(int cfg) { return kCfgBK[cfg]; }

hipError_t igemm_launch(const IGemmArgs& a, int a_mode, int cfg, hipStream_t s) {
  switch (a_mode) {
    case kADense: return launch_mode<kADense>(a, cfg, s);
    case kAIm2col: return launch_mode<kAIm2col>(a, cfg, s);
    case kAStemF32: return launch_mode<kAStemF32>(a, cfg, s);
    case kAStem7x7x3: return launch_mode<kAStem7x7x3>(a, cfg, s);
    case kAC4: return launch_mode<kAC4>(a, cfg, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t splitk_reduce_launch(const IGemmArgs& a, hipStream_t s) {
  const long work = long(a.M) * ((a.N + 7) / 8);
  long g = (work + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(int(g < 1 ? 1 : g)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace tfsk
