// Pipelined MFMA conv / GEMM for MI355X (gfx950): bf16 operands, fp32 accumulate.
//
// C[M][N] = epilogue( A[M][K] * B[N][K]^T ), the same contract as igemm.hip, for
// the 64-aligned cases that make up almost all of ResNet-50 / BERT:
//   A dense row-major (K % 64 == 0), or the implicit im2col of an NHWC tensor
//   with C % 64 == 0, so one 64-deep k-tile is exactly one filter tap x 64
//   channels;  B = weights [Cout][ldb].
//
// Why a second kernel: rocprofv3 PMC of igemm on the ResNet 3x3 layers showed
// ~90 SALU+VALU instructions per 16 MFMAs and a vmcnt(0) drain every k-tile
// (SQ_ACTIVE_INST_ANY 44 %, SQ_WAIT_ANY 41 %, MFMA busy 11-16 % of wave
// cycles).  This kernel is built so the steady-state k-tile costs little more
// than its MFMAs:
//   * S-deep ring of direct-to-LDS DMAs (buffer_load ... lds): the wait before
//     tile t is a counted vmcnt((S-2) * pieces) — never a drain — followed by a
//     bare s_barrier;
//   * every per-lane DMA offset is precomputed once (voffset) and the k-tile
//     advance is a wave-uniform scalar (soffset): no VALU address math per tile;
//   * im2col padding = one precomputed tap-validity bit mask per DMA row
//     (3 VALU per piece), the tap walk runs in SGPRs, and the buffer
//     descriptor is rebased by the top/left padding so every in-image offset is
//     non-negative; invalid taps read through an out-of-range voffset (zeros);
//   * the loop is unrolled by S, so ring slots and all LDS fragment offsets
//     are compile-time immediates;
//   * LDS rows are 128 B with 16-B chunks XOR-swizzled by (row & 7): the DMA
//     lane writes slot l&7 of row l>>3 from source chunk (l&7)^(l>>3), the
//     ds_read_b128 fragment reads undo it (conflict-free);
//   * 4 or 8 waves per workgroup, each owning a WM x WN sub-tile of
//     v_mfma_f32_16x16x32_bf16 accumulators; bijective XCD-aware tile remap +
//     GROUP_M ordering; epilogue staged through LDS as fp32 for coalesced
//     16-B bias/residual/activation/store row chunks (residual prefetched into
//     registers before the K loop).
#include "gemm_common.h"
#include "cgemm.h"

namespace tfsk {

namespace {

using namespace gemm;
constexpr int kGroupM = 8;

template <int BM, int BN, int WGM, int WGN, int S>
struct CG {
  static constexpr int NW = WGM * WGN, NT = 64 * NW;
  static constexpr int WM = BM / WGM, WN = BN / WGN;
  static constexpr int TM = WM / 16, TN = WN / 16;
  static constexpr int APW = BM / (8 * NW), BPW = BN / (8 * NW);   // 1-KB DMA pieces per wave per stage
  static constexpr int PPW = APW + BPW;
  static constexpr int A_ST = BM * KT, B_ST = BN * KT;            // elements per ring slot
  static constexpr int LDS_MAIN = S * (A_ST + B_ST) * 2;
  static constexpr int CS_LD = BN + 4;
  // the fp32 tile is staged through LDS for the epilogue; a tile whose fp32
  // image does not fit next to nothing (256 x 192: 196 KB) goes in two row
  // passes (each wave's rows fall in one pass)
  static constexpr int LDS_EPI_FULL = BM * CS_LD * 4;
  static constexpr int PASSES = LDS_EPI_FULL > 160 * 1024 ? 2 : 1;
  static constexpr int RPP = BM / PASSES;
  static constexpr int LDS_EPI = RPP * CS_LD * 4;
  static constexpr int LDS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
  static_assert(RPP % WM == 0, "epilogue passes split the tile at wave-row boundaries");
  static_assert(APW >= 1 && BPW >= 1 && BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "DMA piece split");
  static_assert(TM >= 1 && TN >= 1 && WM % 16 == 0 && WN % 16 == 0, "wave tile");
  static_assert(S >= 2 && (S - 2) * PPW < 64, "ring depth / vmcnt range");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

template <int BM, int BN, int NT>
__device__ __forceinline__ void prefetch_residual(const IGemmArgs& p, int m0, int n0, int tid,
                                                  uint4 (&rpre)[Epi<BM, BN, NT>::PRE > 0 ? Epi<BM, BN, NT>::PRE : 1]) {
  using E = Epi<BM, BN, NT>;
  if (E::PRE == 0 || !p.residual || p.splits > 1 || (p.N % 8) || (p.ldr % 8)) return;
#pragma unroll
  for (int it = 0; it < E::PRE; ++it) {
    int row, col;
    const bool in = epi_rowcol<BM, BN, NT>(tid, it, row, col);
    const int m = m0 + row, n = n0 + col;
    rpre[it] = (in && m < p.M && n + 8 <= p.N) ? *reinterpret_cast<const uint4*>(p.residual + size_t(m) * p.ldr + n)
                                          : make_uint4(0, 0, 0, 0);
  }
}

// Cheap activations (none / ReLU / GELU-tanh / tanh -- the last two are an exp
// and a rcp, common.h sigm2): fully unrolled over the thread's chunks, residual
// from the registers prefetched before the K loop.  erf GELU (Keras FFNs): a
// rolled loop, so the erf expansion is emitted once instead of ITERS x 8 times.
template <int BM, int BN, int NT, int CS_LD, int ACT, bool USE_PRE = true>
__device__ __forceinline__ void epilogue_rows(const IGemmArgs& p, const float* Cs, int m0, int n0, int tid,
                                              const uint4 (&rpre)[Epi<BM, BN, NT>::PRE > 0 ? Epi<BM, BN, NT>::PRE : 1],
                                              const float4 b0, const float4 b1) {
  using E = Epi<BM, BN, NT>;
  constexpr int PRE = USE_PRE ? E::PRE : 0;
  const int M = p.M, N = p.N;
  const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  constexpr bool cheap = (ACT != kActGeluErf);   // GELU-tanh / tanh are exp + rcp (common.h sigm2)
  if constexpr (cheap) {
#pragma unroll
    for (int it = 0; it < E::ITERS; ++it) {
      int row, col;
      if (!epi_rowcol<BM, BN, NT>(tid, it, row, col)) continue;
      const int m = m0 + row, n = n0 + col;
      if (m >= M || n >= N) continue;
      uint4 rr = make_uint4(0, 0, 0, 0);
      if (p.residual)
        rr = PRE > 0 ? rpre[PRE > 0 ? it : 0] : *reinterpret_cast<const uint4*>(p.residual + size_t(m) * p.ldr + n);
      epi_chunk<ACT>(p, Cs + row * CS_LD + col, m, n, bv, rr);
    }
  } else {
#pragma unroll 1
    for (int it = 0; it < E::ITERS; ++it) {
      int row, col;
      if (!epi_rowcol<BM, BN, NT>(tid, it, row, col)) continue;
      const int m = m0 + row, n = n0 + col;
      if (m >= M || n >= N) continue;
      const uint4 rr = p.residual ? *reinterpret_cast<const uint4*>(p.residual + size_t(m) * p.ldr + n)
                                  : make_uint4(0, 0, 0, 0);
      epi_chunk<ACT>(p, Cs + row * CS_LD + col, m, n, bv, rr);
    }
  }
}

// Waves per SIMD the register allocation must leave room for: the 4-wave
// 32-KB tiles (64x64, 2 slots) fit 5 workgroups per CU by LDS, i.e. 5 waves
// per SIMD, which needs <= 102 VGPRs (unconstrained they took 128: 4 per CU)
template <int BM, int BN, int WGM, int WGN, int S, bool PF>
constexpr int cg_waves_per_eu() {
  return (!PF && WGM * WGN == 4 && CG<BM, BN, WGM, WGN, S>::LDS <= 32 * 1024) ? 5 : 1;
}

// PF: fragment-prefetch step pipeline -- step t's fragments are read from LDS
// right after its barrier while the MFMAs of step t - 1 (fragments already in
// registers) issue, so neither the LDS read latency nor the barrier sits
// between a k-tile landing and its MFMAs (halo.hip uses the same scheme).
template <int BM, int BN, int WGM, int WGN, int S, int AM, bool PF>
__global__ __launch_bounds__(64 * WGM * WGN, (cg_waves_per_eu<BM, BN, WGM, WGN, S, PF>())) void cgemm_kernel(IGemmArgs p) {
  using G = CG<BM, BN, WGM, WGN, S>;
  constexpr bool IM2COL = (AM == 1), DUAL = (AM == 2), STEM = (AM == 3);
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  char* const smem = reinterpret_cast<char*>(smem_raw);
  typedef __attribute__((address_space(3))) void* lds_ptr_t;

  // ---- tile of this workgroup (XCD remap + GROUP_M ordering)
  const int M = p.M, N = p.N;
  const int nbm = (M + BM - 1) / BM, nbn = (N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int per_group = kGroupM * nbn;
  const int first_m = (wg / per_group) * kGroupM;
  const int gsz = min(nbm - first_m, kGroupM);
  const int bm = first_m + (wg % per_group) % gsz;
  const int bn = (wg % per_group) / gsz;
  const int m0 = bm * BM, n0 = bn * BN;

  // profiling ablations (act >= 100): bit 0 skips the operand DMAs, bit 1 the
  // LDS reads + MFMAs, bit 2 exits right away, bit 3 skips the epilogue, bit 4
  // exits after the per-lane setup
  // (timing only; results are garbage)
  const int dbg = p.act >= 100 ? p.act - 100 : 0;
  if (dbg & 4) return;
  trace_stamp(p, 0);
  const bool do_dma = !(dbg & 1), do_mma = !(dbg & 2);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  // DMA lane -> row (lane >> 3) of its 8-row piece, LDS slot (lane & 7) holding
  // logical chunk (lane & 7) ^ (row & 7)
  const int prow = lane >> 3;
  const uint32_t kc = uint32_t(((lane & 7) ^ prow) * 8);

  // ---- buffer descriptors (wave-uniform: kernel args only)
  const char* abase = static_cast<const char*>(p.a);
  uint32_t arec = uint32_t(p.a_bytes);
  if (IM2COL) {
    const uint32_t shift = uint32_t((p.PT * p.W + p.PL) * p.C) * 2u;
    abase -= shift;
    arec += shift;
  }
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(abase), 0, int(arec), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.b), 0, int(p.b_bytes), 0x00020000);
  // dual mode: second A source (1x1 / strided samples of an NHWC tensor)
  const __amdgpu_buffer_rsrc_t rsA2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(DUAL ? p.a2 : p.a), 0, int(DUAL ? p.a2_bytes : p.a_bytes), 0x00020000);

  // ---- per-lane DMA offsets (computed once)
  const float inv_hw = 1.f / float(p.Ho * p.Wo), inv_wo = 1.f / float(p.Wo);
  uint32_t a_off[G::APW], a_msk[G::APW], a_off2[DUAL ? G::APW : 1];
#pragma unroll
  for (int j = 0; j < G::APW; ++j) {
    const int m = m0 + (wid * G::APW + j) * 8 + prow;
    const bool ok = m < M;
    a_msk[j] = 0;
    if (STEM) {
      // pre-padded bf16 RGBA, k = kh*32 + kw*4 + c: a k-tile is filter rows
      // (2t, 2t+1) x 8 taps x 4 channels = 2 runs of 64 contiguous bytes; this
      // lane's logical chunk lc holds row lc>>2, pixels 2*(lc&3) .. +1
      const int lc = (lane & 7) ^ prow;
      const int mm = ok ? m : 0;
      const int hw = p.Ho * p.Wo;
      const int n = fdiv(mm, hw, inv_hw), r = mm - n * hw;
      const int ho = fdiv(r, p.Wo, inv_wo), wo = r - ho * p.Wo;
      a_off[j] = ok ? uint32_t(((n * p.H + ho * p.SH + (lc >> 2)) * p.W + wo * p.SW + (lc & 3) * 2) * 4) * 2u : kOOB;
    } else if (!IM2COL) {
      a_off[j] = ok ? (uint32_t(m) * uint32_t(p.lda) + kc) * 2u : kOOB;
      if constexpr (DUAL) {
        const int mm = ok ? m : 0;
        const int hw = p.Ho * p.Wo;
        const int n = fdiv(mm, hw, inv_hw), r = mm - n * hw;
        const int ho = fdiv(r, p.Wo, inv_wo), wo = r - ho * p.Wo;
        a_off2[j] = ok ? (uint32_t((n * p.H + ho * p.SH) * p.W + wo * p.SW) * uint32_t(p.C) + kc) * 2u : kOOB;
      }
    } else {
      const int mm = ok ? m : 0;
      const int hw = p.Ho * p.Wo;
      const int n = fdiv(mm, hw, inv_hw), r = mm - n * hw;
      const int ho = fdiv(r, p.Wo, inv_wo), wo = r - ho * p.Wo;
      const int hb = ho * p.SH, wb = wo * p.SW;          // tap (0,0) in padded coordinates
      a_off[j] = (uint32_t((n * p.H + hb) * p.W + wb) * uint32_t(p.C) + kc) * 2u;
      // tap t = kh*KW + kw is valid iff row hi0+kh and column wi0+kw are inside
      const int hi0 = hb - p.PT, wi0 = wb - p.PL;
      uint32_t wbits = 0;
      for (int kw = 0; kw < p.KW; ++kw) wbits |= uint32_t((unsigned)(wi0 + kw) < (unsigned)p.W) << kw;
      uint32_t msk = 0;
      for (int kh = 0; kh < p.KH; ++kh)
        if ((unsigned)(hi0 + kh) < (unsigned)p.H) msk |= wbits << (kh * p.KW);
      a_msk[j] = ok ? msk : 0u;
    }
  }
  uint32_t b_off[G::BPW];
#pragma unroll
  for (int j = 0; j < G::BPW; ++j) {
    const int n = n0 + (wid * G::BPW + j) * 8 + prow;
    b_off[j] = n < N ? (uint32_t(n) * uint32_t(p.ldb) + kc) * 2u : kOOB;
  }

  // ---- k range of this workgroup (split-K: blockIdx.y selects a slice)
  const int nk_all = p.K / KT;
  int kt0 = 0, nk = nk_all;
  if (p.splits > 1) {
    kt0 = blockIdx.y * p.kt_per_split;
    nk = min(nk_all - kt0, p.kt_per_split);
  }

  // ---- scalar producer walk: k element offset; im2col tap (kh, kw) + channel offset
  int w_k = kt0 * KT;
  int w_ci = 0, w_kh = 0, w_kw = 0, w_tap = 0;
  if (IM2COL) {
    w_tap = w_k / p.C;
    w_ci = w_k - w_tap * p.C;
    w_kh = w_tap / p.KW;
    w_kw = w_tap - w_kh * p.KW;
  }

  auto issue = [&](int slot) {
    const uint32_t a_soff = IM2COL ? uint32_t((w_kh * p.W + w_kw) * p.C + w_ci) * 2u
                            : STEM ? uint32_t(w_k >> 6) * uint32_t(p.W) * 16u   // 2 filter rows per k-tile
                                   : uint32_t(w_k) * 2u;
    const uint32_t b_soff = uint32_t(w_k) * 2u;
    if (DUAL && w_k >= p.K1) {   // wave-uniform: the k-tile lies in the second source
      const uint32_t soff2 = uint32_t(w_k - p.K1) * 2u;
#pragma unroll
      for (int j = 0; j < G::APW; ++j) {
        const uint32_t v = a_off2[DUAL ? j : 0];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsA2, (lds_ptr_t)(smem + (slot * G::A_ST + (wid * G::APW + j) * 512) * 2), 16, v, soff2, 0, 0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < G::APW; ++j) {
        uint32_t v = a_off[j];
        if (IM2COL) v = ((a_msk[j] >> w_tap) & 1u) ? v : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsA, (lds_ptr_t)(smem + (slot * G::A_ST + (wid * G::APW + j) * 512) * 2), 16, v, a_soff, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < G::BPW; ++j) {
      // (a named local, not b_off[j] in the call: with the array element as a
      // builtin argument hipcc's host pass silently drops the kernel stub)
      const uint32_t v = b_off[j];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (lds_ptr_t)(smem + (S * G::A_ST + slot * G::B_ST + (wid * G::BPW + j) * 512) * 2), 16, v, b_soff,
          0, 0);
    }
    w_k += KT;
    if (IM2COL) {
      w_ci += KT;
      if (w_ci == p.C) {
        w_ci = 0;
        ++w_tap;
        if (++w_kw == p.KW) {
          w_kw = 0;
          ++w_kh;
        }
      }
    }
  };

  // ---- consumer: per-lane fragment byte offsets within a ring slot (k-subtile 0 / 1)
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t ra0 = uint32_t(((wm * G::WM + fr) * KT + ((fq ^ (fr & 7)) * 8)) * 2);
  const uint32_t ra1 = uint32_t(((wm * G::WM + fr) * KT + (((4 + fq) ^ (fr & 7)) * 8)) * 2);
  const uint32_t rb0 = uint32_t(((wn * G::WN + fr) * KT + ((fq ^ (fr & 7)) * 8)) * 2);
  const uint32_t rb1 = uint32_t(((wn * G::WN + fr) * KT + (((4 + fq) ^ (fr & 7)) * 8)) * 2);

  f32x4 acc[G::TM][G::TN];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int slot) {
    const char* sa = smem + slot * G::A_ST * 2;
    const char* sb = smem + (S * G::A_ST + slot * G::B_ST) * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[G::TM], bfr[G::TN];
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(sa + (kk ? ra1 : ra0) + i * 16 * KT * 2);
#pragma unroll
      for (int j = 0; j < G::TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(sb + (kk ? rb1 : rb0) + j * 16 * KT * 2);
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  struct Frags {
    bf16x8 a[2][G::TM], b[2][G::TN];
  };
  auto load_frags = [&](Frags& f, int slot) {
    const char* sa = smem + slot * G::A_ST * 2;
    const char* sb = smem + (S * G::A_ST + slot * G::B_ST) * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
        f.a[kk][i] = *reinterpret_cast<const bf16x8*>(sa + (kk ? ra1 : ra0) + i * 16 * KT * 2);
#pragma unroll
      for (int j = 0; j < G::TN; ++j)
        f.b[kk][j] = *reinterpret_cast<const bf16x8*>(sb + (kk ? rb1 : rb0) + j * 16 * KT * 2);
    }
  };
  auto mma = [&](const Frags& f) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[kk][i], f.b[kk][j], acc[i][j], 0, 0, 0);
  };
  Frags prev;

  uint4 rpre[Epi<BM, BN, G::NT>::PRE > 0 ? Epi<BM, BN, G::NT>::PRE : 1];
  if constexpr (G::PASSES == 1) prefetch_residual<BM, BN, G::NT>(p, m0, n0, tid, rpre);
  float4 bias0, bias1;
  prefetch_bias<BM, BN, G::NT>(p, n0, tid, bias0, bias1);

  if (dbg & 16) {   // ablation: setup only (keep the per-lane state live)
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < G::APW; ++j) keep ^= a_off[j] ^ a_msk[j];
#pragma unroll
    for (int j = 0; j < G::BPW; ++j) keep ^= b_off[j];
    asm volatile("" ::"v"(keep), "v"(ra0), "v"(rb1), "s"(w_tap), "s"(w_ci));
    return;
  }

  // ---- prologue: S-1 k-tiles in flight
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk && do_dma) issue(s);

  // ---- main loop, unrolled by the ring depth (slot indices are immediates)
  for (int kt = 0; kt < nk; kt += S) {
#pragma unroll
    for (int u = 0; u < S; ++u) {
      const int t = kt + u;
      if (t < nk) {
        // tile t landed (this wave's DMAs) once only the younger groups remain
        if (t + S - 2 < nk) wait_vmcnt<(S - 2) * G::PPW>();
        else wait_vmcnt<0>();
        // ... and every wave's (and every wave is done reading slot (t-1) % S)
        lds_barrier();
        if (t == 0) trace_stamp(p, 1);
        if (t + S - 1 < nk && do_dma) issue((u + S - 1) % S);
        if constexpr (PF) {
          // pinned: the scheduler would hoist the register-only MFMAs above
          // the barrier and sink the reads to their uses
          __builtin_amdgcn_sched_barrier(0);
          Frags cur;
          load_frags(cur, u);
          __builtin_amdgcn_sched_barrier(0);
          if (t > 0 && do_mma) mma(prev);
          __builtin_amdgcn_sched_barrier(0);
          prev = cur;
        } else {
          if (do_mma) compute(u);
        }
      }
    }
  }
  if constexpr (PF) {
    if (nk > 0 && do_mma) mma(prev);
  }
  wait_vmcnt<0>();
  __syncthreads();
  trace_stamp(p, 2);
  if (dbg & 8) return;
  // ---- epilogue: stage the fp32 tile in LDS, then coalesced row chunks
  // (G::PASSES row passes of G::RPP rows when the whole fp32 tile does not fit)
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int RPP = G::RPP;
#pragma unroll
  for (int ps = 0; ps < G::PASSES; ++ps) {
    if (ps > 0) __syncthreads();    // the previous pass has read Cs
    if (G::PASSES == 1 || (wm * G::WM) / RPP == ps) {
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(wm * G::WM - ps * RPP + i * 16 + fq * 4 + r) * G::CS_LD + wn * G::WN + j * 16 + fr] = acc[i][j][r];
    }
    __syncthreads();
    const int mp = m0 + ps * RPP;

    if (p.splits > 1) {
      // raw (alpha-scaled) partial slab of this K slice; splitk_reduce applies the epilogue
      const float alpha = p.alpha;
      float* ws = p.ws + size_t(blockIdx.y) * M * N;
      const __amdgpu_buffer_rsrc_t wsr = splitk_rsrc(p);
      constexpr int CPR = BN / 8;
      const bool v4 = (N % 4 == 0);
      for (int c = tid; c < RPP * CPR; c += G::NT) {
        const int row = c / CPR, col = (c - row * CPR) * 8;
        const int m = mp + row, n = n0 + col;
        if (m >= M || n >= N) continue;
        const float* src = Cs + row * G::CS_LD + col;
        float* dst = ws + size_t(m) * N + n;
        if (v4 && n + 8 <= N) {
          float4 a = *reinterpret_cast<const float4*>(src);
          float4 b = *reinterpret_cast<const float4*>(src + 4);
          a.x *= alpha; a.y *= alpha; a.z *= alpha; a.w *= alpha;
          b.x *= alpha; b.y *= alpha; b.z *= alpha; b.w *= alpha;
          if (p.counters != nullptr) {
            splitk_store8(p, wsr, m, n, a, b);
          } else {
            *reinterpret_cast<float4*>(dst) = a;
            *reinterpret_cast<float4*>(dst + 4) = b;
          }
        } else {
          for (int e = 0; e < 8 && n + e < N; ++e) dst[e] = src[e] * alpha;
        }
      }
      if constexpr (G::PASSES == 1) {
        if (p.counters != nullptr) {
          if (!splitk_arrive(p, blockIdx.x)) {
            trace_stamp(p, 3);
            return;
          }
          // the last slice: every slab of the tile summed into Cs, then the
          // epilogue (unrolled: every chunk's slab loads in flight together)
#pragma unroll
          for (int c = tid; c < RPP * CPR; c += G::NT) {
            const int row = c / CPR, col = (c - row * CPR) * 8;
            const int m = mp + row, n = n0 + col;
            if (m >= M || n >= N) continue;
            float4 lo, hi;
            splitk_sum8(p, wsr, m, n, lo, hi);
            *reinterpret_cast<float4*>(Cs + row * G::CS_LD + col) = lo;
            *reinterpret_cast<float4*>(Cs + row * G::CS_LD + col + 4) = hi;
          }
          __syncthreads();
          IGemmArgs q = p;
          q.splits = 1;
          q.alpha = 1.f;                      // the slabs carry alpha already
          float4 qb0, qb1;
          prefetch_bias<BM, BN, G::NT>(q, n0, tid, qb0, qb1);
          using RP1 = uint4[Epi<RPP, BN, G::NT>::PRE > 0 ? Epi<RPP, BN, G::NT>::PRE : 1];
          const RP1& r1 = *reinterpret_cast<const RP1*>(rpre);   // not read (USE_PRE = false)
          switch (q.act) {
            case kActRelu: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActRelu, false>(q, Cs, mp, n0, tid, r1, qb0, qb1); break;
            case kActGeluTanh: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActGeluTanh, false>(q, Cs, mp, n0, tid, r1, qb0, qb1); break;
            case kActGeluErf: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActGeluErf, false>(q, Cs, mp, n0, tid, r1, qb0, qb1); break;
            case kActTanh: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActTanh, false>(q, Cs, mp, n0, tid, r1, qb0, qb1); break;
            default: epilogue_rows<RPP, BN, G::NT, G::CS_LD, 0, false>(q, Cs, mp, n0, tid, r1, qb0, qb1); break;
          }
          trace_stamp(p, 3);
          return;
        }
      }
      continue;
    }
    constexpr bool P1 = G::PASSES == 1;
    using RP = uint4[Epi<RPP, BN, G::NT>::PRE > 0 ? Epi<RPP, BN, G::NT>::PRE : 1];
    const RP& rp = *reinterpret_cast<const RP*>(rpre);   // only read when PASSES == 1 (RPP == BM)
    switch (p.act) {
      case kActRelu: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActRelu, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1); break;
      case kActGeluTanh: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActGeluTanh, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1); break;
      case kActGeluErf: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActGeluErf, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1); break;
      case kActTanh: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActTanh, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1); break;
      default: epilogue_rows<RPP, BN, G::NT, G::CS_LD, 0, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1); break;
    }
  }
  trace_stamp(p, 3);
}

template <int BM, int BN, int WGM, int WGN, int S, int AM, bool PF = false>
hipError_t launch_cfg(const IGemmArgs& a0, hipStream_t s) {
  using G = CG<BM, BN, WGM, WGN, S>;
  IGemmArgs a = a0;
  const int nk = a.K / KT;
  const int splits = a.splits > 1 ? a.splits : 1;
  if (splits > 1) a.kt_per_split = (nk + splits - 1) / splits;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (tiles == 0) return hipSuccess;
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&cgemm_kernel<BM, BN, WGM, WGN, S, AM, PF>), G::LDS);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((cgemm_kernel<BM, BN, WGM, WGN, S, AM, PF>), dim3(tiles, splits), dim3(G::NT), G::LDS, s, a);
  return hipGetLastError();
}

// Config table (tile BM x BN, wave grid, ring depth).  LDS per workgroup =
// S * (BM + BN) * 128 B (or the fp32 epilogue tile if larger).
constexpr int kAll = kNumCGemmConfigs + kNumCGemmConfigs2;
constexpr int kBM[kAll] = {128, 128, 64, 128, 64, 256, 128, 128, 64, 256, 64, 64, 128, 128, 128, 64,
                           64, 64, 64, 128, 64, 128, 64, 64, 256};
constexpr int kBN[kAll] = {128, 128, 128, 64, 64, 128, 256, 128, 256, 64, 64, 128, 64, 96, 96, 96,
                           64, 64, 64, 64, 128, 64, 128, 64, 192};

// PF config ids kCGemmPfCfgBase + i: the fragment-prefetch build of table index kPfOf[i]
// (the 8-wave 256 x 128 / 128 x 256 / 256 x 192 tiles spill with two fragment sets: not built)
constexpr int kPfOf[kNumCGemmPfConfigs] = {0, 2, 3, 4, 7, 9, 10, 11, 12, 13, 23};

// config id -> index into the tables (all id ranges)
int cfg_index(int cfg) {
  if (cfg >= kCGemmPfCfgBase) return kPfOf[cfg - kCGemmPfCfgBase];
  return cfg < kCGemmCfgBase2 ? cfg - kCGemmCfgBase : kNumCGemmConfigs + (cfg - kCGemmCfgBase2);
}

template <int AM>
hipError_t launch_mode_pf(const IGemmArgs& a, int idx, hipStream_t s) {
  switch (idx) {
    case 0: return launch_cfg<128, 128, 2, 2, 3, AM, true>(a, s);
    case 2: return launch_cfg<64, 128, 2, 2, 4, AM, true>(a, s);
    case 3: return launch_cfg<128, 64, 2, 2, 4, AM, true>(a, s);
    case 4: return launch_cfg<64, 64, 2, 2, 4, AM, true>(a, s);
    case 7: return launch_cfg<128, 128, 2, 4, 4, AM, true>(a, s);
    case 9: return launch_cfg<256, 64, 4, 1, 3, AM, true>(a, s);
    case 10: return launch_cfg<64, 64, 2, 2, 2, AM, true>(a, s);
    case 11: return launch_cfg<64, 128, 2, 2, 2, AM, true>(a, s);
    case 12: return launch_cfg<128, 64, 2, 2, 2, AM, true>(a, s);
    case 13: return launch_cfg<128, 96, 2, 2, 3, AM, true>(a, s);
    case 23: return launch_cfg<64, 64, 2, 2, 3, AM, true>(a, s);
    default: return hipErrorInvalidValue;
  }
}

template <int AM>
hipError_t launch_mode(const IGemmArgs& a, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_cfg<128, 128, 2, 2, 3, AM>(a, s);   // 96 KB, wave 64x64
    case 1: return launch_cfg<128, 128, 2, 2, 2, AM>(a, s);   // 64 KB (2 WG/CU)
    case 2: return launch_cfg<64, 128, 2, 2, 4, AM>(a, s);    // 96 KB, wave 32x64
    case 3: return launch_cfg<128, 64, 2, 2, 4, AM>(a, s);    // 96 KB, wave 64x32
    case 4: return launch_cfg<64, 64, 2, 2, 4, AM>(a, s);     // 64 KB, wave 32x32
    case 5: return launch_cfg<256, 128, 4, 2, 3, AM>(a, s);   // 144 KB, 8 waves of 64x64
    case 6: return launch_cfg<128, 256, 2, 4, 3, AM>(a, s);   // 144 KB, 8 waves of 64x64
    case 7: return launch_cfg<128, 128, 2, 4, 4, AM>(a, s);   // 128 KB, 8 waves of 64x32
    case 8: return launch_cfg<64, 256, 1, 4, 3, AM>(a, s);    // 120 KB, wave 64x64
    case 9: return launch_cfg<256, 64, 4, 1, 3, AM>(a, s);    // 120 KB, wave 64x64
    // double-buffered, small LDS: several workgroups per CU overlap each
    // other's prologue / barrier / epilogue latency
    case 10: return launch_cfg<64, 64, 2, 2, 2, AM>(a, s);    // 32 KB (5 WG/CU)
    case 11: return launch_cfg<64, 128, 2, 2, 2, AM>(a, s);   // 48 KB (3 WG/CU)
    case 12: return launch_cfg<128, 64, 2, 2, 2, AM>(a, s);   // 48 KB (3 WG/CU)
    // 96-wide tiles: N = 768 (BERT-base hidden) is 8 of them, so an M = 4096
    // GEMM is exactly 256 tiles of 128 x 96 -- one per CU -- where 128 x 128
    // leaves a quarter of the CUs idle (192 tiles) and 128 x 64 needs 1.5 waves
    case 13: return launch_cfg<128, 96, 2, 2, 3, AM>(a, s);   // 84 KB, wave 64x48
    case 14: return launch_cfg<128, 96, 2, 2, 4, AM>(a, s);   // 112 KB
    case 15: return launch_cfg<64, 96, 2, 2, 3, AM>(a, s);    // 60 KB, wave 32x48
    // two waves per workgroup: a 64x64 tile as two 64x32 wave tiles reads 24 KB
    // of LDS fragments per k-step instead of the 32 KB four 32x32 waves read
    // (whose LDS reads take as long as their MFMAs at 256 B/clk)
    case 16: return launch_cfg<64, 64, 1, 2, 2, AM>(a, s);    // 32 KB, wave 64x32
    case 17: return launch_cfg<64, 64, 1, 2, 3, AM>(a, s);    // 48 KB
    case 18: return launch_cfg<64, 64, 2, 1, 3, AM>(a, s);    // 48 KB, wave 32x64
    case 19: return launch_cfg<128, 64, 2, 1, 2, AM>(a, s);   // 48 KB, wave 64x64
    case 20: return launch_cfg<64, 128, 1, 2, 2, AM>(a, s);   // 48 KB, wave 64x64
    case 21: return launch_cfg<128, 64, 2, 1, 3, AM>(a, s);   // 72 KB, wave 64x64
    case 22: return launch_cfg<64, 128, 1, 2, 3, AM>(a, s);   // 72 KB, wave 64x64
    case 23: return launch_cfg<64, 64, 2, 2, 3, AM>(a, s);    // 48 KB, wave 32x32
    // 8 waves of 64x96 (BERT's 2304 / 3072-wide projections at M = 4096: 192 /
    // 256 tiles, one per CU); 112 KB ring, epilogue in two 128-row passes
    case 24: return launch_cfg<256, 192, 4, 2, 2, AM>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool cgemm_fixup_ok(int cfg) {
  // the in-kernel split-K fixup needs the whole fp32 tile in LDS at once (one pass)
  const int i = cfg_index(cfg);
  return size_t(kBM[i]) * (kBN[i] + 4) * 4 <= 160 * 1024;
}

bool cgemm_supported(const IGemmArgs& a, int a_mode) {
  if (a.K <= 0 || a.K % KT || a.ldb % 8 || a.ldb < a.K) return false;
  if (a.N % 8 || a.ldc % 8 || (a.residual && a.ldr % 8)) return false;   // 16-B epilogue chunks only
  if (a.M >= (1 << 23)) return false;   // fdiv() row-index decomposition is exact below 2^23
  if (a_mode == kADense) return a.lda % 8 == 0 && a.lda >= a.K;
  if (a_mode == kAIm2col)
    return a.C % KT == 0 && a.KH * a.KW <= 32 && a.K == a.KH * a.KW * a.C &&
           a.a_bytes + int64_t(a.PT * a.W + a.PL) * a.C * 2 < 0x7ffffff0LL;
  if (a_mode == kAC4)
    return a.C == 4 && a.KW == 8 && a.KH % 2 == 0 && a.K == a.KH * 32 && a.PT == 0 && a.PL == 0 &&
           a.H >= (a.Ho - 1) * a.SH + a.KH && a.W >= (a.Wo - 1) * a.SW + a.KW;
  if (a_mode == kADual)
    return a.a2 && a.K1 > 0 && a.K1 % KT == 0 && a.lda % 8 == 0 && a.lda >= a.K1 && a.C % KT == 0 &&
           a.K == a.K1 + a.C && a.KH == 1 && a.KW == 1 && a.PT == 0 && a.PL == 0 && a.a2_bytes < 0x7ffffff0LL;
  return false;
}

int cgemm_config_bm(int cfg) { return kBM[cfg_index(cfg)]; }
int cgemm_config_bn(int cfg) { return kBN[cfg_index(cfg)]; }

hipError_t cgemm_launch(const IGemmArgs& a, int a_mode, int cfg, hipStream_t s) {
  if (!cgemm_cfg_id(cfg) || !cgemm_supported(a, a_mode)) return hipErrorInvalidValue;
  if (cfg >= kCGemmPfCfgBase) {
    const int idx = cfg_index(cfg);
    switch (a_mode) {
      case kAIm2col: return launch_mode_pf<1>(a, idx, s);
      case kADual: return launch_mode_pf<2>(a, idx, s);
      case kAC4: return launch_mode_pf<3>(a, idx, s);
      default: return launch_mode_pf<0>(a, idx, s);
    }
  }
  cfg = cfg_index(cfg);
  switch (a_mode) {
    case kAIm2col: return launch_mode<1>(a, cfg, s);
    case kADual: return launch_mode<2>(a, cfg, s);
    case kAC4: return launch_mode<3>(a, cfg, s);
    default: return launch_mode<0>(a, cfg, s);
  }
}

}  // namespace tfsk
