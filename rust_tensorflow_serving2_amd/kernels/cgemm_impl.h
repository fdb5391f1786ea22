// The pipelined MFMA conv / GEMM kernel template (cgemm.hip's header comment
// describes it) and its launcher, shared by the translation units that
// instantiate its configurations: cgemm.hip (16x16x32 MFMA builds) and
// cgemm32.hip (32x32x16 builds), compiled in parallel.
#pragma once
#include <type_traits>

#include "gemm_common.h"
#include "cgemm.h"

namespace tfsk {
namespace cgemm_impl {


using namespace gemm;
constexpr int kGroupM = 8;

template <int A>
struct ActC {
  static constexpr int value = A;
};

template <int BM, int BN, int WGM, int WGN, int S, int MF = 16, int KTT = 64>
struct CG {
  static constexpr int NW = WGM * WGN, NT = 64 * NW;
  static constexpr int WM = BM / WGM, WN = BN / WGN;
  // MF = 16: v_mfma_f32_16x16x32_bf16 tiles; MF = 32: v_mfma_f32_32x32x16_bf16
  static constexpr int TM = WM / MF, TN = WN / MF;
  // KTT: k-tile depth (LDS row = KTT * 2 bytes).  64 = one 128-B row per ring
  // slot row; 32 halves a ring slot, so the same LDS holds twice the slots:
  // the 256 x 192 tile then keeps 4 k-tiles in flight instead of 1
  static constexpr int CPR = KTT / 8;                              // 16-B chunks per LDS row
  static constexpr int RPD = 64 / CPR;                             // rows per 1-KB DMA piece
  // 1-KB DMA pieces per stage (NAP of A, NBP of B) over NW waves.  An even
  // split gives wave w the contiguous pieces w * APW ..; an uneven one (the
  // 192-row B tile in 16-row pieces: 12 over 8 waves) deals piece j * NW + w,
  // so some waves issue one piece more: every vmcnt wait then counts the
  // fewest pieces any wave issues per stage (PPW), which over-waits, never under
  static constexpr int NAP = BM / RPD, NBP = BN / RPD;
  static constexpr bool A_EVEN = NAP % NW == 0, B_EVEN = NBP % NW == 0;
  static constexpr int APW = (NAP + NW - 1) / NW, BPW = (NBP + NW - 1) / NW;   // per wave (at most)
  static constexpr int PPW = NAP / NW + NBP / NW;
  static constexpr int A_ST = BM * KTT, B_ST = BN * KTT;          // elements per ring slot
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
  // deferred LayerNorm: 3 x BM float2 (A stats, residual stats, output sums)
  // and 3 x BN floats (colsum, gamma, beta of the tile's columns) past
  // everything else (staged before the K loop); such launches ask for LDS_LNX
  static constexpr int LDS_LNX = LDS + 24 * BM + 12 * BN;
  static_assert(RPP % WM == 0, "epilogue passes split the tile at wave-row boundaries");
  static_assert(KTT == 64 || KTT == 32, "k-tile depth");
  static_assert(BM % RPD == 0 && BN % RPD == 0 && NAP >= NW && NBP >= NW, "DMA piece split");
  static_assert(MF == 16 || MF == 32, "MFMA shape");
  static_assert(TM >= 1 && TN >= 1 && WM % MF == 0 && WN % MF == 0, "wave tile");
  static_assert(S >= 2 && (S - 2) * PPW < 64 && (S - 2) * (APW + BPW) < 64, "ring depth / vmcnt range");
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

// Deferred-LayerNorm epilogue (IGemmArgs::st_out / a_st / r_st; the launcher
// admits dense, one-slice launches): `ln` = the LDS block ln_stage filled --
// this tile's rows' (mean, rstd) of A and of the residual, the rows' output
// (sum, sum sq) accumulators, and the tile columns' colsum / gamma / beta.
// Register budget: round 3's fold kept the column vectors in registers over
// the epilogue and spilled in the 8-wave tiles (256 VGPRs, 43-52 spills,
// profiles/round3/ln_fold.md), which cost QKV / FFN1 their best tile; here
// every chunk re-reads them from LDS (ds_read_b128; an opaque zero offset
// keeps the compiler from merging the unrolled chunks' identical reads into
// one hoisted, long-lived copy).  The per-row output sums: the 4 lanes of a row
// group (CPR = BN / 8 chunk lanes per row, 4-aligned) pre-reduce by xor
// shuffles, then one LDS float atomic per group; the loop body has no
// `continue`, so every lane reaches the shuffles.
template <int BM, int BN>
struct LnLds {
  float2* sa;      // [rows] (mean, rstd) of A
  float2* sr;      // [rows] (mean, rstd) of the residual
  float* red;      // [rows][2] output (sum, sum sq)
  const float* cs; // [BN] colsum / gamma / beta of the tile's columns
  const float* rg;
  const float* rb;
};

template <int BM, int BN, int NT, int CS_LD, int ACT, bool USE_PRE, int TBM, int TBN>
__device__ __forceinline__ void epilogue_lnx(const IGemmArgs& p, const float* Cs, int m0, int n0, int tid,
                                             const uint4 (&rpre)[Epi<BM, BN, NT>::PRE > 0 ? Epi<BM, BN, NT>::PRE : 1],
                                             const float4 b0, const float4 b1, const LnLds<TBM, TBN>& ln) {
  using E = Epi<BM, BN, NT>;
  constexpr int PRE = USE_PRE ? E::PRE : 0;
  static_assert(E::CPR % 4 == 0 && E::NTE % 4 == 0, "row groups of 4 chunk lanes");
  const int M = p.M, N = p.N;
  const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  auto chunk = [&](int it, bool use_pre) __attribute__((always_inline)) {
    int row, col;
    bool in = epi_rowcol<BM, BN, NT>(tid, it, row, col);
    const int m = m0 + row, n = n0 + col;
    in = in && m < M && n < N;
    float s = 0.f, q = 0.f;
    if (in) {
      int z;
      asm volatile("v_mov_b32 %0, 0" : "=v"(z));
      const int c = col + z;
      float v[8];
      load8f(Cs + row * CS_LD + col, v);
      const float alpha = p.alpha;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= alpha;
      if (p.a_st) {
        const float2 st = ln.sa[row];
        float cs[8];
        load8f(ln.cs + c, cs);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = st.y * (v[e] - st.x * cs[e]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bv[e];
      if (p.residual) {
        const uint4 rr = use_pre ? rpre[PRE > 0 ? it : 0]
                                 : *reinterpret_cast<const uint4*>(p.residual + size_t(m) * p.ldr + n);
        const uint32_t w[4] = {rr.x, rr.y, rr.z, rr.w};
        float r[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          r[2 * e] = __uint_as_float(w[e] << 16);
          r[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
        }
        if (p.r_st) {
          const float2 st = ln.sr[row];
          float g[8], b[8];
          load8f(ln.rg + c, g);
          load8f(ln.rb + c, b);
#pragma unroll
          for (int e = 0; e < 8; ++e) r[e] = (r[e] - st.x) * st.y * g[e] + b[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = act_fn<ACT>(v[e]);
      store_chunk(p, p.out, m, n, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = static_cast<float>(static_cast<__bf16>(v[e]));   // the value stored
        s += f;
        q += f * f;
      }
    }
    if (p.st_out) {
      s += __shfl_xor(s, 1, 64);
      q += __shfl_xor(q, 1, 64);
      s += __shfl_xor(s, 2, 64);
      q += __shfl_xor(q, 2, 64);
      if (in && (tid & 3) == 0) {
        atomicAdd(ln.red + 2 * row, s);
        atomicAdd(ln.red + 2 * row + 1, q);
      }
    }
  };
  // (unrolled: every chunk's residual load in flight at once.  The 8-wave
  // 256 x 192 tile spills ~37 VGPRs with this epilogue, 10 without -- all
  // stored after the K loop and reloaded in the epilogue, none in the MFMA
  // loop: -Rpass-analysis=kernel-resource-usage + the ISA, round 5)
  if constexpr (ACT != kActGeluErf) {
#pragma unroll
    for (int it = 0; it < E::ITERS; ++it) chunk(it, PRE > 0);
  } else {
#pragma unroll 1
    for (int it = 0; it < E::ITERS; ++it) chunk(it, false);
  }
}

// Deferred-LayerNorm staging, in two halves around the prologue's DMA issue:
// ln_fetch (kernel start) loads this thread's row partials (thread r < BM:
// tile row r; up to kLnPre partials per side as 16-B buffer loads, lanes past
// a row's partials read past the resource: zeros) and column values (thread
// c < BN); ln_stage (after the prologue's DMAs are issued) reduces them into
// LnLds.  The loads are the oldest in flight, so the compiler's vmcnt wait
// before the stage lets the k-tile DMAs keep flying; an epilogue-time fetch
// stalled every workgroup for ~3 dependent memory round trips (round 5:
// QKV / FFN1 +5-7 us each).  More partials than kLnPre: read in ln_stage.
constexpr int kLnPre = 8;

struct LnPre {
  u32x4 a[kLnPre / 2], r[kLnPre / 2];
  float cs, g, b;
};

__device__ __forceinline__ void ln_fetch_rows(const float* st, int parts, int M, int m, bool on, u32x4 (&v)[kLnPre / 2]) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(st), 0, int(long(M) * parts * 8), 0x00020000);
  const uint32_t base = uint32_t(m) * uint32_t(parts) * 8u;
#pragma unroll
  for (int j = 0; j < kLnPre / 2; ++j)
    v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, on && 2 * j < parts ? base + 16u * j : kOOB, 0, 0);
}

template <int BM, int BN>
__device__ __forceinline__ void ln_fetch(const IGemmArgs& p, int m0, int n0, int tid, LnPre& f) {
  const int m = min(m0 + tid, p.M - 1);
  const bool row = tid < BM;
  if (p.a_st) ln_fetch_rows(p.a_st, p.a_parts, p.M, m, row && p.a_parts <= kLnPre, f.a);
  if (p.r_st) ln_fetch_rows(p.r_st, p.r_parts, p.M, m, row && p.r_parts <= kLnPre, f.r);
  const uint32_t c = tid < BN && n0 + tid < p.N ? uint32_t(n0 + tid) * 4u : kOOB;
  const int nb = p.N * 4;
  f.cs = f.g = f.b = 0.f;
  if (p.a_st)
    f.cs = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.a_colsum), 0, nb, 0x00020000), c, 0, 0));
  if (p.r_st) {
    f.g = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.r_gamma), 0, nb, 0x00020000), c, 0, 0));
    f.b = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.r_beta), 0, nb, 0x00020000), c, 0, 0));
  }
}

__device__ __forceinline__ float2 ln_finish(const u32x4 (&v)[kLnPre / 2], int parts, float inv_len, float eps) {
  float a = 0.f, b = 0.f;
#pragma unroll
  for (int j = 0; j < kLnPre / 2; ++j) {
    a += __uint_as_float(v[j].x);
    b += __uint_as_float(v[j].y);
    if (2 * j + 1 < parts) {            // the upper half belongs to the next row past the last partial
      a += __uint_as_float(v[j].z);
      b += __uint_as_float(v[j].w);
    }
  }
  const float mean = a * inv_len;
  return make_float2(mean, rsqrtf(fmaxf(b * inv_len - mean * mean, 0.f) + eps));
}

template <int BM, int BN, int NT>
__device__ __forceinline__ LnLds<BM, BN> ln_stage(const IGemmArgs& p, int m0, int tid, char* base, const LnPre& f) {
  static_assert(BM <= NT && BN <= NT, "one tile row / column per thread");
  LnLds<BM, BN> l;
  float2* st = reinterpret_cast<float2*>(base);
  float* vec = reinterpret_cast<float*>(st + 3 * BM);
  l.sa = st;
  l.sr = st + BM;
  l.red = reinterpret_cast<float*>(st + 2 * BM);
  l.cs = vec;
  l.rg = vec + BN;
  l.rb = vec + 2 * BN;
  if (tid < BM) {
    const int m = min(m0 + tid, p.M - 1);
    if (p.a_st)
      st[tid] = p.a_parts <= kLnPre ? ln_finish(f.a, p.a_parts, 1.f / float(p.K), p.a_eps)
                                    : ln_row_stats(p.a_st, p.a_parts, m, 1.f / float(p.K), p.a_eps);
    if (p.r_st)
      st[BM + tid] = p.r_parts <= kLnPre ? ln_finish(f.r, p.r_parts, 1.f / float(p.N), p.r_eps)
                                         : ln_row_stats(p.r_st, p.r_parts, m, 1.f / float(p.N), p.r_eps);
    st[2 * BM + tid] = make_float2(0.f, 0.f);
  }
  if (tid < BN) {
    vec[tid] = f.cs;
    vec[BN + tid] = f.g;
    vec[2 * BN + tid] = f.b;
  }
  return l;
}

// Waves per SIMD the register allocation must leave room for: the 4-wave
// 32-KB tiles (64x64, 2 slots) fit 5 workgroups per CU by LDS, i.e. 5 waves
// per SIMD, which needs <= 102 VGPRs (unconstrained they took 128: 4 per CU)
template <int BM, int BN, int WGM, int WGN, int S, bool PF, int MF = 16, int KTT = 64>
constexpr int cg_waves_per_eu() {
  return (!PF && WGM * WGN == 4 && CG<BM, BN, WGM, WGN, S, MF, KTT>::LDS <= 32 * 1024) ? 5 : 1;
}

// LDS image swizzle: 16-B chunk c of tile row r sits in slot c ^ swz(r).  The
// 16x16x32 fragment reads (16 rows x 4 chunks per 64 lanes) are conflict-free
// with r & 7; the 32x32x16 reads (32 rows x 2 chunks) are 2-way with it and
// conflict-free with (r >> 1) & 7, which also keeps the 16x16 reads
// conflict-free (ds_read_b128 lane groups, MI355X_MICROARCH.md LDS table;
// checked by brute force over every group and k-subtile).
// 64-B rows (KTT = 32; 4 chunks, a 256-B bank row holds 4 rows): chunk c of
// row r in slot c ^ (bit 3 of r) * 2 ^ (bit 4 of r), conflict-free for both
// MFMA shapes (same brute-force check).
template <int MF, int KTT = 64>
__device__ __forceinline__ int lds_swz(int r) {
  if constexpr (KTT == 32) return (((r >> 3) & 1) << 1) | ((r >> 4) & 1);
  return MF == 32 ? (r >> 1) & 7 : r & 7;
}

// PF: fragment-prefetch step pipeline -- step t's fragments are read from LDS
// right after its barrier while the MFMAs of step t - 1 (fragments already in
// registers) issue, so neither the LDS read latency nor the barrier sits
// between a k-tile landing and its MFMAs (halo.hip uses the same scheme).
// LNX: the deferred-LayerNorm build (dense only, launch_cfg picks it when the
// launch carries statistics): its epilogue / staging registers would
// otherwise count against every launch -- with the LN code in all builds the
// 64 x 64 four-slot tiles dropped from 4 to 3 waves per SIMD (VGPRs 107 -> 109
// next to 20 AGPRs) and ResNet-50 b1 slowed from 0.375 to 0.400 ms (round 5)
template <int BM, int BN, int WGM, int WGN, int S, int AM, bool PF, int MF = 16, int KTT = 64, bool LNX = false>
__global__ __launch_bounds__(64 * WGM * WGN, (cg_waves_per_eu<BM, BN, WGM, WGN, S, PF, MF, KTT>())) void cgemm_kernel(IGemmArgs p) {
  using G = CG<BM, BN, WGM, WGN, S, MF, KTT>;
  static_assert((MF == 16 && KTT == 64) || !PF, "the fragment-prefetch variant is built for 16x16x32, 64-deep only");
  constexpr bool IM2COL = (AM == 1), DUAL = (AM == 2), STEM = (AM == 3);
  static_assert(KTT == 64 || !STEM, "the stem operand layout packs two filter rows per 64-deep k-tile");
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
  // DMA lane -> row (lane / CPR) of its RPD-row piece, LDS slot (lane % CPR)
  // holding logical chunk (lane % CPR) ^ swz(row)
  const int prow = lane / G::CPR;
  auto kc_of = [&](int piece) -> uint32_t {
    return uint32_t(((lane % G::CPR) ^ lds_swz<MF, KTT>(piece * G::RPD + prow)) * 8);
  };

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
  auto a_piece = [&](int j) { return G::A_EVEN ? wid * G::APW + j : j * G::NW + wid; };
  auto b_piece = [&](int j) { return G::B_EVEN ? wid * G::BPW + j : j * G::NW + wid; };
  uint32_t a_off[G::APW], a_msk[G::APW], a_off2[DUAL ? G::APW : 1];
#pragma unroll
  for (int j = 0; j < G::APW; ++j) {
    const int m = m0 + a_piece(j) * G::RPD + prow;
    const bool ok = m < M;
    const uint32_t kc = kc_of(a_piece(j));
    a_msk[j] = 0;
    if (STEM) {
      // pre-padded bf16 RGBA, k = kh*32 + kw*4 + c: a k-tile is filter rows
      // (2t, 2t+1) x 8 taps x 4 channels = 2 runs of 64 contiguous bytes; this
      // lane's logical chunk lc holds row lc>>2, pixels 2*(lc&3) .. +1
      const int lc = int(kc >> 3);
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
    const int n = n0 + b_piece(j) * G::RPD + prow;
    b_off[j] = n < N ? (uint32_t(n) * uint32_t(p.ldb) + kc_of(b_piece(j))) * 2u : kOOB;
  }

  // ---- k range of this workgroup (split-K: blockIdx.y selects a slice)
  const int nk_all = p.K / KTT;
  int kt0 = 0, nk = nk_all;
  if (p.splits > 1) {
    kt0 = blockIdx.y * p.kt_per_split;
    nk = min(nk_all - kt0, p.kt_per_split);
  }

  // ---- scalar producer walk: k element offset; im2col tap (kh, kw) + channel offset
  int w_k = kt0 * KTT;
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
        if (!G::A_EVEN && a_piece(j) >= G::NAP) continue;   // wave-uniform
        const uint32_t v = a_off2[DUAL ? j : 0];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsA2, (lds_ptr_t)(smem + (slot * G::A_ST + a_piece(j) * 512) * 2), 16, v, soff2, 0, 0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < G::APW; ++j) {
        if (!G::A_EVEN && a_piece(j) >= G::NAP) continue;   // wave-uniform
        uint32_t v = a_off[j];
        if (IM2COL) v = ((a_msk[j] >> w_tap) & 1u) ? v : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsA, (lds_ptr_t)(smem + (slot * G::A_ST + a_piece(j) * 512) * 2), 16, v, a_soff, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < G::BPW; ++j) {
      if (!G::B_EVEN && b_piece(j) >= G::NBP) continue;     // wave-uniform
      // (a named local, not b_off[j] in the call: with the array element as a
      // builtin argument hipcc's host pass silently drops the kernel stub)
      const uint32_t v = b_off[j];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (lds_ptr_t)(smem + (S * G::A_ST + slot * G::B_ST + b_piece(j) * 512) * 2), 16, v, b_soff,
          0, 0);
    }
    w_k += KTT;
    if (IM2COL) {
      w_ci += KTT;
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
  // 32x32x16 fragments: lane l holds row l & 31 at k = 16 kk + 8 (l >> 5) .. + 7
  // (chunk 2 kk + (l >> 5)); the wave's row offsets are multiples of 32, so
  // the swizzle term depends on l only
  const int r32 = lane & 31, h32 = lane >> 5;
  constexpr int KK32 = KTT / 16;                 // 32x32x16 k-subtiles per k-tile
  uint32_t ra32[KK32], rb32[KK32];
#pragma unroll
  for (int kk = 0; kk < KK32; ++kk) {
    const uint32_t ch = uint32_t(((2 * kk + h32) ^ lds_swz<MF, KTT>(r32)) * 16);
    ra32[kk] = uint32_t((wm * G::WM + r32) * KTT * 2) + ch;
    rb32[kk] = uint32_t((wn * G::WN + r32) * KTT * 2) + ch;
  }
  // 16x16x32 on 64-B rows: one k-subtile per k-tile, and the swizzle reads
  // row bits 3-4, which the fragment index i (16 rows) changes
  uint32_t ra16[KTT == 32 ? G::TM : 1], rb16[KTT == 32 ? G::TN : 1];
  if constexpr (KTT == 32) {
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int r = wm * G::WM + i * 16 + fr;
      ra16[i] = uint32_t((r * KTT + ((fq ^ lds_swz<MF, KTT>(r)) * 8)) * 2);
    }
#pragma unroll
    for (int j = 0; j < G::TN; ++j) {
      const int r = wn * G::WN + j * 16 + fr;
      rb16[j] = uint32_t((r * KTT + ((fq ^ lds_swz<MF, KTT>(r)) * 8)) * 2);
    }
  }

  using AccT = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  AccT acc[G::TM][G::TN];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j) acc[i][j] = AccT{};

  auto compute = [&](int slot) {
    const char* sa = smem + slot * G::A_ST * 2;
    const char* sb = smem + (S * G::A_ST + slot * G::B_ST) * 2;
    if constexpr (MF == 32) {
#pragma unroll
      for (int kk = 0; kk < KK32; ++kk) {
        bf16x8 af[G::TM], bfr[G::TN];
#pragma unroll
        for (int i = 0; i < G::TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sa + ra32[kk] + i * 32 * KTT * 2);
#pragma unroll
        for (int j = 0; j < G::TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sb + rb32[kk] + j * 32 * KTT * 2);
#pragma unroll
        for (int i = 0; i < G::TM; ++i)
#pragma unroll
          for (int j = 0; j < G::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
      return;
    } else if constexpr (KTT == 32) {
      bf16x8 af[G::TM], bfr[G::TN];
#pragma unroll
      for (int i = 0; i < G::TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sa + ra16[i]);
#pragma unroll
      for (int j = 0; j < G::TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sb + rb16[j]);
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      return;
    } else {
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
    if constexpr (MF == 16) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < G::TM; ++i)
#pragma unroll
          for (int j = 0; j < G::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[kk][i], f.b[kk][j], acc[i][j], 0, 0, 0);
    }
  };
  Frags prev;

  uint4 rpre[Epi<BM, BN, G::NT>::PRE > 0 ? Epi<BM, BN, G::NT>::PRE : 1];
  if constexpr (G::PASSES == 1) prefetch_residual<BM, BN, G::NT>(p, m0, n0, tid, rpre);
  float4 bias0, bias1;
  // two-pass tiles run each pass's epilogue on that pass's own waves (see the
  // epilogue): a thread's epilogue column then follows its index in its half
  const int etid = G::PASSES == 2 ? tid - ((wm * G::WM) / G::RPP) * (G::NT / 2) : tid;
  if constexpr (G::PASSES == 2)
    prefetch_bias<BM, BN, G::NT / 2>(p, n0, etid, bias0, bias1);
  else
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

  // deferred LayerNorm (runtime-uniform; the launcher admits it for dense,
  // one-slice tiles only): row statistics and column vectors fetched now,
  // staged into the LDS past the ring / fp32 tile once the prologue is issued
  const bool lnx = LNX && !STEM && (p.st_out != nullptr || p.a_st != nullptr || p.r_st != nullptr);
  LnPre lpre;
  if (lnx) ln_fetch<BM, BN>(p, m0, n0, tid, lpre);

  // ---- prologue: S-1 k-tiles in flight
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk && do_dma) issue(s);
  LnLds<BM, BN> ln{};
  if (lnx) ln = ln_stage<BM, BN, G::NT>(p, m0, tid, smem + G::LDS, lpre);

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
  auto stage = [&](int ps) __attribute__((always_inline)) {    // this wave's accumulators of pass ps -> Cs
    if constexpr (MF == 32) {
      // C/D of 32x32x16: column lane & 31, row (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            Cs[(wm * G::WM - ps * RPP + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32) * G::CS_LD + wn * G::WN +
               j * 32 + r32] = acc[i][j][r];
    } else {
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(wm * G::WM - ps * RPP + i * 16 + fq * 4 + r) * G::CS_LD + wn * G::WN + j * 16 + fr] = acc[i][j][r];
    }
  };
  if constexpr (MF == 16 && BM * (BN + 8) * 2 <= G::LDS && (BM * (BN / 8)) % G::NT == 0) {
    // Plain bf16 output (no residual / second output / deferred LayerNorm,
    // activation without erf): bias and activation applied in registers and
    // the bf16 tile staged in ONE pass by every wave, half the LDS bytes of
    // the fp32 image.  The 256 x 192 tile's two-pass fp32 path below runs
    // its passes on half the waves each, one after the other: its epilogue
    // took 5.7 of 23.4 us of the workgroup's life, 2.8 us this way
    // (profiles/round5/s2/wgt.log, s49/wgt.log).  Same arithmetic as
    // epi_chunk (fma(acc, alpha, bias) + 0, act, RNE to bf16).
    if (p.splits <= 1 && !lnx && p.residual == nullptr && p.out2 == nullptr && !p.out_f32 && p.out != nullptr &&
        p.act != kActGeluErf && !p.epi_f32) {
      constexpr int CB_LD = BN + 8;
      uint16_t* Cb = reinterpret_cast<uint16_t*>(smem);
      const bool use_b = p.bias != nullptr && p.N % 8 == 0;
      const __amdgpu_buffer_rsrc_t rsb =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.bias), 0, use_b ? p.N * 4 : 0, 0x00020000);
      float bj[G::TN];
#pragma unroll
      for (int j = 0; j < G::TN; ++j)
        bj[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            rsb, uint32_t(n0 + wn * G::WN + j * 16 + fr) * 4u, 0, 0));
      const float alpha = p.alpha;
      auto stage_bf16 = [&](auto actc) __attribute__((always_inline)) {
        constexpr int ACT = decltype(actc)::value;
#pragma unroll
        for (int i = 0; i < G::TM; ++i)
#pragma unroll
          for (int j = 0; j < G::TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = act_fn<ACT>(acc[i][j][r] * alpha + bj[j] + 0.f);
              Cb[(wm * G::WM + i * 16 + fq * 4 + r) * CB_LD + wn * G::WN + j * 16 + fr] =
                  __builtin_bit_cast(uint16_t, static_cast<__bf16>(v));
            }
      };
      switch (p.act) {
        case kActRelu: stage_bf16(ActC<kActRelu>{}); break;
        case kActGeluTanh: stage_bf16(ActC<kActGeluTanh>{}); break;
        case kActTanh: stage_bf16(ActC<kActTanh>{}); break;
        default: stage_bf16(ActC<0>{}); break;
      }
      __syncthreads();
      constexpr int CPRB = BN / 8;
#pragma unroll
      for (int it = 0; it < BM * CPRB / G::NT; ++it) {
        const int c = tid + it * G::NT, row = c / CPRB, ch = c - row * CPRB;
        const int m = m0 + row, n = n0 + ch * 8;
        if (m < M && n < N)
          *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p.out) + size_t(m) * p.ldc + n) =
              *reinterpret_cast<const uint4*>(Cb + row * CB_LD + ch * 8);
      }
      trace_stamp(p, 3);
      return;
    }
  }
  if constexpr (G::PASSES == 2) {
    if (p.splits <= 1) {
      // Two-pass tiles (256 x 192): pass ps's rows belong to half of the waves.
      // Each half stages its accumulators and runs its pass's epilogue alone,
      // on two wave-uniform paths with matching barriers: the other half's
      // accumulators are not live during an epilogue, which kept the 8-wave
      // tile's epilogue from spilling (10 VGPRs with the plain epilogue, 37
      // with the deferred-LayerNorm one when all waves ran both passes).
      constexpr int ENT = G::NT / 2;
      using RPn = uint4[Epi<RPP, BN, ENT>::PRE > 0 ? Epi<RPP, BN, ENT>::PRE : 1];
      const RPn& rpn = *reinterpret_cast<const RPn*>(rpre);   // not read (USE_PRE = false)
      auto epi = [&](int ps) __attribute__((always_inline)) {
        const int mp = m0 + ps * RPP;
        bool done = false;
        if constexpr (LNX) if (lnx) {
          done = true;
          LnLds<BM, BN> lp = ln;
          lp.sa += ps * RPP;
          lp.sr += ps * RPP;
          lp.red += 2 * ps * RPP;
          switch (p.act) {
            case kActRelu: epilogue_lnx<RPP, BN, ENT, G::CS_LD, kActRelu, false>(p, Cs, mp, n0, etid, rpn, bias0, bias1, lp); break;
            case kActGeluTanh: epilogue_lnx<RPP, BN, ENT, G::CS_LD, kActGeluTanh, false>(p, Cs, mp, n0, etid, rpn, bias0, bias1, lp); break;
            case kActGeluErf: epilogue_lnx<RPP, BN, ENT, G::CS_LD, kActGeluErf, false>(p, Cs, mp, n0, etid, rpn, bias0, bias1, lp); break;
            case kActTanh: epilogue_lnx<RPP, BN, ENT, G::CS_LD, kActTanh, false>(p, Cs, mp, n0, etid, rpn, bias0, bias1, lp); break;
            default: epilogue_lnx<RPP, BN, ENT, G::CS_LD, 0, false>(p, Cs, mp, n0, etid, rpn, bias0, bias1, lp); break;
          }
        }
        if (!done) {
          switch (p.act) {
            case kActRelu: epilogue_rows<RPP, BN, ENT, G::CS_LD, kActRelu, false>(p, Cs, mp, n0, etid, rpn, bias0, bias1); break;
            case kActGeluTanh: epilogue_rows<RPP, BN, ENT, G::CS_LD, kActGeluTanh, false>(p, Cs, mp, n0, etid, rpn, bias0, bias1); break;
            case kActGeluErf: epilogue_rows<RPP, BN, ENT, G::CS_LD, kActGeluErf, false>(p, Cs, mp, n0, etid, rpn, bias0, bias1); break;
            case kActTanh: epilogue_rows<RPP, BN, ENT, G::CS_LD, kActTanh, false>(p, Cs, mp, n0, etid, rpn, bias0, bias1); break;
            default: epilogue_rows<RPP, BN, ENT, G::CS_LD, 0, false>(p, Cs, mp, n0, etid, rpn, bias0, bias1); break;
          }
        }
      };
      if (__builtin_amdgcn_readfirstlane((wm * G::WM) / RPP) == 0) {
        stage(0);
        __syncthreads();          // B1: pass 0 staged
        epi(0);
        __syncthreads();          // B2: pass 0 read
        __syncthreads();          // B3
        __syncthreads();          // B4
      } else {
        __syncthreads();          // B1
        __syncthreads();          // B2
        stage(1);
        __syncthreads();          // B3: pass 1 staged
        epi(1);
        __syncthreads();          // B4: pass 1 done
      }
      if (lnx && p.st_out != nullptr) {
        const float2* red = reinterpret_cast<const float2*>(ln.red);
        for (int r = tid; r < BM; r += G::NT)
          if (m0 + r < M) reinterpret_cast<float2*>(p.st_out)[size_t(m0 + r) * nbn + bn] = red[r];
      }
      trace_stamp(p, 3);
      return;
    }
  }
#pragma unroll
  for (int ps = 0; ps < G::PASSES; ++ps) {
    if (ps > 0) __syncthreads();    // the previous pass has read Cs
    if (G::PASSES == 1 || (wm * G::WM) / RPP == ps) stage(ps);
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
    if constexpr (LNX) if (lnx) {
      LnLds<BM, BN> lp = ln;                 // this pass's rows
      lp.sa += ps * RPP;
      lp.sr += ps * RPP;
      lp.red += 2 * ps * RPP;
      switch (p.act) {
        case kActRelu: epilogue_lnx<RPP, BN, G::NT, G::CS_LD, kActRelu, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1, lp); break;
        case kActGeluTanh: epilogue_lnx<RPP, BN, G::NT, G::CS_LD, kActGeluTanh, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1, lp); break;
        case kActGeluErf: epilogue_lnx<RPP, BN, G::NT, G::CS_LD, kActGeluErf, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1, lp); break;
        case kActTanh: epilogue_lnx<RPP, BN, G::NT, G::CS_LD, kActTanh, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1, lp); break;
        default: epilogue_lnx<RPP, BN, G::NT, G::CS_LD, 0, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1, lp); break;
      }
      continue;
    }
    switch (p.act) {
      case kActRelu: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActRelu, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1); break;
      case kActGeluTanh: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActGeluTanh, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1); break;
      case kActGeluErf: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActGeluErf, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1); break;
      case kActTanh: epilogue_rows<RPP, BN, G::NT, G::CS_LD, kActTanh, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1); break;
      default: epilogue_rows<RPP, BN, G::NT, G::CS_LD, 0, P1>(p, Cs, mp, n0, tid, rp, bias0, bias1); break;
    }
  }
  if (lnx && p.st_out != nullptr) {
    // this tile's (sum, sum sq) of each of its rows -> slot bn of the row
    __syncthreads();
    const float2* red = reinterpret_cast<const float2*>(ln.red);
    for (int r = tid; r < BM; r += G::NT)
      if (m0 + r < M) reinterpret_cast<float2*>(p.st_out)[size_t(m0 + r) * nbn + bn] = red[r];
  }
  trace_stamp(p, 3);
}

template <int BM, int BN, int WGM, int WGN, int S, int AM, bool PF = false, int MF = 16, int KTT = 64>
hipError_t launch_cfg(const IGemmArgs& a0, hipStream_t s) {
  using G = CG<BM, BN, WGM, WGN, S, MF, KTT>;
  const bool lnx = a0.st_out != nullptr || a0.a_st != nullptr || a0.r_st != nullptr;
  if (lnx && (AM != 0 || (BN / 8) % 4 != 0 || a0.splits > 1 || a0.out2 != nullptr || G::LDS_LNX > 160 * 1024 ||
              (a0.st_out != nullptr && (a0.out_f32 || a0.out == nullptr)) ||
              (a0.a_st != nullptr && (a0.a_colsum == nullptr || a0.a_parts < 1)) ||
              (a0.r_st != nullptr && (a0.residual == nullptr || a0.r_gamma == nullptr || a0.r_beta == nullptr ||
                                      a0.r_parts < 1)) ||
              a0.N % 8 != 0))
    return hipErrorInvalidValue;                    // deferred LayerNorm: dense, one K slice, bf16 sums
  const int lds = lnx ? G::LDS_LNX : G::LDS;
  IGemmArgs a = a0;
  a.epi_f32 = epi_f32_env();
  const int nk = a.K / KTT;
  const int splits = a.splits > 1 ? a.splits : 1;
  if (splits > 1) a.kt_per_split = (nk + splits - 1) / splits;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (tiles == 0) return hipSuccess;
  if constexpr (AM == 0 && (BN / 8) % 4 == 0) {     // (epilogue_lnx row groups of 4 chunk lanes)
    if (lnx) {
      hipError_t e = ensure_dyn_lds(
          reinterpret_cast<const void*>(&cgemm_kernel<BM, BN, WGM, WGN, S, AM, PF, MF, KTT, true>), lds);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL((cgemm_kernel<BM, BN, WGM, WGN, S, AM, PF, MF, KTT, true>), dim3(tiles, splits), dim3(G::NT),
                         lds, s, a);
      return hipGetLastError();
    }
  }
  hipError_t e =
      ensure_dyn_lds(reinterpret_cast<const void*>(&cgemm_kernel<BM, BN, WGM, WGN, S, AM, PF, MF, KTT>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((cgemm_kernel<BM, BN, WGM, WGN, S, AM, PF, MF, KTT>), dim3(tiles, splits), dim3(G::NT), lds,
                     s, a);
  return hipGetLastError();
}

}  // namespace cgemm_impl
}  // namespace tfsk
