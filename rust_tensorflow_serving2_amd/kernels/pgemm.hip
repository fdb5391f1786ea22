// Persistent multi-tile MFMA conv / GEMM (config ids kPGemmCfgBase + idx;
// cgemm_launch dispatches here).
//
// Why: at ResNet-50 b32 a cgemm launch is one wave of workgroups that all
// start together and run fill -> K loop -> epilogue in lockstep; per-workgroup
// phase traces put fill + epilogue at 30-42 % of a launch span
// (docs/benchmarks.md, "Where a conv / GEMM launch spends its time"), and the
// many-tile layers (stage 2-3: 1-4 k-steps per 64x64 tile, 1.5k-6k tiles) pay
// the fill latency once per tile.  Here a grid of (co-resident) workgroups
// loops over the tiles, and the DMA ring runs over the FLATTENED (tile, k-step)
// sequence: while tile i's last k-steps compute and its epilogue stores, the
// ring already holds the first S - 1 k-tiles of tile i + 1, so only a
// workgroup's first tile waits for a fill.  The fp32 epilogue staging area is
// its own LDS region (not aliased with the ring) for that reason.
//
// Same operand contract as cgemm (dense / im2col / dual A modes, 64-aligned;
// cgemm_supported), same epilogue (bias, residual, activation, post output),
// 16x16x32 MFMA, 64-deep k-tiles, no split-K (each tile's K loop is whole).
//
// Waits: the ring wait counts only the younger DMA loads (S - 2 k-tiles of
// pieces).  The epilogue's stores sit in the same vmcnt counter; a pending
// store only makes such a wait longer (loads complete in order among
// themselves, so "at most N pending" still implies the awaited k-tile
// landed), never shorter -- the count never includes stores.
#include "cgemm_impl.h"

namespace tfsk {

namespace {

using namespace gemm;
using cgemm_impl::CG;
using cgemm_impl::epilogue_rows;
using cgemm_impl::kGroupM;

template <int BM, int BN, int WGM, int WGN, int S>
struct PG {
  using G = CG<BM, BN, WGM, WGN, S, 16, 64>;
  static constexpr int CS_LD = BN + 4;
  static constexpr int RING = G::LDS_MAIN;                 // bytes of the DMA ring
  static constexpr int EPI = BM * CS_LD * 4;               // fp32 staging, after the ring
  static constexpr int LDS = RING + EPI;
  static_assert(LDS <= 160 * 1024, "LDS budget (ring + separate epilogue staging)");
  static_assert(S >= 2 && S <= 4, "ring depth (the tail waits cover up to 2 younger k-tiles)");
};

// tile `t` of the launch (logical order) -> (m0, n0): GROUP_M column sweeps
template <int BM, int BN>
__device__ __forceinline__ void tile_mn(int t, int nbm, int nbn, int& m0, int& n0) {
  const int per_group = kGroupM * nbn;
  const int first_m = (t / per_group) * kGroupM;
  const int gsz = min(nbm - first_m, kGroupM);
  m0 = (first_m + (t % per_group) % gsz) * BM;
  n0 = ((t % per_group) / gsz) * BN;
}

template <int BM, int BN, int WGM, int WGN, int S, int AM>
__global__ __launch_bounds__(64 * WGM * WGN) void pgemm_kernel(IGemmArgs p) {
  using P = PG<BM, BN, WGM, WGN, S>;
  using G = typename P::G;
  constexpr bool IM2COL = (AM == 1), DUAL = (AM == 2);
  static_assert(AM == 0 || AM == 1 || AM == 2, "dense / im2col / dual operands");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  char* const smem = reinterpret_cast<char*>(smem_raw);
  float* const Cs = reinterpret_cast<float*>(smem + P::RING);
  typedef __attribute__((address_space(3))) void* lds_ptr_t;

  const int M = p.M, N = p.N;
  const int nbm = (M + BM - 1) / BM, nbn = (N + BN - 1) / BN;
  const int ntiles = nbm * nbn;
  // this workgroup's tiles: slot, slot + G, ... (slot = XCD-remapped block id,
  // so the workgroups of one XCD work on neighbouring tiles in each round)
  const int slot = xcd_remap(blockIdx.x, gridDim.x);
  const int mine = slot < ntiles ? (ntiles - slot + int(gridDim.x) - 1) / int(gridDim.x) : 0;
  const int nk = p.K / KT;
  const int T = mine * nk;                         // flattened (tile, k-step) sequence
  trace_stamp(p, 0);
  if (T == 0) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int prow = lane / G::CPR;
  auto kc_of = [&](int piece) -> uint32_t {
    return uint32_t(((lane % G::CPR) ^ cgemm_impl::lds_swz<16, 64>(piece * G::RPD + prow)) * 8);
  };

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
  const __amdgpu_buffer_rsrc_t rsA2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(DUAL ? p.a2 : p.a), 0, int(DUAL ? p.a2_bytes : p.a_bytes), 0x00020000);

  const float inv_hw = 1.f / float(p.Ho * p.Wo), inv_wo = 1.f / float(p.Wo);
  auto a_piece = [&](int j) { return G::A_EVEN ? wid * G::APW + j : j * G::NW + wid; };
  auto b_piece = [&](int j) { return G::B_EVEN ? wid * G::BPW + j : j * G::NW + wid; };

  // ---- producer: per-lane DMA offsets of the tile it fills, and its k walk
  uint32_t a_off[G::APW], a_msk[G::APW], a_off2[DUAL ? G::APW : 1], b_off[G::BPW];
  int w_k = 0, w_ci = 0, w_kh = 0, w_kw = 0, w_tap = 0;
  int p_i = 0, p_k = 0;                            // producer: my tile index, k-step in it
  auto set_producer_tile = [&](int i) {
    int m0, n0;
    tile_mn<BM, BN>(slot + i * int(gridDim.x), nbm, nbn, m0, n0);
#pragma unroll
    for (int j = 0; j < G::APW; ++j) {
      const int m = m0 + a_piece(j) * G::RPD + prow;
      const bool ok = m < M;
      const uint32_t kc = kc_of(a_piece(j));
      a_msk[j] = 0;
      if (!IM2COL) {
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
        const int hb = ho * p.SH, wb = wo * p.SW;
        a_off[j] = (uint32_t((n * p.H + hb) * p.W + wb) * uint32_t(p.C) + kc) * 2u;
        const int hi0 = hb - p.PT, wi0 = wb - p.PL;
        uint32_t wbits = 0;
        for (int kw = 0; kw < p.KW; ++kw) wbits |= uint32_t((unsigned)(wi0 + kw) < (unsigned)p.W) << kw;
        uint32_t msk = 0;
        for (int kh = 0; kh < p.KH; ++kh)
          if ((unsigned)(hi0 + kh) < (unsigned)p.H) msk |= wbits << (kh * p.KW);
        a_msk[j] = ok ? msk : 0u;
      }
    }
#pragma unroll
    for (int j = 0; j < G::BPW; ++j) {
      const int n = n0 + b_piece(j) * G::RPD + prow;
      b_off[j] = n < N ? (uint32_t(n) * uint32_t(p.ldb) + kc_of(b_piece(j))) * 2u : kOOB;
    }
    w_k = 0;
    w_ci = w_kh = w_kw = w_tap = 0;
  };

  // DMA of the producer's next k-tile into ring slot `rs`; then advance
  auto issue = [&](int rs) {
    const uint32_t a_soff = IM2COL ? uint32_t((w_kh * p.W + w_kw) * p.C + w_ci) * 2u : uint32_t(w_k) * 2u;
    const uint32_t b_soff = uint32_t(w_k) * 2u;
    char* const sa = smem + rs * G::A_ST * 2;
    char* const sb = smem + (S * G::A_ST + rs * G::B_ST) * 2;
    if (DUAL && w_k >= p.K1) {
      const uint32_t soff2 = uint32_t(w_k - p.K1) * 2u;
#pragma unroll
      for (int j = 0; j < G::APW; ++j) {
        if (!G::A_EVEN && a_piece(j) >= G::NAP) continue;
        const uint32_t v = a_off2[DUAL ? j : 0];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA2, (lds_ptr_t)(sa + a_piece(j) * 1024), 16, v, soff2, 0, 0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < G::APW; ++j) {
        if (!G::A_EVEN && a_piece(j) >= G::NAP) continue;
        uint32_t v = a_off[j];
        if (IM2COL) v = ((a_msk[j] >> w_tap) & 1u) ? v : kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_ptr_t)(sa + a_piece(j) * 1024), 16, v, a_soff, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < G::BPW; ++j) {
      if (!G::B_EVEN && b_piece(j) >= G::NBP) continue;
      const uint32_t v = b_off[j];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_ptr_t)(sb + b_piece(j) * 1024), 16, v, b_soff, 0, 0);
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
    if (++p_k == nk) {                             // the next DMA belongs to the producer's next tile
      p_k = 0;
      if (++p_i < mine) set_producer_tile(p_i);
    }
  };

  // ---- consumer fragments (16x16x32, 128-B rows, r & 7 swizzle)
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
  auto compute = [&](int rs) {
    const char* sa = smem + rs * G::A_ST * 2;
    const char* sb = smem + (S * G::A_ST + rs * G::B_ST) * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[G::TM], bfr[G::TN];
#pragma unroll
      for (int i = 0; i < G::TM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sa + (kk ? ra1 : ra0) + i * 16 * KT * 2);
#pragma unroll
      for (int j = 0; j < G::TN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sb + (kk ? rb1 : rb0) + j * 16 * KT * 2);
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // epilogue of the consumer's tile `i`: the accumulators through the separate
  // fp32 staging area (the ring keeps filling), then bias / residual / act rows
  float4 bias0, bias1;
  int c_m0, c_n0;
  tile_mn<BM, BN>(slot, nbm, nbn, c_m0, c_n0);
  cgemm_impl::prefetch_bias<BM, BN, G::NT>(p, c_n0, tid, bias0, bias1);
  using RP = uint4[Epi<BM, BN, G::NT>::PRE > 0 ? Epi<BM, BN, G::NT>::PRE : 1];
  RP rdummy;
  auto epilogue = [&]() {
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int j = 0; j < G::TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          Cs[(wm * G::WM + i * 16 + fq * 4 + r) * P::CS_LD + wn * G::WN + j * 16 + fr] = acc[i][j][r];
          acc[i][j][r] = 0.f;
        }
    // (an LDS barrier, not __syncthreads(): its fence would drain the next
    // tile's DMAs in flight with vmcnt(0))
    lds_barrier();
    switch (p.act) {
      case kActRelu: epilogue_rows<BM, BN, G::NT, P::CS_LD, kActRelu, false>(p, Cs, c_m0, c_n0, tid, rdummy, bias0, bias1); break;
      case kActGeluTanh: epilogue_rows<BM, BN, G::NT, P::CS_LD, kActGeluTanh, false>(p, Cs, c_m0, c_n0, tid, rdummy, bias0, bias1); break;
      case kActGeluErf: epilogue_rows<BM, BN, G::NT, P::CS_LD, kActGeluErf, false>(p, Cs, c_m0, c_n0, tid, rdummy, bias0, bias1); break;
      case kActTanh: epilogue_rows<BM, BN, G::NT, P::CS_LD, kActTanh, false>(p, Cs, c_m0, c_n0, tid, rdummy, bias0, bias1); break;
      default: epilogue_rows<BM, BN, G::NT, P::CS_LD, 0, false>(p, Cs, c_m0, c_n0, tid, rdummy, bias0, bias1); break;
    }
  };

  // ---- prologue: S - 1 k-tiles of the flattened sequence in flight
  set_producer_tile(0);
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < T) issue(s);

  int c_k = 0, c_i = 0;
  for (int g = 0; g < T; ++g) {
    const int rs = g % S;
    // k-tile g landed once only the younger DMAs remain (stores never counted)
    const int younger = min(S - 2, T - 1 - g);
    if (younger == S - 2) {
      wait_vmcnt<(S - 2) * G::PPW>();
    } else if (S >= 4 && younger == 2) {
      wait_vmcnt<(S >= 4 ? 2 : 0) * G::PPW>();
    } else if (S >= 3 && younger == 1) {
      wait_vmcnt<(S >= 3 ? 1 : 0) * G::PPW>();
    } else {
      wait_vmcnt<0>();
    }
    lds_barrier();
    if (g == 0) trace_stamp(p, 1);
    if (g + S - 1 < T) issue((g + S - 1) % S);
    compute(rs);
    if (++c_k == nk) {
      c_k = 0;
      epilogue();
      if (++c_i < mine) {
        tile_mn<BM, BN>(slot + c_i * int(gridDim.x), nbm, nbn, c_m0, c_n0);
        cgemm_impl::prefetch_bias<BM, BN, G::NT>(p, c_n0, tid, bias0, bias1);
      }
    }
  }
  trace_stamp(p, 3);
}

template <int BM, int BN, int WGM, int WGN, int S, int AM>
hipError_t launch_pg(const IGemmArgs& a, hipStream_t s) {
  using P = PG<BM, BN, WGM, WGN, S>;
  if (a.splits > 1 || a.st_out != nullptr || a.a_st != nullptr || a.r_st != nullptr)
    return hipErrorInvalidValue;   // whole K loops only, no deferred LayerNorm
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (tiles == 0) return hipSuccess;
  const void* fn = reinterpret_cast<const void*>(&pgemm_kernel<BM, BN, WGM, WGN, S, AM>);
  hipError_t e = ensure_dyn_lds(fn, P::LDS);
  if (e != hipSuccess) return e;
  // one resident round of workgroups (per device and kernel, queried once)
  static int per_cu[16] = {0};
  static int cus[16] = {0};
  int dev = 0;
  e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const int di = dev & 15;
  if (per_cu[di] == 0) {
    int n = 0, c = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 64 * WGM * WGN, P::LDS);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    cus[di] = c > 0 ? c : 256;
    per_cu[di] = n > 0 ? n : 1;
  }
  const int grid = tiles < per_cu[di] * cus[di] ? tiles : per_cu[di] * cus[di];
  hipLaunchKernelGGL((pgemm_kernel<BM, BN, WGM, WGN, S, AM>), dim3(grid), dim3(64 * WGM * WGN), P::LDS, s, a);
  return hipGetLastError();
}

template <int AM>
hipError_t launch_mode_pg(const IGemmArgs& a, int idx, hipStream_t s) {
  switch (idx) {
    case 0: return launch_pg<64, 64, 2, 2, 3, AM>(a, s);     // 48 KB ring + 17 KB staging, waves 32x32
    case 1: return launch_pg<64, 64, 2, 2, 4, AM>(a, s);     // 64 + 17 KB
    case 2: return launch_pg<64, 128, 2, 2, 3, AM>(a, s);    // 72 + 33 KB, waves 32x64
    case 3: return launch_pg<128, 64, 2, 2, 3, AM>(a, s);    // 72 + 34 KB, waves 64x32
    case 4: return launch_pg<128, 128, 2, 2, 2, AM>(a, s);   // 64 + 66 KB, waves 64x64
    case 5: return launch_pg<128, 128, 2, 4, 2, AM>(a, s);   // 64 + 66 KB, 8 waves of 64x32
    case 6: return launch_pg<64, 256, 1, 4, 2, AM>(a, s);    // 80 + 66 KB, waves 64x64
    case 7: return launch_pg<64, 64, 2, 2, 2, AM>(a, s);     // 32 + 17 KB
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t pgemm_launch(const IGemmArgs& a, int a_mode, int idx, hipStream_t s) {
  switch (a_mode) {
    case kAIm2col: return launch_mode_pg<1>(a, idx, s);
    case kADual: return launch_mode_pg<2>(a, idx, s);
    case kADense: return launch_mode_pg<0>(a, idx, s);
    default: return hipErrorInvalidValue;              // the stem layout stays on cgemm
  }
}

}  // namespace tfsk
