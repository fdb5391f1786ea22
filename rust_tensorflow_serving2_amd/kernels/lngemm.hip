// GEMM + residual + LayerNorm in one launch for MI355X (gfx950):
//   y[M][N] = LN(x[M][K] w[N][K]^T + bias + r[M][N]) * gamma + beta
// (w passed fragment-major: see w_off below)
// bf16 operands / output, fp32 accumulate and statistics.
//
// Why: BERT's attention-output projection (M = 128 x batch, N = K = 768) is
// followed by a residual add and a LayerNorm over the 768 columns.  As two
// launches it costs 12-14 us (64 x 64 cgemm tiles) + 5.4-7.2 us
// (layernorm_fit_kernel) per layer at b32 (profiles/round6/r6d/
// replay_bert_b32.txt); the LayerNorm re-reads the GEMM output and the
// residual from HBM / Infinity Cache and pays a launch boundary.  Here one
// workgroup owns BM whole rows, so the row statistics never leave the CU:
//
//   * 8 waves side by side along N, wave w owns columns [w N/8, (w+1) N/8)
//     (TN 16-wide MFMA tiles) for all BM rows: v_mfma_f32_16x16x32_bf16,
//     BM/16 x TN accumulators;
//   * the weights are read ONCE per workgroup and by one wave each (no wave
//     shares a column), so they skip LDS: every wave streams its own [N/8][K]
//     slice straight into VGPRs (16-B buffer loads, a 5-slot register ring,
//     loads issued 3 K-steps ahead and pinned above the MFMAs, one counted
//     vmcnt per K-step);
//   * x (BM x K) and the residual tile (BM x N, one contiguous range: whole
//     rows) go to LDS by buffer_load ... lds in the prologue, x as k-tile
//     images of 128-B rows with 16-B chunks XOR-swizzled by (row & 7) (the
//     conflict-free ds_read_b128 fragment reads of cgemm);
//   * epilogue: v = acc + bias + r in registers; two-pass mean / variance
//     (a 16-lane xor reduction, then the 8 waves' partials through LDS);
//     the normalized bf16 rows are staged over the residual tile and leave
//     as 16-B row stores.
// Cost model (BERT-base b32, BM = 32: 128 workgroups): each streams the 1.2 MB
// weight matrix from L2 (16 per XCD: ~19 MB per XCD of L2 reads), 37.7 MFLOP
// per workgroup -- about 5-6 us against the 17-21 us of the two launches.
#include <algorithm>

#include "common.h"
#include "gemm_common.h"
#include "launch.h"

namespace tfsk {

namespace {

using gemm::kOOB;

template <int BM, int TN>
struct LG {
  static constexpr int NW = 8, NT = 512;
  static constexpr int WN = TN * 16, N = NW * WN;   // columns per wave / per row
  static constexpr int MT = BM / 16;                // m-tiles
  static constexpr int SLOTS = 5, AHEAD = 3;        // register ring of K-steps (32 deep); loads AHEAD steps out
  static constexpr int R_B = BM * N * 2;            // residual / output staging tile
  static constexpr int ST_B = 2 * NW * BM * 4;      // per-wave row partials (sum, then squares)
  static constexpr int MV_B = 2 * BM * 4;           // mean, rstd per row
  static_assert(BM % 16 == 0 && BM >= 16 && BM <= 64, "BM");
  static_assert(R_B % 1024 == 0, "residual tile in whole 1-KB DMA pieces");
};

template <int BM, int TN>
__global__ __launch_bounds__(512, 1) void lngemm_kernel(LnGemmArgs p) {
  using G = LG<BM, TN>;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  char* const smem = reinterpret_cast<char*>(smem_raw);
  typedef __attribute__((address_space(3))) void* lds_ptr_t;

  const int K = p.K, M = p.M;
  const int A_B = BM * K * 2;                       // x tile bytes
  char* const As = smem;                            // [K/64][BM][64] swizzled
  char* const Rs = smem + A_B;                      // [BM][N] bf16 (residual, then the output)
  float* const St = reinterpret_cast<float*>(Rs + G::R_B);     // [2][NW][BM]
  float* const Mv = St + 2 * G::NW * BM;                       // [2][BM]

  const int m0 = blockIdx.x * BM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  const __amdgpu_buffer_rsrc_t rsX =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.x), 0, int(long(M) * p.ldx * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.w), 0, int(long(G::N) * K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsR = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(p.r), 0, p.r ? int(long(M) * G::N * 2) : 0, 0x00020000);

  // ---- weights: this wave's columns n = wid * WN + j * 16 + fr, k chunk fq
  const int nks = K / 32;
  // fragment-major weights (host pre-shuffle, graph/fused.py ln_weight_frags):
  // the B fragment of (n-tile nt, K-step t) is one contiguous KB, lane l at
  // ((nt * nks + t) * 64 + l) * 16 -- every load instruction reads 8 whole
  // 128-B lines instead of 16 half lines of 16 rows (the [N][K] layout ran
  // 42-46 us per workgroup, profiles/round6/r6h-r6i)
  uint32_t w_off[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) w_off[j] = (uint32_t((wid * TN + j) * nks) * 64u + lane) * 16u;
  // register ring of SLOTS K-steps: at step t the loads of step t + AHEAD go
  // into the slot step t - 2 used (its MFMAs issued two steps back), then the
  // wave waits for step t's own loads (vmcnt = the AHEAD younger steps)
  u32x4 bq[G::SLOTS][TN];
  auto load_b = [&](int slot, int t) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bq[slot][j] = __builtin_amdgcn_raw_buffer_load_b128(rsW, w_off[j], min(t, nks - 1) * 1024, 0);
  };
#pragma unroll
  for (int d = 0; d < G::AHEAD; ++d) load_b(d, d);

  // ---- x k-tile images and the residual tile by LDS-DMA (issued after the
  // first weight loads, so both are in flight together; one vmcnt(0) below)
  {
    const int pieces = (K / 64) * (BM / 8);
    for (int pc = wid; pc < pieces; pc += G::NW) {
      const int kt = pc / (BM / 8), rb = pc - kt * (BM / 8);
      const int row = rb * 8 + (lane >> 3);
      const int m = m0 + row;
      const uint32_t src = m < M ? (uint32_t(m) * uint32_t(p.ldx) + kt * 64 + (((lane & 7) ^ (row & 7)) * 8)) * 2u
                                 : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsX, (lds_ptr_t)(As + pc * 1024), 16, src, 0, 0, 0);
    }
    if (p.r != nullptr) {
      const uint32_t base = uint32_t(m0) * uint32_t(G::N) * 2u;
      for (int pc = wid; pc < G::R_B / 1024; pc += G::NW)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsR, (lds_ptr_t)(Rs + pc * 1024), 16,
                                                 base + uint32_t(pc * 1024 + lane * 16), 0, 0, 0);
    }
  }
  gemm::wait_vmcnt<0>();
  __syncthreads();

  // ---- main loop: K-steps of 32; A fragments from LDS, B from the register ring
  f32x4 acc[G::MT][TN];
#pragma unroll
  for (int i = 0; i < G::MT; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint32_t ra = uint32_t(fr * 128);
  for (int t0 = 0; t0 < nks; t0 += G::SLOTS) {
#pragma unroll
    for (int d = 0; d < G::SLOTS; ++d) {
      const int t = t0 + d;
      // unconditional, clamped at the tail: a branch around the loads made
      // hipcc wait vmcnt(0) at every loop head (one K-step in flight, 38 us
      // per workgroup, profiles/round6/r6g)
      __builtin_amdgcn_sched_barrier(0);
      load_b((d + G::AHEAD) % G::SLOTS, t + G::AHEAD);
      __builtin_amdgcn_sched_barrier(0);
      gemm::wait_vmcnt<G::AHEAD * TN>();
      if (t < nks) {
        const int kt = t >> 1, ch = (t & 1) * 4 + fq;
        bf16x8 a[G::MT];
#pragma unroll
        for (int i = 0; i < G::MT; ++i) {
          const int row = i * 16 + fr;
          a[i] = *reinterpret_cast<const bf16x8*>(As + (kt * BM + i * 16) * 128 + ra + ((ch ^ (row & 7)) << 4));
        }
#pragma unroll
        for (int i = 0; i < G::MT; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], __builtin_bit_cast(bf16x8, bq[d][j]),
                                                                acc[i][j], 0, 0, 0);
      }
    }
  }
  gemm::wait_vmcnt<0>();

  // ---- epilogue: v = acc + bias + residual; row (i, r) = i * 16 + fq * 4 + r
  const uint16_t* Rh = reinterpret_cast<const uint16_t*>(Rs);
  float bj[TN], gj[TN], ej[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wid * G::WN + j * 16 + fr;
    bj[j] = p.bias ? p.bias[col] : 0.f;
    gj[j] = p.gamma[col];
    ej[j] = p.beta[col];
  }
  const bool has_r = p.r != nullptr;
#pragma unroll
  for (int i = 0; i < G::MT; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + fq * 4 + r, col = wid * G::WN + j * 16 + fr;
        const float rv = has_r ? bf16_to_f32(Rh[row * G::N + col]) : 0.f;
        acc[i][j][r] += bj[j] + rv;
      }
  // row partial of this wave -> St[pass][wid][row]; then thread row < BM folds the 8 waves
  auto reduce_rows = [&](int pass, const float (&part)[G::MT][4]) {
#pragma unroll
    for (int i = 0; i < G::MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = part[i][r];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        if (fr == 0) St[(pass * G::NW + wid) * BM + i * 16 + fq * 4 + r] = s;
      }
  };
  float part[G::MT][4];
#pragma unroll
  for (int i = 0; i < G::MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) s += acc[i][j][r];
      part[i][r] = s;
    }
  reduce_rows(0, part);
  __syncthreads();                       // (also: every residual read above is done)
  const float inv_n = 1.f / float(G::N);
  if (tid < BM) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < G::NW; ++w) s += St[w * BM + tid];
    Mv[tid] = s * inv_n;
  }
  __syncthreads();
  float mean[G::MT][4];
#pragma unroll
  for (int i = 0; i < G::MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mean[i][r] = Mv[i * 16 + fq * 4 + r];
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float dv = acc[i][j][r] - mean[i][r];
        s += dv * dv;
      }
      part[i][r] = s;
    }
  reduce_rows(1, part);
  __syncthreads();
  if (tid < BM) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < G::NW; ++w) s += St[(G::NW + w) * BM + tid];
    Mv[BM + tid] = rsqrtf(s * inv_n + p.eps);
  }
  __syncthreads();
  uint16_t* Ys = reinterpret_cast<uint16_t*>(Rs);
#pragma unroll
  for (int i = 0; i < G::MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = i * 16 + fq * 4 + r;
      const float rs = Mv[BM + row];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float y = (acc[i][j][r] - mean[i][r]) * rs * gj[j] + ej[j];
        Ys[row * G::N + wid * G::WN + j * 16 + fr] = __builtin_bit_cast(uint16_t, static_cast<__bf16>(y));
      }
    }
  __syncthreads();
  constexpr int CPR = G::N / 8;
#pragma unroll 2
  for (int c = tid; c < BM * CPR; c += G::NT) {
    const int row = c / CPR, ch = c - row * CPR;
    const int m = m0 + row;
    if (m < M)
      *reinterpret_cast<uint4*>(p.y + size_t(m) * G::N + ch * 8) =
          *reinterpret_cast<const uint4*>(Ys + row * G::N + ch * 8);
  }
}

template <int BM, int TN>
hipError_t launch_lg(const LnGemmArgs& a, hipStream_t s) {
  using G = LG<BM, TN>;
  const int lds = BM * a.K * 2 + G::R_B + G::ST_B + G::MV_B;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&lngemm_kernel<BM, TN>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((lngemm_kernel<BM, TN>), dim3((a.M + BM - 1) / BM), dim3(G::NT), lds, s, a);
  return hipGetLastError();
}

template <int BM>
hipError_t launch_lg_n(const LnGemmArgs& a, hipStream_t s) {
  switch (a.N) {
    case 512: return launch_lg<BM, 4>(a, s);
    case 768: return launch_lg<BM, 6>(a, s);
    case 1024: return launch_lg<BM, 8>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool lngemm_supported(int M, int N, int K, int bm) {
  if (M <= 0 || K <= 0 || K % 128 || !(N == 512 || N == 768 || N == 1024)) return false;
  if (!(bm == 16 || bm == 32 || bm == 64)) return false;
  const int lds = bm * K * 2 + bm * N * 2 + 2 * 8 * bm * 4 + 2 * bm * 4;
  return lds <= 160 * 1024 && long(M) * K * 2 < 0x7fffffffL && long(N) * K * 2 < 0x7fffffffL &&
         long(M) * N * 2 < 0x7fffffffL;
}

hipError_t lngemm_launch(const LnGemmArgs& a, int bm, hipStream_t s) {
  if (!lngemm_supported(a.M, a.N, a.K, bm) || a.ldx < a.K || a.ldx % 8)
    return hipErrorInvalidValue;
  switch (bm) {
    case 16: return launch_lg_n<16>(a, s);
    case 32: return launch_lg_n<32>(a, s);
    case 64: return launch_lg_n<64>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tfsk
