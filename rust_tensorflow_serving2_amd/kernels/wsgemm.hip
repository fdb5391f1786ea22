// Weight-stationary GEMM for MI355X (gfx950): C[M][N] = act(A[M][K] B[N][K]^T
// + bias + residual), bf16 operands, fp32 MFMA accumulate.  The 1x1 convs of
// ResNet-50 (dense NHWC rows, kADense) and the K <= 1024 projections of BERT.
//
// Why: the pipelined cgemm kernel streams BOTH operands through an LDS-DMA
// ring with a workgroup barrier per 64-deep k-tile; for these shapes (K 64 ..
// 2048, N 64 .. 2048, M up to 10^5 rows) the weight slice a workgroup needs is
// small (BN x K x 2 B <= 128 KB), so here it is loaded into LDS ONCE and
// stays: the workgroup then walks a contiguous range of rows (persistent over
// M), each wave on its own 16 x TM-row groups, streaming its A rows straight
// from memory into the MFMA A registers (two k-tiles ahead, compiler-counted
// vmcnt waits).  No LDS ring, no barrier after the prologue, no LDS-DMA for
// the activations; the waves never wait for each other.
//
//   * A fragments are loaded in the channel permutation of halo.hip's
//     register operands (lane group fq takes 16 channels of a k-tile, kk the
//     8-channel half: two adjacent 16-B loads per lane) and the B fragment
//     reads from LDS apply the same permutation;
//   * B lives in LDS as k-tiles of BN rows x 128 B, 16-B chunks XOR-swizzled
//     by row & 7 (the conflict-free image cgemm uses);
//   * the epilogue stages each 16-row slice through a per-wave fp32 slab and
//     writes 16-B bf16 row chunks (bias + residual + activation).
#include "gemm_common.h"
#include "cgemm.h"

namespace tfsk {
namespace {

using namespace gemm;

constexpr int kWsNT = 256;

template <int BN, int TM>
struct WS {
  static constexpr int TN = BN / 16;
  static constexpr int ROWS = 16 * TM;               // rows per wave step
  static constexpr int SLD = BN + 4;                 // slab row stride (floats)
  static constexpr int SLAB_B = 16 * SLD * 4;        // one wave's slab
  static constexpr int EPI_IT = (16 * (BN / 8) + 63) / 64;   // 16-B chunks per lane per 16-row slice
  static_assert(BN % 16 == 0 && BN >= 16, "BN");
  static int lds(int K) { return BN * K * 2 + 4 * SLAB_B; }
};

template <int BN, int TM>
__global__ __launch_bounds__(kWsNT) void wsgemm_kernel(IGemmArgs p, int rows_per_wg) {
  using G = WS<BN, TM>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  const int M = p.M, N = p.N, K = p.K;
  const int nkt = K / KT;
  const int nbn = (N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int bn = wg % nbn, mg = wg / nbn;
  const int n0 = bn * BN;
  const int m_begin = mg * rows_per_wg, m_end = min(M, m_begin + rows_per_wg);
  if (m_begin >= m_end) return;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int prow = lane >> 3;
  const uint32_t kc = uint32_t(((lane & 7) ^ prow) * 8);

  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.a), 0, int(p.a_bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.b), 0, int(p.b_bytes), 0x00020000);

  // ---- prologue: this workgroup's weight slice [BN][K] -> LDS (k-tile kt at
  // kt * BN * 128 B; 8-row pieces of 1 KB spread over the 4 waves)
  {
    const int pieces = nkt * (BN / 8);
    for (int q = wid; q < pieces; q += 4) {
      const int kt = q / (BN / 8), pc = q - kt * (BN / 8);
      const int n = n0 + pc * 8 + prow;
      const uint32_t v = n < N ? (uint32_t(n) * uint32_t(p.ldb) + uint32_t(kt * KT) + kc) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_ptr_t)(smem + (kt * BN + pc * 8) * KT * 2), 16, v, 0, 0, 0);
    }
  }
  dma_fence();                          // the A loads below stay behind the weight DMAs (gemm_common.h)

  // ---- this wave's row groups: rows [m, m + ROWS) for m = m_begin + (wid + 4 j) * ROWS
  const int ngroups = (m_end - m_begin + G::ROWS - 1) / G::ROWS;
  const int my_groups = ngroups > wid ? (ngroups - wid + 3) / 4 : 0;
  const int steps = my_groups * nkt;                  // (group, k-tile) steps of this wave

  // A fragment loads of step s -> registers (kk halves of lane group fq's 16 channels)
  typedef bf16x8 AFrag[TM][2];
  const int lda2 = p.lda * 2;
  auto load_a = [&](int s, AFrag& dst) {
    const int gi = s / nkt, kt = s - gi * nkt;
    const int mrow = m_begin + (wid + 4 * gi) * G::ROWS + fr;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = mrow + i * 16;
      const uint32_t v = m < m_end ? uint32_t(m) * uint32_t(lda2) + uint32_t(kt * KT * 2 + fq * 32) : kOOB;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        dst[i][kk] = __builtin_bit_cast(bf16x8, ordered_load16(rsA, v + kk * 16u, 0));
    }
  };

  AFrag aq[3];
  if (steps > 0) load_a(0, aq[0]);
  if (steps > 1) load_a(1, aq[1]);
  // the weight DMAs were issued first: once only this wave's A loads remain
  // in flight its share of the slice has landed; the barrier makes it every wave's
  dma_fence();
  if (steps > 1) wait_vmcnt<4 * TM < 63 ? 4 * TM : 63>();
  else if (steps == 1) wait_vmcnt<2 * TM < 63 ? 2 * TM : 63>();
  else wait_vmcnt<0>();
  __syncthreads();

  float* slab = reinterpret_cast<float*>(smem + BN * K * 2) + wid * 16 * G::SLD;

  f32x4 acc[TM][G::TN];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < G::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto compute = [&](int kt, const AFrag& a) {
    const char* sb = smem + kt * BN * KT * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 bfr[G::TN];
#pragma unroll
      for (int j = 0; j < G::TN; ++j) {
        const int row = j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(sb + (row * KT + (((fq * 2 + kk) ^ (row & 7)) * 8)) * 2);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][kk], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  auto epilogue = [&](int gi) {
    const int mbase = m_begin + (wid + 4 * gi) * G::ROWS;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < G::TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[(fq * 4 + r) * G::SLD + j * 16 + fr] = acc[i][j][r];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int it = 0; it < G::EPI_IT; ++it) {
        const int item = lane + 64 * it;
        if (item < 16 * (BN / 8)) {
          const int rl = item / (BN / 8), c8 = item % (BN / 8);
          const int m = mbase + i * 16 + rl, n = n0 + c8 * 8;
          if (m < m_end && n < N) {
            float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (p.bias) {
              const float4 b0 = *reinterpret_cast<const float4*>(p.bias + n);
              const float4 b1 = *reinterpret_cast<const float4*>(p.bias + n + 4);
              bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
              bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
            }
            const uint4 rr = p.residual ? *reinterpret_cast<const uint4*>(p.residual + size_t(m) * p.ldr + n)
                                        : make_uint4(0, 0, 0, 0);
            switch (p.act) {
              case kActRelu: epi_chunk<kActRelu>(p, slab + rl * G::SLD + c8 * 8, m, n, bv, rr); break;
              case kActGeluTanh: epi_chunk<kActGeluTanh>(p, slab + rl * G::SLD + c8 * 8, m, n, bv, rr); break;
              case kActGeluErf: epi_chunk<kActGeluErf>(p, slab + rl * G::SLD + c8 * 8, m, n, bv, rr); break;
              case kActTanh: epi_chunk<kActTanh>(p, slab + rl * G::SLD + c8 * 8, m, n, bv, rr); break;
              default: epi_chunk<kActNone>(p, slab + rl * G::SLD + c8 * 8, m, n, bv, rr); break;
            }
          }
        }
      }
      __builtin_amdgcn_wave_barrier();   // slab reads done before the next slice overwrites it
    }
  };

  // ---- main loop: steps s = (group, k-tile), A two steps ahead in 3 register
  // slots (unrolled by 3 so the slots are static)
  zero();
  for (int s0 = 0; s0 < steps; s0 += 3) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int s = s0 + u;
      if (s < steps) {
        if (s + 2 < steps) load_a(s + 2, aq[(u + 2) % 3]);
        const int gi = s / nkt, kt = s - gi * nkt;
        compute(kt, aq[u]);
        if (kt == nkt - 1) {
          epilogue(gi);
          zero();
        }
      }
    }
  }
}

template <int BN, int TM>
hipError_t launch_ws(const IGemmArgs& a, hipStream_t s) {
  using G = WS<BN, TM>;
  const int lds = G::lds(a.K);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int nbn = (a.N + BN - 1) / BN;
  // rows per workgroup: ~512 workgroups (2 per CU) in all, whole 4-wave
  // rounds of row groups each
  const int unit = 4 * G::ROWS;
  long groups = (512 + nbn - 1) / nbn;
  if (groups < 1) groups = 1;
  long rows = (a.M + groups - 1) / groups;
  rows = (rows + unit - 1) / unit * unit;
  const long mgs = (a.M + rows - 1) / rows;
  const long tiles = mgs * nbn;
  if (tiles <= 0) return hipSuccess;
  if (tiles >= (1L << 31)) return hipErrorInvalidValue;
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&wsgemm_kernel<BN, TM>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((wsgemm_kernel<BN, TM>), dim3(unsigned(tiles)), dim3(kWsNT), lds, s, a, int(rows));
  return hipGetLastError();
}

constexpr int kWBN[kNumWsConfigs] = {64, 128, 64, 128, 256, 32, 96};
constexpr int kWTM[kNumWsConfigs] = {2, 2, 4, 1, 1, 4, 2};

}  // namespace

bool ws_supported(const IGemmArgs& a, int cfg) {
  const int c = cfg - kWsCfgBase;
  if (c < 0 || c >= kNumWsConfigs) return false;
  const int bn = kWBN[c];
  return a.K > 0 && a.K % KT == 0 && a.lda % 8 == 0 && a.lda >= a.K && a.ldb % 8 == 0 && a.ldb >= a.K &&
         a.N % 8 == 0 && a.ldc % 8 == 0 && (!a.residual || a.ldr % 8 == 0) && a.splits <= 1 && !a.out2 &&
         a.alpha == 1.f && bn * a.K * 2 + 4 * 16 * (bn + 4) * 4 <= 160 * 1024 && a.M < (1 << 30) &&
         a.a_bytes < 0x7ffffff0LL && a.b_bytes < 0x7ffffff0LL;
}

int ws_config_bn(int cfg) { return kWBN[cfg - kWsCfgBase]; }
int ws_config_bm(int cfg) { return 64 * kWTM[cfg - kWsCfgBase]; }

hipError_t ws_launch(const IGemmArgs& a, int cfg, hipStream_t s) {
  if (!ws_supported(a, cfg)) return hipErrorInvalidValue;
  switch (cfg - kWsCfgBase) {
    case 0: return launch_ws<64, 2>(a, s);
    case 1: return launch_ws<128, 2>(a, s);
    case 2: return launch_ws<64, 4>(a, s);
    case 3: return launch_ws<128, 1>(a, s);
    case 4: return launch_ws<256, 1>(a, s);
    case 5: return launch_ws<32, 4>(a, s);
    case 6: return launch_ws<96, 2>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tfsk
