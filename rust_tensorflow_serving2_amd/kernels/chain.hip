// Two chained 1x1 convs (plain GEMMs on NHWC rows) in ONE kernel:
//
//   Y1 = act1(X  W1^T + b1 + R)       [M][N1]   (a bottleneck's expand conv + shortcut)
//   Y2 = act2(Y1 W2^T + b2)           [M][N2]   (the NEXT bottleneck's reduce conv)
//
// In ResNet-50 v1.5 the reduce 1x1 of block i+1 reads exactly the rows the
// expand 1x1 of block i has just written: as two launches the reduce re-reads
// the whole expand output (stage 1 at b32: 51 MB) and pays a kernel boundary.
// Here a workgroup owns 64 full rows of Y1 (all N1 columns), keeps them in LDS
// as bf16 (the A operand of the second GEMM, in the swizzled layout the MFMA
// fragment reads expect) and streams W2 through a small LDS-DMA ring, so Y1 is
// written once and never read back.  Stage-1/2 shapes: K1 in {64, 128},
// N1 in {256, 512}, N2 in {64, 128, 256}.
//
//   * phase 1: X tile [64][K1] and all of W1 [N1][K1] land in LDS by direct
//     DMA (buffer_load ... lds, 16-B chunks XOR-swizzled by row & 7), the
//     residual chunks and biases this lane will need are loaded into registers
//     meanwhile; 4 waves each own 64 rows x N1/4 columns of v_mfma_f32_16x16x32_bf16
//     accumulators;
//   * phase 2: each wave stages its accumulators 16 rows x 64 columns at a time
//     through a private fp32 LDS slab (no workgroup barrier), applies bias +
//     residual + act, stores Y1 with 16-B row chunks and writes the same bf16
//     chunk into the LDS chain tile;
//   * phase 3: Y1(LDS) x W2(ring) on a 2 x 2 wave grid, then the Y2 epilogue
//     through the same per-wave slab.
// Y2 is computed from the bf16 Y1 values, exactly what the separate reduce
// conv would read.
#include "gemm_common.h"

namespace tfsk {
namespace {

using namespace gemm;

struct ChainArgs {
  const uint16_t* x;     // [M][K1] bf16
  const uint16_t* w1;    // [N1][ldw1] bf16
  const float* b1;       // [N1]
  const uint16_t* res;   // [M][N1] bf16 or nullptr
  uint16_t* y1;          // [M][N1] bf16
  const uint16_t* w2;    // [N2][ldw2] bf16
  const float* b2;       // [N2]
  uint16_t* y2;          // [M][N2] bf16
  int M, ldw1, ldw2;
  float lo1, lo2;        // activation floors: 0 (ReLU) or -inf (none)
};

constexpr int kBM = 64, kNT = 256, kStgLd = 68;   // fp32 slab row stride (floats): 16-B aligned rows

template <int K1, int N1, int N2>
struct CH {
  static constexpr int KT1 = K1 / KT, KT2 = N1 / KT;
  static constexpr int A_BYTES = KT1 * kBM * KT * 2;
  static constexpr int W1_BYTES = KT1 * N1 * KT * 2;
  static constexpr int P1 = A_BYTES + W1_BYTES;
  static constexpr int CHAIN = KT2 * kBM * KT * 2;             // Y1 tile, bf16
  static constexpr int STG = 4 * 16 * kStgLd * 4;              // one 16-row slab per wave
  static constexpr int S2 = N2 <= 128 ? 3 : 2;                 // W2 ring depth
  static constexpr int W2_SLOT = N2 * KT * 2;
  // the W2 ring and the per-wave epilogue slabs share one region (the ring is
  // idle during both epilogues): 80 KB for the stage-1 shapes = 2 workgroups per CU
  static constexpr int RING_OFF = CHAIN;
  static constexpr int P23 = CHAIN + (STG > S2 * W2_SLOT ? STG : S2 * W2_SLOT);
  static constexpr int LDS = P1 > P23 ? P1 : P23;
  static constexpr int WN1 = N1 / 4, TN1 = WN1 / 16, U1 = WN1 / 64;   // GEMM1: wave = 64 rows x WN1
  static constexpr int WN2 = N2 / 2, TN2 = WN2 / 16;                  // GEMM2: wave = 32 rows x WN2
  static constexpr int UW2 = WN2 < 64 ? WN2 : 64, U2 = WN2 / UW2;
  static constexpr int APW = KT1 * (kBM / 8) / 4, W1PW = KT1 * (N1 / 8) / 4, W2PW = N2 / 32;
  static_assert(K1 % KT == 0 && N1 % 256 == 0 && N2 % 64 == 0, "chain shape");
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert((S2 - 2) * W2PW < 64, "vmcnt range");
};

template <int K1, int N1, int N2>
__global__ __launch_bounds__(256, 1) void conv_chain_kernel(ChainArgs p) {
  using G = CH<K1, N1, N2>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int prow = lane >> 3;
  const uint32_t kc = uint32_t(((lane & 7) ^ prow) * 8);
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * kBM;
  const int M = p.M;

  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(p.x), 0, int(long(M) * K1 * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW1 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(p.w1), 0, int(long(N1) * p.ldw1 * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(p.w2), 0, int(long(N2) * p.ldw2 * 2), 0x00020000);

  // ---- phase 1 DMAs: piece q (8 rows x 128 B) of k-tile kt lands at LDS
  // rows [8q, 8q + 8) of that k-tile's image
#pragma unroll
  for (int j = 0; j < G::APW; ++j) {
    const int q = wid * G::APW + j;                 // over KT1 x 8 pieces
    const int kt = q / (kBM / 8), pc = q % (kBM / 8);
    const int m = m0 + pc * 8 + prow;
    const uint32_t v = m < M ? (uint32_t(m) * K1 + uint32_t(kt * KT) + kc) * 2u : kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsX, (lds_ptr_t)(smem + kt * kBM * KT * 2 + pc * 1024), 16, v, 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < G::W1PW; ++j) {
    const int q = wid * G::W1PW + j;                // over KT1 x N1/8 pieces
    const int kt = q / (N1 / 8), pc = q % (N1 / 8);
    const int n = pc * 8 + prow;
    const uint32_t v = (uint32_t(n) * uint32_t(p.ldw1) + uint32_t(kt * KT) + kc) * 2u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW1, (lds_ptr_t)(smem + G::A_BYTES + kt * N1 * KT * 2 + pc * 1024), 16,
                                             v, 0, 0, 0);
  }

  // ---- this lane's epilogue-1 operands, loaded while the DMAs fly: unit
  // (i, c) = rows [16i, 16i + 16) x wave columns [64c, 64c + 64); a lane owns
  // chunk column c8 = lane & 7 of rows (lane >> 3) and (lane >> 3) + 8
  const int c8 = lane & 7, rl = lane >> 3;
  float4 bias1[G::U1][2];
#pragma unroll
  for (int c = 0; c < G::U1; ++c) {
    const int n = wid * G::WN1 + c * 64 + c8 * 8;
    bias1[c][0] = *reinterpret_cast<const float4*>(p.b1 + n);
    bias1[c][1] = *reinterpret_cast<const float4*>(p.b1 + n + 4);
  }
  const __amdgpu_buffer_rsrc_t rsR = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(p.res), 0, p.res ? int(long(M) * N1 * 2) : 0, 0x00020000);
  u32x4 rr[4][G::U1][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int c = 0; c < G::U1; ++c)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int m = m0 + i * 16 + rl + 8 * k;
        const int n = wid * G::WN1 + c * 64 + c8 * 8;
        const uint32_t v = m < M ? (uint32_t(m) * N1 + uint32_t(n)) * 2u : kOOB;
        rr[i][c][k] = __builtin_amdgcn_raw_buffer_load_b128(rsR, v, 0, 0);
      }

  wait_vmcnt<0>();
  __syncthreads();

  // ---- GEMM1: 64 rows x this wave's WN1 columns
  f32x4 acc[4][G::TN1];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < G::TN1; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint32_t ro0 = uint32_t((fr * KT + ((fq ^ (fr & 7)) * 8)) * 2);
  const uint32_t ro1 = uint32_t((fr * KT + (((4 + fq) ^ (fr & 7)) * 8)) * 2);
#pragma unroll
  for (int kt = 0; kt < G::KT1; ++kt) {
    const char* sa = smem + kt * kBM * KT * 2;
    const char* sb = smem + G::A_BYTES + kt * N1 * KT * 2 + wid * G::WN1 * KT * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[G::TN1];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sa + (kk ? ro1 : ro0) + i * 16 * KT * 2);
#pragma unroll
      for (int j = 0; j < G::TN1; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sb + (kk ? ro1 : ro0) + j * 16 * KT * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < G::TN1; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();   // every wave is done with the phase-1 images

  auto issue_w2 = [&](int kt2, int slot) {
#pragma unroll
    for (int j = 0; j < G::W2PW; ++j) {
      const int pc = wid * G::W2PW + j;
      const int n = pc * 8 + prow;
      const uint32_t v = (uint32_t(n) * uint32_t(p.ldw2) + uint32_t(kt2 * KT) + kc) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW2, (lds_ptr_t)(smem + G::RING_OFF + slot * G::W2_SLOT + pc * 1024),
                                               16, v, 0, 0, 0);
    }
  };

  // ---- epilogue 1 through this wave's fp32 slab
  float* stg = reinterpret_cast<float*>(smem + G::CHAIN) + wid * 16 * kStgLd;
  char* chain = smem;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int c = 0; c < G::U1; ++c) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) stg[(fq * 4 + r) * kStgLd + jj * 16 + fr] = acc[i][c * 4 + jj][r];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int row = i * 16 + rl + 8 * k;
        const float* src = stg + (rl + 8 * k) * kStgLd + c8 * 8;
        const float4 lo = *reinterpret_cast<const float4*>(src);
        const float4 hi = *reinterpret_cast<const float4*>(src + 4);
        const float bv[8] = {bias1[c][0].x, bias1[c][0].y, bias1[c][0].z, bias1[c][0].w,
                             bias1[c][1].x, bias1[c][1].y, bias1[c][1].z, bias1[c][1].w};
        const float a[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        const u32x4 w = rr[i][c][k];
        const uint32_t rw[4] = {w.x, w.y, w.z, w.w};
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v0 = fmaxf(a[2 * e] + bv[2 * e] + __uint_as_float(rw[e] << 16), p.lo1);
          const float v1 = fmaxf(a[2 * e + 1] + bv[2 * e + 1] + __uint_as_float(rw[e] & 0xffff0000u), p.lo1);
          o[e] = pack_bf16x2(v0, v1);
        }
        const uint4 ov = make_uint4(o[0], o[1], o[2], o[3]);
        const int n = wid * G::WN1 + c * 64 + c8 * 8;
        const int m = m0 + row;
        if (m < M) *reinterpret_cast<uint4*>(p.y1 + size_t(m) * N1 + n) = ov;
        const int kt2 = n >> 6;
        *reinterpret_cast<uint4*>(chain + ((kt2 * kBM + row) * KT + ((c8 ^ (row & 7)) * 8)) * 2) = ov;
      }
      __builtin_amdgcn_wave_barrier();   // slab reads done before the next unit overwrites it
    }
  }

  // ---- GEMM2: Y1 (LDS) x W2 (ring), wave grid 2 x 2 of 32 x WN2
  const int wm2 = wid >> 1, wn2 = wid & 1;
  f32x4 acc2[2][G::TN2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < G::TN2; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint32_t ra0 = uint32_t(((wm2 * 32 + fr) * KT + ((fq ^ (fr & 7)) * 8)) * 2);
  const uint32_t ra1 = uint32_t(((wm2 * 32 + fr) * KT + (((4 + fq) ^ (fr & 7)) * 8)) * 2);
  const uint32_t rb0 = uint32_t(((wn2 * G::WN2 + fr) * KT + ((fq ^ (fr & 7)) * 8)) * 2);
  const uint32_t rb1 = uint32_t(((wn2 * G::WN2 + fr) * KT + (((4 + fq) ^ (fr & 7)) * 8)) * 2);
  constexpr int S = G::S2;
  // ---- epilogue-2 bias values of this lane's items, issued here so the
  // ring's first wait covers them (plain loads of p.b2 were reloaded next to
  // each store: one serial memory round trip per epilogue item, seen in the
  // gfx950 ISA, scripts/isa_audit.py); buffer loads are not rematerialised
  constexpr int CPR2 = G::UW2 / 8;                  // chunks per slab row (4 or 8)
  constexpr int IT2 = 16 * CPR2 / 64;               // items per lane (1 or 2)
  const __amdgpu_buffer_rsrc_t rsB2 =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.b2), 0, N2 * 4, 0x00020000);
  u32x4 b2v[G::U2][IT2][2];
#pragma unroll
  for (int c = 0; c < G::U2; ++c)
#pragma unroll
    for (int k = 0; k < IT2; ++k) {
      const int cc = (lane + 64 * k) % CPR2;
      const uint32_t n = uint32_t(wn2 * G::WN2 + c * G::UW2 + cc * 8);
      b2v[c][k][0] = __builtin_amdgcn_raw_buffer_load_b128(rsB2, n * 4u, 0, 0);
      b2v[c][k][1] = __builtin_amdgcn_raw_buffer_load_b128(rsB2, n * 4u + 16u, 0, 0);
    }
  // ---- W2 ring prologue, once every wave is done with its slab (same region)
  __syncthreads();
#pragma unroll
  for (int s = 0; s < G::S2 - 1; ++s)
    if (s < G::KT2) issue_w2(s, s);
  // the ring prologue landed and the Y1 stores are drained (a workgroup-scope
  // __syncthreads waits for LDS only, and stores may complete out of order
  // with the DMAs), every wave's chain-tile writes are visible: from here on
  // only ring DMAs are in flight, so the counted waits below see ring slots alone
  wait_vmcnt<0>();
  __syncthreads();
  for (int kt0 = 0; kt0 < G::KT2; kt0 += S) {
#pragma unroll
    for (int u = 0; u < S; ++u) {
      const int t = kt0 + u;
      if (t < G::KT2) {
        // slot t landed once only the younger slots remain in flight (and
        // every wave is done reading slot t - 1, which the issue below reuses)
        if (t + S - 2 < G::KT2) wait_vmcnt<(S - 2) * G::W2PW>();
        else wait_vmcnt<0>();
        lds_barrier();
        if (t + S - 1 < G::KT2) issue_w2(t + S - 1, (u + S - 1) % S);
        const char* sa = chain + t * kBM * KT * 2;
        const char* sb = smem + G::RING_OFF + u * G::W2_SLOT;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          bf16x8 af[2], bfr[G::TN2];
#pragma unroll
          for (int i = 0; i < 2; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sa + (kk ? ra1 : ra0) + i * 16 * KT * 2);
#pragma unroll
          for (int j = 0; j < G::TN2; ++j)
            bfr[j] = *reinterpret_cast<const bf16x8*>(sb + (kk ? rb1 : rb0) + j * 16 * KT * 2);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < G::TN2; ++j)
              acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc2[i][j], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue 2 (its slabs overlay the ring: every wave is done reading it)
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rsY2 =
      __builtin_amdgcn_make_buffer_rsrc(p.y2, 0, int(long(M) * N2 * 2), 0x00020000);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int c = 0; c < G::U2; ++c) {
#pragma unroll
      for (int jj = 0; jj < G::UW2 / 16; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          stg[(fq * 4 + r) * kStgLd + jj * 16 + fr] = acc2[i][c * (G::UW2 / 16) + jj][r];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < IT2; ++k) {
        const int item = lane + 64 * k;
        const int rloc = item / CPR2, cc = item % CPR2;
        const float* src = stg + rloc * kStgLd + cc * 8;
        const float4 lo = *reinterpret_cast<const float4*>(src);
        const float4 hi = *reinterpret_cast<const float4*>(src + 4);
        const int n = wn2 * G::WN2 + c * G::UW2 + cc * 8;
        const u32x4 b0 = b2v[c][k][0], b1 = b2v[c][k][1];
        auto f = [](uint32_t u) { return __uint_as_float(u); };
        u32x4 ov;
        ov.x = pack_bf16x2(fmaxf(lo.x + f(b0.x), p.lo2), fmaxf(lo.y + f(b0.y), p.lo2));
        ov.y = pack_bf16x2(fmaxf(lo.z + f(b0.z), p.lo2), fmaxf(lo.w + f(b0.w), p.lo2));
        ov.z = pack_bf16x2(fmaxf(hi.x + f(b1.x), p.lo2), fmaxf(hi.y + f(b1.y), p.lo2));
        ov.w = pack_bf16x2(fmaxf(hi.z + f(b1.z), p.lo2), fmaxf(hi.w + f(b1.w), p.lo2));
        const int m = m0 + wm2 * 32 + i * 16 + rloc;
        // unconditional store: rows past M go to a dropped out-of-range offset
        __builtin_amdgcn_raw_buffer_store_b128(ov, rsY2, m < M ? (uint32_t(m) * N2 + uint32_t(n)) * 2u : kOOB, 0, 0);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

template <int K1, int N1, int N2>
hipError_t launch_chain(const ChainArgs& a, hipStream_t s) {
  using G = CH<K1, N1, N2>;
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&conv_chain_kernel<K1, N1, N2>), G::LDS);
  if (e != hipSuccess) return e;
  const int tiles = (a.M + kBM - 1) / kBM;
  hipLaunchKernelGGL((conv_chain_kernel<K1, N1, N2>), dim3(tiles), dim3(kNT), G::LDS, s, a);
  return hipGetLastError();
}

}  // namespace

bool conv_chain_supported(int K1, int N1, int N2) {
  return (K1 == 64 && N1 == 256 && (N2 == 64 || N2 == 128)) || (K1 == 128 && N1 == 512 && (N2 == 128 || N2 == 256));
}

hipError_t conv_chain_launch(const uint16_t* x, const uint16_t* w1, int ldw1, const float* b1, const uint16_t* res,
                             uint16_t* y1, const uint16_t* w2, int ldw2, const float* b2, uint16_t* y2, int M, int K1,
                             int N1, int N2, int act1, int act2, hipStream_t s) {
  if (M <= 0) return hipSuccess;
  if (!conv_chain_supported(K1, N1, N2) || ldw1 < K1 || ldw1 % 8 || ldw2 < N1 || ldw2 % 8) return hipErrorInvalidValue;
  if ((act1 != kActNone && act1 != kActRelu) || (act2 != kActNone && act2 != kActRelu)) return hipErrorInvalidValue;
  if (long(M) * N1 * 2 >= 0x7fffffffL) return hipErrorInvalidValue;   // 32-bit buffer offsets
  ChainArgs a{x, w1, b1, res, y1, w2, b2, y2, M, ldw1, ldw2, act1 == kActRelu ? 0.f : -INFINITY,
              act2 == kActRelu ? 0.f : -INFINITY};
  if (K1 == 64 && N1 == 256 && N2 == 64) return launch_chain<64, 256, 64>(a, s);
  if (K1 == 64 && N1 == 256 && N2 == 128) return launch_chain<64, 256, 128>(a, s);
  if (K1 == 128 && N1 == 512 && N2 == 128) return launch_chain<128, 512, 128>(a, s);
  return launch_chain<128, 512, 256>(a, s);
}

}  // namespace tfsk
