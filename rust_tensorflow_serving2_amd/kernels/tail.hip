// A ResNet bottleneck's tail in ONE kernel (gfx950): the 3x3 stride-1 conv
// (+ bias, act) and the expand 1x1 conv that reads exactly its output
// (+ bias, + the block's shortcut, act).
//
//   Y2 = act2(conv3x3(X) + b2)                 [M][C]   never leaves the CU
//   Y3 = act3(Y2 W3^T + b3 + R)                [M][N3]  (N3 = 4 C in ResNet-50)
//
// As two launches the expand re-reads Y2 from memory and pays a kernel
// boundary plus its own prologue; the 3x3's output tile is also written out.
// Here a workgroup owns a TH x TW block of output pixels of one image (BM
// rows) with ALL C channels of the 3x3 (the expand needs every channel of a
// pixel), keeps that tile in LDS as bf16 in the swizzled k-tile layout the
// MFMA fragment reads expect, and runs the expand over N3 in 128-column
// chunks.  Four waves split the columns (WGN = 4): every wave owns all BM rows,
// so the weights of both GEMMs are private per wave and go straight from L2
// into the MFMA B registers (halo.hip's register-B scheme: lane groups fq take
// 16 channels each, kk the 8-channel half, two adjacent 16-B loads per lane;
// the A fragment reads from LDS apply the same channel permutation).  LDS
// holds only the activations: the 3x3 input halo (double buffered per
// 64-channel chunk, by LDS-DMA), then the Y2 tile, plus a 16-row fp32 slab per
// wave for the two epilogues' transposes.
//
// SURVEY.md S8 (fused conv epilogues); the served network is the reference
// client's ResNet (/root/reference/serving/fetch.sh:7, src/lib.rs:229-257).
#include "gemm_common.h"

namespace tfsk {
namespace {

using namespace gemm;

constexpr int kTailNT = 256;          // 4 waves, all splitting columns
constexpr int kTailNC = 128;          // expand columns per chunk (32 per wave)
constexpr int kSlabLd = 68;           // fp32 slab row stride (floats), 16-B aligned rows

struct TailArgs {
  const uint16_t* x;     // 3x3 input, NHWC [nimg][H][W][C] bf16
  const uint16_t* w2;    // 3x3 weights [C][ldw2], k = tap * C + c
  const float* b2;       // [C]
  const uint16_t* w3;    // expand weights [N3][ldw3], k = c
  const float* b3;       // [N3]
  const uint16_t* res;   // shortcut [M][N3] bf16 or nullptr
  uint16_t* y;           // [M][N3] bf16
  int H, W, C, N3, ldw2, ldw3, nimg;
  int TH, TW;            // output block (launcher: pick_block)
  float lo2, lo3;        // activation floors: 0 (ReLU) or -inf (none)
};

template <int C, int BM, int HR>
struct TG {
  static constexpr int TM = BM / 16;
  static constexpr int WN1 = C / 4, TN1 = WN1 / 16;   // 3x3: wave columns
  static constexpr int TN2 = kTailNC / 4 / 16;        // expand: 2 fragments of 16 columns per chunk
  static constexpr int KT1 = C / KT;                  // 64-channel chunks
  static constexpr int HPW = HR / 32;                 // halo 1-KB DMA pieces per wave per chunk
  static constexpr int HALO_B = HR * 128;
  static constexpr int Y2_B = KT1 * BM * KT * 2;      // the 3x3 tile, bf16
  static constexpr int REGION = (2 * HALO_B > Y2_B ? 2 * HALO_B : Y2_B);
  static constexpr int SLAB_OFF = REGION;
  static constexpr int LDS = REGION + 4 * 16 * kSlabLd * 4;
  static_assert(BM % 16 == 0 && C % 64 == 0 && WN1 % 16 == 0 && HR % 32 == 0, "tail shape");
  static_assert(WN1 <= 64, "a wave's 3x3 columns fit one slab row");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

template <int C, int BM, int HR>
__global__ __launch_bounds__(kTailNT) void tail_kernel(TailArgs p) {
  using G = TG<C, BM, HR>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef __attribute__((address_space(3))) void* lds_ptr_t;

  const int TH = p.TH, TW = p.TW, HW2 = TW + 2, H = p.H, W = p.W;
  const int tph = (H + TH - 1) / TH, tpw = (W + TW - 1) / TW;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tw = wg % tpw;
  const int th = (wg / tpw) % tph;
  const int img = wg / (tpw * tph);
  const int h0 = th * TH, w0 = tw * TW;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wn = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int prow = lane >> 3;
  const uint32_t kc = uint32_t(((lane & 7) ^ prow) * 8);
  const int fr = lane & 15, fq = lane >> 4;

  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(p.x), 0, int(long(p.nimg) * H * W * C * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(p.w2), 0, int(long(C) * p.ldw2 * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW3 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(p.w3), 0, int(long(p.N3) * p.ldw3 * 2), 0x00020000);

  // ---- halo DMA offsets: halo row r = pixel (h0 - 1 + r / HW2, w0 - 1 + r % HW2)
  const int hrows = (TH + 2) * HW2;
  const float inv_hw2 = 1.f / float(HW2);
  uint32_t h_off[G::HPW];
#pragma unroll
  for (int j = 0; j < G::HPW; ++j) {
    const int r = (wn * G::HPW + j) * 8 + prow;
    const int rr = fdiv(r, HW2, inv_hw2);
    const int hh = h0 - 1 + rr, ww = w0 - 1 + (r - rr * HW2);
    const bool ok = r < hrows && unsigned(hh) < unsigned(H) && unsigned(ww) < unsigned(W);
    h_off[j] = ok ? (uint32_t((img * H + hh) * W + ww) * uint32_t(C) + kc) * 2u : kOOB;
  }
  auto issue_halo = [&](int c) {
    char* dst = smem + (c & 1) * G::HALO_B;
    const uint32_t soff = uint32_t(c) * (KT * 2);
    dma_fence();                        // the weight loads keep their place around the DMAs (gemm_common.h)
#pragma unroll
    for (int j = 0; j < G::HPW; ++j) {
      const uint32_t v = h_off[j];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsX, (lds_ptr_t)(dst + (wn * G::HPW + j) * 1024), 16, v, soff, 0, 0);
    }
    dma_fence();
  };

  // ---- 3x3 weights: this lane's columns wn * WN1 + j * 16 + fr, channels fq * 16 .. +15 of a chunk
  uint32_t b2_off[G::TN1];
#pragma unroll
  for (int j = 0; j < G::TN1; ++j)
    b2_off[j] = (uint32_t(wn * G::WN1 + j * 16 + fr) * uint32_t(p.ldw2) + uint32_t(fq * 16)) * 2u;
  typedef bf16x8 BFrag1[G::TN1][2];
  auto load_b2 = [&](int c, int u, BFrag1& dst) {
    const uint32_t soff = uint32_t(u * C + c * KT) * 2u;
#pragma unroll
    for (int j = 0; j < G::TN1; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        dst[j][kk] = __builtin_bit_cast(bf16x8, ordered_load16(rsW2, b2_off[j] + kk * 16u, soff));
  };

  // A rows: output pixel i * 16 + fr of the block -> halo row of tap (0, 0)
  int hrow0[G::TM];
#pragma unroll
  for (int i = 0; i < G::TM; ++i) {
    const int px = i * 16 + fr;
    const int ph = px / TW;
    hrow0[i] = px < TH * TW ? ph * HW2 + (px - ph * TW) : 0;
  }

  f32x4 acc[G::TM][G::TN1];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN1; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute1 = [&](const char* hb, const BFrag1& bq, int tap_off) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[G::TM];
#pragma unroll
      for (int i = 0; i < G::TM; ++i) {
        const int hr = hrow0[i] + tap_off;
        af[i] = *reinterpret_cast<const bf16x8*>(hb + uint32_t(hr) * 128u +
                                                 ((uint32_t((fq * 2 + kk) ^ (hr & 7))) << 4));
      }
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN1; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bq[j][kk], acc[i][j], 0, 0, 0);
    }
  };

  // ---- GEMM 1: the 3x3 over KT1 chunks x 9 taps (halo.hip halo_rb_kernel's
  // schedule: B two taps ahead in 3 register slots, one barrier per chunk)
  BFrag1 bq[3];
  issue_halo(0);
  load_b2(0, 0, bq[0]);
  load_b2(0, 1, bq[1]);
  constexpr int WAIT_HALO = 2 * 2 * G::TN1 < 63 ? 2 * 2 * G::TN1 : 63;
  auto chunk = [&](auto last_tag, int c) {
    constexpr bool LAST = decltype(last_tag)::value;
    const char* hb = smem + (c & 1) * G::HALO_B;
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      if (u == 0) {
        dma_fence();
        wait_vmcnt<WAIT_HALO>();
        lds_barrier();
        if (!LAST) issue_halo(c + 1);
      }
      if (u + 2 < 9) load_b2(c, u + 2, bq[(u + 2) % 3]);
      else if (!LAST) load_b2(c + 1, u + 2 - 9, bq[(u + 2) % 3]);
      compute1(hb, bq[u % 3], (u / 3) * HW2 + (u % 3));
    }
  };
  for (int c = 0; c < G::KT1 - 1; ++c) chunk(std::false_type{}, c);
  chunk(std::true_type{}, G::KT1 - 1);
  wait_vmcnt<0>();
  __syncthreads();                      // every wave is done with the halo buffers

  // ---- epilogue 1: bias + act -> bf16 Y2 tile in LDS (k-tile kt = channel / 64,
  // rows of 128 B, 16-B chunks swizzled by row & 7), through this wave's slab
  float* slab = reinterpret_cast<float*>(smem + G::SLAB_OFF) + wn * 16 * kSlabLd;
  char* y2t = smem;
  {
    constexpr int CPR = G::WN1 / 8;                    // 8-channel chunks per slab row (2..8)
    constexpr int IT = (16 * CPR + 63) / 64;
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
#pragma unroll
      for (int j = 0; j < G::TN1; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[(fq * 4 + r) * kSlabLd + j * 16 + fr] = acc[i][j][r];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < IT; ++k) {
        const int item = lane + 64 * k;
        if (item < 16 * CPR) {
          const int rl = item / CPR, cc = item % CPR;
          const float* src = slab + rl * kSlabLd + cc * 8;
          const float4 lo = *reinterpret_cast<const float4*>(src);
          const float4 hi = *reinterpret_cast<const float4*>(src + 4);
          const int n = wn * G::WN1 + cc * 8;
          const float4 c0 = *reinterpret_cast<const float4*>(p.b2 + n);
          const float4 c1 = *reinterpret_cast<const float4*>(p.b2 + n + 4);
          const uint4 ov = make_uint4(pack_bf16x2(fmaxf(lo.x + c0.x, p.lo2), fmaxf(lo.y + c0.y, p.lo2)),
                                      pack_bf16x2(fmaxf(lo.z + c0.z, p.lo2), fmaxf(lo.w + c0.w, p.lo2)),
                                      pack_bf16x2(fmaxf(hi.x + c1.x, p.lo2), fmaxf(hi.y + c1.y, p.lo2)),
                                      pack_bf16x2(fmaxf(hi.z + c1.z, p.lo2), fmaxf(hi.w + c1.w, p.lo2)));
          const int row = i * 16 + rl;
          const int kt = n >> 6, ch = (n & 63) >> 3;
          *reinterpret_cast<uint4*>(y2t + ((kt * BM + row) * KT + ((ch ^ (row & 7)) * 8)) * 2) = ov;
        }
      }
      __builtin_amdgcn_wave_barrier();   // slab reads done before the next rows overwrite it
    }
  }
  __syncthreads();                      // the whole Y2 tile is in LDS

  // ---- GEMM 2: Y2 (LDS) x W3^T, 128-column chunks; this wave's 32 columns
  // of a chunk, all BM rows; K = C in 32-deep MFMA steps (kk)
  constexpr int KK2 = C / 32;
  const int n_chunks = p.N3 / kTailNC;
  uint32_t b3_off[G::TN2];
#pragma unroll
  for (int j = 0; j < G::TN2; ++j)
    b3_off[j] = (uint32_t(wn * 32 + j * 16 + fr) * uint32_t(p.ldw3) + uint32_t(fq * 16)) * 2u;
  typedef bf16x8 BFrag2[G::TN2][KK2];
  auto load_b3 = [&](int nc, BFrag2& dst) {
    const uint32_t soff = uint32_t(nc * kTailNC) * uint32_t(p.ldw3) * 2u;
#pragma unroll
    for (int j = 0; j < G::TN2; ++j)
#pragma unroll
      for (int kk = 0; kk < KK2; ++kk)   // kk = 2 * k-tile + half: channels 64 * (kk / 2) + fq * 16 + 8 * (kk % 2)
        dst[j][kk] = __builtin_bit_cast(
            bf16x8, ordered_load16(rsW3, b3_off[j] + uint32_t((kk >> 1) * 128 + (kk & 1) * 16), soff));
  };
  // this lane's epilogue item: slab row rl2, 8-column chunk cc2 of the wave's 32
  const int rl2 = lane >> 2, cc2 = lane & 3;
  const __amdgpu_buffer_rsrc_t rsR = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(p.res), 0, p.res ? int(long(p.nimg) * H * W * p.N3 * 2) : 0, 0x00020000);
  auto out_row = [&](int row) -> int {   // global row of block row `row`, or -1
    if (row >= TH * TW) return -1;
    const int ph = row / TW, pw = row - ph * TW;
    const int h = h0 + ph, w = w0 + pw;
    if (h >= H || w >= W) return -1;
    return (img * H + h) * W + w;
  };

  BFrag2 b3q[2];
  load_b3(0, b3q[0]);
  auto chunk2 = [&](int nc, const BFrag2& bw) {
    f32x4 acc2[G::TM][G::TN2];
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int j = 0; j < G::TN2; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KK2; ++kk) {
      const char* sa = y2t + (kk >> 1) * BM * KT * 2;
      bf16x8 af[G::TM];
#pragma unroll
      for (int i = 0; i < G::TM; ++i) {
        const int row = i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(sa + (row * KT + (((fq * 2 + (kk & 1)) ^ (row & 7)) * 8)) * 2);
      }
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN2; ++j)
          acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bw[j][kk], acc2[i][j], 0, 0, 0);
    }
    // epilogue 2: + bias + shortcut, act, 16-B bf16 row chunks
    const int n = nc * kTailNC + wn * 32 + cc2 * 8;
    const float4 c0 = *reinterpret_cast<const float4*>(p.b3 + n);
    const float4 c1 = *reinterpret_cast<const float4*>(p.b3 + n + 4);
    const float bv[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int m = out_row(i * 16 + rl2);
      const u32x4 rr = __builtin_amdgcn_raw_buffer_load_b128(
          rsR, m >= 0 ? (uint32_t(m) * uint32_t(p.N3) + uint32_t(n)) * 2u : kOOB, 0, 0);
#pragma unroll
      for (int j = 0; j < G::TN2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab[(fq * 4 + r) * kSlabLd + j * 16 + fr] = acc2[i][j][r];
      __builtin_amdgcn_wave_barrier();
      const float* src = slab + rl2 * kSlabLd + cc2 * 8;
      const float4 lo = *reinterpret_cast<const float4*>(src);
      const float4 hi = *reinterpret_cast<const float4*>(src + 4);
      const float a[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      const uint32_t rw[4] = {rr.x, rr.y, rr.z, rr.w};
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v0 = fmaxf(a[2 * e] + bv[2 * e] + __uint_as_float(rw[e] << 16), p.lo3);
        const float v1 = fmaxf(a[2 * e + 1] + bv[2 * e + 1] + __uint_as_float(rw[e] & 0xffff0000u), p.lo3);
        o[e] = pack_bf16x2(v0, v1);
      }
      if (m >= 0) *reinterpret_cast<uint4*>(p.y + size_t(m) * p.N3 + n) = make_uint4(o[0], o[1], o[2], o[3]);
      __builtin_amdgcn_wave_barrier();   // slab reads done before the next rows overwrite it
    }
  };
  // two register sets of W3 fragments: the next chunk's loads fly while this
  // chunk computes (the loop is unrolled by 2 so the sets are static)
  for (int nc = 0; nc < n_chunks; nc += 2) {
    if (nc + 1 < n_chunks) load_b3(nc + 1, b3q[1]);
    chunk2(nc, b3q[0]);
    if (nc + 1 < n_chunks) {
      if (nc + 2 < n_chunks) load_b3(nc + 2, b3q[0]);
      chunk2(nc + 1, b3q[1]);
    }
  }
}

// Output block for a BM-pixel tile whose halo fits HR rows (halo.hip's rule:
// fewest tiles, then the smallest halo, blocks balanced).
bool tail_block(int H, int W, int BM, int HR, int& TH, int& TW) {
  long best_tiles = -1, best_halo = 0;
  for (int tw = 1; tw <= W; ++tw) {
    int th = BM / tw < H ? BM / tw : H;
    while (th >= 1 && (th + 2) * (tw + 2) > HR) --th;
    if (th < 1) continue;
    const int nh = (H + th - 1) / th, nw = (W + tw - 1) / tw;
    const int bh = (H + nh - 1) / nh, bw = (W + nw - 1) / nw;
    const long tiles = long(nh) * nw, halo = long(bh + 2) * (bw + 2);
    if (best_tiles < 0 || tiles < best_tiles || (tiles == best_tiles && halo < best_halo)) {
      best_tiles = tiles;
      best_halo = halo;
      TH = bh;
      TW = bw;
    }
  }
  return best_tiles > 0;
}

template <int C, int BM, int HR>
hipError_t launch_tail(TailArgs a, hipStream_t s) {
  using G = TG<C, BM, HR>;
  if (!tail_block(a.H, a.W, BM, HR, a.TH, a.TW)) return hipErrorInvalidValue;
  const long tiles = long(a.nimg) * ((a.H + a.TH - 1) / a.TH) * ((a.W + a.TW - 1) / a.TW);
  if (tiles <= 0) return hipSuccess;
  if (tiles >= (1L << 31)) return hipErrorInvalidValue;
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&tail_kernel<C, BM, HR>), G::LDS);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((tail_kernel<C, BM, HR>), dim3(unsigned(tiles)), dim3(kTailNT), G::LDS, s, a);
  return hipGetLastError();
}

}  // namespace

// (C, config) pairs: config 0 = the larger pixel block, 1 = the smaller
bool tail_supported(int C, int N3, int cfg) {
  return (C == 64 || C == 128 || C == 256) && N3 % kTailNC == 0 && N3 > 0 && (cfg == 0 || cfg == 1);
}

hipError_t tail_launch(const uint16_t* x, const uint16_t* w2, int ldw2, const float* b2, const uint16_t* w3,
                       int ldw3, const float* b3, const uint16_t* res, uint16_t* y, int nimg, int H, int W, int C,
                       int N3, int act2, int act3, int cfg, hipStream_t s) {
  if (nimg <= 0) return hipSuccess;
  if (!tail_supported(C, N3, cfg) || ldw2 < 9 * C || ldw2 % 8 || ldw3 < C || ldw3 % 8) return hipErrorInvalidValue;
  if ((act2 != kActNone && act2 != kActRelu) || (act3 != kActNone && act3 != kActRelu)) return hipErrorInvalidValue;
  if (long(nimg) * H * W * (N3 > C ? N3 : C) * 2 >= 0x7fffffffL) return hipErrorInvalidValue;   // 32-bit offsets
  TailArgs a{x, w2, b2, w3, b3, res, y, H, W, C, N3, ldw2, ldw3, nimg, 0, 0,
             act2 == kActRelu ? 0.f : -INFINITY, act3 == kActRelu ? 0.f : -INFINITY};
  switch (C * 2 + cfg) {
    case 128: return launch_tail<64, 224, 320>(a, s);     // stage 2: 4 rows x 56 (halo 6 x 58 = 348 > 320 -> 3 rows)
    case 129: return launch_tail<64, 128, 192>(a, s);
    case 256: return launch_tail<128, 112, 192>(a, s);    // stage 3: 4 rows x 28, halo 6 x 30 = 180
    case 257: return launch_tail<128, 64, 128>(a, s);
    case 512: return launch_tail<256, 64, 128>(a, s);     // stage 4: 4 rows x 14 (56 px), halo 6 x 16 = 96
    case 513: return launch_tail<256, 32, 64>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tfsk
