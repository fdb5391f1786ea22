// Halo-tiled 3x3 stride-1 convolution for MI355X (gfx950): bf16 NHWC operands,
// fp32 MFMA accumulate, the cgemm epilogue (bias / residual / act, split-K).
//
// Why: the implicit-GEMM (im2col) path streams every input pixel into LDS nine
// times (once per filter tap).  Per-CU LDS-DMA intake tops out at ~70 GB/s
// (MI355X_MICROARCH.md, "indexed rows" / ldsdma-fill), and the round-1
// rocprofv3 replay (profiles/r50_b32_replay_round1_final.txt) put the ResNet-50
// 3x3 layers at 10-13 TB/s of chip-wide intake: 115-236 MB per layer at b32,
// i.e. intake-bound at 3-8x their MFMA time.  Here a workgroup owns a TH x TW
// block of output pixels of one image (+ a BN slice of output channels); per
// 64-channel chunk it DMAs the (TH+2) x (TW+2) input halo into LDS ONCE and
// runs all nine taps against it — the A operand of tap (kh, kw) is the halo
// shifted by kh*(TW+2) + kw rows.  A-intake drops ~9x -> ~1.3-1.9x of the
// input; only the weight slices (B) stream per tap.
//
//   * K loop = (chunk c, tap u) steps; B ring of S = 3 or 9 slots with S - 1
//     weight tiles in flight.  Depth matters: a CU takes in ~55 GB/s with 16 KB of
//     LDS-DMA in flight but 100-125 GB/s with 32-64 KB
//     (scripts/intake_bench.hip, profiles/round2/intake_bench.log); the first
//     version kept two 8-KB B tiles in flight and ran the 3x3 layers B-bound;
//   * the halo of chunk c+1 is DMA'd into the other halo buffer while chunk c
//     computes (one buffer when C == 64: no next chunk);
//   * counted vmcnt waits: with the taps unrolled and a separate body for the
//     last chunk, the number of DMAs issued after B(step) is a compile-time
//     constant per tap (a run-time switch over it cost ~12 scalar branches per
//     step and made the kernel slower than the 2-deep original);
//   * LDS rows are 128 B with 16-B chunks XOR-swizzled by a per-row key.  The
//     key is NOT the storage row (row & 7, cgemm's image): 16 output pixels of
//     a fragment sit on consecutive halo rows only inside one tile row, and a
//     TW -> TW + 2 jump at each tile-row end put two lanes of an 8-lane LDS
//     group on the same bank slot (rocprofv3: 1.4-2.3 SQ_LDS_BANK_CONFLICT
//     cycles per LDS instruction at ResNet-50 stage 3, 9e5 per launch;
//     profiles/round6/r6e).  halo_key uses the halo pixel's index in the
//     tile's TW-wide numbering instead, (ii TH + h) TW + w: a fragment's 16
//     rows then carry 16 consecutive keys at every tap (the tap adds
//     kh TW + kw to all of them), so every 8-lane group hits 8 distinct slots.
//     The DMA applies the key on the source address (lane-linear LDS image);
//   * tile -> workgroup: XCD-aware remap, output-channel slices innermost so
//     the workgroups sharing one halo run on one XCD (shared L2);
//   * split-K over channel chunks (gridDim.y), partial slabs indexed by the
//     output pixel row, reduced by splitk_reduce like every other GEMM.
#include <algorithm>
#include <type_traits>

#include "gemm_common.h"
#include "cgemm.h"

namespace tfsk {

namespace {

using namespace gemm;

// XOR key of a halo row from its pixel index in the tile's TW-wide numbering
// (see the header: conflict-free fragment reads across tile-row ends)
__device__ __forceinline__ int halo_key(int lin) { return lin & 7; }

template <int BM, int BN, int WGM, int WGN, int HR, int S_>
struct HG {
  static constexpr int NW = WGM * WGN, NT = 64 * NW;
  static constexpr int WM = BM / WGM, WN = BN / WGN;
  static constexpr int TM = WM / 16, TN = WN / 16;
  static constexpr int HPW = HR / (8 * NW);        // halo 1-KB DMA pieces per wave per chunk
  static constexpr int BPW = BN / (8 * NW);        // B pieces per wave per step
  static constexpr int S = S_;                     // B ring depth (S - 1 tiles in flight)
  static_assert(S == 3 || S == 9, "ring depth must divide the 9 taps (static slots)");
  static constexpr int HALO_B = HR * 128;          // bytes of one halo buffer
  static constexpr int B_B = BN * 128;             // bytes of one B ring slot
  static constexpr int CS_LD = BN + 4;
  static constexpr int LDS_EPI = BM * CS_LD * 4;
  static constexpr int lds(int nbuf) {
    return (nbuf * HALO_B + S * B_B) > LDS_EPI ? (nbuf * HALO_B + S * B_B) : LDS_EPI;
  }
  static_assert(HPW >= 1 && HR % (8 * NW) == 0, "halo DMA split");
  static_assert(BPW >= 1 && BN % (8 * NW) == 0, "B DMA split");
  static_assert(TM >= 1 && TN >= 1 && WM % 16 == 0 && WN % 16 == 0, "wave tile");
  static_assert(HPW + BPW * (S - 2) <= 39, "vmcnt immediate range");
  static_assert(lds(2) <= 160 * 1024, "LDS budget");
};

// Shared epilogue of the halo kernels: the fp32 accumulator tile staged in LDS
// (row = output pixel of the TH x TW block), split-K slab / in-kernel fixup,
// then bias / residual / activation row chunks.  The caller has drained its
// DMAs and met a barrier, so the LDS is free.
template <int BM, int BN, int NT, int TM, int TN, int WM, int WN>
__device__ __forceinline__ void halo_epilogue(const IGemmArgs& p, const f32x4 (&acc)[TM][TN], char* smem, int h0,
                                              int w0, int img, int n0, int wm, int wn, int tid, float4 bias0,
                                              float4 bias1) {
  constexpr int CS_LD = BN + 4;
  const int TH = p.TH, TW = p.TW, Ho = p.Ho, Wo = p.Wo;
  const int TI = p.TI > 1 ? p.TI : 1, nimg = p.M / (Ho * Wo);
  const int lane = tid & 63, fr = lane & 15, fq = lane >> 4;
  auto out_row = [&](int row) -> int {   // global GEMM row of tile row `row`, or -1
    if (row >= TI * TH * TW) return -1;
    const int ii = row / (TH * TW), r2 = row - ii * (TH * TW);
    const int ph = r2 / TW, pw = r2 - ph * TW;
    const int h = h0 + ph, w = w0 + pw;
    if (h >= Ho || w >= Wo || img + ii >= nimg) return -1;
    return ((img + ii) * Ho + h) * Wo + w;
  };

  // ---- plain bf16 output (no split, residual or second output; any
  // activation but erf: the 3x3 convs of a bottleneck): bias and activation
  // in registers, the bf16 tile staged once (half the LDS bytes of the fp32
  // image), whole 16-B row chunks out.  Same arithmetic as epi_chunk (see
  // cgemm_impl.h, the one-pass bf16 epilogue).
  if (p.splits <= 1 && p.residual == nullptr && p.out2 == nullptr && !p.out_f32 && p.out != nullptr &&
      p.act != kActGeluErf && !p.epi_f32) {
    constexpr int CB_LD = BN + 8;
    uint16_t* Cb = reinterpret_cast<uint16_t*>(smem);
    const bool use_b = p.bias != nullptr && p.N % 8 == 0;
    const __amdgpu_buffer_rsrc_t rsb =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.bias), 0, use_b ? p.N * 4 : 0, 0x00020000);
    float bj[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bj[j] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(rsb, uint32_t(n0 + wn * WN + j * 16 + fr) * 4u, 0, 0));
    const float alpha = p.alpha;
    auto stage = [&](auto act_tag) __attribute__((always_inline)) {
      constexpr int ACT = decltype(act_tag)::value;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = act_fn<ACT>(acc[i][j][r] * alpha + bj[j] + 0.f);
            Cb[(wm * WM + i * 16 + fq * 4 + r) * CB_LD + wn * WN + j * 16 + fr] =
                __builtin_bit_cast(uint16_t, static_cast<__bf16>(v));
          }
    };
    switch (p.act) {
      case kActRelu: stage(std::integral_constant<int, kActRelu>{}); break;
      case kActGeluTanh: stage(std::integral_constant<int, kActGeluTanh>{}); break;
      case kActTanh: stage(std::integral_constant<int, kActTanh>{}); break;
      default: stage(std::integral_constant<int, kActNone>{}); break;
    }
    __syncthreads();
    constexpr int CPRB = BN / 8;
#pragma unroll 4
    for (int c = tid; c < BM * CPRB; c += NT) {
      const int row = c / CPRB, ch = c - row * CPRB;
      const int m = out_row(row), n = n0 + ch * 8;
      if (m >= 0 && n < p.N)
        *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p.out) + size_t(m) * p.ldc + n) =
            *reinterpret_cast<const uint4*>(Cb + row * CB_LD + ch * 8);
    }
    return;
  }

  // ---- epilogue: fp32 tile staged in LDS; row = output pixel of the block
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * WM + i * 16 + fq * 4 + r) * CS_LD + wn * WN + j * 16 + fr] = acc[i][j][r];
  __syncthreads();

  using E = Epi<BM, BN, NT>;
  IGemmArgs q = p;                      // the epilogue's view (split-K fixup: splits 1, alpha 1)
  if (p.splits > 1) {
    const float alpha = p.alpha;
    float* ws = p.ws + size_t(blockIdx.y) * p.M * p.N;
    const __amdgpu_buffer_rsrc_t wsr = splitk_rsrc(p);
#pragma unroll 1
    for (int it = 0; it < E::ITERS; ++it) {
      int row, col;
      if (!epi_rowcol<BM, BN, NT>(tid, it, row, col)) continue;
      const int m = out_row(row), n = n0 + col;
      if (m < 0 || n >= p.N) continue;
      const float* src = Cs + row * CS_LD + col;
      float4 a = *reinterpret_cast<const float4*>(src);
      float4 b = *reinterpret_cast<const float4*>(src + 4);
      a.x *= alpha; a.y *= alpha; a.z *= alpha; a.w *= alpha;
      b.x *= alpha; b.y *= alpha; b.z *= alpha; b.w *= alpha;
      float* dst = ws + size_t(m) * p.N + n;
      if (p.counters != nullptr) {
        splitk_store8(p, wsr, m, n, a, b);
      } else {
        *reinterpret_cast<float4*>(dst) = a;
        *reinterpret_cast<float4*>(dst + 4) = b;
      }
    }
    if (p.counters == nullptr || !splitk_arrive(p, blockIdx.x)) {
      trace_stamp(p, 3);
      return;
    }
    // the last slice of this tile: every slab summed back into Cs, then the
    // epilogue below with the bias the split path did not prefetch
    // (unrolled: every chunk's slab loads in flight together)
#pragma unroll
    for (int it = 0; it < E::ITERS; ++it) {
      int row, col;
      if (!epi_rowcol<BM, BN, NT>(tid, it, row, col)) continue;
      const int m = out_row(row), n = n0 + col;
      if (m < 0 || n >= p.N) continue;
      float4 lo, hi;
      splitk_sum8(p, wsr, m, n, lo, hi);
      *reinterpret_cast<float4*>(Cs + row * CS_LD + col) = lo;
      *reinterpret_cast<float4*>(Cs + row * CS_LD + col + 4) = hi;
    }
    __syncthreads();
    q.splits = 1;
    q.alpha = 1.f;                      // the slabs carry alpha already
    prefetch_bias<BM, BN, NT>(q, n0, tid, bias0, bias1);
  }
  const float bv[8] = {bias0.x, bias0.y, bias0.z, bias0.w, bias1.x, bias1.y, bias1.z, bias1.w};
  auto run = [&](auto act_tag) {
    constexpr int ACT = decltype(act_tag)::value;
#pragma unroll 2
    for (int it = 0; it < E::ITERS; ++it) {
      int row, col;
      if (!epi_rowcol<BM, BN, NT>(tid, it, row, col)) continue;
      const int m = out_row(row), n = n0 + col;
      if (m < 0 || n >= q.N) continue;
      const uint4 rr = q.residual ? *reinterpret_cast<const uint4*>(q.residual + size_t(m) * q.ldr + n)
                                  : make_uint4(0, 0, 0, 0);
      epi_chunk<ACT>(q, Cs + row * CS_LD + col, m, n, bv, rr);
    }
  };
  switch (q.act) {
    case kActRelu: run(std::integral_constant<int, kActRelu>{}); break;
    case kActGeluTanh: run(std::integral_constant<int, kActGeluTanh>{}); break;
    case kActGeluErf: run(std::integral_constant<int, kActGeluErf>{}); break;
    case kActTanh: run(std::integral_constant<int, kActTanh>{}); break;
    default: run(std::integral_constant<int, kActNone>{}); break;
  }
}

template <int BM, int BN, int WGM, int WGN, int HR, int S, bool PF>
__global__ __launch_bounds__(64 * WGM * WGN) void halo_conv_kernel(IGemmArgs p) {
  using G = HG<BM, BN, WGM, WGN, HR, S>;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  char* const smem = reinterpret_cast<char*>(smem_raw);
  typedef __attribute__((address_space(3))) void* lds_ptr_t;

  const int TH = p.TH, TW = p.TW, HW2 = TW + 2;
  const int Ho = p.Ho, Wo = p.Wo, H = p.H, W = p.W, C = p.C;
  const int tph = (Ho + TH - 1) / TH, tpw = (Wo + TW - 1) / TW;
  const int nbn = (p.N + BN - 1) / BN;
  const int TI = p.TI > 1 ? p.TI : 1, nimg = p.M / (Ho * Wo);
  const int HB = (TH + 2) * HW2;                  // halo rows of one image's block

  // ---- tile of this workgroup: (image, tile row, tile col, channel slice)
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int bn = wg % nbn;
  int r_ = wg / nbn;
  const int tw = r_ % tpw;
  r_ /= tpw;
  const int th = r_ % tph;
  const int img = (r_ / tph) * TI;                // first image of the tile
  const int h0 = th * TH, w0 = tw * TW, n0 = bn * BN;

  trace_stamp(p, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int prow = lane >> 3;
  const uint32_t kc = uint32_t(((lane & 7) ^ prow) * 8);

  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.a), 0, int(p.a_bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.b), 0, int(p.b_bytes), 0x00020000);

  // ---- per-lane halo DMA offsets: halo row r = image ii = r / HB of the tile,
  // pixel (h0 - PT + q / HW2, w0 - PL + q % HW2) with q = r % HB
  const int hrows = TI * HB;
  const float inv_hw2 = 1.f / float(HW2), inv_hb = 1.f / float(HB);
  uint32_t h_off[G::HPW];
#pragma unroll
  for (int j = 0; j < G::HPW; ++j) {
    const int r = (wid * G::HPW + j) * 8 + prow;
    const int ii = TI > 1 ? fdiv(r, HB, inv_hb) : 0;
    const int q = r - ii * HB;
    const int rr = fdiv(q, HW2, inv_hw2);
    const int hh = h0 - p.PT + rr, ww = w0 - p.PL + (q - rr * HW2);
    const bool ok = r < hrows && img + ii < nimg && unsigned(hh) < unsigned(H) && unsigned(ww) < unsigned(W);
    const uint32_t kh = uint32_t(((lane & 7) ^ halo_key(ii * TH * TW + rr * TW + (q - rr * HW2))) * 8);
    h_off[j] = ok ? (uint32_t(((img + ii) * H + hh) * W + ww) * uint32_t(C) + kh) * 2u : kOOB;
  }
  uint32_t b_off[G::BPW];
#pragma unroll
  for (int j = 0; j < G::BPW; ++j) {
    const int n = n0 + (wid * G::BPW + j) * 8 + prow;
    b_off[j] = n < p.N ? (uint32_t(n) * uint32_t(p.ldb) + kc) * 2u : kOOB;
  }

  // ---- channel-chunk range (split-K: blockIdx.y selects a slice of chunks)
  const int nch = C / KT;
  int c0 = 0, c1 = nch;
  if (p.splits > 1) {
    c0 = blockIdx.y * p.kt_per_split;
    c1 = min(nch, c0 + p.kt_per_split);
  }
  const int nbuf = (c1 - c0) > 1 ? 2 : 1;
  char* const ring = smem + nbuf * G::HALO_B;

  auto issue_halo = [&](int c) {
    char* dst = smem + ((c - c0) & 1) * G::HALO_B;
    const uint32_t soff = uint32_t(c) * (KT * 2);
#pragma unroll
    for (int j = 0; j < G::HPW; ++j) {
      const uint32_t v = h_off[j];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_ptr_t)(dst + (wid * G::HPW + j) * 1024), 16, v, soff, 0, 0);
    }
  };
  // weights k = tap * C + channel
  auto issue_b = [&](int c, int u, int slot) {
    const uint32_t soff = uint32_t(u * C + c * KT) * 2u;
#pragma unroll
    for (int j = 0; j < G::BPW; ++j) {
      const uint32_t v = b_off[j];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_ptr_t)(ring + slot * G::B_B + (wid * G::BPW + j) * 1024),
                                               16, v, soff, 0, 0);
    }
  };

  // ---- consumer fragments: A rows are output pixels -> halo rows (tap (0,0))
  const int fr = lane & 15, fq = lane >> 4;
  int hrow0[G::TM], kpx0[G::TM];
#pragma unroll
  for (int i = 0; i < G::TM; ++i) {
    const int px = wm * G::WM + i * 16 + fr;
    const int ii = px / (TH * TW), p2 = px - ii * (TH * TW);
    const int ph = p2 / TW;
    hrow0[i] = px < TI * TH * TW ? ii * HB + ph * HW2 + (p2 - ph * TW) : 0;
    kpx0[i] = px;
  }
  const uint32_t rb0 = uint32_t(((wn * G::WN + fr) * KT + ((fq ^ (fr & 7)) * 8)) * 2);
  const uint32_t rb1 = uint32_t(((wn * G::WN + fr) * KT + (((4 + fq) ^ (fr & 7)) * 8)) * 2);

  f32x4 acc[G::TM][G::TN];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one tap's operand fragments (both 32-deep k halves of the 64-channel chunk)
  struct Frags {
    bf16x8 a[2][G::TM], b[2][G::TN];
  };
  auto load_frags = [&](Frags& f, const char* hb, const char* sb, int tap_off, int tap_key) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < G::TM; ++i) {
        const int hr = hrow0[i] + tap_off;
        const uint32_t addr = uint32_t(hr) * 128u + ((uint32_t((kk * 4 + fq) ^ halo_key(kpx0[i] + tap_key))) << 4);
        f.a[kk][i] = *reinterpret_cast<const bf16x8*>(hb + addr);
      }
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
  auto compute = [&](const char* hb, const char* sb, int tap_off, int tap_key) {
    Frags f;
    load_frags(f, hb, sb, tap_off, tap_key);
    mma(f);
  };
  // PF: the fragments of step t are read from LDS right after step t's
  // barrier, and the MFMAs of step t - 1 (fragments already in registers) run
  // while those reads are in flight -- the LDS latency and the barrier no
  // longer sit between a step's data landing and its MFMAs
  Frags prev;

  float4 bias0, bias1;
  prefetch_bias<BM, BN, G::NT>(p, n0, tid, bias0, bias1);

  // ---- steps t = (chunk c0 + t / 9, tap u = t % 9); B(t) lands in slot
  // t % S = u % S (S divides 9), D = S - 1 tiles issued ahead.  Every chunk but
  // the last has the same DMA schedule, so the taps are unrolled and every
  // wait count is an immediate: DMAs younger than B(t) are B(t+1 .. t+D-1)
  // (fewer in the last chunk's tail) plus this chunk's halo issue when it went
  // out after B(t), i.e. at tap 0 with 1 <= u < D.
  constexpr int D = G::S - 1;
  const int nck = c1 - c0;
  issue_halo(c0);
#pragma unroll
  for (int j = 0; j < D; ++j)
    if (j < nck * 9) issue_b(c0 + j / 9, j % 9, j % G::S);

  auto chunk = [&](auto last_tag, int c) {
    constexpr bool LAST = decltype(last_tag)::value;
    const char* hb = smem + ((c - c0) & 1) * G::HALO_B;
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      const int nb = LAST ? (D - 1 < 8 - u ? D - 1 : 8 - u) : D - 1;
      const int younger = G::BPW * nb + ((!LAST && u >= 1 && u < D) ? G::HPW : 0);
      switch (younger) {   // folds to one immediate per unrolled tap
#define TFSK_W(k) case k: wait_vmcnt<k>(); break;
        TFSK_W(0) TFSK_W(1) TFSK_W(2) TFSK_W(3) TFSK_W(4) TFSK_W(5) TFSK_W(6) TFSK_W(7) TFSK_W(8) TFSK_W(9)
        TFSK_W(10) TFSK_W(11) TFSK_W(12) TFSK_W(13) TFSK_W(14) TFSK_W(15) TFSK_W(16) TFSK_W(17) TFSK_W(18)
        TFSK_W(19) TFSK_W(20) TFSK_W(21) TFSK_W(22) TFSK_W(23) TFSK_W(24) TFSK_W(25) TFSK_W(26) TFSK_W(27)
        TFSK_W(28) TFSK_W(29) TFSK_W(30) TFSK_W(31) TFSK_W(32) TFSK_W(33) TFSK_W(34) TFSK_W(35) TFSK_W(36)
        TFSK_W(37) TFSK_W(38) TFSK_W(39)
#undef TFSK_W
        default: wait_vmcnt<40>(); break;
      }
      lds_barrier();   // every wave's DMAs landed; the slot / buffer about to be refilled is read-free
      if (u == 0 && c == c0) trace_stamp(p, 1);
      if (!LAST && u == 0) issue_halo(c + 1);
      if (!LAST || u + D < 9) issue_b(c + (u + D) / 9, (u + D) % 9, (u + D) % G::S);
      if constexpr (PF) {
        // the scheduler would hoist the (register-only) MFMAs of the previous
        // step above the barrier and sink these reads to their uses: pin both
        __builtin_amdgcn_sched_barrier(0);
        Frags cur;
        load_frags(cur, hb, ring + (u % G::S) * G::B_B, (u / 3) * HW2 + (u % 3), (u / 3) * TW + (u % 3));
        __builtin_amdgcn_sched_barrier(0);
        if (u > 0 || c > c0) mma(prev);
        __builtin_amdgcn_sched_barrier(0);   // (and keep them above the next step's barrier)
        prev = cur;
      } else {
        compute(hb, ring + (u % G::S) * G::B_B, (u / 3) * HW2 + (u % 3), (u / 3) * TW + (u % 3));
      }
    }
  };
  for (int c = c0; c < c1 - 1; ++c) chunk(std::false_type{}, c);
  chunk(std::true_type{}, c1 - 1);
  if constexpr (PF) mma(prev);
  wait_vmcnt<0>();
  __syncthreads();
  trace_stamp(p, 2);

  halo_epilogue<BM, BN, G::NT, G::TM, G::TN, G::WM, G::WN>(p, acc, smem, h0, w0, img, n0, wm, wn, tid, bias0,
                                                              bias1);
  trace_stamp(p, 3);
}

// ---------------------------------------------------------------- persistent halo conv
// halo_persist_kernel (id kHaloPersistCfg): the 3x3 layers whose whole filter
// fits in LDS -- one 64-channel input chunk and 64 output channels (ResNet-50
// stage 1, 56x56x64 -> 64: 9 taps x 64 x 64 bf16 = 72 KB).  halo_conv_kernel
// runs them as ~1.75 waves of workgroups that all wait for their first halo at
// once, compute, then all store at once: 17-18 us at b32 for 7.4 GFLOP
// (profiles/round6/r6n/replay_r50_b32.txt), the halo latency and the store
// tail exposed in every workgroup.  Here one workgroup per CU:
//   * the 9 taps' weights are DMA'd ONCE into 9 resident slots (the image of
//     halo_conv_kernel's B ring), so the K loop of a tile has no barrier;
//   * the workgroup walks its tiles (tile = blockIdx.x + k * gridDim.x) with
//     two halo buffers: tile k+1's halo goes out right after tile k's opening
//     barrier and lands while tile k computes;
//   * epilogue: bias + act in registers, the bf16 tile staged in its own LDS
//     region, 16-B buffer stores -- unconditional (rows past the output go to
//     an out-of-range offset and are dropped), so each lane has exactly
//     kStores stores in flight and the next tile's opening wait is the counted
//     vmcnt(kStores): the stores drain while the next tile computes;
//   * raw s_barrier (lds_barrier) only: a __syncthreads() would drain vmcnt.
// Plain bf16 output only (bias, act != erf; no residual / second output /
// split): the launcher rejects the rest, which the tuner skips.
constexpr int kPersistBM = 128, kPersistBN = 64, kPersistHR = 192;
struct HPs {
  static constexpr int BM = kPersistBM, BN = kPersistBN, HR = kPersistHR;
  static constexpr int WGM = 4, WGN = 2, NW = 8, NT = 512;
  static constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  static constexpr int HPW = HR / (8 * NW), BPW = BN / (8 * NW);
  static constexpr int B_B = BN * 128, HALO_B = HR * 128;
  static constexpr int CB_LD = BN + 8;
  static constexpr int STG_B = BM * CB_LD * 2;
  static constexpr int OFF_HALO = 9 * B_B, OFF_STG = OFF_HALO + 2 * HALO_B;
  static constexpr int LDS = OFF_STG + STG_B;
  static constexpr int kStores = BM * (BN / 8) / NT;     // 16-B stores per thread per tile
  static_assert(HPW * 8 * NW == HR && BPW == 1 && kStores * NT == BM * (BN / 8), "persistent halo split");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

__global__ __launch_bounds__(512, 1) void halo_persist_kernel(IGemmArgs p, int ntiles) {
  using G = HPs;
  constexpr int BM = G::BM, BN = G::BN;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  char* const smem = reinterpret_cast<char*>(smem_raw);
  typedef __attribute__((address_space(3))) void* lds_ptr_t;

  const int TH = p.TH, TW = p.TW, HW2 = TW + 2;
  const int Ho = p.Ho, Wo = p.Wo, H = p.H, W = p.W, C = p.C;
  const int tph = (Ho + TH - 1) / TH, tpw = (Wo + TW - 1) / TW;
  const int TI = p.TI > 1 ? p.TI : 1, nimg = p.M / (Ho * Wo);
  const int HB = (TH + 2) * HW2, hrows = TI * HB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / G::WGN, wn = wid % G::WGN;
  const int prow = lane >> 3;
  const int fr = lane & 15, fq = lane >> 4;

  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.a), 0, int(p.a_bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p.b), 0, int(p.b_bytes), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsO =
      __builtin_amdgcn_make_buffer_rsrc(p.out, 0, int(long(p.M) * p.ldc * 2), 0x00020000);
  const bool use_b = p.bias != nullptr;
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.bias), 0, use_b ? BN * 4 : 0, 0x00020000);

  // bias first (a VGPR-destination load: issued and used before any DMA, so
  // no wait on it lands inside the DMA pipeline)
  float bj[G::TN];
#pragma unroll
  for (int j = 0; j < G::TN; ++j)
    bj[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsb, uint32_t(wn * G::WN + j * 16 + fr) * 4u, 0, 0));
  const float alpha = p.alpha;
  gemm::wait_vmcnt<0>();

  // ---- the filter: 9 resident slots, slot u = tap u (k = u * C + channel), rows n swizzled by n & 7
  {
    const uint32_t kc = uint32_t(((lane & 7) ^ prow) * 8);
    const int n = wid * 8 + prow;
    const uint32_t boff = (uint32_t(n) * uint32_t(p.ldb) + kc) * 2u;
#pragma unroll
    for (int u = 0; u < 9; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_ptr_t)(smem + u * G::B_B + wid * 1024), 16, boff,
                                               uint32_t(u * C) * 2u, 0, 0);
  }
  // ---- halo DMA of tile t into buffer b (halo_key swizzle, as halo_conv_kernel)
  const float inv_hw2 = 1.f / float(HW2), inv_hb = 1.f / float(HB);
  auto issue_halo = [&](int t, int b) {
    int r_ = t;
    const int tw = r_ % tpw;
    r_ /= tpw;
    const int th = r_ % tph;
    const int img = (r_ / tph) * TI;
    const int h0 = th * TH, w0 = tw * TW;
    char* dst = smem + G::OFF_HALO + b * G::HALO_B;
#pragma unroll
    for (int j = 0; j < G::HPW; ++j) {
      const int r = (wid * G::HPW + j) * 8 + prow;
      const int ii = TI > 1 ? fdiv(r, HB, inv_hb) : 0;
      const int q = r - ii * HB;
      const int rr = fdiv(q, HW2, inv_hw2);
      const int hh = h0 - p.PT + rr, ww = w0 - p.PL + (q - rr * HW2);
      const bool ok = r < hrows && img + ii < nimg && unsigned(hh) < unsigned(H) && unsigned(ww) < unsigned(W);
      const uint32_t kh = uint32_t(((lane & 7) ^ halo_key(ii * TH * TW + rr * TW + (q - rr * HW2))) * 8);
      const uint32_t off = ok ? (uint32_t(((img + ii) * H + hh) * W + ww) * uint32_t(C) + kh) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_ptr_t)(dst + (wid * G::HPW + j) * 1024), 16, off, 0, 0, 0);
    }
  };

  // ---- consumer fragment rows (tile-invariant): output pixel -> halo row, swizzle key
  int hrow0[G::TM], kpx0[G::TM];
#pragma unroll
  for (int i = 0; i < G::TM; ++i) {
    const int px = wm * G::WM + i * 16 + fr;
    const int ii = px / (TH * TW), p2 = px - ii * (TH * TW);
    const int ph = p2 / TW;
    hrow0[i] = px < TI * TH * TW ? ii * HB + ph * HW2 + (p2 - ph * TW) : 0;
    kpx0[i] = px;
  }
  const uint32_t rb0 = uint32_t(((wn * G::WN + fr) * KT + ((fq ^ (fr & 7)) * 8)) * 2);
  const uint32_t rb1 = uint32_t(((wn * G::WN + fr) * KT + (((4 + fq) ^ (fr & 7)) * 8)) * 2);
  // epilogue store rows of this thread (tile-invariant): chunk c = tid + it * NT
  constexpr int CPRB = BN / 8;
  uint16_t* const Cb = reinterpret_cast<uint16_t*>(smem + G::OFF_STG);

  int t = blockIdx.x;
  if (t < ntiles) issue_halo(t, 0);
  for (int k = 0; t < ntiles; t += gridDim.x, ++k) {
    const int b = k & 1;
    // tile t's halo (and, on the first tile, the filter) landed; the previous
    // tile's kStores stores stay in flight
    if (k == 0) gemm::wait_vmcnt<0>();
    else gemm::wait_vmcnt<G::kStores>();
    gemm::lds_barrier();   // every wave's DMAs landed; halo buffer b^1 and the staging tile are read-free
    const int tn = t + gridDim.x;
    if (tn < ntiles) issue_halo(tn, b ^ 1);
    __builtin_amdgcn_sched_barrier(0);

    f32x4 acc[G::TM][G::TN];
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int j = 0; j < G::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* hb = smem + G::OFF_HALO + b * G::HALO_B;
    // the nine taps, software-pipelined: tap u + 1's fragment reads are issued
    // ahead of tap u's MFMAs (pinned by sched_barrier), so the LDS latency of a
    // tap runs under the previous tap's matrix work
    struct TapFrags {
      bf16x8 a[2][G::TM], b[2][G::TN];
    };
    auto load_tap = [&](TapFrags& f, int u) __attribute__((always_inline)) {
      const int tap_off = (u / 3) * HW2 + (u % 3), tap_key = (u / 3) * TW + (u % 3);
      const char* sb = smem + u * G::B_B;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < G::TM; ++i) {
          const int hr = hrow0[i] + tap_off;
          const uint32_t addr = uint32_t(hr) * 128u + ((uint32_t((kk * 4 + fq) ^ halo_key(kpx0[i] + tap_key))) << 4);
          f.a[kk][i] = *reinterpret_cast<const bf16x8*>(hb + addr);
        }
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
          f.b[kk][j] = *reinterpret_cast<const bf16x8*>(sb + (kk ? rb1 : rb0) + j * 16 * KT * 2);
      }
    };
    TapFrags fr2[2];
    load_tap(fr2[0], 0);
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      __builtin_amdgcn_sched_barrier(0);
      if (u < 8) load_tap(fr2[(u + 1) & 1], u + 1);
      __builtin_amdgcn_sched_barrier(0);
      const TapFrags& f = fr2[u & 1];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < G::TM; ++i)
#pragma unroll
          for (int j = 0; j < G::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[kk][i], f.b[kk][j], acc[i][j], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- epilogue: bias + act -> bf16 staging -> 16-B buffer stores
    auto stage = [&](auto act_tag) __attribute__((always_inline)) {
      constexpr int ACT = decltype(act_tag)::value;
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = act_fn<ACT>(acc[i][j][r] * alpha + bj[j] + 0.f);
            Cb[(wm * G::WM + i * 16 + fq * 4 + r) * G::CB_LD + wn * G::WN + j * 16 + fr] =
                __builtin_bit_cast(uint16_t, static_cast<__bf16>(v));
          }
    };
    switch (p.act) {
      case kActRelu: stage(std::integral_constant<int, kActRelu>{}); break;
      case kActGeluTanh: stage(std::integral_constant<int, kActGeluTanh>{}); break;
      case kActTanh: stage(std::integral_constant<int, kActTanh>{}); break;
      default: stage(std::integral_constant<int, kActNone>{}); break;
    }
    gemm::lds_barrier();
    {
      int r_ = t;
      const int tw = r_ % tpw;
      r_ /= tpw;
      const int th = r_ % tph;
      const int img = (r_ / tph) * TI;
      const int h0 = th * TH, w0 = tw * TW;
#pragma unroll
      for (int it = 0; it < G::kStores; ++it) {
        const int c = tid + it * G::NT, row = c / CPRB, ch = c - row * CPRB;
        int m = -1;
        if (row < TI * TH * TW) {
          const int ii = row / (TH * TW), r2 = row - ii * (TH * TW);
          const int ph = r2 / TW, pw = r2 - ph * TW;
          const int h = h0 + ph, w = w0 + pw;
          if (h < Ho && w < Wo && img + ii < nimg) m = ((img + ii) * Ho + h) * Wo + w;
        }
        const uint32_t off = m >= 0 ? (uint32_t(m) * uint32_t(p.ldc) + uint32_t(ch * 8)) * 2u : kOOB;
        const u32x4 v = *reinterpret_cast<const u32x4*>(Cb + row * G::CB_LD + ch * 8);
        __builtin_amdgcn_raw_buffer_store_b128(v, rsO, off, 0, 0);
      }
    }
  }
  gemm::wait_vmcnt<0>();
}

// (the ping-pong halo kernel, ids 144/145, was removed in round 6: 0 picks in
// the round-6 tile tables, slower than halo_conv_kernel on every ResNet-50
// 3x3 layer -- profiles/round6/r6f/conv.log; it stays in git history)


// Output block (TH, TW) for a BM-pixel tile whose halo fits HR rows: fewest
// tiles first, then the smallest halo (least re-read input).
bool pick_block(int Ho, int Wo, int BM, int HR, int& TH, int& TW) {
  long best_tiles = -1, best_halo = 0;
  for (int tw = 1; tw <= Wo; ++tw) {
    int th = BM / tw < Ho ? BM / tw : Ho;
    while (th >= 1 && (th + 2) * (tw + 2) > HR) --th;
    if (th < 1) continue;
    // the same tile counts with balanced blocks (9 + 5 rows -> 7 + 7): a
    // smaller halo and no mostly-empty last row of tiles
    const int nh = (Ho + th - 1) / th, nw = (Wo + tw - 1) / tw;
    const int bh = (Ho + nh - 1) / nh, bw = (Wo + nw - 1) / nw;
    const long tiles = long(nh) * nw;
    const long halo = long(bh + 2) * (bw + 2);
    if (best_tiles < 0 || tiles < best_tiles || (tiles == best_tiles && halo < best_halo)) {
      best_tiles = tiles;
      best_halo = halo;
      TH = bh;
      TW = bw;
    }
  }
  return best_tiles > 0;
}

// Whole images per tile when one image's output block and halo fit BM / HR
// several times (7x7 and 14x14 maps): the tile's weight stream then serves TI
// images, cutting the layer's weight traffic (= M-tiles x weights) by TI; the
// launcher's split-K restores the workgroup count.  1 otherwise.
int pick_images(const IGemmArgs& a, int BM, int HR) {
  if (a.TH != a.Ho || a.TW != a.Wo) return 1;
  const int nimg = a.M / (a.Ho * a.Wo);
  int ti = std::min(BM / (a.Ho * a.Wo), HR / ((a.Ho + 2) * (a.Wo + 2)));
  ti = std::min(ti, nimg);
  return ti > 1 ? ti : 1;
}

template <int BM, int BN, int WGM, int WGN, int HR, int S, bool PF = false>
hipError_t launch_halo_cfg(const IGemmArgs& a0, hipStream_t s) {
  using G = HG<BM, BN, WGM, WGN, HR, S>;
  IGemmArgs a = a0;
  a.epi_f32 = epi_f32_env();
  if (!pick_block(a.Ho, a.Wo, BM, HR, a.TH, a.TW)) return hipErrorInvalidValue;
  a.TI = pick_images(a, BM, HR);
  const int nch = a.C / KT;
  const int splits = a.splits > 1 ? a.splits : 1;
  if (splits > 1 && a.kt_per_split <= 0) return hipErrorInvalidValue;
  const int per = splits > 1 ? a.kt_per_split : nch;
  const int nimg = a.M / (a.Ho * a.Wo);
  const long tiles = long((nimg + a.TI - 1) / a.TI) * ((a.Ho + a.TH - 1) / a.TH) * ((a.Wo + a.TW - 1) / a.TW) *
                     ((a.N + BN - 1) / BN);
  if (tiles == 0) return hipSuccess;
  if (tiles >= (1L << 31)) return hipErrorInvalidValue;
  const int lds = G::lds(per > 1 ? 2 : 1);
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&halo_conv_kernel<BM, BN, WGM, WGN, HR, S, PF>), G::lds(2));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((halo_conv_kernel<BM, BN, WGM, WGN, HR, S, PF>), dim3(unsigned(tiles), splits), dim3(G::NT), lds, s,
                     a);
  return hipGetLastError();
}

hipError_t launch_halo_persist(const IGemmArgs& a0, hipStream_t s) {
  using G = HPs;
  IGemmArgs a = a0;
  // the configuration it is built for: one 64-channel chunk, 64 output
  // channels, plain bf16 output (see halo_persist_kernel)
  if (a.C != KT || a.N != G::BN || a.splits > 1 || a.residual != nullptr || a.out2 != nullptr || a.out_f32 ||
      a.out == nullptr || a.act == kActGeluErf || epi_f32_env() || a.counters != nullptr || a.ldc % 8)
    return hipErrorInvalidValue;
  if (long(a.M) * a.ldc * 2 >= 0x7fffffffL) return hipErrorInvalidValue;
  if (!pick_block(a.Ho, a.Wo, G::BM, G::HR, a.TH, a.TW)) return hipErrorInvalidValue;
  a.TI = pick_images(a, G::BM, G::HR);
  const int nimg = a.M / (a.Ho * a.Wo);
  const long tiles = long((nimg + a.TI - 1) / a.TI) * ((a.Ho + a.TH - 1) / a.TH) * ((a.Wo + a.TW - 1) / a.TW);
  if (tiles == 0) return hipSuccess;
  if (tiles >= (1L << 30)) return hipErrorInvalidValue;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || n <= 0)
      n = 256;
    cus = n;
  }
  const int grid = int(tiles < cus ? tiles : cus);
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&halo_persist_kernel), G::LDS);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(halo_persist_kernel, dim3(unsigned(grid)), dim3(G::NT), G::LDS, s, a, int(tiles));
  return hipGetLastError();
}

// per config index (halo_cfg_index)
constexpr int kHBM[kNumHaloConfigs] = {256, 128, 128, 64, 256, 64, 64, 128, 256, 128, 128};
constexpr int kHBN[kNumHaloConfigs] = {64, 128, 64, 64, 128, 128, 64, 64, 64, 64, 64};
constexpr int kHHR[kNumHaloConfigs] = {320, 192, 192, 128, 320, 128, 128, 192, 320, 192, 192};     // halo rows (HR)

int halo_cfg_index(int cfg) {
  if (cfg >= kHaloCfgBase && cfg < kHaloCfgBase + kNumHaloConfigs) return cfg - kHaloCfgBase;
  if (cfg >= kHaloPfCfgBase && cfg < kHaloPfCfgBase + kNumHaloConfigs) return cfg - kHaloPfCfgBase;
  return -1;
}

}  // namespace

long halo_tiles(const IGemmArgs& a0, int cfg) {
  IGemmArgs a = a0;
  a.epi_f32 = epi_f32_env();
  if (cfg == kHaloPersistCfg) return 0;   // no split-K (no fixup counters)
  const int c = halo_cfg_index(cfg);
  if (c < 0) return 0;
  if (!pick_block(a.Ho, a.Wo, kHBM[c], kHHR[c], a.TH, a.TW)) return 0;
  const int nimg = a.M / (a.Ho * a.Wo);
  const int ti = pick_images(a, kHBM[c], kHHR[c]);
  return long((nimg + ti - 1) / ti) * ((a.Ho + a.TH - 1) / a.TH) * ((a.Wo + a.TW - 1) / a.TW) *
         ((a.N + kHBN[c] - 1) / kHBN[c]);
}

bool halo_supported(const IGemmArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.SH == 1 && a.SW == 1 && a.C % KT == 0 && a.K == 9 * a.C && a.ldb >= a.K &&
         a.ldb % 8 == 0 && a.N % 8 == 0 && a.ldc % 8 == 0 && (!a.residual || a.ldr % 8 == 0) && a.PT >= 0 &&
         a.PT <= 2 && a.PL >= 0 && a.PL <= 2 && a.Ho > 0 && a.Wo > 0 && a.M % (a.Ho * a.Wo) == 0 &&
         a.M < (1 << 23) && int64_t(a.M / (a.Ho * a.Wo)) * a.H * a.W * a.C < (1LL << 30);
}

int halo_config_bm(int cfg) { return cfg == kHaloPersistCfg ? kPersistBM : kHBM[halo_cfg_index(cfg)]; }
int halo_config_bn(int cfg) { return cfg == kHaloPersistCfg ? kPersistBN : kHBN[halo_cfg_index(cfg)]; }

hipError_t halo_launch(const IGemmArgs& a, int cfg, hipStream_t s) {
  if (!halo_cfg_id(cfg) || !halo_supported(a)) return hipErrorInvalidValue;
  if (cfg == kHaloPersistCfg) return launch_halo_persist(a, s);
  if (cfg >= kHaloPfCfgBase) {
    switch (halo_cfg_index(cfg)) {   // the same tiles with the fragment-prefetch step pipeline
      case 0: return launch_halo_cfg<256, 64, 4, 1, 320, 3, true>(a, s);
      case 1: return launch_halo_cfg<128, 128, 2, 2, 192, 3, true>(a, s);
      case 2: return launch_halo_cfg<128, 64, 2, 2, 192, 3, true>(a, s);
      case 3: return launch_halo_cfg<64, 64, 2, 2, 128, 3, true>(a, s);
      // (4: the 8-wave 256 x 128 tile spills with two fragment sets; not built)
      case 5: return launch_halo_cfg<64, 128, 2, 2, 128, 3, true>(a, s);
      case 6: return launch_halo_cfg<64, 64, 2, 2, 128, 9, true>(a, s);
      case 7: return launch_halo_cfg<128, 64, 2, 2, 192, 9, true>(a, s);
      case 8: return launch_halo_cfg<256, 64, 4, 1, 320, 9, true>(a, s);
      case 9: return launch_halo_cfg<128, 64, 4, 2, 192, 3, true>(a, s);
      case 10: return launch_halo_cfg<128, 64, 4, 2, 192, 9, true>(a, s);
      default: return hipErrorInvalidValue;
    }
  }
  switch (halo_cfg_index(cfg)) {
    // LDS = 2 halo buffers (HR x 128 B; one when C == 64) + S B slots (BN x 128 B)
    case 0: return launch_halo_cfg<256, 64, 4, 1, 320, 3>(a, s);    // 104 KB (64 KB for C == 64), waves 64x64
    case 1: return launch_halo_cfg<128, 128, 2, 2, 192, 3>(a, s);   // 96 KB, waves 64x64
    case 2: return launch_halo_cfg<128, 64, 2, 2, 192, 3>(a, s);    // 72 KB (48 KB), waves 64x32
    case 3: return launch_halo_cfg<64, 64, 2, 2, 128, 3>(a, s);     // 56 KB (40 KB), waves 32x32
    case 4: return launch_halo_cfg<256, 128, 4, 2, 320, 3>(a, s);   // 135 KB, 8 waves of 64x64
    case 5: return launch_halo_cfg<64, 128, 2, 2, 128, 3>(a, s);    // 80 KB, waves 32x64
    // 9-slot rings: 8 weight tiles in flight (16 x 1-KB DMAs per wave)
    case 6: return launch_halo_cfg<64, 64, 2, 2, 128, 9>(a, s);     // 104 KB, waves 32x32
    case 7: return launch_halo_cfg<128, 64, 2, 2, 192, 9>(a, s);    // 120 KB, waves 64x32
    case 8: return launch_halo_cfg<256, 64, 4, 1, 320, 9>(a, s);    // 152 KB, waves 64x64
    // 8 waves of 32x32 on the 128 x 64 tile: two waves per SIMD where the
    // 4-wave build waits 40 % of its cycles (the stage-2 / 3 3x3 convs,
    // profiles/round4/s5/pmc_r50_b32_mfma.txt)
    case 9: return launch_halo_cfg<128, 64, 4, 2, 192, 3>(a, s);    // 72 KB
    case 10: return launch_halo_cfg<128, 64, 4, 2, 192, 9>(a, s);   // 120 KB
    default: return hipErrorInvalidValue;
  }
}

}  // namespace tfsk
