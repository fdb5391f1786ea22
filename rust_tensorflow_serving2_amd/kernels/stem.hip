// ResNet stem in ONE kernel: fp32 RGB request -> 7x7/2 conv (+folded BN, act)
// -> 3x3/2 max pool (+ optional folded BN/act after the max, ResNet v2).
//
// The unfused path ran three launches and moved the 112x112x64 conv output
// through memory twice (b32: ingest 12.4 us + stem cgemm 34.6 us + maxpool
// 17.7 us, profiles/round2/r50_b32_replay_head_halo9.txt).  Here a workgroup
// owns a 4 x 8 tile of POOLED outputs: it computes the 9 x 17 conv pixels
// under that tile's pooling windows (1.2x recompute of the shared border),
// keeps them in LDS, and writes only the pooled tile.
//
//   * input patch: the 23 x 40 fp32 pixels under those conv windows, read
//     straight from the request tensor (out-of-image -> 0, the conv's zero
//     padding), cast to bf16 and padded to 4 channels in LDS (8 B / pixel);
//   * the K order is [kh][kw (7 -> 8, tap 7 has zero weight)][4 ch], so one
//     32-deep MFMA k-step is one filter row and a lane's 8 k-values are two
//     horizontally adjacent pixels: one 16-B LDS read per A fragment;
//   * weights (<= 64 x 224 bf16) live in registers for the workgroup's whole
//     life: the grid is persistent (<= 2 workgroups per CU), each workgroup
//     walks a contiguous run of tiles and prefetches the next tile's patch
//     into registers while its MFMAs run;
//   * waves split the 10 row groups of 16 conv pixels (3/3/2/2) and each
//     computes all output channels, so a patch fragment is read from LDS once
//     per use by 1-4 MFMAs;
//   * C = W x patch^T: a lane's accumulator is 4 consecutive channels of one
//     pixel, stored to LDS packed (v_cvt_pk_bf16_f32) as order-preserving
//     int16 keys, so the 3x3 max runs as packed v_pk_max_i16 (the first
//     version's per-value conversions / stores made it VALU-issue bound:
//     62 us at b32);
//   * conv pixels outside the conv's output range are stored as -inf, so the
//     pooling max ignores them (TF SAME/VALID pooling semantics).
//
// The op replaces _FusedConv2D(7x7/2, C <= 4) -> _MaxPool(3x3/2) in the graph
// (graph/fused.py fuse_stem_pool); the model is the one the reference serves
// (/root/reference/serving/fetch.sh:7, resnet_v2_fp32_savedmodel_NHWC) and the
// request tensor is the one its client sends (src/lib.rs:229-257).
#include "common.h"
#include "launch.h"

namespace tfsk {
namespace {

constexpr int kTPY = 4, kTPX = 8;                   // pooled tile
constexpr int kCR = 2 * kTPY + 1, kCC = 2 * kTPX + 1;  // conv pixels under it: 9 x 17
constexpr int kNPix = kCR * kCC;                    // 153
constexpr int kNRG = (kNPix + 15) / 16;             // 10 row groups of 16
constexpr int kIR = 2 * (kCR - 1) + 7;              // 23 input rows
constexpr int kIC = 2 * (kCC - 1) + 8;              // 40 input cols (tap 7 is padding)
constexpr int kPatch = kIR * kIC;                   // 920 pixels
constexpr int kSlots = (kPatch + 255) / 256;        // 4 per thread
constexpr int kKSteps = 7;                          // filter rows

struct StemArgs {
  const void* x;        // [N][H][W][C] fp32, or bf16 (XB16: converted on ingest, csrc/ingest.h)
  const uint16_t* w;    // [Cout][ldw] bf16, k = kh*32 + kw*4 + c
  const float* bias;    // [Cout]
  uint16_t* y;          // [N][Hp][Wp][Cout] bf16
  const float* pscale;  // optional [Cout] (after the max)
  const float* pshift;
  int N, H, W, C, ldw;
  int pt, pl, Hc, Wc;   // conv padding (top / left) and output size
  int ppt, ppl, Hp, Wp; // pool padding (top / left) and output size
  int tiles_y, tiles_x, tiles;
  float lo, plo;        // activation as a floor: 0 (ReLU) or -inf (none)
  int dbg;              // profiling ablations (TFSK_STEM_DBG; 0 in production)
};

typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) short s16x2;

// two f32 -> packed bf16 (v_cvt_pk_bf16_f32, round-to-nearest-even)
__device__ __forceinline__ uint32_t cvt2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
// order-preserving bf16 <-> int16 key (self-inverse): negative values get
// their magnitude bits flipped, so a signed 16-bit max is the float max and
// the pool runs on packed v_pk_max_i16 (two channels per instruction)
__device__ __forceinline__ uint32_t okey(uint32_t u) {
  const s16x2 v = __builtin_bit_cast(s16x2, u);
  return __builtin_bit_cast(uint32_t, v ^ ((v >> 15) & (s16x2){0x7fff, 0x7fff}));
}
// key pair of two bf16 -inf (0xff80): what conv pixels outside the output hold
constexpr uint32_t kNegInfKey2 = 0x807f807fu;
__device__ __forceinline__ uint32_t kmax(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2, a),
                                                                __builtin_bit_cast(s16x2, b)));
}

// s_waitcnt vmcnt(N) only (gfx9 encoding: expcnt / lgkmcnt at their maxima)
template <int N>
__device__ __forceinline__ void stem_wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ u32x4 make_u32x4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  u32x4 v;
  v.x = a; v.y = b; v.z = c; v.w = d;
  return v;
}

template <int NCG, bool XB16>
__global__ __launch_bounds__(256, 2) void stem_pool_kernel(StemArgs p) {
  constexpr int COUT = NCG * 16;
  constexpr int CS = COUT + 8;                      // conv tile row stride (halves), 16-B aligned rows
  __shared__ uint2 patch[kPatch];
  __shared__ __attribute__((aligned(16))) uint16_t ctile[kNRG * 16 * CS];   // rows >= 153: scratch

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar branches)
  const int fr = lane & 15, fq = lane >> 4;

  // ---- this workgroup's run of tiles (XCD-aware: neighbouring runs share an L2)
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int t_begin = int(long(wg) * p.tiles / gridDim.x);
  const int t_end = int(long(wg + 1) * p.tiles / gridDim.x);
  if (t_begin >= t_end) return;

  // ---- this lane's conv pixel in each of the wave's row groups (B operand
  // columns); pixels past 153 clamp their reads and store to scratch rows
  constexpr int kRGW = (kNRG + 3) / 4;              // row groups per wave (max)
  int aoff[kRGW], pcy[kRGW], pcx[kRGW];
#pragma unroll
  for (int i = 0; i < kRGW; ++i) {
    const int px = min((wid + 4 * i) * 16 + fr, kNPix - 1);
    pcy[i] = px / kCC;
    pcx[i] = px - pcy[i] * kCC;
    aoff[i] = 2 * pcy[i] * kIC + 2 * pcx[i] + 2 * fq;
  }

  // request tensor as a buffer resource: an out-of-image pixel or a channel
  // >= C reads through an out-of-range offset and gets the conv's zero padding
  // from the hardware.  (The first version loaded through plain pointers and
  // selected afterwards; hipcc turned that into per-slot conditional blocks
  // that waited for their loads on the spot, so the "prefetch" of the next
  // tile's patch was serial memory round trips: b32 47.5 -> 38.5 us in graph
  // replay with this form.  Ablations after the change, b32 eager 35.5 us:
  // without the loads 30.1, the MFMAs 26.5, the pool 31.6, the conv-tile
  // stores 30.0, all four 12.6 -- profiles/round2/stem_ablate.log)
  // A bf16 request (rounded on ingest exactly as cvt2 rounds below) is read
  // as the two aligned dwords covering the pixel's channels -- 2 loads per
  // pixel instead of one per channel -- and its bf16 halves are staged as
  // they are: the same patch bits as the fp32 path.  (The record count is
  // rounded up to whole dwords: with an odd element count the last pixel's
  // second dword runs 2 B past the tensor; the binding requires the storage to
  // extend that far -- bindings.cpp stem_pool.)
  constexpr uint32_t kEsz = XB16 ? 2u : 4u;
  const long xbytes = long(p.N) * p.H * p.W * p.C * kEsz;
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(p.x), 0, int(XB16 ? (xbytes + 3) & ~3L : xbytes), 0x00020000);
  constexpr uint32_t kOff = 0x80000000u;
  float pf[XB16 ? 1 : kSlots][4] = {};
  uint32_t pv[XB16 ? kSlots : 1][2] = {};
  uint32_t podd[XB16 ? kSlots : 1] = {};
  auto load_patch = [&](int t) {
    const int n = t / (p.tiles_y * p.tiles_x);
    const int rem = t - n * p.tiles_y * p.tiles_x;
    const int ty = rem / p.tiles_x, tx = rem - ty * p.tiles_x;
    const int iy0 = 2 * (2 * ty * kTPY - p.ppt) - p.pt;
    const int ix0 = 2 * (2 * tx * kTPX - p.ppl) - p.pl;
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      const int q = tid + s * 256;
      const int r = q / kIC, c = q - r * kIC;
      const int gy = iy0 + r, gx = ix0 + c;
      const bool ok = q < kPatch && (unsigned)gy < (unsigned)p.H && (unsigned)gx < (unsigned)p.W;
      if constexpr (XB16) {
        const uint32_t e0 = uint32_t(((n * p.H + gy) * p.W + gx) * p.C);
        const uint32_t base = (e0 & ~1u) * 2u;
        pv[s][0] = __builtin_amdgcn_raw_buffer_load_b32(rsX, ok ? base : kOff, 0, 0);
        pv[s][1] = __builtin_amdgcn_raw_buffer_load_b32(rsX, ok ? base + 4u : kOff, 0, 0);
        podd[s] = e0 & 1u;
      } else {
        const uint32_t pix = uint32_t(((n * p.H + gy) * p.W + gx) * p.C) * kEsz;
#pragma unroll
        for (int ch = 0; ch < 4; ++ch) {
          const uint32_t voff = ok && ch < p.C ? pix + uint32_t(ch) * kEsz : kOff;
          pf[s][ch] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsX, voff, 0, 0));
        }
      }
    }
  };

  // ablations (timing only, results are garbage): bit 0 skips the patch
  // loads, bit 1 the MFMAs, bit 2 the pool phase, bit 3 the conv-tile stores
  const int dbg = p.dbg;
  // the conv activation's floor as a packed key pair (ReLU: +0 -> key 0;
  // none: -inf -> the smallest key, a no-op under the max)
  const uint32_t lokey = okey(cvt2(p.lo, p.lo));
  // pooled-tile stores: with COUT = 64 every thread stores exactly SPT 16-B
  // items per tile (out-of-range items to an out-of-range offset: dropped), so
  // the next tile's patch wait is an exact vmcnt(SPT) -- the stores stay in
  // flight.  (vmcnt counts stores too on gfx950: the plain vmcnt(0) there
  // waited for the previous tile's write acknowledgements every tile.)
  constexpr int C8 = COUT / 8;
  constexpr int kItems = kTPY * kTPX * C8;
  constexpr bool kExactStores = kItems % 256 == 0;
  constexpr int SPT = kItems / 256;
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(
      p.y, 0, int(long(p.N) * p.Hp * p.Wp * COUT * 2), 0x00020000);
  if (!(dbg & 1)) load_patch(t_begin);
  // ---- weights (MFMA A operand: rows = output channels) and bias in registers
  // for the whole run.  C = W x patch^T, so a lane's accumulator holds 4
  // CONSECUTIVE channels of one conv pixel: one packed 8-B LDS store each.
  bf16x8 wf[kKSteps][NCG];
  float4 bias[NCG];
#pragma unroll
  for (int j = 0; j < NCG; ++j) {
    const uint16_t* wr = p.w + long(j * 16 + fr) * p.ldw + fq * 8;
#pragma unroll
    for (int kh = 0; kh < kKSteps; ++kh) wf[kh][j] = *reinterpret_cast<const bf16x8*>(wr + kh * 32);
    bias[j] = *reinterpret_cast<const float4*>(p.bias + j * 16 + fq * 4);
  }

  // the weights, the bias and the first patch, one round trip; the explicit
  // wait also tells the compiler's wait-count pass that the weight / bias
  // registers are complete.  (Without it the loop body waited for them --
  // vmcnt(4) in the MFMAs, vmcnt(0) in the epilogue -- and so for most of the
  // next tile's patch prefetch, every tile.)
  stem_wait_vmcnt<0>();
  for (int t = t_begin; t < t_end; ++t) {
    // ---- stage the prefetched patch (the previous tile's MFMA reads ended at
    // its post-epilogue barrier)
    if constexpr (kExactStores) {
      if (t == t_begin) stem_wait_vmcnt<0>();
      else stem_wait_vmcnt<SPT>();
    }
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
      const int q = tid + s * 256;
      if constexpr (XB16) {
        // halves h0..h3 cover elements (e0 & ~1) .. +3: channels start at h[odd]
        const uint64_t v = (uint64_t(pv[s][1]) << 32) | pv[s][0];
        uint64_t c4 = v >> (16 * podd[s]);
        c4 &= p.C >= 4 ? ~0ull : (1ull << (16 * p.C)) - 1ull;      // channels >= C are zero
        if (q < kPatch) patch[q] = make_uint2(uint32_t(c4), uint32_t(c4 >> 32));
      } else {
        if (q < kPatch) patch[q] = make_uint2(cvt2(pf[s][0], pf[s][1]), cvt2(pf[s][2], pf[s][3]));
      }
    }
    __syncthreads();
    if (t + 1 < t_end && !(dbg & 1)) load_patch(t + 1);   // in flight during the MFMAs

    // ---- conv: 7 k-steps x (2-3 row groups) x NCG channel groups
    f32x4 acc[kRGW][NCG];
#pragma unroll
    for (int i = 0; i < kRGW; ++i)
#pragma unroll
      for (int j = 0; j < NCG; ++j) acc[i][j] = f32x4{bias[j].x, bias[j].y, bias[j].z, bias[j].w};   // bias in the accumulator
    const char* pb = reinterpret_cast<const char*>(patch);
    // patch fragments read one filter row ahead, unconditionally (a wave's
    // missing third row group reads a clamped pixel, never used): with the
    // read inside each group's wave-uniform branch every group waited
    // lgkmcnt(0) for its own read, 21 LDS round trips per tile
    bf16x8 afr[2][kRGW];
#pragma unroll
    for (int i = 0; i < kRGW; ++i) afr[0][i] = *reinterpret_cast<const bf16x8*>(pb + size_t(aoff[i]) * 8);
#pragma unroll
    for (int kh = 0; kh < kKSteps; ++kh) {
      if (kh + 1 < kKSteps) {
#pragma unroll
        for (int i = 0; i < kRGW; ++i)
          afr[(kh + 1) & 1][i] = *reinterpret_cast<const bf16x8*>(pb + size_t(aoff[i] + (kh + 1) * kIC) * 8);
      }
#pragma unroll
      for (int i = 0; i < kRGW; ++i) {
        if (wid + 4 * i >= kNRG || (dbg & 2)) continue;   // wave-uniform
#pragma unroll
        for (int j = 0; j < NCG; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kh][j], afr[kh & 1][i], acc[i][j], 0, 0, 0);
      }
    }

    // ---- epilogue -> LDS conv tile as order keys (bias, act; outside the
    // conv output: -inf)
    const int n = t / (p.tiles_y * p.tiles_x);
    const int rem = t - n * p.tiles_y * p.tiles_x;
    const int ty = rem / p.tiles_x, tx = rem - ty * p.tiles_x;
    const int cy0 = 2 * ty * kTPY - p.ppt, cx0 = 2 * tx * kTPX - p.ppl;
#pragma unroll
    for (int i = 0; i < kRGW; ++i) {
      if (wid + 4 * i >= kNRG || (dbg & 8)) continue;
      const int px = (wid + 4 * i) * 16 + fr;
      const bool in = (unsigned)(cy0 + pcy[i]) < (unsigned)p.Hc && (unsigned)(cx0 + pcx[i]) < (unsigned)p.Wc;
#pragma unroll
      for (int j = 0; j < NCG; ++j) {
        // keys of the biased conv values; -inf keys outside the conv output.
        // The activation floor is applied after the max (max and ReLU
        // commute; bf16 rounding is monotonic): ~10 fewer VALU ops per 4 values
        const uint32_t k01 = okey(cvt2(acc[i][j][0], acc[i][j][1]));
        const uint32_t k23 = okey(cvt2(acc[i][j][2], acc[i][j][3]));
        *reinterpret_cast<uint2*>(ctile + px * CS + j * 16 + fq * 4) =
            make_uint2(in ? k01 : kNegInfKey2, in ? k23 : kNegInfKey2);
      }
    }
    __syncthreads();

    // ---- 3x3/2 max over the conv tile -> pooled tile (16 B = 8 channels per
    // item).  Pooled column fastest across lanes: neighbouring lanes read conv
    // pixels 2 apart (288 B = bank offset 8 for COUT 64), so 8 lanes x 16 B
    // cover all 64 banks; channel-chunk-fastest order had 2-way conflicts
    // (SQ_LDS_BANK_CONFLICT 2.1M cycles per launch at b32)
    auto pool_item = [&](int idx, bool out_ok, int qx, int c8, int qy, int py, int px) {
      const uint16_t* c0 = ctile + (2 * qy * kCC + 2 * qx) * CS + c8 * 8;
      uint4 m = *reinterpret_cast<const uint4*>(c0);
#pragma unroll
      for (int tap = 1; tap < 9; ++tap) {
        const uint4 v = *reinterpret_cast<const uint4*>(c0 + ((tap / 3) * kCC + tap % 3) * CS);
        m = make_uint4(kmax(m.x, v.x), kmax(m.y, v.y), kmax(m.z, v.z), kmax(m.w, v.w));
      }
      m = make_uint4(kmax(m.x, lokey), kmax(m.y, lokey), kmax(m.z, lokey), kmax(m.w, lokey));   // the conv's act
      uint32_t o[4] = {okey(m.x), okey(m.y), okey(m.z), okey(m.w)};
      if (p.pscale) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = c8 * 8 + 2 * e;
          const float lo = fmaxf(__uint_as_float(o[e] << 16) * p.pscale[c] + p.pshift[c], p.plo);
          const float hi = fmaxf(__uint_as_float(o[e] & 0xffff0000u) * p.pscale[c + 1] + p.pshift[c + 1], p.plo);
          o[e] = cvt2(lo, hi);
        }
      }
      if constexpr (kExactStores) {
        const uint32_t yoff = out_ok ? uint32_t(((long(n) * p.Hp + py) * p.Wp + px) * COUT + c8 * 8) * 2u : kOff;
        __builtin_amdgcn_raw_buffer_store_b128(make_u32x4(o[0], o[1], o[2], o[3]), rsY, yoff, 0, 0);
      } else {
        *reinterpret_cast<uint4*>(p.y + ((long(n) * p.Hp + py) * p.Wp + px) * COUT + c8 * 8) =
            make_uint4(o[0], o[1], o[2], o[3]);
      }
    };
    if constexpr (kExactStores) {
      // exactly SPT items per thread, no branch around the stores (the wait
      // count above relies on it; TFSK_STEM_DBG bit 2 does not apply here)
#pragma unroll
      for (int it = 0; it < SPT; ++it) {
        const int idx = tid + it * 256;
        const int qx = idx % kTPX, c8 = (idx / kTPX) % C8, qy = idx / (kTPX * C8);
        const int py = ty * kTPY + qy, px = tx * kTPX + qx;
        pool_item(idx, py < p.Hp && px < p.Wp, qx, c8, qy, py, px);
      }
    } else {
      for (int idx = tid; idx < kItems && !(dbg & 4); idx += 256) {
        const int qx = idx % kTPX, c8 = (idx / kTPX) % C8, qy = idx / (kTPX * C8);
        const int py = ty * kTPY + qy, px = tx * kTPX + qx;
        if (py >= p.Hp || px >= p.Wp) continue;
        pool_item(idx, true, qx, c8, qy, py, px);
      }
    }
    // the next iteration's barrier (after its patch store) orders these ctile
    // reads before its epilogue's writes
  }
}

int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;   // benign race: every writer stores the same value
  }
  return cached[dev];
}

}  // namespace

hipError_t stem_pool_launch(const void* x, bool x_bf16, const uint16_t* w, int ldw, const float* bias, uint16_t* y,
                            int N, int H, int W, int C, int cout, int pt, int pl, int Hc, int Wc, int ppt, int ppl,
                            int Hp, int Wp, int act, const float* pscale, const float* pshift, int pact,
                            hipStream_t s) {
  if (N <= 0 || Hp <= 0 || Wp <= 0) return hipSuccess;
  if (C < 1 || C > 4 || cout % 16 || cout < 16 || cout > 64 || ldw < kKSteps * 32 || ldw % 8 ||
      (pscale == nullptr) != (pshift == nullptr) || ppt < 0 || ppl < 0 || pt < 0 || pl < 0)
    return hipErrorInvalidValue;
  if (Hc <= 0 || Wc <= 0 || ppt > 2 || ppl > 2) return hipErrorInvalidValue;
  if ((act != kActNone && act != kActRelu) || (pact != kActNone && pact != kActRelu)) return hipErrorInvalidValue;
  StemArgs a{x, w, bias, y, pscale, pshift, N, H, W, C, ldw, pt, pl, Hc, Wc, ppt, ppl, Hp, Wp, 0, 0, 0,
             act == kActRelu ? 0.f : -INFINITY, pact == kActRelu ? 0.f : -INFINITY, 0};
  static const int dbg = [] {
    const char* e = getenv("TFSK_STEM_DBG");
    return e ? atoi(e) : 0;
  }();
  a.dbg = dbg;
  a.tiles_y = (Hp + kTPY - 1) / kTPY;
  a.tiles_x = (Wp + kTPX - 1) / kTPX;
  const long tiles = long(N) * a.tiles_y * a.tiles_x;
  if (tiles > (1L << 30)) return hipErrorInvalidValue;
  if (long(N) * H * W * C * (x_bf16 ? 2 : 4) >= 0x7fffffffL) return hipErrorInvalidValue;   // 32-bit buffer offsets
  if (long(N) * Hp * Wp * cout * 2 >= 0x7fffffffL) return hipErrorInvalidValue;
  a.tiles = int(tiles);
  const int grid = int(tiles < 2L * cu_count() ? tiles : 2L * cu_count());
  if (x_bf16) {
    switch (cout / 16) {
      case 1: hipLaunchKernelGGL((stem_pool_kernel<1, true>), dim3(grid), dim3(256), 0, s, a); break;
      case 2: hipLaunchKernelGGL((stem_pool_kernel<2, true>), dim3(grid), dim3(256), 0, s, a); break;
      case 3: hipLaunchKernelGGL((stem_pool_kernel<3, true>), dim3(grid), dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL((stem_pool_kernel<4, true>), dim3(grid), dim3(256), 0, s, a); break;
    }
  } else {
    switch (cout / 16) {
      case 1: hipLaunchKernelGGL((stem_pool_kernel<1, false>), dim3(grid), dim3(256), 0, s, a); break;
      case 2: hipLaunchKernelGGL((stem_pool_kernel<2, false>), dim3(grid), dim3(256), 0, s, a); break;
      case 3: hipLaunchKernelGGL((stem_pool_kernel<3, false>), dim3(grid), dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL((stem_pool_kernel<4, false>), dim3(grid), dim3(256), 0, s, a); break;
    }
  }
  return hipGetLastError();
}

}  // namespace tfsk
