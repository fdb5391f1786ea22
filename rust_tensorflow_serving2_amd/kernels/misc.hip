// Memory-bound companion kernels (gfx950): pooling, classifier head, casts,
// LayerNorm, embedding+LN.  All bf16 traffic is 16-B vectorised (8 elements
// per lane), reductions are wave64 shuffles.
#include <type_traits>

#include "common.h"
#include "gemm_common.h"
#include "launch.h"

namespace tfsk {

namespace {

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = bf16_to_f32(uint16_t(w[e] & 0xffff));
    f[2 * e + 1] = bf16_to_f32(uint16_t(w[e] >> 16));
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint16_t b[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = f32_to_bf16(f[e]);
  return make_uint4(b[0] | (uint32_t(b[1]) << 16), b[2] | (uint32_t(b[3]) << 16),
                    b[4] | (uint32_t(b[5]) << 16), b[6] | (uint32_t(b[7]) << 16));
}

// ---------------------------------------------------------------- max pool
// One block row per output row (n, ho): threads cover that row's Wo * C/8
// 16-byte chunks, so the only per-thread index math is one 32-bit division by
// C/8 (the grid-stride version spent three 64-bit div/mods per output chunk,
// emulated in ~40 VALU ops each).  Rows beyond the grid's y extent loop.
__global__ __launch_bounds__(256) void maxpool_nhwc_kernel(const uint16_t* __restrict__ x,
                                                           uint16_t* __restrict__ y, int N, int H, int W,
                                                           int C, int KH, int KW, int SH, int SW, int PT,
                                                           int PL, int Ho, int Wo,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift, int act) {
  const int C8 = C / 8;
  const int row_items = Wo * C8;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= row_items) return;
  const int wo = j / C8;
  const int c8 = j - wo * C8;
  // optional folded BN (+ReLU) after the max: this thread's 8 channels are fixed
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale ? scale[c8 * 8 + e] : 1.f;
    sh[e] = scale ? shift[c8 * 8 + e] : 0.f;
  }
  for (int r = blockIdx.y; r < N * Ho; r += gridDim.y) {
    const int n = r / Ho;
    const int ho = r - n * Ho;
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    if (KH == 3 && KW == 3) {
      // the ResNet stem pool: all nine 16-B loads issued before any max (the
      // generic loop below has run-time trip counts, so its loads went out one
      // at a time, each paying the full latency); out-of-range taps load a
      // clamped in-range address and are masked
      uint4 v[9];
      bool ok[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int hi = ho * SH - PT + t / 3, wi = wo * SW - PL + t % 3;
        ok[t] = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
        const int hc = min(max(hi, 0), H - 1), wc = min(max(wi, 0), W - 1);
        v[t] = *reinterpret_cast<const uint4*>(x + ((long(n) * H + hc) * W + wc) * long(C) + c8 * 8);
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (!ok[t]) continue;
        float f[8];
        unpack8(v[t], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], f[e]);
      }
    } else
    for (int kh = 0; kh < KH; ++kh) {
      const int hi = ho * SH - PT + kh;
      if ((unsigned)hi >= (unsigned)H) continue;
      const uint16_t* xrow = x + (long(n) * H + hi) * long(W) * C + c8 * 8;
      for (int kw = 0; kw < KW; ++kw) {
        const int wi = wo * SW - PL + kw;
        if ((unsigned)wi >= (unsigned)W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(xrow + long(wi) * C), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], f[e]);
      }
    }
    if (scale) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        m[e] = m[e] * sc[e] + sh[e];
        if (act == kActRelu) m[e] = fmaxf(m[e], 0.f);
      }
    }
    *reinterpret_cast<uint4*>(y + (long(r) * Wo * C8 + j) * 8) = pack8(m);
  }
}

// ---------------------------------------------------------------- global avg pool
// Block = 4 waves on one (image, 512-channel chunk): lane owns 8 channels, the
// 4 waves split the HW positions (loads unrolled so several are in flight),
// partial sums meet in LDS.  N*C/512 blocks (e.g. 128 for ResNet-50 b32)
// instead of one serial 49-load chain per thread.
__global__ __launch_bounds__(256) void gap_nhwc_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                       int N, int HW, int C) {
  __shared__ float part[3][64][8];
  const int C8 = C / 8;
  const int chunks = (C8 + 63) / 64;
  const int n = blockIdx.x / chunks;
  const int c8 = (blockIdx.x - n * chunks) * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c8 < C8) {
    const uint16_t* p = x + long(n) * HW * C + c8 * 8;
#pragma unroll 4
    for (int h = w; h < HW; h += 4) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(p + long(h) * C), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += f[e];
    }
  }
  if (w > 0)
#pragma unroll
    for (int e = 0; e < 8; ++e) part[w - 1][threadIdx.x & 63][e] = s[e];
  __syncthreads();
  if (w == 0 && c8 < C8) {
    const float inv = 1.f / float(HW);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = (s[e] + part[0][threadIdx.x][e] + part[1][threadIdx.x][e] +
                                        part[2][threadIdx.x][e]) * inv;
    *reinterpret_cast<uint4*>(y + long(n) * C + c8 * 8) = pack8(s);
  }
}

// ---------------------------------------------------------------- softmax + argmax
// One 256-thread block per row: every logit is loaded exactly once into
// registers (up to 16 per thread, i.e. rows of <= 4096 classes stay in
// registers), max/argmax and the exp-sum are block reductions (wave shuffles
// + LDS).  ArgMax ties resolve to the smallest index (TF semantics).
// With `parts`, a logit is bias[c] + the sum of `nparts` split-K partial rows
// (parts[p * part_stride + row * ld + c]): the classifier head's reduction.
// PER = register-tile logits per thread: 4 for rows of <= 1024 classes (the
// ResNet head's 1001), so a thread issues 4 x (NPARTS + 1) loads instead of 16
// x (NPARTS + 1) mostly-clamped duplicates (80 loads > the 63 vmcnt slots at
// NPARTS = 4: the wave stalled on a second round trip).
constexpr int kSmPer = 16, kSmPerSmall = 4;
template <int NPARTS, int PER = kSmPer>
__global__ __launch_bounds__(256) void softmax_argmax_kernel(const void* __restrict__ logits, int in_bf16,
                                                             float* __restrict__ probs,
                                                             int64_t* __restrict__ classes, int rows, int cols,
                                                             long ld, const float* __restrict__ parts,
                                                             long part_stride, const float* __restrict__ bias) {
  __shared__ float smx[4];
  __shared__ int sarg[4];
  __shared__ float ssum[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (row >= rows) return;
  auto load = [&](int c) -> float {
    if constexpr (NPARTS > 0) {
      float a = bias[c];
      const float* q = parts + long(row) * ld + c;
#pragma unroll
      for (int p = 0; p < NPARTS; ++p) a += q[p * part_stride];
      return a;
    }
    return in_bf16 ? bf16_to_f32(static_cast<const uint16_t*>(logits)[long(row) * ld + c])
                   : static_cast<const float*>(logits)[long(row) * ld + c];
  };
  float v[PER];
  float mx = -INFINITY;
  int arg = 0x7fffffff;
  // every load of the register tile issued before any compare: unconditional
  // loads of clamped columns, masked afterwards (`if (c < cols) x = load(c)`
  // compiled to one conditional block per k that waited for its loads, i.e.
  // PER serial memory round trips per row)
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = k * 256 + tid;
    v[k] = load(c < cols ? c : cols - 1);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = k * 256 + tid;
    const float x = c < cols ? v[k] : -INFINITY;
    v[k] = x;
    if (c < cols && (x > mx || (x == mx && c < arg))) { mx = x; arg = c; }
  }
  // columns beyond the register tile (cols > 4096): strided tail, recomputed below
  for (int c = PER * 256 + tid; c < cols; c += 256) {
    const float x = load(c);
    if (x > mx || (x == mx && c < arg)) { mx = x; arg = c; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
  }
  if (lane == 0) { smx[w] = mx; sarg[w] = arg; }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float om = smx[k];
    const int oa = sarg[k];
    if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    v[k] = (k * 256 + tid < cols) ? __expf(v[k] - mx) : 0.f;
    s += v[k];
  }
  for (int c = PER * 256 + tid; c < cols; c += 256) s += __expf(load(c) - mx);
  s = wave_sum(s);
  if (lane == 0) ssum[w] = s;
  __syncthreads();
  const float inv = 1.f / (ssum[0] + ssum[1] + ssum[2] + ssum[3]);
  if (probs) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = k * 256 + tid;
      if (c < cols) probs[long(row) * cols + c] = v[k] * inv;
    }
    for (int c = PER * 256 + tid; c < cols; c += 256) probs[long(row) * cols + c] = __expf(load(c) - mx) * inv;
  }
  if (classes && tid == 0) classes[row] = arg;
}

// ---------------------------------------------------------------- classifier head
// GlobalAvgPool -> dense -> (softmax + argmax), the ResNet head, as three short
// launches that each fill the chip, instead of gap + a 16-workgroup GEMM with
// a 2048-deep serial K loop (17.6 us at b32) + softmax:
//   1. gap_rows: workgroup (row, 64-channel slice), 32 lane groups split the
//      HW positions (<= 2 loads per lane for 7x7), bf16 pooled rows [M][K];
//   2. fc_partial: workgroup (K slice, 32 columns), one v_mfma 16x16x32 tile
//      pair per 32 rows, operands straight from global (every load of the
//      slice in flight at once), 4 waves split the slice and meet in LDS ->
//      f32 partial rows [KS][M][Np];
//   3. softmax_argmax<KS> above: bias + the KS partials per logit.
// Deterministic (no atomics).  Measured on the way (b32, rocprofv3): a fused
// pool + 32-slice VALU version took 15 + 35 us, a VALU dot-product version
// 27 us (LDS-read bound) for the middle kernel.
constexpr int kHeadKS = 4, kHeadCols = 32;
__global__ __launch_bounds__(256) void gap_rows_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ pooled,
                                                       int HW, int K, float inv_hw) {
  __shared__ float part[32][8][9];
  const int m = blockIdx.x, k0 = blockIdx.y * 64;
  const int tid = threadIdx.x, cg = tid & 7, hs = tid >> 3;
  float s8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint16_t* p = x + long(m) * HW * K + k0 + cg * 8;
  // the first two positions of this lane group (all of them for HW <= 64,
  // e.g. ResNet's 7x7) load together from clamped rows, masked afterwards: the
  // rolled loop issued one load per trip and waited for it (2 serial round trips)
  {
    const uint4 v0 = *reinterpret_cast<const uint4*>(p + long(min(hs, HW - 1)) * K);
    const uint4 v1 = *reinterpret_cast<const uint4*>(p + long(min(hs + 32, HW - 1)) * K);
    __builtin_amdgcn_sched_barrier(0);
    float f0[8], f1[8];
    unpack8(v0, f0);
    unpack8(v1, f1);
    const bool in0 = hs < HW, in1 = hs + 32 < HW;
#pragma unroll
    for (int e = 0; e < 8; ++e) s8[e] = (in0 ? f0[e] : 0.f) + (in1 ? f1[e] : 0.f);
  }
  for (int hw = hs + 64; hw < HW; hw += 32) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(p + long(hw) * K), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) s8[e] += f[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[hs][cg][e] = s8[e];
  __syncthreads();
  if (tid < 64) {
    const int g = tid >> 3, e = tid & 7;
    float a = 0.f;
#pragma unroll 8
    for (int h = 0; h < 32; ++h) a += part[h][g][e];
    pooled[long(m) * K + k0 + tid] = f32_to_bf16(a * inv_hw);
  }
}

// K slice = K / kHeadKS channels, split over the 4 waves (kw = K slice / 4 each,
// a multiple of 32); a wave holds 2 x 2 16x16 accumulators (32 rows x 32 cols).
template <int KSTEPS, int KS>
__global__ __launch_bounds__(256) void fc_partial_kernel(const uint16_t* __restrict__ pooled,
                                                         const uint16_t* __restrict__ w, float* __restrict__ part,
                                                         int M, int K, int Np) {
  __shared__ float red[3][32][33];
  const int ks = blockIdx.x, ns = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int kslice = K / KS, kw = kslice / 4;
  const int k0 = ks * kslice + wid * kw;
  const int n0 = ns * kHeadCols;
  // B fragments of this wave's K range: rows n0 + j*16 + fr (zero past Np)
  bf16x8 bfr[KSTEPS][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + j * 16 + fr;
#pragma unroll
    for (int t = 0; t < KSTEPS; ++t)
      bfr[t][j] = n < Np ? *reinterpret_cast<const bf16x8*>(w + long(n) * K + k0 + t * 32 + fq * 8)
                         : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  for (int m0 = 0; m0 < M; m0 += 32) {
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 afr[KSTEPS][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + i * 16 + fr;
#pragma unroll
      for (int t = 0; t < KSTEPS; ++t)
        afr[t][i] = m < M ? *reinterpret_cast<const bf16x8*>(pooled + long(m) * K + k0 + t * 32 + fq * 8)
                          : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int t = 0; t < KSTEPS; ++t)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[t][i], bfr[t][j], acc[i][j], 0, 0, 0);
    // waves 1..3 hand their tiles to wave 0 (C layout: row fq*4 + r, column fr)
    if (wid > 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[wid - 1][i * 16 + fq * 4 + r][j * 16 + fr] = acc[i][j][r];
    }
    __syncthreads();
    if (wid == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rr = i * 16 + fq * 4 + r, cc = j * 16 + fr;
            const int m = m0 + rr, n = n0 + cc;
            if (m < M && n < Np)
              part[(long(ks) * M + m) * Np + n] = acc[i][j][r] + red[0][rr][cc] + red[1][rr][cc] + red[2][rr][cc];
          }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- casts
__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, long n) {
  const long n8 = n / 8;
  for (long i = blockIdx.x * long(blockDim.x) + threadIdx.x; i < n8; i += long(gridDim.x) * blockDim.x) {
    const float4 a = reinterpret_cast<const float4*>(x)[2 * i];
    const float4 b = reinterpret_cast<const float4*>(x)[2 * i + 1];
    const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
  for (long i = n8 * 8 + blockIdx.x * long(blockDim.x) + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x)
    y[i] = f32_to_bf16(x[i]);
}

__global__ void cast_bf16_f32_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, long n) {
  for (long i = blockIdx.x * long(blockDim.x) + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x)
    y[i] = bf16_to_f32(x[i]);
}

// ---------------------------------------------------------------- BERT head
// Classifier + softmax over a few labels (BERT's num_labels = 2): one
// workgroup per row; each thread accumulates its k-slice of every label's dot
// product from the fp32 pooled row (vectorised float4 / 4-bf16 loads), a
// wave-shuffle + LDS reduction combines them, one lane applies the softmax.
// Replaces cast + a mostly-empty GEMM tile + torch's softmax (3 launches).
constexpr int kDsMaxN = 16;

__global__ __launch_bounds__(256) void dense_softmax_kernel(const float* __restrict__ x, int ldx,
                                                            const uint16_t* __restrict__ w, int ldw,
                                                            const float* __restrict__ bias, float* __restrict__ probs,
                                                            int N, int K) {
  __shared__ float red[4][kDsMaxN];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* xr = x + size_t(row) * ldx;
  float acc[kDsMaxN];
#pragma unroll
  for (int n = 0; n < kDsMaxN; ++n) acc[n] = 0.f;
  for (int k = tid * 4; k < K; k += 256 * 4) {        // K % 4 == 0 (host check)
    const float4 xv = *reinterpret_cast<const float4*>(xr + k);
#pragma unroll
    for (int n = 0; n < kDsMaxN; ++n) {
      if (n < N) {
        const uint2 wv4 = *reinterpret_cast<const uint2*>(w + size_t(n) * ldw + k);
        acc[n] += xv.x * bf16_to_f32(uint16_t(wv4.x & 0xffff)) + xv.y * bf16_to_f32(uint16_t(wv4.x >> 16)) +
                  xv.z * bf16_to_f32(uint16_t(wv4.y & 0xffff)) + xv.w * bf16_to_f32(uint16_t(wv4.y >> 16));
      }
    }
  }
#pragma unroll
  for (int n = 0; n < kDsMaxN; ++n) {
    float v = acc[n];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[wv][n] = v;
  }
  __syncthreads();
  if (tid == 0) {
    float logit[kDsMaxN], mx = -INFINITY;
    for (int n = 0; n < N; ++n) {
      logit[n] = red[0][n] + red[1][n] + red[2][n] + red[3][n] + (bias ? bias[n] : 0.f);
      mx = fmaxf(mx, logit[n]);
    }
    float sum = 0.f;
    for (int n = 0; n < N; ++n) {
      logit[n] = __expf(logit[n] - mx);
      sum += logit[n];
    }
    const float inv = 1.f / sum;
    for (int n = 0; n < N; ++n) probs[size_t(row) * N + n] = logit[n] * inv;
  }
}

// BERT attention adder from a key mask X [B, 1, S] (int32 or f32):
// (one - X) * scale, one launch instead of cast + mul + add.
__global__ void key_mask_adder_kernel(const void* __restrict__ m, int is_int, float one, float scale,
                                      float* __restrict__ out, long n) {
  for (long i = blockIdx.x * long(blockDim.x) + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x) {
    const float v = is_int ? float(static_cast<const int*>(m)[i]) : static_cast<const float*>(m)[i];
    out[i] = (one - v) * scale;
  }
}

// ---------------------------------------------------------------- LayerNorm
// One wave per row, y = LN(x + r). Rows up to 64 * 8 * kLnChunks columns are
// read once into registers (16-B loads), statistics are two-pass from the
// registers, gamma/beta come in as float4 pairs; longer rows stream twice.
constexpr int kLnChunks = 4;

__device__ __forceinline__ void ln_load(const uint16_t* xr, const uint16_t* rr, int c, float* f) {
  unpack8(*reinterpret_cast<const uint4*>(xr + c), f);
  if (rr) {
    float g[8];
    unpack8(*reinterpret_cast<const uint4*>(rr + c), g);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] += g[e];
  }
}

__device__ __forceinline__ void ln_store(uint16_t* yr, int c, const float* f, float mean, float inv,
                                         const float* __restrict__ gamma, const float* __restrict__ beta) {
  const float4 g0 = *reinterpret_cast<const float4*>(gamma + c), g1 = *reinterpret_cast<const float4*>(gamma + c + 4);
  const float4 b0 = *reinterpret_cast<const float4*>(beta + c), b1 = *reinterpret_cast<const float4*>(beta + c + 4);
  const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
  const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = (f[e] - mean) * inv * g[e] + bb[e];
  *reinterpret_cast<uint4*>(yr + c) = pack8(o);
}

__global__ __launch_bounds__(256) void layernorm_kernel(const uint16_t* __restrict__ x,
                                                        const uint16_t* __restrict__ r,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        uint16_t* __restrict__ y, int rows, int cols, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const uint16_t* xr = x + long(row) * cols;
  const uint16_t* rr = r ? r + long(row) * cols : nullptr;
  uint16_t* yr = y + long(row) * cols;
  if (cols <= 64 * 8 * kLnChunks) {
    float v[kLnChunks][8];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kLnChunks; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < cols) {
        ln_load(xr, rr, c, v[k]);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += v[k][e];
      }
    }
    const float mean = wave_sum(s) / cols;
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < kLnChunks; ++k)
      if ((k * 64 + lane) * 8 < cols) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float d = v[k][e] - mean; ss += d * d; }
      }
    const float inv = rsqrtf(wave_sum(ss) / cols + eps);
#pragma unroll
    for (int k = 0; k < kLnChunks; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < cols) ln_store(yr, c, v[k], mean, inv, gamma, beta);
    }
    return;
  }
  float s = 0.f, ss = 0.f;
  for (int c = lane * 8; c < cols; c += 512) {
    float f[8];
    ln_load(xr, rr, c, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) { s += f[e]; ss += f[e] * f[e]; }
  }
  s = wave_sum(s);
  ss = wave_sum(ss);
  const float mean = s / cols;
  const float inv = rsqrtf(fmaxf(ss / cols - mean * mean, 0.f) + eps);
  for (int c = lane * 8; c < cols; c += 512) {
    float f[8];
    ln_load(xr, rr, c, f);
    ln_store(yr, c, f, mean, inv, gamma, beta);
  }
}

// Sum over aligned groups of LPR lanes, every lane of a group getting the
// total: DPP lane swaps within 16-lane rows (quad xor 1 / 2, half-row mirror,
// row mirror: a few cycles each) and ds_bpermute only across rows.  The
// __shfl_xor butterfly was 5 LDS round trips per sum, each waited for alone.
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
  static_assert(LPR == 16 || LPR == 32 || LPR == 64, "lane group");
  auto dpp = [](float x, auto ctrl) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), decltype(ctrl)::value, 0xf, 0xf, false));
  };
  v += dpp(v, std::integral_constant<int, 0xb1>{});    // quad_perm [1, 0, 3, 2]
  v += dpp(v, std::integral_constant<int, 0x4e>{});    // quad_perm [2, 3, 0, 1]
  v += dpp(v, std::integral_constant<int, 0x141>{});   // row_half_mirror: quad 0 <-> 1
  v += dpp(v, std::integral_constant<int, 0x140>{});   // row_mirror: half-row 0 <-> 1
  if constexpr (LPR >= 32) v += __shfl_xor(v, 16, 64);
  if constexpr (LPR >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}

// Exact-fit rows (cols == LPR * 8 * CH, e.g. BERT-base 768 = 32 lanes x 3
// chunks): LPR lanes per row, 64 / LPR rows per wave, gamma / beta loaded into
// registers before the row arrives (their latency hides under the row's), no
// idle lanes in the last chunk (the one-wave-per-row kernel above leaves half
// of a wave idle for 768 columns).  Two-pass statistics from registers.
template <int LPR, int CH, int RG = 1>
__global__ __launch_bounds__(256) void layernorm_fit_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ r,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            uint16_t* __restrict__ y, int rows, float eps) {
  constexpr int COLS = LPR * 8 * CH;
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const int sub = lane / LPR, l = lane % LPR;
  // RG row groups per wave (TFSERVE_LN_RW): the gamma / beta registers serve
  // RG x RPW rows instead of RPW
  const int row0 = ((blockIdx.x * 4 + (threadIdx.x >> 6)) * RG) * RPW + sub;
  // gamma / beta through buffer loads: plain loads of the restrict-const
  // pointers were rematerialised by the register allocator next to their use,
  // after the row reduction (one more serial round trip per row group)
  float g[CH][8], b[CH][8];
  const __amdgpu_buffer_rsrc_t rsG =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(gamma), 0, COLS * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(beta), 0, COLS * 4, 0x00020000);
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const uint32_t c4 = uint32_t((k * LPR + l) * 8) * 4u;
    const u32x4 g0 = __builtin_amdgcn_raw_buffer_load_b128(rsG, c4, 0, 0);
    const u32x4 g1 = __builtin_amdgcn_raw_buffer_load_b128(rsG, c4 + 16u, 0, 0);
    const u32x4 b0 = __builtin_amdgcn_raw_buffer_load_b128(rsB, c4, 0, 0);
    const u32x4 b1 = __builtin_amdgcn_raw_buffer_load_b128(rsB, c4 + 16u, 0, 0);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      g[k][e] = __uint_as_float(g0[e]); g[k][4 + e] = __uint_as_float(g1[e]);
      b[k][e] = __uint_as_float(b0[e]); b[k][4 + e] = __uint_as_float(b1[e]);
    }
  }
  // every row load (x chunks and residual chunks, all RG groups) in flight at
  // once: the residual goes through a buffer resource (0 records when there
  // is none -> zeros), because `if (r) load` compiled to per-chunk
  // conditional blocks that each waited for their load -- 2 x CH serial
  // memory round trips per row
  const __amdgpu_buffer_rsrc_t rsR = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(r), 0, r ? int(long(rows) * COLS * 2) : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(y, 0, int(long(rows) * COLS * 2), 0x00020000);
  uint4 xv[RG][CH];
  u32x4 rv[RG][CH];
  long base[RG];
  bool ok[RG];
#pragma unroll
  for (int q = 0; q < RG; ++q) {
    const int row = row0 + q * RPW;
    ok[q] = row < rows;
    base[q] = long(ok[q] ? row : 0) * COLS;
#pragma unroll
    for (int k = 0; k < CH; ++k) xv[q][k] = *reinterpret_cast<const uint4*>(x + base[q] + (k * LPR + l) * 8);
#pragma unroll
    for (int k = 0; k < CH; ++k)
      rv[q][k] = __builtin_amdgcn_raw_buffer_load_b128(rsR, uint32_t(base[q] + (k * LPR + l) * 8) * 2u, 0, 0);
  }
  // keep the gamma/beta loads above ahead of the row math (the scheduler sank
  // them below the reduction: one more serial round trip before the stores)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < RG; ++q) {
    float v[CH][8];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      float rf[8];
      unpack8(xv[q][k], v[k]);
      unpack8(make_uint4(rv[q][k].x, rv[q][k].y, rv[q][k].z, rv[q][k].w), rf);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[k][e] += rf[e];
        s += v[k][e];
      }
    }
    s = group_sum<LPR>(s);
    const float mean = s * (1.f / COLS);
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < CH; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[k][e] - mean; ss += d * d; }
    ss = group_sum<LPR>(ss);
    const float inv = rsqrtf(ss * (1.f / COLS) + eps);
    // no branch around the stores (rows past the end store to an out-of-range
    // offset, dropped): with `if (ok) store` the gamma / beta loads above were
    // sunk into that branch -- issued after the row reduction, one more serial
    // memory round trip (seen in the gfx950 ISA, scripts/isa_audit.py)
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      float o8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o8[e] = (v[k][e] - mean) * inv * g[k][e] + b[k][e];
      const uint4 pk = pack8(o8);
      u32x4 pv;
      pv.x = pk.x; pv.y = pk.y; pv.z = pk.z; pv.w = pk.w;
      __builtin_amdgcn_raw_buffer_store_b128(
          pv, rsY, ok[q] ? uint32_t(base[q] + (k * LPR + l) * 8) * 2u : 0x80000000u, 0, 0);
    }
  }
}

// ---------------------------------------------------------------- embedding + LN
// One wave per token: y[t] = LN(word[ids[t]] + type[tids[t]] + pos[t % seq]).
// An id outside its table contributes a zero row (TF's GPU GatherV2 reads zeros
// there and never faults); `tids` / `pos` may be null. The row sum stays in
// registers (hidden <= 64 * 8 * kEmbChunks) so the variance is two-pass.
constexpr int kEmbChunks = 4;

__global__ __launch_bounds__(256) void embed_ln_kernel(const int* __restrict__ ids, const int* __restrict__ tids,
                                                       const uint16_t* __restrict__ word,
                                                       const uint16_t* __restrict__ pos,
                                                       const uint16_t* __restrict__ type,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, uint16_t* __restrict__ y,
                                                       int tokens, int seq, int hidden, int vocab, int ntypes,
                                                       float eps) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= tokens) return;
  const int id = ids[t];
  const bool wok = id >= 0 && id < vocab;
  const int tt = tids ? tids[t] : -1;
  const bool tok = tt >= 0 && tt < ntypes;
  const int p = t % seq;
  // every table row chunk (word, type, position) and gamma/beta in flight at
  // once: buffer loads whose out-of-range offsets read zeros stand in for the
  // `if (c < hidden) { if (wok) ... }` blocks, which waited for each load in
  // turn (an absent table is a 0-record descriptor)
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(word), 0, vocab * hidden * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsT = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(type), 0, type ? ntypes * hidden * 2 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsP =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(pos), 0, pos ? seq * hidden * 2 : 0, 0x00020000);
  u32x4 rw[kEmbChunks], rt[kEmbChunks], rp[kEmbChunks];
  float4 gl[kEmbChunks][2], bl[kEmbChunks][2];
#pragma unroll
  for (int k = 0; k < kEmbChunks; ++k) {
    const int c = (k * 64 + lane) * 8;
    const bool in = c < hidden;
    rw[k] = __builtin_amdgcn_raw_buffer_load_b128(rsW, in && wok ? uint32_t(id * hidden + c) * 2u : 0x80000000u, 0, 0);
    rt[k] = __builtin_amdgcn_raw_buffer_load_b128(rsT, in && tok ? uint32_t(tt * hidden + c) * 2u : 0x80000000u, 0, 0);
    rp[k] = __builtin_amdgcn_raw_buffer_load_b128(rsP, in ? uint32_t(p * hidden + c) * 2u : 0x80000000u, 0, 0);
    const int cc = in ? c : 0;
    gl[k][0] = *reinterpret_cast<const float4*>(gamma + cc);
    gl[k][1] = *reinterpret_cast<const float4*>(gamma + cc + 4);
    bl[k][0] = *reinterpret_cast<const float4*>(beta + cc);
    bl[k][1] = *reinterpret_cast<const float4*>(beta + cc + 4);
  }
  __builtin_amdgcn_sched_barrier(0);
  float v[kEmbChunks][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kEmbChunks; ++k) {
    float a[8], b[8], d[8];
    unpack8(make_uint4(rw[k].x, rw[k].y, rw[k].z, rw[k].w), a);
    unpack8(make_uint4(rt[k].x, rt[k].y, rt[k].z, rt[k].w), b);
    unpack8(make_uint4(rp[k].x, rp[k].y, rp[k].z, rp[k].w), d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[k][e] = a[e] + b[e] + d[e];   // zeros past `hidden`
      s += v[k][e];
    }
  }
  const float mean = wave_sum(s) / hidden;
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < kEmbChunks; ++k)
    if ((k * 64 + lane) * 8 < hidden) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[k][e] - mean; ss += d * d; }
    }
  const float inv = rsqrtf(wave_sum(ss) / hidden + eps);
#pragma unroll
  for (int k = 0; k < kEmbChunks; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < hidden) {
      const float4 g0 = gl[k][0], g1 = gl[k][1], b0 = bl[k][0], b1 = bl[k][1];
      const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[k][e] - mean) * inv * g[e] + bb[e];
      *reinterpret_cast<uint4*>(y + long(t) * hidden + c) = pack8(o);
    }
  }
}

// fp32 NHWC (C <= 4) -> bf16 NHWC C = 4 (zero padded): one pixel per thread,
// one 8-B store; feeds the kAC4 stem gather.
__global__ void ingest_c4_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, long pixels, int C) {
  for (long i = blockIdx.x * long(blockDim.x) + threadIdx.x; i < pixels; i += long(gridDim.x) * blockDim.x) {
    uint16_t v[4] = {0, 0, 0, 0};
    for (int c = 0; c < C; ++c) v[c] = f32_to_bf16(x[i * C + c]);
    reinterpret_cast<uint2*>(y)[i] = make_uint2(v[0] | (uint32_t(v[1]) << 16), v[2] | (uint32_t(v[3]) << 16));
  }
}

// RGB fast path: 4 pixels (48 B = three 16-B loads) per thread step, so the
// reads are wide enough to stream at full rate even when `x` is pinned host
// memory read over PCIe (the zero-copy ingest); 32 B of bf16 RGBA out.
__global__ void ingest_rgb4_kernel(const float4* __restrict__ x, uint4* __restrict__ y, long quads) {
  for (long q = blockIdx.x * long(blockDim.x) + threadIdx.x; q < quads; q += long(gridDim.x) * blockDim.x) {
    const float4 a = x[3 * q], b = x[3 * q + 1], c = x[3 * q + 2];
    const float p[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w[2 * k] = f32_to_bf16(p[3 * k]) | (uint32_t(f32_to_bf16(p[3 * k + 1])) << 16);
      w[2 * k + 1] = f32_to_bf16(p[3 * k + 2]);
    }
    y[2 * q] = make_uint4(w[0], w[1], w[2], w[3]);
    y[2 * q + 1] = make_uint4(w[4], w[5], w[6], w[7]);
  }
}

// fp32 NHWC (C <= 4) -> bf16 RGBA into a zero-bordered [N][Hp][Wp][4] buffer
// (image at row pt, column pl): the stem conv then runs without padding, so
// every 16-B operand chunk it DMAs (2 pixels x 4 channels) is in bounds.
// One block row per padded output row (n, yo), threads across its Wp pixels:
// 32-bit index math only, and border rows / columns store zeros without loads.
__global__ __launch_bounds__(256) void ingest_c4_pad_kernel(const float* __restrict__ x, uint2* __restrict__ y,
                                                            int N, int H, int W, int C, int Hp, int Wp, int pt,
                                                            int pl) {
  const int xo = blockIdx.x * blockDim.x + threadIdx.x;
  if (xo >= Wp) return;
  const int xi = xo - pl;
  for (int r = blockIdx.y; r < N * Hp; r += gridDim.y) {
    const int n = r / Hp;
    const int yi = r - n * Hp - pt;
    uint16_t v[4] = {0, 0, 0, 0};
    if ((unsigned)yi < (unsigned)H && (unsigned)xi < (unsigned)W) {
      const float* src = x + ((long(n) * H + yi) * W + xi) * C;
      if (C == 3) {
        v[0] = f32_to_bf16(src[0]);
        v[1] = f32_to_bf16(src[1]);
        v[2] = f32_to_bf16(src[2]);
      } else {
        for (int c = 0; c < C; ++c) v[c] = f32_to_bf16(src[c]);
      }
    }
    y[long(r) * Wp + xo] = make_uint2(v[0] | (uint32_t(v[1]) << 16), v[2] | (uint32_t(v[3]) << 16));
  }
}

int grid_for(long work, int block) {
  long g = (work + block - 1) / block;
  if (g > 256 * 16) g = 256 * 16;
  return int(g < 1 ? 1 : g);
}

}  // namespace

hipError_t maxpool_nhwc_launch(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, int KH, int KW,
                               int SH, int SW, int PT, int PL, int Ho, int Wo, hipStream_t s, const float* scale,
                               const float* shift, int act) {
  if ((scale == nullptr) != (shift == nullptr)) return hipErrorInvalidValue;
  if (C % 8 || N <= 0 || Ho <= 0 || Wo <= 0) return N <= 0 || Ho <= 0 || Wo <= 0 ? hipSuccess : hipErrorInvalidValue;
  const long row_items = long(Wo) * (C / 8);
  if (row_items > (1L << 30)) return hipErrorInvalidValue;
  const long rows = long(N) * Ho;
  if (rows > (1L << 30)) return hipErrorInvalidValue;
  const dim3 grid(unsigned((row_items + 255) / 256), unsigned(rows < 65535 ? rows : 65535));
  hipLaunchKernelGGL(maxpool_nhwc_kernel, grid, dim3(256), 0, s, x, y, N, H, W, C, KH, KW, SH, SW, PT, PL, Ho, Wo,
                     scale, shift, act);
  return hipGetLastError();
}

hipError_t global_avgpool_nhwc_launch(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t s) {
  const int chunks = (C / 8 + 63) / 64;
  hipLaunchKernelGGL(gap_nhwc_kernel, dim3(N * chunks), dim3(256), 0, s, x, y, N, HW, C);
  return hipGetLastError();
}

hipError_t softmax_argmax_launch(const void* logits, int in_bf16, float* probs, int64_t* classes, int rows,
                                 int cols, long ld, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  if (ld < cols) return hipErrorInvalidValue;
  if (cols <= kSmPerSmall * 256)
    hipLaunchKernelGGL((softmax_argmax_kernel<0, kSmPerSmall>), dim3(rows), dim3(256), 0, s, logits, in_bf16, probs,
                       classes, rows, cols, ld, static_cast<const float*>(nullptr), 0L,
                       static_cast<const float*>(nullptr));
  else
    hipLaunchKernelGGL(softmax_argmax_kernel<0>, dim3(rows), dim3(256), 0, s, logits, in_bf16, probs, classes, rows,
                       cols, ld, static_cast<const float*>(nullptr), 0L, static_cast<const float*>(nullptr));
  return hipGetLastError();
}

// Small-batch head (M <= 16 rows, HW <= 64 positions) in ONE launch instead
// of gap_rows + fc_partial + softmax_argmax (three ~5-us launches at b1):
//   * each fc workgroup (K slice, 32 columns) pools its own K slice first:
//     (row, 8-channel chunk, position quarter) per thread, every position's
//     load in flight, the quarters met in LDS -> bf16 pooled slice in LDS
//     (the same bf16 rounding as gap_rows);
//   * the fc partial as fc_partial_kernel, A fragments from that LDS slice;
//   * partials stored agent-coherent (sc1: visible to the other XCDs), then
//     one arrival count per workgroup; the LAST workgroup to arrive sums the
//     KS partials + bias per logit and runs softmax / argmax for the M rows
//     (the split-K fixup's hand-off, kernels/gemm_common.h), and re-zeroes
//     the counter for the next launch.
constexpr int kHeadSmallM = 16, kHeadSmallHW = 64;
template <int KSTEPS, int PER>
__global__ __launch_bounds__(256) void head_small_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                         const float* __restrict__ bias, float* __restrict__ part,
                                                         float* __restrict__ probs, int64_t* __restrict__ classes,
                                                         int* __restrict__ counter, int M, int HW, int K, int Np,
                                                         int N, float inv_hw, float* __restrict__ probs_h,
                                                         int64_t* __restrict__ classes_h) {
  constexpr int KSLICE = KSTEPS * 32 * 4;            // channels per workgroup (4 waves)
  __shared__ __attribute__((aligned(16))) uint16_t pooled[kHeadSmallM][KSLICE];
  __shared__ float quarter[4][64][9];
  __shared__ float red[3][16][33];
  __shared__ int s_last;
  __shared__ float smx[4], ssum[4];
  __shared__ int sarg[4];
  const int ks = blockIdx.x, ns = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int kbase = ks * KSLICE;
  // weights (B fragments of this wave's K range) and the bias (used by
  // whichever workgroup arrives last) are issued first: their round trips
  // overlap the pooling's instead of following it
  const int kw = KSLICE / 4, kl = wid * kw;       // this wave's offset in the slice
  const int n0 = ns * kHeadCols;
  bf16x8 bfr[KSTEPS][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + j * 16 + fr;
#pragma unroll
    for (int t = 0; t < KSTEPS; ++t)
      bfr[t][j] = n < Np ? *reinterpret_cast<const bf16x8*>(w + long(n) * K + kbase + kl + t * 32 + fq * 8)
                         : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  float bv[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = k * 256 + tid;
    bv[k] = bias[c < N ? c : N - 1];
  }
  // ---- pool this K slice: thread = (chunk of 8 channels, position quarter)
  constexpr int CHUNKS = KSLICE / 8;                // <= 64 at K = 2048
  static_assert(CHUNKS <= 64, "one chunk per lane of a quarter");
  const int ch = tid & 63, qtr = tid >> 6;
  for (int m = 0; m < M; ++m) {
    float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (ch < CHUNKS) {
      const uint16_t* px = x + (long(m) * HW) * K + kbase + ch * 8;
      uint4 v[kHeadSmallHW / 4];
#pragma unroll
      for (int j = 0; j < kHeadSmallHW / 4; ++j) {   // positions qtr, qtr + 4, ...: clamped, masked below
        const int hw = qtr + 4 * j;
        v[j] = *reinterpret_cast<const uint4*>(px + long(hw < HW ? hw : HW - 1) * K);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < kHeadSmallHW / 4; ++j) {
        if (qtr + 4 * j >= HW) continue;
        float f[8];
        unpack8(v[j], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) s8[e] += f[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) quarter[qtr][ch][e] = s8[e];
    __syncthreads();
    if (tid < CHUNKS * 8 / 8) {
      // thread tid: chunk tid, its 8 channels -> bf16 pooled row m
      uint32_t o[4];
#pragma unroll
      for (int e2 = 0; e2 < 4; ++e2) {
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a0 += quarter[q][tid][2 * e2];
          a1 += quarter[q][tid][2 * e2 + 1];
        }
        o[e2] = uint32_t(f32_to_bf16(a0 * inv_hw)) | (uint32_t(f32_to_bf16(a1 * inv_hw)) << 16);
      }
      *reinterpret_cast<uint4*>(&pooled[m][tid * 8]) = make_uint4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();
  }
  // ---- fc partial of this slice (B fragments and bias already in registers)
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int t = 0; t < KSTEPS; ++t) {
    const bf16x8 a = fr < M ? *reinterpret_cast<const bf16x8*>(&pooled[fr][kl + t * 32 + fq * 8])
                            : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[t][j], acc[j], 0, 0, 0);
  }
  if (wid > 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wid - 1][fq * 4 + r][j * 16 + fr] = acc[j][r];
  }
  __syncthreads();
  if (wid == 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = fq * 4 + r, cc = j * 16 + fr, n = n0 + cc;
        if (rr < M && n < Np)
          __hip_atomic_store(part + (long(ks) * M + rr) * Np + n,
                             acc[j][r] + red[0][rr][cc] + red[1][rr][cc] + red[2][rr][cc], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
  }
  // ---- arrival; the last workgroup finishes the head
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (tid == 0) {
    const int total = gridDim.x * gridDim.y;
    const int old = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == total - 1;
    if (s_last) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  for (int m = 0; m < M; ++m) {
    float v[PER];
    float mx = -INFINITY;
    int arg = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = k * 256 + tid, cc = c < N ? c : N - 1;
      float a = bv[k];
#pragma unroll
      for (int q = 0; q < kHeadKS; ++q)
        a += __hip_atomic_load(part + (long(q) * M + m) * Np + cc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v[k] = c < N ? a : -INFINITY;
      if (c < N && (a > mx || (a == mx && c < arg))) { mx = a; arg = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(arg, o, 64);
      if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
    }
    if (lane == 0) { smx[wid] = mx; sarg[wid] = arg; }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float om = smx[k];
      const int oa = sarg[k];
      if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
    }
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      v[k] = (k * 256 + tid < N) ? __expf(v[k] - mx) : 0.f;
      sum += v[k];
    }
    sum = wave_sum(sum);
    if (lane == 0) ssum[wid] = sum;
    __syncthreads();
    const float inv = 1.f / (ssum[0] + ssum[1] + ssum[2] + ssum[3]);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = k * 256 + tid;
      if (c < N) {
        probs[long(m) * N + c] = v[k] * inv;
        if (probs_h) probs_h[long(m) * N + c] = v[k] * inv;
      }
    }
    if (tid == 0) {
      classes[m] = arg;
      if (classes_h) classes_h[m] = arg;
    }
    __syncthreads();   // smx / ssum reused by the next row
  }
  if (probs_h || classes_h) __threadfence_system();   // host rows visible with the kernel's completion
}

bool classifier_head_one_launch(int M, int HW, int K, int Np, int N) {
  if (M <= 0 || HW <= 0 || N <= 0 || N > Np || K % (kHeadKS * 4 * 32)) return false;
  const int ksteps = K / kHeadKS / 4 / 32;
  return M <= kHeadSmallM && HW <= kHeadSmallHW && N <= kSmPer * 256 && (ksteps == 1 || ksteps == 2 || ksteps == 4);
}

static int head_ks(int K) {   // read per launch (captured once into a graph; tests flip it)
  const char* e = getenv("TFSERVE_HEAD_KS");
  const int want = e && std::atoi(e) == 8 ? 8 : kHeadKS;
  return (want == 2 * kHeadKS && K % (2 * kHeadKS * 4 * 32) == 0 && K / (2 * kHeadKS * 4 * 32) <= 4) ? want : kHeadKS;
}

hipError_t classifier_head_launch(const uint16_t* x, const uint16_t* w, const float* bias, float* ws, float* probs,
                                  int64_t* classes, int M, int HW, int K, int Np, int N, hipStream_t s,
                                  int* counter, float* probs_h, int64_t* classes_h) {
  if (M <= 0) return hipSuccess;
  if (K % (kHeadKS * 4 * 32) || N > Np || N <= 0 || HW <= 0) return hipErrorInvalidValue;
  const int ksteps = K / kHeadKS / 4 / 32;        // 32-deep MFMA steps per wave
  uint16_t* pooled = reinterpret_cast<uint16_t*>(ws);
  float* part = ws + (size_t(M) * K + 1) / 2;
  if (counter != nullptr && classifier_head_one_launch(M, HW, K, Np, N)) {
    const dim3 grid(kHeadKS, (Np + kHeadCols - 1) / kHeadCols);
    const float inv_hw = 1.f / float(HW);
    // the last workgroup's softmax tile: 4 logits per thread for N <= 1024
    // (see softmax_argmax_kernel), 16 otherwise
    const bool small = N <= kSmPerSmall * 256;
#define TFSK_HEAD_SMALL(KS, PER)                                                                               \
  hipLaunchKernelGGL((head_small_kernel<KS, PER>), grid, dim3(256), 0, s, x, w, bias, part, probs, classes,   \
                     counter, M, HW, K, Np, N, inv_hw, probs_h, classes_h)
    switch (ksteps) {
      case 1: if (small) TFSK_HEAD_SMALL(1, kSmPerSmall); else TFSK_HEAD_SMALL(1, kSmPer); break;
      case 2: if (small) TFSK_HEAD_SMALL(2, kSmPerSmall); else TFSK_HEAD_SMALL(2, kSmPer); break;
      case 4: if (small) TFSK_HEAD_SMALL(4, kSmPerSmall); else TFSK_HEAD_SMALL(4, kSmPer); break;
      default: return hipErrorInvalidValue;
    }
#undef TFSK_HEAD_SMALL
    return hipGetLastError();
  }
  if (probs_h != nullptr || classes_h != nullptr) return hipErrorNotSupported;
  hipLaunchKernelGGL(gap_rows_kernel, dim3(M, K / 64), dim3(256), 0, s, x, pooled, HW, K, 1.f / float(HW));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // K split: kHeadKS (4) slices, or 8 (TFSERVE_HEAD_KS=8, K a multiple of
  // 1024) for twice the workgroups on the weight stream (A/B switch)
  const int KS = head_ks(K);
  const int ks_steps = K / KS / 4 / 32;
  const dim3 grid(KS, (Np + kHeadCols - 1) / kHeadCols);
#define TFSK_FC(T, KSV) hipLaunchKernelGGL((fc_partial_kernel<T, KSV>), grid, dim3(256), 0, s, pooled, w, part, M, K, Np)
  if (KS == kHeadKS) {
    switch (ks_steps) {
      case 1: TFSK_FC(1, kHeadKS); break;
      case 2: TFSK_FC(2, kHeadKS); break;
      case 4: TFSK_FC(4, kHeadKS); break;
      case 8: TFSK_FC(8, kHeadKS); break;
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (ks_steps) {
      case 1: TFSK_FC(1, 2 * kHeadKS); break;
      case 2: TFSK_FC(2, 2 * kHeadKS); break;
      case 4: TFSK_FC(4, 2 * kHeadKS); break;
      default: return hipErrorInvalidValue;
    }
  }
#undef TFSK_FC
  e = hipGetLastError();
  if (e != hipSuccess) return e;
#define TFSK_SM(NP, PER)                                                                                   \
  hipLaunchKernelGGL((softmax_argmax_kernel<NP, PER>), dim3(M), dim3(256), 0, s,                          \
                     static_cast<const void*>(nullptr), 0, probs, classes, M, N, long(Np),                \
                     static_cast<const float*>(part), long(M) * Np, bias)
  const bool small = N <= kSmPerSmall * 256;
  if (KS == kHeadKS) {
    if (small) TFSK_SM(kHeadKS, kSmPerSmall); else TFSK_SM(kHeadKS, kSmPer);
  } else {
    if (small) TFSK_SM(2 * kHeadKS, kSmPerSmall); else TFSK_SM(2 * kHeadKS, kSmPer);
  }
#undef TFSK_SM
  return hipGetLastError();
}

size_t classifier_head_ws_floats(int M, int K, int Np) {
  return (size_t(M) * K + 1) / 2 + size_t(2 * kHeadKS) * M * Np;   // bf16 pooled rows + f32 partials (<= 8 slices)
}

hipError_t cast_f32_bf16_launch(const float* x, uint16_t* y, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n / 8 + 1, 256)), dim3(256), 0, s, x, y, long(n));
  return hipGetLastError();
}

hipError_t ingest_c4_launch(const float* x, uint16_t* y, int64_t pixels, int C, hipStream_t s) {
  if (C == 3 && pixels % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(y) & 15) == 0) {
    const long quads = long(pixels) / 4;
    hipLaunchKernelGGL(ingest_rgb4_kernel, dim3(grid_for(quads, 256)), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(x), reinterpret_cast<uint4*>(y), quads);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(ingest_c4_kernel, dim3(grid_for(pixels, 256)), dim3(256), 0, s, x, y, long(pixels), C);
  return hipGetLastError();
}

hipError_t ingest_c4_pad_launch(const float* x, uint16_t* y, int N, int H, int W, int C, int Hp, int Wp, int pt,
                               int pl, hipStream_t s) {
  if (N <= 0 || Hp <= 0 || Wp <= 0) return hipSuccess;
  const long rows = long(N) * Hp;
  if (rows > (1L << 30) || Wp > (1 << 30)) return hipErrorInvalidValue;
  const dim3 grid(unsigned((Wp + 255) / 256), unsigned(rows < 65535 ? rows : 65535));
  hipLaunchKernelGGL(ingest_c4_pad_kernel, grid, dim3(256), 0, s, x, reinterpret_cast<uint2*>(y), N, H, W, C, Hp,
                     Wp, pt, pl);
  return hipGetLastError();
}

hipError_t dense_softmax_launch(const float* x, int ldx, const uint16_t* w, int ldw, const float* bias,
                                float* probs, int rows, int N, int K, hipStream_t s) {
  if (N < 1 || N > kDsMaxN || K % 4 || ldx % 4 || ldw % 4) return hipErrorInvalidValue;
  if (rows == 0) return hipSuccess;
  hipLaunchKernelGGL(dense_softmax_kernel, dim3(rows), dim3(256), 0, s, x, ldx, w, ldw, bias, probs, N, K);
  return hipGetLastError();
}

hipError_t key_mask_adder_launch(const void* m, int is_int, float one, float scale, float* out, int64_t n,
                                 hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(key_mask_adder_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, m, is_int, one, scale, out,
                     long(n));
  return hipGetLastError();
}

// ---------------------------------------------------------------- host rows -> device
// A small batch's input rows copied by a kernel inside the bucket's HIP graph
// instead of an SDMA hipMemcpyAsync ahead of it: at batch 1 the copy engine
// took 11.7 us for 301 KB and its completion another 9.8 us to reach the
// graph's first kernel (profiles/round5/s45/c1_timeline.json).  Every load is
// in flight at once (4 x 16 B per thread) and carries system scope (sc0 sc1):
// the host rewrites the same pinned rows for every batch, so a line cached in
// L2 by an earlier replay must never satisfy a later one.
template <int PER>
__global__ __launch_bounds__(256) void h2d_rows_kernel(const void* __restrict__ src, u32x4* __restrict__ dst, int n16) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(src), 0, n16 * 16, 0x00020000);
  const int base = blockIdx.x * (256 * PER) + threadIdx.x;
  u32x4 v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j)
    v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, uint32_t(base + j * 256) * 16u, 0, 17);   // sc0 | sc1
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (base + j * 256 < n16) dst[base + j * 256] = v[j];
}

int epi_f32_env() {
  static const int v = [] {
    const char* e = getenv("TFSERVE_EPI_F32");
    return e != nullptr && atoi(e) != 0 ? 1 : 0;
  }();
  return v;
}

// 16-B pieces per thread: TFSERVE_H2D_PER (1 / 2 / 4; A/B), default 4
int h2d_per() {
  static const int v = [] {
    const char* e = getenv("TFSERVE_H2D_PER");
    const int x = e ? atoi(e) : 4;
    return x == 1 || x == 2 ? x : 4;
  }();
  return v;
}

hipError_t h2d_rows_launch(const void* host, void* dev, int64_t bytes, hipStream_t s) {
  if (bytes <= 0) return hipSuccess;
  if (bytes % 16 != 0 || bytes >= (int64_t(1) << 31) ||
      (reinterpret_cast<uintptr_t>(host) | reinterpret_cast<uintptr_t>(dev)) % 16 != 0)
    return hipErrorInvalidValue;
  const int n16 = int(bytes / 16), per = h2d_per();
  const dim3 grid((n16 + 256 * per - 1) / (256 * per));
  u32x4* d = reinterpret_cast<u32x4*>(dev);
  switch (per) {
    case 1: hipLaunchKernelGGL(h2d_rows_kernel<1>, grid, dim3(256), 0, s, host, d, n16); break;
    case 2: hipLaunchKernelGGL(h2d_rows_kernel<2>, grid, dim3(256), 0, s, host, d, n16); break;
    default: hipLaunchKernelGGL(h2d_rows_kernel<4>, grid, dim3(256), 0, s, host, d, n16); break;
  }
  return hipGetLastError();
}

hipError_t cast_bf16_f32_launch(const uint16_t* x, float* y, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, x, y, long(n));
  return hipGetLastError();
}

// row groups per wave of the exact-fit LayerNorm: TFSERVE_LN_RW (1 / 2; A/B), default 1
int ln_rw() {
  static const int v = [] {
    const char* e = getenv("TFSERVE_LN_RW");
    return e != nullptr && atoi(e) == 2 ? 2 : 1;
  }();
  return v;
}

template <int LPR, int CH>
hipError_t ln_fit(const uint16_t* x, const uint16_t* r, const float* gamma, const float* beta, uint16_t* y, int rows,
                  float eps, hipStream_t s) {
  if (long(rows) * LPR * 8 * CH * 2 >= 0x7fffffffL) {   // residual buffer offsets are 32-bit
    hipLaunchKernelGGL(layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, r, gamma, beta, y, rows,
                       LPR * 8 * CH, eps);
    return hipGetLastError();
  }
  if (ln_rw() == 2) {
    const int per_block = 4 * 2 * (64 / LPR);
    hipLaunchKernelGGL((layernorm_fit_kernel<LPR, CH, 2>), dim3((rows + per_block - 1) / per_block), dim3(256), 0, s,
                       x, r, gamma, beta, y, rows, eps);
    return hipGetLastError();
  }
  const int per_block = 4 * (64 / LPR);
  hipLaunchKernelGGL((layernorm_fit_kernel<LPR, CH>), dim3((rows + per_block - 1) / per_block), dim3(256), 0, s, x, r,
                     gamma, beta, y, rows, eps);
  return hipGetLastError();
}

hipError_t layernorm_launch(const uint16_t* x, const uint16_t* r, const float* gamma, const float* beta,
                            uint16_t* y, int rows, int cols, float eps, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  switch (cols) {
    case 128: return ln_fit<16, 1>(x, r, gamma, beta, y, rows, eps, s);
    case 256: return ln_fit<32, 1>(x, r, gamma, beta, y, rows, eps, s);
    case 384: return ln_fit<16, 3>(x, r, gamma, beta, y, rows, eps, s);
    case 512: return ln_fit<64, 1>(x, r, gamma, beta, y, rows, eps, s);
    case 768: return ln_fit<32, 3>(x, r, gamma, beta, y, rows, eps, s);
    case 1024: return ln_fit<64, 2>(x, r, gamma, beta, y, rows, eps, s);
    case 2048: return ln_fit<64, 4>(x, r, gamma, beta, y, rows, eps, s);
    default: break;
  }
  hipLaunchKernelGGL(layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, r, gamma, beta, y, rows, cols,
                     eps);
  return hipGetLastError();
}

hipError_t embed_ln_launch(const int* ids, const int* type_ids, const uint16_t* word, const uint16_t* pos,
                           const uint16_t* type, const float* gamma, const float* beta, uint16_t* y, int tokens,
                           int seq, int hidden, int vocab, int ntypes, float eps, hipStream_t s) {
  if (hidden % 8 || hidden > 64 * 8 * kEmbChunks || seq <= 0) return hipErrorInvalidValue;
  // 32-bit buffer offsets into the tables
  if (long(vocab) * hidden * 2 >= 0x7fffffffL || long(ntypes) * hidden * 2 >= 0x7fffffffL ||
      long(seq) * hidden * 2 >= 0x7fffffffL)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_ln_kernel, dim3((tokens + 3) / 4), dim3(256), 0, s, ids, type_ids, word, pos, type,
                     gamma, beta, y, tokens, seq, hidden, vocab, ntypes, eps);
  return hipGetLastError();
}

}  // namespace tfsk
