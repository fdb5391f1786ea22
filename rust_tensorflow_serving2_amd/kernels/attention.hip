// Fused multi-head self-attention for encoder models (BERT), gfx950.
//
// Input is the packed output of ONE fused QKV GEMM: qkv[B][S][3*H*D] (bf16,
// Q | K | V column blocks, head h at columns h*D).  One 256-thread workgroup
// per (batch, head, 64-query block); each wave64 owns 16 query rows against
// all S keys:
//   scores^T = K Q^T        v_mfma_f32_16x16x32_bf16, K row-major in LDS
//                           (XOR-swizzled 16-B chunks: conflict-free b128 reads)
//   P = softmax(scores*scale + mask_bias)   in registers: each lane holds one
//                           query's S/16 x 4 keys; row max/sum = 2 xor shuffles
//   ctx^T = V^T P^T         P stays in registers as the B operand (k slots
//                           permuted, the A side reads V^T rows to match); V
//                           stored transposed (Vt[d][key], rows padded by 16 B),
//                           transposed in registers on 8x8 blocks, after the
//                           scores so its loads overlap them
// (attention_plds_kernel: the previous layout, P through a per-wave LDS strip.)
// S in {64, 128, 192, 256} (the whole key row in registers; D == 64), and
// attention_flash_kernel below for any other S up to
// kMaxAttentionSeq.  The S x S matrix never touches HBM.
#include <cstdlib>

#include "common.h"
#include "gemm_common.h"
#include "launch.h"

namespace tfsk {

namespace {

constexpr int D = 64;

// query rows per workgroup (16 per wave) for S != 128 (S = 128: attn_qb).  With
// P through LDS, 64 measured faster than one workgroup per (batch, head) at
// BERT-base b32 (161 vs 182 us per 12 layers); with P in registers, 128 wins
// there (attn_qb below).
constexpr int qb_for(int) { return 64; }

// per-workgroup phase stamps (scripts/wg_trace.py --attention; null: off)
long long* g_attn_trace = nullptr;
int g_attn_trace_cap = 0;
__device__ __forceinline__ void attn_stamp(long long* trace, int cap, int k) {
  if (trace != nullptr && threadIdx.x == 0 && int(blockIdx.x) < cap) {
    long long* d = trace + long(blockIdx.x) * 8;
    d[k] = wall_clock64();
    if (k == 0) d[7] = __smid();
  }
}

// Scores computed transposed (S^T = K Q^T: keys on the MFMA rows, queries on
// the columns), so each lane ends the softmax holding, for ONE query (its
// column fr), the 8 keys {32ks + 4fq + r, 32ks + 16 + 4fq + r} of every 32-key
// block: exactly a B fragment of ctx^T = V^T P^T under a k-slot permutation
// that the A side (V^T rows, two 8-B LDS reads per fragment) repeats.  P never
// goes through LDS and the output leaves in 8-B row pieces straight from the
// accumulators.  Staging is split: Q, K and the key mask land first (one
// barrier), V's loads stay in flight in registers through the scores and the
// softmax and are transposed into LDS behind a second barrier -- the V half of
// the staging overlaps the score math instead of preceding it.
template <int S, int QB>
__global__ __launch_bounds__(QB * 4) void attention_kernel(const uint16_t* __restrict__ qkv,
                                                           const float* __restrict__ mask_bias,
                                                           uint16_t* __restrict__ ctx, int H, float scale,
                                                           long mask_bstride, long mask_qstride,
                                                           long long* __restrict__ trace, int trace_cap) {
  attn_stamp(trace, trace_cap, 0);
  constexpr int NTH = QB * 4;            // QB / 16 waves
  constexpr int VT_LD = S + 8;           // Vt row stride (elements): +16 B pad
  constexpr int NT = S / 16;             // key tiles
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* Ks = reinterpret_cast<uint16_t*>(smem);          // [S][64] swizzled
  uint16_t* Vt = Ks + S * D;                                  // [64][VT_LD]
  float* Ms = reinterpret_cast<float*>(Vt + D * VT_LD);       // [S] key mask adder

  const int qblocks = S / QB;
  const int bid = blockIdx.x;
  const int qb = bid % qblocks;
  const int h = (bid / qblocks) % H;
  const int b = bid / (qblocks * H);
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const long row_stride = 3L * H * D;
  const uint16_t* base = qkv + long(b) * S * row_stride;

  // ---- K rows and the key mask by LDS-DMA: each wave instruction lands 1 KB
  // (8 keys x 128 B) with lane l at chunk l & 7 of key row l >> 3, so lane l
  // fetches chunk (l & 7) ^ (key & 7) -- the XOR-swizzled row.  (Loads into
  // registers were sunk by the compiler to their LDS stores, one serial round
  // trip per chunk, and the mask's behind them.)
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  constexpr int NW = NTH / 64;
  const __amdgpu_buffer_rsrc_t rsQ =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(base), 0, int(S * row_stride * 2), 0x00020000);
  static_assert((S / 8) % NW == 0, "K staging split");
  constexpr int KDMA = S / 8 / NW;
#pragma unroll
  for (int i = 0; i < KDMA; ++i) {
    const int pc = wid + i * NW, key = pc * 8 + (lane >> 3);
    const uint32_t src = uint32_t(long(key) * row_stride + H * D + h * D + (((lane & 7) ^ (key & 7)) * 8)) * 2u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsQ, (lds_ptr_t)(Ks + pc * 512), 16, src, 0, 0, 0);
  }
  // the [B,1,1,S] key mask (BERT's adder, mask_qstride == 0); a 0-record
  // descriptor (zeros) when the mask is per query row or absent.  Lanes past
  // S / 4 land zeros in the region's padding.
  const bool key_mask = mask_bias != nullptr && mask_qstride == 0;
  const __amdgpu_buffer_rsrc_t rsM = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(key_mask ? mask_bias + long(b) * mask_bstride : mask_bias), 0, key_mask ? S * 4 : 0,
      0x00020000);
  static_assert(S * 4 <= 1024, "mask staging");
  if (wid == 0)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsM, (lds_ptr_t)Ms, 16, lane * 16 < S * 4 ? uint32_t(lane * 16) : gemm::kOOB,
                                             0, 0, 0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  // ---- Q fragments (the B operand of K Q^T: column = query fr, k = d)
  const int q0 = qb * QB + wid * 16;
  bf16x8 qf[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
    qf[kk] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                            rsQ, uint32_t(long(q0 + fr) * row_stride + h * D + kk * 32 + fq * 8) * 2u, 0, 0));
  static_assert(S <= NTH, "V staging split");
  // V: an 8-key x 8-dim block per thread (threads >= S load a clamped
  // in-range block whose stores land in the rows' padding), issued now,
  // consumed after the softmax
  const int vblk = tid < S ? tid : S - 1;
  const int kg = vblk >> 3, vch = vblk & 7;
  uint32_t w[8][4];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
        rsQ, uint32_t(long(kg * 8 + k) * row_stride + 2 * H * D + h * D + vch * 8) * 2u, 0, 0);
    w[k][0] = v.x; w[k][1] = v.y; w[k][2] = v.z; w[k][3] = v.w;
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  // K, the mask and Q landed (in order: only the 8 V loads may be younger)
  gemm::wait_vmcnt<8>();
  __syncthreads();
  attn_stamp(trace, trace_cap, 1);          // Q / K / mask staged (V in flight)

  // ---- S^T tiles: lane holds keys nt*16 + 4fq + r of query fr
  f32x4 s[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int key = nt * 16 + fr;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + fq;
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + key * D + ((ch ^ (key & 7)) * 8));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], acc, 0, 0, 0);
    }
    s[nt] = acc;
  }
  // ---- softmax over keys: 32 values per lane, then the 4 lanes of a query
  float mx = -INFINITY;
  if (key_mask) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const f32x4 mb = *reinterpret_cast<const f32x4*>(Ms + nt * 16 + fq * 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = s[nt][r] * scale + mb[r];
        s[nt][r] = v;
        mx = fmaxf(mx, v);
      }
    }
  } else {
    const float* mq = mask_bias ? mask_bias + long(b) * mask_bstride + long(q0 + fr) * mask_qstride : nullptr;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = s[nt][r] * scale + (mq ? mq[nt * 16 + fq * 4 + r] : 0.f);
        s[nt][r] = v;
        mx = fmaxf(mx, v);
      }
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
  bf16x8 pb[S / 32];                        // P^T B fragments, k-slot j -> tile 2ks + (j >> 2), r = j & 3
  // exp(v - mx) as exp2(v log2e - mx log2e): one fma + v_exp_f32 per value
  // (__expf is a subtract, a multiply and the v_exp)
  // (pairs: the arguments and the running sum as packed fp32, v_pk_fma_f32 /
  // v_pk_add_f32, two values per instruction)
  constexpr float kLog2e = 1.4426950408889634f;
  const float mxl = mx * kLog2e;
  typedef __attribute__((ext_vector_type(2))) float f32x2;
  f32x2 sum2 = {0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < S / 32; ++ks) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const f32x2 v = {s[2 * ks + (j >> 2)][j & 3], s[2 * ks + (j >> 2)][(j & 3) + 1]};
      const f32x2 a = v * kLog2e - mxl;
      const f32x2 e = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
      sum2 += e;
      pb[ks][j] = static_cast<__bf16>(e.x);
      pb[ks][j + 1] = static_cast<__bf16>(e.y);
    }
  }
  sum = sum2.x + sum2.y;
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  attn_stamp(trace, trace_cap, 2);          // scores + softmax done

  // ---- V transposed into LDS (8 x 16-B stores per thread) behind the second barrier
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = (d & 1) ? (w[2 * j][d >> 1] >> 16) : (w[2 * j][d >> 1] & 0xffffu);
      const uint32_t hi = (d & 1) ? (w[2 * j + 1][d >> 1] & 0xffff0000u) : (w[2 * j + 1][d >> 1] << 16);
      o[j] = lo | hi;
    }
    const int vcol = tid < S ? kg * 8 : S;
    *reinterpret_cast<uint4*>(Vt + (vch * 8 + d) * VT_LD + vcol) = make_uint4(o[0], o[1], o[2], o[3]);
  }
  __syncthreads();

  // ---- ctx^T = V^T P^T: A = Vt rows dt*16 + fr at the same permuted keys
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the V^T fragments read two 32-key steps ahead of their MFMAs (the
  // compiler's own order left an LDS round trip in front of every MFMA;
  // sched_barriers pin this one)
  constexpr int KS = S / 32;
  bf16x8 va[KS][4];
  auto read_v = [&](int ks) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const uint16_t* vr = Vt + (dt * 16 + fr) * VT_LD + ks * 32 + fq * 4;
      const uint2 lo = *reinterpret_cast<const uint2*>(vr);
      const uint2 hi = *reinterpret_cast<const uint2*>(vr + 16);
      va[ks][dt] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
    }
  };
  read_v(0);
  if (KS > 1) read_v(1);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (ks + 2 < KS) read_v(ks + 2);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va[ks][dt], pb[ks], o[dt], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  attn_stamp(trace, trace_cap, 3);          // P V done (wave 0)
  // ---- normalise; lane holds dims dt*16 + 4fq + [0, 4) of query q0 + fr.
  // Re-laid out through a wave-private 16 x 64 block of the K rows (every
  // wave passed its scores before the second barrier; (wid + 1) * 16 <= S)
  // with 16-B chunks XOR-swizzled by row, then stored as whole 128-B rows:
  // 8-B stores straight from the accumulators touch 16 rows per instruction
  // (0.88 vs 0.24 us for the store phase, profiles/round5/s40/wgN.log)
  const float inv = 1.f / sum;
  uint16_t* os = Ks + wid * 16 * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const uint32_t lo = gemm::pack_bf16x2(o[dt][0] * inv, o[dt][1] * inv);
    const uint32_t hi = gemm::pack_bf16x2(o[dt][2] * inv, o[dt][3] * inv);
    const int chunk = dt * 2 + (fq >> 1);
    *reinterpret_cast<uint2*>(os + fr * D + ((chunk ^ (fr & 7)) * 8) + (fq & 1) * 4) = make_uint2(lo, hi);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);          // lgkmcnt(0): this wave's LDS writes landed
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = j * 64 + lane, row = c >> 3, ch = c & 7;
    *reinterpret_cast<uint4*>(ctx + (long(b) * S + q0 + row) * (long(H) * D) + h * D + ch * 8) =
        *reinterpret_cast<const uint4*>(os + row * D + ((ch ^ (row & 7)) * 8));
  }
  if (trace != nullptr) {
    __builtin_amdgcn_s_waitcnt(0);          // this wave's stores acknowledged
    attn_stamp(trace, trace_cap, 4);
  }
}

// The previous layout (TFSERVE_ATTN_PLDS=1, A/B only): scores un-transposed,
// P re-laid out through a per-wave LDS strip, all staging before one barrier.
template <int S, int QB>
__global__ __launch_bounds__(QB * 4) void attention_plds_kernel(const uint16_t* __restrict__ qkv,
                                                           const float* __restrict__ mask_bias,
                                                           uint16_t* __restrict__ ctx, int H, float scale,
                                                           long mask_bstride, long mask_qstride,
                                                           long long* __restrict__ trace, int trace_cap) {
  attn_stamp(trace, trace_cap, 0);
  constexpr int NTH = QB * 4;            // QB / 16 waves
  constexpr int VT_LD = S + 8;           // Vt row stride (elements): +16 B pad
  constexpr int P_LD = S + 8;
  constexpr int NT = S / 16;             // key tiles
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint16_t* Ks = reinterpret_cast<uint16_t*>(smem);          // [S][64] swizzled
  uint16_t* Vt = Ks + S * D;                                  // [64][VT_LD]
  uint16_t* Ps = Vt + D * VT_LD;                              // [QB/16][16][P_LD]

  const int qblocks = S / QB;
  // (an XCD remap putting a head's two query blocks on one XCD, so the second
  // K / V staging would hit L2, measured neutral: 150.5 vs 149.6 us per 12
  // layers at BERT-base b32, profiles/round5/s9/replay_bert_b32.txt)
  const int bid = blockIdx.x;
  const int qb = bid % qblocks;
  const int h = (bid / qblocks) % H;
  const int b = bid / (qblocks * H);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const long row_stride = 3L * H * D;
  const uint16_t* base = qkv + long(b) * S * row_stride;

  // ---- every staging load (K chunks, this thread's 8x8 V block, Q fragments)
  // issued before the first LDS store: the rolled K loop loaded and stored one
  // chunk per trip, i.e. S * 8 / NTH serial memory round trips before the
  // MFMAs could start (seen in the gfx950 ISA)
  static_assert((S * 8) % NTH == 0 && S <= NTH, "staging split");
  constexpr int KIT = S * 8 / NTH;
  uint4 kv[KIT];
#pragma unroll
  for (int i = 0; i < KIT; ++i) {
    const int c = tid + i * NTH, key = c >> 3, ch = c & 7;
    kv[i] = *reinterpret_cast<const uint4*>(base + long(key) * row_stride + H * D + h * D + ch * 8);
  }
  // V transposed: an 8-key x 8-dim block per thread (threads >= S idle; their
  // loads read a clamped in-range block and are dropped), transposed in
  // registers (8 x 16-B loads in, 8 x 16-B LDS stores out)
  const int vblk = tid < S ? tid : S - 1;
  const int kg = vblk >> 3, vch = vblk & 7;
  uint32_t w[8][4];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 v = *reinterpret_cast<const uint4*>(base + long(kg * 8 + k) * row_stride + 2 * H * D + h * D +
                                                    vch * 8);
    w[k][0] = v.x; w[k][1] = v.y; w[k][2] = v.z; w[k][3] = v.w;
  }
  // ---- Q fragments straight from global (A operand: row = fr, k = 8*fq + j)
  const int q0 = qb * QB + wid * 16;
  bf16x8 qf[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
    qf[kk] = *reinterpret_cast<const bf16x8*>(base + long(q0 + fr) * row_stride + h * D + kk * 32 + fq * 8);
  // the [B,1,1,S] key mask (BERT's adder, mask_qstride == 0) of this lane's
  // key columns, loaded with the operands instead of after the QK^T MFMAs (a
  // 0-record descriptor when the mask is per query row or absent: zeros)
  const bool key_mask = mask_bias != nullptr && mask_qstride == 0;
  const __amdgpu_buffer_rsrc_t rsM = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(key_mask ? mask_bias + long(b) * mask_bstride : mask_bias), 0, key_mask ? S * 4 : 0,
      0x00020000);
  float mbk[S / 16];
#pragma unroll
  for (int nt = 0; nt < S / 16; ++nt)
    mbk[nt] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsM, uint32_t(nt * 16 + fr) * 4u, 0, 0));
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < KIT; ++i) {
    const int c = tid + i * NTH, key = c >> 3, ch = c & 7;
    *reinterpret_cast<uint4*>(Ks + key * D + ((ch ^ (key & 7)) * 8)) = kv[i];
  }
  // (no `if (tid < S)` around the stores: the compiler sank the V loads into
  // any such block; idle threads store into the rows' 16-B padding columns
  // [S, S + 8), which no P.V read touches)
  uint4 vt8[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) {
    uint32_t o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = (d & 1) ? (w[2 * j][d >> 1] >> 16) : (w[2 * j][d >> 1] & 0xffffu);
      const uint32_t hi = (d & 1) ? (w[2 * j + 1][d >> 1] & 0xffff0000u) : (w[2 * j + 1][d >> 1] << 16);
      o[j] = lo | hi;
    }
    vt8[d] = make_uint4(o[0], o[1], o[2], o[3]);
  }
  const int vcol = tid < S ? kg * 8 : S;
#pragma unroll
  for (int d = 0; d < 8; ++d) *reinterpret_cast<uint4*>(Vt + (vch * 8 + d) * VT_LD + vcol) = vt8[d];
  __syncthreads();
  attn_stamp(trace, trace_cap, 1);          // operands staged

  // ---- scores
  f32x4 s[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int key = nt * 16 + fr;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + fq;
      const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + key * D + ((ch ^ (key & 7)) * 8));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[kk], kf, acc, 0, 0, 0);
    }
    s[nt] = acc;
  }
  // ---- softmax (rows fq*4 + r, columns nt*16 + fr)
  float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  const float* mrow = mask_bias ? mask_bias + long(b) * mask_bstride + long(q0 + fq * 4) * mask_qstride : nullptr;
  if (key_mask) {
    // key mask shared by every query row (BERT's [B,1,1,S] adder): prefetched above
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const float mb = mbk[nt];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = s[nt][r] * scale + mb;
        s[nt][r] = v;
        mx[r] = fmaxf(mx[r], v);
      }
    }
  } else {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float mb = mrow ? mrow[long(r) * mask_qstride + nt * 16 + fr] : 0.f;
        const float v = s[nt][r] * scale + mb;
        s[nt][r] = v;
        mx[r] = fmaxf(mx[r], v);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o, 64));
  float sum[4] = {0.f, 0.f, 0.f, 0.f};
  uint16_t* pw = Ps + wid * 16 * P_LD;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = __expf(s[nt][r] - mx[r]);
      sum[r] += e;
      pw[(fq * 4 + r) * P_LD + nt * 16 + fr] = f32_to_bf16(e);
    }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) sum[r] += __shfl_xor(sum[r], o, 64);
  // the P strip is wave-private (this wave's 16 rows) and K / Vt were staged
  // before the barrier above: only this wave's LDS writes must land before
  // its P reads, so no workgroup barrier (waves that finish the softmax early
  // start P V without waiting for the others)
  __builtin_amdgcn_s_waitcnt(0xc07f);          // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  attn_stamp(trace, trace_cap, 2);          // scores + softmax done

  // ---- ctx = P V
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < S / 32; ++ks) {
    const bf16x8 pa = *reinterpret_cast<const bf16x8*>(pw + fr * P_LD + ks * 32 + fq * 8);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 vb = *reinterpret_cast<const bf16x8*>(Vt + (dt * 16 + fr) * VT_LD + ks * 32 + fq * 8);
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[dt], 0, 0, 0);
    }
  }
  // ---- normalise, re-layout through the wave's P strip (its P reads are
  // done: the MFMAs above consumed them) and store 16-B row chunks:
  // rows q0 + i, cols h*D + [0, 64)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float inv = 1.f / sum[r];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) pw[(fq * 4 + r) * P_LD + dt * 16 + fr] = f32_to_bf16(o[dt][r] * inv);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);          // lgkmcnt(0): this wave's LDS writes landed
  __builtin_amdgcn_wave_barrier();
  attn_stamp(trace, trace_cap, 3);          // P V done (wave 0)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = j * 64 + lane, row = c >> 3, ch = c & 7;
    *reinterpret_cast<uint4*>(ctx + (long(b) * S + q0 + row) * (long(H) * D) + h * D + ch * 8) =
        *reinterpret_cast<const uint4*>(pw + row * P_LD + ch * 8);
  }
  if (trace != nullptr) {
    __builtin_amdgcn_s_waitcnt(0);          // this wave's stores acknowledged
    attn_stamp(trace, trace_cap, 4);
  }
}

// ---------------------------------------------------------------- long sequences
// S up to 512 (BERT-QA's 384, full 512) or any other S the fixed-S kernel
// above does not cover: a KV-block loop with an online softmax (running row
// max / sum, O rescaled per block), so registers hold one 64-key block of
// scores instead of the whole row and LDS holds one K / V block.  Keys past S
// in the last block are masked to -inf; query rows past S are never stored.
constexpr int FQB = 64, FKB = 64;

__global__ __launch_bounds__(256) void attention_flash_kernel(const uint16_t* __restrict__ qkv,
                                                              const float* __restrict__ mask_bias,
                                                              uint16_t* __restrict__ ctx, int S, int H, float scale,
                                                              long mask_bstride, long mask_qstride) {
  constexpr int VT_LD = FKB + 8, P_LD = FKB + 8;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[FKB * D];       // [key][64] swizzled
  __shared__ __attribute__((aligned(16))) uint16_t Vt[D * VT_LD];     // [d][key]
  __shared__ __attribute__((aligned(16))) uint16_t Ps[4 * 16 * P_LD]; // per-wave P / output strips

  const int qblocks = (S + FQB - 1) / FQB;
  const int bid = blockIdx.x;
  const int qb = bid % qblocks;
  const int h = (bid / qblocks) % H;
  const int b = bid / (qblocks * H);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const long row_stride = 3L * H * D;
  const uint16_t* base = qkv + long(b) * S * row_stride;

  const int q0 = qb * FQB + wid * 16;
  bf16x8 qf[2];
  const int qrow = min(q0 + fr, S - 1);            // rows past S load a valid row, never stored
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
    qf[kk] = *reinterpret_cast<const bf16x8*>(base + long(qrow) * row_stride + h * D + kk * 32 + fq * 8);

  float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, l[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint16_t* pw = Ps + wid * 16 * P_LD;
  const float* mrow = mask_bias ? mask_bias + long(b) * mask_bstride : nullptr;

  for (int k0 = 0; k0 < S; k0 += FKB) {
    // ---- stage this block's K (swizzled rows) and V (transposed); keys past S read key S-1
    for (int c = tid; c < FKB * 8; c += 256) {
      const int key = c >> 3, ch = c & 7;
      const int kg = min(k0 + key, S - 1);
      const uint4 kv = *reinterpret_cast<const uint4*>(base + long(kg) * row_stride + H * D + h * D + ch * 8);
      *reinterpret_cast<uint4*>(Ks + key * D + ((ch ^ (key & 7)) * 8)) = kv;
    }
    for (int blk = tid; blk < (FKB / 8) * 8; blk += 256) {
      const int kgrp = blk >> 3, ch = blk & 7;
      uint32_t w[8][4];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int kg = min(k0 + kgrp * 8 + k, S - 1);
        const uint4 v = *reinterpret_cast<const uint4*>(base + long(kg) * row_stride + 2 * H * D + h * D + ch * 8);
        w[k][0] = v.x; w[k][1] = v.y; w[k][2] = v.z; w[k][3] = v.w;
      }
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        uint32_t ov[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t lo = (d & 1) ? (w[2 * j][d >> 1] >> 16) : (w[2 * j][d >> 1] & 0xffffu);
          const uint32_t hi = (d & 1) ? (w[2 * j + 1][d >> 1] & 0xffff0000u) : (w[2 * j + 1][d >> 1] << 16);
          ov[j] = lo | hi;
        }
        *reinterpret_cast<uint4*>(Vt + (ch * 8 + d) * VT_LD + kgrp * 8) = make_uint4(ov[0], ov[1], ov[2], ov[3]);
      }
    }
    __syncthreads();
    // ---- scores of this block
    f32x4 sc[FKB / 16];
#pragma unroll
    for (int nt = 0; nt < FKB / 16; ++nt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int key = nt * 16 + fr;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = kk * 4 + fq;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + key * D + ((ch ^ (key & 7)) * 8));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[kk], kf, acc, 0, 0, 0);
      }
      sc[nt] = acc;
    }
    // ---- online softmax update (rows fq*4 + r, key k0 + nt*16 + fr)
    float bm[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int nt = 0; nt < FKB / 16; ++nt) {
      const int key = k0 + nt * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v;
        if (key < S) {
          const float mb = mrow ? mrow[long(min(q0 + fq * 4 + r, S - 1)) * mask_qstride + key] : 0.f;
          v = sc[nt][r] * scale + mb;
        } else {
          v = -INFINITY;
        }
        sc[nt][r] = v;
        bm[r] = fmaxf(bm[r], v);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) bm[r] = fmaxf(bm[r], __shfl_xor(bm[r], off, 64));
    float alpha[4], bs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mn = fmaxf(m[r], bm[r]);
      alpha[r] = __expf(m[r] - mn);            // exp(-inf) = 0 on the first block
      m[r] = mn;
      bs[r] = 0.f;
    }
#pragma unroll
    for (int nt = 0; nt < FKB / 16; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __expf(sc[nt][r] - m[r]);
        bs[r] += e;
        pw[(fq * 4 + r) * P_LD + nt * 16 + fr] = f32_to_bf16(e);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) bs[r] += __shfl_xor(bs[r], off, 64);
      l[r] = l[r] * alpha[r] + bs[r];
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] *= alpha[r];
    __builtin_amdgcn_s_waitcnt(0xc07f);       // this wave's P strip writes landed
    __builtin_amdgcn_wave_barrier();
    // ---- o += P V over the block's 64 keys
#pragma unroll
    for (int ks = 0; ks < FKB / 32; ++ks) {
      const bf16x8 pa = *reinterpret_cast<const bf16x8*>(pw + fr * P_LD + ks * 32 + fq * 8);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 vb = *reinterpret_cast<const bf16x8*>(Vt + (dt * 16 + fr) * VT_LD + ks * 32 + fq * 8);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[dt], 0, 0, 0);
      }
    }
    __syncthreads();                          // every wave is done with Ks / Vt before the next block
  }
  // ---- normalise and store (through the wave's strip for 16-B row chunks)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float inv = 1.f / l[r];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) pw[(fq * 4 + r) * P_LD + dt * 16 + fr] = f32_to_bf16(o[dt][r] * inv);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = j * 64 + lane, row = c >> 3, ch = c & 7;
    if (q0 + row < S)
      *reinterpret_cast<uint4*>(ctx + (long(b) * S + q0 + row) * (long(H) * D) + h * D + ch * 8) =
          *reinterpret_cast<const uint4*>(pw + row * P_LD + ch * 8);
  }
}

// -1: TFSERVE_ATTN_PLDS decides (default off); 0 / 1 forced (attention_set_plds)
int g_attn_plds = -1;
bool attn_plds() {
  static const bool env = [] {
    const char* e = getenv("TFSERVE_ATTN_PLDS");
    return e != nullptr && atoi(e) != 0;
  }();
  return g_attn_plds < 0 ? env : g_attn_plds != 0;
}

template <int S, int QB = qb_for(S)>
hipError_t launch_s(const uint16_t* qkv, const float* mb, uint16_t* ctx, int B, int H, float scale, long bs, long qs,
                    hipStream_t st) {
  static_assert(S % QB == 0, "attention tile");
  const int grid = B * H * (S / QB);
  if (attn_plds()) {
    constexpr int lds = (S * D + D * (S + 8) + (QB / 16) * 16 * (S + 8)) * 2;
    static_assert(lds <= 160 * 1024, "attention tile");
    hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&attention_plds_kernel<S, QB>), lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((attention_plds_kernel<S, QB>), dim3(grid), dim3(QB * 4), lds, st, qkv, mb, ctx, H, scale, bs,
                       qs, g_attn_trace, g_attn_trace_cap);
    return hipGetLastError();
  }
  constexpr int lds = (S * D + D * (S + 8)) * 2 + 1024;          // + the key mask's 1-KB DMA image
  static_assert(lds <= 160 * 1024, "attention tile");
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&attention_kernel<S, QB>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((attention_kernel<S, QB>), dim3(grid), dim3(QB * 4), lds, st, qkv, mb, ctx, H, scale, bs, qs,
                     g_attn_trace, g_attn_trace_cap);
  return hipGetLastError();
}

// query rows per workgroup at S = 128: TFSERVE_ATTN_QB (32 / 64 / 128) when
// set, else 128 (one workgroup per (batch, head): K / V staged once) when that
// still gives every CU a workgroup, 64 below (twice the workgroups for small
// batches).  b32 BERT-base: 10.2 vs 11.4 us per layer (profiles/round5/s41/).
int attn_qb(int BH) {
  static const int v = [] {
    const char* e = getenv("TFSERVE_ATTN_QB");
    return e ? atoi(e) : 0;
  }();
  return v ? v : (BH >= 256 ? 128 : 64);
}

}  // namespace

int attention_set_plds(int mode) {
  const int prev = g_attn_plds;
  g_attn_plds = mode < 0 ? -1 : (mode ? 1 : 0);
  return prev;
}

void attention_set_trace(long long* trace, int cap) {
  g_attn_trace = trace;
  g_attn_trace_cap = trace ? cap : 0;
}

hipError_t attention_launch(const uint16_t* qkv, const float* mask_bias, uint16_t* ctx, int B, int S, int H,
                            int Dh, float scale, long mask_bstride, long mask_qstride, hipStream_t st) {
  if (Dh != D) return hipErrorInvalidValue;
  const long bs = mask_bstride, qs = mask_qstride;
  switch (S) {
    case 64: return launch_s<64>(qkv, mask_bias, ctx, B, H, scale, bs, qs, st);
    case 128:
      // query rows per workgroup (TFSERVE_ATTN_QB: 32 / 64 / 128; experiments)
      switch (attn_qb(B * H)) {
        case 32: return launch_s<128, 32>(qkv, mask_bias, ctx, B, H, scale, bs, qs, st);
        case 128: return launch_s<128, 128>(qkv, mask_bias, ctx, B, H, scale, bs, qs, st);
        default: return launch_s<128>(qkv, mask_bias, ctx, B, H, scale, bs, qs, st);
      }
    case 192: return launch_s<192>(qkv, mask_bias, ctx, B, H, scale, bs, qs, st);
    case 256: return launch_s<256>(qkv, mask_bias, ctx, B, H, scale, bs, qs, st);
    default: {
      if (S <= 0 || S > kMaxAttentionSeq) return hipErrorInvalidValue;
      const long grid = long(B) * H * ((S + FQB - 1) / FQB);
      if (grid >= (1L << 31)) return hipErrorInvalidValue;
      hipLaunchKernelGGL(attention_flash_kernel, dim3(unsigned(grid)), dim3(256), 0, st, qkv, mask_bias, ctx, S, H,
                         scale, bs, qs);
      return hipGetLastError();
    }
  }
}

}  // namespace tfsk
