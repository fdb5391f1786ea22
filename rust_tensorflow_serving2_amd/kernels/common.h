// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace tfsk {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef uint16_t bf16_t;   // storage type on the host-visible side

constexpr int kWave = 64;
constexpr int kNumXcd = 8;

enum Act : int { kActNone = 0, kActRelu = 1, kActGeluTanh = 2, kActGeluErf = 3, kActTanh = 4 };

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
  return __uint_as_float(uint32_t(v) << 16);
}

// round-to-nearest-even f32 -> bf16 (NaN stays NaN): gfx950's
// v_cvt_pk_bf16_f32.  (The integer form -- add 0x7fff + lsb, NaN check --
// compiled to ~12 instructions and a branch per value: a third of the
// attention softmax's VALU work.)
__device__ __forceinline__ bf16_t f32_to_bf16(float f) { return __builtin_bit_cast(bf16_t, static_cast<__bf16>(f)); }

// 1 / (1 + exp(-2u)): one v_exp_f32 + one v_rcp_f32 (both ~1 ulp; the
// epilogues round to bf16). 0.5 x (1 + tanh u) == x * sigm2(u) and
// tanh x == 2 sigm2(x) - 1, so GELU-tanh / tanh cost two transcendental ops
// instead of ocml tanhf's branchy expansion (which made BERT's FFN1 epilogue
// a visible share of the GEMM). exp overflow -> rcp(inf) = 0: correct limits.
__device__ __forceinline__ float sigm2(float u) { return __builtin_amdgcn_rcpf(1.f + __expf(-2.f * u)); }

// GELU-tanh as x * sigm2(u) with the constants folded into one polynomial in
// x^2 and exp2: x * rcp(1 + exp2(x (k0 + k1 x^2))), k0 = -2 sqrt(2/pi) log2(e),
// k1 = 0.044715 k0.  5 plain VALU ops + v_exp + v_rcp per element against 8 +
// 2 for the textbook form (the FFN1 epilogue of BERT, 12.6 M elements per
// forward, is VALU-bound behind the last MFMA: 32.6 vs 28.9 us without the
// activation, profiles/round5/s41/blt.log).  Limits: x -> -inf gives
// rcp(inf) = 0, x -> +inf gives x.
__device__ __forceinline__ float gelu_tanh(float x) {
  const float t = fmaf(x * x, -0.1029432395800235f, -2.302208198144325f);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * t));
}

__device__ __forceinline__ float apply_act(float x, int act) {
  switch (act) {
    case kActRelu: return x > 0.f ? x : 0.f;
    case kActGeluTanh: return gelu_tanh(x);
    case kActGeluErf: return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
    case kActTanh: return 2.f * sigm2(x) - 1.f;
    default: return x;
  }
}

// Compile-time activation (epilogues dispatch on the runtime code once, then
// run branch-free loops).
template <int ACT>
__device__ __forceinline__ float act_fn(float x) {
  if constexpr (ACT == kActRelu) {
    return x > 0.f ? x : 0.f;
  } else if constexpr (ACT == kActGeluTanh) {
    return gelu_tanh(x);
  } else if constexpr (ACT == kActGeluErf) {
    return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
  } else if constexpr (ACT == kActTanh) {
    return 2.f * sigm2(x) - 1.f;
  } else {
    return x;
  }
}

// Bijective XCD-aware remap (MI355X: 8 XCDs, blocks dealt round-robin):
// blocks that share an XCD get a contiguous range of logical tile ids, so
// neighbouring tiles (which share A rows / B columns) hit the same L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / kNumXcd, r = nwg % kNumXcd;
  const int xcd = bid % kNumXcd, idx = bid / kNumXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace tfsk
