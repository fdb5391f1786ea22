// 32-deep k-tile builds of the pipelined conv / GEMM kernel (config ids
// kCGemmKt32CfgBase + idx; cgemm_launch dispatches here).  A ring slot holds
// half the bytes of a 64-deep one, so the same LDS keeps twice the k-tiles in
// flight: the 256 x 192 tile (BERT-base's QKV / FFN1 projections at M = 4096,
// one tile per CU) fits 2 slots of 64-deep k-tiles (112 KB: ONE tile in
// flight while the other computes, DMA-latency bound: ~2 us per 64-deep step
// for ~0.64 us of MFMA per SIMD) but 5 slots of 32-deep ones (140 KB: 4 in
// flight).  The 64-B LDS rows use their own conflict-free swizzle
// (cgemm_impl.h lds_swz).  Own translation unit: compiles in parallel.
#include "cgemm_impl.h"

namespace tfsk {

namespace {

using cgemm_impl::launch_cfg;

template <int AM>
hipError_t launch_mode_kt32(const IGemmArgs& a, int idx, hipStream_t s) {
  switch (idx) {
    case 0: return launch_cfg<256, 192, 4, 2, 5, AM, false, 16, 32>(a, s);   // 140 KB, 8 waves of 64x96
    case 1: return launch_cfg<256, 192, 4, 2, 5, AM, false, 32, 32>(a, s);   // same, 32x32x16 MFMA
    case 2: return launch_cfg<256, 128, 4, 2, 6, AM, false, 16, 32>(a, s);   // 144 KB, 8 waves of 64x64
    case 3: return launch_cfg<128, 256, 2, 4, 6, AM, false, 32, 32>(a, s);   // 144 KB, 8 waves of 64x64
    case 4: return launch_cfg<128, 128, 2, 2, 6, AM, false, 16, 32>(a, s);   // 96 KB, waves 64x64
    case 5: return launch_cfg<128, 96, 2, 2, 8, AM, false, 16, 32>(a, s);    // 112 KB, waves 64x48
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t cgemm_kt32_launch(const IGemmArgs& a, int a_mode, int idx, hipStream_t s) {
  switch (a_mode) {
    case kAIm2col: return launch_mode_kt32<1>(a, idx, s);
    case kADual: return launch_mode_kt32<2>(a, idx, s);
    case kAC4: return hipErrorInvalidValue;            // stem layout: 64-deep k-tiles only
    default: return launch_mode_kt32<0>(a, idx, s);
  }
}

}  // namespace tfsk
