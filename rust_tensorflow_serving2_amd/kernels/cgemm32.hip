// 32x32x16 MFMA builds of the pipelined conv / GEMM kernel (config ids
// kCGemm32CfgBase + idx; cgemm_launch dispatches here).  Separate translation
// unit so the two families compile in parallel.
#include "cgemm_impl.h"

namespace tfsk {

namespace {

using cgemm_impl::launch_cfg;

template <int AM>
hipError_t launch_mode32(const IGemmArgs& a, int idx, hipStream_t s) {
  switch (idx) {
    case 0: return launch_cfg<64, 64, 2, 2, 4, AM, false, 32>(a, s);     // 64 KB, waves 32x32
    case 1: return launch_cfg<64, 64, 1, 2, 3, AM, false, 32>(a, s);     // 48 KB, waves 64x32
    case 2: return launch_cfg<128, 128, 2, 2, 3, AM, false, 32>(a, s);   // 96 KB, waves 64x64
    case 3: return launch_cfg<128, 64, 2, 2, 4, AM, false, 32>(a, s);    // 96 KB, waves 64x32
    case 4: return launch_cfg<64, 128, 2, 2, 4, AM, false, 32>(a, s);    // 96 KB, waves 32x64
    case 5: return launch_cfg<128, 256, 2, 4, 3, AM, false, 32>(a, s);   // 144 KB, 8 waves of 64x64
    case 6: return launch_cfg<256, 128, 4, 2, 3, AM, false, 32>(a, s);   // 144 KB, 8 waves of 64x64
    case 7: return launch_cfg<256, 64, 4, 1, 3, AM, false, 32>(a, s);    // 120 KB, waves 64x64
    case 8: return launch_cfg<128, 128, 2, 4, 4, AM, false, 32>(a, s);   // 128 KB, 8 waves of 64x32
    case 9: return launch_cfg<64, 128, 2, 2, 2, AM, false, 32>(a, s);    // 48 KB (3 WG/CU)
    case 10: return launch_cfg<128, 64, 2, 2, 2, AM, false, 32>(a, s);   // 48 KB (3 WG/CU)
    case 11: return launch_cfg<256, 192, 4, 2, 2, AM, false, 32>(a, s);  // 112 KB, 8 waves of 64x96
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t cgemm32_launch(const IGemmArgs& a, int a_mode, int idx, hipStream_t s) {
  switch (a_mode) {
    case kAIm2col: return launch_mode32<1>(a, idx, s);
    case kADual: return launch_mode32<2>(a, idx, s);
    case kAC4: return launch_mode32<3>(a, idx, s);
    default: return launch_mode32<0>(a, idx, s);
  }
}

}  // namespace tfsk
