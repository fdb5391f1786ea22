// Pipelined MFMA conv/GEMM (cgemm.hip): the fast path for 64-aligned operands.
#pragma once
#include "launch.h"

namespace tfsk {

// Config ids continue after the igemm ones so one `cfg` integer selects either
// kernel family: cgemm configs are kCGemmCfgBase .. kCGemmCfgBase + kNumCGemmConfigs - 1.
constexpr int kCGemmCfgBase = 32;
constexpr int kNumCGemmConfigs = 16;

// Operand requirements (else cgemm_launch returns hipErrorInvalidValue):
//   dense (a_mode kADense): K % 64 == 0, lda % 8 == 0;
//   im2col (kAIm2col): C % 64 == 0 (a k-tile is one filter tap x 64 channels), KH*KW <= 32;
//   stem (kAC4): zero-bordered bf16 RGBA input (no conv padding), KW == 8, KH even;
//   dual (kADual): see IGemmArgs::a2;
//   weights: ldb % 8 == 0, ldb >= K;  epilogue: N, ldc (and ldr) % 8 == 0.
bool cgemm_supported(const IGemmArgs& a, int a_mode);
int cgemm_config_bm(int cfg);
int cgemm_config_bn(int cfg);
hipError_t cgemm_launch(const IGemmArgs& a, int a_mode, int cfg, hipStream_t stream);

}  // namespace tfsk
