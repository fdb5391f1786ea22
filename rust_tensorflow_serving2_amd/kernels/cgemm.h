// Pipelined MFMA conv/GEMM (cgemm.hip): the fast path for 64-aligned operands.
#pragma once
#include "launch.h"

namespace tfsk {

// Config ids continue after the igemm ones so one `cfg` integer selects either
// kernel family: cgemm configs are kCGemmCfgBase .. kCGemmCfgBase + kNumCGemmConfigs - 1.
constexpr int kCGemmCfgBase = 32;
constexpr int kNumCGemmConfigs = 16;
// a second id range (after the halo ids): 2-wave and 3-deep variants
constexpr int kCGemmCfgBase2 = 64;
constexpr int kNumCGemmConfigs2 = 12;
// a third range: fragment-prefetch (PF) builds of 11 of the tiles above
constexpr int kCGemmPfCfgBase = 96;
constexpr int kNumCGemmPfConfigs = 11;
// a fourth range: v_mfma_f32_32x32x16_bf16 builds (wave tiles in 32x32 blocks)
constexpr int kCGemm32CfgBase = 112;
constexpr int kNumCGemm32Configs = 12;
// ids 124..137 are retired: the 32-deep k-tile builds (124..129) and the
// persistent multi-tile kernel (130..137) took 0 of 192 picks in the round-5
// tile table (ops/tuned_mi355x.json) and were removed in round 6
// a seventh range: the big-tile ping-pong GEMM (bgemm.hip; dense operands, no split-K fixup)
constexpr int kBGemmCfgBase = 140;
constexpr int kNumBGemmConfigs = 3;
inline bool cgemm_cfg_id(int cfg) {
  return (cfg >= kCGemmCfgBase && cfg < kCGemmCfgBase + kNumCGemmConfigs) ||
         (cfg >= kCGemmCfgBase2 && cfg < kCGemmCfgBase2 + kNumCGemmConfigs2) ||
         (cfg >= kCGemmPfCfgBase && cfg < kCGemmPfCfgBase + kNumCGemmPfConfigs) ||
         (cfg >= kCGemm32CfgBase && cfg < kCGemm32CfgBase + kNumCGemm32Configs) ||
         (cfg >= kBGemmCfgBase && cfg < kBGemmCfgBase + kNumBGemmConfigs);
}

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
// the 32x32x16 builds (cgemm32.hip), table index idx = cfg - kCGemm32CfgBase
hipError_t cgemm32_launch(const IGemmArgs& a, int a_mode, int idx, hipStream_t stream);
// the big-tile ping-pong builds (bgemm.hip), idx = cfg - kBGemmCfgBase
hipError_t bgemm_launch(const IGemmArgs& a, int a_mode, int idx, hipStream_t stream);
// the config can finish split-K in-kernel (IGemmArgs::counters)
bool cgemm_fixup_ok(int cfg);
// workgroups (= tiles) of a halo launch (its split-K counters)
long halo_tiles(const IGemmArgs& a, int cfg);

// Halo-tiled 3x3 stride-1 conv (halo.hip): an NHWC bf16 input with C % 64 == 0
// and the im2col weight layout ([Cout][9 * C]); the workgroup tile is a block
// of output pixels (TH x TW, picked by the launcher) x a BN slice of Cout.
// Config ids kHaloCfgBase .. + kNumHaloConfigs - 1; split-K splits the channel
// chunks (kt_per_split counts 64-channel chunks).
constexpr int kHaloCfgBase = 48;
constexpr int kNumHaloConfigs = 11;
// the same halo tiles with the fragment-prefetch step pipeline (PF)
constexpr int kHaloPfCfgBase = 80;
// the PF build of tile 4 (256x128, 8 waves) does not fit the register budget
// and is not instantiated: id 84 is not a config
constexpr int kHaloPfMissing = 4;
// the persistent halo kernel (halo.hip halo_persist_kernel): 128 pixels x 64
// channels, C == 64 only, the whole filter resident in LDS
constexpr int kHaloPersistCfg = 146;
inline bool halo_cfg_id(int cfg) {
  return (cfg >= kHaloCfgBase && cfg < kHaloCfgBase + kNumHaloConfigs) || cfg == kHaloPersistCfg ||
         (cfg >= kHaloPfCfgBase && cfg < kHaloPfCfgBase + kNumHaloConfigs && cfg != kHaloPfCfgBase + kHaloPfMissing);
}
bool halo_supported(const IGemmArgs& a);
int halo_config_bm(int cfg);
int halo_config_bn(int cfg);
hipError_t halo_launch(const IGemmArgs& a, int cfg, hipStream_t stream);

}  // namespace tfsk
