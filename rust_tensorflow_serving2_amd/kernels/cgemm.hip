// Pipelined MFMA conv / GEMM for MI355X (gfx950): bf16 operands, fp32 accumulate.
//
// C[M][N] = epilogue( A[M][K] * B[N][K]^T ), the same contract as igemm.hip, for
// the 64-aligned cases that make up almost all of ResNet-50 / BERT:
//   A dense row-major (K % 64 == 0), or the implicit im2col of an NHWC tensor
//   with C % 64 == 0, so one 64-deep k-tile is exactly one filter tap x 64
//   channels;  B = weights [Cout][ldb].
//
// Why a second kernel: rocprofv3 PMC of igemm on the ResNet 3x3 layers showed
// ~90 SALU+VALU instructions per 16 MFMAs and a vmcnt(0) drain every k-tile
// (SQ_ACTIVE_INST_ANY 44 %, SQ_WAIT_ANY 41 %, MFMA busy 11-16 % of wave
// cycles).  This kernel is built so the steady-state k-tile costs little more
// than its MFMAs:
//   * S-deep ring of direct-to-LDS DMAs (buffer_load ... lds): the wait before
//     tile t is a counted vmcnt((S-2) * pieces) — never a drain — followed by a
//     bare s_barrier;
//   * every per-lane DMA offset is precomputed once (voffset) and the k-tile
//     advance is a wave-uniform scalar (soffset): no VALU address math per tile;
//   * im2col padding = one precomputed tap-validity bit mask per DMA row
//     (3 VALU per piece), the tap walk runs in SGPRs, and the buffer
//     descriptor is rebased by the top/left padding so every in-image offset is
//     non-negative; invalid taps read through an out-of-range voffset (zeros);
//   * the loop is unrolled by S, so ring slots and all LDS fragment offsets
//     are compile-time immediates;
//   * LDS rows are 128 B with 16-B chunks XOR-swizzled by (row & 7): the DMA
//     lane writes slot l&7 of row l>>3 from source chunk (l&7)^(l>>3), the
//     ds_read_b128 fragment reads undo it (conflict-free);
//   * 4 or 8 waves per workgroup, each owning a WM x WN sub-tile of
//     v_mfma_f32_16x16x32_bf16 accumulators; bijective XCD-aware tile remap +
//     GROUP_M ordering; epilogue staged through LDS as fp32 for coalesced
//     16-B bias/residual/activation/store row chunks (residual prefetched into
//     registers before the K loop).
#include "cgemm_impl.h"

namespace tfsk {

namespace {

using namespace gemm;
using cgemm_impl::launch_cfg;

// Config table (tile BM x BN, wave grid, ring depth).  LDS per workgroup =
// S * (BM + BN) * 128 B (or the fp32 epilogue tile if larger).
constexpr int kAll = kNumCGemmConfigs + kNumCGemmConfigs2;
constexpr int kBM[kAll] = {128, 128, 64, 128, 64, 256, 128, 128, 64, 256, 64, 64, 128, 128, 128, 64,
                           64, 64, 64, 128, 64, 128, 64, 64, 256, 256, 128, 128};
constexpr int kBN[kAll] = {128, 128, 128, 64, 64, 128, 256, 128, 256, 64, 64, 128, 64, 96, 96, 96,
                           64, 64, 64, 64, 128, 64, 128, 64, 192, 144, 96, 96};

// PF config ids kCGemmPfCfgBase + i: the fragment-prefetch build of table index kPfOf[i]
// (the 8-wave 256 x 128 / 128 x 256 / 256 x 192 tiles spill with two fragment sets: not built)
constexpr int kPfOf[kNumCGemmPfConfigs] = {0, 2, 3, 4, 7, 9, 10, 11, 12, 13, 23};

// 32x32x16 MFMA builds (ids kCGemm32CfgBase + i): BM x BN, wave grid, ring depth
constexpr int k32BM[kNumCGemm32Configs] = {64, 64, 128, 128, 64, 128, 256, 256, 128, 64, 128, 256};
constexpr int k32BN[kNumCGemm32Configs] = {64, 64, 128, 64, 128, 256, 128, 64, 128, 128, 64, 192};

// big-tile ping-pong builds (ids kBGemmCfgBase + i, bgemm.hip)
constexpr int kBBM[kNumBGemmConfigs] = {256, 256, 256};
constexpr int kBBN[kNumBGemmConfigs] = {256, 128, 192};

// config id -> index into the tables (all id ranges; the 32x32 range indexes k32BM / k32BN)
int cfg_index(int cfg) {
  if (cfg >= kBGemmCfgBase) return cfg - kBGemmCfgBase;
  if (cfg >= kCGemm32CfgBase) return cfg - kCGemm32CfgBase;
  if (cfg >= kCGemmPfCfgBase) return kPfOf[cfg - kCGemmPfCfgBase];
  return cfg < kCGemmCfgBase2 ? cfg - kCGemmCfgBase : kNumCGemmConfigs + (cfg - kCGemmCfgBase2);
}

template <int AM>
hipError_t launch_mode_pf(const IGemmArgs& a, int idx, hipStream_t s) {
  switch (idx) {
    case 0: return launch_cfg<128, 128, 2, 2, 3, AM, true>(a, s);
    case 2: return launch_cfg<64, 128, 2, 2, 4, AM, true>(a, s);
    case 3: return launch_cfg<128, 64, 2, 2, 4, AM, true>(a, s);
    case 4: return launch_cfg<64, 64, 2, 2, 4, AM, true>(a, s);
    case 7: return launch_cfg<128, 128, 2, 4, 4, AM, true>(a, s);
    case 9: return launch_cfg<256, 64, 4, 1, 3, AM, true>(a, s);
    case 10: return launch_cfg<64, 64, 2, 2, 2, AM, true>(a, s);
    case 11: return launch_cfg<64, 128, 2, 2, 2, AM, true>(a, s);
    case 12: return launch_cfg<128, 64, 2, 2, 2, AM, true>(a, s);
    case 13: return launch_cfg<128, 96, 2, 2, 3, AM, true>(a, s);
    case 23: return launch_cfg<64, 64, 2, 2, 3, AM, true>(a, s);
    default: return hipErrorInvalidValue;
  }
}

template <int AM>
hipError_t launch_mode(const IGemmArgs& a, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_cfg<128, 128, 2, 2, 3, AM>(a, s);   // 96 KB, wave 64x64
    case 1: return launch_cfg<128, 128, 2, 2, 2, AM>(a, s);   // 64 KB (2 WG/CU)
    case 2: return launch_cfg<64, 128, 2, 2, 4, AM>(a, s);    // 96 KB, wave 32x64
    case 3: return launch_cfg<128, 64, 2, 2, 4, AM>(a, s);    // 96 KB, wave 64x32
    case 4: return launch_cfg<64, 64, 2, 2, 4, AM>(a, s);     // 64 KB, wave 32x32
    case 5: return launch_cfg<256, 128, 4, 2, 3, AM>(a, s);   // 144 KB, 8 waves of 64x64
    case 6: return launch_cfg<128, 256, 2, 4, 3, AM>(a, s);   // 144 KB, 8 waves of 64x64
    case 7: return launch_cfg<128, 128, 2, 4, 4, AM>(a, s);   // 128 KB, 8 waves of 64x32
    case 8: return launch_cfg<64, 256, 1, 4, 3, AM>(a, s);    // 120 KB, wave 64x64
    case 9: return launch_cfg<256, 64, 4, 1, 3, AM>(a, s);    // 120 KB, wave 64x64
    // double-buffered, small LDS: several workgroups per CU overlap each
    // other's prologue / barrier / epilogue latency
    case 10: return launch_cfg<64, 64, 2, 2, 2, AM>(a, s);    // 32 KB (5 WG/CU)
    case 11: return launch_cfg<64, 128, 2, 2, 2, AM>(a, s);   // 48 KB (3 WG/CU)
    case 12: return launch_cfg<128, 64, 2, 2, 2, AM>(a, s);   // 48 KB (3 WG/CU)
    // 96-wide tiles: N = 768 (BERT-base hidden) is 8 of them, so an M = 4096
    // GEMM is exactly 256 tiles of 128 x 96 -- one per CU -- where 128 x 128
    // leaves a quarter of the CUs idle (192 tiles) and 128 x 64 needs 1.5 waves
    case 13: return launch_cfg<128, 96, 2, 2, 3, AM>(a, s);   // 84 KB, wave 64x48
    case 14: return launch_cfg<128, 96, 2, 2, 4, AM>(a, s);   // 112 KB
    case 15: return launch_cfg<64, 96, 2, 2, 3, AM>(a, s);    // 60 KB, wave 32x48
    // two waves per workgroup: a 64x64 tile as two 64x32 wave tiles reads 24 KB
    // of LDS fragments per k-step instead of the 32 KB four 32x32 waves read
    // (whose LDS reads take as long as their MFMAs at 256 B/clk)
    case 16: return launch_cfg<64, 64, 1, 2, 2, AM>(a, s);    // 32 KB, wave 64x32
    case 17: return launch_cfg<64, 64, 1, 2, 3, AM>(a, s);    // 48 KB
    case 18: return launch_cfg<64, 64, 2, 1, 3, AM>(a, s);    // 48 KB, wave 32x64
    case 19: return launch_cfg<128, 64, 2, 1, 2, AM>(a, s);   // 48 KB, wave 64x64
    case 20: return launch_cfg<64, 128, 1, 2, 2, AM>(a, s);   // 48 KB, wave 64x64
    case 21: return launch_cfg<128, 64, 2, 1, 3, AM>(a, s);   // 72 KB, wave 64x64
    case 22: return launch_cfg<64, 128, 1, 2, 3, AM>(a, s);   // 72 KB, wave 64x64
    case 23: return launch_cfg<64, 64, 2, 2, 3, AM>(a, s);    // 48 KB, wave 32x32
    // 8 waves of 64x96 (BERT's 2304 / 3072-wide projections at M = 4096: 192 /
    // 256 tiles, one per CU); 112 KB ring, epilogue in two 128-row passes
    case 24: return launch_cfg<256, 192, 4, 2, 2, AM>(a, s);
    // 8 waves of 32x144: BERT-base's QKV projection (4096 x 2304) is exactly
    // 256 tiles of 256 x 144, one per CU, where 256 x 192 leaves 64 CUs idle
    // (192 tiles); 150 KB, a 3-slot ring, the fp32 epilogue in one pass
    case 25: return launch_cfg<256, 144, 8, 1, 3, AM>(a, s);
    // 8 waves of 32x48 on the 128 x 96 tile (N = 768 at M = 4096: 256 tiles):
    // two waves per SIMD to cover the DMA latency the 4-wave 128 x 96 builds
    // (ids 45 / 46) leave exposed over K = 3072; 4- and 5-slot rings
    case 26: return launch_cfg<128, 96, 4, 2, 4, AM>(a, s);   // 112 KB
    case 27: return launch_cfg<128, 96, 4, 2, 5, AM>(a, s);   // 140 KB
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

int cgemm_config_bm(int cfg) {
  return cfg >= kBGemmCfgBase ? kBBM[cfg_index(cfg)]
         : cfg >= kCGemm32CfgBase ? k32BM[cfg_index(cfg)] : kBM[cfg_index(cfg)];
}
int cgemm_config_bn(int cfg) {
  return cfg >= kBGemmCfgBase ? kBBN[cfg_index(cfg)]
         : cfg >= kCGemm32CfgBase ? k32BN[cfg_index(cfg)] : kBN[cfg_index(cfg)];
}

bool cgemm_fixup_ok(int cfg) {
  if (cfg >= kBGemmCfgBase) return false;            // no in-kernel fixup (bgemm)
  // the in-kernel split-K fixup needs the whole fp32 tile in LDS at once (one pass)
  return size_t(cgemm_config_bm(cfg)) * (cgemm_config_bn(cfg) + 4) * 4 <= 160 * 1024;
}

bool cgemm_supported(const IGemmArgs& a, int a_mode) {
  if (a.K <= 0 || a.K % KT || a.ldb % 8 || a.ldb < a.K) return false;
  if (a.N % 8 || a.ldc % 8 || (a.residual && a.ldr % 8)) return false;   // 16-B epilogue chunks only
  if (a.M >= (1 << 23)) return false;   // fdiv() row-index decomposition is exact below 2^23
  if (a_mode == kADense) return a.lda % 8 == 0 && a.lda >= a.K;
  if (a_mode == kAIm2col)
    return a.C % KT == 0 && a.KH * a.KW <= 32 && a.K == a.KH * a.KW * a.C &&
           a.a_bytes + int64_t(a.PT * a.W + a.PL) * a.C * 2 < 0x7ffffff0LL;
  if (a_mode == kAC4)
    return a.C == 4 && a.KW == 8 && a.KH % 2 == 0 && a.K == a.KH * 32 && a.PT == 0 && a.PL == 0 &&
           a.H >= (a.Ho - 1) * a.SH + a.KH && a.W >= (a.Wo - 1) * a.SW + a.KW;
  if (a_mode == kADual)
    return a.a2 && a.K1 > 0 && a.K1 % KT == 0 && a.lda % 8 == 0 && a.lda >= a.K1 && a.C % KT == 0 &&
           a.K == a.K1 + a.C && a.KH == 1 && a.KW == 1 && a.PT == 0 && a.PL == 0 && a.a2_bytes < 0x7ffffff0LL;
  return false;
}


hipError_t cgemm_launch(const IGemmArgs& a, int a_mode, int cfg, hipStream_t s) {
  if (!cgemm_cfg_id(cfg) || !cgemm_supported(a, a_mode)) return hipErrorInvalidValue;
  if (cfg >= kBGemmCfgBase) return bgemm_launch(a, a_mode, cfg_index(cfg), s);
  if (cfg >= kCGemm32CfgBase) return cgemm32_launch(a, a_mode, cfg_index(cfg), s);
  if (cfg >= kCGemmPfCfgBase) {
    const int idx = cfg_index(cfg);
    switch (a_mode) {
      case kAIm2col: return launch_mode_pf<1>(a, idx, s);
      case kADual: return launch_mode_pf<2>(a, idx, s);
      case kAC4: return launch_mode_pf<3>(a, idx, s);
      default: return launch_mode_pf<0>(a, idx, s);
    }
  }
  cfg = cfg_index(cfg);
  switch (a_mode) {
    case kAIm2col: return launch_mode<1>(a, cfg, s);
    case kADual: return launch_mode<2>(a, cfg, s);
    case kAC4: return launch_mode<3>(a, cfg, s);
    default: return launch_mode<0>(a, cfg, s);
  }
}

}  // namespace tfsk
