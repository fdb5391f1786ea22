// Host-side launchers of the HIP kernels (torch-free; bindings.cpp wraps them).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tfsk {

// Implicit-GEMM geometry.  GEMM view: C[M][N] = A[M][K] * B[N][K]^T where
//   A = im2col(x) of an NHWC input (or a dense row-major matrix),
//   B = weights [Cout][ldb] with k = (kh*KW + kw)*C + c (zero padded to ldb).
struct IGemmArgs {
  const void* a;        // bf16 NHWC / dense [M][lda] (fp32 NHWC for the stem mode)
  const uint16_t* b;    // bf16 [N][ldb]
  int M, N, K;
  int lda, ldb;
  // conv geometry (a_mode 1/2)
  int H, W, C, KH, KW, SH, SW, PT, PL, Ho, Wo;
  // epilogue
  const float* bias;    // [N] or nullptr
  const uint16_t* residual;  // bf16 [M][ldr] or nullptr
  int ldr;
  int act;
  void* out;            // bf16 or f32 [M][ldc]
  int ldc;
  int out_f32;
  float alpha;          // scale applied to the accumulator before bias
  // split-K: gridDim.y = splits; split s covers k-tiles [s*kt_per_split, ...).
  // With splits > 1 the kernel stores raw fp32 partials to ws[s][M][N] and
  // splitk_reduce applies the epilogue.
  int splits;
  int kt_per_split;
  float* ws;
  // byte extents of A and B (buffer-descriptor bounds for the direct-to-LDS
  // loads; must be < 2^31)
  int64_t a_bytes;
  int64_t b_bytes;
  // dual-source A (cgemm only): k < K1 reads the dense `a` [M][lda], k >= K1
  // reads `a2`, an NHWC tensor sampled by a 1x1 / stride (SH, SW) conv with the
  // geometry fields above (C = its channels).  One GEMM then computes
  // conv1x1(a) + conv1x1_strided(a2) — a ResNet bottleneck's expand conv and
  // its projection shortcut (K-concatenated weights, summed bias).
  const void* a2;
  int64_t a2_bytes;
  int K1;
  // halo conv (halo.hip): output pixel block per workgroup (set by the launcher);
  // TI > 1: the block is TI whole images (small feature maps: fewer M-tiles,
  // so each weight byte a workgroup streams serves TI images)
  int TH, TW, TI;
  // post-activation output (cgemm / halo / split-K reduce): out2 = act2(v *
  // scale2 + shift2) per output channel, v = the epilogue value stored to
  // `out` — a ResNet v2 block's sum and the next block's pre-activation
  // relu(bn(sum)) from ONE kernel.  out == nullptr: only out2 is written.
  void* out2;
  const float* scale2;
  const float* shift2;
  int act2;
  // split-K without the reduce launch (cgemm / halo, inside HIP graphs): one
  // arrival counter per tile (zero between launches); the last slice to arrive
  // sums the slabs and runs the epilogue, then re-zeroes its counter
  int* counters;
  // profiling (scripts/wg_trace.py): per-workgroup wall-clock stamps, 8 int64
  // per workgroup (blockIdx.y * gridDim.x + blockIdx.x), nullptr in production
  long long* trace;
  int trace_cap;        // workgroups the trace buffer holds
  // 1: the fp32-staged epilogue even where the one-pass bf16 one applies
  // (A/B only: TFSERVE_EPI_F32=1, set by the launchers)
  int epi_f32;
  // deferred LayerNorm (cgemm dense, one K slice; graph/fused.py
  // defer_layernorm).  st_out: [M][ceil(N / BN)][2] fp32 -- per (row, column
  // block) (sum, sum of squares) of the stored bf16 outputs, each slot written
  // once by plain stores (nothing to zero between launches).  a_st / r_st:
  // such partials (a_parts / r_parts per row) of A's rows (length K) / of the
  // residual's rows (length N), tensors whose LayerNorm was never stored: the
  // epilogue applies it -- v = rstd_a (acc - mean_a a_colsum[n]) + bias (the
  // LN's gamma folded into the weights, beta into the bias, a_colsum = the
  // per-column sums of the folded weights) and residual = (r - mean_r) rstd_r
  // r_gamma + r_beta.  All nullptr: a plain epilogue.
  float* st_out;
  const float* a_st;
  const float* a_colsum;
  int a_parts;
  float a_eps;
  const float* r_st;
  const float* r_gamma;
  const float* r_beta;
  int r_parts;
  float r_eps;
};

// Per-device pool of zeroed split-K arrival counters: a launch captured into a
// HIP graph takes a slice for good (its replays are ordered on its stream, and
// each tile's last arriver re-zeroes its counter); an eager launch takes the
// next slice of a ring.  nullptr when the pool is missing or exhausted: the
// caller then uses the separate reduce launch.
int* splitk_counters(int n, hipStream_t s);
// Allocates and zeroes this device's pool (no-op while `s` is capturing).
void splitk_counters_prepare(hipStream_t s);
// Captured slices taken on this thread while `owner` != 0 belong to that
// owner; splitk_counters_release(owner) returns them to the pool (call it when
// the graph captured under the token is destroyed).  Returns the ints freed.
// Released slices are not reused at once: a replay of the dropped graph may
// still be queued on a lane, or a lane abandoned mid-count may have left a
// counter non-zero.  Reclamation is stream-ordered, not timed: the streams the
// owner's graph replays on (the capturing stream, recorded automatically, plus
// any added with splitk_counters_add_stream) each get a fence event at the
// first splitk_counters_reclaim() after the release; once every fence has
// completed the slices are zeroed on the first of those streams (the lane's
// own), and once that memset has completed they join the free list.  A fence
// behind a hung kernel never completes, so a hung lane's slices are never
// handed out again.  splitk_counters_reclaim never blocks (call it outside any
// capture on this thread; the runtime calls it before each capture).
void splitk_counters_set_owner(int64_t owner);
void splitk_counters_add_stream(int64_t owner, hipStream_t s);
int64_t splitk_counters_release(int64_t owner);
int64_t splitk_counters_reclaim();
int64_t splitk_counters_pending();
int64_t splitk_counters_captured_in_use();

// kAStem7x7x3: fp32 NHWC input with C == 3 and a 7-wide filter (the ResNet
// stem) — compile-time geometry for the operand gather.
// kAC4: bf16 NHWC with exactly 4 channels (RGB + zero pad, written by
// ingest_c4) and KW <= 8; k = kh*32 + kw*4 + c, so one 16-B operand chunk is
// two 8-B filter taps and kh = k >> 5 (no division in the gather).
enum AMode : int { kADense = 0, kAIm2col = 1, kAStemF32 = 2, kAStem7x7x3 = 3, kAC4 = 4, kADual = 5 };

// fp32 NHWC with C <= 4 channels -> bf16 NHWC with 4 channels (zero padded).
hipError_t ingest_c4_launch(const float* x, uint16_t* y, int64_t pixels, int C, hipStream_t stream);

// Same into a zero-bordered [N][Hp][Wp][4] buffer (image placed at row pt, column pl).
hipError_t ingest_c4_pad_launch(const float* x, uint16_t* y, int N, int H, int W, int C, int Hp, int Wp, int pt,
                               int pl, hipStream_t stream);

// Sum split-K partial slabs and apply the epilogue (bias, residual, act, store).
hipError_t splitk_reduce_launch(const IGemmArgs& args, hipStream_t stream);

// Tile configs (BM x BN, DMA ring depth): 0..3 = 128x128, 128x64, 64x128,
// 64x64 double-buffered; 4 = 128x128x3, 5 = 64x64x4, 6 = 128x64x3, 7 = 64x128x3;
// wide: 8 = 64x256, 9 = 256x64, 10 = 128x256, 11 = 256x128 (dense / im2col only)
// deep k-tiles (BK): 12 = 64x64/128, 13 = 64x64/256, 14 = 64x128/128, 15 = 128x64/128, 16 = 128x128/128
constexpr int kNumIGemmConfigs = 17;
int igemm_config_bm(int cfg);
int igemm_config_bn(int cfg);
int igemm_config_stages(int cfg);
int igemm_config_bk(int cfg);
hipError_t igemm_launch(const IGemmArgs& args, int a_mode, int cfg, hipStream_t stream);

// Fused ResNet stem (stem.hip): fp32 [N][H][W][C<=4] -> 7x7/2 conv (weights
// [cout][ldw] bf16, k = kh*32 + kw*4 + c, cout in {16,32,48,64}) + bias + act
// -> 3x3/2 max pool (+ optional scale/shift/act after the max) -> bf16
// [N][Hp][Wp][cout].  pt/pl: conv padding; ppt/ppl: pool padding.
hipError_t stem_pool_launch(const void* x, bool x_bf16, const uint16_t* w, int ldw, const float* bias, uint16_t* y,
                            int N, int H, int W, int C, int cout, int pt, int pl, int Hc, int Wc, int ppt, int ppl,
                            int Hp, int Wp, int act, const float* pscale, const float* pshift, int pact,
                            hipStream_t s);
// Two chained 1x1 convs in one launch (chain.hip): y1 = act1(x w1^T + b1 + res),
// y2 = act2(y1 w2^T + b2); (K1, N1, N2) in conv_chain_supported().
bool conv_chain_supported(int K1, int N1, int N2);
hipError_t conv_chain_launch(const uint16_t* x, const uint16_t* w1, int ldw1, const float* b1, const uint16_t* res,
                             uint16_t* y1, const uint16_t* w2, int ldw2, const float* b2, uint16_t* y2, int M, int K1,
                             int N1, int N2, int act1, int act2, hipStream_t s);
// NHWC bf16 max-pool (TF SAME/VALID padding given explicitly).  With `scale`
// (and `shift`): y = act(max * scale[c] + shift[c]) — a folded inference
// BatchNorm (+ ReLU when act == 1) applied after the pooling.
hipError_t maxpool_nhwc_launch(const uint16_t* x, uint16_t* y, int N, int H, int W, int C,
                               int KH, int KW, int SH, int SW, int PT, int PL, int Ho, int Wo,
                               hipStream_t stream, const float* scale = nullptr, const float* shift = nullptr,
                               int act = 0);
// Mean over H,W of NHWC bf16 -> [N][C] (bf16).
hipError_t global_avgpool_nhwc_launch(const uint16_t* x, uint16_t* y, int N, int HW, int C,
                                      hipStream_t stream);
// Row softmax (fp32 in) -> probs f32 + argmax int64 (the classifier head).
// GlobalAvgPool + dense + softmax/argmax (misc.hip): x [M][HW][K] bf16 (NHWC
// feature map, K % 256 == 0), w [Np][K] bf16, bias [Np] f32, ws = f32
// workspace of classifier_head_ws_floats(M, K, Np); probs [M][N] f32 and
// classes [M] for the first N <= Np columns.
// `counter` (a zeroed int, re-zeroed by the kernel; nullptr: three launches):
// M <= 16 rows and HW <= 64 run as ONE launch (misc.hip head_small_kernel),
// which also stores the rows into pinned host buffers `probs_h` / `classes_h`
// when given (a serving lane's output rows: no D2H copies after the graph).
// Returns hipErrorNotSupported when host rows are asked of the 3-launch path.
hipError_t classifier_head_launch(const uint16_t* x, const uint16_t* w, const float* bias, float* ws,
                                  float* probs, int64_t* classes, int M, int HW, int K, int Np, int N,
                                  hipStream_t s, int* counter = nullptr, float* probs_h = nullptr,
                                  int64_t* classes_h = nullptr);
size_t classifier_head_ws_floats(int M, int K, int Np);
// The shapes classifier_head_launch runs as ONE launch (given a counter): the
// only path that can store host rows.  Callers decide on host rows with it.
bool classifier_head_one_launch(int M, int HW, int K, int Np, int N);
// BERT head: probs[r] = softmax(x[r] @ w^T + bias) over N <= 16 labels (x fp32)
hipError_t dense_softmax_launch(const float* x, int ldx, const uint16_t* w, int ldw, const float* bias,
                                float* probs, int rows, int N, int K, hipStream_t s);
// (one - m) * scale over a key mask (int32 when is_int, else f32) -> f32
hipError_t key_mask_adder_launch(const void* m, int is_int, float one, float scale, float* out, int64_t n,
                                 hipStream_t s);
hipError_t softmax_argmax_launch(const void* logits, int in_bf16, float* probs, int64_t* classes,
                                 int rows, int cols, long ld, hipStream_t stream);
// fp32 -> bf16 cast (vectorized).
hipError_t cast_f32_bf16_launch(const float* x, uint16_t* y, int64_t n, hipStream_t stream);
hipError_t cast_bf16_f32_launch(const uint16_t* x, float* y, int64_t n, hipStream_t stream);
// `bytes` (16-B multiple, 16-B aligned) of pinned host memory -> device, as a
// kernel (system-scope loads): the small-bucket graphs' input copy
// TFSERVE_EPI_F32 (read once): force the fp32-staged GEMM / conv epilogue
int epi_f32_env();
hipError_t h2d_rows_launch(const void* host, void* dev, int64_t bytes, hipStream_t stream);

// LayerNorm over the last dim (bf16 in/out, f32 gamma/beta), optional fused residual add:
// y = LN(x + r) ; if `sum_out` != nullptr the pre-norm sum is also written.
hipError_t layernorm_launch(const uint16_t* x, const uint16_t* r, const float* gamma, const float* beta,
                            uint16_t* y, int rows, int cols, float eps, hipStream_t stream);
// Embedding: y[t] = LN(word[ids[t]] + pos[t % S] + type[tt[t]]) (bf16 tables, f32 LN params;
// int32 ids, out-of-range ids add a zero row; type_ids / pos may be null; hidden % 8 == 0, <= 2048)
hipError_t embed_ln_launch(const int* ids, const int* type_ids, const uint16_t* word,
                           const uint16_t* pos, const uint16_t* type, const float* gamma,
                           const float* beta, uint16_t* y, int tokens, int seq, int hidden,
                           int vocab, int ntypes, float eps, hipStream_t stream);
// GEMM + residual + LayerNorm over whole rows (kernels/lngemm.hip):
// y[M][N] = LN(x[M][K] w[N][K]^T + bias + r[M][N]) * gamma + beta, bf16 in/out,
// f32 bias / gamma / beta; N in {512, 768, 1024}, K % 128 == 0; one workgroup
// per `bm` rows (16 / 32 / 64).  r, bias may be null.
struct LnGemmArgs {
  const uint16_t* x = nullptr;   // [M][ldx]
  const uint16_t* w = nullptr;   // fragment-major [N/16][K/32][64 lanes][8] (lngemm.hip w_off)
  const float* bias = nullptr;
  const uint16_t* r = nullptr;   // [M][N]
  const float* gamma = nullptr;
  const float* beta = nullptr;
  uint16_t* y = nullptr;         // [M][N]
  int M = 0, N = 0, K = 0, ldx = 0;
  float eps = 1e-12f;
};
bool lngemm_supported(int M, int N, int K, int bm);
hipError_t lngemm_launch(const LnGemmArgs& a, int bm, hipStream_t stream);
constexpr int kMaxAttentionSeq = 4096;
// Fused multi-head attention over a packed QKV buffer [B*S][3*H*D] (bf16):
// ctx[b,q,h,:] = softmax(Q K^T * scale + mask[b*bstride + q*qstride + key]) V
// (additive f32 mask; strides 0 broadcast, e.g. BERT's [B,1,S,S] adder or a [B,S] key mask)
hipError_t attention_launch(const uint16_t* qkv, const float* mask_bias, uint16_t* ctx, int B, int S,
                            int H, int D, float scale, long mask_bstride, long mask_qstride,
                            hipStream_t stream);
// per-workgroup phase stamps of the following fixed-S attention launches
// (entry, staged, softmax, P V, stored; [7] = CU id); nullptr: off
void attention_set_trace(long long* trace, int cap);
// fixed-S attention layout: 1 = P through LDS (previous kernel), 0 = P in
// registers (default), -1 = env TFSERVE_ATTN_PLDS; returns the previous mode
int attention_set_plds(int mode);

}  // namespace tfsk
