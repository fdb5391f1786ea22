// torch bindings of the gfx950 kernels (`_hip`).  (ROCm torch exposes HIP
// devices as "cuda": guards/streams use the MasqueradingAsCUDA variants.)  Every op launches on the
// caller's current HIP stream, allocates nothing inside the launch function
// beyond the output tensor (so callers can capture them in HIP graphs with
// pre-allocated outputs via the `out=` forms), and validates shapes on the host
// before anything touches the GPU.
#include <cstdlib>
#include <algorithm>
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "launch.h"
#include "cgemm.h"

namespace {

using torch::Tensor;

hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e));
}

// Launch with optional split-K: raw fp32 slabs in a workspace + reduce/epilogue kernel.
// cfg < kNumIGemmConfigs: igemm.hip (any operand mode); cfg in [kCGemmCfgBase,
// kCGemmCfgBase + kNumCGemmConfigs): the pipelined cgemm.hip kernel (64-aligned operands).
bool is_cgemm_cfg(int64_t cfg) {
  return cfg >= 0 && cfg < (1 << 20) && tfsk::cgemm_cfg_id(int(cfg));
}

// halo-tiled 3x3 stride-1 conv configs (halo.hip)
bool is_halo_cfg(int64_t cfg) {
  return cfg >= 0 && cfg < (1 << 20) && tfsk::halo_cfg_id(int(cfg));
}

hipError_t launch_any(const tfsk::IGemmArgs& a, int a_mode, int64_t cfg, hipStream_t st) {
  if (is_halo_cfg(cfg)) return tfsk::halo_launch(a, int(cfg), st);
  return is_cgemm_cfg(cfg) ? tfsk::cgemm_launch(a, a_mode, int(cfg), st) : tfsk::igemm_launch(a, a_mode, int(cfg), st);
}

// Split-K finishing in-kernel (the last slice of a tile sums the slabs and
// runs the epilogue; no reduce launch).  TFSERVE_SPLITK_FIXUP: "1" always,
// "0" never.  Otherwise the serving runtime decides per batch bucket while it
// tunes and captures (set_splitk_fixup: on for the small buckets, whose few
// workgroups each run a long K loop -- b1 0.371-0.374 vs 0.391-0.394 ms per
// replay -- off for the large ones, where the write-through slab traffic cost
// more than the reduce launch when every small launch used it: b32 0.816-0.824 vs 0.780-0.786 ms; per bucket: 0.771-0.773 vs 0.781-0.794,
// profiles/round4/s13), and outside that launches of fewer than
// kFixupAutoTiles tiles use it.
constexpr long kFixupAutoTiles = 128;
// per thread: the serving runtime sets it around ONE bucket's tuning + capture
// on the capturing thread; eager launches of other threads (another
// servable's warm-up / tuning) keep the default rule and never take eager
// ring slices under a capture's mode
thread_local int g_fixup_override = -1;
int split_fixup_mode() {
  const char* v = std::getenv("TFSERVE_SPLITK_FIXUP");
  if (v && v[0] == '1') return 1;
  if (v && v[0] == '0') return 0;
  if (g_fixup_override >= 0) return g_fixup_override;
  return 2;
}

// scripts/wg_trace.py: per-workgroup phase stamps of the next GEMM / conv
// launches (a device int64 buffer of 8 per workgroup; None turns it off)
long long* g_trace = nullptr;
int g_trace_cap = 0;

void run_igemm(tfsk::IGemmArgs& a, int a_mode, int64_t cfg, int64_t splits, const Tensor& like, hipStream_t st) {
  a.trace = g_trace;
  a.trace_cap = g_trace_cap;
  TORCH_CHECK((cfg >= 0 && cfg < tfsk::kNumIGemmConfigs) || is_cgemm_cfg(cfg) || is_halo_cfg(cfg),
              "bad tile config ", cfg);
  TORCH_CHECK(!is_cgemm_cfg(cfg) || tfsk::cgemm_supported(a, a_mode),
              "tile config ", cfg, " needs 64-aligned operands (K % 64, C % 64)");
  TORCH_CHECK(!is_halo_cfg(cfg) || (a_mode == tfsk::kAIm2col && tfsk::halo_supported(a)),
              "halo config ", cfg, " needs a 3x3 stride-1 conv with C % 64 == 0");
  // split-K granule: 64-deep k-tiles, or 64-channel chunks (9 taps each) for the halo conv
  const int nk = is_halo_cfg(cfg) ? a.C / 64 : (a.K + 63) / 64;
  if (splits > nk) splits = nk;
  if (splits <= 1) {
    a.splits = 1;
    a.kt_per_split = nk;
    a.ws = nullptr;
    TORCH_CHECK(launch_any(a, a_mode, cfg, st) == hipSuccess, "conv/GEMM launch failed");
    return;
  }
  const int per = (nk + splits - 1) / splits;
  splits = (nk + per - 1) / per;
  Tensor ws = torch::empty({splits * int64_t(a.M) * a.N}, like.options().dtype(at::kFloat));
  a.splits = int(splits);
  a.kt_per_split = per;
  a.ws = ws.data_ptr<float>();
  // With the fixup on (split_fixup_mode: launches under kFixupAutoTiles tiles by default) cgemm /
  // halo finish split-K in-kernel (the last slice of each tile reduces): one
  // launch instead of two; eager launches (autotuning) then use the fixup too,
  // so the tuner times the split-K candidates as the graph runs them.
  // Otherwise, or when no counters are left, a separate reduce launch.
  a.counters = nullptr;
  const int fixup = split_fixup_mode();
  if (fixup != 0 && a.N % 8 == 0 && ((is_cgemm_cfg(cfg) && tfsk::cgemm_fixup_ok(int(cfg))) || is_halo_cfg(cfg))) {
    long tiles = 0;
    if (is_halo_cfg(cfg)) {
      tiles = tfsk::halo_tiles(a, int(cfg));
    } else {
      const int bm = tfsk::cgemm_config_bm(int(cfg)), bn = tfsk::cgemm_config_bn(int(cfg));
      tiles = long((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
    }
    if (tiles > 0 && tiles < (1L << 24) && (fixup == 1 || tiles < kFixupAutoTiles)) {
      tfsk::splitk_counters_prepare(st);
      a.counters = tfsk::splitk_counters(int(tiles), st);
    }
  }
  TORCH_CHECK(launch_any(a, a_mode, cfg, st) == hipSuccess, "conv/GEMM (split-K) launch failed");
  if (a.counters == nullptr)
    TORCH_CHECK(tfsk::splitk_reduce_launch(a, st) == hipSuccess, "split-K reduce launch failed");
}

void need(const Tensor& t, at::ScalarType st, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

bool aligned16(const Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; }

const uint16_t* bf16p(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }

// Post-activation output (ResNet v2): out2 = act2(y * scale + shift) per output
// channel, written by the same GEMM epilogue.  post_only: `y` itself receives
// the post-activated values (the raw sum is not stored).  cgemm / halo configs
// (or split-K, whose reduce applies the epilogue) only.
void set_post(tfsk::IGemmArgs& a, const c10::optional<Tensor>& scale, const c10::optional<Tensor>& shift,
              int64_t act2, const c10::optional<Tensor>& out2, bool post_only, const Tensor& y, int64_t cfg,
              int64_t splits, int cout) {
  if (!scale.has_value()) {
    TORCH_CHECK(!shift.has_value() && !out2.has_value() && !post_only, "post output needs post_scale");
    return;
  }
  TORCH_CHECK(shift.has_value(), "post_scale needs post_shift");
  need(*scale, at::kFloat, "post_scale");
  need(*shift, at::kFloat, "post_shift");
  TORCH_CHECK(scale->numel() == cout && shift->numel() == cout, "post scale / shift must have Cout entries");
  TORCH_CHECK(aligned16(*scale) && aligned16(*shift), "post scale / shift must be 16-B aligned");
  TORCH_CHECK(cfg >= tfsk::kCGemmCfgBase || splits > 1, "the post-activation output needs a cgemm / halo config");
  a.scale2 = scale->data_ptr<float>();
  a.shift2 = shift->data_ptr<float>();
  a.act2 = int(act2);
  if (post_only) {
    TORCH_CHECK(!out2.has_value(), "post_only writes the post output to `out`");
    a.out2 = y.data_ptr();
    a.out = nullptr;
  } else {
    TORCH_CHECK(out2.has_value(), "dual output needs out2");
    TORCH_CHECK(out2->scalar_type() == y.scalar_type() && out2->numel() == y.numel() && out2->is_contiguous(),
                "out2 must match the output");
    a.out2 = out2->data_ptr();
  }
}
uint16_t* bf16p_mut(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

// x: NHWC bf16 (or fp32 when stem=true), w: [Cout][ldb] bf16, bias: [Cout] f32
Tensor conv2d(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias,
              const c10::optional<Tensor>& residual, int64_t KH, int64_t KW, int64_t SH, int64_t SW,
              int64_t PT, int64_t PB, int64_t PL, int64_t PR, int64_t act, int64_t cfg,
              const c10::optional<Tensor>& out, bool out_f32, int64_t splits,
              const c10::optional<Tensor>& post_scale, const c10::optional<Tensor>& post_shift, int64_t post_act,
              const c10::optional<Tensor>& out2, bool post_only) {
  const bool stem = x.scalar_type() == at::kFloat;
  need(x, stem ? at::kFloat : at::kBFloat16, "x");
  need(w, at::kBFloat16, "w");
  TORCH_CHECK(x.dim() == 4, "x must be NHWC");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = (H + PT + PB - KH) / SH + 1, Wo = (W + PL + PR - KW) / SW + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty conv output");
  const int Cout = w.size(0), ldb = w.size(1);
  const bool c4 = !stem && C == 4;
  TORCH_CHECK(!c4 || KW <= 8, "4-channel (RGBA) conv supports KW <= 8");
  const int K = c4 ? KH * 32 : KH * KW * C;   // c4 weights: [Cout][kh][8 taps][4 ch]
  TORCH_CHECK(ldb >= K && ldb % 8 == 0, "weight rows must hold K=", K, " (padded to a multiple of 8)");
  int a_mode;
  if (stem) {
    a_mode = (C == 3 && KH == 7 && KW == 7) ? tfsk::kAStem7x7x3 : tfsk::kAStemF32;
  } else if (c4) {
    a_mode = tfsk::kAC4;
  } else {
    TORCH_CHECK(C % 8 == 0, "conv input channels must be a multiple of 8 (got ", C, ")");
    a_mode = (KH == 1 && KW == 1 && SH == 1 && SW == 1 && PT == 0 && PL == 0) ? tfsk::kADense : tfsk::kAIm2col;
  }
  Tensor y = out.has_value() ? *out
                             : torch::empty({N, Ho, Wo, Cout}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  need(y, out_f32 ? at::kFloat : at::kBFloat16, "out");
  TORCH_CHECK(y.numel() == int64_t(N) * Ho * Wo * Cout, "out has the wrong size");
  tfsk::IGemmArgs a{};
  a.a = x.data_ptr();
  a.b = bf16p(w);
  a.a_bytes = x.numel() * x.element_size();
  a.b_bytes = w.numel() * 2;
  TORCH_CHECK(a.a_bytes < 0x7ffffff0LL && a.b_bytes < 0x7ffffff0LL, "conv operands must be < 2 GiB");
  a.M = N * Ho * Wo; a.N = Cout; a.K = K; a.lda = C; a.ldb = ldb;
  a.H = H; a.W = W; a.C = C; a.KH = KH; a.KW = KW; a.SH = SH; a.SW = SW; a.PT = PT; a.PL = PL;
  a.Ho = Ho; a.Wo = Wo;
  if (bias.has_value()) {
    need(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == Cout, "bias size");
    a.bias = bias->data_ptr<float>();
  }
  if (residual.has_value()) {
    need(*residual, at::kBFloat16, "residual");
    TORCH_CHECK(residual->numel() == y.numel(), "residual shape must match the output");
    a.residual = bf16p(*residual);
    a.ldr = Cout;
  }
  a.act = act; a.out = y.data_ptr(); a.ldc = Cout; a.out_f32 = out_f32; a.alpha = 1.f;
  set_post(a, post_scale, post_shift, post_act, out2, post_only, y, cfg, splits, Cout);
  run_igemm(a, a_mode, cfg, splits, x, cur_stream(x));
  return y;
}

// ResNet bottleneck tail in one GEMM: act(conv1x1(h) + conv1x1_stride(x) + bias)
// with w = [Cout][C_h + C_x] (expand weights | projection weights).
// h: NHWC [N][Ho][Wo][C_h] bf16 (dense rows), x: NHWC [N][H][W][C_x] bf16
// sampled at (ho*SH, wo*SW).  cgemm configs only (C_h, C_x % 64 == 0).
Tensor conv2d_dual(const Tensor& h, const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias,
                   int64_t SH, int64_t SW, int64_t act, int64_t cfg, const c10::optional<Tensor>& out, int64_t splits,
                   const c10::optional<Tensor>& post_scale, const c10::optional<Tensor>& post_shift,
                   int64_t post_act, const c10::optional<Tensor>& out2, bool post_only) {
  need(h, at::kBFloat16, "h");
  need(x, at::kBFloat16, "x");
  need(w, at::kBFloat16, "w");
  TORCH_CHECK(h.dim() == 4 && x.dim() == 4 && h.size(0) == x.size(0), "conv2d_dual: NHWC h and x, same batch");
  TORCH_CHECK(is_cgemm_cfg(cfg), "conv2d_dual needs a cgemm tile config");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(h.device());
  const int N = h.size(0), Ho = h.size(1), Wo = h.size(2), C1 = h.size(3);
  const int H = x.size(1), W = x.size(2), C2 = x.size(3);
  TORCH_CHECK(SH >= 1 && SW >= 1 && (H - 1) / SH + 1 == Ho && (W - 1) / SW + 1 == Wo,
              "conv2d_dual: x sampled at stride (SH, SW) must give h's spatial size");
  const int Cout = w.size(0), ldb = w.size(1);
  TORCH_CHECK(ldb >= C1 + C2 && ldb % 8 == 0, "conv2d_dual: weights must hold K = C_h + C_x");
  Tensor y = out.has_value() ? *out : torch::empty({N, Ho, Wo, Cout}, h.options());
  need(y, at::kBFloat16, "out");
  TORCH_CHECK(y.numel() == int64_t(N) * Ho * Wo * Cout, "out has the wrong size");
  tfsk::IGemmArgs a{};
  a.a = h.data_ptr(); a.a_bytes = h.numel() * 2;
  a.a2 = x.data_ptr(); a.a2_bytes = x.numel() * 2;
  a.b = bf16p(w); a.b_bytes = w.numel() * 2;
  TORCH_CHECK(a.a_bytes < 0x7ffffff0LL && a.a2_bytes < 0x7ffffff0LL && a.b_bytes < 0x7ffffff0LL,
              "conv2d_dual operands must be < 2 GiB");
  a.M = N * Ho * Wo; a.N = Cout; a.K = C1 + C2; a.K1 = C1; a.lda = C1; a.ldb = ldb;
  a.H = H; a.W = W; a.C = C2; a.KH = 1; a.KW = 1; a.SH = SH; a.SW = SW; a.PT = 0; a.PL = 0; a.Ho = Ho; a.Wo = Wo;
  if (bias.has_value()) {
    need(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == Cout, "bias size");
    a.bias = bias->data_ptr<float>();
  }
  a.act = act; a.out = y.data_ptr(); a.ldc = Cout; a.out_f32 = 0; a.alpha = 1.f;
  set_post(a, post_scale, post_shift, post_act, out2, post_only, y, cfg, splits, Cout);
  run_igemm(a, tfsk::kADual, cfg, splits, h, cur_stream(h));
  return y;
}

// x: [M][K] bf16 (any leading dims), w: [N][ldb] bf16 -> [.., N]
Tensor linear(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias,
              const c10::optional<Tensor>& residual, int64_t act, int64_t cfg, bool out_f32, double alpha,
              const c10::optional<Tensor>& out, int64_t splits) {
  // x: contiguous, or a row-strided 2-D view (x[r][k] at r * lda + k; e.g.
  // BERT's pooler reads every sequence's first token straight from [B, S, H])
  const bool strided = !x.is_contiguous();
  if (strided) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1 &&
                    x.stride(0) >= x.size(1) && x.stride(0) % 8 == 0,
                "x must be contiguous or a row-strided 2-D bf16 view");
  } else {
    need(x, at::kBFloat16, "x");
  }
  need(w, at::kBFloat16, "w");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int K = x.size(-1);
  const int M = x.numel() / K;
  const int lda = strided ? int(x.stride(0)) : K;
  const int N = w.size(0), ldb = w.size(1);
  TORCH_CHECK(ldb >= K && K % 8 == 0 && ldb % 8 == 0, "linear: K must be a multiple of 8 and fit in w");
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  Tensor y = out.has_value() ? *out : torch::empty(sizes, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  need(y, out_f32 ? at::kFloat : at::kBFloat16, "out");
  TORCH_CHECK(y.numel() == int64_t(M) * N, "out has the wrong size");
  tfsk::IGemmArgs a{};
  a.a = x.data_ptr(); a.b = bf16p(w);
  a.a_bytes = M > 0 ? (int64_t(M - 1) * lda + K) * 2 : 0;
  a.b_bytes = w.numel() * 2;
  TORCH_CHECK(a.a_bytes < 0x7ffffff0LL && a.b_bytes < 0x7ffffff0LL, "linear operands must be < 2 GiB");
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb;
  if (bias.has_value()) {
    need(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == N, "bias size");
    a.bias = bias->data_ptr<float>();
  }
  if (residual.has_value()) {
    need(*residual, at::kBFloat16, "residual");
    TORCH_CHECK(residual->numel() == y.numel(), "residual shape must match the output");
    a.residual = bf16p(*residual);
    a.ldr = N;
  }
  a.act = act; a.out = y.data_ptr(); a.ldc = N; a.out_f32 = out_f32; a.alpha = float(alpha);
  run_igemm(a, tfsk::kADense, cfg, splits, x, cur_stream(x));
  return y;
}


// Deferred-LayerNorm GEMM (graph/fused.py defer_layernorm): y = epilogue(x @
// w^T) where the rows of x (a_st) and / or of the residual (r_st) are sums
// whose LayerNorm was never stored -- their statistics come along as [M][P][2]
// (sum, sum sq) partials and the epilogue applies the normalisation (x's via
// the gamma-folded weights w, the beta-folded bias and a_colsum = per-column
// sums of w; the residual's via r_gamma / r_beta) -- and, with stats, y's own
// row partials are returned for the next consumer.  cgemm configs (not the
// persistent ones), one K slice.  Returns {y, y's partials (empty without stats)}.
std::vector<Tensor> linear_lnx(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias,
                               const c10::optional<Tensor>& residual, int64_t act, int64_t cfg, bool out_f32,
                               const c10::optional<Tensor>& out, const c10::optional<Tensor>& a_st,
                               const c10::optional<Tensor>& a_colsum, double a_eps,
                               const c10::optional<Tensor>& r_st, const c10::optional<Tensor>& r_gamma,
                               const c10::optional<Tensor>& r_beta, double r_eps, bool stats) {
  need(x, at::kBFloat16, "x");
  need(w, at::kBFloat16, "w");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int K = x.size(-1);
  const int M = x.numel() / K;
  const int N = w.size(0), ldb = w.size(1);
  TORCH_CHECK(ldb >= K && K % 64 == 0 && ldb % 8 == 0 && N % 8 == 0,
              "linear_lnx: K % 64 == 0 (fitting in w), N % 8 == 0");
  TORCH_CHECK(is_cgemm_cfg(cfg) && !(cfg >= tfsk::kBGemmCfgBase && cfg < tfsk::kBGemmCfgBase + tfsk::kNumBGemmConfigs),
              "linear_lnx: a cgemm tile config");
  TORCH_CHECK(!(stats && out_f32), "linear_lnx: row statistics of bf16 outputs only");
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  Tensor y = out.has_value() ? *out : torch::empty(sizes, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  need(y, out_f32 ? at::kFloat : at::kBFloat16, "out");
  TORCH_CHECK(y.numel() == int64_t(M) * N, "out has the wrong size");
  auto parts_of = [&](const Tensor& t, const char* what) {
    need(t, at::kFloat, what);
    TORCH_CHECK(t.dim() == 3 && t.size(0) == M && t.size(2) == 2 && t.size(1) >= 1,
                "linear_lnx: ", what, " must be [M][parts][2]");
    return int(t.size(1));
  };
  auto vec_n = [&](const c10::optional<Tensor>& t, const char* what) {
    TORCH_CHECK(t.has_value(), "linear_lnx: ", what, " missing");
    need(*t, at::kFloat, what);
    TORCH_CHECK(t->numel() == N && aligned16(*t), "linear_lnx: ", what, " must be N floats, 16-B aligned");
    return t->data_ptr<float>();
  };
  tfsk::IGemmArgs a{};
  a.a = x.data_ptr(); a.b = bf16p(w);
  a.a_bytes = int64_t(M) * K * 2;
  a.b_bytes = w.numel() * 2;
  TORCH_CHECK(a.a_bytes < 0x7ffffff0LL && a.b_bytes < 0x7ffffff0LL, "linear_lnx operands must be < 2 GiB");
  a.M = M; a.N = N; a.K = K; a.lda = K; a.ldb = ldb;
  if (bias.has_value()) {
    need(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == N, "bias size");
    a.bias = bias->data_ptr<float>();
  }
  if (residual.has_value()) {
    need(*residual, at::kBFloat16, "residual");
    TORCH_CHECK(residual->numel() == y.numel(), "residual shape must match the output");
    a.residual = bf16p(*residual);
    a.ldr = N;
  }
  if (a_st.has_value()) {
    a.a_parts = parts_of(*a_st, "a_st");
    a.a_st = a_st->data_ptr<float>();
    a.a_colsum = vec_n(a_colsum, "a_colsum");
    a.a_eps = float(a_eps);
  }
  if (r_st.has_value()) {
    TORCH_CHECK(residual.has_value(), "linear_lnx: r_st normalises the residual: give one");
    a.r_parts = parts_of(*r_st, "r_st");
    a.r_st = r_st->data_ptr<float>();
    a.r_gamma = vec_n(r_gamma, "r_gamma");
    a.r_beta = vec_n(r_beta, "r_beta");
    a.r_eps = float(r_eps);
  }
  Tensor st;
  if (stats) {
    const int bn = tfsk::cgemm_config_bn(int(cfg));
    st = torch::empty({M, (N + bn - 1) / bn, 2}, x.options().dtype(at::kFloat));
    a.st_out = st.data_ptr<float>();
  } else {
    st = torch::empty({0}, x.options().dtype(at::kFloat));
  }
  a.act = act; a.out = y.data_ptr(); a.ldc = N; a.out_f32 = out_f32; a.alpha = 1.f;
  run_igemm(a, tfsk::kADense, cfg, 1, x, cur_stream(x));
  return {y, st};
}

Tensor dense_softmax(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, int64_t n) {
  need(x, at::kFloat, "x");
  need(w, at::kBFloat16, "w");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && w.size(1) >= x.size(1) && w.size(0) >= n && n >= 1 && n <= 16,
              "dense_softmax: x [B, K] f32, w [>= n, >= K] bf16, 1 <= n <= 16");
  TORCH_CHECK(x.size(1) % 4 == 0 && w.size(1) % 4 == 0, "dense_softmax: K % 4 == 0");
  const float* b = nullptr;
  if (bias.has_value()) {
    need(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() >= n, "bias size");
    b = bias->data_ptr<float>();
  }
  Tensor probs = torch::empty({x.size(0), n}, x.options());
  TORCH_CHECK(tfsk::dense_softmax_launch(x.data_ptr<float>(), int(x.size(1)), bf16p(w), int(w.size(1)), b,
                                         probs.data_ptr<float>(), int(x.size(0)), int(n), int(x.size(1)),
                                         cur_stream(x)) == hipSuccess, "dense_softmax launch failed");
  return probs;
}

Tensor key_mask_adder(const Tensor& m, double one, double scale) {
  TORCH_CHECK(m.is_cuda() && m.is_contiguous() && (m.scalar_type() == at::kInt || m.scalar_type() == at::kFloat),
              "key mask must be a contiguous int32 / f32 GPU tensor");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(m.device());
  Tensor out = torch::empty(m.sizes(), m.options().dtype(at::kFloat));
  TORCH_CHECK(tfsk::key_mask_adder_launch(m.data_ptr(), m.scalar_type() == at::kInt, float(one), float(scale),
                                          out.data_ptr<float>(), m.numel(), cur_stream(m)) == hipSuccess,
              "key_mask_adder launch failed");
  return out;
}

Tensor maxpool(const Tensor& x, int64_t KH, int64_t KW, int64_t SH, int64_t SW, int64_t PT, int64_t PB,
               int64_t PL, int64_t PR, const c10::optional<Tensor>& out, const c10::optional<Tensor>& post_scale,
               const c10::optional<Tensor>& post_shift, int64_t post_act) {
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "maxpool: NHWC with C % 8 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = (H + PT + PB - KH) / SH + 1, Wo = (W + PL + PR - KW) / SW + 1;
  Tensor y = out.has_value() ? *out : torch::empty({N, Ho, Wo, C}, x.options());
  need(y, at::kBFloat16, "out");
  TORCH_CHECK(y.numel() == int64_t(N) * Ho * Wo * C, "out has the wrong size");
  const float* sc = nullptr;
  const float* sh = nullptr;
  if (post_scale.has_value()) {
    TORCH_CHECK(post_shift.has_value(), "post_scale needs post_shift");
    need(*post_scale, at::kFloat, "post_scale");
    need(*post_shift, at::kFloat, "post_shift");
    TORCH_CHECK(post_scale->numel() == C && post_shift->numel() == C, "post scale / shift must have C entries");
    sc = post_scale->data_ptr<float>();
    sh = post_shift->data_ptr<float>();
  }
  check(tfsk::maxpool_nhwc_launch(bf16p(x), bf16p_mut(y), N, H, W, C, KH, KW, SH, SW, PT, PL, Ho, Wo,
                                  cur_stream(x), sc, sh, int(post_act)), "maxpool");
  return y;
}

// ResNet stem: conv 7x7/2 (+bias, act) -> max pool 3x3/2 (+post) in one kernel
// (stem.hip).  x: fp32 NHWC request with C <= 4 (or that request converted to
// bf16 on ingest, csrc/ingest.h); w: [cout][ldw] bf16 in the padded-RGBA order
// of the c4 stem ([kh][8 taps][4 ch]).
Tensor stem_pool(const Tensor& x, const Tensor& w, const Tensor& bias, int64_t PT, int64_t PB, int64_t PL, int64_t PR,
                 int64_t act, int64_t PPT, int64_t PPB, int64_t PPL, int64_t PPR,
                 const c10::optional<Tensor>& post_scale, const c10::optional<Tensor>& post_shift, int64_t post_act) {
  const bool xb16 = x.scalar_type() == at::kBFloat16;
  need(x, xb16 ? at::kBFloat16 : at::kFloat, "x");
  need(w, at::kBFloat16, "w");
  need(bias, at::kFloat, "bias");
  TORCH_CHECK(x.dim() == 4 && x.size(3) >= 1 && x.size(3) <= 4, "stem_pool: x must be NHWC with C <= 4");
  TORCH_CHECK(w.dim() == 2 && w.size(0) % 16 == 0 && w.size(0) >= 16 && w.size(0) <= 64 && w.size(1) >= 224 &&
              w.size(1) % 8 == 0, "stem_pool: w must be [cout in 16..64 step 16][>= 224, % 8]");
  TORCH_CHECK(bias.numel() == w.size(0), "stem_pool: bias must have cout entries");
  TORCH_CHECK(PT >= 0 && PB >= 0 && PL >= 0 && PR >= 0 && PPT >= 0 && PPT <= 2 && PPL >= 0 && PPL <= 2 &&
              PPB >= 0 && PPR >= 0, "stem_pool: bad padding");
  TORCH_CHECK(w.device() == x.device() && bias.device() == x.device(), "stem_pool: tensors on different devices");
  Tensor xin = x;
  if (xb16 && x.numel() % 2) {
    // the bf16 path reads whole aligned dwords: an odd element count's last
    // pixel reads 2 B past the tensor, which must still lie in its storage;
    // otherwise the kernel reads a copy with one element of padding (the
    // serving path's ingest buffers are padded, so it never copies)
    const int64_t avail = int64_t(x.storage().nbytes()) - int64_t(x.storage_offset()) * 2;
    if (avail < x.numel() * 2 + 2 || !x.is_contiguous()) {
      Tensor padded = torch::zeros({x.numel() + 1}, x.options());
      padded.narrow(0, 0, x.numel()).copy_(x.reshape({-1}));
      xin = padded.narrow(0, 0, x.numel()).view(x.sizes());
    }
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), cout = w.size(0);
  const int Hc = (H + PT + PB - 7) / 2 + 1, Wc = (W + PL + PR - 7) / 2 + 1;
  TORCH_CHECK(Hc >= 1 && Wc >= 1, "stem_pool: input smaller than the filter");
  const int Hp = (Hc + PPT + PPB - 3) / 2 + 1, Wp = (Wc + PPL + PPR - 3) / 2 + 1;
  TORCH_CHECK(Hp >= 1 && Wp >= 1, "stem_pool: conv output smaller than the pool window");
  Tensor y = torch::empty({N, Hp, Wp, cout}, x.options().dtype(at::kBFloat16));
  const float* sc = nullptr;
  const float* sh = nullptr;
  if (post_scale.has_value()) {
    TORCH_CHECK(post_shift.has_value(), "post_scale needs post_shift");
    need(*post_scale, at::kFloat, "post_scale");
    need(*post_shift, at::kFloat, "post_shift");
    TORCH_CHECK(post_scale->numel() == cout && post_shift->numel() == cout, "post scale / shift must have cout entries");
    sc = post_scale->data_ptr<float>();
    sh = post_shift->data_ptr<float>();
  }
  check(tfsk::stem_pool_launch(xin.data_ptr(), xb16, bf16p(w), int(w.size(1)), bias.data_ptr<float>(), bf16p_mut(y), N,
                               H, W, C, cout, int(PT), int(PL), Hc, Wc, int(PPT), int(PPL), Hp, Wp, int(act), sc, sh,
                               int(post_act), cur_stream(x)), "stem_pool");
  return y;
}

// A bottleneck's expand 1x1 (+ shortcut, act) and the next bottleneck's
// reduce 1x1 (+ act) as one kernel (chain.hip): returns (y1, y2), NHWC bf16.
std::vector<Tensor> conv_chain(const Tensor& x, const Tensor& w1, const Tensor& b1,
                               const c10::optional<Tensor>& residual, int64_t act1, const Tensor& w2,
                               const Tensor& b2, int64_t act2) {
  need(x, at::kBFloat16, "x");
  need(w1, at::kBFloat16, "w1");
  need(w2, at::kBFloat16, "w2");
  need(b1, at::kFloat, "b1");
  need(b2, at::kFloat, "b2");
  TORCH_CHECK(x.dim() == 4, "conv_chain: x must be NHWC");
  const int K1 = x.size(3), N1 = w1.size(0), N2 = w2.size(0);
  TORCH_CHECK(w1.dim() == 2 && w2.dim() == 2 && w1.size(1) >= K1 && w2.size(1) >= N1 && w1.size(1) % 8 == 0 &&
                  w2.size(1) % 8 == 0, "conv_chain: w1 [N1][>= K1], w2 [N2][>= N1]");
  TORCH_CHECK(tfsk::conv_chain_supported(K1, N1, N2), "conv_chain: unsupported shape K1=", K1, " N1=", N1, " N2=", N2);
  TORCH_CHECK(b1.numel() == N1 && b2.numel() == N2, "conv_chain: bias sizes");
  TORCH_CHECK(w1.device() == x.device() && w2.device() == x.device() && b1.device() == x.device() &&
                  b2.device() == x.device(), "conv_chain: tensors on different devices");
  const uint16_t* rp = nullptr;
  if (residual.has_value()) {
    need(*residual, at::kBFloat16, "residual");
    TORCH_CHECK(residual->dim() == 4 && residual->size(0) == x.size(0) && residual->size(1) == x.size(1) &&
                    residual->size(2) == x.size(2) && residual->size(3) == N1, "conv_chain: residual [n][h][w][N1]");
    rp = bf16p(*residual);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int M = x.size(0) * x.size(1) * x.size(2);
  Tensor y1 = torch::empty({x.size(0), x.size(1), x.size(2), N1}, x.options());
  Tensor y2 = torch::empty({x.size(0), x.size(1), x.size(2), N2}, x.options());
  check(tfsk::conv_chain_launch(bf16p(x), bf16p(w1), int(w1.size(1)), b1.data_ptr<float>(), rp, bf16p_mut(y1),
                                bf16p(w2), int(w2.size(1)), b2.data_ptr<float>(), bf16p_mut(y2), M, K1, N1, N2,
                                int(act1), int(act2), cur_stream(x)),
        "conv_chain");
  return {y1, y2};
}

Tensor global_avgpool(const Tensor& x, const c10::optional<Tensor>& out) {
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "global_avgpool: NHWC with C % 8 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  Tensor y = out.has_value() ? *out : torch::empty({N, C}, x.options());
  need(y, at::kBFloat16, "out");
  check(tfsk::global_avgpool_nhwc_launch(bf16p(x), bf16p_mut(y), N, HW, C, cur_stream(x)), "gap");
  return y;
}

std::vector<Tensor> softmax_argmax(const Tensor& logits, bool want_probs, bool want_classes,
                                   const c10::optional<Tensor>& probs_out,
                                   const c10::optional<Tensor>& classes_out) {
  // rows may be strided (a [M, N] view of a GEMM output padded to ldc > N)
  TORCH_CHECK(logits.is_cuda() && logits.dim() >= 1 && logits.stride(-1) == 1 &&
                  (logits.is_contiguous() || logits.dim() == 2),
              "logits must be a GPU tensor with unit column stride (contiguous, or 2-D with a row stride)");
  const bool bf = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == at::kFloat, "logits must be f32 or bf16");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  const int cols = logits.size(-1);
  const int rows = logits.numel() / cols;
  const long ld = logits.dim() == 2 ? long(logits.stride(0)) : long(cols);
  TORCH_CHECK(ld >= cols, "logits row stride");
  Tensor probs, classes;
  if (want_probs) {
    probs = probs_out.has_value() ? *probs_out : torch::empty(logits.sizes(), logits.options().dtype(at::kFloat));
    need(probs, at::kFloat, "probs");
  }
  if (want_classes) {
    auto sz = logits.sizes().vec();
    sz.pop_back();
    classes = classes_out.has_value() ? *classes_out : torch::empty(sz, logits.options().dtype(at::kLong));
    need(classes, at::kLong, "classes");
  }
  check(tfsk::softmax_argmax_launch(logits.data_ptr(), bf, want_probs ? probs.data_ptr<float>() : nullptr,
                                    want_classes ? classes.data_ptr<int64_t>() : nullptr, rows, cols, ld,
                                    cur_stream(logits)), "softmax_argmax");
  return {probs, classes};
}

// ResNet-style head: probs, classes = softmax/argmax(mean_hw(x) @ w^T + bias)[:, :n]
// With `probs_host` / `classes_host` (pinned host addresses of >= M rows, 0:
// none) the one-launch head also stores its rows there; the returned flag
// says whether it did (only the one-launch path can).
std::tuple<Tensor, Tensor, bool> classifier_head_impl(const Tensor& x, const Tensor& w, const Tensor& bias, int64_t n,
                                                      int64_t probs_host, int64_t classes_host);

std::vector<Tensor> classifier_head(const Tensor& x, const Tensor& w, const Tensor& bias, int64_t n) {
  auto r = classifier_head_impl(x, w, bias, n, 0, 0);
  return {std::get<0>(r), std::get<1>(r)};
}

std::tuple<Tensor, Tensor, bool> classifier_head_impl(const Tensor& x, const Tensor& w, const Tensor& bias, int64_t n,
                                                      int64_t probs_host, int64_t classes_host) {
  need(x, at::kBFloat16, "x");
  need(w, at::kBFloat16, "w");
  need(bias, at::kFloat, "bias");
  TORCH_CHECK(x.dim() == 4, "classifier_head: x must be NHWC");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int M = x.size(0), HW = x.size(1) * x.size(2), K = x.size(3);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K && (K == 512 || K == 1024 || K == 2048 || K == 4096),
              "classifier_head: w [Np][K] with K in {512, 1024, 2048, 4096}");
  const int Np = w.size(0);
  TORCH_CHECK(bias.numel() == Np && n >= 1 && n <= Np, "classifier_head: bias [Np], 1 <= n <= Np");
  Tensor part = torch::empty({int64_t(tfsk::classifier_head_ws_floats(M, K, Np))}, x.options().dtype(at::kFloat));
  Tensor probs = torch::empty({M, n}, x.options().dtype(at::kFloat));
  Tensor classes = torch::empty({M}, x.options().dtype(at::kLong));
  // small batches: one launch that hands off through an arrival counter (its
  // last workgroup runs the softmax rows serially, so only up to
  // TFSERVE_HEAD_FUSED rows, default 4, at most 16; 0 keeps three launches)
  int* counter = nullptr;
  const char* hf = std::getenv("TFSERVE_HEAD_FUSED");
  const int fused_max = hf && hf[0] ? std::min(16, std::atoi(hf)) : 4;
  if (M <= fused_max) {
    tfsk::splitk_counters_prepare(cur_stream(x));
    counter = tfsk::splitk_counters(1, cur_stream(x));
  }
  // host rows only where the one-launch path runs (same conditions as the launcher)
  const bool to_host = counter != nullptr && (probs_host != 0 || classes_host != 0) &&
                       tfsk::classifier_head_one_launch(M, HW, K, Np, int(n));
  check(tfsk::classifier_head_launch(bf16p(x), bf16p(w), bias.data_ptr<float>(), part.data_ptr<float>(),
                                     probs.data_ptr<float>(), classes.data_ptr<int64_t>(), M, HW, K, Np, int(n),
                                     cur_stream(x), counter,
                                     to_host ? reinterpret_cast<float*>(probs_host) : nullptr,
                                     to_host ? reinterpret_cast<int64_t*>(classes_host) : nullptr),
        "classifier_head");
  return {probs, classes, to_host};
}

Tensor ingest_c4(const Tensor& x, const c10::optional<Tensor>& out) {
  need(x, at::kFloat, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) <= 4, "ingest_c4: NHWC with C <= 4");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = out.has_value() ? *out : torch::empty({x.size(0), x.size(1), x.size(2), 4}, x.options().dtype(at::kBFloat16));
  need(y, at::kBFloat16, "out");
  check(tfsk::ingest_c4_launch(x.data_ptr<float>(), bf16p_mut(y), x.numel() / x.size(3), x.size(3), cur_stream(x)),
        "ingest_c4");
  return y;
}

// Zero-copy ingest: the kernel reads fp32 rows straight out of a *pinned host*
// tensor (device-accessible; e.g. a lane's request staging buffer) over PCIe,
// instead of an SDMA copy followed by a device pass.
void need_pinned_f32(const Tensor& x, const char* name) {
  TORCH_CHECK(x.device().is_cpu() && x.is_pinned(), name, " must be a pinned host tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous(), name, " must be contiguous float32");
}

void ingest_c4_from_host(const Tensor& x, const Tensor& out) {
  need_pinned_f32(x, "x");
  need(out, at::kBFloat16, "out");
  TORCH_CHECK(x.dim() == 4 && x.size(3) >= 1 && x.size(3) <= 4, "ingest_c4_from_host: x must be NHWC with C <= 4");
  const int64_t pixels = x.numel() / x.size(3);
  TORCH_CHECK(out.numel() == pixels * 4, "ingest_c4_from_host: out must hold pixels x 4 channels");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(out.device());
  check(tfsk::ingest_c4_launch(x.data_ptr<float>(), bf16p_mut(out), pixels, int(x.size(3)), cur_stream(out)),
        "ingest_c4_from_host");
}

Tensor ingest_c4_padded(const Tensor& x, int64_t Hp, int64_t Wp, int64_t pt, int64_t pl) {
  need(x, at::kFloat, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) >= 1 && x.size(3) <= 4, "ingest_c4_padded: NHWC with C <= 4");
  TORCH_CHECK(pt >= 0 && pl >= 0 && Hp >= pt + x.size(1) && Wp >= pl + x.size(2), "ingest_c4_padded: padding");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = torch::empty({x.size(0), Hp, Wp, 4}, x.options().dtype(at::kBFloat16));
  check(tfsk::ingest_c4_pad_launch(x.data_ptr<float>(), bf16p_mut(y), x.size(0), x.size(1), x.size(2), x.size(3),
                                   Hp, Wp, pt, pl, cur_stream(x)),
        "ingest_c4_padded");
  return y;
}

void cast_bf16_from_host(const Tensor& x, const Tensor& out) {
  need_pinned_f32(x, "x");
  need(out, at::kBFloat16, "out");
  TORCH_CHECK(out.numel() == x.numel(), "cast_bf16_from_host: size mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(out.device());
  check(tfsk::cast_f32_bf16_launch(x.data_ptr<float>(), bf16p_mut(out), x.numel(), cur_stream(out)),
        "cast_bf16_from_host");
}

void h2d_rows(const Tensor& host, const Tensor& dev) {
  TORCH_CHECK(host.device().is_cpu() && host.is_pinned() && host.is_contiguous(), "h2d_rows: host must be a "
              "contiguous pinned CPU tensor");
  TORCH_CHECK(dev.is_cuda() && dev.is_contiguous(), "h2d_rows: dev must be a contiguous device tensor");
  const int64_t bytes = host.numel() * host.element_size();
  TORCH_CHECK(bytes == dev.numel() * dev.element_size(), "h2d_rows: size mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dev.device());
  check(tfsk::h2d_rows_launch(host.data_ptr(), dev.data_ptr(), bytes, cur_stream(dev)), "h2d_rows");
}

Tensor cast_bf16(const Tensor& x, const c10::optional<Tensor>& out) {
  need(x, at::kFloat, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Tensor y = out.has_value() ? *out : torch::empty(x.sizes(), x.options().dtype(at::kBFloat16));
  need(y, at::kBFloat16, "out");
  check(tfsk::cast_f32_bf16_launch(x.data_ptr<float>(), bf16p_mut(y), x.numel(), cur_stream(x)), "cast");
  return y;
}

// y = LN(x @ w^T + bias + residual) * gamma + beta in one launch (lngemm.hip);
// x [.., K] contiguous bf16, w_frag = w [N][K] bf16 pre-shuffled fragment-major
// ([N/16][K/32][4][16][8]: graph/fused.py ln_weight_frags), bias / gamma / beta f32 [N]
Tensor linear_ln(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias,
                 const c10::optional<Tensor>& residual, const Tensor& gamma, const Tensor& beta, double eps,
                 int64_t bm, const c10::optional<Tensor>& out) {
  need(x, at::kBFloat16, "x");
  need(w, at::kBFloat16, "w");
  need(gamma, at::kFloat, "gamma");
  need(beta, at::kFloat, "beta");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int K = x.size(-1), M = x.numel() / K, N = w.size(0);
  TORCH_CHECK(w.is_contiguous() && w.numel() == int64_t(N) * K, "linear_ln: w_frag must be a contiguous [N][K]");
  TORCH_CHECK(tfsk::lngemm_supported(M, N, K, int(bm)), "linear_ln: unsupported shape M=", M, " N=", N, " K=", K,
              " bm=", bm);
  TORCH_CHECK(gamma.numel() == N && beta.numel() == N, "linear_ln: gamma / beta size");
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  Tensor y = out.has_value() ? *out : torch::empty(sizes, x.options());
  need(y, at::kBFloat16, "out");
  TORCH_CHECK(y.numel() == int64_t(M) * N, "linear_ln: out has the wrong size");
  tfsk::LnGemmArgs a;
  a.x = bf16p(x); a.w = bf16p(w); a.gamma = gamma.data_ptr<float>(); a.beta = beta.data_ptr<float>();
  a.y = bf16p_mut(y); a.M = M; a.N = N; a.K = K; a.ldx = K; a.eps = float(eps);
  if (bias.has_value()) {
    need(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == N, "linear_ln: bias size");
    a.bias = bias->data_ptr<float>();
  }
  if (residual.has_value()) {
    need(*residual, at::kBFloat16, "residual");
    TORCH_CHECK(residual->numel() == y.numel(), "linear_ln: residual shape must match the output");
    a.r = bf16p(*residual);
  }
  check(tfsk::lngemm_launch(a, int(bm), cur_stream(x)), "linear_ln");
  return y;
}

Tensor layernorm(const Tensor& x, const c10::optional<Tensor>& residual, const Tensor& gamma, const Tensor& beta,
                 double eps, const c10::optional<Tensor>& out) {
  need(x, at::kBFloat16, "x");
  need(gamma, at::kFloat, "gamma");
  need(beta, at::kFloat, "beta");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int cols = x.size(-1);
  TORCH_CHECK(cols % 8 == 0 && gamma.numel() == cols && beta.numel() == cols, "layernorm shapes");
  TORCH_CHECK(aligned16(gamma) && aligned16(beta), "layernorm: gamma / beta must be 16-B aligned");
  const int rows = x.numel() / cols;
  const uint16_t* r = nullptr;
  if (residual.has_value()) {
    need(*residual, at::kBFloat16, "residual");
    TORCH_CHECK(residual->numel() == x.numel(), "residual shape");
    r = bf16p(*residual);
  }
  Tensor y = out.has_value() ? *out : torch::empty_like(x);
  need(y, at::kBFloat16, "out");
  check(tfsk::layernorm_launch(bf16p(x), r, gamma.data_ptr<float>(), beta.data_ptr<float>(), bf16p_mut(y), rows,
                               cols, float(eps), cur_stream(x)), "layernorm");
  return y;
}

// ids / type_ids: int32, any shape, flattened to tokens; pos: [>= seq, Hd] rows
// indexed by token % seq. Returns ids.shape + [Hd].
Tensor embed_ln(const Tensor& ids, const c10::optional<Tensor>& type_ids, const Tensor& word,
                const c10::optional<Tensor>& pos, const c10::optional<Tensor>& type, const Tensor& gamma,
                const Tensor& beta, double eps, int64_t seq) {
  need(ids, at::kInt, "ids");
  need(word, at::kBFloat16, "word");
  need(gamma, at::kFloat, "gamma");
  need(beta, at::kFloat, "beta");
  TORCH_CHECK(word.dim() == 2, "word table must be 2-D");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(ids.device());
  const int64_t tokens = ids.numel(), Hd = word.size(1);
  TORCH_CHECK(Hd % 8 == 0 && Hd <= 2048, "embed_ln: hidden must be a multiple of 8 and <= 2048");
  TORCH_CHECK(gamma.numel() == Hd && beta.numel() == Hd, "embed_ln: LN params shape");
  TORCH_CHECK(aligned16(gamma) && aligned16(beta), "embed_ln: gamma / beta must be 16-B aligned");
  TORCH_CHECK(seq > 0 && tokens % seq == 0 && tokens < (int64_t(1) << 31), "embed_ln: tokens must be batch * seq");
  const int* tt = nullptr;
  const uint16_t *pp = nullptr, *tp = nullptr;
  int ntypes = 0;
  if (type_ids.has_value()) {
    TORCH_CHECK(type.has_value(), "embed_ln: type_ids without a type table");
    need(*type_ids, at::kInt, "type_ids");
    need(*type, at::kBFloat16, "type");
    TORCH_CHECK(type_ids->numel() == tokens && type->dim() == 2 && type->size(1) == Hd, "embed_ln: type shapes");
    tt = type_ids->data_ptr<int>();
    tp = bf16p(*type);
    ntypes = type->size(0);
  }
  if (pos.has_value()) {
    need(*pos, at::kBFloat16, "pos");
    TORCH_CHECK(pos->dim() == 2 && pos->size(1) == Hd && pos->size(0) >= seq, "embed_ln: pos shape");
    pp = bf16p(*pos);
  }
  auto shape = ids.sizes().vec();
  shape.push_back(Hd);
  Tensor y = torch::empty(shape, word.options());
  check(tfsk::embed_ln_launch(ids.data_ptr<int>(), tt, bf16p(word), pp, tp, gamma.data_ptr<float>(),
                              beta.data_ptr<float>(), bf16p_mut(y), tokens, seq, Hd, word.size(0), ntypes,
                              float(eps), cur_stream(ids)), "embed_ln");
  return y;
}

Tensor attention(const Tensor& qkv, const c10::optional<Tensor>& mask_bias, int64_t heads, double scale,
                 const c10::optional<Tensor>& out, int64_t mask_bstride, int64_t mask_qstride) {
  need(qkv, at::kBFloat16, "qkv");
  TORCH_CHECK(qkv.dim() == 3, "qkv must be [B, S, 3*H*D]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  const int B = qkv.size(0), S = qkv.size(1), HD3 = qkv.size(2);
  TORCH_CHECK(HD3 % (3 * heads) == 0, "qkv width must be 3*heads*head_dim");
  const int D = HD3 / (3 * heads);
  TORCH_CHECK(D == 64, "attention kernel supports head_dim 64");
  TORCH_CHECK(S >= 1 && S <= tfsk::kMaxAttentionSeq, "attention kernel supports 1 <= S <= ", tfsk::kMaxAttentionSeq);
  const float* mb = nullptr;
  if (mask_bias.has_value()) {
    need(*mask_bias, at::kFloat, "mask_bias");
    // largest index the kernel reads must be inside the mask tensor
    const int64_t last = int64_t(B - 1) * mask_bstride + int64_t(S - 1) * mask_qstride + (S - 1);
    TORCH_CHECK(mask_bstride >= 0 && mask_qstride >= 0 && last < mask_bias->numel(),
                "mask strides exceed the mask tensor");
    mb = mask_bias->data_ptr<float>();
  }
  Tensor y = out.has_value() ? *out : torch::empty({B, S, heads * D}, qkv.options());
  need(y, at::kBFloat16, "out");
  check(tfsk::attention_launch(bf16p(qkv), mb, bf16p_mut(y), B, S, heads, D, float(scale), mask_bstride,
                               mask_qstride, cur_stream(qkv)),
        "attention");
  return y;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 HIP kernels (MFMA implicit-GEMM conv/GEMM, attention, norms, pooling)";
  m.def("conv2d", &conv2d, "NHWC implicit-GEMM conv (+bias +residual +act)", py::arg("x"), py::arg("w"),
        py::arg("bias"), py::arg("residual"), py::arg("kh"), py::arg("kw"), py::arg("sh"), py::arg("sw"),
        py::arg("pt"), py::arg("pb"), py::arg("pl"), py::arg("pr"), py::arg("act") = 0, py::arg("cfg") = 0,
        py::arg("out") = py::none(), py::arg("out_f32") = false, py::arg("splits") = 1,
        py::arg("post_scale") = py::none(), py::arg("post_shift") = py::none(), py::arg("post_act") = 0,
        py::arg("out2") = py::none(), py::arg("post_only") = false);
  m.def("conv_chain", &conv_chain, "expand 1x1 (+residual, act) -> next reduce 1x1 (+act) in one kernel",
        py::arg("x"), py::arg("w1"), py::arg("b1"), py::arg("residual"), py::arg("act1"), py::arg("w2"),
        py::arg("b2"), py::arg("act2"));
  m.def("conv_chain_supported", [](int64_t k1, int64_t n1, int64_t n2) {
    return tfsk::conv_chain_supported(int(k1), int(n1), int(n2));
  });
  m.def("conv2d_dual", &conv2d_dual, "act(conv1x1(h) + conv1x1_stride(x) + bias) as one K-concatenated GEMM",
        py::arg("h"), py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("sh"), py::arg("sw"), py::arg("act") = 0,
        py::arg("cfg") = 36, py::arg("out") = py::none(), py::arg("splits") = 1,
        py::arg("post_scale") = py::none(), py::arg("post_shift") = py::none(), py::arg("post_act") = 0,
        py::arg("out2") = py::none(), py::arg("post_only") = false);
  m.def("linear_lnx", &linear_lnx,
        "GEMM whose A / residual rows are LayerNorm inputs (statistics as partials), optionally "
        "returning its own rows' partials: {y, partials}",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("residual"), py::arg("act"), py::arg("cfg"),
        py::arg("out_f32") = false, py::arg("out") = py::none(), py::arg("a_st") = py::none(),
        py::arg("a_colsum") = py::none(), py::arg("a_eps") = 1e-12, py::arg("r_st") = py::none(),
        py::arg("r_gamma") = py::none(), py::arg("r_beta") = py::none(), py::arg("r_eps") = 1e-12,
        py::arg("stats") = false);
  m.def("linear", &linear,"x @ w^T (+bias +residual +act)", py::arg("x"), py::arg("w"), py::arg("bias"),
        py::arg("residual") = py::none(), py::arg("act") = 0, py::arg("cfg") = 0, py::arg("out_f32") = false,
        py::arg("alpha") = 1.0, py::arg("out") = py::none(), py::arg("splits") = 1);
  m.def("stem_pool", &stem_pool, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("pt"), py::arg("pb"),
        py::arg("pl"), py::arg("pr"), py::arg("act"), py::arg("ppt"), py::arg("ppb"), py::arg("ppl"), py::arg("ppr"),
        py::arg("post_scale") = py::none(), py::arg("post_shift") = py::none(), py::arg("post_act") = 0);
  m.def("maxpool", &maxpool, py::arg("x"), py::arg("kh"), py::arg("kw"), py::arg("sh"), py::arg("sw"),
        py::arg("pt"), py::arg("pb"), py::arg("pl"), py::arg("pr"), py::arg("out") = py::none(),
        py::arg("post_scale") = py::none(), py::arg("post_shift") = py::none(), py::arg("post_act") = 0);
  m.def("global_avgpool", &global_avgpool, py::arg("x"), py::arg("out") = py::none());
  m.def("classifier_head", &classifier_head, "softmax/argmax(mean_hw(x) @ w^T + bias)[:, :n]", py::arg("x"),
        py::arg("w"), py::arg("bias"), py::arg("n"));
  m.def("softmax_argmax", &softmax_argmax, py::arg("logits"), py::arg("want_probs") = true,
        py::arg("want_classes") = true, py::arg("probs_out") = py::none(), py::arg("classes_out") = py::none());
  m.def("dense_softmax", &dense_softmax, "softmax(x @ w[:n]^T + bias[:n]) for n <= 16 labels (x f32)",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("n"));
  m.def("key_mask_adder", &key_mask_adder, "(one - m) * scale as f32", py::arg("m"), py::arg("one"),
        py::arg("scale"));
  m.def("cast_bf16", &cast_bf16, py::arg("x"), py::arg("out") = py::none());
  m.def("ingest_c4", &ingest_c4, "fp32 NHWC (C<=4) -> bf16 NHWC C=4", py::arg("x"), py::arg("out") = py::none());
  m.def("ingest_c4_padded", &ingest_c4_padded, "fp32 NHWC (C<=4) -> zero-bordered bf16 RGBA [N][Hp][Wp][4]",
        py::arg("x"), py::arg("hp"), py::arg("wp"), py::arg("pt"), py::arg("pl"));
  m.def("ingest_c4_from_host", &ingest_c4_from_host, "ingest_c4 reading a pinned host tensor (zero-copy)",
        py::arg("x"), py::arg("out"));
  m.def("h2d_rows", &h2d_rows, py::arg("host"), py::arg("dev"),
        "copy a pinned host tensor into a device tensor with a kernel (system-scope loads; capturable)");
  m.def("cast_bf16_from_host", &cast_bf16_from_host, "fp32 pinned host tensor -> bf16 device tensor",
        py::arg("x"), py::arg("out"));
  m.def("linear_ln", &linear_ln, "LN(x @ w^T + bias + residual) * gamma + beta, whole rows per workgroup",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("residual"), py::arg("gamma"), py::arg("beta"),
        py::arg("eps"), py::arg("bm") = 32, py::arg("out") = py::none());
  m.def("linear_ln_supported", [](int64_t M, int64_t N, int64_t K, int64_t bm) {
    return tfsk::lngemm_supported(int(M), int(N), int(K), int(bm));
  });
  m.def("layernorm", &layernorm, py::arg("x"), py::arg("residual"), py::arg("gamma"), py::arg("beta"),
        py::arg("eps"), py::arg("out") = py::none());
  m.def("embed_ln", &embed_ln, py::arg("ids"), py::arg("type_ids"), py::arg("word"), py::arg("pos"),
        py::arg("type"), py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("seq"));
  m.def("classifier_head_to_host", &classifier_head_impl, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("n"),
        py::arg("probs_host"), py::arg("classes_host"),
        "classifier_head that also stores its rows into pinned host memory when it runs as one launch: "
        "(probs, classes, wrote_host)");
  m.def("attention", &attention, py::arg("qkv"), py::arg("mask_bias"), py::arg("heads"), py::arg("scale"),
        py::arg("out") = py::none(), py::arg("mask_bstride") = 0, py::arg("mask_qstride") = 0);
  m.def("splitk_counters_set_owner", [](int64_t owner) { tfsk::splitk_counters_set_owner(owner); },
        "tag the split-K counter slices this thread's captures take (0 = none)");
  m.def("splitk_counters_release", [](int64_t owner) { return tfsk::splitk_counters_release(owner); },
        "return an owner's captured split-K counter slices to the pool");
  m.def("splitk_counters_captured_in_use", []() { return tfsk::splitk_counters_captured_in_use(); });
  m.def("splitk_counters_reclaim", []() { return tfsk::splitk_counters_reclaim(); },
        "advance released captured slices (fence on their replay streams -> zero on the lane's stream -> free); "
        "never blocks; call outside any capture on this thread; returns the ints made reusable");
  m.def("splitk_counters_add_stream", [](int64_t owner, int64_t stream) {
          tfsk::splitk_counters_add_stream(owner, reinterpret_cast<hipStream_t>(stream));
        }, py::arg("owner"), py::arg("stream"),
        "another stream the owner's graph replays on (its fence must complete before the slices are reused)");
  m.def("splitk_counters_pending", []() { return tfsk::splitk_counters_pending(); });
  m.def("set_wg_trace", [](const c10::optional<Tensor>& t) {
    if (!t.has_value()) {
      g_trace = nullptr;
      g_trace_cap = 0;
      tfsk::attention_set_trace(nullptr, 0);
      return;
    }
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->is_contiguous(), "trace: int64 device tensor");
    g_trace = reinterpret_cast<long long*>(t->data_ptr<int64_t>());
    g_trace_cap = int(std::min<int64_t>(t->numel() / 8, 1 << 30));
    tfsk::attention_set_trace(g_trace, g_trace_cap);
  }, "per-workgroup wall-clock stamps of the following GEMM / conv launches (None: off)");
  m.def("set_attention_plds", [](int64_t mode) { return tfsk::attention_set_plds(int(mode)); },
        "fixed-S attention: 1 = the P-through-LDS kernel, 0 = P in registers (default), -1 = env; returns the "
        "previous mode (process-wide; set it outside captures)");
  m.def("set_splitk_fixup", [](int64_t mode) {
    const int prev = g_fixup_override;
    g_fixup_override = mode < 0 ? -1 : (mode ? 1 : 0);
    return prev;
  }, "in-kernel split-K for this thread's following launches: 1 on, 0 off, -1 default (env, else small "
     "launches); returns the previous mode (restore it when done)");
  m.def("get_splitk_fixup", []() { return g_fixup_override; });
  m.def("classifier_head_one_launch", [](int64_t M, int64_t HW, int64_t K, int64_t Np, int64_t n) {
    return tfsk::classifier_head_one_launch(int(M), int(HW), int(K), int(Np), int(n));
  });
  m.def("num_configs", []() { return tfsk::kNumIGemmConfigs; });
  m.def("cgemm_configs", []() {
    std::vector<int> v;
    for (int c = 0; c < tfsk::kNumCGemmConfigs; ++c) v.push_back(tfsk::kCGemmCfgBase + c);
    for (int c = 0; c < tfsk::kNumCGemmConfigs2; ++c) v.push_back(tfsk::kCGemmCfgBase2 + c);
    for (int c = 0; c < tfsk::kNumCGemmPfConfigs; ++c) v.push_back(tfsk::kCGemmPfCfgBase + c);
    for (int c = 0; c < tfsk::kNumCGemm32Configs; ++c) v.push_back(tfsk::kCGemm32CfgBase + c);
    for (int c = 0; c < tfsk::kNumBGemmConfigs; ++c) v.push_back(tfsk::kBGemmCfgBase + c);
    return v;
  });
  m.def("halo_configs", []() {
    std::vector<int> v;
    for (int c = 0; c < tfsk::kNumHaloConfigs; ++c) v.push_back(tfsk::kHaloCfgBase + c);
    for (int c = 0; c < tfsk::kNumHaloConfigs; ++c)
      if (tfsk::halo_cfg_id(tfsk::kHaloPfCfgBase + c)) v.push_back(tfsk::kHaloPfCfgBase + c);
    v.push_back(tfsk::kHaloPersistCfg);
    return v;
  });
  m.def("config_tile", [](int cfg) {
    if (is_halo_cfg(cfg)) return std::make_pair(tfsk::halo_config_bm(cfg), tfsk::halo_config_bn(cfg));
    if (is_cgemm_cfg(cfg)) return std::make_pair(tfsk::cgemm_config_bm(cfg), tfsk::cgemm_config_bn(cfg));
    return std::make_pair(tfsk::igemm_config_bm(cfg), tfsk::igemm_config_bn(cfg));
  });
}
