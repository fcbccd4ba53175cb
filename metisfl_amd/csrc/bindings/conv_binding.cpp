// torch binding for the implicit-GEMM convolution kernels (conv.hip) and the
// dense GEMM kernels (gemm.hip).  Geometry is validated here, on the host,
// before any launch: the kernels index with 32-bit offsets and trust M/K/Ng.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "bindings/opt_tail_args.h"
#include "kernels/conv.h"
#include "kernels/gemm.h"

namespace {

hipStream_t cur_stream(const torch::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}
uint16_t* bf(const torch::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

void check_bf16(const torch::Tensor& t, int64_t numel, const char* nm) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), nm, " must be a contiguous device tensor");
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, nm, " must be bf16");
  TORCH_CHECK(t.numel() == numel, nm, " has ", t.numel(), " elements, expected ", numel);
}
void check_f32(const torch::Tensor& t, int64_t min_numel, const char* nm) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), nm, " must be a contiguous device tensor");
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, nm, " must be fp32");
  TORCH_CHECK(t.numel() >= min_numel, nm, " too small: ", t.numel(), " < ", min_numel);
}

int out_dim(int64_t in, int64_t k, int64_t stride, int64_t pad) {
  return (int)((in + 2 * pad - k) / stride + 1);
}

mfl::ConvGeom fwd_geom(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co, int64_t R,
                       int64_t S, int64_t stride, int64_t pad) {
  TORCH_CHECK(C % 8 == 0, "conv input channels must be a multiple of 8 (got ", C, ")");
  TORCH_CHECK(Co % 8 == 0, "conv output channels must be a multiple of 8 (got ", Co, ")");
  mfl::ConvGeom g{};
  g.N = (int)N; g.H = (int)H; g.W = (int)W; g.C = (int)C;
  g.P = out_dim(H, R, stride, pad);
  g.Q = out_dim(W, S, stride, pad);
  g.R = (int)R; g.S = (int)S; g.stride = (int)stride; g.pad = (int)pad;
  g.M = (int)(N * g.P * g.Q);
  g.K = (int)(R * S * C);
  g.Ng = (int)Co;
  TORCH_CHECK((int64_t)N * H * W * C < (1LL << 31), "activation too large for 32-bit indexing");
  return g;
}

// dgrad: rows over dX (H x W), source dY (P x Q x Co), B = W^T [Cin][R][S][Co]
mfl::ConvGeom dgrad_geom(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co, int64_t R,
                         int64_t S, int64_t stride, int64_t pad) {
  mfl::ConvGeom f = fwd_geom(N, H, W, C, Co, R, S, stride, pad);
  mfl::ConvGeom g{};
  g.N = f.N; g.H = f.P; g.W = f.Q; g.C = (int)Co;
  g.P = (int)H; g.Q = (int)W;
  g.R = f.R; g.S = f.S; g.stride = f.stride; g.pad = f.pad;
  g.M = (int)(N * H * W);
  g.K = (int)(R * S * Co);
  g.Ng = (int)C;
  return g;
}

// The counter block has ONE fixed size for every plan: a workspace is shared
// by all layers of a model, and a per-plan size would let one layer's slabs
// overlap (and poison) another layer's counters.  Split plans have < 256
// tiles (plan_conv_gemm only splits while tiles * splits < 256).
constexpr int64_t kCounterWords = 1024;
int64_t counter_words(const mfl::ConvGeom& g, const mfl::ConvPlan& p) {
  TORCH_CHECK(mfl::conv_counter_slots(g, p) <= kCounterWords, "split-K plan has too many tiles");
  return kCounterWords;
}
int64_t workspace_floats(const mfl::ConvGeom& g, const mfl::ConvPlan& p) {
  if (p.splits <= 1) return 0;
  return counter_words(g, p) + (int64_t)p.splits * mfl::conv_counter_slots(g, p) * p.bm * p.bn;
}

std::vector<int64_t> plan_vec(const mfl::ConvPlan& p, int64_t ws_floats, int64_t stats_rows) {
  return {p.bm, p.bn, p.splits, p.kchunk, stats_rows, ws_floats};
}

// mode 0 = fwd, 1 = dgrad, 2 = wgrad.  Returns
// [bm, bn, splits, kchunk, stats_rows, workspace_floats].
std::vector<int64_t> conv_plan(int64_t mode, int64_t N, int64_t H, int64_t W, int64_t C,
                               int64_t Co, int64_t R, int64_t S, int64_t stride, int64_t pad) {
  if (mode == 2) {
    mfl::ConvGeom g = fwd_geom(N, H, W, C, Co, R, S, stride, pad);
    auto p = mfl::plan_conv_wgrad(g);
    return plan_vec(p, 0, 0);
  }
  mfl::ConvGeom g = mode == 0 ? fwd_geom(N, H, W, C, Co, R, S, stride, pad)
                              : dgrad_geom(N, H, W, C, Co, R, S, stride, pad);
  auto p = mfl::plan_conv_gemm(g, mode == 1);
  return plan_vec(p, workspace_floats(g, p), 1);
}

void run_gemm(const mfl::ConvGeom& g, bool dgrad, const torch::Tensor& src, const torch::Tensor& w,
              const torch::Tensor& y, const c10::optional<torch::Tensor>& ws,
              const c10::optional<torch::Tensor>& stats, bool accum,
              const mfl::BnBwdFusion* bnb = nullptr) {
  auto p = mfl::plan_conv_gemm(g, dgrad);
  float* wsp = nullptr;
  int* counters = nullptr;
  if (p.splits > 1) {
    // layout: [arrival counters, padded to 64 words][fp32 slabs]; the
    // counters must be zero when first used (allocate with torch.zeros) and
    // are re-armed by the reducing workgroup, so the buffer is reusable.
    TORCH_CHECK(ws.has_value() && ws->defined(), "split-K workspace required");
    check_f32(*ws, workspace_floats(g, p), "workspace");
    counters = reinterpret_cast<int*>(ws->data_ptr<float>());
    wsp = ws->data_ptr<float>() + counter_words(g, p);
  }
  double* st = nullptr;
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats->is_cuda() && stats->is_contiguous() &&
                    stats->scalar_type() == torch::kFloat64 && stats->numel() >= 2 * g.Ng,
                "stats must be a contiguous fp64 device tensor of >= 2*Cout elements");
    st = stats->data_ptr<double>();
  }
  if (bnb != nullptr)
    mfl::launch_conv_dgrad_bnb(g, p, bf(src), bf(w), bf(y), wsp, counters, accum, *bnb, cur_stream(y));
  else
    mfl::launch_conv_gemm(g, dgrad, p, bf(src), bf(w), bf(y), wsp, counters, st, accum,
                          cur_stream(y));
}

// split-K workspace / stats pointers of a forward plan (as run_gemm)
void gemm_ptrs(const mfl::ConvGeom& g, const mfl::ConvPlan& p, const c10::optional<torch::Tensor>& ws,
               const c10::optional<torch::Tensor>& stats, float*& wsp, int*& counters, double*& st) {
  wsp = nullptr;
  counters = nullptr;
  st = nullptr;
  if (p.splits > 1) {
    TORCH_CHECK(ws.has_value() && ws->defined(), "split-K workspace required");
    check_f32(*ws, workspace_floats(g, p), "workspace");
    counters = reinterpret_cast<int*>(ws->data_ptr<float>());
    wsp = ws->data_ptr<float>() + counter_words(g, p);
  }
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats->is_cuda() && stats->is_contiguous() &&
                    stats->scalar_type() == torch::kFloat64 && stats->numel() >= 2 * g.Ng,
                "stats must be a contiguous fp64 device tensor of >= 2*Cout elements");
    st = stats->data_ptr<double>();
  }
}

// A downsampling block's conv1 (3x3, stride 2, pad 1) and projection shortcut
// (1x1, stride 2) of the same x: one paired launch, else two.
void conv_forward_pair(torch::Tensor x, torch::Tensor w1, torch::Tensor y1, c10::optional<torch::Tensor> ws1,
                       c10::optional<torch::Tensor> stats1, torch::Tensor w2, torch::Tensor y2,
                       c10::optional<torch::Tensor> ws2, c10::optional<torch::Tensor> stats2, int64_t N,
                       int64_t H, int64_t W, int64_t C, int64_t Co) {
  auto g1 = fwd_geom(N, H, W, C, Co, 3, 3, 2, 1);
  auto g2 = fwd_geom(N, H, W, C, Co, 1, 1, 2, 0);
  TORCH_CHECK(g1.M == g2.M, "conv1 / shortcut output sizes differ");
  check_bf16(x, N * H * W * C, "x");
  check_bf16(w1, Co * 9 * C, "w1");
  check_bf16(w2, Co * C, "w2");
  check_bf16(y1, (int64_t)g1.M * Co, "y1");
  check_bf16(y2, (int64_t)g2.M * Co, "y2");
  const auto p1 = mfl::plan_conv_gemm(g1, false), p2 = mfl::plan_conv_gemm(g2, false);
  float *ys1, *ys2;
  int *c1, *c2;
  double *st1, *st2;
  gemm_ptrs(g1, p1, ws1, stats1, ys1, c1, st1);
  gemm_ptrs(g2, p2, ws2, stats2, ys2, c2, st2);
  if (mfl::launch_conv_fwd_pair(g1, p1, bf(w1), bf(y1), ys1, c1, st1, g2, p2, bf(w2), bf(y2), ys2, c2, st2,
                                bf(x), cur_stream(x)))
    return;
  run_gemm(g1, false, x, w1, y1, ws1, stats1, false);
  run_gemm(g2, false, x, w2, y2, ws2, stats2, false);
}

void conv_forward(torch::Tensor x, torch::Tensor w, torch::Tensor y,
                  c10::optional<torch::Tensor> ws, c10::optional<torch::Tensor> stats, int64_t N,
                  int64_t H, int64_t W, int64_t C, int64_t Co, int64_t R, int64_t S,
                  int64_t stride, int64_t pad) {
  auto g = fwd_geom(N, H, W, C, Co, R, S, stride, pad);
  check_bf16(x, N * H * W * C, "x");
  check_bf16(w, Co * R * S * C, "w");
  check_bf16(y, (int64_t)g.M * Co, "y");
  run_gemm(g, false, x, w, y, ws, stats, false);
}

// fused BN-backward target of a dgrad (all optional; bn_acc undefined: off)
bool bnb_args(int64_t M, int64_t C, const c10::optional<torch::Tensor>& bn_z,
              const c10::optional<torch::Tensor>& bn_y, const c10::optional<torch::Tensor>& bn_mean,
              const c10::optional<torch::Tensor>& bn_invstd, const c10::optional<torch::Tensor>& bn_acc,
              mfl::BnBwdFusion& f) {
  if (!(bn_acc.has_value() && bn_acc->defined())) return false;
  TORCH_CHECK(bn_z.has_value() && bn_mean.has_value() && bn_invstd.has_value(), "bn fusion args");
  check_bf16(*bn_z, M * C, "bn_z");
  f.z = bf(*bn_z);
  if (bn_y.has_value() && bn_y->defined()) {
    check_bf16(*bn_y, M * C, "bn_y");
    f.y = bf(*bn_y);
  }
  check_f32(*bn_mean, C, "bn_mean");
  check_f32(*bn_invstd, C, "bn_invstd");
  f.mean = bn_mean->data_ptr<float>();
  f.invstd = bn_invstd->data_ptr<float>();
  TORCH_CHECK(bn_acc->is_cuda() && bn_acc->is_contiguous() && bn_acc->scalar_type() == torch::kFloat64 &&
                  bn_acc->numel() >= 2 * C, "bn_acc must be a contiguous fp64 tensor of >= 2*C");
  f.acc = bn_acc->data_ptr<double>();
  return true;
}

void conv_dgrad(torch::Tensor dy, torch::Tensor wt, torch::Tensor dx,
                c10::optional<torch::Tensor> ws, int64_t N, int64_t H, int64_t W, int64_t C,
                int64_t Co, int64_t R, int64_t S, int64_t stride, int64_t pad, bool accumulate,
                c10::optional<torch::Tensor> bn_z, c10::optional<torch::Tensor> bn_y,
                c10::optional<torch::Tensor> bn_mean, c10::optional<torch::Tensor> bn_invstd,
                c10::optional<torch::Tensor> bn_acc) {
  auto g = dgrad_geom(N, H, W, C, Co, R, S, stride, pad);
  check_bf16(dy, (int64_t)N * g.H * g.W * Co, "dy");
  check_bf16(wt, C * R * S * Co, "wt");
  check_bf16(dx, N * H * W * C, "dx");
  if (bn_acc.has_value() && bn_acc->defined()) {
    // fused BN-backward reductions of the layer whose output gradient dx is
    mfl::BnBwdFusion f;
    TORCH_CHECK(bn_z.has_value() && bn_mean.has_value() && bn_invstd.has_value(), "bn fusion args");
    check_bf16(*bn_z, N * H * W * C, "bn_z");
    f.z = bf(*bn_z);
    if (bn_y.has_value() && bn_y->defined()) {
      check_bf16(*bn_y, N * H * W * C, "bn_y");
      f.y = bf(*bn_y);
    }
    check_f32(*bn_mean, C, "bn_mean");
    check_f32(*bn_invstd, C, "bn_invstd");
    f.mean = bn_mean->data_ptr<float>();
    f.invstd = bn_invstd->data_ptr<float>();
    TORCH_CHECK(bn_acc->is_cuda() && bn_acc->is_contiguous() && bn_acc->scalar_type() == torch::kFloat64 &&
                    bn_acc->numel() >= 2 * C, "bn_acc must be a contiguous fp64 tensor of >= 2*C");
    f.acc = bn_acc->data_ptr<double>();
    run_gemm(g, true, dy, wt, dx, ws, c10::nullopt, accumulate, &f);
    return;
  }
  run_gemm(g, true, dy, wt, dx, ws, c10::nullopt, accumulate);
}

// accumulate=false zeroes dw first when the plan splits the reduction (the
// training step passes true: its gradient buffer is zeroed by the optimizer).
void conv_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor dw, int64_t N, int64_t H,
                int64_t W, int64_t C, int64_t Co, int64_t R, int64_t S, int64_t stride,
                int64_t pad, bool accumulate) {
  auto g = fwd_geom(N, H, W, C, Co, R, S, stride, pad);
  check_bf16(x, N * H * W * C, "x");
  check_bf16(dy, (int64_t)g.M * Co, "dy");
  check_f32(dw, Co * R * S * C, "dw");
  TORCH_CHECK(dw.numel() == Co * R * S * C, "dw size");
  auto p = mfl::plan_conv_wgrad(g);
  if (p.splits > 1 && !accumulate)
    (void)hipMemsetAsync(dw.data_ptr<float>(), 0, dw.numel() * sizeof(float), cur_stream(x));
  mfl::launch_conv_wgrad(g, p, bf(x), bf(dy), dw.data_ptr<float>(), cur_stream(x));
}

// A layer's backward GEMMs: dw += dy^T im2col(x) (dw zero on entry, the
// training step's gradient buffer) and dx (+)= conv_transpose(dy, W) with the
// optional fused BN-backward reductions -- in one paired launch when the
// shapes allow (launch_conv_bwd_pair), else as the two launches.
void conv_backward_pair(torch::Tensor x, torch::Tensor dy, torch::Tensor dw, torch::Tensor wt,
                        torch::Tensor dx, c10::optional<torch::Tensor> ws, int64_t N, int64_t H, int64_t W,
                        int64_t C, int64_t Co, int64_t R, int64_t S, int64_t stride, int64_t pad,
                        bool accumulate, c10::optional<torch::Tensor> bn_z, c10::optional<torch::Tensor> bn_y,
                        c10::optional<torch::Tensor> bn_mean, c10::optional<torch::Tensor> bn_invstd,
                        c10::optional<torch::Tensor> bn_acc, c10::optional<torch::Tensor> opt_p,
                        c10::optional<torch::Tensor> opt_g, c10::optional<torch::Tensor> opt_m,
                        c10::optional<torch::Tensor> opt_v, c10::optional<torch::Tensor> opt_anchor,
                        c10::optional<torch::Tensor> opt_mirror, c10::optional<torch::Tensor> opt_lr_scale,
                        c10::optional<torch::Tensor> opt_step, int64_t opt_mode, std::vector<double> opt_hyper,
                        bool opt_zero_grad) {
  auto gw = fwd_geom(N, H, W, C, Co, R, S, stride, pad);
  auto gd = dgrad_geom(N, H, W, C, Co, R, S, stride, pad);
  mfl::OptTail ot;  // optimizer tail (opt_tail.h), bf16 compute-copy mirror
  const bool tail = opt_tail_args(ot, opt_p, opt_g, opt_m, opt_v, opt_anchor, opt_mirror, opt_lr_scale, opt_step,
                                  opt_mode, opt_hyper, opt_zero_grad);
  check_bf16(x, N * H * W * C, "x");
  check_bf16(dy, (int64_t)gw.M * Co, "dy");
  check_f32(dw, Co * R * S * C, "dw");
  TORCH_CHECK(dw.numel() == Co * R * S * C, "dw size");
  check_bf16(wt, C * R * S * Co, "wt");
  check_bf16(dx, N * H * W * C, "dx");
  mfl::BnBwdFusion f;
  const bool fused = bnb_args(N * H * W, C, bn_z, bn_y, bn_mean, bn_invstd, bn_acc, f);
  auto pd = mfl::plan_conv_gemm(gd, true);
  float* wsp = nullptr;
  int* counters = nullptr;
  if (pd.splits > 1) {
    TORCH_CHECK(ws.has_value() && ws->defined(), "split-K workspace required");
    check_f32(*ws, workspace_floats(gd, pd), "workspace");
    counters = reinterpret_cast<int*>(ws->data_ptr<float>());
    wsp = ws->data_ptr<float>() + counter_words(gd, pd);
  }
  if (mfl::launch_conv_bwd_pair(gd, pd, bf(dy), bf(wt), bf(dx), wsp, counters, accumulate, fused ? &f : nullptr,
                                gw, bf(x), dw.data_ptr<float>(), cur_stream(dx), tail ? &ot : nullptr))
    return;
  mfl::launch_conv_wgrad(gw, mfl::plan_conv_wgrad(gw), bf(x), bf(dy), dw.data_ptr<float>(), cur_stream(x));
  if (fused) run_gemm(gd, true, dy, wt, dx, ws, c10::nullopt, accumulate, &f);
  else run_gemm(gd, true, dy, wt, dx, ws, c10::nullopt, accumulate);
  if (tail) opt_tail_fallback(ot, cur_stream(dx));
}

void transpose_krsc(torch::Tensor w, torch::Tensor wt, int64_t Co, int64_t RS, int64_t Ci) {
  check_bf16(w, Co * RS * Ci, "w");
  check_bf16(wt, Co * RS * Ci, "wt");
  mfl::launch_transpose_krsc(bf(w), bf(wt), (int)Co, (int)RS, (int)Ci, cur_stream(w));
}

// ---------------------------------------------------------------------------
// Dense GEMM  C[M][N] = A[M][K] . B[N][K]^T  (+bias, +gelu, ...), bf16 in/out.
void gemm_nt(torch::Tensor a, torch::Tensor b, torch::Tensor c, c10::optional<torch::Tensor> bias,
             int64_t M, int64_t N, int64_t K, int64_t epilogue, c10::optional<torch::Tensor> aux) {
  check_bf16(a, M * K, "a");
  check_bf16(b, N * K, "b");
  check_bf16(c, M * N, "c");
  TORCH_CHECK(K % 8 == 0 && N % 8 == 0, "gemm K and N must be multiples of 8");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_f32(*bias, N, "bias");
    bp = bias->data_ptr<float>();
  }
  uint16_t* ap = nullptr;
  if (aux.has_value() && aux->defined()) {
    check_bf16(*aux, M * N, "aux");
    ap = bf(*aux);
  }
  mfl::launch_gemm_nt(bf(a), bf(b), bf(c), bp, ap, (int)M, (int)N, (int)K, (int)epilogue,
                      cur_stream(c));
}

}  // namespace

void register_conv(pybind11::module& m) {
  m.def("conv_plan", &conv_plan);
  m.def("set_conv_plan_targets", [](int64_t conv_target, int64_t wgrad_target) {
    mfl::set_conv_plan_targets((int)conv_target, (int)wgrad_target);
  });
  m.def("conv_forward", &conv_forward);
  m.def("conv_dgrad", &conv_dgrad);
  m.def("conv_wgrad", &conv_wgrad);
  m.def("conv_backward_pair", &conv_backward_pair);
  m.def("conv_forward_pair", &conv_forward_pair);
  m.def("transpose_krsc", &transpose_krsc);
}

void register_gemm(pybind11::module& m) { m.def("gemm_nt", &gemm_nt); }
