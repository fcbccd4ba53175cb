// torch binding for the fp32 (reference-precision) learner kernels:
// conv32.hip (fwd / dgrad / wgrad), bn32.hip, the fp32 head and the batch
// gather.  As in the other bindings, shapes / dtypes are validated on the
// host before any launch (the kernels index with 32-bit offsets and trust
// their geometry) and every launch goes to the caller's current HIP stream.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/conv32.h"
#include "kernels/launchers.h"
#include "bindings/opt_tail_args.h"

namespace {

// Convolution product mode of the fp32 path: 0 = exact fp32 MFMA (mfl::c32x),
// 1 = bf16x3 split products with fp32 accumulation (mfl::c32s).  Process-wide,
// set before a model captures its graph.
int g_c32_mode = 0;
#define C32_CALL(fn, ...) (g_c32_mode ? mfl::c32s::fn(__VA_ARGS__) : mfl::c32x::fn(__VA_ARGS__))

void set_conv32_pair_ring(int64_t ns) {
  TORCH_CHECK(ns == 0 || ns == 2 || ns == 3, "pair ring depth is 0 (build default), 2 or 3");
  mfl::c32x::set_conv32_pair_ring((int)ns);
  mfl::c32s::set_conv32_pair_ring((int)ns);
}

void set_conv32_plan_overrides(const std::string& spec) {
  mfl::c32x::set_conv32_plan_overrides(spec.c_str());
  mfl::c32s::set_conv32_plan_overrides(spec.c_str());
}

void set_conv32_mode(int64_t m) {
  TORCH_CHECK(m == 0 || m == 1, "conv32 mode is 0 (exact fp32) or 1 (bf16x3)");
  g_c32_mode = (int)m;
}
int64_t conv32_mode() { return g_c32_mode; }

hipStream_t cur_stream(const torch::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_f32(const torch::Tensor& t, int64_t numel, const char* nm, bool exact = true) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), nm, " must be a contiguous device tensor");
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, nm, " must be fp32");
  if (exact) {
    TORCH_CHECK(t.numel() == numel, nm, " has ", t.numel(), " elements, expected ", numel);
  } else {
    TORCH_CHECK(t.numel() >= numel, nm, " too small: ", t.numel(), " < ", numel);
  }
}
float* fp(const torch::Tensor& t) { return t.data_ptr<float>(); }
template <typename T>
T* opt_ptr(const c10::optional<torch::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->is_contiguous(), "optional operand must be a contiguous device tensor");
  return reinterpret_cast<T*>(t->data_ptr());
}

int out_dim(int64_t in, int64_t k, int64_t stride, int64_t pad) { return (int)((in + 2 * pad - k) / stride + 1); }

mfl::ConvGeom fwd_geom(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co, int64_t R, int64_t S, int64_t stride,
                       int64_t pad) {
  TORCH_CHECK(C % 4 == 0 && Co % 4 == 0, "fp32 conv channels must be multiples of 4 (got ", C, ", ", Co, ")");
  TORCH_CHECK(R == S && (R == 1 || R == 3) && (stride == 1 || stride == 2),
              "fp32 conv supports 1x1 / 3x3 kernels at stride 1 / 2");
  mfl::ConvGeom g{};
  g.N = (int)N; g.H = (int)H; g.W = (int)W; g.C = (int)C;
  g.P = out_dim(H, R, stride, pad);
  g.Q = out_dim(W, S, stride, pad);
  g.R = (int)R; g.S = (int)S; g.stride = (int)stride; g.pad = (int)pad;
  g.M = (int)(N * g.P * g.Q);
  g.K = (int)(R * S * C);
  g.Ng = (int)Co;
  TORCH_CHECK((int64_t)N * H * W * C * 4 < (1LL << 31) && (int64_t)g.M * Co * 4 < (1LL << 31),
              "activation too large for 32-bit byte offsets");
  return g;
}
mfl::ConvGeom dgrad_geom(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co, int64_t R, int64_t S,
                         int64_t stride, int64_t pad) {
  const mfl::ConvGeom f = fwd_geom(N, H, W, C, Co, R, S, stride, pad);
  mfl::ConvGeom g{};
  g.N = f.N; g.H = f.P; g.W = f.Q; g.C = (int)Co;
  g.P = (int)H; g.Q = (int)W;
  g.R = f.R; g.S = f.S; g.stride = f.stride; g.pad = f.pad;
  g.M = (int)(N * H * W);
  g.K = (int)(R * S * Co);
  g.Ng = (int)C;
  return g;
}

constexpr int64_t kCounterWords = 1024;
int64_t ws_floats(const mfl::ConvGeom& g, const mfl::ConvPlan& p) {
  if (p.splits <= 1) return 0;
  TORCH_CHECK(C32_CALL(conv32_counter_slots, g, p) <= kCounterWords, "split-K plan has too many tiles");
  return kCounterWords + (int64_t)p.splits * C32_CALL(conv32_counter_slots, g, p) * p.bm * p.bn;
}

// mode 0 fwd / 1 dgrad / 2 wgrad -> [bm, bn, splits, kchunk, stats_rows, workspace_floats]
std::vector<int64_t> conv32_plan(int64_t mode, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co, int64_t R,
                                 int64_t S, int64_t stride, int64_t pad) {
  if (mode == 2) {
    const auto g = fwd_geom(N, H, W, C, Co, R, S, stride, pad);
    const auto p = C32_CALL(plan_conv32, g, 2);
    TORCH_CHECK(p.kchunk > 0, "no feasible conv32 plan for this shape");
    return {p.bm, p.bn, p.splits, p.kchunk, 0, 0};
  }
  const auto g = mode == 0 ? fwd_geom(N, H, W, C, Co, R, S, stride, pad) : dgrad_geom(N, H, W, C, Co, R, S, stride, pad);
  const auto p = C32_CALL(plan_conv32, g, (int)mode);
  TORCH_CHECK(p.kchunk > 0, "no feasible conv32 plan for this shape");
  // workspace for the larger of the regime's plan and the table's
  const auto pt = C32_CALL(plan_conv32_table, g, (int)mode);
  const int64_t ws = std::max(ws_floats(g, p), pt.kchunk > 0 ? ws_floats(g, pt) : (int64_t)0);
  return {p.bm, p.bn, p.splits, p.kchunk, mode == 0 ? 1 : 0, ws};
}

// fwd / dgrad B operand: the fp32 weights (exact mode), or in bf16x3 mode their
// packed hi|lo split -- the model's optimizer-maintained mirror when given
// (wp, int32), else packed here into a temporary (stream-ordered lifetime)
const float* wsrc(const torch::Tensor& w, const c10::optional<torch::Tensor>& wp, torch::Tensor& tmp) {
  if (!g_c32_mode) return fp(w);
  if (wp.has_value() && wp->defined()) {
    TORCH_CHECK(wp->is_cuda() && wp->is_contiguous() && wp->scalar_type() == torch::kInt32 &&
                    wp->numel() == w.numel(),
                "packed weights: contiguous int32 device tensor of the weights' size");
    return reinterpret_cast<const float*>(wp->data_ptr());
  }
  TORCH_CHECK(w.numel() % 4 == 0, "weights are packed in groups of 4");
  tmp = torch::empty({w.numel()}, w.options().dtype(torch::kInt32));
  mfl::launch_split_pack(fp(w), reinterpret_cast<uint32_t*>(tmp.data_ptr()), w.numel(), cur_stream(w));
  return reinterpret_cast<const float*>(tmp.data_ptr());
}

// dgrad / wgrad dY operand: fp32 (exact mode); in bf16x3 mode its packed hi|lo
// split -- as the layer's fp32 BN backward wrote it when dy is an int32 view of
// that buffer (bn32_backward with an int32 dx), else packed here into a
// temporary (stream-ordered lifetime)
// The same holds for the activation operand X of fwd / wgrad (int32: the
// packed mirror the fp32 BN apply wrote next to its output).
const float* dysrc(const torch::Tensor& dy, int64_t n, torch::Tensor& tmp, const char* nm = "dy") {
  if (dy.scalar_type() == torch::kInt32) {
    TORCH_CHECK(g_c32_mode, "a packed (int32) conv operand needs the bf16x3 conv product mode: ", nm);
    TORCH_CHECK(dy.is_cuda() && dy.is_contiguous() && dy.numel() == n,
                "packed operand: contiguous int32 device tensor of the operand's size: ", nm);
    return reinterpret_cast<const float*>(dy.data_ptr());
  }
  check_f32(dy, n, nm);
  if (!g_c32_mode) return fp(dy);
  TORCH_CHECK(n % 4 == 0, "dY is packed in groups of 4");
  tmp = torch::empty({n}, dy.options().dtype(torch::kInt32));
  mfl::launch_split_pack(fp(dy), reinterpret_cast<uint32_t*>(tmp.data_ptr()), n, cur_stream(dy));
  return reinterpret_cast<const float*>(tmp.data_ptr());
}

void run(const mfl::ConvGeom& g, bool dgrad, const float* src, const float* wptr, const torch::Tensor& y,
         const c10::optional<torch::Tensor>& ws, double* stats, bool accum, const mfl::BnBwdFusion32* bnb,
         int stats_reps = 1) {
  const auto p = C32_CALL(plan_conv32, g, dgrad ? 1 : 0);
  float* slab = nullptr;
  int* counters = nullptr;
  if (p.splits > 1) {
    TORCH_CHECK(ws.has_value() && ws->defined(), "split-K workspace required");
    check_f32(*ws, ws_floats(g, p), "workspace", false);
    counters = reinterpret_cast<int*>(ws->data_ptr<float>());
    slab = ws->data_ptr<float>() + kCounterWords;
  }
  C32_CALL(launch_conv32_gemm, g, dgrad, p, src, wptr, fp(y), slab, counters, stats, accum, bnb, cur_stream(y),
                          stats_reps);
}

// BN accumulators may hold R replicas [R][2][C] (R = numel / 2C)
int reps_of(const torch::Tensor& acc, int64_t C) { return (int)std::max<int64_t>(1, acc.numel() / (2 * C)); }

double* stats_ptr(const c10::optional<torch::Tensor>& st, int64_t C) {
  if (!st.has_value() || !st->defined()) return nullptr;
  TORCH_CHECK(st->is_cuda() && st->is_contiguous() && st->scalar_type() == torch::kFloat64 && st->numel() >= 2 * C,
              "stats must be a contiguous fp64 device tensor of >= 2*C elements");
  return st->data_ptr<double>();
}

void conv32_forward(torch::Tensor x, torch::Tensor w, torch::Tensor y, c10::optional<torch::Tensor> ws,
                    c10::optional<torch::Tensor> stats, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co,
                    int64_t R, int64_t S, int64_t stride, int64_t pad, c10::optional<torch::Tensor> wp) {
  const auto g = fwd_geom(N, H, W, C, Co, R, S, stride, pad);
  torch::Tensor xtmp;
  const float* xs = dysrc(x, (int64_t)N * H * W * C, xtmp, "x");
  check_f32(w, (int64_t)Co * R * S * C, "w");
  check_f32(y, (int64_t)g.M * Co, "y");
  torch::Tensor tmp;
  run(g, false, xs, wsrc(w, wp, tmp), y, ws, stats_ptr(stats, Co), false, nullptr,
      stats.has_value() && stats->defined() ? reps_of(*stats, Co) : 1);
}

void conv32_dgrad(torch::Tensor dy, torch::Tensor w, torch::Tensor dx, c10::optional<torch::Tensor> ws, int64_t N,
                  int64_t H, int64_t W, int64_t C, int64_t Co, int64_t R, int64_t S, int64_t stride, int64_t pad,
                  bool accumulate, c10::optional<torch::Tensor> bn_z, c10::optional<torch::Tensor> bn_y,
                  c10::optional<torch::Tensor> bn_mean, c10::optional<torch::Tensor> bn_invstd,
                  c10::optional<torch::Tensor> bn_acc, c10::optional<torch::Tensor> wp) {
  const auto g = dgrad_geom(N, H, W, C, Co, R, S, stride, pad);
  torch::Tensor dtmp;
  const float* dyp = dysrc(dy, (int64_t)N * g.H * g.W * Co, dtmp);
  check_f32(w, (int64_t)Co * R * S * C, "w");
  check_f32(dx, (int64_t)N * H * W * C, "dx");
  mfl::BnBwdFusion32 f;
  const bool fuse = bn_acc.has_value() && bn_acc->defined();
  if (fuse) {
    TORCH_CHECK(bn_z.has_value() && bn_mean.has_value() && bn_invstd.has_value(), "bn fusion operands");
    check_f32(*bn_z, dx.numel(), "bn_z");
    if (bn_y.has_value() && bn_y->defined()) check_f32(*bn_y, dx.numel(), "bn_y");
    check_f32(*bn_mean, C, "bn_mean");
    check_f32(*bn_invstd, C, "bn_invstd");
    f.z = fp(*bn_z);
    f.y = opt_ptr<float>(bn_y);
    f.mean = fp(*bn_mean);
    f.invstd = fp(*bn_invstd);
    f.acc = stats_ptr(bn_acc, C);
    f.reps = reps_of(*bn_acc, C);
  }
  torch::Tensor tmp;
  run(g, true, dyp, wsrc(w, wp, tmp), dx, ws, nullptr, accumulate, fuse ? &f : nullptr);
}

// A layer's dgrad (+ fused consumer-BN reductions) and wgrad (dw zero on
// entry or a running sum) -- one paired launch when both plans allow it.
void conv32_backward_pair(torch::Tensor x, torch::Tensor dy, torch::Tensor dw, torch::Tensor w, torch::Tensor dx,
                          c10::optional<torch::Tensor> ws, int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co,
                          int64_t R, int64_t S, int64_t stride, int64_t pad, bool accumulate,
                          c10::optional<torch::Tensor> bn_z, c10::optional<torch::Tensor> bn_y,
                          c10::optional<torch::Tensor> bn_mean, c10::optional<torch::Tensor> bn_invstd,
                          c10::optional<torch::Tensor> bn_acc, c10::optional<torch::Tensor> wp,
                          c10::optional<torch::Tensor> opt_p, c10::optional<torch::Tensor> opt_g,
                          c10::optional<torch::Tensor> opt_m, c10::optional<torch::Tensor> opt_v,
                          c10::optional<torch::Tensor> opt_anchor, c10::optional<torch::Tensor> opt_mirror,
                          c10::optional<torch::Tensor> opt_lr_scale, c10::optional<torch::Tensor> opt_step,
                          int64_t opt_mode, std::vector<double> opt_hyper, bool opt_zero_grad) {
  const auto gf = fwd_geom(N, H, W, C, Co, R, S, stride, pad);
  const auto gd = dgrad_geom(N, H, W, C, Co, R, S, stride, pad);
  // optimizer tail (opt_tail.h): a flat-model range whose gradients are
  // final, updated by extra workgroups of this launch
  mfl::OptTail ot;
  const bool tail = opt_tail_args(ot, opt_p, opt_g, opt_m, opt_v, opt_anchor, opt_mirror, opt_lr_scale, opt_step,
                                  opt_mode, opt_hyper, opt_zero_grad);
  torch::Tensor xtmp, dtmp;
  const float* xs = dysrc(x, (int64_t)N * H * W * C, xtmp, "x");
  const float* dyp = dysrc(dy, (int64_t)gf.M * Co, dtmp);
  check_f32(dw, (int64_t)Co * R * S * C, "dw");
  check_f32(w, (int64_t)Co * R * S * C, "w");
  check_f32(dx, (int64_t)N * H * W * C, "dx");
  mfl::BnBwdFusion32 f;
  const bool fuse = bn_acc.has_value() && bn_acc->defined();
  if (fuse) {
    TORCH_CHECK(bn_z.has_value() && bn_mean.has_value() && bn_invstd.has_value(), "bn fusion operands");
    check_f32(*bn_z, dx.numel(), "bn_z");
    if (bn_y.has_value() && bn_y->defined()) check_f32(*bn_y, dx.numel(), "bn_y");
    check_f32(*bn_mean, C, "bn_mean");
    check_f32(*bn_invstd, C, "bn_invstd");
    f.z = fp(*bn_z);
    f.y = opt_ptr<float>(bn_y);
    f.mean = fp(*bn_mean);
    f.invstd = fp(*bn_invstd);
    f.acc = stats_ptr(bn_acc, C);
    f.reps = reps_of(*bn_acc, C);
  }
  const auto pd = C32_CALL(plan_conv32, gd, 1);
  const auto pw = C32_CALL(plan_conv32, gf, 2);
  float* slab = nullptr;
  int* counters = nullptr;
  if (pd.splits > 1) {
    TORCH_CHECK(ws.has_value() && ws->defined(), "split-K workspace required");
    check_f32(*ws, ws_floats(gd, pd), "workspace", false);
    counters = reinterpret_cast<int*>(ws->data_ptr<float>());
    slab = ws->data_ptr<float>() + kCounterWords;
  }
  torch::Tensor tmp;
  const float* wb = wsrc(w, wp, tmp);
  if (C32_CALL(launch_conv32_bwd_pair, gd, pd, gf, pw, dyp, wb, fp(dx), slab, counters, accumulate,
                                  fuse ? &f : nullptr, xs, fp(dw), cur_stream(dx), tail ? &ot : nullptr))
    return;
  C32_CALL(launch_conv32_wgrad, gf, pw, xs, dyp, fp(dw), true, cur_stream(dw));
  C32_CALL(launch_conv32_gemm, gd, true, pd, dyp, wb, fp(dx), slab, counters, nullptr, accumulate,
                          fuse ? &f : nullptr, cur_stream(dx));
  if (tail) opt_tail_fallback(ot, cur_stream(dx));
}

void conv32_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor dw, int64_t N, int64_t H, int64_t W, int64_t C,
                  int64_t Co, int64_t R, int64_t S, int64_t stride, int64_t pad, bool accumulate) {
  const auto g = fwd_geom(N, H, W, C, Co, R, S, stride, pad);
  torch::Tensor xtmp, dtmp;
  const float* xs = dysrc(x, (int64_t)N * H * W * C, xtmp, "x");
  const float* dyp = dysrc(dy, (int64_t)g.M * Co, dtmp);
  check_f32(dw, (int64_t)Co * R * S * C, "dw");
  const auto p = C32_CALL(plan_conv32, g, 2);
  if (!accumulate && p.splits > 1) dw.zero_();
  C32_CALL(launch_conv32_wgrad, g, p, xs, dyp, fp(dw), accumulate, cur_stream(dw));
}

// ---- BatchNorm -----------------------------------------------------------
void check_nhwc32(const torch::Tensor& x, int64_t C) {
  check_f32(x, 0, "activation", false);
  TORCH_CHECK(x.numel() % C == 0, "NHWC tensor not divisible by C");
  TORCH_CHECK(C % 4 == 0 && C <= 4096, "BN channels must be a multiple of 4, <= 4096");
}
void check_pc(const torch::Tensor& t, int64_t C, const char* nm) { check_f32(t, C, nm); }
const double* acc_ptr(const torch::Tensor& acc, int64_t C) {
  TORCH_CHECK(acc.is_cuda() && acc.is_contiguous() && acc.scalar_type() == torch::kFloat64 && acc.numel() >= 2 * C,
              "BN accumulator must be a contiguous fp64 device tensor of >= 2*C elements");
  return acc.data_ptr<double>();
}

void bn32_stats(torch::Tensor x, int64_t C, torch::Tensor acc) {
  check_nhwc32(x, C);
  acc_ptr(acc, C);
  mfl::launch_bn32_stats(fp(x), x.numel() / C, (int)C, acc.data_ptr<double>(), cur_stream(x), reps_of(acc, C));
}

mfl::BnFwdArgs32 bn32_args(torch::Tensor x, int64_t C, c10::optional<torch::Tensor> acc, torch::Tensor gamma,
                           torch::Tensor beta, torch::Tensor mean, torch::Tensor invstd, torch::Tensor run_mean,
                           torch::Tensor run_var, c10::optional<torch::Tensor> residual, torch::Tensor y, bool relu,
                           bool train, double momentum, double eps) {
  check_nhwc32(x, C);
  check_nhwc32(y, C);
  TORCH_CHECK(y.numel() == x.numel(), "bn y size");
  for (auto* t : {&gamma, &beta, &mean, &invstd, &run_mean, &run_var}) check_pc(*t, C, "bn param");
  mfl::BnFwdArgs32 a{};
  a.x = fp(x);
  if (residual.has_value() && residual->defined()) {
    check_nhwc32(*residual, C);
    TORCH_CHECK(residual->numel() == x.numel(), "residual size");
    a.residual = fp(*residual);
  }
  a.y = fp(y);
  if (train) {
    TORCH_CHECK(acc.has_value() && acc->defined(), "train-mode BN needs the statistics accumulator");
    a.acc = acc_ptr(*acc, C);
    a.reps = reps_of(*acc, C);
    TORCH_CHECK(a.reps <= 8, "at most 8 BN accumulator replicas");
  }
  a.gamma = fp(gamma);
  a.beta = fp(beta);
  a.mean = fp(mean);
  a.invstd = fp(invstd);
  a.run_mean = fp(run_mean);
  a.run_var = fp(run_var);
  a.M = x.numel() / C;
  a.C = (int)C;
  a.momentum = (float)momentum;
  a.eps = (float)eps;
  a.train = train ? 1 : 0;
  a.relu = relu ? 1 : 0;
  return a;
}

// yp (optional, int32 of y's size): also write y's packed bf16x3 split
uint32_t* yp_ptr(const c10::optional<torch::Tensor>& yp, const torch::Tensor& y) {
  if (!yp.has_value() || !yp->defined()) return nullptr;
  TORCH_CHECK(yp->is_cuda() && yp->is_contiguous() && yp->scalar_type() == torch::kInt32 && yp->numel() == y.numel(),
              "yp: contiguous int32 device tensor of y's size");
  return reinterpret_cast<uint32_t*>(yp->data_ptr());
}

void bn32_apply(torch::Tensor x, int64_t C, c10::optional<torch::Tensor> acc, torch::Tensor gamma, torch::Tensor beta,
                torch::Tensor mean, torch::Tensor invstd, torch::Tensor run_mean, torch::Tensor run_var,
                c10::optional<torch::Tensor> residual, torch::Tensor y, bool relu, bool train, double momentum,
                double eps, c10::optional<torch::Tensor> yp) {
  auto a = bn32_args(x, C, acc, gamma, beta, mean, invstd, run_mean, run_var, residual, y, relu, train, momentum, eps);
  a.yp = yp_ptr(yp, y);
  mfl::launch_bn32_apply(a, cur_stream(x));
}

// shortcut BN (no ReLU) + conv1 BN (ReLU) of a downsampling block in one launch
void bn32_apply_pair(torch::Tensor x1, torch::Tensor gamma1, torch::Tensor beta1, torch::Tensor mean1,
                     torch::Tensor invstd1, torch::Tensor rm1, torch::Tensor rv1, c10::optional<torch::Tensor> acc1,
                     torch::Tensor y1, torch::Tensor x2, torch::Tensor gamma2, torch::Tensor beta2,
                     torch::Tensor mean2, torch::Tensor invstd2, torch::Tensor rm2, torch::Tensor rv2,
                     c10::optional<torch::Tensor> acc2, torch::Tensor y2, int64_t C, bool train, double momentum,
                     double eps, c10::optional<torch::Tensor> yp2) {
  const auto a1 = bn32_args(x1, C, acc1, gamma1, beta1, mean1, invstd1, rm1, rv1, c10::nullopt, y1, false, train,
                            momentum, eps);
  auto a2 = bn32_args(x2, C, acc2, gamma2, beta2, mean2, invstd2, rm2, rv2, c10::nullopt, y2, true, train,
                      momentum, eps);
  a2.yp = yp_ptr(yp2, y2);
  mfl::launch_bn32_apply_pair(a1, a2, cur_stream(x1));
}

// conv1 (3x3 / s2) + projection shortcut (1x1 / s2) of one x: one launch when both plans pair
void conv32_forward_pair(torch::Tensor x, torch::Tensor w1, torch::Tensor y1, c10::optional<torch::Tensor> ws1,
                         c10::optional<torch::Tensor> stats1, torch::Tensor w2, torch::Tensor y2,
                         c10::optional<torch::Tensor> ws2, c10::optional<torch::Tensor> stats2, int64_t N, int64_t H,
                         int64_t W, int64_t C, int64_t Co, c10::optional<torch::Tensor> wp1,
                         c10::optional<torch::Tensor> wp2) {
  const auto g1 = fwd_geom(N, H, W, C, Co, 3, 3, 2, 1);
  const auto g2 = fwd_geom(N, H, W, C, Co, 1, 1, 2, 0);
  TORCH_CHECK(g1.M == g2.M, "conv1 / shortcut output sizes differ");
  torch::Tensor xtmp;
  const float* xs = dysrc(x, N * H * W * C, xtmp, "x");
  check_f32(w1, Co * 9 * C, "w1");
  check_f32(w2, Co * C, "w2");
  check_f32(y1, (int64_t)g1.M * Co, "y1");
  check_f32(y2, (int64_t)g2.M * Co, "y2");
  const auto p1 = C32_CALL(plan_conv32, g1, 0), p2 = C32_CALL(plan_conv32, g2, 0);
  auto slab = [&](const mfl::ConvGeom& g, const mfl::ConvPlan& p, const c10::optional<torch::Tensor>& ws,
                  float*& ys, int*& cn) {
    ys = nullptr;
    cn = nullptr;
    if (p.splits > 1) {
      TORCH_CHECK(ws.has_value() && ws->defined(), "split-K workspace required");
      check_f32(*ws, ws_floats(g, p), "workspace", false);
      cn = reinterpret_cast<int*>(ws->data_ptr<float>());
      ys = ws->data_ptr<float>() + kCounterWords;
    }
  };
  float *ys1, *ys2;
  int *c1, *c2;
  slab(g1, p1, ws1, ys1, c1);
  slab(g2, p2, ws2, ys2, c2);
  double* st1 = stats_ptr(stats1, Co);
  double* st2 = stats_ptr(stats2, Co);
  const int r1 = st1 ? reps_of(*stats1, Co) : 1, r2 = st2 ? reps_of(*stats2, Co) : 1;
  torch::Tensor t1, t2;
  const float* wb1 = wsrc(w1, wp1, t1);
  const float* wb2 = wsrc(w2, wp2, t2);
  if (C32_CALL(launch_conv32_fwd_pair, g1, p1, wb1, fp(y1), ys1, c1, st1, r1, g2, p2, wb2, fp(y2), ys2, c2, st2, r2,
                                  xs, cur_stream(y1)))
    return;
  run(g1, false, xs, wb1, y1, ws1, st1, false, nullptr, r1);
  run(g2, false, xs, wb2, y2, ws2, st2, false, nullptr, r2);
}

// Validated BN-backward apply arguments (and, unless presummed, the reduce
// launch that completes `acc` first).
static mfl::BnBwdArgs32 bn32_bwd_args(torch::Tensor dy, torch::Tensor x, c10::optional<torch::Tensor> y, int64_t C,
                                      torch::Tensor gamma, torch::Tensor mean, torch::Tensor invstd, torch::Tensor acc,
                                      c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta,
                                      torch::Tensor dx, c10::optional<torch::Tensor> dy_masked, bool presummed,
                                      c10::optional<torch::Tensor> z2, c10::optional<torch::Tensor> mean2,
                                      c10::optional<torch::Tensor> invstd2, c10::optional<torch::Tensor> acc2) {
  check_nhwc32(dy, C);
  check_nhwc32(x, C);
  // an int32 dx receives the packed bf16x3 split of the gradient: the dY
  // operand of the layer's bf16x3 dgrad / wgrad (see dysrc)
  const bool pack_dx = dx.scalar_type() == torch::kInt32;
  if (pack_dx) {
    TORCH_CHECK(dx.is_cuda() && dx.is_contiguous(), "packed dx: contiguous int32 device tensor");
  } else {
    check_nhwc32(dx, C);
  }
  TORCH_CHECK(dy.numel() == x.numel() && dx.numel() == x.numel(), "bn bwd sizes");
  for (auto* t : {&gamma, &mean, &invstd}) check_pc(*t, C, "bn param");
  mfl::BnBwdArgs32 a{};
  a.dy = fp(dy);
  a.x = fp(x);
  if (y.has_value() && y->defined()) {
    check_nhwc32(*y, C);
    TORCH_CHECK(y->numel() == x.numel(), "bn bwd y");
    a.y = fp(*y);
  }
  if (dy_masked.has_value() && dy_masked->defined()) {
    check_nhwc32(*dy_masked, C);
    TORCH_CHECK(dy_masked->numel() == x.numel(), "dy_masked size");
    a.dy_masked = fp(*dy_masked);
  }
  if (dgamma.has_value() && dgamma->defined()) { check_pc(*dgamma, C, "dgamma"); a.dgamma = fp(*dgamma); }
  if (dbeta.has_value() && dbeta->defined()) { check_pc(*dbeta, C, "dbeta"); a.dbeta = fp(*dbeta); }
  a.acc = acc_ptr(acc, C);
  a.reps = reps_of(acc, C);
  TORCH_CHECK(a.reps <= 8, "at most 8 BN accumulator replicas");
  a.gamma = fp(gamma);
  a.mean = fp(mean);
  a.invstd = fp(invstd);
  a.dx = reinterpret_cast<float*>(dx.data_ptr());
  a.pack_dx = pack_dx ? 1 : 0;
  a.M = x.numel() / C;
  a.C = (int)C;
  if (acc2.has_value() && acc2->defined()) {
    TORCH_CHECK(a.dy_masked != nullptr, "the side reduction runs over dy_masked");
    TORCH_CHECK(C / 4 <= 256 && 256 % (C / 4) == 0, "side reduction needs C / 4 dividing 256");
    TORCH_CHECK(z2.has_value() && mean2.has_value() && invstd2.has_value(), "side reduction operands");
    check_nhwc32(*z2, C);
    TORCH_CHECK(z2->numel() == x.numel(), "side z size");
    check_pc(*mean2, C, "mean2");
    check_pc(*invstd2, C, "invstd2");
    a.z2 = fp(*z2);
    a.mean2 = fp(*mean2);
    a.invstd2 = fp(*invstd2);
    a.acc2 = const_cast<double*>(acc_ptr(*acc2, C));
    a.reps2 = reps_of(*acc2, C);
  }
  if (!presummed)
    mfl::launch_bn32_bwd_reduce(a.dy, a.x, a.y, a.mean, a.invstd, a.M, a.C, acc.data_ptr<double>(), cur_stream(x),
                                a.reps);
  return a;
}

void bn32_backward_side(torch::Tensor dy, torch::Tensor x, c10::optional<torch::Tensor> y, int64_t C,
                        torch::Tensor gamma, torch::Tensor mean, torch::Tensor invstd, torch::Tensor acc,
                        c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta, torch::Tensor dx,
                        c10::optional<torch::Tensor> dy_masked, bool presummed, c10::optional<torch::Tensor> z2,
                        c10::optional<torch::Tensor> mean2, c10::optional<torch::Tensor> invstd2,
                        c10::optional<torch::Tensor> acc2) {
  const auto a = bn32_bwd_args(dy, x, y, C, gamma, mean, invstd, acc, dgamma, dbeta, dx, dy_masked, presummed, z2,
                               mean2, invstd2, acc2);
  mfl::launch_bn32_bwd_apply(a, cur_stream(x));
}

// Two presummed BN-backward applies in one launch (bn32.hip
// bn32_bwd_apply_pair_kernel): role 1 a downsampling block's conv1 (with its
// ReLU mask y1, or none when dy1 arrives masked), role 2 its projection
// shortcut (no ReLU).
void bn32_backward_pair(torch::Tensor dy1, torch::Tensor x1, c10::optional<torch::Tensor> y1, int64_t C1,
                        torch::Tensor gamma1,
                        torch::Tensor mean1, torch::Tensor invstd1, torch::Tensor acc1, torch::Tensor dgamma1,
                        torch::Tensor dbeta1, torch::Tensor dx1, torch::Tensor dy2, torch::Tensor x2, int64_t C2,
                        torch::Tensor gamma2, torch::Tensor mean2, torch::Tensor invstd2, torch::Tensor acc2,
                        torch::Tensor dgamma2, torch::Tensor dbeta2, torch::Tensor dx2) {
  const auto a1 = bn32_bwd_args(dy1, x1, y1, C1, gamma1, mean1, invstd1, acc1, dgamma1, dbeta1, dx1, c10::nullopt,
                                true, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt);
  const auto a2 = bn32_bwd_args(dy2, x2, c10::nullopt, C2, gamma2, mean2, invstd2, acc2, dgamma2, dbeta2, dx2,
                                c10::nullopt, true, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt);
  TORCH_CHECK(a1.pack_dx == a2.pack_dx, "bn backward pair: both dx packed or both fp32");
  mfl::launch_bn32_bwd_apply_pair(a1, a2, cur_stream(x1));
}

void bn32_backward(torch::Tensor dy, torch::Tensor x, c10::optional<torch::Tensor> y, int64_t C, torch::Tensor gamma,
                   torch::Tensor mean, torch::Tensor invstd, torch::Tensor acc, c10::optional<torch::Tensor> dgamma,
                   c10::optional<torch::Tensor> dbeta, torch::Tensor dx, c10::optional<torch::Tensor> dy_masked,
                   bool presummed) {
  bn32_backward_side(dy, x, y, C, gamma, mean, invstd, acc, dgamma, dbeta, dx, dy_masked, presummed, c10::nullopt,
                     c10::nullopt, c10::nullopt, c10::nullopt);
}

// The stem's BatchNorm(+ReLU) backward and its 3x3 weight gradient in one
// launch (bn32.hip stem_bwd32_kernel); `acc` holds the complete backward sums
// (presummed by the first block's dgrad); dw (KRSC, zero on entry) += ...
bool stem_backward32_ok(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Co) {
  return mfl::stem_bwd32_ok((int)N, (int)H, (int)W, (int)Cin, (int)Co);
}

void stem_backward32(torch::Tensor dy, torch::Tensor z, torch::Tensor y, torch::Tensor gamma, torch::Tensor mean,
                     torch::Tensor invstd, torch::Tensor acc, c10::optional<torch::Tensor> dgamma,
                     c10::optional<torch::Tensor> dbeta, torch::Tensor x, torch::Tensor dw,
                     c10::optional<torch::Tensor> opt_p, c10::optional<torch::Tensor> opt_g,
                     c10::optional<torch::Tensor> opt_m, c10::optional<torch::Tensor> opt_v,
                     c10::optional<torch::Tensor> opt_anchor, c10::optional<torch::Tensor> opt_mirror,
                     c10::optional<torch::Tensor> opt_lr_scale, c10::optional<torch::Tensor> opt_step,
                     int64_t opt_mode, std::vector<double> opt_hyper, bool opt_zero_grad) {
  TORCH_CHECK(z.dim() == 4 && x.dim() == 4, "stem backward: NHWC tensors");
  const int64_t N = z.size(0), H = z.size(1), W = z.size(2), Co = z.size(3), Cin = x.size(3);
  TORCH_CHECK(x.size(0) == N && x.size(1) == H && x.size(2) == W, "stem backward: x / z shapes");
  TORCH_CHECK(stem_backward32_ok(N, H, W, Cin, Co), "stem backward: unsupported shape");
  // fp32 activations, or the bf16 option's (dy, z, y, x all bf16)
  const bool bf = z.scalar_type() == torch::kBFloat16;
  for (auto* t : {&dy, &z, &y, &x}) {
    if (bf) {
      TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == torch::kBFloat16,
                  "stem backward: contiguous bf16 device tensors expected");
    } else {
      check_nhwc32(*t, t == &x ? Cin : Co);
    }
  }
  TORCH_CHECK(dy.numel() == z.numel() && y.numel() == z.numel(), "stem backward sizes");
  TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == torch::kFloat32 && dw.is_contiguous() && dw.numel() == Co * 9 * Cin,
              "stem backward: dw [Co][3][3][Cin] fp32");
  for (auto* t : {&gamma, &mean, &invstd}) check_pc(*t, Co, "bn param");
  mfl::BnBwdArgs32 a{};
  a.dy = reinterpret_cast<const float*>(dy.data_ptr());
  a.x = reinterpret_cast<const float*>(z.data_ptr());
  a.y = reinterpret_cast<const float*>(y.data_ptr());
  a.acc = acc_ptr(acc, Co);
  a.reps = reps_of(acc, Co);
  TORCH_CHECK(a.reps <= 8, "at most 8 BN accumulator replicas");
  a.gamma = fp(gamma);
  a.mean = fp(mean);
  a.invstd = fp(invstd);
  if (dgamma.has_value() && dgamma->defined()) { check_pc(*dgamma, Co, "dgamma"); a.dgamma = fp(*dgamma); }
  if (dbeta.has_value() && dbeta->defined()) { check_pc(*dbeta, Co, "dbeta"); a.dbeta = fp(*dbeta); }
  a.M = z.numel() / Co;
  a.C = (int)Co;
  // optimizer tail: the rest of the model (every variable but the stem's),
  // final by now, rides in this launch (opt_tail.h)
  mfl::OptTail ot;
  const bool tail = opt_tail_args(ot, opt_p, opt_g, opt_m, opt_v, opt_anchor, opt_mirror, opt_lr_scale, opt_step,
                                  opt_mode, opt_hyper, opt_zero_grad);
  if (bf)
    mfl::launch_stem_bwd_bf16(a, reinterpret_cast<const uint16_t*>(x.data_ptr()), (int)N, fp(dw), cur_stream(z),
                              tail ? &ot : nullptr);
  else
    mfl::launch_stem_bwd32(a, fp(x), (int)N, (int)H, (int)W, (int)Cin, fp(dw), cur_stream(z), tail ? &ot : nullptr);
}

// ---- head / data ---------------------------------------------------------
void head32_forward_backward(torch::Tensor x, int64_t B, int64_t HW, int64_t C, torch::Tensor W,
                             c10::optional<torch::Tensor> bias, torch::Tensor labels,
                             c10::optional<torch::Tensor> feat, c10::optional<torch::Tensor> dlogits,
                             c10::optional<torch::Tensor> dx, c10::optional<torch::Tensor> stats, bool backward,
                             c10::optional<torch::Tensor> dW, c10::optional<torch::Tensor> db) {
  check_f32(x, B * HW * C, "head x");
  check_f32(W, 0, "head W", false);
  TORCH_CHECK(W.numel() % C == 0, "head W");
  const int64_t K = W.numel() / C;
  TORCH_CHECK(labels.is_cuda() && labels.is_contiguous() && labels.scalar_type() == torch::kInt32 &&
                  labels.numel() >= B, "labels");
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && K <= 1024, "head: C must be a multiple of 8 (<= 2048), K <= 1024");
  const bool fuse = dW.has_value() && dW->defined();
  if (fuse) {
    check_f32(*dW, K * C, "head dW");
    if (db.has_value() && db->defined()) check_f32(*db, K, "head db");
  }
  if (backward) {
    TORCH_CHECK(feat.has_value() && dlogits.has_value() && dx.has_value(), "bwd buffers");
    TORCH_CHECK(feat->numel() >= B * C && dlogits->numel() >= B * K, "bwd buffer sizes");
    check_f32(*dx, x.numel(), "head dx");
  }
  mfl::launch_head32_fwd_bwd(fp(x), (int)B, (int)HW, (int)C, fp(W), opt_ptr<float>(bias), (int)K,
                             labels.data_ptr<int>(), opt_ptr<float>(feat), opt_ptr<float>(dlogits),
                             opt_ptr<float>(dx), opt_ptr<float>(stats), backward, cur_stream(x),
                             fuse ? fp(*dW) : nullptr, fuse ? opt_ptr<float>(db) : nullptr);
}

// The fp32 head with the last block's BatchNorm (+ residual, + ReLU) applied
// in its pooling loop and, in train mode, the BN-backward sums of dx added
// into acc_b (the caller then runs that BN's backward presummed).
void head32_forward_backward_bn(int64_t B, int64_t HW, int64_t C, torch::Tensor W, c10::optional<torch::Tensor> bias,
                                torch::Tensor labels, c10::optional<torch::Tensor> feat,
                                c10::optional<torch::Tensor> dlogits, c10::optional<torch::Tensor> dx,
                                c10::optional<torch::Tensor> stats, bool backward, c10::optional<torch::Tensor> dW,
                                c10::optional<torch::Tensor> db, torch::Tensor z, torch::Tensor res,
                                c10::optional<torch::Tensor> acc, torch::Tensor gamma, torch::Tensor beta,
                                torch::Tensor mean, torch::Tensor invstd, torch::Tensor run_mean,
                                torch::Tensor run_var, double momentum, double eps, bool train, torch::Tensor y,
                                c10::optional<torch::Tensor> acc_b) {
  const int64_t n = B * HW * C;
  // fp32 activations, or the bf16 option's (z / res / y / dx bf16)
  const bool bf = z.scalar_type() == torch::kBFloat16;
  auto check_act = [&](const torch::Tensor& t, const char* nm) {
    if (!bf) return check_f32(t, n, nm);
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kBFloat16 && t.numel() == n, nm,
                ": contiguous bf16 device tensor of ", n, " elements expected");
  };
  check_act(z, "head z");
  check_act(res, "head res");
  check_act(y, "head y");
  for (auto* t : {&gamma, &beta, &mean, &invstd, &run_mean, &run_var}) check_pc(*t, C, "head bn param");
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "head: C must be a multiple of 8 (<= 2048)");
  check_f32(W, 0, "head W", false);
  TORCH_CHECK(W.numel() % C == 0, "head W");
  const int64_t K = W.numel() / C;
  TORCH_CHECK(K <= 1024, "head: K <= 1024");
  TORCH_CHECK(labels.is_cuda() && labels.is_contiguous() && labels.scalar_type() == torch::kInt32 &&
                  labels.numel() >= B, "labels");
  mfl::HeadBn hb;
  hb.z = reinterpret_cast<const float*>(z.data_ptr());
  hb.res = reinterpret_cast<const float*>(res.data_ptr());
  if (train) {
    TORCH_CHECK(acc.has_value() && acc->defined(), "train-mode BN needs its statistics accumulator");
    hb.acc = acc_ptr(*acc, C);
    hb.reps = reps_of(*acc, C);
    TORCH_CHECK(hb.reps <= 8, "at most 8 BN accumulator replicas");
  }
  hb.gamma = fp(gamma);
  hb.beta = fp(beta);
  hb.mean = fp(mean);
  hb.invstd = fp(invstd);
  hb.run_mean = fp(run_mean);
  hb.run_var = fp(run_var);
  hb.momentum = (float)momentum;
  hb.eps = (float)eps;
  hb.train = train ? 1 : 0;
  hb.y = reinterpret_cast<float*>(y.data_ptr());
  if (backward && acc_b.has_value() && acc_b->defined()) {
    hb.acc_b = const_cast<double*>(acc_ptr(*acc_b, C));
    hb.reps_b = reps_of(*acc_b, C);
  }
  const bool fuse = dW.has_value() && dW->defined();
  if (fuse) {
    check_f32(*dW, K * C, "head dW");
    if (db.has_value() && db->defined()) check_f32(*db, K, "head db");
  }
  if (backward) {
    TORCH_CHECK(feat.has_value() && dlogits.has_value() && dx.has_value(), "bwd buffers");
    TORCH_CHECK(feat->numel() >= B * C && dlogits->numel() >= B * K, "bwd buffer sizes");
    check_act(*dx, "head dx");
  }
  // split head scratch: [B][C / 128][K] partial logits (stream-ordered lifetime)
  torch::Tensor lpart;
  if (C % 128 == 0 && feat.has_value() && feat->defined() && feat->numel() >= B * C)
    lpart = torch::empty({B * (C / 128) * K}, z.options().dtype(torch::kFloat32));
  float* lp = lpart.defined() ? lpart.data_ptr<float>() : nullptr;
  if (bf) {
    mfl::launch_head_fwd_bwd(reinterpret_cast<const uint16_t*>(y.data_ptr()), (int)B, (int)HW, (int)C, fp(W),
                             opt_ptr<float>(bias), (int)K, labels.data_ptr<int>(), opt_ptr<float>(feat),
                             opt_ptr<float>(dlogits),
                             backward ? reinterpret_cast<uint16_t*>(dx->data_ptr()) : nullptr,
                             opt_ptr<float>(stats), backward, cur_stream(z), fuse ? fp(*dW) : nullptr,
                             fuse ? opt_ptr<float>(db) : nullptr, &hb, lp);
    return;
  }
  mfl::launch_head32_fwd_bwd(fp(y), (int)B, (int)HW, (int)C, fp(W), opt_ptr<float>(bias), (int)K,
                             labels.data_ptr<int>(), opt_ptr<float>(feat), opt_ptr<float>(dlogits),
                             opt_ptr<float>(dx), opt_ptr<float>(stats), backward, cur_stream(z),
                             fuse ? fp(*dW) : nullptr, fuse ? opt_ptr<float>(db) : nullptr, &hb, lp);
}

// fp32 rows are gathered as 16-B units, like the bf16 ones
void gather_batch32(torch::Tensor shard, torch::Tensor labels, torch::Tensor perm, torch::Tensor step,
                    int64_t steps_per_epoch, int64_t B, torch::Tensor xb, torch::Tensor yb,
                    c10::optional<torch::Tensor> xp) {
  check_f32(shard, 0, "shard", false);
  check_f32(xb, 0, "xb", false);
  for (auto* t : {&labels, &perm, &step, &yb})
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == torch::kInt32, "int32 operand");
  const int64_t n = labels.numel();
  TORCH_CHECK(n > 0 && shard.numel() % n == 0, "shard rows");
  const int64_t row = shard.numel() / n;
  TORCH_CHECK(row % 4 == 0, "row must be a multiple of 4 fp32 elements");
  TORCH_CHECK(xb.numel() == B * row && yb.numel() >= B, "batch buffers");
  TORCH_CHECK(perm.numel() >= steps_per_epoch * B, "permutation too short");
  mfl::launch_gather_batch(reinterpret_cast<const uint16_t*>(shard.data_ptr()), labels.data_ptr<int>(),
                           perm.data_ptr<int>(), step.data_ptr<int>(), (int)steps_per_epoch, (int)B, row * 2,
                           reinterpret_cast<uint16_t*>(xb.data_ptr()), yb.data_ptr<int>(), cur_stream(shard),
                           yp_ptr(xp, xb));
}

}  // namespace

void register_fp32(pybind11::module& m) {
  m.def("set_conv32_mode", &set_conv32_mode);
  m.def("set_conv32_pair_ring", &set_conv32_pair_ring);
  m.def("set_conv32_plan_overrides", &set_conv32_plan_overrides);
  m.def("set_bn32_grid_cap", [](int64_t cap) { mfl::set_bn32_grid_cap((int)cap); });
  m.def("conv32_mode", &conv32_mode);
  m.def("conv32_plan", &conv32_plan);
  m.def("conv32_forward", &conv32_forward);
  m.def("conv32_dgrad", &conv32_dgrad);
  m.def("conv32_wgrad", &conv32_wgrad);
  m.def("conv32_backward_pair", &conv32_backward_pair);
  m.def("bn32_stats", &bn32_stats);
  m.def("bn32_apply", &bn32_apply);
  m.def("bn32_apply_pair", &bn32_apply_pair);
  m.def("conv32_forward_pair", &conv32_forward_pair);
  m.def("bn32_backward", &bn32_backward);
  m.def("bn32_backward_side", &bn32_backward_side);
  m.def("bn32_backward_pair", &bn32_backward_pair);
  m.def("stem_backward32", &stem_backward32);
  m.def("stem_backward32_ok", &stem_backward32_ok);
  m.def("head32_forward_backward", &head32_forward_backward);
  m.def("head32_forward_backward_bn", &head32_forward_backward_bn);
  m.def("gather_batch32", &gather_batch32);
}
