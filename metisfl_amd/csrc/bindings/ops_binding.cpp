// torch binding for the metisfl_amd HIP kernels (module ``metisfl_amd._ops``).
//
// Every entry point validates shapes/dtypes on the host BEFORE launching (a
// mis-shaped launch of a hand-written kernel can fault the whole GPU), then
// launches on the caller's current HIP stream so that the call is capturable
// into a hipGraph.  No function here allocates device memory.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <vector>

#include "kernels/launchers.h"

namespace {

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a device tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_T(t, dt) \
  TORCH_CHECK((t).scalar_type() == (dt), #t " has dtype ", (t).scalar_type(), ", expected ", dt)
#define CHECK_IN(t, dt) \
  do {                  \
    CHECK_DEV(t);       \
    CHECK_CONTIG(t);    \
    CHECK_T(t, dt);     \
  } while (0)

hipStream_t cur_stream(const torch::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

template <typename T>
T* ptr_or_null(const c10::optional<torch::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_DEV(*t);
  CHECK_CONTIG(*t);
  return reinterpret_cast<T*>(t->data_ptr());
}

uint16_t* bf(const torch::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

// --------------------------------------------------------------------------
void fused_optimizer(int64_t mode, torch::Tensor p, torch::Tensor g,
                     c10::optional<torch::Tensor> m, c10::optional<torch::Tensor> v,
                     c10::optional<torch::Tensor> anchor, c10::optional<torch::Tensor> p16,
                     double lr, double l1, double l2, double momentum, double mu, double beta1,
                     double beta2, double eps, double wd, c10::optional<torch::Tensor> lr_scale,
                     c10::optional<torch::Tensor> step, bool zero_grad,
                     c10::optional<torch::Tensor> zero_region, bool tick) {
  CHECK_IN(p, torch::kFloat32);
  CHECK_IN(g, torch::kFloat32);
  const int64_t n = p.numel();
  TORCH_CHECK(g.numel() == n, "grad size mismatch");
  TORCH_CHECK(n % 4 == 0, "flat buffers must be padded to a multiple of 4 elements");
  auto need = [&](const c10::optional<torch::Tensor>& t, const char* nm) {
    TORCH_CHECK(t.has_value() && t->defined(), nm, " is required for this optimizer");
    CHECK_IN((*t), torch::kFloat32);
    TORCH_CHECK(t->numel() == n, nm, " size mismatch");
  };
  if (mode == mfl::OPT_MOMENTUM) need(m, "momentum buffer");
  if (mode == mfl::OPT_FEDPROX) need(anchor, "proximal anchor");
  if (mode == mfl::OPT_ADAM || mode == mfl::OPT_ADAMW) {
    need(m, "m");
    need(v, "v");
  }
  int mirror = 0;
  if (p16.has_value() && p16->defined()) {  // bf16 compute copy, or the int32 packed bf16x3 split
    TORCH_CHECK(p16->is_cuda() && p16->is_contiguous(), "weight mirror must be a contiguous device tensor");
    TORCH_CHECK(p16->scalar_type() == torch::kBFloat16 || p16->scalar_type() == torch::kInt32,
                "weight mirror is bf16 or int32 (packed split)");
    TORCH_CHECK(p16->numel() == n, "weight mirror size mismatch");
    mirror = p16->scalar_type() == torch::kInt32 ? 2 : 1;
  }
  if (lr_scale.has_value() && lr_scale->defined()) CHECK_IN((*lr_scale), torch::kFloat32);
  if (step.has_value() && step->defined()) CHECK_IN((*step), torch::kInt32);
  TORCH_CHECK(!tick || (step.has_value() && step->defined()), "tick needs the step counter");
  mfl::OptHyper h;
  h.lr = (float)lr; h.l1 = (float)l1; h.l2 = (float)l2; h.momentum = (float)momentum;
  h.mu = (float)mu; h.beta1 = (float)beta1; h.beta2 = (float)beta2; h.eps = (float)eps;
  h.wd = (float)wd;
  mfl::launch_fused_optimizer((int)mode, p.data_ptr<float>(), g.data_ptr<float>(),
                              ptr_or_null<float>(m), ptr_or_null<float>(v),
                              ptr_or_null<float>(anchor), mirror ? p16->data_ptr() : nullptr, n, h,
                              ptr_or_null<float>(lr_scale), ptr_or_null<int>(step), zero_grad,
                              zero_region.has_value() && zero_region->defined() ? zero_region->data_ptr() : nullptr,
                              zero_region.has_value() && zero_region->defined()
                                  ? (int64_t)(zero_region->numel() * zero_region->element_size()) / 16 * 16
                                  : 0,
                              cur_stream(p), tick ? step->data_ptr<int>() : nullptr, mirror);
}

void split_pack_f32(torch::Tensor x, torch::Tensor y) {
  CHECK_IN(x, torch::kFloat32);
  CHECK_IN(y, torch::kInt32);
  TORCH_CHECK(x.numel() == y.numel() && x.numel() % 4 == 0, "split pack size");
  mfl::launch_split_pack(x.data_ptr<float>(), reinterpret_cast<uint32_t*>(y.data_ptr()), x.numel(), cur_stream(x));
}

void cast_f32_bf16(torch::Tensor x, torch::Tensor y) {
  CHECK_IN(x, torch::kFloat32);
  CHECK_IN(y, torch::kBFloat16);
  TORCH_CHECK(x.numel() == y.numel() && x.numel() % 4 == 0, "cast size");
  mfl::launch_cast_f32_bf16(x.data_ptr<float>(), bf(y), x.numel(), cur_stream(x));
}

void scale_f32(torch::Tensor x, double w, c10::optional<torch::Tensor> wdev) {
  CHECK_IN(x, torch::kFloat32);
  TORCH_CHECK(x.numel() % 4 == 0, "scale size");
  mfl::launch_scale_f32(x.data_ptr<float>(), x.numel(), (float)w, ptr_or_null<float>(wdev),
                        cur_stream(x));
}

void tick(torch::Tensor step, int64_t inc) {
  CHECK_IN(step, torch::kInt32);
  mfl::launch_tick(step.data_ptr<int>(), (int)inc, cur_stream(step));
}

// --------------------------------------------------------------------------
int dtype_code(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kInt8: return 0;
    case torch::kInt16: return 1;
    case torch::kInt32: return 2;
    case torch::kInt64: return 3;
    case torch::kUInt8: return 4;
    case torch::kUInt16: return 5;
    case torch::kUInt32: return 6;
    case torch::kUInt64: return 7;
    case torch::kFloat32: return 8;
    case torch::kFloat64: return 9;
    default: TORCH_CHECK(false, "unsupported dtype for aggregation: ", t.scalar_type());
  }
  return -1;
}

void weighted_sum(torch::Tensor out, std::vector<torch::Tensor> xs, std::vector<double> ws) {
  CHECK_DEV(out);
  CHECK_CONTIG(out);
  TORCH_CHECK(xs.size() == ws.size() && !xs.empty(), "inputs/weights mismatch");
  const int code = dtype_code(out);
  const int64_t n = out.numel();
  for (auto& x : xs) {
    CHECK_DEV(x);
    CHECK_CONTIG(x);
    TORCH_CHECK(x.scalar_type() == out.scalar_type() && x.numel() == n, "input mismatch");
  }
  // Process learners in the reference's order, 16 per launch, accumulating.
  for (size_t base = 0; base < xs.size(); base += mfl::kMaxAggInputs) {
    mfl::AggInputs in{};
    in.count = (int)std::min<size_t>(mfl::kMaxAggInputs, xs.size() - base);
    for (int k = 0; k < in.count; ++k) {
      in.ptr[k] = xs[base + k].data_ptr();
      in.w[k] = ws[base + k];
    }
    mfl::launch_weighted_sum(code, out.data_ptr(), in, n, base > 0, cur_stream(out));
  }
}

void rolling_op(torch::Tensor y, c10::optional<torch::Tensor> x, int64_t op, double w) {
  CHECK_DEV(y);
  CHECK_CONTIG(y);
  const void* xp = nullptr;
  if (op <= 1) {
    TORCH_CHECK(x.has_value() && x->defined(), "merge needs x");
    CHECK_DEV(*x);
    CHECK_CONTIG(*x);
    TORCH_CHECK(x->scalar_type() == y.scalar_type() && x->numel() == y.numel(), "merge mismatch");
    xp = x->data_ptr();
  }
  mfl::launch_axpby(dtype_code(y), y.data_ptr(), xp, (double)op, w, y.numel(), cur_stream(y));
}

void count_zeros(torch::Tensor x, torch::Tensor tile_seg, torch::Tensor tile_beg,
                 torch::Tensor tile_end, torch::Tensor counts) {
  CHECK_DEV(x);
  CHECK_CONTIG(x);
  CHECK_IN(tile_seg, torch::kInt64);
  CHECK_IN(tile_beg, torch::kInt64);
  CHECK_IN(tile_end, torch::kInt64);
  CHECK_IN(counts, torch::kInt64);
  const int nt = (int)tile_seg.numel();
  TORCH_CHECK(tile_beg.numel() == nt && tile_end.numel() == nt, "tile table");
  mfl::launch_count_zeros(dtype_code(x), x.data_ptr(), tile_seg.data_ptr<int64_t>(),
                          tile_beg.data_ptr<int64_t>(), tile_end.data_ptr<int64_t>(), nt,
                          reinterpret_cast<unsigned long long*>(counts.data_ptr<int64_t>()),
                          cur_stream(x));
}

void ckks_pwa(torch::Tensor ptrs, torch::Tensor wq, torch::Tensor out, torch::Tensor moduli,
              int64_t nlimbs, int64_t ncoef, int64_t nct) {
  CHECK_IN(ptrs, torch::kInt64);
  CHECK_IN(wq, torch::kInt64);
  CHECK_IN(out, torch::kInt64);
  CHECK_IN(moduli, torch::kInt64);
  const int L = (int)ptrs.numel();
  TORCH_CHECK(wq.numel() == (int64_t)L * nlimbs * 2, "wq size");
  TORCH_CHECK(out.numel() == nct * 2 * nlimbs * ncoef, "out size");
  TORCH_CHECK(moduli.numel() == nlimbs, "moduli size");
  mfl::launch_ckks_pwa(reinterpret_cast<const uint64_t* const*>(ptrs.data_ptr<int64_t>()),
                       reinterpret_cast<const uint64_t*>(wq.data_ptr<int64_t>()), L,
                       reinterpret_cast<uint64_t*>(out.data_ptr<int64_t>()),
                       reinterpret_cast<const uint64_t*>(moduli.data_ptr<int64_t>()), (int)nlimbs,
                       ncoef, nct, cur_stream(out));
}

// --------------------------------------------------------------------------
void check_nhwc(const torch::Tensor& x, int64_t C) {
  CHECK_IN(x, torch::kBFloat16);
  TORCH_CHECK(x.numel() % C == 0, "NHWC tensor not divisible by C");
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "BN channels must be a multiple of 8, <= 2048");
}

void check_acc(const torch::Tensor& acc, int64_t C) {
  TORCH_CHECK(acc.is_cuda() && acc.is_contiguous() && acc.scalar_type() == torch::kFloat64,
              "BN accumulator must be a contiguous fp64 device tensor");
  TORCH_CHECK(acc.numel() >= 2 * C, "BN accumulator needs 2*C elements");
}
void check_pc(const torch::Tensor& t, int64_t C, const char* nm) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kFloat32, nm,
              " must be a contiguous fp32 device tensor");
  TORCH_CHECK(t.numel() == C, nm, " must have C elements");
}

// acc[0:C] += sum x, acc[C:2C] += sum x^2 over the M rows of an NHWC tensor.
void bn_stats(torch::Tensor x, int64_t C, torch::Tensor acc) {
  check_nhwc(x, C);
  check_acc(acc, C);
  mfl::launch_bn_stats(bf(x), x.numel() / C, (int)C, acc.data_ptr<double>(), cur_stream(x));
}

// y = relu?(bn(x) (+ residual)).  train: statistics from acc (sums over M rows),
// publishes mean/invstd and updates running stats; eval: running statistics.
mfl::BnFwdArgs bn_fwd_args(torch::Tensor x, int64_t C, c10::optional<torch::Tensor> acc, torch::Tensor gamma,
                           torch::Tensor beta, torch::Tensor mean, torch::Tensor invstd,
                           torch::Tensor run_mean, torch::Tensor run_var, c10::optional<torch::Tensor> residual,
                           torch::Tensor y, bool relu, bool train, double momentum, double eps);

void bn_apply(torch::Tensor x, int64_t C, c10::optional<torch::Tensor> acc, torch::Tensor gamma,
              torch::Tensor beta, torch::Tensor mean, torch::Tensor invstd,
              torch::Tensor run_mean, torch::Tensor run_var, c10::optional<torch::Tensor> residual,
              torch::Tensor y, bool relu, bool train, double momentum, double eps) {
  mfl::launch_bn_apply(bn_fwd_args(x, C, acc, gamma, beta, mean, invstd, run_mean, run_var, residual, y, relu,
                                   train, momentum, eps),
                       cur_stream(x));
}

// shortcut BN (no ReLU) + conv1 BN (ReLU) of a downsampling block, one launch
void bn_apply_pair(torch::Tensor x1, torch::Tensor gamma1, torch::Tensor beta1, torch::Tensor mean1,
                   torch::Tensor invstd1, torch::Tensor rm1, torch::Tensor rv1, c10::optional<torch::Tensor> acc1,
                   torch::Tensor y1, torch::Tensor x2, torch::Tensor gamma2, torch::Tensor beta2,
                   torch::Tensor mean2, torch::Tensor invstd2, torch::Tensor rm2, torch::Tensor rv2,
                   c10::optional<torch::Tensor> acc2, torch::Tensor y2, int64_t C, bool train, double momentum,
                   double eps) {
  const auto a1 = bn_fwd_args(x1, C, acc1, gamma1, beta1, mean1, invstd1, rm1, rv1, c10::nullopt, y1, false,
                              train, momentum, eps);
  const auto a2 = bn_fwd_args(x2, C, acc2, gamma2, beta2, mean2, invstd2, rm2, rv2, c10::nullopt, y2, true,
                              train, momentum, eps);
  mfl::launch_bn_apply_pair(a1, a2, cur_stream(x1));
}

mfl::BnFwdArgs bn_fwd_args(torch::Tensor x, int64_t C, c10::optional<torch::Tensor> acc, torch::Tensor gamma,
                           torch::Tensor beta, torch::Tensor mean, torch::Tensor invstd,
                           torch::Tensor run_mean, torch::Tensor run_var, c10::optional<torch::Tensor> residual,
                           torch::Tensor y, bool relu, bool train, double momentum, double eps) {
  check_nhwc(x, C);
  check_nhwc(y, C);
  TORCH_CHECK(y.numel() == x.numel(), "bn y size");
  for (auto* t : {&gamma, &beta, &mean, &invstd, &run_mean, &run_var}) check_pc(*t, C, "bn param");
  mfl::BnFwdArgs a{};
  a.x = bf(x);
  a.y = bf(y);
  if (train) {
    TORCH_CHECK(acc.has_value() && acc->defined(), "training BN needs the statistics accumulator");
    check_acc(*acc, C);
    a.acc = acc->data_ptr<double>();
  }
  if (residual.has_value() && residual->defined()) {
    check_nhwc(*residual, C);
    TORCH_CHECK(residual->numel() == x.numel(), "residual size");
    a.residual = bf(*residual);
  }
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.mean = mean.data_ptr<float>();
  a.invstd = invstd.data_ptr<float>();
  a.run_mean = run_mean.data_ptr<float>();
  a.run_var = run_var.data_ptr<float>();
  a.M = x.numel() / C;
  a.C = (int)C;
  a.momentum = (float)momentum;
  a.eps = (float)eps;
  a.train = train ? 1 : 0;
  a.relu = relu ? 1 : 0;
  return a;
}

// BN(+ReLU) backward: reduce into acc (fp64 atomics; must be zero on entry),
// then dx and (optionally) the masked dy for a residual shortcut.
void bn_backward(torch::Tensor dy, torch::Tensor x, c10::optional<torch::Tensor> y, int64_t C,
                 torch::Tensor gamma, torch::Tensor mean, torch::Tensor invstd, torch::Tensor acc,
                 c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta,
                 torch::Tensor dx, c10::optional<torch::Tensor> dy_masked, bool presummed) {
  check_nhwc(dy, C);
  check_nhwc(x, C);
  check_nhwc(dx, C);
  check_acc(acc, C);
  TORCH_CHECK(dy.numel() == x.numel() && dx.numel() == x.numel(), "bn bwd sizes");
  for (auto* t : {&gamma, &mean, &invstd}) check_pc(*t, C, "bn param");
  mfl::BnBwdArgs a{};
  a.dy = bf(dy);
  a.x = bf(x);
  if (y.has_value() && y->defined()) {
    check_nhwc(*y, C);
    TORCH_CHECK(y->numel() == x.numel(), "bn bwd y");
    a.y = bf(*y);
  }
  if (dy_masked.has_value() && dy_masked->defined()) {
    check_nhwc(*dy_masked, C);
    // (without y: dy arrives masked and is copied as is)
    a.dy_masked = bf(*dy_masked);
  }
  if (dgamma.has_value() && dgamma->defined()) { check_pc(*dgamma, C, "dgamma"); a.dgamma = dgamma->data_ptr<float>(); }
  if (dbeta.has_value() && dbeta->defined()) { check_pc(*dbeta, C, "dbeta"); a.dbeta = dbeta->data_ptr<float>(); }
  a.acc = acc.data_ptr<double>();
  a.gamma = gamma.data_ptr<float>();
  a.mean = mean.data_ptr<float>();
  a.invstd = invstd.data_ptr<float>();
  a.dx = bf(dx);
  a.M = x.numel() / C;
  a.C = (int)C;
  auto s = cur_stream(x);
  // presummed: the producer of dy (a conv dgrad epilogue) already added
  // sum(g) / sum(g*xhat) into acc
  if (!presummed)
    mfl::launch_bn_bwd_reduce(a.dy, a.x, a.y, a.mean, a.invstd, a.M, a.C, acc.data_ptr<double>(), s);
  mfl::launch_bn_bwd_apply(a, s);
}

void head_forward_backward(torch::Tensor x, int64_t B, int64_t HW, int64_t C, torch::Tensor W,
                           c10::optional<torch::Tensor> bias, torch::Tensor labels,
                           c10::optional<torch::Tensor> feat, c10::optional<torch::Tensor> dlogits,
                           c10::optional<torch::Tensor> dx, c10::optional<torch::Tensor> stats,
                           bool backward, c10::optional<torch::Tensor> dW,
                           c10::optional<torch::Tensor> db) {
  CHECK_IN(x, torch::kBFloat16);
  TORCH_CHECK(x.numel() == B * HW * C, "head x size");
  CHECK_IN(W, torch::kFloat32);
  TORCH_CHECK(W.numel() % C == 0, "head W");
  const int64_t K = W.numel() / C;
  CHECK_IN(labels, torch::kInt32);
  TORCH_CHECK(labels.numel() >= B, "labels");
  TORCH_CHECK(C % 8 == 0 && C <= 2048 && K <= 1024, "head: C must be a multiple of 8 (<= 2048), K <= 1024");
  const bool fuse = dW.has_value() && dW->defined();
  if (fuse) {
    CHECK_IN((*dW), torch::kFloat32);
    TORCH_CHECK(dW->numel() == K * C, "head dW size");
    if (db.has_value() && db->defined()) {
      CHECK_IN((*db), torch::kFloat32);
      TORCH_CHECK(db->numel() == K, "head db size");
    }
  }
  if (backward) {
    TORCH_CHECK(feat.has_value() && dlogits.has_value() && dx.has_value(), "bwd buffers");
    TORCH_CHECK(feat->numel() >= B * C && dlogits->numel() >= B * K, "bwd buffer sizes");
    CHECK_IN((*dx), torch::kBFloat16);
    TORCH_CHECK(dx->numel() == x.numel(), "dx size");
  }
  mfl::launch_head_fwd_bwd(bf(x), (int)B, (int)HW, (int)C, W.data_ptr<float>(),
                           ptr_or_null<float>(bias), (int)K, labels.data_ptr<int>(),
                           ptr_or_null<float>(feat), ptr_or_null<float>(dlogits),
                           dx.has_value() && dx->defined() ? bf(*dx) : nullptr,
                           ptr_or_null<float>(stats), backward, cur_stream(x),
                           fuse ? dW->data_ptr<float>() : nullptr, fuse ? ptr_or_null<float>(db) : nullptr);
}

void head_wgrad(torch::Tensor feat, torch::Tensor dlogits, int64_t B, int64_t C, int64_t K,
                torch::Tensor dW, c10::optional<torch::Tensor> db) {
  CHECK_IN(feat, torch::kFloat32);
  CHECK_IN(dlogits, torch::kFloat32);
  CHECK_IN(dW, torch::kFloat32);
  TORCH_CHECK(feat.numel() >= B * C && dlogits.numel() >= B * K && dW.numel() == K * C, "wgrad");
  mfl::launch_head_wgrad(feat.data_ptr<float>(), dlogits.data_ptr<float>(), (int)B, (int)C, (int)K,
                         dW.data_ptr<float>(), ptr_or_null<float>(db), cur_stream(feat));
}

void gather_batch(torch::Tensor shard, torch::Tensor labels, torch::Tensor perm,
                  torch::Tensor step, int64_t steps_per_epoch, int64_t B, torch::Tensor xb,
                  torch::Tensor yb) {
  CHECK_IN(shard, torch::kBFloat16);
  CHECK_IN(labels, torch::kInt32);
  CHECK_IN(perm, torch::kInt32);
  CHECK_IN(step, torch::kInt32);
  CHECK_IN(xb, torch::kBFloat16);
  CHECK_IN(yb, torch::kInt32);
  const int64_t n = labels.numel();
  TORCH_CHECK(n > 0 && shard.numel() % n == 0, "shard rows");
  const int64_t row = shard.numel() / n;
  TORCH_CHECK(row % 8 == 0, "row must be a multiple of 8 elements");
  TORCH_CHECK(xb.numel() == B * row && yb.numel() >= B, "batch buffers");
  TORCH_CHECK(perm.numel() >= steps_per_epoch * B, "permutation too short");
  TORCH_CHECK(perm.numel() <= n || true, "");
  mfl::launch_gather_batch(bf(shard), labels.data_ptr<int>(), perm.data_ptr<int>(),
                           step.data_ptr<int>(), (int)steps_per_epoch, (int)B, row, bf(xb),
                           yb.data_ptr<int>(), cur_stream(shard));
}

}  // namespace

void register_conv(pybind11::module& m);
void register_gemm(pybind11::module& m);
void register_layers(pybind11::module& m);
void register_bert(pybind11::module& m);
void register_ckks(pybind11::module& m);
void register_fp32(pybind11::module& m);
void register_hconv(pybind11::module& m);

PYBIND11_MODULE(_ops, m) {
  m.doc() = "metisfl_amd hand-written HIP (gfx950) kernels";
  m.def("fused_optimizer", &fused_optimizer);
  m.def("split_pack_f32", &split_pack_f32);
  m.def("bn_apply_pair", &bn_apply_pair);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("scale_f32", &scale_f32);
  m.def("tick", &tick);
  m.def("weighted_sum", &weighted_sum);
  m.def("rolling_op", &rolling_op);
  m.def("count_zeros", &count_zeros);
  m.def("ckks_pwa", &ckks_pwa);
  m.def("bn_stats", &bn_stats);
  m.def("bn_apply", &bn_apply);
  m.def("bn_backward", &bn_backward);
  m.def("head_forward_backward", &head_forward_backward, pybind11::arg("x"), pybind11::arg("B"),
        pybind11::arg("HW"), pybind11::arg("C"), pybind11::arg("W"), pybind11::arg("bias"),
        pybind11::arg("labels"), pybind11::arg("feat"), pybind11::arg("dlogits"), pybind11::arg("dx"),
        pybind11::arg("stats"), pybind11::arg("backward"), pybind11::arg("dW") = pybind11::none(),
        pybind11::arg("db") = pybind11::none());
  m.def("head_wgrad", &head_wgrad);
  m.def("gather_batch", &gather_batch);
  register_conv(m);
  register_gemm(m);
  register_layers(m);
  register_bert(m);
  register_ckks(m);
  register_fp32(m);
  register_hconv(m);
}
