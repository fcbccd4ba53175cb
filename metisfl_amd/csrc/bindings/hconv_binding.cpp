// torch binding of the halo-tiled fp32 (bf16x3-product) convolutions with the
// producer's BatchNorm fused into the operand fill (kernels/hconv.hip).
// Shapes / dtypes / sizes are validated here, before any launch: the kernels
// trust their geometry and index with 32-bit byte offsets.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/hconv.h"

namespace {

using OptT = c10::optional<torch::Tensor>;

hipStream_t cur_stream(const torch::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check(const torch::Tensor& t, c10::ScalarType st, int64_t numel, const char* nm) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), nm, " must be a contiguous device tensor");
  TORCH_CHECK(t.scalar_type() == st, nm, " has the wrong dtype");
  TORCH_CHECK(numel < 0 || t.numel() == numel, nm, " has ", t.numel(), " elements, expected ", numel);
}
bool has(const OptT& t) { return t.has_value() && t->defined(); }

// BatchNorm source from (acc fp64 [reps][2][C], gamma, beta, mean, invstd, run_mean, run_var)
mfl::hc::BnSrc bn_src(const OptT& acc, const torch::Tensor& gamma, const torch::Tensor& beta,
                      const torch::Tensor& mean, const torch::Tensor& invstd, const torch::Tensor& rm,
                      const torch::Tensor& rv, int64_t C, bool train, double momentum, double eps) {
  for (auto* p : {&gamma, &beta, &mean, &invstd, &rm, &rv}) check(*p, torch::kFloat32, C, "bn parameter");
  mfl::hc::BnSrc b;
  if (train) {
    TORCH_CHECK(has(acc), "train-mode BN needs the statistics accumulator");
    check(*acc, torch::kFloat64, -1, "bn acc");
    TORCH_CHECK(acc->numel() % (2 * C) == 0, "bn acc holds [reps][2][C]");
    b.acc = acc->data_ptr<double>();
    b.reps = (int)(acc->numel() / (2 * C));
    TORCH_CHECK(b.reps >= 1 && b.reps <= 8, "1..8 BN accumulator replicas");
  }
  b.gamma = gamma.data_ptr<float>();
  b.beta = beta.data_ptr<float>();
  b.mean = mean.data_ptr<float>();
  b.invstd = invstd.data_ptr<float>();
  b.run_mean = rm.data_ptr<float>();
  b.run_var = rv.data_ptr<float>();
  b.momentum = (float)momentum;
  b.eps = (float)eps;
  return b;
}

int64_t hconv_fwd_workspace(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co) {
  return mfl::hc::hconv_fwd_workspace((int)N, (int)H, (int)W, (int)C, (int)Co);
}

// out = conv3x3(T(z), W) with T(z) = relu?(BN(z) [+ res | + BN_r(zr)]); y / yp
// (optional) receive T(z) and its packed split; stats (optional, train) the
// output's BN sums.  bn: (acc, gamma, beta, mean, invstd, run_mean, run_var)
// of z's BatchNorm; bnr: the same for zr's (projection-shortcut residual).
void hconv_forward(torch::Tensor z, torch::Tensor wp, torch::Tensor out, OptT ws, OptT stats, int64_t N, int64_t H,
                   int64_t W, int64_t C, int64_t Co, bool train, bool relu, OptT acc, torch::Tensor gamma,
                   torch::Tensor beta, torch::Tensor mean, torch::Tensor invstd, torch::Tensor run_mean,
                   torch::Tensor run_var, double momentum, double eps, OptT res, OptT zr, OptT acc2, OptT gamma2,
                   OptT beta2, OptT mean2, OptT invstd2, OptT run_mean2, OptT run_var2, OptT y, OptT yp,
                   OptT stamps) {
  const int64_t ws_need = mfl::hc::hconv_fwd_workspace((int)N, (int)H, (int)W, (int)C, (int)Co);
  TORCH_CHECK(ws_need >= 0, "halo conv: unsupported geometry N=", N, " H=", H, " W=", W, " C=", C, " Co=", Co);
  const int64_t nin = N * H * W * C, nout = N * H * W * Co;
  TORCH_CHECK(nin * 4 < (1LL << 31) && nout * 4 < (1LL << 31), "activation too large for 32-bit byte offsets");
  // fp32 activations with the packed bf16x3 weight mirror, or the bf16
  // option: bf16 activations, residual, output and weights
  const bool bf = z.scalar_type() == torch::kBFloat16;
  const auto act = bf ? torch::kBFloat16 : torch::kFloat32;
  check(z, act, nin, "z");
  check(wp, bf ? torch::kBFloat16 : torch::kInt32, Co * 9 * C, "weights");
  check(out, act, nout, "out");
  mfl::hc::FwdArgs a{};
  a.bf16 = bf ? 1 : 0;
  a.N = (int)N; a.H = (int)H; a.W = (int)W; a.C = (int)C; a.Co = (int)Co;
  a.x.z = reinterpret_cast<const float*>(z.data_ptr());
  a.x.has_bn = 1;
  a.x.bn = bn_src(acc, gamma, beta, mean, invstd, run_mean, run_var, C, train, momentum, eps);
  if (has(res)) {
    check(*res, act, nin, "res");
    a.x.res = reinterpret_cast<const float*>(res->data_ptr());
  }
  if (has(zr)) {
    TORCH_CHECK(!has(res), "one residual: res or zr");
    check(*zr, act, nin, "zr");
    TORCH_CHECK(has(gamma2) && has(beta2) && has(mean2) && has(invstd2) && has(run_mean2) && has(run_var2),
                "zr needs its BN parameters");
    a.x.zr = reinterpret_cast<const float*>(zr->data_ptr());
    a.x.bnr = bn_src(acc2, *gamma2, *beta2, *mean2, *invstd2, *run_mean2, *run_var2, C, train, momentum, eps);
  }
  a.x.relu = relu ? 1 : 0;
  a.x.train = train ? 1 : 0;
  a.x.M = (int)(N * H * W);
  if (has(y)) {
    check(*y, act, nin, "y");
    a.x.y = reinterpret_cast<float*>(y->data_ptr());
  }
  if (has(yp)) {
    TORCH_CHECK(!bf, "the bf16 option has no packed mirror");
    TORCH_CHECK(has(y), "yp is written with y");
    check(*yp, torch::kInt32, nin, "yp");
    a.x.yp = reinterpret_cast<uint32_t*>(yp->data_ptr());
  }
  a.wp = reinterpret_cast<const uint32_t*>(wp.data_ptr());
  a.out = reinterpret_cast<float*>(out.data_ptr());
  a.reps = 1;
  if (has(stats)) {
    TORCH_CHECK(train, "output statistics are a train-mode product");
    check(*stats, torch::kFloat64, -1, "stats");
    TORCH_CHECK(stats->numel() % (2 * Co) == 0, "stats hold [reps][2][Co]");
    a.stats = stats->data_ptr<double>();
    a.reps = (int)(stats->numel() / (2 * Co));
  }
  if (ws_need > 0) {
    TORCH_CHECK(has(ws), "split-K workspace required");
    check(*ws, torch::kFloat32, -1, "workspace");
    TORCH_CHECK(ws->numel() >= ws_need, "workspace too small: ", ws->numel(), " < ", ws_need);
    a.counters = reinterpret_cast<int*>(ws->data_ptr<float>());
    a.slab = ws->data_ptr<float>() + 1024;
  }
  if (has(stamps)) {  // profiling: [grid][16] int64 phase stamps
    check(*stamps, torch::kInt64, -1, "stamps");
    TORCH_CHECK(stamps->numel() >= 16 * 2048, "stamps: at least 16 x 2048 slots");
    a.stamps = reinterpret_cast<long long*>(stamps->data_ptr<int64_t>());
  }
  if (const char* e = getenv("MFL_HC_DBG")) a.dbg = atoi(e);  // timing ablations only
  if (const char* e = getenv("MFL_HC_XCD")) a.xcd = atoi(e);
  mfl::hc::launch_hconv_fwd(a, cur_stream(out));
}

// dx (+)= conv3x3^T(dz, W), dz = BN_bwd(dy [* (ymask > 0)]) applied in the
// operand fill from (acc: complete sums of g and g * xhat [reps][2][C],
// gamma, mean, invstd); dgamma / dbeta published.  Owner tiles write dz's
// packed split (dzp, the wgrad operand) and g (dres).  bnb_*: the consumer
// BN-backward reductions of dx in the epilogue.
void hconv_dgrad(torch::Tensor dy, OptT ymask, torch::Tensor z, torch::Tensor wp, torch::Tensor out, OptT ws,
                 int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co, torch::Tensor acc, torch::Tensor gamma,
                 torch::Tensor mean, torch::Tensor invstd, OptT dgamma, OptT dbeta, OptT dres, OptT dzp,
                 bool accumulate, OptT bnb_z, OptT bnb_y, OptT bnb_mean, OptT bnb_invstd, OptT bnb_acc,
                 OptT stamps) {
  const int64_t ws_need = mfl::hc::hconv_fwd_workspace((int)N, (int)H, (int)W, (int)C, (int)Co);
  TORCH_CHECK(ws_need >= 0, "halo dgrad: unsupported geometry N=", N, " H=", H, " W=", W, " C=", C, " Co=", Co);
  const int64_t nin = N * H * W * C, nout = N * H * W * Co;
  TORCH_CHECK(nin * 4 < (1LL << 31) && nout * 4 < (1LL << 31), "activation too large for 32-bit byte offsets");
  check(dy, torch::kFloat32, nin, "dy");
  check(z, torch::kFloat32, nin, "z");
  check(wp, torch::kInt32, C * 9 * Co, "packed weights");
  check(out, torch::kFloat32, nout, "out");
  mfl::hc::DgArgs a{};
  a.N = (int)N; a.H = (int)H; a.W = (int)W; a.C = (int)C; a.Co = (int)Co;
  a.x.dy = dy.data_ptr<float>();
  a.x.z = z.data_ptr<float>();
  if (has(ymask)) {
    check(*ymask, torch::kFloat32, nin, "ymask");
    a.x.ymask = ymask->data_ptr<float>();
  }
  check(acc, torch::kFloat64, -1, "bn acc");
  TORCH_CHECK(acc.numel() % (2 * C) == 0, "bn acc holds [reps][2][C]");
  a.x.bn.acc = acc.data_ptr<double>();
  a.x.bn.reps = (int)(acc.numel() / (2 * C));
  TORCH_CHECK(a.x.bn.reps >= 1 && a.x.bn.reps <= 8, "1..8 BN accumulator replicas");
  for (auto* p : {&gamma, &mean, &invstd}) check(*p, torch::kFloat32, C, "bn parameter");
  a.x.bn.gamma = gamma.data_ptr<float>();
  a.x.bn.mean = mean.data_ptr<float>();
  a.x.bn.invstd = invstd.data_ptr<float>();
  if (has(dgamma)) { check(*dgamma, torch::kFloat32, C, "dgamma"); a.x.bn.dgamma = dgamma->data_ptr<float>(); }
  if (has(dbeta)) { check(*dbeta, torch::kFloat32, C, "dbeta"); a.x.bn.dbeta = dbeta->data_ptr<float>(); }
  a.x.M = (int)(N * H * W);
  if (has(dres)) {
    check(*dres, torch::kFloat32, nin, "dres");
    a.x.dres = dres->data_ptr<float>();
  }
  if (has(dzp)) {
    check(*dzp, torch::kInt32, nin, "dzp");
    a.x.dzp = reinterpret_cast<uint32_t*>(dzp->data_ptr());
  }
  a.wp = reinterpret_cast<const uint32_t*>(wp.data_ptr());
  a.out = out.data_ptr<float>();
  a.accumulate = accumulate ? 1 : 0;
  if (has(bnb_acc)) {
    TORCH_CHECK(has(bnb_z) && has(bnb_mean) && has(bnb_invstd), "consumer BN reductions need z, mean, invstd");
    check(*bnb_z, torch::kFloat32, nout, "bnb z");
    if (has(bnb_y)) {
      check(*bnb_y, torch::kFloat32, nout, "bnb y");
      a.bnb.y = bnb_y->data_ptr<float>();
    }
    check(*bnb_mean, torch::kFloat32, Co, "bnb mean");
    check(*bnb_invstd, torch::kFloat32, Co, "bnb invstd");
    check(*bnb_acc, torch::kFloat64, -1, "bnb acc");
    TORCH_CHECK(bnb_acc->numel() % (2 * Co) == 0, "bnb acc holds [reps][2][Co]");
    a.bnb.z = bnb_z->data_ptr<float>();
    a.bnb.mean = bnb_mean->data_ptr<float>();
    a.bnb.invstd = bnb_invstd->data_ptr<float>();
    a.bnb.acc = bnb_acc->data_ptr<double>();
    a.bnb.reps = (int)(bnb_acc->numel() / (2 * Co));
  }
  if (ws_need > 0) {
    TORCH_CHECK(has(ws), "split-K workspace required");
    check(*ws, torch::kFloat32, -1, "workspace");
    TORCH_CHECK(ws->numel() >= ws_need, "workspace too small: ", ws->numel(), " < ", ws_need);
    a.counters = reinterpret_cast<int*>(ws->data_ptr<float>());
    a.slab = ws->data_ptr<float>() + 1024;
  }
  if (has(stamps)) {
    check(*stamps, torch::kInt64, -1, "stamps");
    TORCH_CHECK(stamps->numel() >= 16 * 2048, "stamps: at least 16 x 2048 slots");
    a.stamps = reinterpret_cast<long long*>(stamps->data_ptr<int64_t>());
  }
  if (const char* e = getenv("MFL_HC_DBG")) a.dbg = atoi(e);
  if (const char* e = getenv("MFL_HC_XCD")) a.xcd = atoi(e);
  mfl::hc::launch_hconv_dgrad(a, cur_stream(out));
}

}  // namespace

void register_hconv(pybind11::module& m) {
  m.def("hconv_fwd_workspace", &hconv_fwd_workspace);
  m.def("hconv_forward", &hconv_forward);
  m.def("hconv_dgrad", &hconv_dgrad);
}
