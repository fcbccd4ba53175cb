// torch binding for the example-model layer kernels (layers.hip).  Shapes are
// validated here before any launch.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/launchers.h"

namespace {

hipStream_t stream_of(const torch::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}
uint16_t* bfp(const torch::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

void need(const torch::Tensor& t, torch::ScalarType dt, const char* nm) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), nm, " must be a contiguous device tensor");
  TORCH_CHECK(t.scalar_type() == dt, nm, " has the wrong dtype");
}

void bias_act(torch::Tensor y, torch::Tensor bias, int64_t N, int64_t act) {
  need(y, torch::kBFloat16, "y");
  need(bias, torch::kFloat32, "bias");
  TORCH_CHECK(N % 8 == 0 && y.numel() % N == 0 && bias.numel() >= N, "bias_act shapes");
  mfl::launch_bias_act_fwd(bfp(y), bias.data_ptr<float>(), y.numel() / N, (int)N, (int)act, stream_of(y));
}

void bias_act_backward(torch::Tensor dy, torch::Tensor y, torch::Tensor dz, torch::Tensor dbias, int64_t N,
                       int64_t act) {
  need(dy, torch::kBFloat16, "dy");
  need(y, torch::kBFloat16, "y");
  need(dz, torch::kBFloat16, "dz");
  need(dbias, torch::kFloat32, "dbias");
  TORCH_CHECK(N % 8 == 0 && N <= 2048 && dy.numel() % N == 0 && dy.numel() == y.numel() &&
                  dz.numel() == dy.numel() && dbias.numel() >= N,
              "bias_act_backward shapes (N <= 2048, multiple of 8)");
  mfl::launch_bias_act_bwd(bfp(dy), bfp(y), bfp(dz), dbias.data_ptr<float>(), dy.numel() / N, (int)N,
                           (int)act, stream_of(dy));
}

void maxpool2(torch::Tensor x, torch::Tensor y, int64_t N, int64_t H, int64_t W, int64_t C) {
  need(x, torch::kBFloat16, "x");
  need(y, torch::kBFloat16, "y");
  TORCH_CHECK(C % 8 == 0 && H % 2 == 0 && W % 2 == 0 && x.numel() == N * H * W * C &&
                  y.numel() == N * (H / 2) * (W / 2) * C,
              "maxpool2 shapes");
  mfl::launch_maxpool2(bfp(x), bfp(y), (int)N, (int)H, (int)W, (int)C, stream_of(x));
}

void maxpool2_backward(torch::Tensor dy, torch::Tensor x, torch::Tensor y, torch::Tensor dx, int64_t N,
                       int64_t H, int64_t W, int64_t C) {
  for (auto* t : {&dy, &x, &y, &dx}) need(*t, torch::kBFloat16, "maxpool tensor");
  TORCH_CHECK(C % 8 == 0 && H % 2 == 0 && W % 2 == 0 && x.numel() == N * H * W * C &&
                  dx.numel() == x.numel() && y.numel() == N * (H / 2) * (W / 2) * C && dy.numel() == y.numel(),
              "maxpool2_backward shapes");
  mfl::launch_maxpool2_bwd(bfp(dy), bfp(x), bfp(y), bfp(dx), (int)N, (int)H, (int)W, (int)C, stream_of(x));
}

void dropout(torch::Tensor in, torch::Tensor out, double p, int64_t seed, c10::optional<torch::Tensor> step) {
  need(in, torch::kBFloat16, "in");
  need(out, torch::kBFloat16, "out");
  TORCH_CHECK(in.numel() == out.numel() && in.numel() % 8 == 0, "dropout shapes");
  const int* sp = nullptr;
  if (step.has_value() && step->defined()) {
    need(*step, torch::kInt32, "step");
    sp = step->data_ptr<int>();
  }
  mfl::launch_dropout(bfp(in), bfp(out), in.numel(), (float)p, (uint32_t)seed, sp, stream_of(in));
}

void xent(torch::Tensor logits, torch::Tensor labels, int64_t B, int64_t Kp, int64_t K,
          c10::optional<torch::Tensor> dlogits, torch::Tensor stats) {
  need(logits, torch::kBFloat16, "logits");
  need(labels, torch::kInt32, "labels");
  need(stats, torch::kFloat32, "stats");
  TORCH_CHECK(logits.numel() == B * Kp && labels.numel() >= B && K <= Kp && stats.numel() >= 3, "xent shapes");
  uint16_t* dl = nullptr;
  if (dlogits.has_value() && dlogits->defined()) {
    need(*dlogits, torch::kBFloat16, "dlogits");
    TORCH_CHECK(dlogits->numel() == B * Kp, "dlogits shape");
    dl = bfp(*dlogits);
  }
  mfl::launch_xent(bfp(logits), labels.data_ptr<int>(), (int)B, (int)Kp, (int)K, dl, stats.data_ptr<float>(),
                   dl != nullptr, stream_of(logits));
}

void mse(torch::Tensor pred, torch::Tensor target, int64_t B, int64_t Kp, c10::optional<torch::Tensor> dpred,
         torch::Tensor stats) {
  need(pred, torch::kBFloat16, "pred");
  TORCH_CHECK(target.is_cuda() && target.is_contiguous() && target.element_size() == 4 && target.numel() >= B,
              "target must hold B 4-byte values (fp32 targets, possibly viewed as int32)");
  need(stats, torch::kFloat32, "stats");
  TORCH_CHECK(pred.numel() == B * Kp, "pred shape");
  uint16_t* dp = nullptr;
  if (dpred.has_value() && dpred->defined()) {
    need(*dpred, torch::kBFloat16, "dpred");
    dp = bfp(*dpred);
  }
  mfl::launch_mse(bfp(pred), reinterpret_cast<const float*>(target.data_ptr()), (int)B, (int)Kp, dp,
                  stats.data_ptr<float>(), dp != nullptr, stream_of(pred));
}

}  // namespace

void register_layers(pybind11::module& m) {
  m.def("bias_act", &bias_act);
  m.def("bias_act_backward", &bias_act_backward);
  m.def("maxpool2", &maxpool2);
  m.def("maxpool2_backward", &maxpool2_backward);
  m.def("dropout", &dropout);
  m.def("xent", &xent);
  m.def("mse", &mse);
}
