// torch binding for the throughput-regime backward convolutions (tconv.hip):
// a 3x3 / stride-1 layer's weight gradient and input gradient (with the
// consumer-BN fusion of the fp32 dgrad epilogue) from the packed bf16x3
// operands the fp32 path already writes.  Used by the co-located learners
// (models/colocated.py -> ops/nn.py set_throughput_conv); shapes / dtypes are
// validated here before any launch, and every launch goes to the caller's
// current HIP stream.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/tconv.h"

namespace {

hipStream_t cur_stream(const torch::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check(const torch::Tensor& t, int64_t numel, c10::ScalarType ty, const char* nm, bool exact = true) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), nm, " must be a contiguous device tensor");
  TORCH_CHECK(t.scalar_type() == ty, nm, " has dtype ", t.scalar_type(), ", expected ", ty);
  if (exact) {
    TORCH_CHECK(t.numel() == numel, nm, " has ", t.numel(), " elements, expected ", numel);
  } else {
    TORCH_CHECK(t.numel() >= numel, nm, " too small: ", t.numel(), " < ", numel);
  }
}
// packed operands arrive as int32 tensors, or as the fp32 buffer the BN
// backward wrote them into (same 4 bytes per element)
const uint32_t* packed(const torch::Tensor& t, int64_t numel, const char* nm) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.numel() == numel, nm,
              " must be a contiguous device tensor of ", numel, " packed elements");
  TORCH_CHECK(t.scalar_type() == torch::kInt32 || t.scalar_type() == torch::kFloat32, nm, " must be int32 / fp32");
  return reinterpret_cast<const uint32_t*>(t.data_ptr());
}

mfl::tc::Geom geom(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co, int64_t R, int64_t S, int64_t stride,
                   int64_t pad) {
  mfl::tc::Geom g{};
  g.N = (int)N;
  g.H = (int)H;
  g.W = (int)W;
  g.C = (int)C;
  g.Co = (int)Co;
  g.KS = (int)R;
  g.ST = (int)stride;
  g.pad = (int)pad;
  g.P = (int)((H + 2 * pad - R) / stride + 1);
  g.Q = (int)((W + 2 * pad - S) / stride + 1);
  TORCH_CHECK(R == S, "square filters only");
  TORCH_CHECK((int64_t)N * H * W * std::max(C, Co) * 4 < (1LL << 31), "activation too large for 32-bit offsets");
  return g;
}

bool tconv_backward_ok(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co, int64_t R, int64_t S, int64_t stride,
                       int64_t pad) {
  if (R != S) return false;
  const auto g = geom(N, H, W, C, Co, R, S, stride, pad);
  return mfl::tc::wgrad_ok(g) && mfl::tc::dgrad_ok(g);
}

// (workspace floats, counter ints) of the planned dgrad
std::tuple<int64_t, int64_t> tconv_workspace(int64_t N, int64_t H, int64_t W, int64_t C, int64_t Co, int64_t R,
                                             int64_t S, int64_t stride, int64_t pad) {
  const auto g = geom(N, H, W, C, Co, R, S, stride, pad);
  const int sp = mfl::tc::dgrad_default_splits(g);
  return {mfl::tc::dgrad_workspace(g, sp), sp > 1 ? mfl::tc::dgrad_counters(g) : 0};
}

void tconv_backward(torch::Tensor xp, torch::Tensor dyp, torch::Tensor dw, torch::Tensor wp, torch::Tensor dx,
                    c10::optional<torch::Tensor> ws, c10::optional<torch::Tensor> counters, int64_t N, int64_t H,
                    int64_t W, int64_t C, int64_t Co, int64_t R, int64_t S, int64_t stride, int64_t pad,
                    bool accumulate, c10::optional<torch::Tensor> bn_z, c10::optional<torch::Tensor> bn_y,
                    c10::optional<torch::Tensor> bn_mean, c10::optional<torch::Tensor> bn_invstd,
                    c10::optional<torch::Tensor> bn_acc) {
  const auto g = geom(N, H, W, C, Co, R, S, stride, pad);
  TORCH_CHECK(mfl::tc::wgrad_ok(g) && mfl::tc::dgrad_ok(g), "tconv: unsupported layer shape");
  const int64_t nx = (int64_t)N * H * W * C, ny = (int64_t)N * g.P * g.Q * Co, nw = (int64_t)Co * R * S * C;
  const uint32_t* x = packed(xp, nx, "xp");
  const uint32_t* dy = packed(dyp, ny, "dyp");
  const uint32_t* w = packed(wp, nw, "wp");
  check(dw, nw, torch::kFloat32, "dw");
  check(dx, nx, torch::kFloat32, "dx");
  mfl::tc::Bnb f;
  const bool fuse = bn_acc.has_value() && bn_acc->defined();
  if (fuse) {
    TORCH_CHECK(bn_z.has_value() && bn_mean.has_value() && bn_invstd.has_value(), "bn fusion operands");
    check(*bn_z, nx, torch::kFloat32, "bn_z");
    if (bn_y.has_value() && bn_y->defined()) {
      check(*bn_y, nx, torch::kFloat32, "bn_y");
      f.y = bn_y->data_ptr<float>();
    }
    check(*bn_mean, C, torch::kFloat32, "bn_mean");
    check(*bn_invstd, C, torch::kFloat32, "bn_invstd");
    check(*bn_acc, 2 * C, torch::kFloat64, "bn_acc", false);
    f.z = bn_z->data_ptr<float>();
    f.mean = bn_mean->data_ptr<float>();
    f.invstd = bn_invstd->data_ptr<float>();
    f.acc = bn_acc->data_ptr<double>();
    f.reps = (int)std::max<int64_t>(1, bn_acc->numel() / (2 * C));
  }
  const int sp = mfl::tc::dgrad_default_splits(g);
  float* slab = nullptr;
  int* cnt = nullptr;
  if (sp > 1) {
    TORCH_CHECK(ws.has_value() && ws->defined() && counters.has_value() && counters->defined(),
                "tconv: split-K workspace and counters required");
    check(*ws, mfl::tc::dgrad_workspace(g, sp), torch::kFloat32, "ws", false);
    check(*counters, mfl::tc::dgrad_counters(g), torch::kInt32, "counters", false);
    slab = ws->data_ptr<float>();
    cnt = counters->data_ptr<int>();
  }
  const hipStream_t s = cur_stream(dx);
  mfl::tc::launch_wgrad(g, x, dy, dw.data_ptr<float>(), 0, s);
  mfl::tc::launch_dgrad(g, dy, w, dx.data_ptr<float>(), accumulate, fuse ? &f : nullptr, slab, cnt, sp, s);
}

}  // namespace

void register_tconv(pybind11::module& m) {
  m.def("tconv_backward_ok", &tconv_backward_ok);
  m.def("tconv_workspace", &tconv_workspace);
  m.def("tconv_backward", &tconv_backward);
}
