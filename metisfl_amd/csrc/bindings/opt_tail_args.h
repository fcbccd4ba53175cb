// Torch-facing construction of an optimizer tail (kernels/opt_tail.h) from
// the trailing arguments of the paired backward bindings (fp32 and bf16).
#pragma once
#include <torch/extension.h>

#include <algorithm>
#include <vector>

#include "kernels/launchers.h"
#include "kernels/opt_tail.h"

// -> whether a tail was given; mirror: int32 = packed bf16x3 split, bf16 =
// the bf16 compute copy
static inline bool opt_tail_args(mfl::OptTail& ot, const c10::optional<torch::Tensor>& opt_p,
                                 const c10::optional<torch::Tensor>& opt_g, const c10::optional<torch::Tensor>& opt_m,
                                 const c10::optional<torch::Tensor>& opt_v,
                                 const c10::optional<torch::Tensor>& opt_anchor,
                                 const c10::optional<torch::Tensor>& opt_mirror,
                                 const c10::optional<torch::Tensor>& opt_lr_scale,
                                 const c10::optional<torch::Tensor>& opt_step, int64_t opt_mode,
                                 const std::vector<double>& opt_hyper, bool opt_zero_grad) {
  if (!(opt_p.has_value() && opt_p->defined())) return false;
  const int64_t n = opt_p->numel();
  TORCH_CHECK(opt_p->is_cuda() && opt_p->is_contiguous() && opt_p->scalar_type() == torch::kFloat32, "opt p");
  TORCH_CHECK(n % 4 == 0 && (reinterpret_cast<uintptr_t>(opt_p->data_ptr()) & 15) == 0, "opt range: 16-B float4s");
  TORCH_CHECK(opt_hyper.size() == 9, "opt hyper: lr l1 l2 momentum mu beta1 beta2 eps wd");
  auto same = [&](const c10::optional<torch::Tensor>& t, const char* nm) -> void* {
    if (!(t.has_value() && t->defined())) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->numel() == n, "opt ", nm, " range");
    return t->data_ptr();
  };
  ot.p = opt_p->data_ptr<float>();
  ot.g = static_cast<float*>(same(opt_g, "g"));
  TORCH_CHECK(ot.g != nullptr, "opt tail needs the gradient range");
  ot.m = static_cast<float*>(same(opt_m, "m"));
  ot.v = static_cast<float*>(same(opt_v, "v"));
  ot.anchor = static_cast<const float*>(same(opt_anchor, "anchor"));
  ot.mirror = same(opt_mirror, "mirror");
  ot.mirror_kind = 0;
  if (ot.mirror) {
    const auto dt = opt_mirror->scalar_type();
    TORCH_CHECK(dt == torch::kInt32 || dt == torch::kBFloat16, "opt tail mirror: packed split or bf16 copy");
    ot.mirror_kind = dt == torch::kInt32 ? 2 : 1;
  }
  ot.mode = (int)opt_mode;
  TORCH_CHECK(ot.mode != mfl::OPT_MOMENTUM || ot.m, "momentum buffer");
  TORCH_CHECK(ot.mode != mfl::OPT_FEDPROX || ot.anchor, "proximal anchor");
  TORCH_CHECK((ot.mode != mfl::OPT_ADAM && ot.mode != mfl::OPT_ADAMW) || (ot.m && ot.v), "adam slots");
  ot.h.lr = (float)opt_hyper[0]; ot.h.l1 = (float)opt_hyper[1]; ot.h.l2 = (float)opt_hyper[2];
  ot.h.momentum = (float)opt_hyper[3]; ot.h.mu = (float)opt_hyper[4]; ot.h.beta1 = (float)opt_hyper[5];
  ot.h.beta2 = (float)opt_hyper[6]; ot.h.eps = (float)opt_hyper[7]; ot.h.wd = (float)opt_hyper[8];
  ot.lr_ptr = opt_lr_scale.has_value() && opt_lr_scale->defined() ? opt_lr_scale->data_ptr<float>() : nullptr;
  ot.step_ptr = opt_step.has_value() && opt_step->defined() ? opt_step->data_ptr<int>() : nullptr;
  ot.zero_grad = opt_zero_grad ? 1 : 0;
  ot.n4 = n / 4;
  // ~4 float4 per thread: enough workgroups to stream at full rate, few
  // enough to land in the GEMMs' tail
  ot.nblk = (int)std::max<int64_t>(16, std::min<int64_t>(256, ot.n4 / (256 * 4)));
  return true;
}

// the pair did not launch: the range's optimizer as its own launch
static inline void opt_tail_fallback(const mfl::OptTail& ot, hipStream_t s) {
  mfl::launch_fused_optimizer(ot.mode, ot.p, ot.g, ot.m, ot.v, ot.anchor, ot.mirror, ot.n4 * 4, ot.h, ot.lr_ptr,
                              ot.step_ptr, ot.zero_grad != 0, nullptr, 0, s, nullptr, ot.mirror_kind);
}
