// K3/K4/K5 element math shared by the fused optimizer launch (optim.hip) and
// the optimizer-tail role of the fp32 paired backward launch (conv32.hip
// conv32_bwd_pair_kernel): one float4 of the flat master / gradient / slots.
#pragma once
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace mfl {

// One float4 of every operand an update reads (opt_load4), so a loop can
// have the next element's loads in flight while it updates and stores this
// one (opt_apply4).
struct OptIn4 {
  float4 p, g, m, v, a;
};

template <int MODE>
__device__ __forceinline__ OptIn4 opt_load4(const float* __restrict__ p, const float* __restrict__ g,
                                            const float* __restrict__ m, const float* __restrict__ v,
                                            const float* __restrict__ anchor, int64_t i) {
  OptIn4 r;
  r.p = reinterpret_cast<const float4*>(p)[i];
  r.g = reinterpret_cast<const float4*>(g)[i];
  if (MODE == OPT_MOMENTUM || MODE == OPT_ADAM || MODE == OPT_ADAMW) r.m = reinterpret_cast<const float4*>(m)[i];
  if (MODE == OPT_ADAM || MODE == OPT_ADAMW) r.v = reinterpret_cast<const float4*>(v)[i];
  if (MODE == OPT_FEDPROX) r.a = reinterpret_cast<const float4*>(anchor)[i];
  return r;
}

// MIRROR: 0 none, 1 bf16 compute copy, 2 packed bf16x3 split (split_pack)
template <int MODE, int MIRROR>
__device__ __forceinline__ void opt_apply4(OptIn4 in, float* __restrict__ p, float* __restrict__ g,
                                           float* __restrict__ m, float* __restrict__ v,
                                           void* __restrict__ mirror, int64_t i, const OptHyper& h, float lr,
                                           float bc1, float bc2, bool zero_grad) {
  float4 pv = in.p;
  const float4 gv = in.g;
  if (zero_grad) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  float* pp = &pv.x;
  const float* gg = &gv.x;
  if (MODE == OPT_SGD) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gr = gg[k] + h.l2 * pp[k];
      if (h.l1 != 0.f) gr += h.l1 * ((pp[k] > 0.f) - (pp[k] < 0.f));
      pp[k] -= lr * gr;
    }
  } else if (MODE == OPT_MOMENTUM) {
    // Keras SGD(momentum) form: v = mu*v - lr*g ; p += v
    float4 mv = in.m;
    float* mm = &mv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mm[k] = h.momentum * mm[k] - lr * gg[k];
      pp[k] += mm[k];
    }
    reinterpret_cast<float4*>(m)[i] = mv;
  } else if (MODE == OPT_FEDPROX) {
    const float4 av = in.a;
    const float* aa = &av.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) pp[k] -= lr * (gg[k] + h.mu * (pp[k] - aa[k]));
  } else {  // Adam / AdamW
    float4 mv = in.m;
    float4 vv = in.v;
    float* mm = &mv.x;
    float* vq = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mm[k] = h.beta1 * mm[k] + (1.f - h.beta1) * gg[k];
      vq[k] = h.beta2 * vq[k] + (1.f - h.beta2) * gg[k] * gg[k];
      const float mh = mm[k] / bc1;
      const float vh = vq[k] / bc2;
      float upd = mh / (sqrtf(vh) + h.eps);
      if (MODE == OPT_ADAMW) upd += h.wd * pp[k];
      pp[k] -= lr * upd;
    }
    reinterpret_cast<float4*>(m)[i] = mv;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  reinterpret_cast<float4*>(p)[i] = pv;
  if (MIRROR == 1) {
    uint2 o;
    o.x = pack2bf(pp[0], pp[1]);
    o.y = pack2bf(pp[2], pp[3]);
    reinterpret_cast<uint2*>(mirror)[i] = o;
  } else if (MIRROR == 2) {
    reinterpret_cast<uint4*>(mirror)[i] =
        make_uint4(split_pack(pp[0]), split_pack(pp[1]), split_pack(pp[2]), split_pack(pp[3]));
  }
}

template <int MODE, int MIRROR>
__device__ __forceinline__ void opt_update4(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                            float* __restrict__ v, const float* __restrict__ anchor,
                                            void* __restrict__ mirror, int64_t i, const OptHyper& h, float lr,
                                            float bc1, float bc2, bool zero_grad) {
  opt_apply4<MODE, MIRROR>(opt_load4<MODE>(p, g, m, v, anchor, i), p, g, m, v, mirror, i, h, lr, bc1, bc2,
                           zero_grad);
}

// Adam bias corrections 1 - beta^t for step t = step_ptr[0] + 1
__device__ __forceinline__ void opt_bias_corr(int mode, const OptHyper& h, const int* step_ptr, float& bc1,
                                              float& bc2) {
  bc1 = bc2 = 1.f;
  if (mode == OPT_ADAM || mode == OPT_ADAMW) {
    const float t = (float)(step_ptr ? step_ptr[0] + 1 : 1);
    bc1 = 1.f - powf(h.beta1, t);
    bc2 = 1.f - powf(h.beta2, t);
  }
}

}  // namespace mfl
