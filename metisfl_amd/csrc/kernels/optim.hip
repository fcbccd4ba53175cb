// K3/K4/K5: fused multi-tensor optimizers over a flat fp32 master buffer.
//
// Replaces the per-variable optimizer application the reference delegates to
// Keras (metisfl/models/keras/keras_model_ops.py:245-283) and the FedProx
// optimizer (metisfl/models/keras/optimizers/fed_prox.py:50-60).  Every
// trainable variable of a learner lives in ONE flat fp32 buffer, so a whole
// optimizer step is a single streaming launch that also refreshes the bf16
// compute copy of the weights (no separate cast pass).  The learning rate and
// the step counter are read from device memory so the launch can sit inside a
// captured hipGraph and still follow a schedule.
//
// FedProx deviation (documented): the proximal anchor is
// the community model the learner received this round, not a zero slot.
#include "kernels/common.h"
#include "kernels/launchers.h"
#include "kernels/opt_body.h"

namespace mfl {

// split_pack (common.h): the packed bf16x3 weight mirror

// MIRROR: 0 none, 1 bf16 compute copy (p16), 2 packed bf16x3 split (ps)
template <int MODE, int MIRROR>
__global__ __launch_bounds__(256) void fused_opt_kernel(
    float* __restrict__ p, float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    const float* __restrict__ anchor, void* __restrict__ mirror, int64_t n4, OptHyper h,
    const float* __restrict__ lr_ptr, const int* __restrict__ step_ptr, int zero_grad,
    uint4* __restrict__ zero, int64_t zero16, int* __restrict__ tick_step) {
  const float lr = lr_ptr ? lr_ptr[0] * h.lr : h.lr;
  float bc1, bc2;
  opt_bias_corr(MODE, h, step_ptr, bc1, bc2);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = tid; i < zero16; i += stride) zero[i] = make_uint4(0, 0, 0, 0);
  // software-pipelined (the next element's operands in flight while this
  // one is updated: BERT's AdamW runs ~50 elements per thread)
  if (tid < n4) {
    OptIn4 cur = opt_load4<MODE>(p, g, m, v, anchor, tid);
    for (int64_t i = tid; i < n4; i += stride) {
      const bool more = i + stride < n4;
      OptIn4 nxt;
      if (more) nxt = opt_load4<MODE>(p, g, m, v, anchor, i + stride);
      opt_apply4<MODE, MIRROR>(cur, p, g, m, v, mirror, i, h, lr, bc1, bc2, zero_grad != 0);
      if (more) cur = nxt;
    }
  }
  // the step-counter increment that used to be its own launch; these modes
  // never read the counter, so one lane bumps it (Adam / AdamW read it in
  // every block: their launcher ticks in a separate launch -- a last-block
  // arrival counter over 2048 blocks serialised ~23 us of same-word atomics)
  if (MODE != OPT_ADAM && MODE != OPT_ADAMW && tick_step && blockIdx.x == 0 && threadIdx.x == 0)
    atomicAdd(tick_step, 1);
}

template <int MODE>
static void launch_mode(float* p, float* g, float* m, float* v, const float* anchor,
                        void* p16, int mirror, int64_t n, const OptHyper& h, const float* lr_ptr,
                        const int* step_ptr, bool zg, void* zero, int64_t zero_bytes,
                        hipStream_t s, int* tick_step) {
  const int64_t n4 = n / 4;
  const int64_t z16 = zero ? zero_bytes / 16 : 0;
  // MFL_OPT_GRID_CAP: workgroup cap of the grid-stride loop (A/B knob)
  static const int cap = [] {
    const char* e = getenv("MFL_OPT_GRID_CAP");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 2048;
  }();
  const unsigned grid = stream_grid(n4 > z16 ? n4 : z16, 256, cap);
  uint4* z = reinterpret_cast<uint4*>(zero);
  if (p16 && mirror == 2)
    fused_opt_kernel<MODE, 2><<<grid, 256, 0, s>>>(p, g, m, v, anchor, p16, n4, h, lr_ptr, step_ptr, zg ? 1 : 0,
                                                   z, z16, tick_step);
  else if (p16)
    fused_opt_kernel<MODE, 1><<<grid, 256, 0, s>>>(p, g, m, v, anchor, p16, n4, h, lr_ptr, step_ptr, zg ? 1 : 0,
                                                   z, z16, tick_step);
  else
    fused_opt_kernel<MODE, 0><<<grid, 256, 0, s>>>(p, g, m, v, anchor, p16, n4, h, lr_ptr, step_ptr, zg ? 1 : 0,
                                                   z, z16, tick_step);
}

void launch_fused_optimizer(int mode, float* p, float* g, float* m, float* v,
                            const float* anchor, void* p16, int64_t n, const OptHyper& h,
                            const float* lr_ptr, const int* step_ptr, bool zero_grad, void* zero,
                            int64_t zero_bytes, hipStream_t s, int* tick_step, int mirror) {
#define MFL_OPT_CASE(M_) \
  case M_: launch_mode<M_>(p, g, m, v, anchor, p16, mirror, n, h, lr_ptr, step_ptr, zero_grad, zero, zero_bytes, \
                           s, tick_step); break;
  switch (mode) {
    MFL_OPT_CASE(OPT_SGD)
    MFL_OPT_CASE(OPT_MOMENTUM)
    MFL_OPT_CASE(OPT_FEDPROX)
    MFL_OPT_CASE(OPT_ADAM)
    MFL_OPT_CASE(OPT_ADAMW)
    default: break;
  }
#undef MFL_OPT_CASE
  if (tick_step && (mode == OPT_ADAM || mode == OPT_ADAMW)) launch_tick(tick_step, 1, s);
}

// fp32 -> packed bf16x3 split mirror of a flat buffer (initial weights, a
// received community model)
__global__ __launch_bounds__(256) void split_pack_kernel(const float4* __restrict__ x, uint4* __restrict__ y,
                                                         int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = x[i];
    y[i] = make_uint4(split_pack(v.x), split_pack(v.y), split_pack(v.z), split_pack(v.w));
  }
}
void launch_split_pack(const float* x, uint32_t* y, int64_t n, hipStream_t s) {
  const int64_t n4 = n / 4;
  split_pack_kernel<<<stream_grid(n4), 256, 0, s>>>(reinterpret_cast<const float4*>(x), reinterpret_cast<uint4*>(y),
                                                    n4);
}

// ---------------------------------------------------------------------------
// fp32 -> bf16 cast of a flat buffer (community-model refresh of the compute
// copy after the RCCL all-reduce), optionally scaled.
__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ x,
                                                         uint16_t* __restrict__ y, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 a = reinterpret_cast<const float4*>(x)[i];
    uint2 o;
    o.x = pack2bf(a.x, a.y);
    o.y = pack2bf(a.z, a.w);
    reinterpret_cast<uint2*>(y)[i] = o;
  }
}

void launch_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t s) {
  const int64_t n4 = n / 4;
  cast_bf16_kernel<<<stream_grid(n4), 256, 0, s>>>(x, y, n4);
}

// In-place x *= w  (K1 pre-scale before the all-reduce).  The weight comes
// from device memory when wptr != nullptr so it can be decided on device.
__global__ __launch_bounds__(256) void scale_kernel(float* __restrict__ x, int64_t n4, float w,
                                                     const float* __restrict__ wptr) {
  const float a = wptr ? wptr[0] : w;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = reinterpret_cast<float4*>(x)[i];
    v.x *= a; v.y *= a; v.z *= a; v.w *= a;
    reinterpret_cast<float4*>(x)[i] = v;
  }
}

void launch_scale_f32(float* x, int64_t n, float w, const float* wptr, hipStream_t s) {
  const int64_t n4 = n / 4;
  scale_kernel<<<stream_grid(n4), 256, 0, s>>>(x, n4, w, wptr);
}

// Scale + cast in one pass: y16 = bf16(x), used after the all-reduce when the
// averaged model must be copied into the compute copy.
__global__ void tick_kernel(int* step, int inc) {
  if (threadIdx.x == 0 && blockIdx.x == 0) step[0] += inc;
}

void launch_tick(int* step, int inc, hipStream_t s) { tick_kernel<<<1, 64, 0, s>>>(step, inc); }

}  // namespace mfl
