// Device pass of an optimizer tail (opt_tail.h), for the .hip kernels.
#pragma once
#include "kernels/opt_body.h"
#include "kernels/opt_tail.h"

namespace mfl {

namespace opt_tail_detail {
// The optimizer tail's grid-stride pass over its range (workgroup t of n).
// (software-pipelined: the next element's operands are loaded before this
// one is updated and stored -- the stores could alias them, so otherwise
// every element of a thread's range paid a full memory latency)
template <int MODE, int MIRROR>
static __device__ __forceinline__ void opt_tail_loop(const OptTail& o, int t, int n, float lr, float bc1, float bc2) {
  const int64_t stride = (int64_t)n * blockDim.x;
  int64_t i = (int64_t)t * blockDim.x + threadIdx.x;
  if (i >= o.n4) return;
  OptIn4 cur = opt_load4<MODE>(o.p, o.g, o.m, o.v, o.anchor, i);
  for (; i < o.n4; i += stride) {
    const bool more = i + stride < o.n4;
    OptIn4 nxt;
    if (more) nxt = opt_load4<MODE>(o.p, o.g, o.m, o.v, o.anchor, i + stride);
    opt_apply4<MODE, MIRROR>(cur, o.p, o.g, o.m, o.v, o.mirror, i, o.h, lr, bc1, bc2, o.zero_grad != 0);
    if (more) cur = nxt;
  }
}
template <int MIRROR>
static __device__ __forceinline__ void opt_tail_mirror(const OptTail& o, int t, int n) {
  const float lr = o.lr_ptr ? o.lr_ptr[0] * o.h.lr : o.h.lr;
  float bc1, bc2;
  opt_bias_corr(o.mode, o.h, o.step_ptr, bc1, bc2);
  switch (o.mode) {
    case OPT_SGD: opt_tail_loop<OPT_SGD, MIRROR>(o, t, n, lr, bc1, bc2); break;
    case OPT_MOMENTUM: opt_tail_loop<OPT_MOMENTUM, MIRROR>(o, t, n, lr, bc1, bc2); break;
    case OPT_FEDPROX: opt_tail_loop<OPT_FEDPROX, MIRROR>(o, t, n, lr, bc1, bc2); break;
    case OPT_ADAM: opt_tail_loop<OPT_ADAM, MIRROR>(o, t, n, lr, bc1, bc2); break;
    default: opt_tail_loop<OPT_ADAMW, MIRROR>(o, t, n, lr, bc1, bc2); break;
  }
}
static __device__ __forceinline__ void opt_tail_body(const OptTail& o, int t) {
  if (o.mirror_kind == 2) opt_tail_mirror<2>(o, t, o.nblk);
  else if (o.mirror_kind == 1) opt_tail_mirror<1>(o, t, o.nblk);
  else opt_tail_mirror<0>(o, t, o.nblk);
}

}  // namespace opt_tail_detail
using opt_tail_detail::opt_tail_body;

}  // namespace mfl
