// Optimizer tails (see OptTail): shared by the fp32 (conv32.hip) and bf16
// (conv.hip) paired backward launches.  Host-safe (the bindings include it);
// the device pass is opt_tail_dev.h.
#pragma once
#include "kernels/launchers.h"

namespace mfl {

// Optimizer tail of a paired backward launch: workgroups appended after the
// dgrad / wgrad ones apply the fused optimizer (opt_body.h) to a range of the
// flat model whose gradients are already final (a later layer's), so its
// HBM-bound pass fills the CUs the latency-bound GEMMs leave idle instead of
// running as the step's last launch.  nblk == 0: no tail.
struct OptTail {
  float* p = nullptr;
  float* g = nullptr;
  float* m = nullptr;
  float* v = nullptr;
  const float* anchor = nullptr;
  void* mirror = nullptr;
  int64_t n4 = 0;        // float4 elements
  OptHyper h{};
  const float* lr_ptr = nullptr;
  const int* step_ptr = nullptr;
  int mode = 0;          // OptMode
  int mirror_kind = 0;   // 0 none, 1 bf16 compute copy, 2 packed bf16x3 split
  int zero_grad = 1;
  int nblk = 0;
};



}  // namespace mfl
