// fp32 (reference-precision) convolution: geometry reuse of conv.h, fp32
// operand pointers.  Shared by conv32.hip and its torch binding.
#pragma once
#include "kernels/conv.h"
#include "kernels/launchers.h"
#include "kernels/opt_tail.h"

namespace mfl {

// Branch-free division by a runtime divisor d >= 1 for 0 <= x < 2^31:
// q = (umulhi(x, m) >> sh) + (x & id), with m = ceil(2^(31+s) / d),
// s = ceil(log2 d), sh = s - 1 (d = 1: m = 0, id = ~0).  Replaces the
// shift-or-divide branches in the DMA address math, which split the k-loop
// into basic blocks the scheduler could not interleave with the MFMAs.
struct FastDiv {
  uint32_t m;
  int sh;
  uint32_t id;
};

struct Conv32Args {
  ConvGeom g;          // fwd geometry, or the role-swapped dgrad geometry (conv.h)
  const float* src;    // fwd: X; dgrad: dY
  const float* wgt;    // OHWI weights [Cout][R][S][Cin]
  float* y;            // fwd: Y; dgrad: dX
  float* ysplit;       // split-K slabs [splits][tiles][BM*BN]
  int* counters;       // split-K arrival tickets, zero between launches
  double* stats;       // fwd: BN sums of Y (sum, sumsq) [2][Ng]
  // dgrad: BN-backward reductions of the consumer layer (see conv.h ConvArgs)
  const float* bn_z;
  const float* bn_y;
  const float* bn_mean;
  const float* bn_invstd;
  double* bn_acc;
  uint32_t src_bytes, wgt_bytes;
  int kchunk;
  int accum;
  int par_mc;
  FastDiv dc, dq, dpq;  // / C, / Q, / (P*Q)
  int reps;             // BN accumulator replicas ([reps][2][Ng]; workgroup b adds into replica b % reps)
};

struct BnBwdFusion32 {
  const float* z = nullptr;
  const float* y = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  double* acc = nullptr;
  int reps = 1;
};

// The API exists twice: mfl::c32x (exact fp32 MFMA) and mfl::c32s (fp32
// operands split into bf16 hi + lo, three bf16 MFMA products, fp32
// accumulation); conv32.hip is compiled once per variant.
namespace c32x {
#include "kernels/conv32_api.inc"
}
namespace c32s {
#include "kernels/conv32_api.inc"
}

}  // namespace mfl
