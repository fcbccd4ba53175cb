// fp32 (reference-precision) convolution: geometry reuse of conv.h, fp32
// operand pointers.  Shared by conv32.hip and its torch binding.
#pragma once
#include "kernels/conv.h"

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

// mode 0 fwd, 1 dgrad, 2 wgrad.  kchunk in k elements (multiple of 32).
ConvPlan plan_conv32(const ConvGeom& g, int mode);
int conv32_counter_slots(const ConvGeom& g, const ConvPlan& p);

// stats: [stats_reps][2][Ng] fp64 BN sums of the forward output (replicated
// so that hundreds of workgroups do not serialise on the same 2*Ng addresses)
void launch_conv32_gemm(const ConvGeom& g, bool dgrad, const ConvPlan& p, const float* src, const float* wgt,
                        float* y, float* ysplit, int* counters, double* stats, bool accum,
                        const BnBwdFusion32* bnb, hipStream_t s, int stats_reps = 1);
// dw (fp32 OHWI); accumulate: dw holds a running sum (zero for a fresh step)
// and every slice adds atomically; otherwise the split-1 plan stores and a
// split plan requires dw zeroed by the caller.
void launch_conv32_wgrad(const ConvGeom& g, const ConvPlan& p, const float* x, const float* dy, float* dw,
                         bool accumulate, hipStream_t s);
// dgrad (gd, pd; role-swapped geometry) + wgrad (gf = the forward geometry,
// pw; dw must hold zeros or a running sum: slices add atomically) of one
// layer in one launch.  Returns false (nothing launched) when the two plans
// do not both run 64x64 tiles on the fast address paths.
// conv1 (3x3/s2, g1) + projection shortcut (1x1/s2, g2) of one x in one
// launch; false (nothing launched) when the plans do not pair.
bool launch_conv32_fwd_pair(const ConvGeom& g1, const ConvPlan& p1, const float* w1, float* y1, float* ys1,
                            int* c1, double* st1, int reps1, const ConvGeom& g2, const ConvPlan& p2,
                            const float* w2, float* y2, float* ys2, int* c2, double* st2, int reps2,
                            const float* x, hipStream_t s);
bool launch_conv32_bwd_pair(const ConvGeom& gd, const ConvPlan& pd, const ConvGeom& gf, const ConvPlan& pw,
                            const float* dy, const float* w, float* dx, float* ysplit, int* counters, bool accum,
                            const BnBwdFusion32* bnb, const float* x, float* dw, hipStream_t s);

}  // namespace mfl
