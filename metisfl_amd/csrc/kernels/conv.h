// Convolution geometry / launch plans shared by conv.hip and its binding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfl {

// Implicit-GEMM geometry.  For the forward pass (and wgrad):
//   H, W, C : input activation dims (NHWC, C % 8 == 0)
//   P, Q    : output spatial dims
//   M       : N * P * Q      (GEMM rows; for wgrad the reduction length)
//   K       : R * S * C      (GEMM reduction; for wgrad the output columns)
//   Ng      : Cout
// For dgrad the roles swap: H, W, C describe dY, P, Q the dX spatial dims,
// Ng = Cin and K = R * S * Cout.
struct ConvGeom {
  int N, H, W, C;
  int P, Q;
  int R, S, stride, pad;
  int M, K, Ng;
};

struct ConvPlan {
  int bm = 64, bn = 64;
  int splits = 1;
  int kchunk = 0;      // reduction elements per split (multiple of 64)
  int stats_rows = 0;  // 1 = the epilogue accumulates BN statistics
  int bk = 64;         // k-tile depth (64 or 128)
  int par_mc = 0;      // stride-2 dgrad parity decomposition: rows per class (0 = off)
  int stages = 3;      // LDS ring depth (conv32.hip)
};

// Kernel argument block.  *_shift = log2 of the divisor when it is a power of
// two (wave-uniform shift instead of an integer division), else -1.
struct ConvArgs {
  ConvGeom g;
  const uint16_t* src;
  const uint16_t* wgt;
  uint16_t* y;
  float* ysplit;   // split-K slabs [splits][tiles][BM*BN]
  int* counters;   // split-K arrival tickets [tiles], zero between launches
  double* stats;
  // dgrad epilogue fusion of the NEXT BatchNorm backward's reductions: dX is
  // the upstream gradient dy of the layer that produced this conv's input,
  // so while writing the final dX tile the epilogue adds
  //   sum(g) and sum(g * xhat),  g = dX * [y > 0],  xhat = (z - mean) * invstd
  // into bn_acc[2][Ng] (fp64 atomics).  bn_acc == nullptr: off.
  const uint16_t* bn_z;
  const uint16_t* bn_y;  // nullptr: that layer has no ReLU
  const float* bn_mean;
  const float* bn_invstd;
  double* bn_acc;
  // dense-GEMM epilogue (1x1 geometry, BERT path): y = acc + bias[col] +
  // resid[row][col]; act_out (optional) = gelu(y).  All nullptr on conv paths.
  const float* bias;
  const uint16_t* resid;
  uint16_t* act_out;
  uint32_t src_bytes, wgt_bytes;  // buffer-descriptor ranges of src / wgt
  int kchunk;
  int accum;
  int dbg;  // timing experiments only (MFL_CONV_DEBUG): bit0 skip MFMAs, bit1 skip operand DMA
  int par_mc;  // stride-2 dgrad parity decomposition: rows per class (0 = off)
  int c_shift, q_shift, pq_shift;
};

ConvPlan plan_conv_gemm(const ConvGeom& g, bool dgrad = false);
ConvPlan plan_conv_wgrad(const ConvGeom& g, int target_blocks = 0);
// split-K workgroup targets of the bf16 forward / dgrad and weight-gradient
// plans (0: the defaults, 256 / 512); MFL_CONV_TARGET_BLOCKS /
// MFL_WGRAD_TARGET_BLOCKS override
void set_conv_plan_targets(int conv_target, int wgrad_target);
// number of output tiles (= split-K counter slots) of a gemm plan
int conv_counter_slots(const ConvGeom& g, const ConvPlan& p);

// y (bf16 [M][Ng]) and, when stats != nullptr, fp64 atomic accumulation of the
// per-channel BatchNorm sums into stats[0..Ng) / stats[Ng..2Ng).  With
// p.splits > 1, ysplit holds splits*slots*bm*bn floats and counters `slots`
// zero-initialised ints (the kernel re-arms them).
void launch_conv_gemm(const ConvGeom& g, bool dgrad, const ConvPlan& p, const uint16_t* src,
                      const uint16_t* wgt, uint16_t* y, float* ysplit, int* counters,
                      double* stats, bool accum, hipStream_t s);
struct BnBwdFusion {
  const uint16_t* z = nullptr;
  const uint16_t* y = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  double* acc = nullptr;
};
// A layer's dgrad (geometry gd, plan pd as sized for the caller's workspace,
// optional fused BN-backward reductions f) and wgrad (forward geometry gw,
// dw += ..., zero on entry) in one launch.  false: not supported for this
// shape (or MFL_CONV_PAIR=0) -- nothing was launched.
// ot (optional): an optimizer tail run by extra workgroups of the same launch
// (opt_tail.h; mirror_kind 1 = the bf16 compute copy)
struct OptTail;
bool launch_conv_bwd_pair(const ConvGeom& gd, const ConvPlan& pd, const uint16_t* dy, const uint16_t* wt,
                          uint16_t* dx, float* ysplit, int* counters, bool accum, const BnBwdFusion* f,
                          const ConvGeom& gw, const uint16_t* x, float* dw, hipStream_t s,
                          const OptTail* ot = nullptr);
// A downsampling block's 3x3/s2 conv1 (g1) and 1x1/s2 shortcut (g2) forward
// convolutions of the same input x in one launch (plans / workspaces / stats
// as for launch_conv_gemm); false: not supported -- nothing was launched.
bool launch_conv_fwd_pair(const ConvGeom& g1, const ConvPlan& p1, const uint16_t* w1, uint16_t* y1, float* ys1,
                          int* cnt1, double* st1, const ConvGeom& g2, const ConvPlan& p2, const uint16_t* w2,
                          uint16_t* y2, float* ys2, int* cnt2, double* st2, const uint16_t* x, hipStream_t s);
// dgrad with the fused BN-backward reductions of the consumer layer
void launch_conv_dgrad_bnb(const ConvGeom& g, const ConvPlan& p, const uint16_t* dy,
                           const uint16_t* wgt, uint16_t* dx, float* ysplit, int* counters,
                           bool accum, const BnBwdFusion& f, hipStream_t s);
struct GemmEpilogueArgs {
  const float* bias = nullptr;
  const uint16_t* resid = nullptr;
  uint16_t* act_out = nullptr;
};
// forward implicit GEMM with the dense epilogue (bias / residual / GELU copy)
void launch_conv_gemm_epi(const ConvGeom& g, const ConvPlan& p, const uint16_t* src,
                          const uint16_t* wgt, uint16_t* y, float* ysplit, int* counters,
                          const GemmEpilogueArgs& e, hipStream_t s);
// dw (fp32 [Cout][R][S][Cin]); must be zeroed first when p.splits > 1.
void launch_conv_wgrad(const ConvGeom& g, const ConvPlan& p, const uint16_t* x, const uint16_t* dy,
                       float* dw, hipStream_t s, bool accumulate = false);
void launch_transpose_krsc(const uint16_t* w, uint16_t* wt, int Co, int RS, int Ci, hipStream_t s);

}  // namespace mfl
