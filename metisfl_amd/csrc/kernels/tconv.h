// Throughput-regime fp32 convolutions (tconv.hip): the backward GEMMs of a
// ResNet layer built for the co-located regime, where several learners'
// launches share the GPU and what counts is MFMA work per operand byte, not
// per-launch latency (profiles/ANALYSIS.md, round 5).
//
// Operands are the packed bf16x3 encodings the rest of the fp32 path already
// writes (dword = hi << 16 | lo, common.h split_pack): activations (BN apply
// mirror), dY (fp32 BN backward) and weights (optimizer mirror, OHWI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfl {
namespace tc {

// Forward geometry of one conv layer (NHWC input [N][H][W][C], OHWI weights
// [Co][KS][KS][C], output [N][P][Q][Co]).
struct Geom {
  int N, H, W, C, Co, KS, ST, pad;
  int P, Q;
};

// The consumer BatchNorm whose backward sums a dgrad epilogue fuses (as
// conv32.h BnBwdFusion32): dX is stored as g = dX [y > 0] (y given) and
// acc[rep][0][c] += sum g, acc[rep][1][c] += sum g (z - mean) invstd.
struct Bnb {
  const float* z = nullptr;
  const float* y = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  double* acc = nullptr;
  int reps = 1;
};

// Shapes the kernels take (3x3 / stride 1 / pad 1, power-of-two spatial
// sizes, channel counts multiples of 64).
bool wgrad_ok(const Geom& g);
bool dgrad_ok(const Geom& g);

// Tile configurations (cfg < 0: the planner's choice; sweeps index them).
int num_wgrad_cfgs();
int num_dgrad_cfgs();
bool wgrad_cfg_fits(const Geom& g, int cfg);
bool dgrad_cfg_fits(const Geom& g, int cfg);

// dw[Co][KS][KS][C] += sum_m dY[m][co] * im2col(X)[m][(r, s, c)].
// dw must hold zeros or a running sum (split slices add atomically).
// splits <= 0: the built-in plan.
void launch_wgrad(const Geom& g, const uint32_t* xp, const uint32_t* dyp, float* dw, int splits,
                  hipStream_t s, int cfg = -1);
int wgrad_default_splits(const Geom& g, int cfg = -1);

// dX[N][H][W][C] (+)= conv_transpose(dY, W) with the fused consumer-BN sums.
// ws / counters: split-K slabs and arrival tickets (dgrad_workspace floats /
// dgrad_counters ints; counters zero between launches).
void launch_dgrad(const Geom& g, const uint32_t* dyp, const uint32_t* wp, float* dx, bool accum, const Bnb* bnb,
                  float* ws, int* counters, int splits, hipStream_t s, int cfg = -1);
int dgrad_default_splits(const Geom& g, int cfg = -1);
int64_t dgrad_workspace(const Geom& g, int splits, int cfg = -1);
int dgrad_counters(const Geom& g, int cfg = -1);

}  // namespace tc
}  // namespace mfl
