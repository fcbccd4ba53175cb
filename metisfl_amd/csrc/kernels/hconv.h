// Halo-tiled fp32 convolutions on bf16x3 products with the producer's
// BatchNorm applied in the operand fill (hconv.hip).  Shared by the kernels
// and their torch binding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfl {
namespace hc {

// Per-channel BatchNorm source.  Train: batch statistics from the fp64 sums
// [reps][2][C] the producing convolution's epilogue accumulated; one block
// publishes mean / inv-std and updates the running averages.  Eval: the
// running statistics.
struct BnSrc {
  const double* acc = nullptr;
  int reps = 1;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  float* mean = nullptr;
  float* invstd = nullptr;
  float* run_mean = nullptr;
  float* run_var = nullptr;
  float momentum = 0.1f;
  float eps = 1e-5f;
};

// Forward input transform (applied once per element as it enters LDS):
//   v = relu?(z * sc + sh  [+ res | + (zr * sc2 + sh2)])
// zero outside the image (padding is in the post-activation domain).  The
// owner tiles (interior pixels, first output-channel tile) also write v (fp32,
// y) and its packed hi|lo split (yp): the backward's ReLU mask / residual and
// wgrad operand.
struct FwdXform {
  const float* z = nullptr;   // [N][H][W][C]
  int has_bn = 0;             // 0: z is already the activation (sc = 1, sh = 0)
  BnSrc bn;
  const float* res = nullptr;  // fp32 residual [N][H][W][C]
  const float* zr = nullptr;   // residual = BN_r(zr) (a projection shortcut's pre-BN output)
  BnSrc bnr;
  int relu = 0;
  float* y = nullptr;
  uint32_t* yp = nullptr;
  int train = 1;
  int M = 0;  // rows of the statistics (N*H*W)
};

struct FwdArgs {
  int N, H, W, C, Co;
  FwdXform x;
  const uint32_t* wp;  // packed (hi << 16 | lo) weight mirror [Co][3][3][C]
  float* out;          // pre-BN output [N][H][W][Co]
  double* stats;       // output BN sums [reps][2][Co] (nullptr: eval)
  int reps;
  float* slab;         // split-K slabs
  int* counters;       // split-K arrival tickets (zero between launches)
  long long* stamps = nullptr;  // profiling: per-workgroup phase timestamps [grid][16] (core clock)
  int dbg = 0;                  // ablation (timing only): 1 skip MFMAs, 2 skip fragment reads, 4 skip fills,
                                // 8 the first (bank-conflicting) weight-fill item order
  int xcd = 1;                  // XCD-grouped tile order (MFL_HC_XCD=0: hardware order)
  int bf16 = 0;                 // the bf16 option: z / res / zr / y / out bf16, wp = the bf16 weights
};

// ---- backward data (dgrad) -------------------------------------------------
// The BatchNorm whose backward the dgrad's operand fill applies: the sums
// [reps][2][C] of g and g * xhat are complete when the launch starts (the
// producer of dy accumulated them); one block publishes dgamma / dbeta.
struct BnBwdSrc {
  const double* acc = nullptr;
  int reps = 1;
  const float* gamma = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  float* dgamma = nullptr;
  float* dbeta = nullptr;
};

// Consumer BatchNorm-backward reductions in the dgrad epilogue (the BN whose
// upstream gradient dx is): acc += (sum g, sum g * xhat), g = dx [* (y > 0)].
struct BnSums {
  const float* z = nullptr;
  const float* y = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  double* acc = nullptr;
  int reps = 1;
};

// dgrad input transform (once per element, as it enters LDS):
//   g = dy [* (y > 0)],  dz = gamma * invstd * (g - mean(g) - xhat * mean(g * xhat))
// zero outside the image.  Owner tiles write dz's packed split (dzp: the
// layer's wgrad operand) and g (dres: the residual branch's gradient).
struct DgXform {
  const float* dy = nullptr;     // [N][H][W][C] gradient w.r.t. the layer output
  const float* ymask = nullptr;  // post-activation output (ReLU mask) or nullptr
  const float* z = nullptr;      // pre-BN conv output
  BnBwdSrc bn;
  int M = 0;
  float* dres = nullptr;
  uint32_t* dzp = nullptr;
};

// dx = conv3x3^T(dz, W) (+ dx when accumulate): C = dz channels (the layer's
// output channels, the reduction), Co = dx channels (the layer's input).
struct DgArgs {
  int N, H, W, C, Co;
  DgXform x;
  const uint32_t* wp;  // the layer's packed weight mirror [C][3][3][Co]
  float* out;
  int accumulate = 0;
  BnSums bnb;
  float* slab;
  int* counters;
  long long* stamps = nullptr;
  int dbg = 0;
  int xcd = 1;
};

// Geometry supported by the halo kernels (3x3, stride 1, pad 1, square
// CIFAR-ResNet stages); returns the split-K workspace floats (incl. 1024
// counter words) or -1 when unsupported.
int64_t hconv_fwd_workspace(int N, int H, int W, int C, int Co);
void launch_hconv_fwd(const FwdArgs& a, hipStream_t s);
void launch_hconv_dgrad(const DgArgs& a, hipStream_t s);

}  // namespace hc
}  // namespace mfl
