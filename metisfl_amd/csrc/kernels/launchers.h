// Host-callable launch functions for the HIP kernels.  Every launcher takes
// the HIP stream explicitly, allocates nothing and never synchronises, so all
// of them are legal inside hipGraph capture (cdna_hip_programming.md G9).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfl {

enum OptMode { OPT_SGD = 0, OPT_MOMENTUM = 1, OPT_FEDPROX = 2, OPT_ADAM = 3, OPT_ADAMW = 4 };

struct OptHyper {
  float lr = 0.01f;
  float l1 = 0.f, l2 = 0.f;
  float momentum = 0.f;
  float mu = 0.f;
  float beta1 = 0.9f, beta2 = 0.999f, eps = 1e-7f;
  float wd = 0.f;
};

// ---- optim.hip -----------------------------------------------------------
// zero_grad: write 0 back into g after use (next step's atomics start from 0);
// zero/zero_bytes: an extra region (BN accumulators) zeroed by the same launch.
// p16: the weight mirror written from the updated fp32 values -- bf16 (mirror
// 1) or the packed bf16x3 split (mirror 2, conv32.hip c32s); nullptr: none
void launch_fused_optimizer(int mode, float* p, float* g, float* m, float* v,
                            const float* anchor, void* p16, int64_t n, const OptHyper& h,
                            const float* lr_ptr, const int* step_ptr, bool zero_grad, void* zero,
                            int64_t zero_bytes, hipStream_t s, int* tick_step = nullptr, int mirror = 1);
void launch_split_pack(const float* x, uint32_t* y, int64_t n, hipStream_t s);
// tick_step: also increment *tick_step once, after the optimizer's reads of
// step_ptr (in the same launch for the modes that never read it)
void launch_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t s);
void launch_scale_f32(float* x, int64_t n, float w, const float* wptr, hipStream_t s);
void launch_tick(int* step, int inc, hipStream_t s);

// ---- aggregate.hip -------------------------------------------------------
// dtype codes follow metisfl DType.Type (model.proto): INT8=0 .. FLOAT64=9
constexpr int kMaxAggInputs = 16;
struct AggInputs {
  const void* ptr[kMaxAggInputs];
  double w[kMaxAggInputs];
  int count;
};
void launch_weighted_sum(int dtype, void* out, const AggInputs& in, int64_t n, bool accumulate,
                         hipStream_t s);
void launch_axpby(int dtype, void* y, const void* x, double a, double b, int64_t n, hipStream_t s);
void launch_count_zeros(int dtype, const void* x, const int64_t* tile_seg, const int64_t* tile_beg,
                        const int64_t* tile_end, int ntiles, unsigned long long* counts,
                        hipStream_t s);
// Exact-form fp32 scaled all-reduce pre-pass: y = (float)((double)x * w)
void launch_ckks_pwa(const uint64_t* const* cts, const uint64_t* wq, int nlearners, uint64_t* out,
                     const uint64_t* moduli, int nlimbs, int64_t coeffs_per_limb, int64_t nct,
                     hipStream_t s);

// ---- bn.hip --------------------------------------------------------------
struct BnFwdArgs {
  const uint16_t* x;
  const uint16_t* residual;  // optional
  uint16_t* y;
  const double* acc;         // [2][C] sum / sumsq (train)
  const float* gamma;
  const float* beta;
  float* mean;               // saved for backward (train)
  float* invstd;
  float* run_mean;           // updated (train) / read (eval)
  float* run_var;
  int64_t M;
  int C;
  float momentum, eps;
  int train, relu;
};
struct BnBwdArgs {
  const uint16_t* dy;
  const uint16_t* x;   // BN input (pre-normalisation)
  const uint16_t* y;   // BN(+res)(+relu) output: ReLU mask, optional
  const double* acc;   // [2][C] sum dyr / sum dyr*xhat
  const float* gamma;
  const float* mean;
  const float* invstd;
  float* dgamma;
  float* dbeta;
  uint16_t* dx;
  uint16_t* dy_masked;  // optional
  int64_t M;
  int C;
};
int bn_stats_blocks(int64_t M, int C);
void launch_bn_stats(const uint16_t* x, int64_t M, int C, double* acc, hipStream_t s);
void launch_bn_apply(const BnFwdArgs& a, hipStream_t s);
// a1: no residual, no ReLU; a2: no residual, ReLU (a downsampling block's
// shortcut and conv1 BatchNorms) in one launch
void launch_bn_apply_pair(const BnFwdArgs& a1, const BnFwdArgs& a2, hipStream_t s);
void launch_bn_bwd_reduce(const uint16_t* dy, const uint16_t* x, const uint16_t* y,
                          const float* mean, const float* invstd, int64_t M, int C, double* acc,
                          hipStream_t s);
void launch_bn_bwd_apply(const BnBwdArgs& a, hipStream_t s);

// ---- bn32.hip (fp32 reference-precision path) -----------------------------
struct BnFwdArgs32 {
  const float* x;
  const float* residual;  // optional
  float* y;
  // optional: y's packed bf16x3 split (split_pack, common.h) -- the activation
  // operand the bf16x3 forward / wgrad convolutions decode without splitting
  uint32_t* yp;
  const double* acc;
  const float* gamma;
  const float* beta;
  float* mean;
  float* invstd;
  float* run_mean;
  float* run_var;
  int64_t M;
  int C;
  float momentum, eps;
  int train, relu;
  int reps;  // acc holds [reps][2][C] replicas, summed here
};
struct BnBwdArgs32 {
  const float* dy;
  const float* x;
  const float* y;
  const double* acc;
  const float* gamma;
  const float* mean;
  const float* invstd;
  float* dgamma;
  float* dbeta;
  float* dx;
  float* dy_masked;
  int64_t M;
  int C;
  int reps;  // acc replicas, as BnFwdArgs32
  // optional side reduction over the masked gradient written to dy_masked:
  // acc2 += (sum g, sum g * (z2 - mean2) * invstd2) -- the BN backward sums
  // of a projection shortcut whose upstream gradient IS dy_masked
  const float* z2;
  const float* mean2;
  const float* invstd2;
  double* acc2;
  int reps2;
  // 1: dx is written as packed bf16x3 splits (split_pack, common.h) -- the
  // dY operand the bf16x3 dgrad / wgrad kernels decode without splitting
  int pack_dx;
};
void launch_bn32_stats(const float* x, int64_t M, int C, double* acc, hipStream_t s, int reps = 1);
void launch_bn32_apply(const BnFwdArgs32& a, hipStream_t s);
// grid cap of the fp32 BatchNorm apply kernels (0: the build default, 512)
void set_bn32_grid_cap(int cap);
void launch_bn32_apply_pair(const BnFwdArgs32& a1, const BnFwdArgs32& a2, hipStream_t s);  // a1 no ReLU, a2 ReLU
void launch_bn32_bwd_reduce(const float* dy, const float* x, const float* y, const float* mean,
                            const float* invstd, int64_t M, int C, double* acc, hipStream_t s, int reps = 1);
void launch_bn32_bwd_apply(const BnBwdArgs32& a, hipStream_t s);
void launch_bn32_bwd_apply_pair(const BnBwdArgs32& a1, const BnBwdArgs32& a2, hipStream_t s);
// The stem's backward in one launch: its BatchNorm(+ReLU) backward (dz, as
// bn32_bwd_apply, never written out) and the 3x3 / stride-1 weight gradient
// dw[Co][3][3][Cin] += sum_p dz[p] x[p + tap] (exact fp32 FMAs).  a.dx: unused;
// x: the stem input [N][H][W][Cin] fp32.  Shapes: stem_bwd32_ok.
bool stem_bwd32_ok(int N, int H, int W, int Cin, int Co);
struct OptTail;  // opt_tail.h: an optimizer tail riding in the stem backward launch (optional)
void launch_stem_bwd32(const BnBwdArgs32& a, const float* x, int N, int H, int W, int Cin, float* dw, hipStream_t s,
                       const OptTail* ot = nullptr);
// the same with the bf16 option's dy / z / y / x (a.dy, a.x, a.y point at bf16)
void launch_stem_bwd_bf16(const BnBwdArgs32& a, const uint16_t* x, int N, float* dw, hipStream_t s,
                          const OptTail* ot = nullptr);

// ---- head.hip ------------------------------------------------------------
// fp32 head whose input is relu(BN(z) + res), applied in its pooling loop
// (the last block's BatchNorm apply folded into the head): writes the
// activation y (the backward's ReLU mask) and, in train mode, publishes the
// BN statistics and adds the BN-backward sums of dx (g = dx * [y > 0]: sum g,
// sum g * xhat) into acc_b.
struct HeadBn {
  const float* z = nullptr;
  const float* res = nullptr;
  const double* acc = nullptr;
  int reps = 1;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  float* mean = nullptr;
  float* invstd = nullptr;
  float* run_mean = nullptr;
  float* run_var = nullptr;
  float momentum = 0.1f, eps = 1e-5f;
  int train = 1;
  float* y = nullptr;
  double* acc_b = nullptr;
  int reps_b = 1;
};
// lpart (fused-BN path): [B][C / 128][K] fp32 scratch of the split head
// (head.hip head_split_*); nullptr: the one-launch head
void launch_head32_fwd_bwd(const float* x, int B, int HW, int C, const float* W, const float* bias, int K,
                           const int* labels, float* feat, float* dlogits, float* dx, float* stats, bool backward,
                           hipStream_t s, float* dW = nullptr, float* db = nullptr, const HeadBn* bn = nullptr,
                           float* lpart = nullptr);
void launch_head_fwd_bwd(const uint16_t* x, int B, int HW, int C, const float* W, const float* bias,
                         int K, const int* labels, float* feat, float* dlogits, uint16_t* dx,
                         float* stats, bool backward, hipStream_t s, float* dW = nullptr,
                         float* db = nullptr, const HeadBn* bn = nullptr, float* lpart = nullptr);
void launch_head_wgrad(const float* feat, const float* dlogits, int B, int C, int K, float* dW,
                       float* db, hipStream_t s);

// ---- data.hip ------------------------------------------------------------
void launch_gather_batch(const uint16_t* shard, const int* labels, const int* perm,
                         const int* step, int steps_per_epoch, int B, int64_t row_elems,
                         uint16_t* xb, int* yb, hipStream_t s, uint32_t* xp = nullptr);

// ---- layers.hip (example-model layers) -------------------------------------
void launch_bias_act_fwd(uint16_t* y, const float* bias, int64_t M, int N, int act, hipStream_t s);
void launch_bias_act_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dz, float* dbias, int64_t M,
                         int N, int act, hipStream_t s);
void launch_maxpool2(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, hipStream_t s);
void launch_maxpool2_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* y, uint16_t* dx, int N,
                         int H, int W, int C, hipStream_t s);
void launch_dropout(const uint16_t* in, uint16_t* out, int64_t n, float p, uint32_t seed, const int* step,
                    hipStream_t s);
void launch_xent(const uint16_t* logits, const int* labels, int B, int Kp, int K, uint16_t* dlogits,
                 float* stats, bool backward, hipStream_t s);
void launch_mse(const uint16_t* pred, const float* target, int B, int Kp, uint16_t* dpred, float* stats,
                bool backward, hipStream_t s);

}  // namespace mfl
