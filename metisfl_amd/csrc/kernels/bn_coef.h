// fp32 BatchNorm coefficient math shared by the kernels that apply a
// BatchNorm (bn32.hip's apply, head.hip's fused input): fp64 statistics from
// the [reps][2][C] replica sums, fp32 scale / shift, and the publication of
// the batch statistics and running averages.  One definition, so every
// consumer derives the same bits (hconv.hip distributes the replica loads
// over its waves but sums them in the same order).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfl {

constexpr int kMaxReps = 8;  // replicas summed per channel (layers.py uses 8 on the fp32 GPU path)

// Sum of a channel's replicas: every load issued before the first add (a
// runtime-bound loop serialised one memory round trip per replica).
__device__ __forceinline__ void rep_sums(const double* acc, int reps, int C, int c, double& s0, double& s1) {
  double a[kMaxReps], b[kMaxReps];
#pragma unroll
  for (int r = 0; r < kMaxReps; ++r) {
    a[r] = r < reps ? acc[(int64_t)r * 2 * C + c] : 0.0;
    b[r] = r < reps ? acc[(int64_t)r * 2 * C + C + c] : 0.0;
  }
  s0 = 0.0;
  s1 = 0.0;
#pragma unroll
  for (int r = 0; r < kMaxReps; ++r) {
    s0 += a[r];
    s1 += b[r];
  }
}

// Channel c's scale / shift (train: batch statistics over M rows, published
// when `publish`; eval: running statistics).
__device__ __forceinline__ void bn_fwd_coef(const double* acc, int reps, int C, int c, int64_t M, bool train,
                                            bool publish, const float* gamma, const float* beta, float* mean,
                                            float* invstd, float* run_mean, float* run_var, float momentum,
                                            float eps, float& sc, float& sh, float* mu_f = nullptr,
                                            float* isd_f = nullptr) {
  double mu, var;
  if (train) {
    double s0, s1;
    rep_sums(acc, reps, C, c, s0, s1);
    const double inv_m = 1.0 / (double)M;
    mu = s0 * inv_m;
    var = s1 * inv_m - mu * mu;
    if (var < 0.0) var = 0.0;
  } else {
    mu = run_mean[c];
    var = run_var[c];
  }
  const double isd = 1.0 / sqrt(var + (double)eps);
  sc = (float)((double)gamma[c] * isd);
  sh = (float)((double)beta[c] - mu * (double)gamma[c] * isd);
  if (mu_f) *mu_f = (float)mu;  // the published values, for a consumer in the same launch
  if (isd_f) *isd_f = (float)isd;
  if (train && publish) {
    mean[c] = (float)mu;
    invstd[c] = (float)isd;
    if (run_mean) {
      const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
      // explicit fma: the halo conv's fill publishes the same bits (hconv.hip)
      run_mean[c] = fmaf(1.f - momentum, run_mean[c], momentum * (float)mu);
      run_var[c] = fmaf(1.f - momentum, run_var[c], momentum * (float)unb);
    }
  }
}

}  // namespace mfl
