// K12: BatchNorm forward/backward for NHWC bf16 activations, fp32 statistics.
//
// The reference only reaches BatchNorm through Keras layers
// (examples/keras/models/cifar_cnn.py:27,32); here it is a first-class
// hand-written kernel family, because ResNet-18 runs 20 of them per step.
//
// Layout: x is [M, C] with M = N*H*W rows and C contiguous channels (NHWC).
// Each lane owns 8 consecutive channels (one 16-B load), a 256-thread block
// covers 256/(C/8) rows per pass.  Reductions are two-level and
// deterministic: per-block partials [nblocks][2][C] -> one finalize block
// (double-precision combine) -> per-channel affine coefficients.
// Fusions: forward apply = affine + optional residual add + optional ReLU;
// backward apply = ReLU mask + dx, and optionally writes the masked dy that
// the residual shortcut consumes (so the add+relu needs no kernel of its own).
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace mfl {

__host__ __device__ static inline int tpr_of(int C) { return C / 8; }

int bn_stats_blocks(int64_t M, int C) {
  const int tpr = tpr_of(C);
  const int rpp = 256 / tpr;
  int64_t nb = (M + (int64_t)rpp * 8 - 1) / ((int64_t)rpp * 8);
  if (nb > 512) nb = 512;
  if (nb < 1) nb = 1;
  return (int)nb;
}

// Shared epilogue: reduce the per-thread [8] accumulators a0/a1 over the rows
// of the block and store partial[blockIdx][0|1][C].
__device__ __forceinline__ void block_channel_reduce(const float* a0, const float* a1, int C,
                                                     int tpr, int rpp, float* partial) {
  __shared__ float sh[2][256 * 8];
  const int t = threadIdx.x;
  const bool act = t < rpp * tpr;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sh[0][t * 8 + k] = act ? a0[k] : 0.f;
    sh[1][t * 8 + k] = act ? a1[k] : 0.f;
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float s0 = 0.f, s1 = 0.f;
    const int cg = c >> 3, ck = c & 7;
    for (int r = 0; r < rpp; ++r) {
      s0 += sh[0][(r * tpr + cg) * 8 + ck];
      s1 += sh[1][(r * tpr + cg) * 8 + ck];
    }
    partial[(int64_t)blockIdx.x * 2 * C + c] = s0;
    partial[(int64_t)blockIdx.x * 2 * C + C + c] = s1;
  }
}

__global__ __launch_bounds__(256) void bn_stats_kernel(const uint16_t* __restrict__ x, int64_t M,
                                                       int C, float* __restrict__ partial) {
  const int tpr = tpr_of(C);
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int cg = t % tpr;
  const int r0 = t / tpr;
  float s[8] = {0}, q[8] = {0};
  if (r0 < rpp) {
    for (int64_t row = (int64_t)blockIdx.x * rpp + r0; row < M; row += (int64_t)gridDim.x * rpp) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + row * C + cg * 8);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += f[k];
        q[k] += f[k] * f[k];
      }
    }
  }
  block_channel_reduce(s, q, C, tpr, rpp, partial);
}

void launch_bn_stats(const uint16_t* x, int64_t M, int C, float* partial, int nblocks,
                     hipStream_t s) {
  bn_stats_kernel<<<nblocks, 256, 0, s>>>(x, M, C, partial);
}

__global__ __launch_bounds__(256) void bn_finalize_kernel(
    const float* __restrict__ partial, int nblocks, int64_t M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ mean, float* __restrict__ invstd,
    float* __restrict__ scale, float* __restrict__ shift, float* __restrict__ run_mean,
    float* __restrict__ run_var, float momentum, float eps) {
  // one wave per channel: lanes stride over the partial rows, then reduce
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  {
    double s = 0.0, q = 0.0;
    for (int b = lane; b < nblocks; b += 64) {
      s += partial[(int64_t)b * 2 * C + c];
      q += partial[(int64_t)b * 2 * C + C + c];
    }
    s = wave_sum(s);
    q = wave_sum(q);
    if (lane != 0) return;
    const double mu = s / (double)M;
    double var = q / (double)M - mu * mu;
    if (var < 0.0) var = 0.0;
    const float is = (float)(1.0 / sqrt(var + (double)eps));
    mean[c] = (float)mu;
    invstd[c] = is;
    const float g = gamma[c];
    scale[c] = g * is;
    shift[c] = beta[c] - (float)mu * g * is;
    if (run_mean) {
      const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mu;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
    }
  }
}

void launch_bn_finalize(const float* partial, int nblocks, int64_t M, int C, const float* gamma,
                        const float* beta, float* mean, float* invstd, float* scale, float* shift,
                        float* run_mean, float* run_var, float momentum, float eps, hipStream_t s) {
  bn_finalize_kernel<<<(C + 3) / 4, 256, 0, s>>>(partial, nblocks, M, C, gamma, beta, mean, invstd, scale,
                                       shift, run_mean, run_var, momentum, eps);
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void bn_apply_kernel(const uint16_t* __restrict__ x,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const uint16_t* __restrict__ res,
                                                       uint16_t* __restrict__ y, int64_t nvec, int C) {
  extern __shared__ __attribute__((aligned(16))) float coef[];  // [2][C]
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    coef[c] = scale[c];
    coef[C + c] = shift[c];
  }
  __syncthreads();
  const int tpr = C / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int cg = (int)(i % tpr);
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(x)[i], f);
    float r[8];
    if (RES) unpack8(reinterpret_cast<const uint4*>(res)[i], r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = f[k] * coef[cg * 8 + k] + coef[C + cg * 8 + k];
      if (RES) v += r[k];
      if (RELU) v = fmaxf(v, 0.f);
      f[k] = v;
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
}

void launch_bn_apply(const uint16_t* x, const float* scale, const float* shift,
                     const uint16_t* residual, uint16_t* y, int64_t M, int C, bool relu,
                     hipStream_t s) {
  const int64_t nvec = M * C / 8;
  const unsigned g = stream_grid(nvec, 256, 2048);
  const size_t sm = 2 * C * sizeof(float);
  if (residual) {
    if (relu) bn_apply_kernel<true, true><<<g, 256, sm, s>>>(x, scale, shift, residual, y, nvec, C);
    else bn_apply_kernel<true, false><<<g, 256, sm, s>>>(x, scale, shift, residual, y, nvec, C);
  } else {
    if (relu) bn_apply_kernel<false, true><<<g, 256, sm, s>>>(x, scale, shift, residual, y, nvec, C);
    else bn_apply_kernel<false, false><<<g, 256, sm, s>>>(x, scale, shift, residual, y, nvec, C);
  }
}

// ---------------------------------------------------------------------------
// Backward.  y (post-activation output) supplies the ReLU mask when non-null.
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, const uint16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, int64_t M, int C,
    float* __restrict__ partial) {
  const int tpr = tpr_of(C);
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int cg = t % tpr;
  const int r0 = t / tpr;
  float s[8] = {0}, q[8] = {0};
  if (r0 < rpp) {
    float mu[8], is[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mu[k] = mean[cg * 8 + k];
      is[k] = invstd[cg * 8 + k];
    }
    for (int64_t row = (int64_t)blockIdx.x * rpp + r0; row < M; row += (int64_t)gridDim.x * rpp) {
      const int64_t off = row * C + cg * 8;
      float g[8], xv[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + off), g);
      unpack8(*reinterpret_cast<const uint4*>(x + off), xv);
      if (y) {
        float yv[8];
        unpack8(*reinterpret_cast<const uint4*>(y + off), yv);
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += g[k];
        q[k] += g[k] * (xv[k] - mu[k]) * is[k];
      }
    }
  }
  block_channel_reduce(s, q, C, tpr, rpp, partial);
}

void launch_bn_bwd_reduce(const uint16_t* dy, const uint16_t* x, const uint16_t* y,
                          const float* mean, const float* invstd, int64_t M, int C, float* partial,
                          int nblocks, hipStream_t s) {
  bn_bwd_reduce_kernel<<<nblocks, 256, 0, s>>>(dy, x, y, mean, invstd, M, C, partial);
}

__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(
    const float* __restrict__ partial, int nblocks, int64_t M, int C, const float* __restrict__ gamma,
    const float* __restrict__ invstd, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ coef) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  {
    double s = 0.0, q = 0.0;
    for (int b = lane; b < nblocks; b += 64) {
      s += partial[(int64_t)b * 2 * C + c];
      q += partial[(int64_t)b * 2 * C + C + c];
    }
    s = wave_sum(s);
    q = wave_sum(q);
    if (lane != 0) return;
    if (dgamma) dgamma[c] = (float)q;
    if (dbeta) dbeta[c] = (float)s;
    coef[c] = gamma[c] * invstd[c];
    coef[C + c] = (float)(s / (double)M);
    coef[2 * C + c] = (float)(q / (double)M);
  }
}

void launch_bn_bwd_finalize(const float* partial, int nblocks, int64_t M, int C,
                            const float* gamma, const float* invstd, float* dgamma, float* dbeta,
                            float* coef, hipStream_t s) {
  bn_bwd_finalize_kernel<<<(C + 3) / 4, 256, 0, s>>>(partial, nblocks, M, C, gamma, invstd, dgamma, dbeta,
                                           coef);
}

template <bool MASK, bool WRITE_DYM>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, const uint16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ coef,
    uint16_t* __restrict__ dx, uint16_t* __restrict__ dym, int64_t nvec, int C) {
  extern __shared__ __attribute__((aligned(16))) float sc[];  // [5][C]: k1,k2,k3,mean,invstd
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    sc[c] = coef[c];
    sc[C + c] = coef[C + c];
    sc[2 * C + c] = coef[2 * C + c];
    sc[3 * C + c] = mean[c];
    sc[4 * C + c] = invstd[c];
  }
  __syncthreads();
  const int tpr = C / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int cb = (int)(i % tpr) * 8;
    float g[8], xv[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[i], g);
    unpack8(reinterpret_cast<const uint4*>(x)[i], xv);
    if (MASK) {
      float yv[8];
      unpack8(reinterpret_cast<const uint4*>(y)[i], yv);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
      if (WRITE_DYM) reinterpret_cast<uint4*>(dym)[i] = pack8(g);
    }
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = cb + k;
      const float xh = (xv[k] - sc[3 * C + c]) * sc[4 * C + c];
      o[k] = sc[c] * (g[k] - sc[C + c] - xh * sc[2 * C + c]);
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(o);
  }
}

void launch_bn_bwd_apply(const uint16_t* dy, const uint16_t* x, const uint16_t* y,
                         const float* mean, const float* invstd, const float* coef, uint16_t* dx,
                         uint16_t* dy_masked, int64_t M, int C, hipStream_t s) {
  const int64_t nvec = M * C / 8;
  const unsigned g = stream_grid(nvec, 256, 2048);
  const size_t sm = 5 * C * sizeof(float);
  if (y) {
    if (dy_masked)
      bn_bwd_apply_kernel<true, true><<<g, 256, sm, s>>>(dy, x, y, mean, invstd, coef, dx, dy_masked, nvec, C);
    else
      bn_bwd_apply_kernel<true, false><<<g, 256, sm, s>>>(dy, x, y, mean, invstd, coef, dx, dy_masked, nvec, C);
  } else {
    bn_bwd_apply_kernel<false, false><<<g, 256, sm, s>>>(dy, x, y, mean, invstd, coef, dx, dy_masked, nvec, C);
  }
}

}  // namespace mfl
