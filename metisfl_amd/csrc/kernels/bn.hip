// K12: BatchNorm forward/backward for NHWC bf16 activations.
//
// The reference only reaches BatchNorm through Keras layers
// (examples/keras/models/cifar_cnn.py:27,32); here it is a first-class
// hand-written kernel family, because ResNet-18 runs 20 of them per step.
//
// Launch-count design (a graph node costs ~4 us on this chip regardless of
// work, so a BN that is "stats -> finalize -> apply" is mostly overhead):
//  * per-channel sums (sum x, sum x^2) are accumulated with fp64 atomics
//    into a small [2][C] buffer -- by the producing conv's epilogue
//    (kernels/conv.hip) in the training step, or by bn_stats here;
//  * the apply kernel derives mean / inv-std / scale / shift from those sums
//    in its prologue (C <= 2048 values per block) and block 0 publishes the
//    saved mean / inv-std and updates the running statistics: no finalize
//    launch;
//  * backward: one reduce (fp64 atomics) + one apply that also forms
//    dgamma / dbeta and optionally the masked dy for a residual shortcut.
// The accumulators are zeroed by the fused optimizer launch at the end of the
// step (kernels/optim.hip), so zeroing costs no launch either.
//
// Layout: x is [M, C] with M = N*H*W rows and C contiguous channels (NHWC);
// each lane owns 8 consecutive channels (one 16-B load).
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

// Reduce the per-thread [8] accumulators a0/a1 over the rows of the block
// and add them into acc[0|1][C] (fp64 atomics).
__device__ __forceinline__ void block_channel_atomic(const float* a0, const float* a1, int C,
                                                     int tpr, int rpp, double* acc) {
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
    atomicAdd(&acc[c], (double)s0);
    atomicAdd(&acc[C + c], (double)s1);
  }
}

__global__ __launch_bounds__(256) void bn_stats_kernel(const uint16_t* __restrict__ x, int64_t M,
                                                       int C, double* __restrict__ acc) {
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
  block_channel_atomic(s, q, C, tpr, rpp, acc);
}

void launch_bn_stats(const uint16_t* x, int64_t M, int C, double* acc, hipStream_t s) {
  bn_stats_kernel<<<bn_stats_blocks(M, C), 256, 0, s>>>(x, M, C, acc);
}

// ---------------------------------------------------------------------------
// Forward apply: y = relu?(x * scale + shift (+ residual)).
// train: statistics from acc (sum, sumsq over M rows); else from running stats.
template <bool RES, bool RELU>
__device__ __forceinline__ void bn_apply_body(const BnFwdArgs& a, int64_t nvec, int bx, int gx,
                                              float* coef /* [2][C] LDS */) {
  const int C = a.C;
  const uint4* X = reinterpret_cast<const uint4*>(a.x);
  const uint4* R = reinterpret_cast<const uint4*>(a.residual);
  // The first vectors go out before the per-channel prologue: its acc loads
  // and fp64 math then overlap the activation loads instead of preceding them
  // (at ResNet-18 sizes every thread handles one or two vectors).
  const int64_t stride = (int64_t)gx * blockDim.x;
  int64_t i = (int64_t)bx * blockDim.x + threadIdx.x;
  uint4 xv = {0, 0, 0, 0}, rv = {0, 0, 0, 0};
  if (i < nvec) {
    xv = X[i];
    if (RES) rv = R[i];
  }
  const double inv_m = 1.0 / (double)a.M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double mu, var;
    if (a.train) {
      mu = a.acc[c] * inv_m;
      var = a.acc[C + c] * inv_m - mu * mu;
      if (var < 0.0) var = 0.0;
    } else {
      mu = a.run_mean[c];
      var = a.run_var[c];
    }
    const float is = (float)(1.0 / sqrt(var + (double)a.eps));
    const float g = a.gamma[c];
    const float sc = g * is;
    coef[c] = sc;
    coef[C + c] = a.beta[c] - (float)mu * sc;
    if (a.train && bx == 0) {
      a.mean[c] = (float)mu;
      a.invstd[c] = is;
      if (a.run_mean) {
        const double unb = a.M > 1 ? var * (double)a.M / (double)(a.M - 1) : var;
        a.run_mean[c] = (1.f - a.momentum) * a.run_mean[c] + a.momentum * (float)mu;
        a.run_var[c] = (1.f - a.momentum) * a.run_var[c] + a.momentum * (float)unb;
      }
    }
  }
  __syncthreads();
  const int tpr = C / 8;
  for (; i < nvec; i += stride) {
    const uint4 xc = xv, rc = rv;
    if (i + stride < nvec) {  // one vector of prefetch
      xv = X[i + stride];
      if (RES) rv = R[i + stride];
    }
    const int cg = (int)(i % tpr);
    float f[8];
    unpack8(xc, f);
    float r[8];
    if (RES) unpack8(rc, r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = f[k] * coef[cg * 8 + k] + coef[C + cg * 8 + k];
      if (RES) v += r[k];
      if (RELU) v = fmaxf(v, 0.f);
      f[k] = v;
    }
    reinterpret_cast<uint4*>(a.y)[i] = pack8(f);
  }
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void bn_apply_kernel(BnFwdArgs a, int64_t nvec) {
  extern __shared__ __attribute__((aligned(16))) float coef[];  // [2][C]
  bn_apply_body<RES, RELU>(a, nvec, blockIdx.x, gridDim.x, coef);
}

// A downsampling block's two BatchNorms (projection shortcut: no ReLU; conv1:
// ReLU; neither with a residual) in one launch: blocks [0, g1) apply a1.
__global__ __launch_bounds__(256) void bn_apply_pair_kernel(BnFwdArgs a1, int64_t n1, int g1, BnFwdArgs a2,
                                                            int64_t n2) {
  extern __shared__ __attribute__((aligned(16))) float coef[];  // [2][max C]
  if ((int)blockIdx.x < g1) bn_apply_body<false, false>(a1, n1, blockIdx.x, g1, coef);
  else bn_apply_body<false, true>(a2, n2, blockIdx.x - g1, gridDim.x - g1, coef);
}

void launch_bn_apply_pair(const BnFwdArgs& a1, const BnFwdArgs& a2, hipStream_t s) {
  const int64_t n1 = a1.M * a1.C / 8, n2 = a2.M * a2.C / 8;
  const unsigned g1 = stream_grid(n1, 256, 512), g2 = stream_grid(n2, 256, 512);
  const size_t sm = 2 * (size_t)(a1.C > a2.C ? a1.C : a2.C) * sizeof(float);
  bn_apply_pair_kernel<<<g1 + g2, 256, sm, s>>>(a1, n1, (int)g1, a2, n2);
}

void launch_bn_apply(const BnFwdArgs& a, hipStream_t s) {
  const int64_t nvec = a.M * a.C / 8;
  const unsigned g = stream_grid(nvec, 256, 512);  // see bn32.hip apply_grid
  const size_t sm = 2 * a.C * sizeof(float);
  if (a.residual) {
    if (a.relu) bn_apply_kernel<true, true><<<g, 256, sm, s>>>(a, nvec);
    else bn_apply_kernel<true, false><<<g, 256, sm, s>>>(a, nvec);
  } else {
    if (a.relu) bn_apply_kernel<false, true><<<g, 256, sm, s>>>(a, nvec);
    else bn_apply_kernel<false, false><<<g, 256, sm, s>>>(a, nvec);
  }
}

// ---------------------------------------------------------------------------
// Backward reduce: acc_b[c] += sum dyr, acc_b[C+c] += sum dyr * xhat, where
// dyr = dy masked by (y > 0) when y is given (fused ReLU backward).
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, const uint16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ invstd, int64_t M, int C,
    double* __restrict__ acc) {
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
  block_channel_atomic(s, q, C, tpr, rpp, acc);
}

void launch_bn_bwd_reduce(const uint16_t* dy, const uint16_t* x, const uint16_t* y,
                          const float* mean, const float* invstd, int64_t M, int C, double* acc,
                          hipStream_t s) {
  bn_bwd_reduce_kernel<<<bn_stats_blocks(M, C), 256, 0, s>>>(dy, x, y, mean, invstd, M, C, acc);
}

// Backward apply: dx = gamma*invstd*(dyr - mean(dyr) - xhat*mean(dyr*xhat)).
template <bool MASK, bool WRITE_DYM>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BnBwdArgs a, int64_t nvec) {
  extern __shared__ __attribute__((aligned(16))) float sc[];  // [5][C]: k1,k2,k3,mean,invstd
  const int C = a.C;
  const uint4* DY = reinterpret_cast<const uint4*>(a.dy);
  const uint4* X = reinterpret_cast<const uint4*>(a.x);
  const uint4* Y = reinterpret_cast<const uint4*>(a.y);
  // first vectors in flight across the prologue (see bn_apply_kernel)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4 gv = {0, 0, 0, 0}, xv = {0, 0, 0, 0}, yv = {0, 0, 0, 0};
  if (i < nvec) {
    gv = DY[i];
    xv = X[i];
    if (MASK) yv = Y[i];
  }
  const double inv_m = 1.0 / (double)a.M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const double s = a.acc[c], q = a.acc[C + c];
    sc[c] = a.gamma[c] * a.invstd[c];
    sc[C + c] = (float)(s * inv_m);
    sc[2 * C + c] = (float)(q * inv_m);
    sc[3 * C + c] = a.mean[c];
    sc[4 * C + c] = a.invstd[c];
    if (blockIdx.x == 0) {
      if (a.dgamma) a.dgamma[c] = (float)q;
      if (a.dbeta) a.dbeta[c] = (float)s;
    }
  }
  __syncthreads();
  const int tpr = C / 8;
  for (; i < nvec; i += stride) {
    const uint4 gc = gv, xc = xv, yc = yv;
    if (i + stride < nvec) {
      gv = DY[i + stride];
      xv = X[i + stride];
      if (MASK) yv = Y[i + stride];
    }
    const int cb = (int)(i % tpr) * 8;
    float g[8], xf[8];
    unpack8(gc, g);
    unpack8(xc, xf);
    if (MASK) {
      float yf[8];
      unpack8(yc, yf);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = yf[k] > 0.f ? g[k] : 0.f;
    }
    // !MASK: dy arrives masked (its producing dgrad applied the mask)
    if (WRITE_DYM) reinterpret_cast<uint4*>(a.dy_masked)[i] = pack8(g);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = cb + k;
      const float xh = (xf[k] - sc[3 * C + c]) * sc[4 * C + c];
      o[k] = sc[c] * (g[k] - sc[C + c] - xh * sc[2 * C + c]);
    }
    reinterpret_cast<uint4*>(a.dx)[i] = pack8(o);
  }
}

void launch_bn_bwd_apply(const BnBwdArgs& a, hipStream_t s) {
  const int64_t nvec = a.M * a.C / 8;
  const unsigned g = stream_grid(nvec, 256, 512);  // see bn32.hip apply_grid
  const size_t sm = 5 * a.C * sizeof(float);
  if (a.y) {
    if (a.dy_masked) bn_bwd_apply_kernel<true, true><<<g, 256, sm, s>>>(a, nvec);
    else bn_bwd_apply_kernel<true, false><<<g, 256, sm, s>>>(a, nvec);
  } else {
    if (a.dy_masked) bn_bwd_apply_kernel<false, true><<<g, 256, sm, s>>>(a, nvec);
    else bn_bwd_apply_kernel<false, false><<<g, 256, sm, s>>>(a, nvec);
  }
}

}  // namespace mfl
