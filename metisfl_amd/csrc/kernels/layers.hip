// Kernels for the reference's Keras-style example models (CifarCNN,
// FashionMNIST FC, HousingMLP: examples/keras/models/*.py) on the static
// executor.  Dense layers run on the MFMA implicit-GEMM conv kernels as
// 1x1 convolutions; this file holds the memory-bound pieces around them:
//   * bias + activation (forward, in place) and its backward with the fused
//     bias-gradient column reduction,
//   * 2x2/2 max pooling forward / backward (NHWC, argmax recomputed),
//   * dropout with a counter-based hash RNG keyed by the device step counter
//     (graph-replay safe, no mask tensor: backward recomputes the mask),
//   * softmax cross-entropy over padded logits and mean-squared error heads
//     (loss / accuracy accumulated on device like the ResNet head).
// All activations bf16, 8 elements (16 B) per thread.
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace mfl {

// ---- bias + activation --------------------------------------------------------
template <int ACT>
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(uint16_t* __restrict__ y,
                                                           const float* __restrict__ bias,
                                                           int64_t nvec, int N) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int c0 = (int)((i * 8) % N);
    float f[8];
    uint4 v = reinterpret_cast<uint4*>(y)[i];
    unpack8(v, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      f[k] += bias[c0 + k];
      if (ACT == 1) f[k] = fmaxf(f[k], 0.f);
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(f);
  }
}

void launch_bias_act_fwd(uint16_t* y, const float* bias, int64_t M, int N, int act, hipStream_t s) {
  const int64_t nvec = M * N / 8;
  const unsigned grid = stream_grid(nvec);
  if (act == 1) bias_act_fwd_kernel<1><<<grid, 256, 0, s>>>(y, bias, nvec, N);
  else bias_act_fwd_kernel<0><<<grid, 256, 0, s>>>(y, bias, nvec, N);
}

// dz = dy * act'(y); dbias[c] += sum_rows dz[:, c].  A block owns a fixed
// group of 8 columns per thread (N/8 threads across, the rest down the rows).
template <int ACT>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(const uint16_t* __restrict__ dy,
                                                           const uint16_t* __restrict__ y,
                                                           uint16_t* __restrict__ dz,
                                                           float* __restrict__ dbias, int64_t M,
                                                           int N) {
  __shared__ float red[256 * 8];
  const int cpr = N / 8;                       // column groups
  const int tpc = blockDim.x / cpr;            // threads per column group (>= 1)
  const int cg = threadIdx.x % cpr, tr = threadIdx.x / cpr;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (tr < tpc) {
    for (int64_t r = (int64_t)blockIdx.x * tpc + tr; r < M; r += (int64_t)gridDim.x * tpc) {
      const int64_t off = r * N + cg * 8;
      float g[8], yy[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + off), g);
      if (ACT == 1) {
        unpack8(*reinterpret_cast<const uint4*>(y + off), yy);
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = yy[k] > 0.f ? g[k] : 0.f;
      }
      const uint4 p = pack8(g);
      *reinterpret_cast<uint4*>(dz + off) = p;
      unpack8(p, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += g[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[threadIdx.x * 8 + k] = s[k];
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += blockDim.x) {
    const int g0 = c / 8, k = c % 8;
    float a = 0.f;
    for (int t = 0; t < tpc; ++t) a += red[(t * cpr + g0) * 8 + k];
    atomicAdd(&dbias[c], a);
  }
}

void launch_bias_act_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dz, float* dbias, int64_t M,
                         int N, int act, hipStream_t s) {
  // N <= 2048 (one 8-column group per thread; checked by the binding)
  const int tpc = 256 / (N / 8);
  unsigned grid = (unsigned)((M + tpc - 1) / tpc);
  if (grid > 1024) grid = 1024;
  if (act == 1) bias_act_bwd_kernel<1><<<grid, 256, 0, s>>>(dy, y, dz, dbias, M, N);
  else bias_act_bwd_kernel<0><<<grid, 256, 0, s>>>(dy, y, dz, dbias, M, N);
}

// ---- 2x2 stride-2 max pooling (NHWC) ------------------------------------------------
__global__ __launch_bounds__(256) void maxpool2_fwd_kernel(const uint16_t* __restrict__ x,
                                                           uint16_t* __restrict__ y, int N, int H,
                                                           int W, int C) {
  const int P = H / 2, Q = W / 2, cv = C / 8;
  const int64_t total = (int64_t)N * P * Q * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % cv);
    int64_t t = i / cv;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float m[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = -INFINITY;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(x + (((int64_t)n * H + 2 * p + dy) * W + 2 * q + dx) * C + c8 * 8), f);
#pragma unroll
        for (int k = 0; k < 8; ++k) m[k] = fmaxf(m[k], f[k]);
      }
    *reinterpret_cast<uint4*>(y + i * 8) = pack8(m);
  }
}

// the gradient goes to the FIRST maximal element of each window (TF / PyTorch
// pick one argmax too)
__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(const uint16_t* __restrict__ dy_,
                                                           const uint16_t* __restrict__ x,
                                                           const uint16_t* __restrict__ y,
                                                           uint16_t* __restrict__ dx_, int N, int H,
                                                           int W, int C) {
  const int P = H / 2, Q = W / 2, cv = C / 8;
  const int64_t total = (int64_t)N * P * Q * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % cv);
    int64_t t = i / cv;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float g[8], m[8];
    unpack8(*reinterpret_cast<const uint4*>(dy_ + i * 8), g);
    unpack8(*reinterpret_cast<const uint4*>(y + i * 8), m);
    bool taken[8] = {false, false, false, false, false, false, false, false};
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int64_t off = (((int64_t)n * H + 2 * p + dy) * W + 2 * q + dx) * C + c8 * 8;
        float f[8], o[8];
        unpack8(*reinterpret_cast<const uint4*>(x + off), f);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const bool hit = !taken[k] && f[k] == m[k];
          o[k] = hit ? g[k] : 0.f;
          taken[k] = taken[k] || hit;
        }
        *reinterpret_cast<uint4*>(dx_ + off) = pack8(o);
      }
  }
}

void launch_maxpool2(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, hipStream_t s) {
  const int64_t total = (int64_t)N * (H / 2) * (W / 2) * (C / 8);
  maxpool2_fwd_kernel<<<stream_grid(total), 256, 0, s>>>(x, y, N, H, W, C);
}
void launch_maxpool2_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* y, uint16_t* dx, int N,
                         int H, int W, int C, hipStream_t s) {
  const int64_t total = (int64_t)N * (H / 2) * (W / 2) * (C / 8);
  maxpool2_bwd_kernel<<<stream_grid(total), 256, 0, s>>>(dy, x, y, dx, N, H, W, C);
}

// ---- dropout ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {  // lowbias32 finaliser
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool keep_elem(uint32_t seed, int step, int64_t idx, uint32_t thresh) {
  return mix32(seed ^ mix32((uint32_t)step * 0x9E3779B9U ^ (uint32_t)idx ^ (uint32_t)(idx >> 32) * 0x85EBCA6BU)) >= thresh;
}

__global__ __launch_bounds__(256) void dropout_kernel(const uint16_t* __restrict__ in,
                                                      uint16_t* __restrict__ out, int64_t nvec,
                                                      uint32_t thresh, float scale, uint32_t seed,
                                                      const int* __restrict__ step) {
  const int st = step ? step[0] : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(in)[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = keep_elem(seed, st, i * 8 + k, thresh) ? f[k] * scale : 0.f;
    reinterpret_cast<uint4*>(out)[i] = pack8(f);
  }
}

// forward and backward apply the SAME mask (same seed, same device step)
void launch_dropout(const uint16_t* in, uint16_t* out, int64_t n, float p, uint32_t seed, const int* step,
                    hipStream_t s) {
  const uint32_t thresh = (uint32_t)((double)p * 4294967296.0 > 4294967295.0 ? 4294967295.0
                                                                              : (double)p * 4294967296.0);
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  dropout_kernel<<<stream_grid(n / 8), 256, 0, s>>>(in, out, n / 8, thresh, scale, seed, step);
}

// ---- loss heads ---------------------------------------------------------------------
// softmax cross-entropy over logits [B][Kp] (first K valid); one wave per
// sample.  dlogits = (softmax - onehot) / B (zero on padded columns);
// stats[0] += loss, stats[1] += correct, stats[2] += 1.
__global__ __launch_bounds__(64) void xent_kernel(const uint16_t* __restrict__ logits,
                                                  const int* __restrict__ labels, int Kp, int K, int B,
                                                  uint16_t* __restrict__ dlogits,
                                                  float* __restrict__ stats, int backward) {
  const int b = blockIdx.x, l = threadIdx.x;
  const uint16_t* z = logits + (int64_t)b * Kp;
  float mx = -INFINITY;
  for (int k = l; k < K; k += 64) mx = fmaxf(mx, bf2f(z[k]));
  mx = wave_max(mx);
  float se = 0.f;
  for (int k = l; k < K; k += 64) se += __expf(bf2f(z[k]) - mx);
  se = wave_sum(se);
  const int y = labels[b];
  // argmax (first max) for accuracy
  int am = K;
  for (int k = l; k < K; k += 64)
    if (bf2f(z[k]) == mx && k < am) am = k;
  for (int off = 32; off > 0; off >>= 1) am = min(am, __shfl_xor(am, off));
  if (backward) {
    for (int k = l; k < Kp; k += 64) {
      float g = 0.f;
      if (k < K) g = (__expf(bf2f(z[k]) - mx) / se - (k == y ? 1.f : 0.f)) / (float)B;
      dlogits[(int64_t)b * Kp + k] = f2bf(g);
    }
  }
  if (l == 0 && y >= 0) {  // y < 0: evaluation padding row
    const float zy = y < K ? bf2f(z[y]) : mx;
    atomicAdd(&stats[0], __logf(se) + mx - zy);
    atomicAdd(&stats[1], am == y ? 1.f : 0.f);
    atomicAdd(&stats[2], 1.f);
  }
}

void launch_xent(const uint16_t* logits, const int* labels, int B, int Kp, int K, uint16_t* dlogits,
                 float* stats, bool backward, hipStream_t s) {
  xent_kernel<<<B, 64, 0, s>>>(logits, labels, Kp, K, B, dlogits, stats, backward ? 1 : 0);
}

// mean squared error on column 0 of pred [B][Kp]; targets are fp32 (stored
// in the int32 label slots); dpred = 2 (pred - t) / B; stats[0] += se,
// stats[2] += 1 (stats[1] unused).
__global__ __launch_bounds__(256) void mse_kernel(const uint16_t* __restrict__ pred,
                                                  const float* __restrict__ target, int B, int Kp,
                                                  uint16_t* __restrict__ dpred, float* __restrict__ stats,
                                                  int backward) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  float se = 0.f, cnt = 0.f;
  // a NaN target (the int32 -1 label of an evaluation padding row) is skipped
  if (b < B && !__builtin_isnan(target[b])) {
    const float d = bf2f(pred[(int64_t)b * Kp]) - target[b];
    se = d * d;
    cnt = 1.f;
    if (backward)
      for (int k = 0; k < Kp; ++k) dpred[(int64_t)b * Kp + k] = f2bf(k == 0 ? 2.f * d / (float)B : 0.f);
  }
  se = wave_sum(se);
  cnt = wave_sum(cnt);
  if ((threadIdx.x & 63) == 0 && cnt > 0.f) {
    atomicAdd(&stats[0], se);
    atomicAdd(&stats[2], cnt);
  }
}

void launch_mse(const uint16_t* pred, const float* target, int B, int Kp, uint16_t* dpred, float* stats,
                bool backward, hipStream_t s) {
  mse_kernel<<<(B + 255) / 256, 256, 0, s>>>(pred, target, B, Kp, dpred, stats, backward ? 1 : 0);
}

}  // namespace mfl
