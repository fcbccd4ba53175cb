// K14 (+K15 pooling): fused classifier head, forward AND backward.
//
// Global-average-pool -> Linear(C->K) -> softmax cross-entropy -> dlogits ->
// dfeat -> d(pool input) for one sample per workgroup, in ONE launch; a second
// tiny launch forms dW/db.  This replaces the Keras
// SparseCategoricalCrossentropy + Dense + pooling chain the reference trains
// through (examples/keras/models/cifar_cnn.py:35-50).  Loss sum, correct
// count and sample count are accumulated on device (stats[0..2]) so the
// training loop never synchronises with the host per step.
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace mfl {

__global__ __launch_bounds__(256) void head_kernel(const uint16_t* __restrict__ x, int HW, int C,
                                                   const float* __restrict__ W,
                                                   const float* __restrict__ bias, int K,
                                                   const int* __restrict__ labels,
                                                   float* __restrict__ feat, float* __restrict__ dlog,
                                                   uint16_t* __restrict__ dx,
                                                   float* __restrict__ stats, int B, int backward) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // feat[C] | logits[K]
  float* f = sm;
  float* lg = sm + C;
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const float inv_hw = 1.f / (float)HW;
  const uint16_t* xb = x + (int64_t)b * HW * C;
  for (int c = t; c < C; c += 256) {
    float s = 0.f;
    for (int h = 0; h < HW; ++h) s += bf2f(xb[(int64_t)h * C + c]);
    s *= inv_hw;
    f[c] = s;
    if (feat) feat[(int64_t)b * C + c] = s;
  }
  __syncthreads();
  for (int k = wv; k < K; k += 4) {
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += f[c] * W[(int64_t)k * C + c];
    s = wave_sum(s);
    if (lane == 0) lg[k] = s + (bias ? bias[k] : 0.f);
  }
  __syncthreads();
  if (wv == 0) {
    float mx = -INFINITY;
    for (int k = lane; k < K; k += 64) mx = fmaxf(mx, lg[k]);
    mx = wave_max(mx);
    float se = 0.f;
    for (int k = lane; k < K; k += 64) se += __expf(lg[k] - mx);
    se = wave_sum(se);
    const int y = labels[b];
    // argmax (first max wins)
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int k = lane; k < K; k += 64) {
      if (lg[k] > best) { best = lg[k]; bi = k; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    const float lse = mx + __logf(se);
    if (lane == 0 && stats) {
      atomicAdd(&stats[0], lse - lg[y]);
      atomicAdd(&stats[1], bi == y ? 1.f : 0.f);
      atomicAdd(&stats[2], 1.f);
    }
    if (backward) {
      const float invB = 1.f / (float)B;
      for (int k = lane; k < K; k += 64) {
        const float p = __expf(lg[k] - lse);
        const float d = (p - (k == y ? 1.f : 0.f)) * invB;
        lg[k] = d;
        dlog[(int64_t)b * K + k] = d;
      }
    }
  }
  if (!backward) return;
  __syncthreads();
  uint16_t* dxb = dx + (int64_t)b * HW * C;
  for (int c = t; c < C; c += 256) {
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += lg[k] * W[(int64_t)k * C + c];
    const uint16_t v = f2bf(s * inv_hw);
    for (int h = 0; h < HW; ++h) dxb[(int64_t)h * C + c] = v;
  }
}

void launch_head_fwd_bwd(const uint16_t* x, int B, int HW, int C, const float* W, const float* bias,
                         int K, const int* labels, float* feat, float* dlogits, uint16_t* dx,
                         float* stats, bool backward, hipStream_t s) {
  const size_t sm = (size_t)(C + K) * sizeof(float);
  head_kernel<<<B, 256, sm, s>>>(x, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, B,
                                 backward ? 1 : 0);
}

__global__ __launch_bounds__(256) void head_wgrad_kernel(const float* __restrict__ feat,
                                                         const float* __restrict__ dlog, int B, int C,
                                                         int K, float* __restrict__ dW,
                                                         float* __restrict__ db) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (int64_t)K * C) {
    const int k = (int)(i / C), c = (int)(i % C);
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dlog[(int64_t)b * K + k] * feat[(int64_t)b * C + c];
    dW[i] = s;
  }
  if (db && i < K) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dlog[(int64_t)b * K + i];
    db[i] = s;
  }
}

void launch_head_wgrad(const float* feat, const float* dlogits, int B, int C, int K, float* dW,
                       float* db, hipStream_t s) {
  const int64_t n = (int64_t)K * C;
  head_wgrad_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(feat, dlogits, B, C, K, dW, db);
}

}  // namespace mfl
