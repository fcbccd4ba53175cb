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

// One sample per workgroup.  Pooling and the dx broadcast move 8 channels
// (16 B) per lane: thread t owns channel group t % G (G = C / 8) and pixel rows
// t / G, t / G + R, ... (R = 256 / G row groups), partial sums meet in LDS.
// With dW != nullptr the weight / bias gradient is fused too: the sample's
// dlogits x feat outer product is added with fp32 atomics (B adders per
// address; dW / db must be zero on entry -- the training step's gradient
// buffer is) and head_wgrad_kernel is not launched.
// Activations arrive as bf16 (mixed-precision path) or fp32 (reference-
// precision path); 8 channels per lane either way.
__device__ __forceinline__ void load8(const uint16_t* p, float* v) { unpack8(*reinterpret_cast<const uint4*>(p), v); }
__device__ __forceinline__ void load8(const float* p, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
struct Pack8 {
  uint4 h;
  float4 a, b;
};
__device__ __forceinline__ void pack_out(const float* v, uint16_t*, Pack8& p) { p.h = pack8(v); }
__device__ __forceinline__ void pack_out(const float* v, float*, Pack8& p) {
  p.a = make_float4(v[0], v[1], v[2], v[3]);
  p.b = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void store8(uint16_t* d, const Pack8& p) { *reinterpret_cast<uint4*>(d) = p.h; }
__device__ __forceinline__ void store8(float* d, const Pack8& p) {
  reinterpret_cast<float4*>(d)[0] = p.a;
  reinterpret_cast<float4*>(d)[1] = p.b;
}

// softmax transcendentals: the fast forms for the bf16 path, full-precision
// libm for the fp32 (reference-precision) path -- only K per sample
template <typename T>
__device__ __forceinline__ float hexp(float x) { return sizeof(T) == 4 ? expf(x) : __expf(x); }
template <typename T>
__device__ __forceinline__ float hlog(float x) { return sizeof(T) == 4 ? logf(x) : __logf(x); }

template <typename T>
__global__ __launch_bounds__(256) void head_kernel(const T* __restrict__ x, int HW, int C,
                                                   const float* __restrict__ W,
                                                   const float* __restrict__ bias, int K,
                                                   const int* __restrict__ labels,
                                                   float* __restrict__ feat, float* __restrict__ dlog,
                                                   T* __restrict__ dx,
                                                   float* __restrict__ stats, int B, int backward,
                                                   float* __restrict__ dW, float* __restrict__ db) {
  // feat[C] | logits[K] | partials[R][C] | W[K][C]
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* f = sm;
  float* lg = sm + C;
  const int G = C >> 3;
  const int R = max(1, 256 / G);
  float* part = sm + C + ((K + 3) & ~3);
  float* Ws = part + R * C;
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & 63, wv = t >> 6;
  const float inv_hw = 1.f / (float)HW;
  const T* xb = x + (int64_t)b * HW * C;
  const int cg = t % G, rg = t / G;
  // the classifier weights go to LDS alongside the pooling loads: the logits
  // and the dx broadcast then read LDS instead of paying two more dependent
  // global round trips in this one-workgroup-per-sample serial chain
  {
    const int n4 = K * C / 4;
    const float4* W4 = reinterpret_cast<const float4*>(W);
    float4* Ws4 = reinterpret_cast<float4*>(Ws);
#pragma unroll 4
    for (int i = t; i < n4; i += 256) Ws4[i] = W4[i];
  }
  if (rg < R) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int h = rg; h < HW; h += R) {
      float v[8];
      load8(xb + (int64_t)h * C + 8 * cg, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += v[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) part[rg * C + 8 * cg + k] = s[k];
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float s = 0.f;
    for (int r = 0; r < R; ++r) s += part[r * C + c];
    s *= inv_hw;
    f[c] = s;
    if (feat) feat[(int64_t)b * C + c] = s;
  }
  __syncthreads();
  for (int k = wv; k < K; k += 4) {
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += f[c] * Ws[k * C + c];
    s = wave_sum(s);
    if (lane == 0) lg[k] = s + (bias ? bias[k] : 0.f);
  }
  __syncthreads();
  if (wv == 0) {
    float mx = -INFINITY;
    for (int k = lane; k < K; k += 64) mx = fmaxf(mx, lg[k]);
    mx = wave_max(mx);
    float se = 0.f;
    for (int k = lane; k < K; k += 64) se += hexp<T>(lg[k] - mx);
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
    const float lse = mx + hlog<T>(se);
    // y < 0: a padding row of the last evaluation batch (DeviceDataset
    // pad_tail) -- excluded from the statistics
    if (lane == 0 && stats && y >= 0) {
      atomicAdd(&stats[0], lse - lg[y]);
      atomicAdd(&stats[1], bi == y ? 1.f : 0.f);
      atomicAdd(&stats[2], 1.f);
    }
    if (backward) {
      const float invB = 1.f / (float)B;
      for (int k = lane; k < K; k += 64) {
        const float p = hexp<T>(lg[k] - lse);
        const float d = (p - (k == y ? 1.f : 0.f)) * invB;
        lg[k] = d;
        dlog[(int64_t)b * K + k] = d;
        if (db) atomicAdd(&db[k], d);
      }
    }
  }
  if (!backward) return;
  __syncthreads();
  if (dW) {
    for (int i = t; i < K * C; i += 256) {
      const int k = i / C, c = i - k * C;
      atomicAdd(&dW[i], lg[k] * f[c]);
    }
  }
  if (rg < R) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float s = 0.f;
      for (int k = 0; k < K; ++k) s += lg[k] * Ws[k * C + 8 * cg + e];
      v[e] = s * inv_hw;
    }
    Pack8 pk;
    T* dxb = dx + (int64_t)b * HW * C + 8 * cg;
    pack_out(v, dxb, pk);
    for (int h = rg; h < HW; h += R) store8(dxb + (int64_t)h * C, pk);
  }
}

template <typename T>
static void head_launch(const T* x, int B, int HW, int C, const float* W, const float* bias, int K,
                        const int* labels, float* feat, float* dlogits, T* dx, float* stats, bool backward,
                        hipStream_t s, float* dW, float* db) {
  const int G = C / 8, R = G >= 256 ? 1 : 256 / G;
  const size_t sm = (size_t)(C + ((K + 3) & ~3) + (size_t)R * C + (size_t)K * C) * sizeof(float);
  static bool attr = false;
  if (!attr && sm > 65536) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&head_kernel<T>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    attr = true;
  }
  head_kernel<T><<<B, 256, sm, s>>>(x, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, B, backward ? 1 : 0,
                                    backward ? dW : nullptr, backward ? db : nullptr);
}

void launch_head_fwd_bwd(const uint16_t* x, int B, int HW, int C, const float* W, const float* bias,
                         int K, const int* labels, float* feat, float* dlogits, uint16_t* dx,
                         float* stats, bool backward, hipStream_t s, float* dW, float* db) {
  head_launch(x, B, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, backward, s, dW, db);
}
void launch_head32_fwd_bwd(const float* x, int B, int HW, int C, const float* W, const float* bias, int K,
                           const int* labels, float* feat, float* dlogits, float* dx, float* stats, bool backward,
                           hipStream_t s, float* dW, float* db) {
  head_launch(x, B, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, backward, s, dW, db);
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
