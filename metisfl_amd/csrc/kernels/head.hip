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
#include "kernels/bn_coef.h"
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

// FUSE: the input is relu(BN(z) + res) (HeadBn; z / res / y in the model's
// activation type T), applied as the pooling loop reads it; the coefficients
// are derived per workgroup with bn32_apply's math (bn_coef.h), workgroup 0
// publishes them.  bf16: the pooled value is the stored (rounded) y.
template <typename T, bool FUSE = false>
__global__ __launch_bounds__(256) void head_kernel(const T* __restrict__ x, int HW, int C,
                                                   const float* __restrict__ W,
                                                   const float* __restrict__ bias, int K,
                                                   const int* __restrict__ labels,
                                                   float* __restrict__ feat, float* __restrict__ dlog,
                                                   T* __restrict__ dx,
                                                   float* __restrict__ stats, int B, int backward,
                                                   float* __restrict__ dW, float* __restrict__ db, HeadBn hb) {
  // feat[C] | logits[K] | partials[R][C] | W[K][C] | FUSE: sc, sh, mean, invstd [4][C]
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* f = sm;
  float* lg = sm + C;
  const int G = C >> 3;
  const int R = max(1, 256 / G);
  float* part = sm + C + ((K + 3) & ~3);
  float* Ws = part + R * C;
  float* bc = Ws + K * C;
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
  if constexpr (FUSE) {
    for (int c = t; c < C; c += 256) {
      float sc, sh, mu, isd;
      bn_fwd_coef(hb.acc, hb.reps, C, c, (int64_t)B * HW, hb.train != 0, b == 0, hb.gamma, hb.beta, hb.mean,
                  hb.invstd, hb.run_mean, hb.run_var, hb.momentum, hb.eps, sc, sh, &mu, &isd);
      bc[c] = sc;
      bc[C + c] = sh;
      bc[2 * C + c] = mu;
      bc[3 * C + c] = isd;
    }
    __syncthreads();
  }
  if (rg < R) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int h = rg; h < HW; h += R) {
      float v[8];
      if constexpr (FUSE) {
        // bn32_apply's element math: fmaf(z, sc, sh) + res, then ReLU
        const int64_t o = ((int64_t)b * HW + h) * C + 8 * cg;
        float zz[8], rr[8];
        load8(reinterpret_cast<const T*>(hb.z) + o, zz);
        load8(reinterpret_cast<const T*>(hb.res) + o, rr);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = fmaxf(fmaf(zz[k], bc[8 * cg + k], bc[C + 8 * cg + k]) + rr[k], 0.f);
        T* yo = reinterpret_cast<T*>(hb.y) + o;
        Pack8 pk;
        pack_out(v, yo, pk);
        store8(yo, pk);
        if constexpr (sizeof(T) == 2) unpack8(pk.h, v);
      } else {
        load8(xb + (int64_t)h * C + 8 * cg, v);
      }
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
  float gs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, gq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
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
    if constexpr (FUSE) {
      if (hb.acc_b) {
        // the last block's BN-backward sums of dx (bn32_bwd_reduce's math):
        // g = dx * [y > 0], sum g and sum g * (z - mean) * invstd per channel
        for (int h = rg; h < HW; h += R) {
          const int64_t o = ((int64_t)b * HW + h) * C + 8 * cg;
          float yy[8], zz[8];
          load8(reinterpret_cast<const T*>(hb.y) + o, yy);
          load8(reinterpret_cast<const T*>(hb.z) + o, zz);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int c = 8 * cg + k;
            const float g = yy[k] > 0.f ? v[k] : 0.f;
            gs[k] += g;
            gq[k] += g * ((zz[k] - bc[2 * C + c]) * bc[3 * C + c]);
          }
        }
      }
    }
  }
  if constexpr (FUSE) {
    if (hb.acc_b) {  // block-uniform: partials meet in LDS, one fp64 atomic per channel
      for (int pass = 0; pass < 2; ++pass) {
        if (rg < R) {
#pragma unroll
          for (int k = 0; k < 8; ++k) part[rg * C + 8 * cg + k] = pass ? gq[k] : gs[k];
        }
        __syncthreads();
        for (int c = t; c < C; c += 256) {
          double a = 0.0;
          for (int r = 0; r < R; ++r) a += part[r * C + c];
          atomicAdd(&hb.acc_b[(int64_t)(b % hb.reps_b) * 2 * C + pass * C + c], a);
        }
        __syncthreads();
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Split head (the fused-BN path, C % 128 == 0): the one-sample-per-workgroup
// kernel above is a serial chain of ~8 dependent phases on 32 of the 256 CUs
// (24.7 us at batch 32, ~2.4 % of the fp32 step).  Here a workgroup owns one
// sample's 128-channel group (B x C/128 workgroups) and the chain is cut in
// two launches: (A) BN coefficients, relu(BN(z) + res) -> y, pooling, and
// the group's partial logits; (B) logits (partials summed in a fixed order,
// so every group of a sample computes identical values), softmax / loss,
// dlogits, dW / db, dx and the BN-backward sums of dx -- each group for its
// own channels.
constexpr int kHeadCW = 128;  // channels per workgroup (16 lane groups x 8)
constexpr int kHeadMaxPix = 4;  // pixel rows per thread kept in registers (HW <= 64)

template <typename T>
__global__ __launch_bounds__(256) void head_split_fwd_kernel(int HW, int C, const float* __restrict__ W, int K,
                                                             float* __restrict__ feat, float* __restrict__ lpart,
                                                             int B, HeadBn hb) {
  __shared__ float sc[kHeadCW], sh[kHeadCW], f[kHeadCW];
  __shared__ float part[16 * kHeadCW];
  const int CG = C / kHeadCW;
  const int b = blockIdx.x / CG, cg = blockIdx.x - b * CG, c0 = cg * kHeadCW;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int lgp = t & 15, rg = t >> 4;  // 8-channel lane group, pixel row group
  // the activation loads go out before the coefficients' fp64 sums
  float zz[kHeadMaxPix][8], rr[kHeadMaxPix][8];
#pragma unroll
  for (int j = 0; j < kHeadMaxPix; ++j) {
    const int h = rg + 16 * j;
    if (h < HW) {
      const int64_t o = ((int64_t)b * HW + h) * C + c0 + 8 * lgp;
      load8(reinterpret_cast<const T*>(hb.z) + o, zz[j]);
      load8(reinterpret_cast<const T*>(hb.res) + o, rr[j]);
    }
  }
  if (t < kHeadCW) {
    float a, bb;
    bn_fwd_coef(hb.acc, hb.reps, C, c0 + t, (int64_t)B * HW, hb.train != 0, b == 0, hb.gamma, hb.beta, hb.mean,
                hb.invstd, hb.run_mean, hb.run_var, hb.momentum, hb.eps, a, bb);
    sc[t] = a;
    sh[t] = bb;
  }
  __syncthreads();
  float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < kHeadMaxPix; ++j) {
    const int h = rg + 16 * j;
    if (h >= HW) break;
    const int64_t o = ((int64_t)b * HW + h) * C + c0 + 8 * lgp;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fmaxf(fmaf(zz[j][k], sc[8 * lgp + k], sh[8 * lgp + k]) + rr[j][k], 0.f);
    T* yo = reinterpret_cast<T*>(hb.y) + o;
    Pack8 pk;
    pack_out(v, yo, pk);
    store8(yo, pk);
    if constexpr (sizeof(T) == 2) unpack8(pk.h, v);  // bf16: the pooled value is the stored y
#pragma unroll
    for (int k = 0; k < 8; ++k) s8[k] += v[k];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) part[rg * kHeadCW + 8 * lgp + k] = s8[k];
  __syncthreads();
  if (t < kHeadCW) {
    float a = 0.f;
    for (int r = 0; r < 16; ++r) a += part[r * kHeadCW + t];
    a *= 1.f / (float)HW;
    f[t] = a;
    feat[(int64_t)b * C + c0 + t] = a;
  }
  __syncthreads();
  for (int k = wv; k < K; k += 4) {
    const float* wr = W + (int64_t)k * C + c0;
    float a = f[lane] * wr[lane] + f[lane + 64] * wr[lane + 64];
    a = wave_sum(a);
    if (lane == 0) lpart[((int64_t)b * CG + cg) * K + k] = a;
  }
}

// Every load that does not depend on the logits (the group's W slice into
// LDS, feat, this thread's y / z pixels, mean / invstd) is issued before the
// partial logits are summed, so their latency overlaps the softmax instead
// of following it (the first version, loading them after, ran 16 us).
template <typename T>
__global__ __launch_bounds__(256) void head_split_bwd_kernel(int HW, int C, const float* __restrict__ W,
                                                             const float* __restrict__ bias, int K,
                                                             const int* __restrict__ labels,
                                                             const float* __restrict__ feat,
                                                             const float* __restrict__ lpart,
                                                             float* __restrict__ dlog, T* __restrict__ dx,
                                                             float* __restrict__ stats, int B, int backward,
                                                             float* __restrict__ dW, float* __restrict__ db,
                                                             HeadBn hb) {
  extern __shared__ __attribute__((aligned(16))) float dyn[];  // lg[K] | Ws[K][128]
  float* lg = dyn;
  float* Ws = dyn + ((K + 3) & ~3);
  __shared__ float part[2][16 * kHeadCW];
  const int CG = C / kHeadCW;
  const int b = blockIdx.x / CG, cg = blockIdx.x - b * CG, c0 = cg * kHeadCW;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int lgp = t & 15, rg = t >> 4;
  const bool sums = backward && hb.acc_b;
  // independent loads first
  float yy[kHeadMaxPix][8], zz[kHeadMaxPix][8], mu[8], isd[8];
  float fc = 0.f;
  if (backward) {
    for (int i = t; i < K * kHeadCW; i += 256) {
      const int k = i / kHeadCW, c = i - k * kHeadCW;
      Ws[i] = W[(int64_t)k * C + c0 + c];
    }
    if (t < kHeadCW) fc = feat[(int64_t)b * C + c0 + t];
    if (sums) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        mu[k] = hb.mean[c0 + 8 * lgp + k];
        isd[k] = hb.invstd[c0 + 8 * lgp + k];
      }
#pragma unroll
      for (int j = 0; j < kHeadMaxPix; ++j) {
        const int h = rg + 16 * j;
        if (h < HW) {
          const int64_t o = ((int64_t)b * HW + h) * C + c0 + 8 * lgp;
          load8(reinterpret_cast<const T*>(hb.y) + o, yy[j]);
          load8(reinterpret_cast<const T*>(hb.z) + o, zz[j]);
        }
      }
    }
  }
  for (int k = t; k < K; k += 256) {
    float a = bias ? bias[k] : 0.f;
    for (int g = 0; g < CG; ++g) a += lpart[((int64_t)b * CG + g) * K + k];
    lg[k] = a;
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
    if (lane == 0 && cg == 0 && stats && y >= 0) {
      atomicAdd(&stats[0], lse - lg[y]);
      atomicAdd(&stats[1], bi == y ? 1.f : 0.f);
      atomicAdd(&stats[2], 1.f);
    }
    if (backward) {
      const float invB = 1.f / (float)B;
      for (int k = lane; k < K; k += 64) {  // each lane reads and writes only its own k
        const float d = (hexp<T>(lg[k] - lse) - (k == y ? 1.f : 0.f)) * invB;
        lg[k] = d;
        if (cg == 0) {
          dlog[(int64_t)b * K + k] = d;
          if (db) atomicAdd(&db[k], d);
        }
      }
    }
  }
  if (!backward) return;
  __syncthreads();
  if (dW && t < kHeadCW) {
    for (int k = 0; k < K; ++k) atomicAdd(&dW[(int64_t)k * C + c0 + t], lg[k] * fc);
  }
  const float inv_hw = 1.f / (float)HW;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float a = 0.f;
    for (int k = 0; k < K; ++k) a += lg[k] * Ws[k * kHeadCW + 8 * lgp + e];
    v[e] = a * inv_hw;
  }
  Pack8 pk;
  T* dxb = dx + (int64_t)b * HW * C + c0 + 8 * lgp;
  pack_out(v, dxb, pk);
  float gs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, gq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < kHeadMaxPix; ++j) {
    const int h = rg + 16 * j;
    if (h >= HW) break;
    store8(dxb + (int64_t)h * C, pk);
    if (sums) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float g = yy[j][k] > 0.f ? v[k] : 0.f;
        gs[k] += g;
        gq[k] += g * ((zz[j][k] - mu[k]) * isd[k]);
      }
    }
  }
  if (!sums) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    part[0][rg * kHeadCW + 8 * lgp + k] = gs[k];
    part[1][rg * kHeadCW + 8 * lgp + k] = gq[k];
  }
  __syncthreads();
  if (t < 2 * kHeadCW) {
    const int pass = t / kHeadCW, c = t - pass * kHeadCW;
    double a = 0.0;
    for (int r = 0; r < 16; ++r) a += part[pass][r * kHeadCW + c];
    atomicAdd(&hb.acc_b[(int64_t)(b % hb.reps_b) * 2 * C + pass * C + c0 + c], a);
  }
}

// MFL_HEAD_SPLIT=0: the one-launch head for A/B runs
static bool head_split_ok(int C, int HW, int K) {
  const char* e = getenv("MFL_HEAD_SPLIT");
  const int on = e && *e ? atoi(e) : 1;
  return on && C % kHeadCW == 0 && HW >= 1 && HW <= 16 * kHeadMaxPix && K <= 64;
}

template <typename T>
static void head_split_launch(int B, int HW, int C, const float* W, const float* bias, int K, const int* labels,
                              float* feat, float* dlogits, T* dx, float* stats, bool backward, hipStream_t s,
                              float* dW, float* db, const HeadBn& hb, float* lpart) {
  const int n = B * (C / kHeadCW);
  head_split_fwd_kernel<T><<<n, 256, 0, s>>>(HW, C, W, K, feat, lpart, B, hb);
  const size_t dyn = ((size_t)((K + 3) & ~3) + (size_t)K * kHeadCW) * sizeof(float);
  head_split_bwd_kernel<T><<<n, 256, dyn, s>>>(HW, C, W, bias, K, labels, feat, lpart,
                                                                    dlogits, dx, stats, B, backward ? 1 : 0,
                                                                    backward ? dW : nullptr,
                                                                    backward ? db : nullptr, hb);
}

template <typename T, bool FUSE>
static void head_launch_t(const T* x, int B, int HW, int C, const float* W, const float* bias, int K,
                          const int* labels, float* feat, float* dlogits, T* dx, float* stats, bool backward,
                          hipStream_t s, float* dW, float* db, const HeadBn& hb) {
  const int G = C / 8, R = G >= 256 ? 1 : 256 / G;
  const size_t sm = (size_t)(C + ((K + 3) & ~3) + (size_t)R * C + (size_t)K * C + (FUSE ? 4 * (size_t)C : 0)) *
                    sizeof(float);
  static bool attr = false;
  if (!attr && sm > 65536) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&head_kernel<T, FUSE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    attr = true;
  }
  head_kernel<T, FUSE><<<B, 256, sm, s>>>(x, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, B,
                                          backward ? 1 : 0, backward ? dW : nullptr, backward ? db : nullptr, hb);
}

template <typename T>
static void head_launch(const T* x, int B, int HW, int C, const float* W, const float* bias, int K,
                        const int* labels, float* feat, float* dlogits, T* dx, float* stats, bool backward,
                        hipStream_t s, float* dW, float* db) {
  head_launch_t<T, false>(x, B, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, backward, s, dW, db, HeadBn{});
}

void launch_head_fwd_bwd(const uint16_t* x, int B, int HW, int C, const float* W, const float* bias,
                         int K, const int* labels, float* feat, float* dlogits, uint16_t* dx,
                         float* stats, bool backward, hipStream_t s, float* dW, float* db, const HeadBn* bn,
                         float* lpart) {
  if (bn) {
    HeadBn hb = *bn;
    if (!backward) hb.acc_b = nullptr;
    if (lpart && feat && head_split_ok(C, HW, K)) {
      head_split_launch<uint16_t>(B, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, backward, s, dW, db, hb,
                                  lpart);
      return;
    }
    head_launch_t<uint16_t, true>(x, B, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, backward, s, dW, db,
                                  hb);
    return;
  }
  head_launch(x, B, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, backward, s, dW, db);
}
void launch_head32_fwd_bwd(const float* x, int B, int HW, int C, const float* W, const float* bias, int K,
                           const int* labels, float* feat, float* dlogits, float* dx, float* stats, bool backward,
                           hipStream_t s, float* dW, float* db, const HeadBn* bn, float* lpart) {
  if (bn) {
    HeadBn hb = *bn;
    if (!backward) hb.acc_b = nullptr;
    if (lpart && feat && head_split_ok(C, HW, K)) {
      head_split_launch<float>(B, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, backward, s, dW, db, hb,
                               lpart);
      return;
    }
    head_launch_t<float, true>(x, B, HW, C, W, bias, K, labels, feat, dlogits, dx, stats, backward, s, dW, db, hb);
    return;
  }
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
