// Shared device helpers for the gfx950 (CDNA4) kernels of metisfl_amd.
//
// Conventions used by every kernel in this directory:
//  * bf16 values travel as raw uint16_t bit patterns; conversion is done with
//    the hip_bf16 intrinsics (the compiler lowers them to v_cvt_pk_bf16_f32 on
//    gfx950, see cdna_hip_programming.md T12 "cvt_pk alone: don't hand-write").
//  * memory-bound kernels move 16 B per lane (8 x bf16 / 4 x fp32)
//    (cdna_hip_programming.md Guideline 13).
//  * wave size is 64 and is hard-coded (Guideline: "Hard-code 64").
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace mfl {

constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(uint16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}

// fp32 -> packed (hi << 16 | lo) bf16 pair, a = hi + lo + O(2^-18 |a|): the
// operand encoding of the bf16x3 fp32 convolutions (conv32.hip c32s decodes it
// with two v_perm per pair instead of splitting in the k-loop).  Written by the
// fused optimizer (weight mirror) and by the fp32 BN backward (the conv's dY).
__device__ __forceinline__ uint32_t split_pack(float a) {
  const uint16_t h = f2bf(a);
  const uint16_t l = f2bf(a - bf2f(h));
  return ((uint32_t)h << 16) | l;
}

// Packs two floats into two bf16 (RNE) in one dword.
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// Exact-erf GELU pieces at bf16-output accuracy: erfc(|z|/sqrt2) by Abramowitz
// & Stegun 7.1.26 (|erf error| <= 1.5e-7; bf16 resolves 2^-9 relative), one
// exp shared by Phi(z) and phi(z), no cancellation in the negative tail.
// ocml's erff is ~3x the VALU work: it made gelu_bwd and the fused GEMM GELU
// epilogues VALU-bound (50M elements per BERT-base FFN).
__device__ __forceinline__ void gelu_parts(float z, float& cdf, float& pdf) {
  const float x = fabsf(z) * 0.70710678f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, x, 1.f));
  const float e = __expf(-x * x);  // exp(-z^2 / 2)
  const float poly =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
               0.254829592f);
  const float q = 0.5f * poly * e;  // Phi(-|z|)
  cdf = z < 0.f ? q : 1.f - q;
  pdf = 0.39894228f * e;
}
__device__ __forceinline__ float gelu_f(float z) {
  float c, p;
  gelu_parts(z, c, p);
  return z * c;
}
__device__ __forceinline__ float gelu_grad_f(float z) {
  float c, p;
  gelu_parts(z, c, p);
  return c + z * p;
}
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2bf(f[0], f[1]);
  r.y = pack2bf(f[2], f[3]);
  r.z = pack2bf(f[4], f[5]);
  r.w = pack2bf(f[6], f[7]);
  return r;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Grid size for a grid-stride memory-bound kernel (Guideline 11: cap ~2048).
inline unsigned stream_grid(int64_t work_items, int block = 256, int cap = 2048) {
  int64_t g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

}  // namespace mfl
