// fp32 BatchNorm(+ReLU) backward apply as a device function, shared by the
// stand-alone launch (bn32.hip bn32_bwd_apply_kernel) and the paired conv
// backward that carries it as a third workgroup role (conv32.hip
// conv32_bwd_pair_kernel, "folded" apply): one definition, so both produce the
// same bits.
//
//   g  = dy [* (y > 0)]                    (dy_masked <- g, optional)
//   dz = gamma invstd (g - mean g - xhat mean(g xhat)),  xhat = (z - mean) invstd
//
// with the per-channel sums (sum g, sum g xhat) read from the fp64 replica
// accumulators the producer of dy added into.  COH: dy and the sums were
// written in the SAME launch by workgroups on other XCDs (device-scope stores
// and memory-side atomics), so they are read with device-scope (sc1) loads
// that look past this XCD's L2; everything else was written by earlier
// launches.
#pragma once
#include "kernels/bn_coef.h"
#include "kernels/common.h"
#include "kernels/launchers.h"
#include "kernels/lds_tiles.h"

namespace mfl {

// per-thread float4 partials (s, q) over rows -> fp64 atomics into acc[0|1][C];
// sh: 2 x 256 float4 of LDS (blockDim.x == 256)
__device__ __forceinline__ void channel_atomic4_lds(float4 s, float4 q, int C, int tpr, int rpp, double* acc,
                                                    float4* sh) {
  const int t = threadIdx.x;
  const bool act = t < rpp * tpr;
  sh[t] = act ? s : make_float4(0.f, 0.f, 0.f, 0.f);
  sh[256 + t] = act ? q : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  const float* s0 = reinterpret_cast<const float*>(sh);
  const float* s1 = reinterpret_cast<const float*>(sh + 256);
  for (int c = t; c < C && c < tpr * 4; c += 256) {
    double a = 0.0, b = 0.0;
    const int cg = c >> 2, k = c & 3;
    for (int r = 0; r < rpp; ++r) {
      a += s0[(r * tpr + cg) * 4 + k];
      b += s1[(r * tpr + cg) * 4 + k];
    }
    atomicAdd(&acc[c], a);
    atomicAdd(&acc[C + c], b);
  }
}

// rep_sums (bn_coef.h) with device-scope loads: same replica order, same bits
__device__ __forceinline__ void rep_sums_coherent(const double* acc, int reps, int C, int c, double& s0,
                                                  double& s1) {
  double a[kMaxReps], b[kMaxReps];
#pragma unroll
  for (int r = 0; r < kMaxReps; ++r) {
    a[r] = r < reps ? __hip_atomic_load(acc + (int64_t)r * 2 * C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                    : 0.0;
    b[r] = r < reps ? __hip_atomic_load(acc + (int64_t)r * 2 * C + C + c, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT)
                    : 0.0;
  }
  s0 = 0.0;
  s1 = 0.0;
#pragma unroll
  for (int r = 0; r < kMaxReps; ++r) {
    s0 += a[r];
    s1 += b[r];
  }
}

// (bid, nblk): this block's index in the apply's own grid; sc: [5][C] floats
// of LDS (k1, mean g, mean g*xhat, mean, invstd); sh: 512 float4 of LDS for
// the side reduction.  blockDim.x == 256.
template <bool MASK, bool WRITE_DYM, bool COH>
__device__ __forceinline__ void bn32_bwd_apply_body(const BnBwdArgs32& a, int64_t nvec, int bid, int nblk,
                                                    float* sc, float4* sh) {
  const int C = a.C;
  const float4* DY = reinterpret_cast<const float4*>(a.dy);
  const float4* X = reinterpret_cast<const float4*>(a.x);
  const float4* Y = reinterpret_cast<const float4*>(a.y);
  const auto rsDY = make_rsrc(a.dy, (uint32_t)(nvec * 16 < 0x7FFFFFF0LL ? nvec * 16 : 0x7FFFFFF0LL));
  auto load_dy = [&](int64_t i) -> float4 {
    if constexpr (COH) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsDY, (int)(i * 16), 0, 16);  // sc1: device scope
      return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                         __uint_as_float(v[3]));
    } else {
      return DY[i];
    }
  };
  const int64_t stride = (int64_t)nblk * blockDim.x;
  int64_t i = (int64_t)bid * blockDim.x + threadIdx.x;
  float4 gv = make_float4(0.f, 0.f, 0.f, 0.f), xv = gv, yv = gv;
  if (i < nvec) {
    gv = load_dy(i);
    xv = X[i];
    if (MASK) yv = Y[i];
  }
  const double inv_m = 1.0 / (double)a.M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double s, q;
    if constexpr (COH) rep_sums_coherent(a.acc, a.reps, C, c, s, q);
    else rep_sums(a.acc, a.reps, C, c, s, q);
    sc[c] = a.gamma[c] * a.invstd[c];
    sc[C + c] = (float)(s * inv_m);
    sc[2 * C + c] = (float)(q * inv_m);
    sc[3 * C + c] = a.mean[c];
    sc[4 * C + c] = a.invstd[c];
    if (bid == 0) {
      if (a.dgamma) a.dgamma[c] = (float)q;
      if (a.dbeta) a.dbeta[c] = (float)s;
    }
  }
  __syncthreads();
  const int tpr = C / 4;
  const bool fixed = (256 % tpr) == 0;
  int cb = fixed ? (int)(threadIdx.x % (unsigned)tpr) * 4 : 0;
  float4 k1, mg, mx, mu, is;
  auto load_coef = [&]() {
    k1 = *reinterpret_cast<const float4*>(sc + cb);
    mg = *reinterpret_cast<const float4*>(sc + C + cb);
    mx = *reinterpret_cast<const float4*>(sc + 2 * C + cb);
    mu = *reinterpret_cast<const float4*>(sc + 3 * C + cb);
    is = *reinterpret_cast<const float4*>(sc + 4 * C + cb);
  };
  load_coef();
  // side reduction (fixed channels only: the bindings check)
  const bool side = WRITE_DYM && a.acc2 != nullptr;
  float4 s2 = make_float4(0.f, 0.f, 0.f, 0.f), q2 = s2, mu2 = s2, is2 = s2;
  if (side) {
    mu2 = *reinterpret_cast<const float4*>(a.mean2 + cb);
    is2 = *reinterpret_cast<const float4*>(a.invstd2 + cb);
  }
  for (; i < nvec; i += stride) {
    float4 g = gv;
    const float4 xc = xv, yc = yv;
    if (i + stride < nvec) {
      gv = load_dy(i + stride);
      xv = X[i + stride];
      if (MASK) yv = Y[i + stride];
    }
    if (!fixed) {
      cb = (int)(i % tpr) * 4;
      load_coef();
    }
    if (MASK) {
      g.x = yc.x > 0.f ? g.x : 0.f;
      g.y = yc.y > 0.f ? g.y : 0.f;
      g.z = yc.z > 0.f ? g.z : 0.f;
      g.w = yc.w > 0.f ? g.w : 0.f;
      if (WRITE_DYM) reinterpret_cast<float4*>(a.dy_masked)[i] = g;
      if (WRITE_DYM && side) {
        const float4 z2 = reinterpret_cast<const float4*>(a.z2)[i];
        s2.x += g.x; s2.y += g.y; s2.z += g.z; s2.w += g.w;
        q2.x += g.x * ((z2.x - mu2.x) * is2.x);
        q2.y += g.y * ((z2.y - mu2.y) * is2.y);
        q2.z += g.z * ((z2.z - mu2.z) * is2.z);
        q2.w += g.w * ((z2.w - mu2.w) * is2.w);
      }
    }
    float4 o;
    o.x = k1.x * fmaf(-((xc.x - mu.x) * is.x), mx.x, g.x - mg.x);
    o.y = k1.y * fmaf(-((xc.y - mu.y) * is.y), mx.y, g.y - mg.y);
    o.z = k1.z * fmaf(-((xc.z - mu.z) * is.z), mx.z, g.z - mg.z);
    o.w = k1.w * fmaf(-((xc.w - mu.w) * is.w), mx.w, g.w - mg.w);
    if (a.pack_dx)  // uniform: the bf16x3 convolutions' dY encoding
      reinterpret_cast<uint4*>(a.dx)[i] = make_uint4(split_pack(o.x), split_pack(o.y), split_pack(o.z), split_pack(o.w));
    else
      reinterpret_cast<float4*>(a.dx)[i] = o;
  }
  if (side) {
    __syncthreads();  // sc[] reads done before the LDS staging
    channel_atomic4_lds(s2, q2, C, tpr, 256 / tpr, a.acc2 + (int64_t)(bid % a.reps2) * 2 * C, sh);
  }
}

}  // namespace mfl
