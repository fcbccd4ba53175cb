// K12 (fp32): BatchNorm forward / backward for NHWC fp32 activations -- the
// reference-precision twin of bn.hip (same launch design: statistics arrive
// as fp64 sums from the producing conv's epilogue, the apply kernel derives
// mean / inv-std / scale / shift in its prologue and block 0 publishes the
// saved statistics and the running averages; backward is one reduce (or
// none, when the dgrad epilogue already summed) plus one apply).
// Each lane moves 4 channels (one 16-B float4).  C % 4 == 0.
#include "kernels/common.h"
#include "kernels/bn_coef.h"
#include "kernels/launchers.h"
#include "kernels/opt_tail_dev.h"

namespace mfl {

namespace {

int blocks_for(int64_t M, int C) {
  const int tpr = C / 4;
  const int rpp = tpr >= 256 ? 1 : 256 / tpr;
  int64_t nb = (M + (int64_t)rpp * 8 - 1) / ((int64_t)rpp * 8);
  if (nb > 512) nb = 512;
  if (nb < 1) nb = 1;
  return (int)nb;
}

// per-thread float4 partials (s, q) over rows -> fp64 atomics into acc[0|1][C]
__device__ __forceinline__ void channel_atomic4(float4 s, float4 q, int C, int tpr, int rpp, double* acc) {
  __shared__ float4 sh[2][256];
  const int t = threadIdx.x;
  const bool act = t < rpp * tpr;
  sh[0][t] = act ? s : make_float4(0.f, 0.f, 0.f, 0.f);
  sh[1][t] = act ? q : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  const float* s0 = reinterpret_cast<const float*>(sh[0]);
  const float* s1 = reinterpret_cast<const float*>(sh[1]);
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

}  // namespace

__global__ __launch_bounds__(256) void bn32_stats_kernel(const float* __restrict__ x, int64_t M, int C,
                                                         double* __restrict__ acc, int reps) {
  // channel groups beyond 256 threads: grid.y slices the channels
  const int tpr_all = C / 4;
  const int tpr = min(tpr_all - (int)blockIdx.y * 256, 256);
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int cg = t % tpr, r0 = t / tpr;
  const int cbase = blockIdx.y * 1024;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
  if (r0 < rpp) {
    for (int64_t row = (int64_t)blockIdx.x * rpp + r0; row < M; row += (int64_t)gridDim.x * rpp) {
      const float4 v = *reinterpret_cast<const float4*>(x + row * C + cbase + cg * 4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      q.x += v.x * v.x; q.y += v.y * v.y; q.z += v.z * v.z; q.w += v.w * v.w;
    }
  }
  channel_atomic4(s, q, C, tpr, rpp, acc + (int64_t)(blockIdx.x % reps) * 2 * C + cbase);
}

void launch_bn32_stats(const float* x, int64_t M, int C, double* acc, hipStream_t s, int reps) {
  // acc + cbase: the [C] halves stay at stride C, so pass the base and C
  const int gy = (C / 4 + 255) / 256;
  bn32_stats_kernel<<<dim3(blocks_for(M, C), gy), 256, 0, s>>>(x, M, C, acc, reps > 0 ? reps : 1);
}


// Grid of the apply kernels.  Every block's prologue re-derives all C
// channels' coefficients from the 8 fp64 replica pairs (16 loads per
// channel): at one float4 per thread (2,048 blocks) that is 2,048 x C x 128 B
// of L2 reads -- 67 MB for a C = 512 layer whose payload is 4 MB.  Capping the
// grid amortises the prologue over several vectors per thread.
#ifndef MFL_BN32_GRID
#define MFL_BN32_GRID 512
#endif
// run-time cap (set_bn32_grid_cap): 256 for 4+ co-located learners, whose
// launches fill the CUs anyway (8 learners 5.391 -> 5.343 ms per 8-learner
// step; one learner 1.038 -> 1.043, so it keeps 512; 1,024 was slower for
// both: profiles/r6/s2/bn32_grid_*.log)
static int g_bn32_grid = MFL_BN32_GRID;
inline unsigned apply_grid(int64_t nvec) { return stream_grid(nvec, 256, g_bn32_grid); }

// Main loops: when C / 4 divides 256 the grid stride is a multiple of C / 4,
// so a lane's channels never change -- its coefficients live in registers
// (no LDS read and no 64-bit modulo per vector).
// (bid, nblk): this block's index in the apply's own grid (the paired launch
// maps one hardware grid onto two applies)
template <bool RES, bool RELU>
__device__ __forceinline__ void bn32_apply_body(const BnFwdArgs32& a, int64_t nvec, int bid, int nblk,
                                                float* coef) {
  const int C = a.C;
  const float4* X = reinterpret_cast<const float4*>(a.x);
  const float4* R = reinterpret_cast<const float4*>(a.residual);
  const int64_t stride = (int64_t)nblk * blockDim.x;
  int64_t i = (int64_t)bid * blockDim.x + threadIdx.x;
  float4 xv = make_float4(0.f, 0.f, 0.f, 0.f), rv = xv;
  if (i < nvec) {  // first vectors in flight across the prologue
    xv = X[i];
    if (RES) rv = R[i];
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float sc, sh;
    bn_fwd_coef(a.acc, a.reps, C, c, a.M, a.train, bid == 0, a.gamma, a.beta, a.mean, a.invstd, a.run_mean,
                a.run_var, a.momentum, a.eps, sc, sh);
    coef[c] = sc;
    coef[C + c] = sh;
  }
  __syncthreads();
  const int tpr = C / 4;
  const bool fixed = (256 % tpr) == 0;  // lane channels constant over the grid stride
  int cb = fixed ? (int)(threadIdx.x % (unsigned)tpr) * 4 : 0;
  float4 sc = *reinterpret_cast<const float4*>(coef + cb);
  float4 sh = *reinterpret_cast<const float4*>(coef + C + cb);
  for (; i < nvec; i += stride) {
    const float4 xc = xv, rc = rv;
    if (i + stride < nvec) {
      xv = X[i + stride];
      if (RES) rv = R[i + stride];
    }
    if (!fixed) {
      cb = (int)(i % tpr) * 4;
      sc = *reinterpret_cast<const float4*>(coef + cb);
      sh = *reinterpret_cast<const float4*>(coef + C + cb);
    }
    float4 v = make_float4(fmaf(xc.x, sc.x, sh.x), fmaf(xc.y, sc.y, sh.y), fmaf(xc.z, sc.z, sh.z),
                           fmaf(xc.w, sc.w, sh.w));
    if (RES) {
      v.x += rc.x; v.y += rc.y; v.z += rc.z; v.w += rc.w;
    }
    if (RELU) {
      v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    }
    reinterpret_cast<float4*>(a.y)[i] = v;
    if (a.yp)  // uniform
      reinterpret_cast<uint4*>(a.yp)[i] = make_uint4(split_pack(v.x), split_pack(v.y), split_pack(v.z), split_pack(v.w));
  }
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void bn32_apply_kernel(BnFwdArgs32 a, int64_t nvec) {
  extern __shared__ __attribute__((aligned(16))) float coef[];  // [2][C]
  bn32_apply_body<RES, RELU>(a, nvec, blockIdx.x, gridDim.x, coef);
}

// A downsampling block's two BatchNorms (shortcut: no ReLU; conv1: ReLU) in
// one launch (the bf16 twin: bn.hip bn_apply_pair_kernel).
__global__ __launch_bounds__(256) void bn32_apply_pair_kernel(BnFwdArgs32 a1, int64_t n1, int g1, BnFwdArgs32 a2,
                                                              int64_t n2) {
  extern __shared__ __attribute__((aligned(16))) float coef[];
  if ((int)blockIdx.x < g1) bn32_apply_body<false, false>(a1, n1, blockIdx.x, g1, coef);
  else bn32_apply_body<false, true>(a2, n2, blockIdx.x - g1, gridDim.x - g1, coef);
}

void launch_bn32_apply_pair(const BnFwdArgs32& a1, const BnFwdArgs32& a2, hipStream_t s) {
  const int64_t n1 = a1.M * a1.C / 4, n2 = a2.M * a2.C / 4;
  const unsigned g1 = apply_grid(n1), g2 = apply_grid(n2);
  const size_t sm = 2 * (size_t)(a1.C > a2.C ? a1.C : a2.C) * sizeof(float);
  bn32_apply_pair_kernel<<<g1 + g2, 256, sm, s>>>(a1, n1, (int)g1, a2, n2);
}

void launch_bn32_apply(const BnFwdArgs32& a, hipStream_t s) {
  const int64_t nvec = a.M * a.C / 4;
  const unsigned g = apply_grid(nvec);
  const size_t sm = 2 * a.C * sizeof(float);
  if (a.residual) {
    if (a.relu) bn32_apply_kernel<true, true><<<g, 256, sm, s>>>(a, nvec);
    else bn32_apply_kernel<true, false><<<g, 256, sm, s>>>(a, nvec);
  } else {
    if (a.relu) bn32_apply_kernel<false, true><<<g, 256, sm, s>>>(a, nvec);
    else bn32_apply_kernel<false, false><<<g, 256, sm, s>>>(a, nvec);
  }
}

// Backward reduce: acc[c] += sum g, acc[C+c] += sum g * xhat, g = dy [* (y > 0)]
__global__ __launch_bounds__(256) void bn32_bwd_reduce_kernel(const float* __restrict__ dy,
                                                              const float* __restrict__ x,
                                                              const float* __restrict__ y,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd, int64_t M,
                                                              int C, double* __restrict__ acc, int reps) {
  const int tpr_all = C / 4;
  const int tpr = min(tpr_all - (int)blockIdx.y * 256, 256);
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int cg = t % tpr, r0 = t / tpr;
  const int cb = blockIdx.y * 1024 + cg * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
  if (r0 < rpp) {
    const float4 mu = *reinterpret_cast<const float4*>(mean + cb);
    const float4 is = *reinterpret_cast<const float4*>(invstd + cb);
    for (int64_t row = (int64_t)blockIdx.x * rpp + r0; row < M; row += (int64_t)gridDim.x * rpp) {
      const int64_t off = row * C + cb;
      float4 g = *reinterpret_cast<const float4*>(dy + off);
      const float4 xv = *reinterpret_cast<const float4*>(x + off);
      if (y) {
        const float4 yv = *reinterpret_cast<const float4*>(y + off);
        g.x = yv.x > 0.f ? g.x : 0.f;
        g.y = yv.y > 0.f ? g.y : 0.f;
        g.z = yv.z > 0.f ? g.z : 0.f;
        g.w = yv.w > 0.f ? g.w : 0.f;
      }
      s.x += g.x; s.y += g.y; s.z += g.z; s.w += g.w;
      q.x += g.x * ((xv.x - mu.x) * is.x);
      q.y += g.y * ((xv.y - mu.y) * is.y);
      q.z += g.z * ((xv.z - mu.z) * is.z);
      q.w += g.w * ((xv.w - mu.w) * is.w);
    }
  }
  channel_atomic4(s, q, C, tpr, rpp, acc + (int64_t)(blockIdx.x % reps) * 2 * C + blockIdx.y * 1024);
}

void launch_bn32_bwd_reduce(const float* dy, const float* x, const float* y, const float* mean,
                            const float* invstd, int64_t M, int C, double* acc, hipStream_t s, int reps) {
  const int gy = (C / 4 + 255) / 256;
  bn32_bwd_reduce_kernel<<<dim3(blocks_for(M, C), gy), 256, 0, s>>>(dy, x, y, mean, invstd, M, C, acc,
                                                                      reps > 0 ? reps : 1);
}

// Backward apply: dx = gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)).
// Workgroup `bid` of `nblk` (a stand-alone launch, or one role of a paired
// launch); sc: [5][C] floats of LDS (k1, mean g, mean g*xh, mean, invstd).
template <bool MASK, bool WRITE_DYM>
__device__ __forceinline__ void bn32_bwd_apply_body(const BnBwdArgs32& a, int64_t nvec, int bid, int nblk,
                                                    float* sc) {
  const int C = a.C;
  const float4* DY = reinterpret_cast<const float4*>(a.dy);
  const float4* X = reinterpret_cast<const float4*>(a.x);
  const float4* Y = reinterpret_cast<const float4*>(a.y);
  const int64_t stride = (int64_t)nblk * blockDim.x;
  int64_t i = (int64_t)bid * blockDim.x + threadIdx.x;
  float4 gv = make_float4(0.f, 0.f, 0.f, 0.f), xv = gv, yv = gv;
  if (i < nvec) {
    gv = DY[i];
    xv = X[i];
    if (MASK) yv = Y[i];
  }
  const double inv_m = 1.0 / (double)a.M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double s, q;
    rep_sums(a.acc, a.reps, C, c, s, q);
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
  // side reduction (fixed channels only: the binding checks)
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
      gv = DY[i + stride];
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
    }
    // !MASK: dy arrives masked (its producing dgrad applied the mask)
    if (WRITE_DYM) reinterpret_cast<float4*>(a.dy_masked)[i] = g;
    if (WRITE_DYM && side) {
      const float4 z2 = reinterpret_cast<const float4*>(a.z2)[i];
      s2.x += g.x; s2.y += g.y; s2.z += g.z; s2.w += g.w;
      q2.x += g.x * ((z2.x - mu2.x) * is2.x);
      q2.y += g.y * ((z2.y - mu2.y) * is2.y);
      q2.z += g.z * ((z2.z - mu2.z) * is2.z);
      q2.w += g.w * ((z2.w - mu2.w) * is2.w);
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
    __syncthreads();  // sc[] reads done before channel_atomic4's LDS staging
    channel_atomic4(s2, q2, C, tpr, 256 / tpr, a.acc2 + (int64_t)(bid % a.reps2) * 2 * C);
  }
}

template <bool MASK, bool WRITE_DYM>
__global__ __launch_bounds__(256) void bn32_bwd_apply_kernel(BnBwdArgs32 a, int64_t nvec) {
  extern __shared__ __attribute__((aligned(16))) float sc[];
  bn32_bwd_apply_body<MASK, WRITE_DYM>(a, nvec, blockIdx.x, gridDim.x, sc);
}

// A downsampling block's conv1 BatchNorm (ReLU) and projection-shortcut
// BatchNorm (no ReLU) backward applies in one launch: both sums are complete
// once conv2's backward has run (conv1's from conv2's dgrad epilogue, the
// shortcut's from conv2's BN-backward side reduction), so the two
// bandwidth-bound passes share one launch instead of two dependent ones.
__global__ __launch_bounds__(256) void bn32_bwd_apply_pair_kernel(BnBwdArgs32 a1, int64_t n1, int g1,
                                                                  BnBwdArgs32 a2, int64_t n2) {
  extern __shared__ __attribute__((aligned(16))) float sc[];
  if ((int)blockIdx.x < g1) {
    if (a1.y) bn32_bwd_apply_body<true, false>(a1, n1, blockIdx.x, g1, sc);
    else bn32_bwd_apply_body<false, false>(a1, n1, blockIdx.x, g1, sc);  // dy arrives masked
  } else {
    bn32_bwd_apply_body<false, false>(a2, n2, blockIdx.x - g1, gridDim.x - g1, sc);
  }
}

// ---------------------------------------------------------------------------
// The stem's backward in ONE launch.  The CIFAR stem (3x3 / stride 1 over the
// 8-channel zero-padded 32x32 input, 64 output channels) has no dgrad, so its
// backward was a BatchNorm backward apply writing dz (5 x 8.4 MB moved at
// batch 32) plus an im2col wgrad over K = 72 that re-reads dz and x per
// split-K slice (~21 us together per step, profiles/r3).  Here workgroup
// (image n, channel group cg) loads dy, z and the ReLU output y of its 8
// output channels over the whole image once, forms dz with bn32_bwd_apply's
// arithmetic (the same fmaf sequence: bit-identical dz) straight into LDS
// next to the image's input (+1-pixel halo), and wave `tap` (9 waves) sums
// dz[p][co] * x[p + tap][ci] over the image with exact fp32 FMAs (lane = pixel
// phase, all 8 x 8 products per lane, a recursive-halving butterfly), then
// one fp32 atomic per (co, tap, ci) and image into dw (zero on entry).
// Work split by (image, 8 output channels): every dw address takes one atomic
// per image (N-way), 576 per workgroup.  (A first version split by 4-row
// pixel strips with all 64 channels per workgroup: 256-way contention on
// every dw address, 1.2M atomics -- slower than the two launches it replaced.)
// Blocks are numbered image-fastest, so with N % 8 == 0 the 8 channel groups
// of an image run on one XCD (round-robin placement) and share its 256-B
// activation rows in that XCD's L2.
// T = uint16_t: the bf16 option's tensors (dy, z, y, x bf16; dz and the
// products stay fp32).
constexpr int kStemCG = 8;  // output channels per workgroup

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld4(const uint16_t* p) {
  const uint2 v = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u), __uint_as_float(v.y << 16),
                     __uint_as_float(v.y & 0xffff0000u));
}

template <typename T>
__global__ __launch_bounds__(576) void stem_bwd32_kernel(BnBwdArgs32 a, const T* __restrict__ x, int N,
                                                         float* __restrict__ dw, OptTail ot) {
  if ((int)blockIdx.x >= (int)gridDim.x - ot.nblk) {  // optimizer tail (opt_tail.h), dispatched last
    opt_tail_body(ot, blockIdx.x - (gridDim.x - ot.nblk));
    return;
  }
  constexpr int H = 32, W = 32, CI = 8, CO = 64, PX = H * W, XW = W + 2, G = kStemCG;
  constexpr int NV = PX * G / 4;            // float4 of dy / z / y per workgroup (2 per pixel)
  constexpr int NU = (NV + 575) / 576;
  constexpr int NX = (H + 2) * XW * CI / 4;  // float4 of the padded input image
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* dzs = sm;                 // [PX][G]
  float* xs = dzs + PX * G;        // [H + 2][XW][CI]
  float* cf = xs + (H + 2) * XW * CI;  // [5][G]: k1, mean g, mean g*xhat, mean, invstd
  const int t = threadIdx.x;
  const int img = blockIdx.x % N, cg = blockIdx.x / N;
  const int co0 = cg * G;
  // operand loads first: float4 i = (pixel i / 2, channels co0 + 4 (i & 1) ..)
  const int64_t pix0 = (int64_t)img * PX;
  float4 g[NU], z[NU], m[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int i = t + 576 * u;
    if (NV % 576 == 0 || i < NV) {
      const int64_t o = (pix0 + (i >> 1)) * CO + co0 + 4 * (i & 1);
      g[u] = ld4(reinterpret_cast<const T*>(a.dy) + o);
      z[u] = ld4(reinterpret_cast<const T*>(a.x) + o);
      m[u] = ld4(reinterpret_cast<const T*>(a.y) + o);
    }
  }
  // the input patch: every load issued before the first LDS store (a
  // load-store loop paid one memory latency per trip)
  constexpr int NXU = (NX + 575) / 576;
  float4 xv[NXU];
#pragma unroll
  for (int u = 0; u < NXU; ++u) {
    const int i = t + 576 * u;
    const int pix = i >> 1, xr = pix / XW, xc = pix - xr * XW;
    const int iy = xr - 1, ix = xc - 1;
    xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < NX && iy >= 0 && iy < H && ix >= 0 && ix < W)
      xv[u] = ld4(x + (pix0 + iy * W + ix) * CI + 4 * (i & 1));
  }
  if (t < G) {
    const int c = co0 + t;
    double s, q;
    rep_sums(a.acc, a.reps, CO, c, s, q);
    const double inv_m = 1.0 / (double)a.M;
    cf[t] = a.gamma[c] * a.invstd[c];
    cf[G + t] = (float)(s * inv_m);
    cf[2 * G + t] = (float)(q * inv_m);
    cf[3 * G + t] = a.mean[c];
    cf[4 * G + t] = a.invstd[c];
    if (img == 0) {
      if (a.dgamma) a.dgamma[c] = (float)q;
      if (a.dbeta) a.dbeta[c] = (float)s;
    }
  }
#pragma unroll
  for (int u = 0; u < NXU; ++u)
    if (t + 576 * u < NX) reinterpret_cast<float4*>(xs)[t + 576 * u] = xv[u];
  __syncthreads();
  // dz = k1 (g - mean g - xhat mean(g xhat)), g = dy [y > 0] (bn32_bwd_apply);
  // 576 is even, so a thread's channel quad (i & 1) is fixed
  const int cb = 4 * (t & 1);
  const float4 k1 = *reinterpret_cast<const float4*>(cf + cb);
  const float4 mg = *reinterpret_cast<const float4*>(cf + G + cb);
  const float4 mx = *reinterpret_cast<const float4*>(cf + 2 * G + cb);
  const float4 mu = *reinterpret_cast<const float4*>(cf + 3 * G + cb);
  const float4 is = *reinterpret_cast<const float4*>(cf + 4 * G + cb);
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int i = t + 576 * u;
    if (NV % 576 == 0 || i < NV) {
      float4 gg = g[u];
      gg.x = m[u].x > 0.f ? gg.x : 0.f;
      gg.y = m[u].y > 0.f ? gg.y : 0.f;
      gg.z = m[u].z > 0.f ? gg.z : 0.f;
      gg.w = m[u].w > 0.f ? gg.w : 0.f;
      float4 o;
      o.x = k1.x * fmaf(-((z[u].x - mu.x) * is.x), mx.x, gg.x - mg.x);
      o.y = k1.y * fmaf(-((z[u].y - mu.y) * is.y), mx.y, gg.y - mg.y);
      o.z = k1.z * fmaf(-((z[u].z - mu.z) * is.z), mx.z, gg.z - mg.z);
      o.w = k1.w * fmaf(-((z[u].w - mu.w) * is.w), mx.w, gg.w - mg.w);
      reinterpret_cast<float4*>(dzs)[i] = o;
    }
  }
  __syncthreads();
  // wave = filter tap (r, s); lane = pixel phase: a lane sums pixels p = lane,
  // lane + 64, ... into all 8 x 8 (co, ci) products of the tap -- dz[p][0..7]
  // and x[p + tap][0..7] are two lane-distinct b128 reads each, 64 FMAs per
  // pixel (a lane-per-output-channel mapping re-read each input row 8 times:
  // LDS-bound) -- then a recursive-halving butterfly leaves output o = lane
  // on each lane (63 shuffles)
  const int tap = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lane = t & 63;
  const int r = tap / 3, sx = tap - 3 * r;
  float acc[G * CI];
#pragma unroll
  for (int o = 0; o < G * CI; ++o) acc[o] = 0.f;
#pragma unroll 2
  for (int p = lane; p < PX; p += 64) {
    const int py = p >> 5, px = p & 31;
    const float4 d0 = *reinterpret_cast<const float4*>(dzs + p * G);
    const float4 d1 = *reinterpret_cast<const float4*>(dzs + p * G + 4);
    const float* xr = xs + ((py + r) * XW + px + sx) * CI;
    const float4 x0 = *reinterpret_cast<const float4*>(xr);
    const float4 x1 = *reinterpret_cast<const float4*>(xr + 4);
    const float dv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
    const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int c = 0; c < G; ++c)
#pragma unroll
      for (int k = 0; k < CI; ++k) acc[c * CI + k] = fmaf(dv[c], xv[k], acc[c * CI + k]);
  }
  // recursive halving over the 64 lanes: at offset d a lane keeps the half of
  // its n values selected by its lane bit d and adds the partner's copy
#pragma unroll
  for (int d = 32, n = 64; d >= 1; d >>= 1, n >>= 1) {
    const bool up = (lane & d) != 0;
#pragma unroll
    for (int j = 0; j < n / 2; ++j) {
      const float send = up ? acc[j] : acc[j + n / 2];
      const float keep = up ? acc[j + n / 2] : acc[j];
      acc[j] = keep + __shfl_xor(send, d, 64);
    }
  }
  // lane = co_local * 8 + ci
  atomicAdd(dw + ((int64_t)(co0 + (lane >> 3)) * 9 + tap) * CI + (lane & 7), acc[0]);  // KRSC [Co][3][3][Cin]
}

bool stem_bwd32_ok(int N, int H, int W, int Cin, int Co) {
  return N > 0 && N < (1 << 24) && H == 32 && W == 32 && Cin == 8 && Co == 64;
}

template <typename T>
static void stem_bwd_launch(const BnBwdArgs32& a, const T* x, int N, float* dw, hipStream_t s, const OptTail* ot) {
  const OptTail tail = ot ? *ot : OptTail{};
  const size_t lds = ((size_t)32 * 32 * kStemCG + (size_t)34 * 34 * 8 + 5 * kStemCG) * sizeof(float);
  static bool init = false;
  if (!init) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_bwd32_kernel<T>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    init = true;
  }
  stem_bwd32_kernel<T><<<(unsigned)(N * (64 / kStemCG) + tail.nblk), 576, lds, s>>>(a, x, N, dw, tail);
}

void launch_stem_bwd32(const BnBwdArgs32& a, const float* x, int N, int H, int W, int Cin, float* dw, hipStream_t s,
                       const OptTail* ot) {
  (void)H;
  (void)W;
  (void)Cin;
  stem_bwd_launch(a, x, N, dw, s, ot);
}

void launch_stem_bwd_bf16(const BnBwdArgs32& a, const uint16_t* x, int N, float* dw, hipStream_t s,
                          const OptTail* ot) {
  stem_bwd_launch(a, x, N, dw, s, ot);
}

void launch_bn32_bwd_apply_pair(const BnBwdArgs32& a1, const BnBwdArgs32& a2, hipStream_t s) {
  const int64_t n1 = a1.M * a1.C / 4, n2 = a2.M * a2.C / 4;
  const unsigned g1 = apply_grid(n1), g2 = apply_grid(n2);
  const size_t sm = 5 * (size_t)(a1.C > a2.C ? a1.C : a2.C) * sizeof(float);
  bn32_bwd_apply_pair_kernel<<<g1 + g2, 256, sm, s>>>(a1, n1, (int)g1, a2, n2);
}

void launch_bn32_bwd_apply(const BnBwdArgs32& a, hipStream_t s) {
  const int64_t nvec = a.M * a.C / 4;
  const unsigned g = apply_grid(nvec);
  const size_t sm = 5 * a.C * sizeof(float);
  if (a.y) {
    if (a.dy_masked) bn32_bwd_apply_kernel<true, true><<<g, 256, sm, s>>>(a, nvec);
    else bn32_bwd_apply_kernel<true, false><<<g, 256, sm, s>>>(a, nvec);
  } else {
    if (a.dy_masked) bn32_bwd_apply_kernel<false, true><<<g, 256, sm, s>>>(a, nvec);
    else bn32_bwd_apply_kernel<false, false><<<g, 256, sm, s>>>(a, nvec);
  }
}

void set_bn32_grid_cap(int cap) { g_bn32_grid = cap > 0 ? cap : MFL_BN32_GRID; }

}  // namespace mfl
