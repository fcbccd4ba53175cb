// K6: NHWC bf16 convolution forward / backward-data / backward-weight as
// implicit GEMMs on the gfx950 matrix cores (v_mfma_f32_16x16x32_bf16).
//
// The reference trains its conv nets through Keras Conv2D layers
// (examples/keras/models/cifar_cnn.py:21-34); the north-star replaces that
// with hand-written CDNA4 kernels.  Design (MI355X-first, not a port):
//
//  * Activations NHWC, weights KRSC ([Cout][R][S][Cin]) so that the GEMM
//    reduction dimension k = (r, s, c) is contiguous in BOTH operands for the
//    forward pass: every lane fetches 16 B (8 channels) per load, and MFMA
//    operand fragments (8 consecutive k per lane) are read from LDS with one
//    ds_read_b128.  Cin must be a multiple of 8 (the 3-channel CIFAR input is
//    zero-padded to 8 channels once, at shard creation).
//  * dgrad is the same kernel with a stride-aware gather of dY; its B operand
//    (W^T) is staged from the KRSC weight as [k][c] tiles and read with the
//    transposing ds_read_b64_tr_b16, so no weight transpose pass exists.
//  * wgrad reduces over the N*P*Q pixels, which are strided in both operands:
//    tiles are staged [m][col] in LDS and the MFMA fragments are formed with
//    the gfx950 transposing LDS read ds_read_b64_tr_b16 (guide T10).
//  * Tiles: 256-thread workgroups (4 waves, 2x2), BK = 64, LDS rows padded to
//    144 B so that a 16-lane ds_read_b128 group touches 16 distinct 4-bank
//    slots (conflict-free, guide Guideline 4), register-staged double
//    buffering with one barrier per k-step (guide T14 / "minimum 2-phase").
//  * Small-M layers (CIFAR 4x4/8x8 stages) use split-K so a launch still
//    fills >= 256 CUs; the split reduction kernel also emits the per-channel
//    BatchNorm sums, and the non-split epilogue emits them directly (fp64
//    atomics into a [2][C] accumulator), so BN never re-reads the conv output
//    for statistics.  wgrad split-K slices accumulate with fp32 atomics into
//    the (pre-zeroed) flat gradient buffer: no reduction launch.
#include "kernels/common.h"
#include "kernels/conv.h"

namespace mfl {

constexpr int kBK = 64;
constexpr int kPad = 8;                 // elements of row padding (16 B)
constexpr int kLdsStride = kBK + kPad;  // 72 bf16 = 144 B

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// Forward / dgrad implicit GEMM:  Y[m][n] = sum_k A[m][k] * B[n][k]
template <int BM, int BN, bool DGRAD>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvGeom g, const uint16_t* __restrict__ src,
                                                        const uint16_t* __restrict__ wgt,
                                                        uint16_t* __restrict__ y,
                                                        float* __restrict__ ysplit,
                                                        double* __restrict__ stats, int kchunk,
                                                        int accum) {
  constexpr int ACH = BM / 32;  // A 16-B chunks per thread per k-step
  constexpr int BCH = BN / 32;
  constexpr int TM = BM / 32;   // 16x16 MFMA tiles per wave along M
  constexpr int TN = BN / 32;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  // buffer b: A tile at smem + b*STAGE, B tile right after it.  Forward: B is
  // [BN][BK] (k-contiguous weight rows).  dgrad: B is staged [BK][BN] straight
  // from the KRSC weight (c-contiguous) and read with ds_read_b64_tr_b16, so no
  // per-step weight transpose is needed.
  constexpr int BST = BN + kPad;
  constexpr int BTILE = DGRAD ? kBK * BST : BN * kLdsStride;
  constexpr int STAGE = BM * kLdsStride + BTILE;
  auto As = [&](int b) { return smem + b * STAGE; };
  auto Bs = [&](int b) { return smem + b * STAGE + BM * kLdsStride; };
  constexpr int BCPR = BN / 8;       // dgrad B: 16-B chunks per k-row
  constexpr int BRPP = 256 / BCPR;   // k-rows per pass
  const int dbch = threadIdx.x % BCPR, dbrow = threadIdx.x / BCPR;

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(g.K, kbeg + kchunk);
  const int nk = (kend - kbeg + kBK - 1) / kBK;

  const int lrow = t >> 3;   // 0..31
  const int lch = t & 7;     // chunk within the BK=64 row
  const int HWC = g.H * g.W * g.C;

  // Per-thread A rows: image base, origin coordinates.
  int a_nb[ACH], a_y0[ACH], a_x0[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int m = m0 + lrow + 32 * i;
    if (m < g.M) {
      const int pq = g.P * g.Q;
      const int n = m / pq;
      const int rem = m - n * pq;
      const int oy = rem / g.Q;
      const int ox = rem - oy * g.Q;
      a_nb[i] = n * HWC;
      if (DGRAD) {
        a_y0[i] = oy + g.pad;
        a_x0[i] = ox + g.pad;
      } else {
        a_y0[i] = oy * g.stride - g.pad;
        a_x0[i] = ox * g.stride - g.pad;
      }
    } else {
      a_nb[i] = 0;
      a_y0[i] = -(1 << 28);
      a_x0[i] = -(1 << 28);
    }
  }

  uint4 ra[ACH], rb[BCH];
  auto load_tile = [&](int kt) {
    const int k = kbeg + kt * kBK + lch * 8;
    const bool kv = k < kend;
    int r = 0, s = 0, c = 0;
    if (kv) {
      const int rs = k / g.C;
      c = k - rs * g.C;
      r = rs / g.S;
      s = rs - r * g.S;
    }
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int iy, ix;
      bool ok = kv;
      if (DGRAD) {
        const int ty = a_y0[i] - r, tx = a_x0[i] - s;
        ok = ok && ty >= 0 && tx >= 0;
        if (g.stride > 1) ok = ok && (ty % g.stride == 0) && (tx % g.stride == 0);
        iy = ty / g.stride;
        ix = tx / g.stride;
      } else {
        iy = a_y0[i] + r;
        ix = a_x0[i] + s;
        ok = ok && iy >= 0 && ix >= 0;
      }
      ok = ok && iy < g.H && ix < g.W;
      if (ok)
        ra[i] = *reinterpret_cast<const uint4*>(src + a_nb[i] + (iy * g.W + ix) * g.C + c);
      else
        ra[i] = make_uint4(0, 0, 0, 0);
    }
    if constexpr (DGRAD) {
      // B[k][n] = W[ko][r][s][n], k = (r, s, ko): rows of the tile are k
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const int kr = kbeg + kt * kBK + dbrow + BRPP * i;
        const int n = n0 + dbch * 8;
        if (kr < kend && n < g.Ng) {
          const int rs = kr / g.C;
          const int ko = kr - rs * g.C;
          rb[i] = *reinterpret_cast<const uint4*>(wgt + ((int64_t)ko * g.R * g.S + rs) * g.Ng + n);
        } else {
          rb[i] = make_uint4(0, 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const int n = n0 + lrow + 32 * i;
        if (kv && n < g.Ng)
          rb[i] = *reinterpret_cast<const uint4*>(wgt + (int64_t)n * g.K + k);
        else
          rb[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < ACH; ++i)
      *reinterpret_cast<uint4*>(As(buf) + (lrow + 32 * i) * kLdsStride + lch * 8) = ra[i];
    if constexpr (DGRAD) {
#pragma unroll
      for (int i = 0; i < BCH; ++i)
        *reinterpret_cast<uint4*>(Bs(buf) + (dbrow + BRPP * i) * BST + dbch * 8) = rb[i];
    } else {
#pragma unroll
      for (int i = 0; i < BCH; ++i)
        *reinterpret_cast<uint4*>(Bs(buf) + (lrow + 32 * i) * kLdsStride + lch * 8) = rb[i];
    }
  };
  typedef short v4s __attribute__((ext_vector_type(4)));

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();
  const int fr = lane & 15;
  const int fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile(kt + 1);
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 32) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As(cur) + (wm * (BM / 2) + 16 * i + fr) * kLdsStride + kk + fk);
      if constexpr (DGRAD) {
        const int grp = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wn * (BN / 2) + 16 * j + 4 * tp;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int row = kk + 8 * grp + 4 * h + tq;
            const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) v4s*)(Bs(cur) + row * BST + col));
            bfr[j][4 * h + 0] = v[0];
            bfr[j][4 * h + 1] = v[1];
            bfr[j][4 * h + 2] = v[2];
            bfr[j][4 * h + 3] = v[3];
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(Bs(cur) + (wn * (BN / 2) + 16 * j + fr) * kLdsStride + kk + fk);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue -----------------------------------------------------------
  const int rbase = m0 + wm * (BM / 2) + (lane >> 4) * 4;
  const int cbase = n0 + wn * (BN / 2) + fr;
  if (ysplit) {
    float* out = ysplit + (int64_t)blockIdx.z * g.M * g.Ng;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = rbase + 16 * i + e, col = cbase + 16 * j;
          if (row < g.M && col < g.Ng) out[(int64_t)row * g.Ng + col] = acc[i][j][e];
        }
    return;
  }
  float cs[TN], cq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) { cs[j] = 0.f; cq[j] = 0.f; }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rbase + 16 * i + e, col = cbase + 16 * j;
        if (row < g.M && col < g.Ng) {
          float a = acc[i][j][e];
          if (accum) a += bf2f(y[(int64_t)row * g.Ng + col]);
          const uint16_t h = f2bf(a);
          y[(int64_t)row * g.Ng + col] = h;
          const float v = bf2f(h);
          cs[j] += v;
          cq[j] += v * v;
        }
      }
  if (!stats) return;
  // lanes l, l^16, l^32, l^48 share a column
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    cs[j] += __shfl_xor(cs[j], 16, 64);
    cs[j] += __shfl_xor(cs[j], 32, 64);
    cq[j] += __shfl_xor(cq[j], 16, 64);
    cq[j] += __shfl_xor(cq[j], 32, 64);
  }
  float* red = reinterpret_cast<float*>(smem);  // [2 wm][2][BN]
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = wn * (BN / 2) + 16 * j + lane;
      red[(wm * 2 + 0) * BN + cl] = cs[j];
      red[(wm * 2 + 1) * BN + cl] = cq[j];
    }
  }
  __syncthreads();
  for (int cl = t; cl < BN; cl += 256) {
    const int col = n0 + cl;
    if (col < g.Ng) {
      atomicAdd(&stats[col], (double)(red[0 * BN + cl] + red[2 * BN + cl]));
      atomicAdd(&stats[g.Ng + col], (double)(red[1 * BN + cl] + red[3 * BN + cl]));
    }
  }
}

// ---------------------------------------------------------------------------
// Split-K reduction: y = bf16(sum_z ysplit[z]) and per-block BN partials.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ysplit,
                                                            int splits, int M, int C,
                                                            uint16_t* __restrict__ y,
                                                            double* __restrict__ stats, int accum) {
  const int tpr = C / 8;
  const int rpp = 256 / tpr;
  const int t = threadIdx.x;
  const int cg = t % tpr;
  const int r0 = t / tpr;
  float s[8] = {0}, q[8] = {0};
  const int64_t MC = (int64_t)M * C;
  if (r0 < rpp) {
    for (int64_t row = (int64_t)blockIdx.x * rpp + r0; row < M; row += (int64_t)gridDim.x * rpp) {
      float v[8] = {0};
      const int64_t off = row * C + cg * 8;
      for (int z = 0; z < splits; ++z) {
        const float4 a = *reinterpret_cast<const float4*>(ysplit + z * MC + off);
        const float4 b = *reinterpret_cast<const float4*>(ysplit + z * MC + off + 4);
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
        v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
      }
      if (accum) {
        float old[8];
        unpack8(*reinterpret_cast<const uint4*>(y + off), old);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += old[k];
      }
      const uint4 o = pack8(v);
      *reinterpret_cast<uint4*>(y + off) = o;
      float f[8];
      unpack8(o, f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += f[k];
        q[k] += f[k] * f[k];
      }
    }
  }
  if (!stats) return;
  __shared__ float sh[2][256 * 8];
  const bool act = r0 < rpp;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sh[0][t * 8 + k] = act ? s[k] : 0.f;
    sh[1][t * 8 + k] = act ? q[k] : 0.f;
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float s0 = 0.f, s1 = 0.f;
    for (int r = 0; r < rpp; ++r) {
      s0 += sh[0][(r * tpr + (c >> 3)) * 8 + (c & 7)];
      s1 += sh[1][(r * tpr + (c >> 3)) * 8 + (c & 7)];
    }
    atomicAdd(&stats[c], (double)s0);
    atomicAdd(&stats[C + c], (double)s1);
  }
}

// ---------------------------------------------------------------------------
// wgrad:  dW[ko][j] = sum_m dY[m][ko] * im2col(X)[m][j],  j = (r, s, c)
template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvGeom g, const uint16_t* __restrict__ x,
                                                         const uint16_t* __restrict__ dy,
                                                         float* __restrict__ dw, int mchunk) {
  // g: H,W,C = X dims; P,Q = dY spatial; Ng = Cout; K = R*S*C; M = N*P*Q
  constexpr int TM = BM / 32;
  constexpr int TN = BN / 32;
  constexpr int AST = BM + kPad;
  constexpr int BST = BN + kPad;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int STAGE = kBK * (AST + BST);
  auto As = [&](int b) { return smem + b * STAGE; };
  auto Bs = [&](int b) { return smem + b * STAGE + kBK * AST; };

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int ko0 = blockIdx.x * BM;
  const int j0 = blockIdx.y * BN;
  const int mbeg = blockIdx.z * mchunk;
  const int mend = min(g.M, mbeg + mchunk);
  const int nk = (mend - mbeg + kBK - 1) / kBK;

  // Load mapping: a [64 m][BN] tile has BN/8 16-B chunks per row, so each
  // thread owns one fixed column chunk and rows brow + BRPP*i; the im2col
  // decomposition (r, s, c) of that column chunk is fixed for the k-loop.
  constexpr int BCPR = BN / 8;
  constexpr int BRPP = 256 / BCPR;
  constexpr int BREP = kBK / BRPP;  // row repetitions
  constexpr int ACPR = BM / 8;
  constexpr int ARPP = 256 / ACPR;
  constexpr int AREP = kBK / ARPP;
  static_assert(BREP * BRPP == kBK && AREP * ARPP == kBK, "tile mapping");
  const int bch = t % BCPR, brow = t / BCPR;
  const int ach = t % ACPR, arow = t / ACPR;
  int b_r, b_s, b_c;
  bool b_ok;
  {
    const int j = j0 + bch * 8;
    b_ok = j < g.K;
    const int rs = b_ok ? j / g.C : 0;
    b_c = b_ok ? j - rs * g.C : 0;
    b_r = b_ok ? rs / g.S : 0;
    b_s = b_ok ? rs - b_r * g.S : 0;
  }
  const int HWC = g.H * g.W * g.C;
  uint4 ra[AREP], rb[BREP];
  auto load_tile = [&](int kt) {
    const int mb = mbeg + kt * kBK;
#pragma unroll
    for (int i = 0; i < AREP; ++i) {
      const int m = mb + arow + ARPP * i;
      const int ko = ko0 + ach * 8;
      if (m < mend && ko < g.Ng)
        ra[i] = *reinterpret_cast<const uint4*>(dy + (int64_t)m * g.Ng + ko);
      else
        ra[i] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BREP; ++i) {
      const int m = mb + brow + BRPP * i;
      bool ok = b_ok && m < mend;
      int n = 0, iy = 0, ix = 0;
      if (ok) {
        const int pq = g.P * g.Q;
        n = m / pq;
        const int rem = m - n * pq;
        const int oy = rem / g.Q;
        const int ox = rem - oy * g.Q;
        iy = oy * g.stride - g.pad + b_r;
        ix = ox * g.stride - g.pad + b_s;
        ok = iy >= 0 && ix >= 0 && iy < g.H && ix < g.W;
      }
      if (ok)
        rb[i] = *reinterpret_cast<const uint4*>(x + (int64_t)n * HWC + (iy * g.W + ix) * g.C + b_c);
      else
        rb[i] = make_uint4(0, 0, 0, 0);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AREP; ++i)
      *reinterpret_cast<uint4*>(As(buf) + (arow + ARPP * i) * AST + ach * 8) = ra[i];
#pragma unroll
    for (int i = 0; i < BREP; ++i)
      *reinterpret_cast<uint4*>(Bs(buf) + (brow + BRPP * i) * BST + bch * 8) = rb[i];
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();
  const int grp = lane >> 4;  // 0..3 -> k = 8*grp + e
  const int li = lane & 15;
  const int tq = li >> 2, tp = li & 3;
  typedef short v4s __attribute__((ext_vector_type(4)));
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile(kt + 1);
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 32) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * (BM / 2) + 16 * i + 4 * tp;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = kk + 8 * grp + 4 * h + tq;
          const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(As(cur) + row * AST + col));
          af[i][4 * h + 0] = v[0];
          af[i][4 * h + 1] = v[1];
          af[i][4 * h + 2] = v[2];
          af[i][4 * h + 3] = v[3];
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / 2) + 16 * j + 4 * tp;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int row = kk + 8 * grp + 4 * h + tq;
          const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4s*)(Bs(cur) + row * BST + col));
          bfr[j][4 * h + 0] = v[0];
          bfr[j][4 * h + 1] = v[1];
          bfr[j][4 * h + 2] = v[2];
          bfr[j][4 * h + 3] = v[3];
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }
  const bool atomic = gridDim.z > 1;  // split-K slices add into the zeroed slot
  const int rbase = ko0 + wm * (BM / 2) + (lane >> 4) * 4;
  const int cbase = j0 + wn * (BN / 2) + li;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rbase + 16 * i + e, col = cbase + 16 * j;
        if (row < g.Ng && col < g.K) {
          if (atomic)
            atomicAdd(&dw[(int64_t)row * g.K + col], acc[i][j][e]);
          else
            dw[(int64_t)row * g.K + col] = acc[i][j][e];
        }
      }
}

// [Cout][R][S][Cin] -> [Cin][R][S][Cout]  (dgrad weight layout)
__global__ __launch_bounds__(256) void transpose_krsc_kernel(const uint16_t* __restrict__ w,
                                                             uint16_t* __restrict__ wt, int Co,
                                                             int RS, int Ci) {
  const int64_t n = (int64_t)Co * RS * Ci;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    // output index i -> (ci, rs, co)
    const int co = (int)(i % Co);
    const int64_t t2 = i / Co;
    const int rs = (int)(t2 % RS);
    const int ci = (int)(t2 / RS);
    wt[i] = w[((int64_t)co * RS + rs) * Ci + ci];
  }
}

// ---------------------------------------------------------------------------
template <int BM, int BN, bool DG>
static void launch_gemm_t(const ConvGeom& g, const uint16_t* src, const uint16_t* wgt, uint16_t* y,
                          float* ysplit, double* stats, int splits, int kchunk, int accum,
                          hipStream_t s) {
  dim3 grid((g.M + BM - 1) / BM, (g.Ng + BN - 1) / BN, splits);
  const size_t btile = DG ? (size_t)kBK * (BN + kPad) : (size_t)BN * kLdsStride;
  const size_t lds = (size_t)2 * ((size_t)BM * kLdsStride + btile) * sizeof(uint16_t);
  static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into
  if (!attr_set && lds > 65536) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_gemm_kernel<BM, BN, DG>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  conv_gemm_kernel<BM, BN, DG><<<grid, 256, lds, s>>>(g, src, wgt, y, ysplit, stats, kchunk, accum);
}

ConvPlan plan_conv_gemm(const ConvGeom& g) {
  ConvPlan p;
  p.bm = g.M >= 8192 ? 128 : 64;
  p.bn = g.Ng >= 128 && g.M >= 8192 ? 128 : 64;
  if (p.bm == 128 && p.bn == 128 && g.M < 16384) p.bn = 64;
  const int tiles = ((g.M + p.bm - 1) / p.bm) * ((g.Ng + p.bn - 1) / p.bn);
  const int ksteps = (g.K + kBK - 1) / kBK;
  int splits = 1;
  while (tiles * splits < 256 && ksteps / (splits * 2) >= 4 && splits < 16) splits *= 2;
  p.splits = splits;
  p.kchunk = ((ksteps + splits - 1) / splits) * kBK;
  p.stats_rows = splits > 1 ? 0 : (g.M + p.bm - 1) / p.bm;
  return p;
}

void launch_conv_gemm(const ConvGeom& g, bool dgrad, const ConvPlan& p, const uint16_t* src,
                      const uint16_t* wgt, uint16_t* y, float* ysplit, double* stats, bool accum,
                      hipStream_t s) {
  const int ac = accum ? 1 : 0;
  float* ys = p.splits > 1 ? ysplit : nullptr;
  double* st = p.splits > 1 ? nullptr : stats;
#define MFL_CONV_CASE(BM_, BN_)                                                                \
  if (p.bm == BM_ && p.bn == BN_) {                                                            \
    if (dgrad) launch_gemm_t<BM_, BN_, true>(g, src, wgt, y, ys, st, p.splits, p.kchunk, ac, s);   \
    else launch_gemm_t<BM_, BN_, false>(g, src, wgt, y, ys, st, p.splits, p.kchunk, ac, s);        \
  }
  MFL_CONV_CASE(128, 128)
  MFL_CONV_CASE(128, 64)
  MFL_CONV_CASE(64, 128)
  MFL_CONV_CASE(64, 64)
#undef MFL_CONV_CASE
  if (p.splits > 1) {
    const int nb = splitk_stats_blocks(g.M, g.Ng);
    splitk_reduce_kernel<<<nb, 256, 0, s>>>(ysplit, p.splits, g.M, g.Ng, y, stats, ac);
  }
}

int splitk_stats_blocks(int M, int C) {
  const int tpr = C / 8;
  const int rpp = 256 / tpr;
  int nb = (M + rpp * 4 - 1) / (rpp * 4);
  return nb < 1 ? 1 : (nb > 512 ? 512 : nb);
}

ConvPlan plan_conv_wgrad(const ConvGeom& g) {
  ConvPlan p;
  p.bm = 64;
  p.bn = 64;
  const int tiles = ((g.Ng + 63) / 64) * ((g.K + 63) / 64);
  const int ksteps = (g.M + kBK - 1) / kBK;
  int splits = 1;
  while (tiles * splits < 512 && ksteps / (splits * 2) >= 8 && splits < 64) splits *= 2;
  p.splits = splits;
  p.kchunk = ((ksteps + splits - 1) / splits) * kBK;
  p.stats_rows = 0;
  return p;
}

// dw must be zero on entry when p.splits > 1 (slices accumulate with fp32
// atomics); the training step gets that for free from the optimizer launch,
// which zeroes the gradient buffer after consuming it.
void launch_conv_wgrad(const ConvGeom& g, const ConvPlan& p, const uint16_t* x, const uint16_t* dy,
                       float* dw, hipStream_t s) {
  dim3 grid((g.Ng + 63) / 64, (g.K + 63) / 64, p.splits);
  const size_t lds = (size_t)2 * kBK * ((64 + kPad) + (64 + kPad)) * sizeof(uint16_t);
  conv_wgrad_kernel<64, 64><<<grid, 256, lds, s>>>(g, x, dy, dw, p.kchunk);
}

void launch_transpose_krsc(const uint16_t* w, uint16_t* wt, int Co, int RS, int Ci, hipStream_t s) {
  const int64_t n = (int64_t)Co * RS * Ci;
  transpose_krsc_kernel<<<stream_grid(n, 256, 4096), 256, 0, s>>>(w, wt, Co, RS, Ci);
}

}  // namespace mfl
