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
//    ds_read_b64_tr_b16 (guide T10).
//  * Index math is kept off the VALU critical path: kernel size and stride are
//    template parameters (constant divisions), channel / spatial divisions by
//    powers of two become shifts (host-computed, wave-uniform).  Round-1
//    profiling showed the generic version spending more VALU cycles on
//    integer division than the MFMAs took.
//  * Tiles: 256-thread workgroups (4 waves, 2x2), BK = 64, LDS rows padded to
//    144 B so that a 16-lane ds_read_b128 group touches 16 distinct 4-bank
//    slots (conflict-free, guide Guideline 4), register-staged double
//    buffering with one barrier per k-step (guide T14 / "minimum 2-phase").
//  * Epilogue through LDS: the fp32 tile is staged in LDS and written as 16-B
//    bf16 vectors; the per-channel BatchNorm sums of the bf16 output are
//    reduced in the same pass and added with fp64 atomics into a [2][C]
//    accumulator (no separate statistics pass).
//  * Small-M layers (CIFAR 4x4 / 8x8 stages) use split-K to fill >= 256 CUs.
//    The reduction happens IN the kernel: every slice stores its fp32 tile
//    slab, then the last-arriving slice (agent-scope release/acquire counter,
//    guide "In-launch split-K reduction") sums the slabs and runs the
//    epilogue -- no reduction launch.  wgrad split-K slices accumulate with
//    fp32 atomics into the pre-zeroed gradient buffer.
#include "kernels/common.h"
#include "kernels/conv.h"

namespace mfl {

constexpr int kBK = 64;
constexpr int kPad = 8;                 // elements of row padding (16 B)
constexpr int kLdsStride = kBK + kPad;  // 72 bf16 = 144 B

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int sdiv(int x, int d, int shift) { return shift >= 0 ? x >> shift : x / d; }

// Vectorised epilogue shared by the direct and the split-K paths:
// out[row][col] = bf16(v (+ y_old)), BN sums of the rounded output.
// `get(row_local, col_local_base, float[8])` supplies 8 consecutive fp32 values.
template <int BM, int BN, typename Getter>
__device__ __forceinline__ void tile_epilogue(const ConvGeom& g, int m0, int n0, uint16_t* y,
                                              double* stats, int accum, float* red, Getter get) {
  constexpr int CPR = BN / 8;        // 16-B column groups per row
  constexpr int RPP = 256 / CPR;     // rows per pass
  const int t = threadIdx.x;
  const int cg = t % CPR, r0 = t / CPR;
  float s[8] = {0}, q[8] = {0};
  const int col = n0 + cg * 8;
  const bool col_ok = col < g.Ng;  // Ng % 8 == 0
  for (int rl = r0; rl < BM; rl += RPP) {
    const int row = m0 + rl;
    if (row >= g.M || !col_ok) continue;
    float v[8];
    get(rl, cg * 8, v);
    uint16_t* dst = y + (int64_t)row * g.Ng + col;
    if (accum) {
      float o[8];
      unpack8(*reinterpret_cast<const uint4*>(dst), o);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += o[k];
    }
    const uint4 packed = pack8(v);
    *reinterpret_cast<uint4*>(dst) = packed;
    if (stats) {
      float f[8];
      unpack8(packed, f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += f[k];
        q[k] += f[k] * f[k];
      }
    }
  }
  if (!stats) return;
  __syncthreads();  // `red` aliases LDS that `get` may have been reading
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[t * 16 + k] = s[k];
    red[t * 16 + 8 + k] = q[k];
  }
  __syncthreads();
  if (t < BN) {
    const int cgi = t >> 3, k = t & 7;
    float a = 0.f, b = 0.f;
    for (int r = 0; r < RPP; ++r) {
      a += red[(r * CPR + cgi) * 16 + k];
      b += red[(r * CPR + cgi) * 16 + 8 + k];
    }
    const int c = n0 + t;
    if (c < g.Ng) {
      atomicAdd(&stats[c], (double)a);
      atomicAdd(&stats[g.Ng + c], (double)b);
    }
  }
}

// ---------------------------------------------------------------------------
// Forward / dgrad implicit GEMM:  Y[m][n] = sum_k A[m][k] * B[n][k]
template <int BM, int BN, bool DGRAD, int KS, int ST>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
  constexpr int ACH = BM / 32;  // A 16-B chunks per thread per k-step
  constexpr int BCH = BN / 32;
  constexpr int TM = BM / 32;   // 16x16 MFMA tiles per wave along M
  constexpr int TN = BN / 32;
  const ConvGeom& g = a.g;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  // buffer b: A tile at smem + b*STAGE, B tile right after it.  Forward: B is
  // [BN][BK] (k-contiguous weight rows).  dgrad: B is [BK][BN] staged from the
  // KRSC weight (c-contiguous) and read with ds_read_b64_tr_b16.
  constexpr int BST = BN + kPad;
  constexpr int BTILE = DGRAD ? kBK * BST : BN * kLdsStride;
  constexpr int STAGE = BM * kLdsStride + BTILE;
  auto As = [&](int b) { return smem + b * STAGE; };
  auto Bs = [&](int b) { return smem + b * STAGE + BM * kLdsStride; };
  constexpr int BCPR = BN / 8;       // dgrad B: 16-B chunks per k-row
  constexpr int BRPP = 256 / BCPR;   // k-rows per pass

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wv = t >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int kbeg = blockIdx.z * a.kchunk;
  const int kend = min(g.K, kbeg + a.kchunk);
  const int nk = (kend - kbeg + kBK - 1) / kBK;
  const int dbch = t % BCPR, dbrow = t / BCPR;

  const int lrow = t >> 3;   // 0..31
  const int lch = t & 7;     // chunk within the BK=64 row
  const int HWC = g.H * g.W * g.C;

  // Per-thread A rows: image base, origin coordinates.
  int a_nb[ACH], a_y0[ACH], a_x0[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int m = m0 + lrow + 32 * i;
    if (m < g.M) {
      const int n = sdiv(m, g.P * g.Q, a.pq_shift);
      const int rem = m - n * g.P * g.Q;
      const int oy = sdiv(rem, g.Q, a.q_shift);
      const int ox = rem - oy * g.Q;
      a_nb[i] = n * HWC;
      if (DGRAD) {
        a_y0[i] = oy + g.pad;
        a_x0[i] = ox + g.pad;
      } else {
        a_y0[i] = oy * ST - g.pad;
        a_x0[i] = ox * ST - g.pad;
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
      const int rs = sdiv(k, g.C, a.c_shift);
      c = k - rs * g.C;
      r = rs / KS;
      s = rs - r * KS;
    }
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int iy, ix;
      bool ok = kv;
      if (DGRAD) {
        const int ty = a_y0[i] - r, tx = a_x0[i] - s;
        ok = ok && ty >= 0 && tx >= 0;
        if (ST > 1) ok = ok && (ty % ST == 0) && (tx % ST == 0);
        iy = ty / ST;
        ix = tx / ST;
      } else {
        iy = a_y0[i] + r;
        ix = a_x0[i] + s;
        ok = ok && iy >= 0 && ix >= 0;
      }
      ok = ok && iy < g.H && ix < g.W;
      if (ok)
        ra[i] = *reinterpret_cast<const uint4*>(a.src + a_nb[i] + (iy * g.W + ix) * g.C + c);
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
          const int rs = sdiv(kr, g.C, a.c_shift);
          const int ko = kr - rs * g.C;
          rb[i] = *reinterpret_cast<const uint4*>(a.wgt + ((int64_t)ko * KS * KS + rs) * g.Ng + n);
        } else {
          rb[i] = make_uint4(0, 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const int n = n0 + lrow + 32 * i;
        if (kv && n < g.Ng)
          rb[i] = *reinterpret_cast<const uint4*>(a.wgt + (int64_t)n * g.K + k);
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
  // fp32 tile in LDS: [BM][BN + 4] (the loop's final barrier freed smem)
  constexpr int TST = BN + 4;
  float* tile = reinterpret_cast<float*>(smem);
  const int rl0 = wm * (BM / 2) + (lane >> 4) * 4;
  const int cl0 = wn * (BN / 2) + fr;
  const int splits = gridDim.z;
  const int tile_id = blockIdx.y * gridDim.x + blockIdx.x;
  if (splits == 1) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) tile[(rl0 + 16 * i + e) * TST + cl0 + 16 * j] = acc[i][j][e];
    __syncthreads();
    tile_epilogue<BM, BN>(g, m0, n0, a.y, a.stats, a.accum, tile + BM * TST,
                          [&](int rl, int cl, float* v) {
                            const float4 p = *reinterpret_cast<const float4*>(tile + rl * TST + cl);
                            const float4 q = *reinterpret_cast<const float4*>(tile + rl * TST + cl + 4);
                            v[0] = p.x; v[1] = p.y; v[2] = p.z; v[3] = p.w;
                            v[4] = q.x; v[5] = q.y; v[6] = q.z; v[7] = q.w;
                          });
    return;
  }
  // split-K: store this slice's slab [BM][BN] (tile-local, row-major)
  const int ntiles = gridDim.x * gridDim.y;
  float* slab = a.ysplit + ((int64_t)blockIdx.z * ntiles + tile_id) * (BM * BN);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) slab[(rl0 + 16 * i + e) * BN + cl0 + 16 * j] = acc[i][j][e];
  // publish: every wave drains its stores, one agent-scope release, then the
  // ticket; the last slice to arrive reduces (guide: In-launch split-K).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(&a.counters[tile_id], 1, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == splits - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // re-arm for the next launch (graph replay): nobody else touches it now
      __hip_atomic_store(&a.counters[tile_id], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    flag[0] = last;
  }
  __syncthreads();
  if (!flag[0]) return;
  const float* base = a.ysplit + (int64_t)tile_id * (BM * BN);
  const int64_t zstride = (int64_t)ntiles * BM * BN;
  tile_epilogue<BM, BN>(g, m0, n0, a.y, a.stats, a.accum, reinterpret_cast<float*>(smem) + 4,
                        [&](int rl, int cl, float* v) {
                          for (int k = 0; k < 8; ++k) v[k] = 0.f;
                          for (int z = 0; z < splits; ++z) {
                            const float* p = base + z * zstride + rl * BN + cl;
                            const float4 x0 = *reinterpret_cast<const float4*>(p);
                            const float4 x1 = *reinterpret_cast<const float4*>(p + 4);
                            v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
                            v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
                          }
                        });
}

// ---------------------------------------------------------------------------
// wgrad:  dW[ko][j] = sum_m dY[m][ko] * im2col(X)[m][j],  j = (r, s, c)
template <int BM, int BN, int KS, int ST>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvArgs a, float* __restrict__ dw) {
  // g: H,W,C = X dims; P,Q = dY spatial; Ng = Cout; K = R*S*C; M = N*P*Q
  constexpr int TM = BM / 32;
  constexpr int TN = BN / 32;
  constexpr int AST = BM + kPad;
  constexpr int BST = BN + kPad;
  const ConvGeom& g = a.g;
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
  const int mbeg = blockIdx.z * a.kchunk;
  const int mend = min(g.M, mbeg + a.kchunk);
  const int nk = (mend - mbeg + kBK - 1) / kBK;

  // A [64 m][BM] and B [64 m][BN] tiles: each thread owns one fixed 16-B
  // column chunk and rows row + RPP*i; the im2col decomposition (r, s, c) of
  // the B column chunk is fixed for the whole k-loop.
  constexpr int BCPR = BN / 8;
  constexpr int BRPP = 256 / BCPR;
  constexpr int BREP = kBK / BRPP;
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
    const int rs = b_ok ? sdiv(j, g.C, a.c_shift) : 0;
    b_c = b_ok ? j - rs * g.C : 0;
    b_r = rs / KS;
    b_s = rs - b_r * KS;
  }
  const int HWC = g.H * g.W * g.C;
  const int PQ = g.P * g.Q;
  uint4 ra[AREP], rb[BREP];
  auto load_tile = [&](int kt) {
    const int mb = mbeg + kt * kBK;
#pragma unroll
    for (int i = 0; i < AREP; ++i) {
      const int m = mb + arow + ARPP * i;
      const int ko = ko0 + ach * 8;
      if (m < mend && ko < g.Ng)
        ra[i] = *reinterpret_cast<const uint4*>(a.src + (int64_t)m * g.Ng + ko);  // src = dY
      else
        ra[i] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BREP; ++i) {
      const int m = mb + brow + BRPP * i;
      bool ok = b_ok && m < mend;
      int n = 0, iy = 0, ix = 0;
      if (ok) {
        n = sdiv(m, PQ, a.pq_shift);
        const int rem = m - n * PQ;
        const int oy = sdiv(rem, g.Q, a.q_shift);
        const int ox = rem - oy * g.Q;
        iy = oy * ST - g.pad + b_r;
        ix = ox * ST - g.pad + b_s;
        ok = iy >= 0 && ix >= 0 && iy < g.H && ix < g.W;
      }
      if (ok)
        rb[i] = *reinterpret_cast<const uint4*>(a.wgt + (int64_t)n * HWC + (iy * g.W + ix) * g.C + b_c);  // wgt = X
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

// [Cout][R][S][Cin] -> [Cin][R][S][Cout]  (layout utility, not on the hot path)
__global__ __launch_bounds__(256) void transpose_krsc_kernel(const uint16_t* __restrict__ w,
                                                             uint16_t* __restrict__ wt, int Co,
                                                             int RS, int Ci) {
  const int64_t n = (int64_t)Co * RS * Ci;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int co = (int)(i % Co);
    const int64_t t2 = i / Co;
    const int rs = (int)(t2 % RS);
    const int ci = (int)(t2 / RS);
    wt[i] = w[((int64_t)co * RS + rs) * Ci + ci];
  }
}

// ---------------------------------------------------------------------------
static int log2_exact(int v) {
  if (v <= 0 || (v & (v - 1))) return -1;
  int s = 0;
  while ((1 << s) < v) ++s;
  return s;
}

static void fill_shifts(ConvArgs& a) {
  a.c_shift = log2_exact(a.g.C);
  a.q_shift = log2_exact(a.g.Q);
  a.pq_shift = log2_exact(a.g.P * a.g.Q);
}

template <int BM, int BN, bool DG, int KS, int ST>
static void launch_gemm_t(const ConvArgs& a, const ConvPlan& p, hipStream_t s) {
  dim3 grid((a.g.M + BM - 1) / BM, (a.g.Ng + BN - 1) / BN, p.splits);
  const size_t btile = DG ? (size_t)kBK * (BN + kPad) : (size_t)BN * kLdsStride;
  size_t lds = (size_t)2 * ((size_t)BM * kLdsStride + btile) * sizeof(uint16_t);
  const size_t epi = ((size_t)BM * (BN + 4) + 256 * 16 + 8) * sizeof(float);
  if (lds < epi) lds = epi;
  static bool attr_set = false;  // > 64 KiB of dynamic LDS must be opted into
  if (!attr_set && lds > 65536) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_gemm_kernel<BM, BN, DG, KS, ST>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  conv_gemm_kernel<BM, BN, DG, KS, ST><<<grid, 256, lds, s>>>(a);
}

template <int BM, int BN, bool DG>
static void launch_gemm_ks(const ConvArgs& a, const ConvPlan& p, hipStream_t s) {
  const int ks = a.g.R, st = a.g.stride;
  if (ks == 3 && st == 1) launch_gemm_t<BM, BN, DG, 3, 1>(a, p, s);
  else if (ks == 3 && st == 2) launch_gemm_t<BM, BN, DG, 3, 2>(a, p, s);
  else if (ks == 1 && st == 1) launch_gemm_t<BM, BN, DG, 1, 1>(a, p, s);
  else if (ks == 1 && st == 2) launch_gemm_t<BM, BN, DG, 1, 2>(a, p, s);
}

bool conv_supported(const ConvGeom& g) {
  return g.R == g.S && (g.R == 1 || g.R == 3) && (g.stride == 1 || g.stride == 2);
}

ConvPlan plan_conv_gemm(const ConvGeom& g) {
  ConvPlan p;
  p.bm = g.M >= 8192 ? 128 : 64;
  p.bn = g.Ng >= 128 && g.M >= 16384 ? 128 : 64;
  const int tiles = ((g.M + p.bm - 1) / p.bm) * ((g.Ng + p.bn - 1) / p.bn);
  const int ksteps = (g.K + kBK - 1) / kBK;
  int splits = 1;
  while (tiles * splits < 256 && ksteps / (splits * 2) >= 4 && splits < 16) splits *= 2;
  p.splits = splits;
  p.kchunk = ((ksteps + splits - 1) / splits) * kBK;
  p.stats_rows = 1;
  return p;
}

int conv_counter_slots(const ConvGeom& g, const ConvPlan& p) {
  return ((g.M + p.bm - 1) / p.bm) * ((g.Ng + p.bn - 1) / p.bn);
}

void launch_conv_gemm(const ConvGeom& g, bool dgrad, const ConvPlan& p, const uint16_t* src,
                      const uint16_t* wgt, uint16_t* y, float* ysplit, int* counters,
                      double* stats, bool accum, hipStream_t s) {
  ConvArgs a{};
  a.g = g;
  a.src = src;
  a.wgt = wgt;
  a.y = y;
  a.ysplit = ysplit;
  a.counters = counters;
  a.stats = stats;
  a.kchunk = p.kchunk;
  a.accum = accum ? 1 : 0;
  fill_shifts(a);
#define MFL_CONV_CASE(BM_, BN_)                                    \
  if (p.bm == BM_ && p.bn == BN_) {                                \
    if (dgrad) launch_gemm_ks<BM_, BN_, true>(a, p, s);            \
    else launch_gemm_ks<BM_, BN_, false>(a, p, s);                 \
  }
  MFL_CONV_CASE(128, 128)
  MFL_CONV_CASE(128, 64)
  MFL_CONV_CASE(64, 64)
#undef MFL_CONV_CASE
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
  ConvArgs a{};
  a.g = g;
  a.src = dy;
  a.wgt = x;
  a.kchunk = p.kchunk;
  fill_shifts(a);
  dim3 grid((g.Ng + 63) / 64, (g.K + 63) / 64, p.splits);
  const size_t lds = (size_t)2 * kBK * ((64 + kPad) + (64 + kPad)) * sizeof(uint16_t);
  const int ks = g.R, st = g.stride;
  if (ks == 3 && st == 1) conv_wgrad_kernel<64, 64, 3, 1><<<grid, 256, lds, s>>>(a, dw);
  else if (ks == 3 && st == 2) conv_wgrad_kernel<64, 64, 3, 2><<<grid, 256, lds, s>>>(a, dw);
  else if (ks == 1 && st == 1) conv_wgrad_kernel<64, 64, 1, 1><<<grid, 256, lds, s>>>(a, dw);
  else if (ks == 1 && st == 2) conv_wgrad_kernel<64, 64, 1, 2><<<grid, 256, lds, s>>>(a, dw);
}

void launch_transpose_krsc(const uint16_t* w, uint16_t* wt, int Co, int RS, int Ci, hipStream_t s) {
  const int64_t n = (int64_t)Co * RS * Ci;
  transpose_krsc_kernel<<<stream_grid(n, 256, 4096), 256, 0, s>>>(w, wt, Co, RS, Ci);
}

}  // namespace mfl
