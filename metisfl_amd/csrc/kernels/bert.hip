// BERT-base training kernels for gfx950 (SURVEY §2.10 K12/K13 LayerNorm, K14
// softmax cross-entropy, K15 fused epilogues, §5.7 fused attention).  The
// reference has no transformer (its largest model is a Keras CNN); SURVEY
// §7.2 step 10 adds BERT-base as the GEMM-heavy workload of the new build.
// The GEMMs run on gemm.hip (MFMA implicit-GEMM core with fused bias /
// residual / GELU epilogue); everything else of a post-LN encoder layer is
// here, each op fused so that one launch reads its inputs once:
//
//  * ln_fwd       LayerNorm (+ the embedding gather word+pos+type for the
//                 first one), mean / rstd saved for backward.
//  * ln_bwd       LayerNorm backward + dgamma / dbeta + the bias gradient of
//                 the GEMM that produced the LN input (= column sums of dx)
//                 + an optional second copy of dx (the residual branch) --
//                 or, for the embedding LN, the scatter of dx into the word /
//                 position / type tables.
//  * gelu_bwd     dz = dh * gelu'(z) and the FFN-1 bias gradient.
//  * attention    seq 128, head dim 64: one workgroup per (sequence, head)
//                 holds K, V (and for backward Q, dO, P, dS) in LDS; QK^T,
//                 PV, dO V^T, dS K, dS^T Q, P^T dO all on MFMA 16x16x32 with
//                 transposing LDS reads for the column-major operands; the
//                 softmax never leaves registers; the qkv bias gradient is
//                 reduced in the same kernel.
//  * mlm_*        gather of the masked positions, vocab-wide softmax CE with
//                 16-B loads, scatter of their gradient back to the sequence.
#include "kernels/common.h"
#include <hipcub/hipcub.hpp>

#include "kernels/bert.h"

#ifndef MFL_BERT_DBG
#define MFL_BERT_DBG 0  // timing experiments only (compile-time)
#endif

namespace mfl {

typedef short v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float hsum32(float v) {  // sum over a 32-lane half-wave
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// =============================================================================
// LayerNorm.  Rows of H = 256 * V elements; a half-wave (32 lanes) per row,
// lane j owns the 16-B column groups (v * 32 + j) for v < V; 8 rows per
// 256-thread block and pass.
template <int V, bool EMB>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LnFwdArgs a) {
  const int hw = threadIdx.x >> 5, j = threadIdx.x & 31;
  const int row = blockIdx.x * 8 + hw;
  if (row >= a.M) return;
  constexpr int H = 256 * V;
  float x[V][8];
  if constexpr (EMB) {
    const int b = row / a.T, t = row - b * a.T;
    const int tok = a.tokens[(int64_t)b * a.tok_stride + t];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = (v * 32 + j) * 8;
      float w[8], p[8], ty[8];
      unpack8(*reinterpret_cast<const uint4*>(a.word + (int64_t)tok * H + c), w);
      unpack8(*reinterpret_cast<const uint4*>(a.pos + (int64_t)t * H + c), p);
      unpack8(*reinterpret_cast<const uint4*>(a.type + c), ty);
#pragma unroll
      for (int k = 0; k < 8; ++k) x[v][k] = w[k] + p[k] + ty[k];
      // keep the (bf16-rounded) LN input for backward
      const uint4 pk = pack8(x[v]);
      *reinterpret_cast<uint4*>(a.xsave + (int64_t)row * H + c) = pk;
      unpack8(pk, x[v]);
    }
  } else {
#pragma unroll
    for (int v = 0; v < V; ++v)
      unpack8(*reinterpret_cast<const uint4*>(a.x + (int64_t)row * H + (v * 32 + j) * 8), x[v]);
  }
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int k = 0; k < 8; ++k) s += x[v][k];
  const float mean = hsum32(s) * (1.f / H);
  float q = 0.f;
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = x[v][k] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(hsum32(q) * (1.f / H) + a.eps);
  if (j == 0) {
    a.mean[row] = mean;
    a.rstd[row] = rstd;
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const int c = (v * 32 + j) * 8;
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (x[v][k] - mean) * rstd * a.gamma[c + k] + a.beta[c + k];
    *reinterpret_cast<uint4*>(a.y + (int64_t)row * H + c) = pack8(o);
  }
}

constexpr int kLnBwdRows = 16;  // rows per block of the embedding variant (pos_reduced needs B % 16 == 0)
// 8 waves per block (16 rows per pass): the block count stays ~256 (each
// block ends with 3 H global atomics) while twice the rows' loads are in
// flight per CU
constexpr int kLnBwdWaves = 8, kLnBwdThreads = 64 * kLnBwdWaves, kLnBwdPass = 2 * kLnBwdWaves;

// Embedding variant with a.pos_reduced (B % kLnBwdRows == 0): rows are
// visited position-major (i -> b = i % B, t = i / B), so a block's rows share
// one position t and the position-table gradient is reduced in the block
// instead of by one atomic per element.
template <int V, bool EMB>
__global__ __launch_bounds__(kLnBwdThreads) void ln_bwd_kernel(LnBwdArgs a) {
  constexpr int H = 256 * V;
  // per-wave column partials [wave][dgamma | dbeta | sum dx][H]; every slot is
  // written exactly once (no zeroing, no LDS atomics)
  __shared__ __attribute__((aligned(16))) float red[kLnBwdWaves][3][H];
  const int hw = threadIdx.x >> 5, j = threadIdx.x & 31;
  float pg[V][8], pb[V][8], pd[V][8];
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int k = 0; k < 8; ++k) pg[v][k] = pb[v][k] = pd[v][k] = 0.f;
  const int rows = EMB ? kLnBwdRows : a.rows;  // multiple of kLnBwdPass
  for (int pass = 0; pass < rows / kLnBwdPass; ++pass) {
    const int i = blockIdx.x * rows + pass * kLnBwdPass + hw;
    if (i >= a.M) break;  // uniform per half-wave
    int row = i, b = 0, t = 0, tok = 0;
    if constexpr (EMB) {
      if (a.pos_reduced) {
        b = i % a.B;
        t = i / a.B;
        row = b * a.T + t;
      } else {
        b = i / a.T;
        t = i - b * a.T;
      }
      tok = a.tokens[(int64_t)b * a.tok_stride + t];
    }
    const float mean = a.mean[row], rstd = a.rstd[row];
    float dy[V][8], xh[V][8], gg[V][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = (v * 32 + j) * 8;
      float xv[8];
      unpack8(*reinterpret_cast<const uint4*>(a.dy + (int64_t)row * H + c), dy[v]);
      unpack8(*reinterpret_cast<const uint4*>(a.x + (int64_t)row * H + c), xv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        xh[v][k] = (xv[k] - mean) * rstd;
        gg[v][k] = dy[v][k] * a.gamma[c + k];
        s1 += gg[v][k];
        s2 += gg[v][k] * xh[v][k];
        pg[v][k] += dy[v][k] * xh[v][k];
        pb[v][k] += dy[v][k];
      }
    }
    const float m1 = hsum32(s1) * (1.f / H), m2 = hsum32(s2) * (1.f / H);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = (v * 32 + j) * 8;
      float dx[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        dx[k] = rstd * (gg[v][k] - m1 - xh[v][k] * m2);
        pd[v][k] += dx[k];
      }
      if constexpr (EMB) {
        if (a.demb) {
          float4* d = reinterpret_cast<float4*>(a.demb + (int64_t)row * H + c);
          d[0] = float4{dx[0], dx[1], dx[2], dx[3]};
          d[1] = float4{dx[4], dx[5], dx[6], dx[7]};
          if (v == 0 && j == 0) {
            a.keys[row] = tok;
            a.vals[row] = row;
          }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (!a.demb) atomicAdd(a.dword + (int64_t)tok * H + c + k, dx[k]);
          if (!a.pos_reduced) atomicAdd(a.dpos + (int64_t)t * H + c + k, dx[k]);
        }
      } else {
        const uint4 pk = pack8(dx);
        *reinterpret_cast<uint4*>(a.dx + (int64_t)row * H + c) = pk;
        if (a.dx2) *reinterpret_cast<uint4*>(a.dx2 + (int64_t)row * H + c) = pk;
      }
    }
  }
  if constexpr (MFL_BERT_DBG & 2) return;
  // Block reduction of the column partials.  The two half-waves of a wave own
  // the same columns: fold them with one cross-half shuffle, write the wave's
  // row of red[w] with 16-B stores, then every thread sums its columns over
  // the 4 waves.  (LDS atomics from all 8 half-waves onto shared columns cost
  // 22 of the kernel's 45 us at the BERT shape: scripts/ln_micro.py.)
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pg[v][k] += __shfl_xor(pg[v][k], 32);
      pb[v][k] += __shfl_xor(pb[v][k], 32);
      pd[v][k] += __shfl_xor(pd[v][k], 32);
    }
  if ((threadIdx.x & 63) < 32) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = (v * 32 + j) * 8;
      float4* r0 = reinterpret_cast<float4*>(&red[w][0][c]);
      float4* r1 = reinterpret_cast<float4*>(&red[w][1][c]);
      float4* r2 = reinterpret_cast<float4*>(&red[w][2][c]);
      r0[0] = float4{pg[v][0], pg[v][1], pg[v][2], pg[v][3]};
      r0[1] = float4{pg[v][4], pg[v][5], pg[v][6], pg[v][7]};
      r1[0] = float4{pb[v][0], pb[v][1], pb[v][2], pb[v][3]};
      r1[1] = float4{pb[v][4], pb[v][5], pb[v][6], pb[v][7]};
      r2[0] = float4{pd[v][0], pd[v][1], pd[v][2], pd[v][3]};
      r2[1] = float4{pd[v][4], pd[v][5], pd[v][6], pd[v][7]};
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 3; ++q)
    for (int c = threadIdx.x; c < H; c += kLnBwdThreads) {
      float t = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < kLnBwdWaves; ++w2) t += red[w2][q][c];
      red[0][q][c] = t;
    }
  __syncthreads();
  if constexpr (MFL_BERT_DBG & 1) return;
  for (int c = threadIdx.x; c < H; c += kLnBwdThreads) {
    atomicAdd(a.dgamma + c, red[0][0][c]);
    atomicAdd(a.dbeta + c, red[0][1][c]);
    // EMB: the type table's gradient (token type 0 for every position);
    // otherwise the bias gradient of the GEMM that produced the LN input
    float* d3 = EMB ? a.dtype : a.dbias_prev;
    if (d3) atomicAdd(d3 + c, red[0][2][c]);
    if (EMB && a.pos_reduced) atomicAdd(a.dpos + (int64_t)((blockIdx.x * kLnBwdRows) / a.B) * H + c, red[0][2][c]);
  }
}

// Segmented reduction of the token-sorted embedding-gradient rows: block =
// 64 consecutive sorted positions x H/4 float4 columns.
constexpr int kEmbChunk = 64;
__global__ __launch_bounds__(256) void emb_word_reduce_kernel(const float* __restrict__ demb,
                                                              const int* __restrict__ skeys,
                                                              const int* __restrict__ svals, int M, int H,
                                                              float* __restrict__ dword) {
  const int c0 = blockIdx.x * kEmbChunk, c1 = min(M, c0 + kEmbChunk);
  const int q = threadIdx.x;
  if (4 * q >= H) return;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  int seg0 = c0;
  for (int p = c0; p < c1; ++p) {
    const int tok = skeys[p];
    const float4 v = *reinterpret_cast<const float4*>(demb + (int64_t)svals[p] * H + 4 * q);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    const bool end = (p + 1 == c1) || (skeys[p + 1] != tok);
    if (!end) continue;
    // a segment touching a chunk edge may continue in the neighbouring chunk
    const bool shared = (seg0 == c0 && c0 > 0 && skeys[c0 - 1] == tok) ||
                        (p + 1 == c1 && c1 < M && skeys[c1] == tok);
    float* d = dword + (int64_t)tok * H + 4 * q;
    if (shared) {
      atomicAdd(d + 0, acc.x); atomicAdd(d + 1, acc.y); atomicAdd(d + 2, acc.z); atomicAdd(d + 3, acc.w);
    } else {  // the only writer of this token's row in this launch
      float4 o = *reinterpret_cast<float4*>(d);
      o.x += acc.x; o.y += acc.y; o.z += acc.z; o.w += acc.w;
      *reinterpret_cast<float4*>(d) = o;
    }
    acc = float4{0.f, 0.f, 0.f, 0.f};
    seg0 = p + 1;
  }
}

size_t emb_sort_temp_bytes(int M, int key_bits) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int*)nullptr, (int*)nullptr,
                                           (const int*)nullptr, (int*)nullptr, M, 0, key_bits);
  return bytes;
}

void launch_emb_word_grad(const float* demb, const int* keys, const int* vals, int* skeys, int* svals,
                          void* tmp, size_t tmp_bytes, int M, int H, int key_bits, float* dword,
                          hipStream_t s) {
  size_t bytes = tmp_bytes;
  (void)hipcub::DeviceRadixSort::SortPairs(tmp, bytes, keys, skeys, vals, svals, M, 0, key_bits, s);
  emb_word_reduce_kernel<<<(M + kEmbChunk - 1) / kEmbChunk, 256, 0, s>>>(demb, skeys, svals, M, H, dword);
}

void launch_ln_fwd(const LnFwdArgs& a, int H, bool emb, hipStream_t s) {
  const unsigned grid = (a.M + 7) / 8;
#define MFL_LN_F(V_)                                                               \
  if (H == 256 * V_) {                                                             \
    if (emb) ln_fwd_kernel<V_, true><<<grid, 256, 0, s>>>(a);                     \
    else ln_fwd_kernel<V_, false><<<grid, 256, 0, s>>>(a);                        \
    return;                                                                        \
  }
  MFL_LN_F(1) MFL_LN_F(2) MFL_LN_F(3) MFL_LN_F(4)
#undef MFL_LN_F
}

void launch_ln_bwd(const LnBwdArgs& args, int H, bool emb, hipStream_t s) {
  // ~256 blocks: enough to fill the CUs, few enough that the per-block
  // column partials (3 H global atomics each) stay cheap
  LnBwdArgs a = args;
  static const int target_blocks = [] {  // env MFL_LN_BWD_BLOCKS (timing experiments)
    const char* v = getenv("MFL_LN_BWD_BLOCKS");
    return v && *v ? atoi(v) : 256;
  }();
  a.rows = max(kLnBwdPass, ((a.M + target_blocks - 1) / target_blocks + kLnBwdPass - 1) / kLnBwdPass * kLnBwdPass);
  static const int dbg = [] {
    const char* v = getenv("MFL_LN_BWD_DEBUG");
    return v && *v ? atoi(v) : 0;
  }();
  a.dbg = dbg;
  const int rows = emb ? kLnBwdRows : a.rows;
  const unsigned grid = (a.M + rows - 1) / rows;
#define MFL_LN_B(V_)                                                               \
  if (H == 256 * V_) {                                                             \
    if (emb) ln_bwd_kernel<V_, true><<<grid, kLnBwdThreads, 0, s>>>(a);           \
    else ln_bwd_kernel<V_, false><<<grid, kLnBwdThreads, 0, s>>>(a);              \
    return;                                                                        \
  }
  MFL_LN_B(1) MFL_LN_B(2) MFL_LN_B(3) MFL_LN_B(4)
#undef MFL_LN_B
}

// =============================================================================
// dz = dh * gelu'(z) (exact erf GELU) and dbias += column sums of dz.
// Block = 512 columns (a wave's 64 lanes x 16 B) x kColRows rows; wave w
// takes rows w, w+4, ... with 4 rows' loads in flight per step, the 4 waves'
// column partials meet in LDS, then one atomic per column per block.
constexpr int kColRows = 64;

template <bool GELU>
__global__ __launch_bounds__(256) void colsum_kernel(const uint16_t* __restrict__ dh,
                                                     const uint16_t* __restrict__ z,
                                                     uint16_t* __restrict__ dz, float* __restrict__ dbias,
                                                     int M, int N, int pre) {
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cv = blockIdx.y * 64 + lane;
  const bool col_ok = cv * 8 < N;
  const int r0 = blockIdx.x * kColRows;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col_ok) {
    for (int rb = r0 + w; rb < min(M, r0 + kColRows); rb += 16) {
      uint4 gv[4], zv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = min(rb + 4 * u, M - 1);  // clamped rows are loaded but not used
        const int64_t off = (int64_t)r * N + cv * 8;
        gv[u] = *reinterpret_cast<const uint4*>(dh + off);
        if (GELU) zv[u] = *reinterpret_cast<const uint4*>(z + off);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rb + 4 * u;
        if (r >= min(M, r0 + kColRows)) break;
        float g[8];
        unpack8(gv[u], g);
        if (GELU) {
          float zz[8];
          unpack8(zv[u], zz);
          if (pre) {  // z holds gelu'(z) (the forward stored it)
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] *= zz[k];
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] *= gelu_grad_f(zz[k]);
          }
          const uint4 pk = pack8(g);
          *reinterpret_cast<uint4*>(dz + (int64_t)r * N + cv * 8) = pk;
          unpack8(pk, g);  // the bias gradient of what the GEMMs consume
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += g[k];
      }
    }
  }
  if (!dbias) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) red[w][lane * 8 + k] = acc[k];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int col = blockIdx.y * 512 + c;
    if (col < N) atomicAdd(dbias + col, red[0][c] + red[1][c] + red[2][c] + red[3][c]);
  }
}

void launch_gelu_bwd(const uint16_t* dh, const uint16_t* z, uint16_t* dz, float* dbias, int M, int N,
                     hipStream_t s, int pre) {
  dim3 grid((M + kColRows - 1) / kColRows, (N + 511) / 512);
  colsum_kernel<true><<<grid, 256, 0, s>>>(dh, z, dz, dbias, M, N, pre);
}

void launch_colsum(const uint16_t* dy, float* dbias, int M, int N, hipStream_t s) {
  dim3 grid((M + kColRows - 1) / kColRows, (N + 511) / 512);
  colsum_kernel<false><<<grid, 256, 0, s>>>(dy, nullptr, nullptr, dbias, M, N, 0);
}

// y <- bf16(gelu'(y)) in place (n % 8 == 0): the conv-core GEMM path's
// stored GELU derivative (launch_gemm_fwd act_grad)
__global__ __launch_bounds__(256) void gelu_grad_inplace_kernel(uint4* __restrict__ y, int64_t n8) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float f[8];
    unpack8(y[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = gelu_grad_f(f[k]);
    y[i] = pack8(f);
  }
}

void launch_gelu_grad_inplace(uint16_t* y, int64_t n, hipStream_t s) {
  const int64_t n8 = n / 8;
  gelu_grad_inplace_kernel<<<stream_grid(n8), 256, 0, s>>>(reinterpret_cast<uint4*>(y), n8);
}

// =============================================================================
// Attention, T = 128 keys, head dim 64.  LDS tiles are row-major bf16 with
// 16-B chunk XOR swizzles (128-B rows: (row>>1)&7, 256-B rows: row&15, the
// conflict-free keys for 16-row b128 fragment reads, see conv.hip).
constexpr int kT = 128, kD = 64;

template <int ROWB>
__device__ __forceinline__ int toff(int row, int col) {
  const int sw = ROWB == 128 ? ((row >> 1) & 7) : (row & 15);
  return row * ROWB + ((((col >> 3) ^ sw)) << 4) + ((col & 7) << 1);
}
// A/B fragment X[r0 + lane%16][k0 + 8*(lane/16) + 0..7] (row-major operand)
template <int ROWB>
__device__ __forceinline__ bf16x8 frag_row(const uint8_t* t, int r0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(t + toff<ROWB>(r0 + (lane & 15), k0 + 8 * (lane >> 4)));
}
// fragment X[k0 + 8*(lane/16) + 0..7][n0 + lane%16] (column-major use of a
// row-major tile) from two transposing reads
template <int ROWB>
__device__ __forceinline__ bf16x8 frag_col(const uint8_t* t, int k0, int n0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  bf16x8 out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4s*)(t + toff<ROWB>(k0 + 8 * g + 4 * h + q, n0 + 4 * p)));
    out[4 * h + 0] = v[0];
    out[4 * h + 1] = v[1];
    out[4 * h + 2] = v[2];
    out[4 * h + 3] = v[3];
  }
  return out;
}
__device__ __forceinline__ f32x4 mma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void st_bf16(uint8_t* t, int off, float v) {
  *reinterpret_cast<uint16_t*>(t + off) = f2bf(v);
}

// stage a [128][64] head slice of a [rows][ld] bf16 matrix into LDS
template <int NT = 256>
__device__ __forceinline__ void load_head(uint8_t* dst, const uint16_t* src, int64_t row0, int ld, int col0) {
  for (int i = threadIdx.x; i < kT * 8; i += NT) {
    const int r = i >> 3, c = (i & 7) * 8;
    *reinterpret_cast<uint4*>(dst + toff<128>(r, c)) =
        *reinterpret_cast<const uint4*>(src + (row0 + r) * ld + col0 + c);
  }
}

constexpr float kLog2e = 1.4426950408889634f;

// One attention item (batch b, head h) once K and V sit in LDS and this
// wave's Q fragments in registers, in two halves: S = Q K^T and the row
// softmax into this wave's P tile (lse saved), then O = P V.
__device__ __forceinline__ void attn_fwd_scores(const AttnArgs& a, int b, int h, const uint8_t* Ks, uint8_t* Pw,
                                                const bf16x8 (&qf)[2][2], int lane, int wave) {
  const int t0 = wave * 32;
  f32x4 s[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jt = 0; jt < 8; ++jt) s[i][jt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int jt = 0; jt < 8; ++jt) {
      const bf16x8 kf = frag_row<128>(Ks, 16 * jt, 32 * kk, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i) s[i][jt] = mma(qf[i][kk], kf, s[i][jt]);
    }
  // row softmax: a row's 128 scores sit in 8 tiles x the 16 lanes of a group
  const float c = a.scale * kLog2e;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float mx = -INFINITY;
#pragma unroll
      for (int jt = 0; jt < 8; ++jt) mx = fmaxf(mx, s[i][jt][e]);
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
      float sum = 0.f;
#pragma unroll
      for (int jt = 0; jt < 8; ++jt) {
        const float p = exp2f((s[i][jt][e] - mx) * c);
        s[i][jt][e] = p;
        sum += p;
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
      const float inv = 1.f / sum;
      const int r = 16 * i + 4 * (lane >> 4) + e;
#pragma unroll
      for (int jt = 0; jt < 8; ++jt) st_bf16(Pw, toff<256>(r, 16 * jt + (lane & 15)), s[i][jt][e] * inv);
      if ((lane & 15) == 0) a.lse[((int64_t)b * a.heads + h) * kT + t0 + r] = mx * a.scale + __logf(sum);
    }
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void attn_fwd_pv(const AttnArgs& a, int b, int h, const uint8_t* Vs, const uint8_t* Pw,
                                            int lane, int wave) {
  const int H = a.heads * kD;
  const int64_t row0 = (int64_t)b * kT;
  const int t0 = wave * 32;
  f32x4 o[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int dj = 0; dj < 4; ++dj) o[i][dj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < kT; kk += 32) {
    bf16x8 pf[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) pf[i] = frag_row<256>(Pw, 16 * i, kk, lane);
#pragma unroll
    for (int dj = 0; dj < 4; ++dj) {
      const bf16x8 vf = frag_col<128>(Vs, kk, 16 * dj, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i) o[i][dj] = mma(pf[i], vf, o[i][dj]);
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int dj = 0; dj < 4; ++dj)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int t = t0 + 16 * i + 4 * (lane >> 4) + e;
        a.ctx[(row0 + t) * H + h * kD + 16 * dj + (lane & 15)] = f2bf(o[i][dj][e]);
      }
}

// this wave's Q fragments of item (b, h), straight from global memory
__device__ __forceinline__ void attn_q_frags(const AttnArgs& a, int b, int h, int lane, int wave, bf16x8 (&qf)[2][2]) {
  const int H = a.heads * kD, ld = 3 * H;
  const int64_t row0 = (int64_t)b * kT;
  const int t0 = wave * 32;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      qf[i][kk] = *reinterpret_cast<const bf16x8*>(a.qkv + (row0 + t0 + 16 * i + (lane & 15)) * ld + h * kD +
                                                   32 * kk + 8 * (lane >> 4));
}

__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* Ks = smem;
  uint8_t* Vs = smem + kT * kD * 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* Pw = smem + 2 * kT * kD * 2 + wave * (32 * kT * 2);  // this wave's [32][128]
  const int b = blockIdx.x / a.heads, h = blockIdx.x - b * a.heads;
  const int H = a.heads * kD, ld = 3 * H;
  const int64_t row0 = (int64_t)b * kT;
  load_head(Ks, a.qkv, row0, ld, H + h * kD);
  load_head(Vs, a.qkv, row0, ld, 2 * H + h * kD);
  bf16x8 qf[2][2];
  attn_q_frags(a, b, h, lane, wave, qf);
  __syncthreads();
  attn_fwd_scores(a, b, h, Ks, Pw, qf, lane, wave);
  attn_fwd_pv(a, b, h, Vs, Pw, lane, wave);
}

// Persistent forward: a workgroup walks items blockIdx.x, + gridDim.x, ...
// with the NEXT item's K / V slices (4 + 4 16-B chunks per thread) in
// flight while it computes this one's P V and writes its context (one item per
// workgroup paid its load latency with nothing to overlap: 2 workgroups per
// CU by LDS).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void attn_fwd_persist_kernel(AttnArgs a, int nitems) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* Ks = smem;
  uint8_t* Vs = smem + kT * kD * 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t* Pw = smem + 2 * kT * kD * 2 + wave * (32 * kT * 2);
  const int H = a.heads * kD, ld = 3 * H;
  const int r = threadIdx.x >> 3, cc = (threadIdx.x & 7) * 8;  // rows r + 32 u, u < 4
  u32x4 kr[4], vr[4];  // (native vectors: HIP uint4 arrays stayed in scratch)
  bf16x8 qf[2][2];
  // (a macro, not a lambda: a lambda capturing the register arrays by
  // reference put them in scratch)
#define MFL_ATTN_FWD_FETCH(ITEM)                                                         \
  {                                                                                      \
    const int b_ = (ITEM) / a.heads, h_ = (ITEM) - b_ * a.heads;                         \
    const uint16_t* base = a.qkv + ((int64_t)b_ * kT + r) * ld + h_ * kD + cc;           \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                      \
      kr[u] = *reinterpret_cast<const u32x4*>(base + (int64_t)32 * u * ld + H);          \
      vr[u] = *reinterpret_cast<const u32x4*>(base + (int64_t)32 * u * ld + 2 * H);      \
    }                                                                                    \
  }
  int it = blockIdx.x;  // grid <= nitems
  MFL_ATTN_FWD_FETCH(it)
#pragma unroll 1
  for (; it < nitems; it += gridDim.x) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      *reinterpret_cast<u32x4*>(Ks + toff<128>(r + 32 * u, cc)) = kr[u];
      *reinterpret_cast<u32x4*>(Vs + toff<128>(r + 32 * u, cc)) = vr[u];
    }
    const int b = it / a.heads, h = it - b * a.heads;
    attn_q_frags(a, b, h, lane, wave, qf);
    __syncthreads();
    attn_fwd_scores(a, b, h, Ks, Pw, qf, lane, wave);
    // the scores are dead once P is in LDS: their registers hold the fetch
    if (it + gridDim.x < nitems) MFL_ATTN_FWD_FETCH(it + gridDim.x)
    attn_fwd_pv(a, b, h, Vs, Pw, lane, wave);
    __syncthreads();  // every wave is done with Ks / Vs / Pw before the next staging
  }
#undef MFL_ATTN_FWD_FETCH
}

template <int NI>
__device__ __forceinline__ void colsum_tile(const f32x4 (&acc)[NI][4], float* cs, int lane, float mul) {
#pragma unroll
  for (int dj = 0; dj < 4; ++dj) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) v += acc[i][dj][e] * mul;
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane < 16) atomicAdd(cs + 16 * dj + lane, v);
  }
}

// NW waves per workgroup, kT / NW query rows (and key rows) per wave.  The
// K/V/Q/dO + P/dS tiles take 130 KiB of LDS (one workgroup per CU), so the
// wave count is the only occupancy lever: NW = 8 runs two waves per SIMD.
//
// attn_bwd_body: one (sequence, head) item whose Q, K, V, dO tiles, D = rowsum
// (dO * O) and lse are staged in LDS and whose bias-gradient partials cs are
// zero.  Its barriers are LDS-only (lgkmcnt + s_barrier): the persistent
// kernel keeps the NEXT item's operand loads and this item's output stores in
// flight across them (__syncthreads would drain vmcnt).
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
}

template <int NW>
__device__ __forceinline__ void attn_bwd_body(const AttnArgs& a, int b, int h, uint8_t* smem, int tid) {
  constexpr int RW = kT / NW, NI = RW / 16;
  constexpr int HT = kT * kD * 2;  // 16 KiB head tile
  uint8_t* Qs = smem;
  uint8_t* Ks = smem + HT;
  uint8_t* Vs = smem + 2 * HT;
  uint8_t* dOs = smem + 3 * HT;
  uint8_t* Ps = smem + 4 * HT;             // [128][128] bf16
  uint8_t* dSs = Ps + kT * kT * 2;          // [128][128] bf16
  float* Dd = reinterpret_cast<float*>(dSs + kT * kT * 2);
  float* Ls = Dd + kT;
  float* cs = Ls + kT;  // [3][64] bias-gradient partials
  const int lane = tid & 63, wave = tid >> 6;
  const int H = a.heads * kD, ld = 3 * H;
  const int64_t row0 = (int64_t)b * kT;
  const int t0 = wave * RW;
  const float c = a.scale * kLog2e;
  {
    f32x4 s[NI][8], dp[NI][8];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int jt = 0; jt < 8; ++jt) s[i][jt] = dp[i][jt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < kD; kk += 32) {
      bf16x8 qf[NI], df[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        qf[i] = frag_row<128>(Qs, t0 + 16 * i, kk, lane);
        df[i] = frag_row<128>(dOs, t0 + 16 * i, kk, lane);
      }
#pragma unroll
      for (int jt = 0; jt < 8; ++jt) {
        const bf16x8 kf = frag_row<128>(Ks, 16 * jt, kk, lane);
        const bf16x8 vf = frag_row<128>(Vs, 16 * jt, kk, lane);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          s[i][jt] = mma(qf[i], kf, s[i][jt]);
          dp[i][jt] = mma(df[i], vf, dp[i][jt]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = t0 + 16 * i + 4 * (lane >> 4) + e;
        const float l2 = Ls[r] * kLog2e, dd = Dd[r];
#pragma unroll
        for (int jt = 0; jt < 8; ++jt) {
          const float p = exp2f(s[i][jt][e] * c - l2);
          const int off = toff<256>(r, 16 * jt + (lane & 15));
          st_bf16(Ps, off, p);
          st_bf16(dSs, off, p * (dp[i][jt][e] - dd));
        }
      }
  }
  __builtin_amdgcn_wave_barrier();
  // dQ = scale * dS K  (this wave's rows; dS rows written by this wave)
  {
    f32x4 acc[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int dj = 0; dj < 4; ++dj) acc[i][dj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < kT; kk += 32) {
      bf16x8 af[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) af[i] = frag_row<256>(dSs, t0 + 16 * i, kk, lane);
#pragma unroll
      for (int dj = 0; dj < 4; ++dj) {
        const bf16x8 kf = frag_col<128>(Ks, kk, 16 * dj, lane);
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i][dj] = mma(af[i], kf, acc[i][dj]);
      }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int dj = 0; dj < 4; ++dj)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int t = t0 + 16 * i + 4 * (lane >> 4) + e;
          a.dqkv[(row0 + t) * ld + h * kD + 16 * dj + (lane & 15)] = f2bf(acc[i][dj][e] * a.scale);
        }
    colsum_tile(acc, cs, lane, a.scale);
  }
  lds_sync();  // every wave's P and dS rows are in LDS
  // dK = scale * dS^T Q and dV = P^T dO for key rows s0 .. s0+31
  {
    const int s0 = wave * RW;
    f32x4 dk[NI][4], dv[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int dj = 0; dj < 4; ++dj) dk[i][dj] = dv[i][dj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < kT; kk += 32) {
      bf16x8 sf[NI], pf[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        sf[i] = frag_col<256>(dSs, kk, s0 + 16 * i, lane);
        pf[i] = frag_col<256>(Ps, kk, s0 + 16 * i, lane);
      }
#pragma unroll
      for (int dj = 0; dj < 4; ++dj) {
        const bf16x8 qf = frag_col<128>(Qs, kk, 16 * dj, lane);
        const bf16x8 of = frag_col<128>(dOs, kk, 16 * dj, lane);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          dk[i][dj] = mma(sf[i], qf, dk[i][dj]);
          dv[i][dj] = mma(pf[i], of, dv[i][dj]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int dj = 0; dj < 4; ++dj)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int sr = s0 + 16 * i + 4 * (lane >> 4) + e;
          uint16_t* rowp = a.dqkv + (row0 + sr) * ld + h * kD + 16 * dj + (lane & 15);
          rowp[H] = f2bf(dk[i][dj][e] * a.scale);
          rowp[2 * H] = f2bf(dv[i][dj][e]);
        }
    colsum_tile(dk, cs + kD, lane, a.scale);
    colsum_tile(dv, cs + 2 * kD, lane, 1.f);
  }
  lds_sync();
  if (a.dbias && tid < 3 * kD) {
    const int part = tid / kD, d = tid - part * kD;
    atomicAdd(a.dbias + part * H + h * kD + d, cs[tid]);
  }
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_bwd_kernel(AttnArgs a) {
  constexpr int NT = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int HT = kT * kD * 2;
  uint8_t* Qs = smem;
  uint8_t* Ks = smem + HT;
  uint8_t* Vs = smem + 2 * HT;
  uint8_t* dOs = smem + 3 * HT;
  float* Dd = reinterpret_cast<float*>(smem + 4 * HT + 2 * kT * kT * 2);
  float* Ls = Dd + kT;
  float* cs = Ls + kT;
  const int b = blockIdx.x / a.heads, h = blockIdx.x - b * a.heads;
  const int H = a.heads * kD, ld = 3 * H;
  const int64_t row0 = (int64_t)b * kT;
  load_head<NT>(Qs, a.qkv, row0, ld, h * kD);
  load_head<NT>(Ks, a.qkv, row0, ld, H + h * kD);
  load_head<NT>(Vs, a.qkv, row0, ld, 2 * H + h * kD);
  if (threadIdx.x < 2 * kT) {
    // dO into LDS and D[t] = sum_d dO[t][d] * O[t][d]: thread -> row tid/2, half tid&1
    const int r = threadIdx.x >> 1, half = threadIdx.x & 1;
    float dsum = 0.f;
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const int col = half * 32 + cc * 8;
      const uint4 dov = *reinterpret_cast<const uint4*>(a.dctx + (row0 + r) * H + h * kD + col);
      const uint4 ov = *reinterpret_cast<const uint4*>(a.ctx + (row0 + r) * H + h * kD + col);
      *reinterpret_cast<uint4*>(dOs + toff<128>(r, col)) = dov;
      float f1[8], f2[8];
      unpack8(dov, f1);
      unpack8(ov, f2);
#pragma unroll
      for (int k = 0; k < 8; ++k) dsum += f1[k] * f2[k];
    }
    dsum += __shfl_xor(dsum, 1);
    if (!half) {
      Dd[r] = dsum;
      Ls[r] = a.lse[((int64_t)b * a.heads + h) * kT + r];
    }
  }
  if (threadIdx.x < 3 * kD) cs[threadIdx.x] = 0.f;
  __syncthreads();
  attn_bwd_body<NW>(a, b, h, smem, threadIdx.x);
}

// Persistent variant (8 waves, one workgroup per CU, grid <= #CUs): each
// workgroup walks items it, it + grid, ...; the NEXT item's Q, K, V, dO, O
// tiles (80 KiB) are requested into registers (10 x 16 B per thread) right
// after the current item's tiles were staged, so the operand latency of item
// i + 1 hides under item i's MFMAs and stores instead of following them (the
// per-item launch pays load -> compute -> store in series, 6 items per CU).
// D = rowsum(dO * O) is reduced from the registers (8 lanes per row).
__device__ __forceinline__ float dot8(const uint4& x, const uint4& y) {
  float f1[8], f2[8];
  unpack8(x, f1);
  unpack8(y, f2);
  float d = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) d += f1[k] * f2[k];
  return d;
}

__device__ __forceinline__ uint4 ldg16(const uint16_t* p) { return *reinterpret_cast<const uint4*>(p); }

__global__ __launch_bounds__(512) void attn_bwd_persist_kernel(AttnArgs a, int nitems) {
  constexpr int HT = kT * kD * 2;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  float* Dd = reinterpret_cast<float*>(smem + 4 * HT + 2 * kT * kT * 2);
  float* Ls = Dd + kT;
  float* cs = Ls + kT;
  const int H = a.heads * kD, ld = 3 * H;
  // per thread: two 16-B chunks (rows r, r + 64; column chunk cc) of each of
  // Q, K, V, dO, O of the next item, and one lse value
  const int r = threadIdx.x >> 3, cc = (threadIdx.x & 7) * 8;
  const int off0 = toff<128>(r, cc), off1 = toff<128>(r + 64, cc);
  uint4 q0, q1, k0, k1, v0, v1, d0, d1, o0, o1;
  float pl;
#define MFL_ATTN_FETCH(ITEM)                                                              \
  {                                                                                       \
    const int b_ = (ITEM) / a.heads, h_ = (ITEM) - b_ * a.heads;                          \
    const uint16_t* qp = a.qkv + ((int64_t)b_ * kT + r) * ld + h_ * kD + cc;              \
    const int64_t q64 = (int64_t)64 * ld;                                                 \
    q0 = ldg16(qp); q1 = ldg16(qp + q64);                                                 \
    k0 = ldg16(qp + H); k1 = ldg16(qp + H + q64);                                         \
    v0 = ldg16(qp + 2 * H); v1 = ldg16(qp + 2 * H + q64);                                 \
    const int64_t o_ = ((int64_t)b_ * kT + r) * H + h_ * kD + cc, o64 = (int64_t)64 * H;  \
    d0 = ldg16(a.dctx + o_); d1 = ldg16(a.dctx + o_ + o64);                               \
    o0 = ldg16(a.ctx + o_); o1 = ldg16(a.ctx + o_ + o64);                                 \
    pl = threadIdx.x < kT ? a.lse[((int64_t)b_ * a.heads + h_) * kT + threadIdx.x] : 0.f; \
  }
  int it = blockIdx.x;  // grid <= nitems
  MFL_ATTN_FETCH(it)
  for (; it < nitems; it += gridDim.x) {
    // stage this item from the registers: Q K V dO tiles at smem + u * HT
    *reinterpret_cast<uint4*>(smem + off0) = q0;
    *reinterpret_cast<uint4*>(smem + off1) = q1;
    *reinterpret_cast<uint4*>(smem + HT + off0) = k0;
    *reinterpret_cast<uint4*>(smem + HT + off1) = k1;
    *reinterpret_cast<uint4*>(smem + 2 * HT + off0) = v0;
    *reinterpret_cast<uint4*>(smem + 2 * HT + off1) = v1;
    *reinterpret_cast<uint4*>(smem + 3 * HT + off0) = d0;
    *reinterpret_cast<uint4*>(smem + 3 * HT + off1) = d1;
    float s0 = dot8(d0, o0), s1 = dot8(d1, o1);  // D = rowsum(dO * O): 8 lanes per row
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) {
      s0 += __shfl_xor(s0, m);
      s1 += __shfl_xor(s1, m);
    }
    if ((threadIdx.x & 7) == 0) {
      Dd[r] = s0;
      Dd[r + 64] = s1;
    }
    if (threadIdx.x < kT) Ls[threadIdx.x] = pl;
    if (threadIdx.x < 3 * kD) cs[threadIdx.x] = 0.f;
    lds_sync();
    const int b = it / a.heads, h = it - b * a.heads;
    // the next item's tiles fly under this item (the last round re-reads its
    // own item: unconditional, so the prefetch stays in registers)
    MFL_ATTN_FETCH(min(it + (int)gridDim.x, nitems - 1))
    // the lane-derived fragment addresses are recomputed per item (an opaque
    // thread id): hoisted out of the item loop they stayed live across the
    // whole body (256 VGPRs + spills instead of ~100 + the prefetch)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    attn_bwd_body<8>(a, b, h, smem, tid);
    lds_sync();  // every wave is done with this item's LDS before the next staging
  }
#undef MFL_ATTN_FETCH
}

static void lds_attr(const void* k, size_t bytes, bool& done) {
  if (!done && bytes > 65536) {
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    done = true;
  }
}

size_t attn_fwd_lds() { return 2 * kT * kD * 2 + 4 * 32 * kT * 2; }
size_t attn_bwd_lds() { return 4 * kT * kD * 2 + 2 * kT * kT * 2 + (2 * kT + 3 * kD) * 4; }

void launch_attn_fwd(const AttnArgs& a, hipStream_t s) {
  // persistent by default (two workgroups per CU, next item prefetched);
  // MFL_ATTN_FWD_PERSIST=0: one item per workgroup
  const char* pv = getenv("MFL_ATTN_FWD_PERSIST");  // read per launch (tests toggle it)
  const int nitems = a.batch * a.heads;
  if (!(pv && *pv == '0')) {
    static const int ncu = [] {
      int dev = 0, n = 256;
      if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      return n > 0 ? n : 256;
    }();
    attn_fwd_persist_kernel<<<std::min(nitems, 2 * ncu), 256, attn_fwd_lds(), s>>>(a, nitems);
    return;
  }
  attn_fwd_kernel<<<nitems, 256, attn_fwd_lds(), s>>>(a);
}

void launch_attn_bwd(const AttnArgs& a, hipStream_t s) {
  // persistent 8-wave kernel by default; MFL_ATTN_BWD_PERSIST=0: one launch
  // item per workgroup (MFL_ATTN_BWD_WAVES=4 for its one-wave-per-SIMD variant)
  const char* pv = getenv("MFL_ATTN_BWD_PERSIST");  // read per launch (tests toggle it)
  const int persist = pv && *pv == '0' ? 0 : 1;
  static const int nw = [] {
    const char* v = getenv("MFL_ATTN_BWD_WAVES");
    return v && *v == '4' ? 4 : 8;
  }();
  static bool done4 = false, done8 = false, donep = false;
  const int nitems = a.batch * a.heads;
  if (persist) {
    static const int ncu = [] {
      int dev = 0, n = 256;
      if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      return n > 0 ? n : 256;
    }();
    lds_attr(reinterpret_cast<const void*>(&attn_bwd_persist_kernel), attn_bwd_lds(), donep);
    attn_bwd_persist_kernel<<<std::min(nitems, ncu), 512, attn_bwd_lds(), s>>>(a, nitems);
    return;
  }
  if (nw == 4) {
    lds_attr(reinterpret_cast<const void*>(&attn_bwd_kernel<4>), attn_bwd_lds(), done4);
    attn_bwd_kernel<4><<<a.batch * a.heads, 256, attn_bwd_lds(), s>>>(a);
  } else {
    lds_attr(reinterpret_cast<const void*>(&attn_bwd_kernel<8>), attn_bwd_lds(), done8);
    attn_bwd_kernel<8><<<a.batch * a.heads, 512, attn_bwd_lds(), s>>>(a);
  }
}

// =============================================================================
// Masked-LM head plumbing.  Batch rows are int32 records
//   [tokens T | mlm positions P | mlm label ids P | inverse map T]
// (inverse map: t -> prediction slot p, or -1).
__global__ __launch_bounds__(256) void mlm_gather_kernel(const uint16_t* __restrict__ x,
                                                         const int* __restrict__ rec, int rec_stride, int T,
                                                         int P, int H, uint16_t* __restrict__ out, int64_t nvec) {
  const int vpr = H / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int r = (int)(i / vpr), cv = (int)(i - (int64_t)r * vpr);
    const int b = r / P, p = r - b * P;
    const int t = rec[(int64_t)b * rec_stride + T + p];
    reinterpret_cast<uint4*>(out)[i] = reinterpret_cast<const uint4*>(x + ((int64_t)b * T + t) * H)[cv];
  }
}

__global__ __launch_bounds__(256) void mlm_scatter_kernel(const uint16_t* __restrict__ dsel,
                                                          const int* __restrict__ rec, int rec_stride, int T,
                                                          int P, int H, uint16_t* __restrict__ dx, int64_t nvec) {
  const int vpr = H / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    const int row = (int)(i / vpr), cv = (int)(i - (int64_t)row * vpr);
    const int b = row / T, t = row - b * T;
    const int p = rec[(int64_t)b * rec_stride + T + 2 * P + t];
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (p >= 0) v = reinterpret_cast<const uint4*>(dsel + ((int64_t)b * P + p) * H)[cv];
    reinterpret_cast<uint4*>(dx)[i] = v;
  }
}

void launch_mlm_gather(const uint16_t* x, const int* rec, int rec_stride, int B, int T, int P, int H,
                       uint16_t* out, hipStream_t s) {
  const int64_t nvec = (int64_t)B * P * H / 8;
  mlm_gather_kernel<<<stream_grid(nvec), 256, 0, s>>>(x, rec, rec_stride, T, P, H, out, nvec);
}

void launch_mlm_scatter(const uint16_t* dsel, const int* rec, int rec_stride, int B, int T, int P, int H,
                        uint16_t* dx, hipStream_t s) {
  const int64_t nvec = (int64_t)B * T * H / 8;
  mlm_scatter_kernel<<<stream_grid(nvec), 256, 0, s>>>(dsel, rec, rec_stride, T, P, H, dx, nvec);
}

// Vocab-wide softmax cross entropy, one 256-thread block per prediction row;
// logits [R][Vp] bf16 with V valid columns; label of row r at
// rec[(r / P) * rec_stride + T + P + r % P] (-1: ignored).  dlogits =
// (softmax - onehot) / R; stats += {loss, correct, count}.
__global__ __launch_bounds__(256) void vocab_xent_kernel(VocabXentArgs a) {
  __shared__ float sm[8], ss[8];
  __shared__ int sa[8];
  const int r = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint16_t* z = a.logits + (int64_t)r * a.Vp;
  const int nv = a.V / 8;  // V % 8 == 0 is not required: the tail is scalar
  // one pass: running max / rescaled sum per 8 logits (one rescale per 8,
  // not per logit) and the first index of this thread's maximum (accuracy);
  // two row vectors in flight per iteration
  float m = -INFINITY, s = 0.f;
  int am = a.V;
  auto fold8 = [&](const float (&f)[8], int base) __attribute__((always_inline)) {
    float m8 = f[0];
    int i8 = base;
#pragma unroll
    for (int k = 1; k < 8; ++k)
      if (f[k] > m8) {
        m8 = f[k];
        i8 = base + k;
      }
    if (m8 > m) am = i8;  // strictly greater: indices rise within a thread
    const float nm = fmaxf(m, m8);
    float e = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) e += __expf(f[k] - nm);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + e;
    m = nm;
  };
  for (int v = t; v < nv; v += 512) {
    const bool two = v + 256 < nv;
    const uint4 u0 = reinterpret_cast<const uint4*>(z)[v];
    uint4 u1 = make_uint4(0u, 0u, 0u, 0u);
    if (two) u1 = reinterpret_cast<const uint4*>(z)[v + 256];
    float f[8];
    unpack8(u0, f);
    fold8(f, v * 8);
    if (two) {
      unpack8(u1, f);
      fold8(f, (v + 256) * 8);
    }
  }
  for (int k = nv * 8 + t; k < a.V; k += 256) {
    const float f = bf2f(z[k]);
    if (f > m) am = k;
    const float nm = fmaxf(m, f);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + __expf(f - nm);
    m = nm;
  }
  // block max / sum
  float bm = wave_max(m);
  if (lane == 0) sm[w] = bm;
  __syncthreads();
  bm = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
  float bs = wave_sum(m == -INFINITY ? 0.f : s * __expf(m - bm));
  if (lane == 0) ss[w] = bs;
  // first index of the row maximum: the smallest index among the threads
  // whose own maximum is it
  if (m != bm) am = a.V;
  for (int o = 32; o > 0; o >>= 1) am = min(am, __shfl_xor(am, o));
  if (lane == 0) sa[w] = am;
  __syncthreads();
  bs = ss[0] + ss[1] + ss[2] + ss[3];
  am = min(min(sa[0], sa[1]), min(sa[2], sa[3]));
  const int b = r / a.P, p = r - b * a.P;
  const int y = a.rec[(int64_t)b * a.rec_stride + a.T + a.P + p];
  const bool valid = y >= 0 && y < a.V;
  const float inv_s = 1.f / bs, inv_r = 1.f / (float)a.R;
  if (a.dlogits) {
    uint16_t* d = a.dlogits + (int64_t)r * a.Vp;
    // (software-pipelined: the next logits vector is requested before this
    // one's gradient is stored -- the store may alias it, so otherwise each
    // of the row's ~15 vectors per thread paid a full load latency)
    const int nvp = a.Vp / 8;
    uint4 nxt = t < nvp ? reinterpret_cast<const uint4*>(z)[t] : make_uint4(0u, 0u, 0u, 0u);
    for (int v = t; v < nvp; v += 256) {
      const uint4 cur = nxt;
      if (v + 256 < nvp) nxt = reinterpret_cast<const uint4*>(z)[v + 256];
      float f[8];
      unpack8(cur, f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int col = v * 8 + k;
        float g = 0.f;
        if (valid && col < a.V) g = (__expf(f[k] - bm) * inv_s - (col == y ? 1.f : 0.f)) * inv_r;
        f[k] = g;
      }
      reinterpret_cast<uint4*>(d)[v] = pack8(f);
    }
  }
  if (t == 0 && valid) {
    atomicAdd(&a.stats[0], __logf(bs) + bm - bf2f(z[y]));
    atomicAdd(&a.stats[1], am == y ? 1.f : 0.f);
    atomicAdd(&a.stats[2], 1.f);
  }
}

void launch_vocab_xent(const VocabXentArgs& a, hipStream_t s) {
  vocab_xent_kernel<<<a.R, 256, 0, s>>>(a);
}

}  // namespace mfl
