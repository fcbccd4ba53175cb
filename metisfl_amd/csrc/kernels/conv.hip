// K6: NHWC bf16 convolution forward / backward-data / backward-weight as
// implicit GEMMs on the gfx950 matrix cores (v_mfma_f32_16x16x32_bf16).
//
// The reference trains its conv nets through Keras Conv2D layers
// (examples/keras/models/cifar_cnn.py:21-34); the north-star replaces that
// with hand-written CDNA4 kernels.  Design (MI355X-first, not a port):
//
//  * Activations NHWC, weights KRSC ([Cout][R][S][Cin]) so that the GEMM
//    reduction dimension k = (r, s, c) is contiguous in BOTH operands for the
//    forward pass: every lane moves 16 B (8 channels) per load, and MFMA
//    operand fragments (8 consecutive k per lane) are read from LDS with one
//    ds_read_b128.  Cin must be a multiple of 8 (the 3-channel CIFAR input is
//    zero-padded to 8 channels once, at shard creation).
//  * dgrad is the same kernel with a stride-aware gather of dY; its B operand
//    (W^T) is staged from the KRSC weight as [k][c] tiles and read with the
//    transposing ds_read_b64_tr_b16, so no weight transpose pass exists.
//  * wgrad reduces over the N*P*Q pixels, which are strided in both operands:
//    tiles are staged [m][col] in LDS and the MFMA fragments are formed with
//    ds_read_b64_tr_b16 (guide T10).
//  * Operand tiles move global -> LDS with LDS-DMA buffer loads
//    (buffer_load_dwordx4 ... lds): no VGPR staging, bounds-checked in
//    hardware (an out-of-range offset reads zeros: padding and ragged edges
//    cost no branch), 3 LDS stages with 2 k-tiles in flight, ONE barrier
//    per k-step and hand-counted vmcnt waits (guide §5 'Async global->LDS
//    copy', Three .s-level traps).  Round-1 measurements: the register-staged
//    version was latency-bound -- hipcc drained vmcnt(0) before every LDS
//    store, serialising the pipeline on the small-M CIFAR layers.
//  * LDS tiles are unpadded 128/256-byte rows (a DMA instruction writes 1 KiB
//    contiguously) with XOR swizzles chosen per read pattern so that both
//    ds_read_b128 fragments and ds_read_b64_tr_b16 fragments are bank-
//    conflict-free (derivation at swz_b128 / swz_tr below).
//  * Index math stays off the VALU critical path: kernel size and stride are
//    template parameters, channel / spatial divisions by powers of two become
//    host-computed shifts.
//  * Epilogue through LDS: the fp32 tile is staged in LDS and written as 16-B
//    bf16 vectors; the per-channel BatchNorm sums of the bf16 output are
//    reduced in the same pass and added with fp64 atomics into a [2][C]
//    accumulator (no separate statistics pass).
//  * Small-M layers (CIFAR 4x4 / 8x8 stages) use split-K to fill >= 256 CUs.
//    The reduction happens IN the kernel: every slice publishes its fp32
//    tile slab with write-through (sc1) stores and draws an arrival ticket;
//    the last-arriving slice (guide "In-launch split-K reduction", write-
//    through form) sums the slabs in slice order with sc1 loads and runs the
//    epilogue -- no reduction launch, no L2 write-back fence.  wgrad split-K
//    slices accumulate with fp32 atomics into the pre-zeroed gradient buffer.
//  * Stride-2 dgrad runs parity-class decomposed (conv_gemm_kernel PAR): no
//    MFMA work or operand traffic on the structurally zero taps.
#include "kernels/common.h"
#include "kernels/conv.h"
#include "kernels/lds_tiles.h"
#include "kernels/opt_tail_dev.h"

#ifndef MFL_CONV_DBG
#define MFL_CONV_DBG 0  // timing experiments only: bit0 skip MFMAs, bit1 skip operand DMA (compile-time: a runtime test split the k-loop into basic blocks)
#endif

namespace mfl {

constexpr int kBK = 64;      // k-tile (elements); one 128-byte bf16 row per operand row
#ifndef MFL_CONV_STAGES
#define MFL_CONV_STAGES 3  // measured: 4 stages (3 tiles in flight) is 4% slower end to end
#endif
constexpr int kStages = MFL_CONV_STAGES;  // LDS ring: tile kt computing, the next kStages-1 landing
static_assert(kStages >= 2 && kStages <= 4, "dma_k_loop counts at most 3 tiles in flight");

__device__ __forceinline__ int sdiv(int x, int d, int shift) { return shift >= 0 ? x >> shift : x / d; }

// GEMM row -> output pixel: identity, or the parity-class order of a
// stride-2 dgrad (see conv_gemm_kernel PAR): row = cls * Mc + (n, y, x) ->
// pixel (n, 2y + cls/2, 2x + cls%2) of the P x Q output.
__device__ __forceinline__ int out_pixel(const ConvArgs& a, int row) {
  if (!a.par_mc) return row;
  const int q2 = a.g.Q >> 1, pq2 = (a.g.P >> 1) * q2;
  const int cls = row / a.par_mc;
  const int mc = row - cls * a.par_mc;
  const int n = mc / pq2;
  const int rem = mc - n * pq2;
  const int y = rem / q2, x = rem - y * q2;
  return (n * a.g.P + 2 * y + (cls >> 1)) * a.g.Q + 2 * x + (cls & 1);
}

// Vectorised epilogue shared by the direct and the split-K paths:
// out[row][col] = bf16(v (+ y_old)), BN sums of the rounded output.
// `get(row_local, col_local_base, float[8])` supplies 8 consecutive fp32 values.
template <int BM, int BN, typename Getter>
__device__ __forceinline__ void tile_epilogue(const ConvArgs& a, int m0, int n0, float* red, Getter get) {
  const ConvGeom& g = a.g;
  uint16_t* y = a.y;
  const int accum = a.accum;
  // per-channel sums: forward BN statistics (v, v^2) of the output, or the
  // fused BN-backward reductions (g, g*xhat) of the consumer layer (dgrad)
  double* stats = a.bn_acc ? a.bn_acc : a.stats;
  constexpr int CPR = BN / 8;        // 16-B column groups per row
  constexpr int RPP = 256 / CPR;     // rows per pass
  const int t = threadIdx.x;
  const int cg = t % CPR, r0 = t / CPR;
  float s[8] = {0}, q[8] = {0};
  const int col = n0 + cg * 8;
  const bool col_ok = col < g.Ng;  // Ng % 8 == 0
  float mu[8], is[8], bv[8];
  if (a.bn_acc && col_ok) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      mu[k] = a.bn_mean[col + k];
      is[k] = a.bn_invstd[col + k];
    }
  }
  if (a.bias && col_ok) {
#pragma unroll
    for (int k = 0; k < 8; ++k) bv[k] = a.bias[col + k];
  }
  // every global read of the output stage (accumulated output, residual, the
  // consumer BN's mask y and input z) is issued for all of this thread's rows
  // before the first store (issued behind each row's possibly-aliasing store
  // they paid one load latency per row; conv32.hip's tile_epilogue32)
  constexpr int NIT = (BM + RPP - 1) / RPP;
  uint4 p_acc[NIT], p_res[NIT], p_y[NIT], p_z[NIT];
  const bool rd_y = a.bn_acc && a.bn_y, rd_z = stats && a.bn_acc;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int rl = r0 + it * RPP, row = m0 + rl;
    p_acc[it] = p_res[it] = p_y[it] = p_z[it] = make_uint4(0u, 0u, 0u, 0u);
    if (rl >= BM || row >= g.M || !col_ok) continue;
    const int64_t off = (int64_t)out_pixel(a, row) * g.Ng + col;
    if (accum) p_acc[it] = *reinterpret_cast<const uint4*>(y + off);
    if (a.resid) p_res[it] = *reinterpret_cast<const uint4*>(a.resid + off);
    if (rd_y) p_y[it] = *reinterpret_cast<const uint4*>(a.bn_y + off);
    if (rd_z) p_z[it] = *reinterpret_cast<const uint4*>(a.bn_z + off);
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int rl = r0 + it * RPP, row = m0 + rl;
    if (rl >= BM || row >= g.M || !col_ok) continue;
    float v[8];
    get(rl, cg * 8, v);
    const int64_t off = (int64_t)out_pixel(a, row) * g.Ng + col;
    uint16_t* dst = y + off;
    if (accum) {
      float o[8];
      unpack8(p_acc[it], o);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += o[k];
    }
    if (a.bias) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += bv[k];
    }
    if (a.resid) {
      float o[8];
      unpack8(p_res[it], o);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += o[k];
    }
    if (rd_y) {
      // the consumer BN's ReLU mask applied on the way out (as conv32.hip):
      // dX is stored as g = dX [y > 0], its BN backward reads no mask
      float ym[8];
      unpack8(p_y[it], ym);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = ym[k] > 0.f ? v[k] : 0.f;
    }
    const uint4 packed = pack8(v);
    *reinterpret_cast<uint4*>(dst) = packed;
    if (a.act_out) {  // exact (erf) GELU of the stored pre-activation
      float f[8], h[8];
      unpack8(packed, f);
#pragma unroll
      for (int k = 0; k < 8; ++k) h[k] = gelu_f(f[k]);
      *reinterpret_cast<uint4*>(a.act_out + off) = pack8(h);
    }
    if (stats) {
      float f[8];
      unpack8(packed, f);
      if (a.bn_acc) {
        float zz[8], ym[8];
        unpack8(p_z[it], zz);
        if (a.bn_y) unpack8(p_y[it], ym);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float gk = (a.bn_y && !(ym[k] > 0.f)) ? 0.f : f[k];
          s[k] += gk;
          q[k] += gk * ((zz[k] - mu[k]) * is[k]);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          s[k] += f[k];
          q[k] += f[k] * f[k];
        }
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

// The k-loop shared by the kernels: `issue(kt, stage)` starts the LDS-DMA of
// k-tile kt (L instructions per thread), `compute(stage)` runs its MFMAs.
//   iteration kt:  wait own DMA of tile kt (vmcnt: tile kt+1 may stay in
//   flight) -> barrier (every wave's tile kt landed AND every wave finished
//   reading stage (kt+2)%3 in iteration kt-1) -> issue tile kt+2 -> compute.
template <int L, typename Issue, typename Compute>
__device__ __forceinline__ void dma_k_loop(int nk, Issue& issue, Compute& compute) {
  constexpr int D = kStages - 1;  // k-tiles in flight
#pragma unroll
  for (int u = 0; u < D; ++u)
    if (u < nk) issue(u, u);
  int stage = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // own DMA of tile kt complete; the younger in-flight tiles may stay
    const int younger = min(D - 1, nk - 1 - kt);
    if (younger >= 2) wait_vmcnt<2 * L>();
    else if (younger == 1) wait_vmcnt<L>();
    else wait_vmcnt<0>();
    lds_barrier();
    if (kt + D < nk) issue(kt + D, stage == 0 ? kStages - 1 : stage - 1);
    compute(stage);
    stage = stage == kStages - 1 ? 0 : stage + 1;
  }
}

// ---------------------------------------------------------------------------
// Forward / dgrad implicit GEMM:  Y[m][n] = sum_k A[m][k] * B[n][k]
//
// PAR (stride-2 dgrad only): parity-class decomposition.  dX pixel (ih, iw)
// only receives the taps r == ih + pad (mod 2), s == iw + pad (mod 2): for a
// 3x3 kernel 4 / 2 / 2 / 1 of the 9 taps, for 1x1 one class gets its single
// tap and three get none.  The M rows are ordered class-major (4 classes of
// N x H/2 x W/2 pixels, a tile never straddles two), each class reduces only
// over its own taps (K_c = taps * Cout), and the epilogue scatters rows back
// to NHWC pixels.  Without it 3/4 of a stride-2 dgrad's MFMA work and operand
// traffic multiplies structural zeros.
// Block coordinates of a workgroup: blockIdx / gridDim of a plain launch, or
// decoded from the linear id of a paired launch (conv_bwd_pair_kernel).
struct BlkCoord {
  int x, y, z, gx, gy, gz;
};
__device__ __forceinline__ BlkCoord hw_coord() {
  return BlkCoord{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z,
                  (int)gridDim.x,  (int)gridDim.y,  (int)gridDim.z};
}

template <int BM, int BN, bool DGRAD, int KS, int ST, int BK, bool PAR = false>
__device__ __forceinline__ void conv_gemm_body(const ConvArgs& a, const BlkCoord bc, uint8_t* smem) {
  // BK = 64 or 128 k-elements per tile: [row][k] tiles have ROWA-byte rows
  constexpr int ROWA = BK * 2;
  constexpr int A_RPI = 1024 / ROWA;   // rows per 1-KiB DMA instruction
  constexpr int A_CPR = ROWA / 16;     // 16-B chunks per row
  constexpr int ACH = BM * BK / 2048;  // A DMA instructions per thread per k-tile
  constexpr int BCH = BN * BK / 2048;  // B DMA instructions per thread per k-tile
  constexpr int TM = BM / 32;          // 16x16 MFMA tiles per wave along M
  constexpr int TN = BN / 32;
  constexpr int A_BYTES = BM * ROWA;
  constexpr int B_ROWB = DGRAD ? BN * 2 : ROWA;  // dgrad B: [BK k][BN] rows
  constexpr int STAGE = A_BYTES + BN * BK * 2;   // both B layouts hold BN*BK bf16
  const ConvGeom& g = a.g;
  const auto rsA = make_rsrc(a.src, a.src_bytes);
  const auto rsB = make_rsrc(a.wgt, a.wgt_bytes);
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = bc.x * BM;
  const int n0 = bc.y * BN;
  const int kbeg = bc.z * a.kchunk;
  // parity class of this tile (block-uniform): first taps r0 / s0, tap counts
  // ns (along s), offsets dh / dw of the dY row / column of tap 0
  int cls = 0, r0 = 0, s0 = 0, ns = 1, dh = 0, dw = 0, kc_end = g.K;
  if constexpr (PAR) {
    cls = m0 / a.par_mc;
    const int qh = cls >> 1, qw = cls & 1;
    r0 = (qh + g.pad) & 1;
    s0 = (qw + g.pad) & 1;
    const int nr = (KS - r0 + 1) >> 1;
    ns = (KS - s0 + 1) >> 1;
    dh = (qh + g.pad - r0) >> 1;
    dw = (qw + g.pad - s0) >> 1;
    kc_end = nr * ns * g.C;
  }
  const int kend = min(kc_end, kbeg + a.kchunk);
  const int nk = max(0, (kend - kbeg + BK - 1) / BK);
  const int HWC = g.H * g.W * g.C;

  // A DMA: instruction i of wave w fills rows (w + 4i)*A_RPI .. (1 KiB); lane
  // -> row lrow + 4*A_RPI*i, physical chunk lane % A_CPR, logical chunk (k
  // offset) below -- the same for every i: the row step (32 or 16) leaves the
  // swizzle bits unchanged.
  constexpr int A_ISTEP = 4 * A_RPI;
  const int lrow = wave * A_RPI + lane / A_CPR;
  const int a_kc = ((lane % A_CPR) ^ swz_b128<ROWA>(lrow)) * 8;
  int a_nb[ACH], a_y0[ACH], a_x0[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int m = m0 + lrow + A_ISTEP * i;
    const int mm = m < g.M ? m : 0;
    if constexpr (PAR) {
      // (n, y, x) inside the class; dY row of tap j_r is y + dh - j_r
      const int q2 = g.Q >> 1;
      const int pq2 = (g.P >> 1) * q2;
      const int mc = mm - cls * a.par_mc;
      const int n = mc / pq2;
      const int rem = mc - n * pq2;
      const int y = rem / q2;
      a_nb[i] = n * HWC;
      a_y0[i] = y + dh;
      a_x0[i] = rem - y * q2 + dw;
      if (m >= g.M) a_y0[i] = -(1 << 28);
      continue;
    }
    const int n = sdiv(mm, g.P * g.Q, a.pq_shift);
    const int rem = mm - n * g.P * g.Q;
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
    if (m >= g.M) a_y0[i] = -(1 << 28);  // forces the OOB offset
  }
  // B DMA mapping.  fwd: rows n (128 B = 64 k), same as A.  dgrad: rows k of
  // B_ROWB bytes; instruction i of wave w fills bytes (w + 4i) KiB.
  constexpr int B_RPI = 1024 / B_ROWB;  // rows per DMA instruction
  constexpr int B_CPR = B_ROWB / 16;    // chunks per row
  const int b_row0 = wave * B_RPI + lane / B_CPR;   // + 4*B_RPI*i
  const int b_pch = lane % B_CPR;

  auto issue = [&](int kt, int stage) {
    if constexpr (MFL_CONV_DBG & 2) return;
    uint8_t* st = smem + stage * STAGE;
    const int kb = kbeg + kt * BK;
    {
      const int k = kb + a_kc;
      const int rs = sdiv(k, g.C, a.c_shift);
      const int c = k - rs * g.C;
      // PAR: rs is the class tap index (j_r, j_s), j_s fastest
      const int r = PAR ? (ns == 2 ? rs >> 1 : rs) : rs / KS;
      const int s = PAR ? rs - r * ns : rs - r * KS;
      const bool kv = k < kend;
#pragma unroll
      for (int i = 0; i < ACH; ++i) {
        int iy, ix;
        bool ok;
        if (PAR) {
          iy = a_y0[i] - r;
          ix = a_x0[i] - s;
          ok = kv & (iy >= 0) & (ix >= 0);
        } else if (DGRAD) {
          const int ty = a_y0[i] - r, tx = a_x0[i] - s;
          ok = kv & (ty >= 0) & (tx >= 0);
          if (ST > 1) ok = ok & ((ty % ST) == 0) & ((tx % ST) == 0);
          iy = ty / ST;
          ix = tx / ST;
        } else {
          iy = a_y0[i] + r;
          ix = a_x0[i] + s;
          ok = kv & (iy >= 0) & (ix >= 0);
        }
        ok = ok & (iy < g.H) & (ix < g.W);
        const uint32_t off = ok ? (uint32_t)(a_nb[i] + (iy * g.W + ix) * g.C + c) * 2u : kOOB;
        dma16(rsA, off, st + (wave + 4 * i) * 1024);
      }
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      uint32_t off;
      if constexpr (DGRAD) {
        // B[k][n] = W[ko][r][s][n], k = (r, s, ko)
        const int row = b_row0 + 4 * B_RPI * i;          // k row within the tile
        const int n = n0 + ((b_pch ^ swz_tr<B_ROWB>(row)) * 8);
        const int kr = kb + row;
        int rs = sdiv(kr, g.C, a.c_shift);
        const int ko = kr - rs * g.C;
        if (PAR) {  // class tap index -> kernel tap (r0 + 2 j_r, s0 + 2 j_s)
          const int jr = ns == 2 ? rs >> 1 : rs;
          rs = (r0 + 2 * jr) * KS + s0 + 2 * (rs - jr * ns);
        }
        off = ((kr < kend) & (n < g.Ng)) ? (uint32_t)((ko * KS * KS + rs) * g.Ng + n) * 2u : kOOB;
      } else {
        const int n = n0 + lrow + A_ISTEP * i;
        const int k = kb + a_kc;
        off = ((k < kend) & (n < g.Ng)) ? (uint32_t)(n * g.K + k) * 2u : kOOB;
      }
      dma16(rsB, off, st + A_BYTES + (wave + 4 * i) * 1024);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) {
    if constexpr (MFL_CONV_DBG & 1) return;
    const uint8_t* As = smem + stage * STAGE;
    const uint8_t* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = b128_frag<ROWA>(As, kk, wm * (BM / 2) + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (DGRAD) bfr[j] = tr_frag<B_ROWB>(Bs, kk, wn * (BN / 2) + 16 * j, lane);
        else bfr[j] = b128_frag<ROWA>(Bs, kk, wn * (BN / 2) + 16 * j, lane);
      }
      if constexpr (DGRAD) frags_ready(bfr);  // asm tr-reads: not tracked by hipcc
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  };
  dma_k_loop<ACH + BCH>(nk, issue, compute);
  __syncthreads();  // every wave done with the ring before smem is reused

  // ---- epilogue -----------------------------------------------------------
  constexpr int TST = BN + 4;
  float* tile = reinterpret_cast<float*>(smem);
  const int fr = lane & 15;
  const int rl0 = wm * (BM / 2) + (lane >> 4) * 4;
  const int cl0 = wn * (BN / 2) + fr;
  const int splits = bc.gz;
  const int tile_id = bc.y * bc.gx + bc.x;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) tile[(rl0 + 16 * i + e) * TST + cl0 + 16 * j] = acc[i][j][e];
  __syncthreads();
  if (splits > 1) {
    // Split-K, in-launch (guide §5 'In-launch split-K reduction', write-
    // through form).  Every slice publishes its fp32 slab [BM][BN] with sc1
    // (write-through) 16-B stores -- no agent release, whose L2 write-back
    // of the freshly dirtied slab measured ~5 µs per launch here -- drains
    // them, and draws a ticket; the last arriver adds the other slabs (sc1
    // loads: misses its own possibly stale L2) onto its own LDS tile.
    constexpr int F = BM * BN / 1024;  // float4 per thread
    constexpr int C4 = BN / 4;
    const int ntiles = bc.gx * bc.gy;
    const int64_t zstride = (int64_t)ntiles * BM * BN * 4;  // bytes between slices
    const auto rsS = make_rsrc(a.ysplit + (int64_t)tile_id * (BM * BN), 0x7FFFFFF0u);
    const uint32_t zoff = (uint32_t)(bc.z * zstride);
#pragma unroll
    for (int u = 0; u < F; ++u) {
      const int f = t + 256 * u;
      const float4 v = *reinterpret_cast<const float4*>(tile + (f / C4) * TST + (f % C4) * 4);
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)},
          rsS, (int)(zoff + f * 16), 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    int* flag = reinterpret_cast<int*>(tile + BM * TST + 256 * 16);
    if (t == 0) {
      const int prev = __hip_atomic_fetch_add(&a.counters[tile_id], 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == splits - 1;
      // re-arm for the next launch (graph replay): nobody else touches it now
      if (last) __hip_atomic_store(&a.counters[tile_id], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    float4 sum[F];
#pragma unroll
    for (int u = 0; u < F; ++u) sum[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    // slices summed in z order whichever slice reduces: bitwise deterministic
    for (int z = 0; z < splits; ++z) {
      float4 r[F];
      if (z == bc.z) {
#pragma unroll
        for (int u = 0; u < F; ++u) {
          const int f = t + 256 * u;
          r[u] = *reinterpret_cast<const float4*>(tile + (f / C4) * TST + (f % C4) * 4);
        }
      } else {
#pragma unroll
        for (int u = 0; u < F; ++u) {
          const u32x4 b =
              __builtin_amdgcn_raw_buffer_load_b128(rsS, (int)(z * zstride + (t + 256 * u) * 16), 0, 16);
          r[u] = make_float4(__uint_as_float(b[0]), __uint_as_float(b[1]), __uint_as_float(b[2]),
                             __uint_as_float(b[3]));
        }
      }
#pragma unroll
      for (int u = 0; u < F; ++u) {
        sum[u].x += r[u].x;
        sum[u].y += r[u].y;
        sum[u].z += r[u].z;
        sum[u].w += r[u].w;
      }
    }
    __syncthreads();  // every thread has read its own-slice values from the tile
#pragma unroll
    for (int u = 0; u < F; ++u) {
      const int f = t + 256 * u;
      *reinterpret_cast<float4*>(tile + (f / C4) * TST + (f % C4) * 4) = sum[u];
    }
    __syncthreads();
  }
  tile_epilogue<BM, BN>(a, m0, n0, tile + BM * TST,
                        [&](int rl, int cl, float* v) {
                          const float4 p = *reinterpret_cast<const float4*>(tile + rl * TST + cl);
                          const float4 q = *reinterpret_cast<const float4*>(tile + rl * TST + cl + 4);
                          v[0] = p.x; v[1] = p.y; v[2] = p.z; v[3] = p.w;
                          v[4] = q.x; v[5] = q.y; v[6] = q.z; v[7] = q.w;
                        });
}

// ---------------------------------------------------------------------------
// wgrad:  dW[ko][j] = sum_m dY[m][ko] * im2col(X)[m][j],  j = (r, s, c)
// Tiles: A = dY [64 m][64 ko], B = im2col(X) [64 m][64 j], both 128-B rows,
// both read with transposing LDS reads.

template <int BM, int BN, bool DGRAD, int KS, int ST, int BK, bool PAR = false>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  conv_gemm_body<BM, BN, DGRAD, KS, ST, BK, PAR>(a, hw_coord(), smem);
}

template <int KS, int ST, int BK>
__device__ __forceinline__ void conv_wgrad_body(const ConvArgs& a, float* __restrict__ dw, const BlkCoord bc,
                                                uint8_t* smem) {
  // g: H,W,C = X dims; P,Q = dY spatial; Ng = Cout; K = R*S*C; M = N*P*Q
  constexpr int BM = 64, BN = 64;
  constexpr int TM = 2, TN = 2;
  constexpr int T_BYTES = BK * 128;   // [BK m][64 cols], 128-B rows
  constexpr int NI = BK / 32;         // DMA instructions per operand per thread
  constexpr int STAGE = 2 * T_BYTES;
  const ConvGeom& g = a.g;
  const auto rsA = make_rsrc(a.src, a.src_bytes);
  const auto rsB = make_rsrc(a.wgt, a.wgt_bytes);
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ko0 = bc.x * BM;
  const int j0 = bc.y * BN;
  const int mbeg = bc.z * a.kchunk;
  const int mend = min(g.M, mbeg + a.kchunk);
  const int nk = (mend - mbeg + BK - 1) / BK;

  // DMA mapping (both operands): instruction i of wave w fills m-rows
  // (w + 4i)*8 .. +8; lane -> row lrow + 32 i, physical chunk lane&7.
  const int lrow = wave * 8 + (lane >> 3);
  const int pch = lane & 7;
  // The swizzle key of row lrow + 32i equals that of lrow (bits 1 and 3).
  const int col = (pch ^ swz_tr<128>(lrow)) * 8;  // column offset inside the tile
  const int ko = ko0 + col;
  const int j = j0 + col;
  const bool j_ok = j < g.K;
  const int rsj = sdiv(j_ok ? j : 0, g.C, a.c_shift);
  const int b_c = (j_ok ? j : 0) - rsj * g.C;
  const int b_r = rsj / KS;
  const int b_s = rsj - b_r * KS;
  const int HWC = g.H * g.W * g.C;
  const int PQ = g.P * g.Q;

  auto issue = [&](int kt, int stage) {
    if constexpr (MFL_CONV_DBG & 2) return;
    uint8_t* st = smem + stage * STAGE;
    const int mb = mbeg + kt * BK;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int m = mb + lrow + 32 * i;
      const bool mv = m < mend;
      dma16(rsA, (mv & (ko < g.Ng)) ? (uint32_t)(m * g.Ng + ko) * 2u : kOOB, st + (wave + 4 * i) * 1024);
      const int n = sdiv(m, PQ, a.pq_shift);
      const int rem = m - n * PQ;
      const int oy = sdiv(rem, g.Q, a.q_shift);
      const int ox = rem - oy * g.Q;
      const int iy = oy * ST - g.pad + b_r;
      const int ix = ox * ST - g.pad + b_s;
      const bool ok = j_ok & mv & (iy >= 0) & (ix >= 0) & (iy < g.H) & (ix < g.W);
      dma16(rsB, ok ? (uint32_t)(n * HWC + (iy * g.W + ix) * g.C + b_c) * 2u : kOOB,
            st + T_BYTES + (wave + 4 * i) * 1024);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jj = 0; jj < TN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int stage) {
    if constexpr (MFL_CONV_DBG & 1) return;
    const uint8_t* As = smem + stage * STAGE;
    const uint8_t* Bs = As + T_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tr_frag<128>(As, kk, wm * (BM / 2) + 16 * i, lane);
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) bfr[jj] = tr_frag<128>(Bs, kk, wn * (BN / 2) + 16 * jj, lane);
      frags_ready(af);  // asm tr-reads: not tracked by hipcc
      frags_ready(bfr);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) acc[i][jj] = mfma16(af[i], bfr[jj], acc[i][jj]);
    }
  };
  dma_k_loop<2 * NI>(nk, issue, compute);

  // split-K slices (or an accumulating caller) add into the gradient slot
  const int rbase = ko0 + wm * (BM / 2) + (lane >> 4) * 4;
  const int cbase = j0 + wn * (BN / 2) + (lane & 15);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int jj = 0; jj < TN; ++jj)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rbase + 16 * i + e, cc = cbase + 16 * jj;
        if (row < g.Ng && cc < g.K) {
          if (bc.gz > 1 || a.accum)
            atomicAdd(&dw[(int64_t)row * g.K + cc], acc[i][jj][e]);
          else
            dw[(int64_t)row * g.K + cc] = acc[i][jj][e];
        }
      }
}

template <int KS, int ST, int BK>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvArgs a, float* __restrict__ dw) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  conv_wgrad_body<KS, ST, BK>(a, dw, hw_coord(), smem);
}

// ---------------------------------------------------------------------------
// A layer's dgrad and wgrad in ONE launch (horizontal fusion).  Both consume
// the same dY and are independent; as two launches each is latency-bound
// (256-576 small workgroups, few k-steps) and the second starts only after
// the first's tail.  In one grid their workgroups share the CUs -- the dgrad
// runs with BK = 64 here so that every workgroup of the launch fits in
// <= 74 KiB of LDS (two per CU).  Block ids [0, nd) are the dgrad grid
// (x fastest, then y, z), [nd, nd + nw) the wgrad grid.  Measured upper bound
// (scripts/conv_pair_probe.py, two unsynchronised streams): 28-30 -> 20-23 us
// per layer pair.
struct PairGrid {
  int dgx, dgy, dgz, wgx, wgy, wgz;
  int order;  // block-id order: 0 dgrad first, 1 wgrad first, 2 alternating (MFL_CONV_PAIR_ORDER)
};
template <int BM, int BN, int KS, int ST, bool PAR>
__global__ __launch_bounds__(256) void conv_bwd_pair_kernel(ConvArgs da, ConvArgs wa, float* __restrict__ dw,
                                                            PairGrid pg, OptTail ot) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int id = blockIdx.x;
  const int nd = pg.dgx * pg.dgy * pg.dgz, nw = pg.wgx * pg.wgy * pg.wgz;
  if (id >= nd + nw) {  // optimizer tail (opt_tail.h), dispatched after both GEMMs
    opt_tail_body(ot, id - nd - nw);
    return;
  }
  bool isd;
  int lid;
  if (pg.order == 0) {
    isd = id < nd;
    lid = isd ? id : id - nd;
  } else if (pg.order == 1) {
    isd = id >= nw;
    lid = isd ? id - nw : id;
  } else {
    const int m = min(nd, nw);
    if (id < 2 * m) {
      isd = !(id & 1);
      lid = id >> 1;
    } else {
      isd = nd > nw;
      lid = id - m;
    }
  }
  if (isd) {
    const int x = lid % pg.dgx, r = lid / pg.dgx;
    conv_gemm_body<BM, BN, true, KS, ST, 64, PAR>(
        da, BlkCoord{x, r % pg.dgy, r / pg.dgy, pg.dgx, pg.dgy, pg.dgz}, smem);
  } else {
    const int x = lid % pg.wgx, r = lid / pg.wgx;
    conv_wgrad_body<KS, ST, 64>(wa, dw, BlkCoord{x, r % pg.wgy, r / pg.wgy, pg.wgx, pg.wgy, pg.wgz}, smem);
  }
}

// Two forward convolutions of one input in ONE launch: a downsampling
// block's 3x3 / stride-2 conv1 and its 1x1 / stride-2 projection shortcut
// (independent, each latency-bound at 64-128 workgroups), BK = 64 for both.
// Block ids [0, n1) run conv1 (grid dgx/dgy/dgz), the rest the shortcut.
template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_fwd_pair_kernel(ConvArgs a1, ConvArgs a2, PairGrid pg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int id = blockIdx.x;
  const int n1 = pg.dgx * pg.dgy * pg.dgz;
  if (id < n1) {
    const int x = id % pg.dgx, r = id / pg.dgx;
    conv_gemm_body<BM, BN, false, 3, 2, 64, false>(
        a1, BlkCoord{x, r % pg.dgy, r / pg.dgy, pg.dgx, pg.dgy, pg.dgz}, smem);
  } else {
    const int lid = id - n1;
    const int x = lid % pg.wgx, r = lid / pg.wgx;
    conv_gemm_body<BM, BN, false, 1, 2, 64, false>(
        a2, BlkCoord{x, r % pg.wgy, r / pg.wgy, pg.wgx, pg.wgy, pg.wgz}, smem);
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

// bf16 element count -> buffer range in bytes (32-bit descriptor range; the
// bindings reject tensors this large before launch)
static uint32_t range_bytes(int64_t elems) {
  const int64_t b = elems * 2;
  return b >= (int64_t)kOOB ? kOOB : (uint32_t)b;
}

static void fill_shifts(ConvArgs& a) {
  a.c_shift = log2_exact(a.g.C);
  a.q_shift = log2_exact(a.g.Q);
  a.pq_shift = log2_exact(a.g.P * a.g.Q);
  static const int dbg = [] {
    const char* v = getenv("MFL_CONV_DEBUG");
    return v && *v ? atoi(v) : 0;
  }();
  a.dbg = dbg;
}

template <typename K>
static void set_lds_limit(K* kernel, size_t lds, bool& done) {
  if (!done && lds > 65536) {  // > 64 KiB of dynamic LDS must be opted into
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    done = true;
  }
}

template <int BM, int BN, bool DG, int KS, int ST, int BK, bool PAR>
static void launch_gemm_t(const ConvArgs& a, const ConvPlan& p, hipStream_t s) {
  dim3 grid((a.g.M + BM - 1) / BM, (a.g.Ng + BN - 1) / BN, p.splits);
  size_t lds = (size_t)kStages * (BM + BN) * BK * 2;
  const size_t epi = ((size_t)BM * (BN + 4) + 256 * 16 + 8) * sizeof(float);
  if (lds < epi) lds = epi;
  static bool attr_set = false;
  set_lds_limit(&conv_gemm_kernel<BM, BN, DG, KS, ST, BK, PAR>, lds, attr_set);
  conv_gemm_kernel<BM, BN, DG, KS, ST, BK, PAR><<<grid, 256, lds, s>>>(a);
}

template <int BM, int BN, bool DG, int KS, int ST>
static void launch_gemm_bk(const ConvArgs& a, const ConvPlan& p, hipStream_t s) {
  if constexpr (DG && ST == 2) {
    if (a.par_mc) {  // parity-decomposed stride-2 dgrad
      if (p.bk == 128) launch_gemm_t<BM, BN, DG, KS, ST, 128, true>(a, p, s);
      else launch_gemm_t<BM, BN, DG, KS, ST, 64, true>(a, p, s);
      return;
    }
  }
  if (p.bk == 128) launch_gemm_t<BM, BN, DG, KS, ST, 128, false>(a, p, s);
  else launch_gemm_t<BM, BN, DG, KS, ST, 64, false>(a, p, s);
}

template <int BM, int BN, bool DG>
static void launch_gemm_ks(const ConvArgs& a, const ConvPlan& p, hipStream_t s) {
  const int ks = a.g.R, st = a.g.stride;
  if (ks == 3 && st == 1) launch_gemm_bk<BM, BN, DG, 3, 1>(a, p, s);
  else if (ks == 3 && st == 2) launch_gemm_bk<BM, BN, DG, 3, 2>(a, p, s);
  else if (ks == 1 && st == 1) launch_gemm_bk<BM, BN, DG, 1, 1>(a, p, s);
  else if (ks == 1 && st == 2) launch_gemm_bk<BM, BN, DG, 1, 2>(a, p, s);
}

bool conv_supported(const ConvGeom& g) {
  return g.R == g.S && (g.R == 1 || g.R == 3) && (g.stride == 1 || g.stride == 2);
}

// Split-K policy.  A block's k-loop is a serial chain of ~latency/2 per
// k-step (two tiles in flight, almost no MFMA work per step at CIFAR sizes),
// so the plan trades k-steps per block for blocks: split until the grid
// reaches `target` workgroups (several per CU to overlap their chains) while
// every slice keeps >= `min_steps` k-steps.  Tunable for sweeps through
// MFL_CONV_TARGET_BLOCKS / MFL_CONV_MIN_KSTEPS / MFL_WGRAD_TARGET_BLOCKS.
static int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

// Run-time split targets (set_conv_plan_targets: the co-located learners'
// regime, models/colocated.py): with several learners' launches sharing the
// CUs, fewer and fuller split-K slices win; the environment variables still
// override both (sweeps).  Targets only lower split counts, so workspaces
// sized for the default plans still fit.
static int g_conv_target_rt = 0, g_wgrad_target_rt = 0;
void set_conv_plan_targets(int conv_target, int wgrad_target) {
  g_conv_target_rt = conv_target;
  g_wgrad_target_rt = wgrad_target;
}

ConvPlan plan_conv_gemm(const ConvGeom& g, bool dgrad) {
  static const int target_env = env_int("MFL_CONV_TARGET_BLOCKS", 0);
  const int target = target_env > 0 ? target_env : (g_conv_target_rt > 0 ? g_conv_target_rt : 256);
  static const int min_steps = env_int("MFL_CONV_MIN_KSTEPS", 4);
  static const int parity_on = env_int("MFL_DGRAD_PARITY", 1);
  ConvPlan p;
  p.bm = g.M >= 8192 ? 128 : 64;
  p.bn = g.Ng >= 128 && g.M >= 16384 ? 128 : 64;
  const int tiles = ((g.M + p.bm - 1) / p.bm) * ((g.Ng + p.bn - 1) / p.bn);
  // stride-2 dgrad: parity classes of N x P/2 x Q/2 rows (whole tiles each);
  // a class reduces over at most ceil(R/2) * ceil(S/2) taps
  int K = g.K;
  // (3x3 only: a 1x1 stride-2 dgrad already skips its zero taps through the
  // out-of-range DMA path, and measured no faster decomposed)
  if (dgrad && parity_on && g.R == 3 && g.stride == 2 && g.P % 2 == 0 && g.Q % 2 == 0) {
    const int mc = g.N * (g.P / 2) * (g.Q / 2);
    if (mc % p.bm == 0) {
      p.par_mc = mc;
      K = ((g.R + 1) / 2) * ((g.S + 1) / 2) * g.C;
    }
  }
  // 128-deep k-tiles halve the serial k-steps (and barriers) of a block when
  // the reduction is long enough; the 128x128 tile keeps BK = 64 (LDS)
  static const int bk128_min_k = env_int("MFL_CONV_BK128_MIN_K", 512);  // measured best (r1 sweep)
  p.bk = (K >= bk128_min_k && !(p.bm == 128 && p.bn == 128)) ? 128 : 64;
  const int ksteps = (K + p.bk - 1) / p.bk;
  int splits = 1;
  while (tiles * splits < target && ksteps / (splits * 2) >= min_steps && splits < 16) splits *= 2;
  p.splits = splits;
  p.kchunk = ((ksteps + splits - 1) / splits) * p.bk;
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
  a.src_bytes = range_bytes((int64_t)g.N * g.H * g.W * g.C);
  a.wgt_bytes = range_bytes((int64_t)g.Ng * g.K);
  a.y = y;
  a.ysplit = ysplit;
  a.counters = counters;
  a.stats = stats;
  a.kchunk = p.kchunk;
  a.accum = accum ? 1 : 0;
  a.par_mc = dgrad ? p.par_mc : 0;
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

void launch_conv_gemm_epi(const ConvGeom& g, const ConvPlan& p, const uint16_t* src,
                          const uint16_t* wgt, uint16_t* y, float* ysplit, int* counters,
                          const GemmEpilogueArgs& e, hipStream_t s) {
  ConvArgs a{};
  a.g = g;
  a.src = src;
  a.wgt = wgt;
  a.src_bytes = range_bytes((int64_t)g.N * g.H * g.W * g.C);
  a.wgt_bytes = range_bytes((int64_t)g.Ng * g.K);
  a.y = y;
  a.ysplit = ysplit;
  a.counters = counters;
  a.kchunk = p.kchunk;
  a.bias = e.bias;
  a.resid = e.resid;
  a.act_out = e.act_out;
  fill_shifts(a);
  if (p.bm == 128 && p.bn == 128) launch_gemm_ks<128, 128, false>(a, p, s);
  else if (p.bm == 128 && p.bn == 64) launch_gemm_ks<128, 64, false>(a, p, s);
  else if (p.bm == 64 && p.bn == 64) launch_gemm_ks<64, 64, false>(a, p, s);
}

void launch_conv_dgrad_bnb(const ConvGeom& g, const ConvPlan& p, const uint16_t* dy,
                           const uint16_t* wgt, uint16_t* dx, float* ysplit, int* counters,
                           bool accum, const BnBwdFusion& f, hipStream_t s) {
  ConvArgs a{};
  a.g = g;
  a.src = dy;
  a.wgt = wgt;
  a.src_bytes = range_bytes((int64_t)g.N * g.H * g.W * g.C);
  a.wgt_bytes = range_bytes((int64_t)g.Ng * g.K);
  a.y = dx;
  a.ysplit = ysplit;
  a.counters = counters;
  a.kchunk = p.kchunk;
  a.accum = accum ? 1 : 0;
  a.bn_z = f.z;
  a.bn_y = f.y;
  a.bn_mean = f.mean;
  a.bn_invstd = f.invstd;
  a.bn_acc = f.acc;
  a.par_mc = p.par_mc;
  fill_shifts(a);
  if (p.bm == 128 && p.bn == 128) launch_gemm_ks<128, 128, true>(a, p, s);
  else if (p.bm == 128 && p.bn == 64) launch_gemm_ks<128, 64, true>(a, p, s);
  else if (p.bm == 64 && p.bn == 64) launch_gemm_ks<64, 64, true>(a, p, s);
}

ConvPlan plan_conv_wgrad(const ConvGeom& g, int target_blocks) {
  static const int target_env = env_int("MFL_WGRAD_TARGET_BLOCKS", 0);
  const int target = target_blocks > 0 ? target_blocks
                     : target_env > 0  ? target_env
                                       : (g_wgrad_target_rt > 0 ? g_wgrad_target_rt : 512);
  static const int min_steps = env_int("MFL_WGRAD_MIN_KSTEPS", 8);
  ConvPlan p;
  p.bm = 64;
  p.bn = 64;
  const int tiles = ((g.Ng + 63) / 64) * ((g.K + 63) / 64);
  static const int bk128_min_m = env_int("MFL_WGRAD_BK128_MIN_M", 1 << 30);
  p.bk = g.M >= bk128_min_m ? 128 : 64;
  const int ksteps = (g.M + p.bk - 1) / p.bk;
  int splits = 1;
  while (tiles * splits < target && ksteps / (splits * 2) >= min_steps && splits < 64) splits *= 2;
  p.splits = splits;
  p.kchunk = ((ksteps + splits - 1) / splits) * p.bk;
  p.stats_rows = 0;
  return p;
}

template <int BK>
static void launch_wgrad_ks(const ConvArgs& a, dim3 grid, int ks, int st, float* dw, hipStream_t s) {
  const size_t lds = (size_t)kStages * 2 * BK * 128;
  static bool attr[4] = {false, false, false, false};
  if (ks == 3 && st == 1) {
    set_lds_limit(&conv_wgrad_kernel<3, 1, BK>, lds, attr[0]);
    conv_wgrad_kernel<3, 1, BK><<<grid, 256, lds, s>>>(a, dw);
  } else if (ks == 3 && st == 2) {
    set_lds_limit(&conv_wgrad_kernel<3, 2, BK>, lds, attr[1]);
    conv_wgrad_kernel<3, 2, BK><<<grid, 256, lds, s>>>(a, dw);
  } else if (ks == 1 && st == 1) {
    set_lds_limit(&conv_wgrad_kernel<1, 1, BK>, lds, attr[2]);
    conv_wgrad_kernel<1, 1, BK><<<grid, 256, lds, s>>>(a, dw);
  } else if (ks == 1 && st == 2) {
    set_lds_limit(&conv_wgrad_kernel<1, 2, BK>, lds, attr[3]);
    conv_wgrad_kernel<1, 2, BK><<<grid, 256, lds, s>>>(a, dw);
  }
}

// dw must be zero on entry when p.splits > 1 (slices accumulate with fp32
// atomics); the training step gets that for free from the optimizer launch,
// which zeroes the gradient buffer after consuming it.
void launch_conv_wgrad(const ConvGeom& g, const ConvPlan& p, const uint16_t* x, const uint16_t* dy,
                       float* dw, hipStream_t s, bool accumulate) {
  ConvArgs a{};
  a.accum = accumulate ? 1 : 0;
  a.g = g;
  a.src = dy;
  a.wgt = x;
  a.src_bytes = range_bytes((int64_t)g.M * g.Ng);
  a.wgt_bytes = range_bytes((int64_t)g.N * g.H * g.W * g.C);
  a.kchunk = p.kchunk;
  fill_shifts(a);
  dim3 grid((g.Ng + 63) / 64, (g.K + 63) / 64, p.splits);
  const int ks = g.R, st = g.stride;
  if (p.bk == 128) launch_wgrad_ks<128>(a, grid, ks, st, dw, s);
  else launch_wgrad_ks<64>(a, grid, ks, st, dw, s);
}

// ---- paired dgrad + wgrad ----------------------------------------------------
namespace {
template <int BM, int BN, int KS, int ST, bool PAR>
void launch_pair_t(const ConvArgs& da, const ConvArgs& wa, float* dw, const PairGrid& pg, hipStream_t s,
                   const OptTail& ot) {
  size_t lds = (size_t)kStages * (BM + BN) * 64 * 2;
  const size_t epi = ((size_t)BM * (BN + 4) + 256 * 16 + 8) * sizeof(float);
  const size_t wl = (size_t)kStages * 2 * 64 * 128;
  lds = std::max(lds, std::max(epi, wl));
  static bool attr = false;
  set_lds_limit(&conv_bwd_pair_kernel<BM, BN, KS, ST, PAR>, lds, attr);
  const unsigned n = (unsigned)(pg.dgx * pg.dgy * pg.dgz + pg.wgx * pg.wgy * pg.wgz + ot.nblk);
  conv_bwd_pair_kernel<BM, BN, KS, ST, PAR><<<n, 256, lds, s>>>(da, wa, dw, pg, ot);
}

template <int BM, int BN>
bool launch_pair_bm(const ConvArgs& da, const ConvArgs& wa, float* dw, const PairGrid& pg, hipStream_t s,
                    const OptTail& ot) {
  const int ks = da.g.R, st = da.g.stride;
  if (ks == 3 && st == 1) launch_pair_t<BM, BN, 3, 1, false>(da, wa, dw, pg, s, ot);
  else if (ks == 3 && st == 2 && da.par_mc) launch_pair_t<BM, BN, 3, 2, true>(da, wa, dw, pg, s, ot);
  else if (ks == 3 && st == 2) launch_pair_t<BM, BN, 3, 2, false>(da, wa, dw, pg, s, ot);
  else if (ks == 1 && st == 2) launch_pair_t<BM, BN, 1, 2, false>(da, wa, dw, pg, s, ot);
  else return false;
  return true;
}
}  // namespace

bool conv_pair_enabled() {
  static const int on = env_int("MFL_CONV_PAIR", 1);
  return on != 0;
}

bool launch_conv_bwd_pair(const ConvGeom& gd, const ConvPlan& pd_in, const uint16_t* dy, const uint16_t* wt,
                          uint16_t* dx, float* ysplit, int* counters, bool accum, const BnBwdFusion* f,
                          const ConvGeom& gw, const uint16_t* x, float* dw, hipStream_t s, const OptTail* ot) {
  if (!conv_pair_enabled()) return false;
  if (!((pd_in.bm == 128 && pd_in.bn == 64) || (pd_in.bm == 64 && pd_in.bn == 64))) return false;
  static const int wg_target = env_int("MFL_PAIR_WGRAD_TARGET", 0);
  const ConvPlan pw = plan_conv_wgrad(gw, wg_target);
  if (pw.bk != 64) return false;
  // the dgrad at BK = 64 with the SAME split count (the caller's workspace
  // and counter slots were sized for this plan)
  ConvPlan pd = pd_in;
  static const int dg_div = env_int("MFL_PAIR_DGRAD_SPLIT_DIV", 1);
  if (dg_div > 1) pd.splits = std::max(1, pd.splits / dg_div);  // fewer slices: fits the same workspace
  const int K = pd.par_mc ? ((gd.R + 1) / 2) * ((gd.S + 1) / 2) * gd.C : gd.K;
  const int ks64 = (K + 63) / 64;
  pd.bk = 64;
  pd.kchunk = ((ks64 + pd.splits - 1) / pd.splits) * 64;
  ConvArgs da{};
  da.g = gd;
  da.src = dy;
  da.wgt = wt;
  da.src_bytes = range_bytes((int64_t)gd.N * gd.H * gd.W * gd.C);
  da.wgt_bytes = range_bytes((int64_t)gd.Ng * gd.K);
  da.y = dx;
  da.ysplit = ysplit;
  da.counters = counters;
  da.kchunk = pd.kchunk;
  da.accum = accum ? 1 : 0;
  if (f) {
    da.bn_z = f->z;
    da.bn_y = f->y;
    da.bn_mean = f->mean;
    da.bn_invstd = f->invstd;
    da.bn_acc = f->acc;
  }
  da.par_mc = pd.par_mc;
  fill_shifts(da);
  ConvArgs wa{};
  // the training step's gradient buffer is zero on entry: split-K slices
  // add atomically (grid z > 1), an unsplit plan stores (as conv32.hip;
  // MFL_C32_WSTORE=0: always atomics)
  wa.accum = env_int("MFL_C32_WSTORE", 1) == 0 ? 1 : 0;
  wa.g = gw;
  wa.src = dy;
  wa.wgt = x;
  wa.src_bytes = range_bytes((int64_t)gw.M * gw.Ng);
  wa.wgt_bytes = range_bytes((int64_t)gw.N * gw.H * gw.W * gw.C);
  wa.kchunk = pw.kchunk;
  fill_shifts(wa);
  PairGrid pg;
  pg.dgx = (gd.M + pd.bm - 1) / pd.bm;
  pg.dgy = (gd.Ng + pd.bn - 1) / pd.bn;
  pg.dgz = pd.splits;
  pg.wgx = (gw.Ng + 63) / 64;
  pg.wgy = (gw.K + 63) / 64;
  pg.wgz = pw.splits;
  static const int order = env_int("MFL_CONV_PAIR_ORDER", 0);
  pg.order = order;
  const OptTail tail = ot ? *ot : OptTail{};
  if (pd.bm == 128) return launch_pair_bm<128, 64>(da, wa, dw, pg, s, tail);
  return launch_pair_bm<64, 64>(da, wa, dw, pg, s, tail);
}

namespace {
template <int BM, int BN>
void launch_fwd_pair_t(const ConvArgs& a1, const ConvArgs& a2, const PairGrid& pg, hipStream_t s) {
  size_t lds = (size_t)kStages * (BM + BN) * 64 * 2;
  const size_t epi = ((size_t)BM * (BN + 4) + 256 * 16 + 8) * sizeof(float);
  lds = std::max(lds, epi);
  static bool attr = false;
  set_lds_limit(&conv_fwd_pair_kernel<BM, BN>, lds, attr);
  const unsigned n = (unsigned)(pg.dgx * pg.dgy * pg.dgz + pg.wgx * pg.wgy * pg.wgz);
  conv_fwd_pair_kernel<BM, BN><<<n, 256, lds, s>>>(a1, a2, pg);
}
}  // namespace

bool launch_conv_fwd_pair(const ConvGeom& g1, const ConvPlan& p1, const uint16_t* w1, uint16_t* y1, float* ys1,
                          int* cnt1, double* st1, const ConvGeom& g2, const ConvPlan& p2, const uint16_t* w2,
                          uint16_t* y2, float* ys2, int* cnt2, double* st2, const uint16_t* x, hipStream_t s) {
  if (!conv_pair_enabled()) return false;
  if (g1.R != 3 || g1.stride != 2 || g2.R != 1 || g2.stride != 2) return false;
  if (p1.bm != p2.bm || p1.bn != p2.bn) return false;
  if (!((p1.bm == 128 && p1.bn == 64) || (p1.bm == 64 && p1.bn == 64))) return false;
  auto mk = [&](const ConvGeom& g, ConvPlan p, const uint16_t* w, uint16_t* y, float* ys, int* cn, double* st,
                ConvArgs& a, int& gx, int& gy, int& gz) {
    const int ks64 = (g.K + 63) / 64;
    p.bk = 64;
    p.kchunk = ((ks64 + p.splits - 1) / p.splits) * 64;  // same slices: the caller's workspace fits
    a = ConvArgs{};
    a.g = g;
    a.src = x;
    a.wgt = w;
    a.src_bytes = range_bytes((int64_t)g.N * g.H * g.W * g.C);
    a.wgt_bytes = range_bytes((int64_t)g.Ng * g.K);
    a.y = y;
    a.ysplit = ys;
    a.counters = cn;
    a.stats = st;
    a.kchunk = p.kchunk;
    fill_shifts(a);
    gx = (g.M + p.bm - 1) / p.bm;
    gy = (g.Ng + p.bn - 1) / p.bn;
    gz = p.splits;
  };
  ConvArgs a1, a2;
  PairGrid pg{};
  mk(g1, p1, w1, y1, ys1, cnt1, st1, a1, pg.dgx, pg.dgy, pg.dgz);
  mk(g2, p2, w2, y2, ys2, cnt2, st2, a2, pg.wgx, pg.wgy, pg.wgz);
  if (p1.bm == 128) launch_fwd_pair_t<128, 64>(a1, a2, pg, s);
  else launch_fwd_pair_t<64, 64>(a1, a2, pg, s);
  return true;
}

void launch_transpose_krsc(const uint16_t* w, uint16_t* wt, int Co, int RS, int Ci, hipStream_t s) {
  const int64_t n = (int64_t)Co * RS * Ci;
  transpose_krsc_kernel<<<stream_grid(n, 256, 4096), 256, 0, s>>>(w, wt, Co, RS, Ci);
}

}  // namespace mfl
