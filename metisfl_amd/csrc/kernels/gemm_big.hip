// K7b: large-tile bf16 GEMM for the BERT-base projections (M = B*T = 16384
// rows, N / K in {768, 2304, 3072}).
//
// The 1x1-conv GEMM path (gemm.hip -> conv.hip, 128x128 tiles, 4 waves) runs
// these shapes at 250-370 TFLOP/s: at 128x128 every k-tile stages 32 KiB per
// 2 MFLOP of work, which pins the CU at its ~64 B/clk L2 load rate.  This
// kernel follows the guide's 256^2 template (cdna_hip_programming.md §5,
// "The 256^2 ... template"): 256x256 output per workgroup, 8 waves as 2(M) x
// 4(N), 128x64 per wave (8x4 v_mfma_f32_16x16x32_bf16 accumulators), BK = 64,
// operand tiles moved global -> LDS with LDS-DMA buffer loads into a 2-stage
// ring (64 KiB per stage), ONE raw barrier per k-step with the next tile's
// DMA in flight across it, an XCD-aware bijective block -> tile remap so the
// tiles that share an A row panel run on one XCD's L2.
//
// Operand layouts (template flags) cover the three training GEMMs of a
// Linear layer with no transpose pass:
//   AK / BK : stored [row][k]  (k contiguous) -> 128-B LDS rows, ds_read_b128
//   AT / BT : stored [k][row]  (rows contiguous) -> 512-B LDS k-rows,
//             ds_read_b64_tr_b16 transposing reads (guide T10)
//   forward  Y[M][N]   = X[M][K] . W[N][K]^T       A = AK, B = BK, bf16 out,
//                        fused bias / residual / GELU epilogue
//   dgrad    dX[M][K]  = dY[M][N] . W[N][K]        A = AK, B = BT, bf16 out (+=)
//   wgrad    dW[N][K] += dY[M][N]^T . X[M][K]      A = AT, B = BT, fp32 out (+=)
// Swizzles (lds_tiles.h) are applied on the DMA source address, so every
// fragment read is bank-conflict-free.  The epilogue stages each wave's fp32
// sub-tile through LDS in 32-row chunks and writes 16-B vectors.
//
// Shapes must tile exactly (M, N multiples of 256, K of 64); gemm.hip routes
// other shapes to the conv-core path.  Reference: the Dense / attention
// projections of SURVEY §2.10 K7 (BERT-base path, §7.2 step 10).
#include "kernels/common.h"
#include "kernels/gemm.h"
#include "kernels/lds_tiles.h"

#ifndef MFL_GB_DBG
#define MFL_GB_DBG 0  // timing experiments only: bit0 skip MFMAs, bit1 skip operand DMA, bit2 skip the output stage (compile-time)
#endif

namespace mfl {

struct BigGemmArgs {
  const uint16_t* a;
  const uint16_t* b;
  int M, N, K;           // C[M][N] = sum_k A(m, k) * B(n, k)
  int lda, ldb;          // row pitch (elements) of the STORED operands
  uint32_t a_bytes, b_bytes;
  uint16_t* c16;         // bf16 output (forward / dgrad)
  float* c32;            // fp32 output (wgrad)
  float* ws;             // split-K partial slabs [splits][M][ldc] (ping-pong kernel), else fp32 atomics
  int ldc;
  const float* bias;     // [N]
  const uint16_t* resid; // [M][ldc]
  uint16_t* act_out;     // [M][ldc] gelu(y)
  int accum;
  int splits;            // split-K slices (fp32 output only; atomics into c32)
  int kt_per_split;      // k-tiles per slice
  int dbg;               // timing experiments (MFL_GB_DEBUG): bit0 skip MFMAs, bit1 skip operand DMA, bit2 skip the output stage (ping-pong kernel)
  // dgrad epilogue fusion of the GELU backward (bf16 output only):
  //   out = bf16(acc * gelu'(z)),  colsum[col] += sum over rows of out
  const uint16_t* gelu_z;
  float* colsum;
  // GELU derivative stored by the forward (FFN1 + GELU): c16 <- gelu'(y)
  // instead of y, and the backward's gelu_z then holds gelu'(z) already
  // (gelu_pre: dz = dh * gelu_z, one multiply instead of the erf / exp
  // evaluation over 50M elements in the output stage)
  int gelu_grad_out;
  int gelu_pre;
};

namespace {

constexpr int GB_BM = 256, GB_BN = 256;
constexpr int GB_EPI_LD = 68;               // fp32 staging row pitch (64 + 4)
constexpr int GB_KQ = 64;                   // K granularity the shapes must meet
#ifndef MFL_GB_PIN_ORDER
#define MFL_GB_PIN_ORDER 1
#endif
constexpr bool kGbPinOrder = MFL_GB_PIN_ORDER;
// Pipeline variants: BK = 64 with a 2-stage ring (one tile in flight across
// the compute), or BK = 32 with a 4-stage ring (three tiles in flight).
template <int BK, int NST>
struct GbCfg {
  static constexpr int TILE = GB_BM * BK * 2;  // bytes of one operand tile
  static constexpr int STAGE = 2 * TILE;       // A + B
  static constexpr int DMA = GB_BM * BK * 2 / 1024 / 8;  // DMA instructions per wave per operand
  static constexpr size_t LDS = (size_t)NST * STAGE > (size_t)8 * 32 * GB_EPI_LD * 4
                                    ? (size_t)NST * STAGE : (size_t)8 * 32 * GB_EPI_LD * 4;
};

// One operand tile (256 rows x BK k) global -> LDS.
template <bool T, int BK>
__device__ __forceinline__ void stage_operand(__amdgpu_buffer_rsrc_t rs, int ld, int row0, int k0,
                                              uint8_t* dst, int wave, int lane) {
  constexpr int NI = GbCfg<BK, 2>::DMA;
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = wave + 8 * u;  // 1-KiB instruction index within the tile
    uint32_t off;
    if constexpr (!T) {
      // [row][k]: 1024 / (2 BK) rows of 2 BK bytes per instruction
      constexpr int RPI = 512 / BK, CPR = BK / 8;
      const int row = RPI * i + lane / CPR;
      const int lc = (lane % CPR) ^ swz_b128<2 * BK>(row);
      off = (uint32_t)((row0 + row) * ld + k0 + 8 * lc) * 2u;
    } else {
      // [k][row]: 2 k-rows of 512 B per instruction
      const int kr = 2 * i + (lane >> 5);
      const int lc = (lane & 31) ^ swz_tr<512>(kr);
      off = (uint32_t)((k0 + kr) * ld + row0 + 8 * lc) * 2u;
    }
    dma16(rs, off, dst + i * 1024);
  }
}

template <bool T, int BK>
__device__ __forceinline__ bf16x8 frag(const uint8_t* tile, int kk, int r0, int lane) {
  if constexpr (T) return tr_frag<512>(tile, kk, r0, lane);
  else return b128_frag<2 * BK>(tile, kk, r0, lane);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Output stage shared by both pipelines: split-K fp32 atomics straight from
// the accumulators, or per wave 4 chunks of 32 rows x 64 cols through LDS
// (the operand ring must be drained) with the fused bias / residual / GELU /
// GELU-backward / column-sum options.  WN = columns per wave (64, or 48 for
// the 256x192 tile); the column-sum option needs WN = 64.
template <bool OUT32, int WN = 64>
__device__ __forceinline__ void big_epilogue(const BigGemmArgs& p, f32x4 (&acc)[8][4], uint8_t* smem, int m0,
                                             int n0, int wm, int wn, int wave, int lane) {
  constexpr int NJ = WN / 16, CG = WN / 8, NU = 32 * CG / 64;
  if constexpr (OUT32) {
    if (p.splits > 1) {
      // split-K: fp32 atomics straight from the accumulators (16 lanes cover
      // 64 contiguous bytes of a row per instruction)
      const int fq = lane >> 4, fr = lane & 15;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = m0 + wm * 128 + 16 * i + 4 * fq + e;
            const int col = n0 + wn * WN + 16 * j + fr;
            if (row < p.M && col < p.N) atomicAdd(p.c32 + (int64_t)row * p.ldc + col, acc[i][j][e]);
          }
      return;
    }
  }

  // ---- epilogue: per wave, 4 chunks of 32 rows x 64 cols through LDS --------
  float* W = reinterpret_cast<float*>(smem) + wave * (32 * GB_EPI_LD);
  const int fq = lane >> 4, fr = lane & 15;
  // every item a lane stores has column group lane & 7 (item = lane + 64 u):
  // per-lane column partial sums for the fused bias gradient
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    // the chunk's global reads (bf16 output: the residual, the GELU
    // pre-activation, the accumulated output) are issued BEFORE it is staged
    // through LDS, so their latency overlaps the staging instead of being
    // exposed item by item after it
    uint4 rd_res[NU], rd_z[NU], rd_acc[NU];
    if constexpr (!OUT32) {
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int item = lane + 64 * u;
        const int rl = item / CG, cg = item - rl * CG;
        const int row = m0 + wm * 128 + 32 * c + rl;
        const int col = n0 + wn * WN + cg * 8;
        rd_res[u] = rd_z[u] = rd_acc[u] = uint4{0u, 0u, 0u, 0u};
        if (row < p.M && col < p.N) {
          const int64_t off = (int64_t)row * p.ldc + col;
          if (p.resid) rd_res[u] = *reinterpret_cast<const uint4*>(p.resid + off);
          if (p.gelu_z) rd_z[u] = *reinterpret_cast<const uint4*>(p.gelu_z + off);
          if (p.accum) rd_acc[u] = *reinterpret_cast<const uint4*>(p.c16 + off);
        }
      }
    }
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          W[(16 * i2 + 4 * fq + e) * GB_EPI_LD + 16 * j + fr] = acc[2 * c + i2][j][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int item = lane + 64 * u;
      const int rl = item / CG, cg = item - rl * CG;
      const float4 lo = *reinterpret_cast<const float4*>(W + rl * GB_EPI_LD + cg * 8);
      const float4 hi = *reinterpret_cast<const float4*>(W + rl * GB_EPI_LD + cg * 8 + 4);
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      const int row = m0 + wm * 128 + 32 * c + rl;
      const int col = n0 + wn * WN + cg * 8;
      if (row >= p.M || col >= p.N) continue;  // ragged edge tiles (N % 8 == 0)
      const int64_t off = (int64_t)row * p.ldc + col;
      if constexpr (OUT32) {
        float4* dst = reinterpret_cast<float4*>(p.c32 + off);
        float4 o0 = {v[0], v[1], v[2], v[3]}, o1 = {v[4], v[5], v[6], v[7]};
        if (p.accum) {
          const float4 a0 = dst[0], a1 = dst[1];
          o0.x += a0.x; o0.y += a0.y; o0.z += a0.z; o0.w += a0.w;
          o1.x += a1.x; o1.y += a1.y; o1.z += a1.z; o1.w += a1.w;
        }
        dst[0] = o0;
        dst[1] = o1;
      } else {
        uint16_t* dst = p.c16 + off;
        if (p.accum) {
          float o[8];
          unpack8(rd_acc[u], o);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += o[k];
        }
        if (p.bias) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += p.bias[col + k];
        }
        if (p.resid) {
          float o[8];
          unpack8(rd_res[u], o);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += o[k];
        }
        if (p.gelu_z) {  // dz = dh * gelu'(z), exact erf GELU
          float zz[8];
          unpack8(rd_z[u], zz);
          if (p.gelu_pre) {  // the forward stored gelu'(z)
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] *= zz[k];
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] *= gelu_grad_f(zz[k]);
          }
        }
        const uint4 packed = pack8(v);
        if (!p.gelu_grad_out) *reinterpret_cast<uint4*>(dst) = packed;
        if (p.colsum) {  // bias gradient of what the next GEMMs consume (rounded)
          float f[8];
          unpack8(packed, f);
#pragma unroll
          for (int k = 0; k < 8; ++k) cs[k] += f[k];
        }
        if (p.act_out) {  // exact (erf) GELU of the stored pre-activation
          float f[8], h[8];
          unpack8(packed, f);
          if (p.gelu_grad_out) {  // and its derivative in place of it
            float gd[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              float c, pd;
              gelu_parts(f[k], c, pd);
              h[k] = f[k] * c;
              gd[k] = c + f[k] * pd;
            }
            *reinterpret_cast<uint4*>(dst) = pack8(gd);
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) h[k] = gelu_f(f[k]);
          }
          *reinterpret_cast<uint4*>(p.act_out + off) = pack8(h);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // reads of this chunk done before the next overwrites W
  }
  if constexpr (!OUT32 && WN == 64) {
    if (p.colsum) {
      // lanes sharing lane & 7 hold the same 8 columns: butterfly over lane >> 3
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float x = cs[k];
        x += __shfl_xor(x, 8, 64);
        x += __shfl_xor(x, 16, 64);
        x += __shfl_xor(x, 32, 64);
        cs[k] = x;
      }
      if (lane < 8 && n0 + wn * 64 + lane * 8 < p.N) {
        const int col = n0 + wn * 64 + lane * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) atomicAdd(p.colsum + col + k, cs[k]);
      }
    }
  }
}

template <bool AT, bool BT, bool OUT32, int BK, int NST>
__global__ __launch_bounds__(512) void gemm_big_kernel(BigGemmArgs p) {
  using C = GbCfg<BK, NST>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  // XCD-aware bijective remap (guide §5: 'XCD swizzle must be bijective'):
  // consecutive tile ids -- same A row panel, N fastest -- share an XCD.
  // blockIdx.y = split-K slice (wgrad: the long M reduction over few output tiles)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int tiles_n = (p.N + GB_BN - 1) / GB_BN;  // ragged last tile: reads OOB-zero / skipped stores
  const int m0 = (wgid / tiles_n) * GB_BM;
  const int n0 = (wgid - (wgid / tiles_n) * tiles_n) * GB_BN;
  const auto rsA = make_rsrc(p.a, p.a_bytes);
  const auto rsB = make_rsrc(p.b, p.b_bytes);
  const int kt0 = blockIdx.y * p.kt_per_split;
  const int nk = min(p.K / BK - kt0, p.kt_per_split);
  if (nk <= 0) return;  // block-uniform: an empty trailing slice

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt, int stage) {
    if constexpr (MFL_GB_DBG & 2) return;
    uint8_t* st = smem + stage * C::STAGE;
    stage_operand<AT, BK>(rsA, p.lda, m0, (kt0 + kt) * BK, st, wave, lane);
    stage_operand<BT, BK>(rsB, p.ldb, n0, (kt0 + kt) * BK, st + C::TILE, wave, lane);
  };
  auto compute = [&](int stage) {
    if constexpr (MFL_GB_DBG & 1) return;
    const uint8_t* As = smem + stage * C::STAGE;
    const uint8_t* Bs = As + C::TILE;
    if constexpr (kGbPinOrder && BK == 64 && !AT && !BT) {
      // Both 32-deep slices' fragments (24 reads) go out before the first
      // MFMA, so slice 1's LDS latency hides under slice 0's 32 MFMAs.
      bf16x8 b0[4], a0[8], b1[4], a1[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) b0[j] = frag<BT, BK>(Bs, 0, wn * 64 + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) a0[i] = frag<AT, BK>(As, 0, wm * 128 + 16 * i, lane);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) b1[j] = frag<BT, BK>(Bs, 32, wn * 64 + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) a1[i] = frag<AT, BK>(As, 32, wm * 128 + 16 * i, lane);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a0[i], b0[j], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a1[i], b1[j], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
      return;
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 bfr[4], af[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BT, BK>(Bs, kk, wn * 64 + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = frag<AT, BK>(As, kk, wm * 128 + 16 * i, lane);
      // transposing reads go through asm (lds_tiles.h): wait for them explicitly
      if constexpr (AT) frags_ready(af);
      if constexpr (BT) frags_ready(bfr);
      // Pin the order: all 12 fragment reads in flight together, then the 32
      // MFMAs.  Left alone, hipcc interleaves read -> lgkmcnt(0) -> 4 MFMAs
      // eight times per slice (register-pressure heuristic), exposing eight
      // LDS latencies per 512 MFMA cycles.
      if constexpr (kGbPinOrder) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      if constexpr (kGbPinOrder) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // NST-stage ring, NST-1 tiles in flight; per tile each thread issues
  // L = 2 * DMA LDS-DMA instructions (counted by vmcnt, hand-waited).
  constexpr int D = NST - 1, L = 2 * C::DMA;
#pragma unroll
  for (int u = 0; u < D; ++u)
    if (u < nk) issue(u, u);
  int stage = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const int younger = min(D - 1, nk - 1 - kt);  // tiles after kt still allowed in flight
    if constexpr (D >= 3) {
      if (younger >= 2) wait_vm<2 * L>();
      else if (younger == 1) wait_vm<L>();
      else wait_vm<0>();
    } else if constexpr (D == 2) {
      if (younger >= 1) wait_vm<L>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own reads of the recycled stage retired
    lds_barrier();  // everyone's tile kt landed; everyone done reading stage (kt-1)%NST
    if (kt + D < nk) issue(kt + D, stage == 0 ? NST - 1 : stage - 1);
    compute(stage);
    stage = stage == NST - 1 ? 0 : stage + 1;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_barrier();  // the ring is free for the epilogue staging

  big_epilogue<OUT32>(p, acc, smem, m0, n0, wm, wn, wave, lane);
}

// ---- half-height tiles, two workgroups per CU (MFL_GB_PIPE=3) -------------------
// 128 x 256 output per workgroup, 4 waves (1 x 4, the same 128 x 64 per wave
// and accumulator layout as the 256^2 kernels), BK = 32 through a 3-stage
// ring: 72 KiB of LDS and <= 128 VGPRs... so TWO workgroups share a CU.  The
// one-workgroup-per-CU kernels run their output stage (100-200 MB per call)
// in lock step on every CU, with no MFMA work beside it (profiles/ANALYSIS.md,
// BERT section: 8-31 us per call); here the two co-resident workgroups drift
// apart, so one's epilogue overlaps the other's k-loop.  Costs 1.5x the
// L2 -> LDS operand bytes of the 256^2 tile (A rows shared by half as many
// columns).  Forward / dgrad (bf16 output) only.  Measured (negative, kept
// opt-in): 15-30 % SLOWER than the ping-pong kernel on every BERT shape
// (qkv fwd 96.0 vs 81.2 us, ffn2 fwd 93.3 vs 68.8;
// profiles/r3/bert/gemm_sweep_h2_vs_pp.log) -- the extra operand traffic and
// the BK = 32 barrier per k-step cost more than the overlap returns.
template <bool T, int BK, int ROWS, int NW>
__device__ __forceinline__ void stage_rows(__amdgpu_buffer_rsrc_t rs, int ld, int row0, int k0, uint8_t* dst,
                                           int wave, int lane) {
  constexpr int NI = ROWS * BK * 2 / 1024 / NW;
  static_assert(!T || ROWS == 256, "[k][row] tiles: 512-B k-rows");
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = wave + NW * u;  // 1-KiB instruction index within the tile
    uint32_t off;
    if constexpr (!T) {
      constexpr int RPI = 512 / BK, CPR = BK / 8;
      const int row = RPI * i + lane / CPR;
      const int lc = (lane % CPR) ^ swz_b128<2 * BK>(row);
      off = (uint32_t)((row0 + row) * ld + k0 + 8 * lc) * 2u;
    } else {
      const int kr = 2 * i + (lane >> 5);
      const int lc = (lane & 31) ^ swz_tr<512>(kr);
      off = (uint32_t)((k0 + kr) * ld + row0 + 8 * lc) * 2u;
    }
    dma16(rs, off, dst + i * 1024);
  }
}

template <bool BT>
__global__ __launch_bounds__(256, 2) void gemm_h2_kernel(BigGemmArgs p) {
  constexpr int BK = 32, NST = 3, BMH = 128;
  constexpr int A_B = BMH * BK * 2, STG = A_B + GB_BN * BK * 2;  // 8 + 16 KiB per stage
  constexpr int L = (A_B + GB_BN * BK * 2) / 1024 / 4;           // DMA instructions per wave per k-tile
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wn = wave;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int tiles_n = (p.N + GB_BN - 1) / GB_BN;
  const int m0 = (wgid / tiles_n) * BMH;
  const int n0 = (wgid - (wgid / tiles_n) * tiles_n) * GB_BN;
  const auto rsA = make_rsrc(p.a, p.a_bytes);
  const auto rsB = make_rsrc(p.b, p.b_bytes);
  const int nk = p.K / BK;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto issue = [&](int kt, int stage) {
    uint8_t* st = smem + stage * STG;
    stage_rows<false, BK, BMH, 4>(rsA, p.lda, m0, kt * BK, st, wave, lane);
    stage_rows<BT, BK, GB_BN, 4>(rsB, p.ldb, n0, kt * BK, st + A_B, wave, lane);
  };
  auto compute = [&](int stage) {
    const uint8_t* As = smem + stage * STG;
    const uint8_t* Bs = As + A_B;
    bf16x8 bfr[4], af[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = frag<BT, BK>(Bs, 0, wn * 64 + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = frag<false, BK>(As, 0, 16 * i, lane);
    if constexpr (BT) frags_ready(bfr);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int D = NST - 1;
#pragma unroll
  for (int u = 0; u < D; ++u)
    if (u < nk) issue(u, u);
  int stage = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (nk - 1 - kt >= 1) wait_vm<L>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_barrier();  // everyone's tile kt landed; everyone done reading stage (kt-1)%NST
    if (kt + D < nk) issue(kt + D, stage == 0 ? NST - 1 : stage - 1);
    compute(stage);
    stage = stage == NST - 1 ? 0 : stage + 1;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_barrier();  // the ring is free for the epilogue staging
  big_epilogue<false, 64>(p, acc, smem, m0, n0, 0, wn, wave, lane);
}

template <bool BT>
void launch_h2_t(const BigGemmArgs& p, hipStream_t s) {
  constexpr size_t kLds = 3 * (128 * 32 * 2 + 256 * 32 * 2);  // 72 KiB (>= the 4-wave epilogue staging)
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_h2_kernel<BT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds);
    attr = true;
  }
  const dim3 grid((unsigned)(((p.M + 127) / 128) * ((p.N + GB_BN - 1) / GB_BN)), 1);
  gemm_h2_kernel<BT><<<grid, 256, kLds, s>>>(p);
}

// ---- ping-pong pipeline (MFL_GB_PIPE=2) ---------------------------------------
// The same 256x256 tile and wave layout, scheduled after the guide's 256^2
// 8-phase template (cdna_hip_programming.md §5): each k-tile is split into 4
// half-tiles of 16 KiB -- A rows {0-63, 128-191} (A0), B cols {64w + 0-31}
// (B0), B cols {64w + 32-63} (B1), A rows {64-127, 192-255} (A1) -- and
// computed in 4 phases, one 64x32 quadrant of every wave's 128x64 output per
// phase: (mi, ni) = (0,0) (0,1) (1,1) (1,0), fragment reads 12 / 4 / 8 / 0.
// A phase is a LOAD section (this phase's fragment reads, ONE half-tile of
// LDS-DMA, vmcnt) and an MFMA section (16 MFMAs), each closed by a barrier.
// Wave rows 0 and 1 share every SIMD (waves w, w + 4) and run one barrier
// apart, so one wave's MFMAs always overlap the other's loads.
//
// Hazards (phase index f, one barrier per section, rows staggered by one):
//  * RAW: the half-tile issued in phase f is retired by vmcnt(8) (4 younger
//    half-tiles in flight) in phase f + 4 and read from phase f + 5 on --
//    every wave's wait precedes a barrier every reader passes before reading.
//  * WAR: a half-tile read in phase f is restaged no earlier than f + 2
//    (both rows' reads have retired by then).
//  Issue order (steady state): phase 4t+0 -> B1(t+1), 4t+1 -> A1(t+1),
//  4t+2 -> A0(t+2), 4t+3 -> B0(t+2); read: A0, B0 at 4t, B1 at 4t+1, A1 at
//  4t+2.  Half-tiles past the slice's last k-tile load out-of-range zeros so
//  the vmcnt count is the same in every phase.
constexpr int PP_HALF = 128 * 64 * 2;  // one half-tile, bytes

// Tile width: 256 (BW = 64 columns per wave) or 192 (BW = 48: the B1
// half-tile then holds 4 x 16 columns, 8 KiB, one DMA instruction per wave --
// N = 768 / 2304 tile into 256 / 768 workgroups instead of 192 / 576).
// Half-tile rows: HR(sub) local rows; local row l -> operand-tile row.
template <bool ISB, int BW>
struct PpHalf {
  static constexpr int W1 = ISB ? BW - 32 : 64;             // rows per wave column in half `sub`
  static __device__ __forceinline__ int rows(int sub) { return ISB ? 4 * (sub ? W1 : 32) : 128; }
  static __device__ __forceinline__ int map(int l, int sub) {
    if constexpr (!ISB) return (l >> 6) * 128 + sub * 64 + (l & 63);
    else return sub ? (l / W1) * BW + 32 + (l % W1) : (l >> 5) * BW + (l & 31);
  }
};

// NR local rows (128, or 64 for a 192-wide B1) x 64 k, 16 B per lane per DMA
// instruction, NR * 128 / 1024 instructions spread over the 8 waves.
template <bool T, bool ISB, int BW, int NR>
__device__ __forceinline__ void pp_stage(__amdgpu_buffer_rsrc_t rs, int ld, int row0, int k0, int sub,
                                         uint8_t* dst, int wave, int lane, bool valid) {
  constexpr int NI = NR * 128 / 1024 / 8;  // instructions per wave
#pragma unroll
  for (int u = 0; u < NI; ++u) {
    const int i = wave + 8 * u;  // 1-KiB instruction index within the half-tile
    uint32_t off;
    if constexpr (!T) {
      // [row][k]: 8 rows of 128 B per instruction
      const int l = 8 * i + (lane >> 3);
      const int lc = (lane & 7) ^ swz_b128<128>(l);
      off = (uint32_t)((row0 + PpHalf<ISB, BW>::map(l, sub)) * ld + k0 + 8 * lc) * 2u;
    } else if constexpr (NR == 128) {
      // [k][row]: 4 k-rows of 256 B per instruction
      const int kr = 4 * i + (lane >> 4);
      const int lc = (lane & 15) ^ swz_tr<256>(kr);
      off = (uint32_t)((k0 + kr) * ld + row0 + PpHalf<ISB, BW>::map(8 * lc, sub)) * 2u;
    } else {
      // [k][row]: 8 k-rows of 128 B per instruction
      const int kr = 8 * i + (lane >> 3);
      const int lc = (lane & 7) ^ swz_tr<128>(kr);
      off = (uint32_t)((k0 + kr) * ld + row0 + PpHalf<ISB, BW>::map(8 * lc, sub)) * 2u;
    }
    dma16(rs, valid ? off : kOOB, dst + i * 1024);
  }
}

template <bool T, int NR = 128>
__device__ __forceinline__ bf16x8 pp_frag(const uint8_t* half, int kk, int r0, int lane) {
  if constexpr (T) return tr_frag<2 * NR>(half, kk, r0, lane);
  else return b128_frag<128>(half, kk, r0, lane);
}

// XCD-aware bijective workgroup -> tile index (tiles sharing an A row panel
// run on one XCD's L2)
__device__ __forceinline__ int pp_wgid() {
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// One 256 x BN output tile (wgid: its index in p's row-major tile grid) of
// split-K slice `split`.
template <bool AT, bool BT, bool OUT32, int BN>
__device__ __forceinline__ void gemm_pp_body(const BigGemmArgs& p, int wgid, int split, uint8_t* smem) {
  constexpr int BW = BN / 4;            // columns per wave
  constexpr int NJ1 = (BW - 32) / 16;   // 16-column tiles of a wave in the B1 half
  constexpr int NR1 = 4 * (BW - 32);    // B1 half-tile rows
  constexpr int VM = 6 + NR1 / 64;      // DMA instructions per wave per k-tile
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int m0 = (wgid / tiles_n) * GB_BM;
  const int n0 = (wgid - (wgid / tiles_n) * tiles_n) * BN;
  const auto rsA = make_rsrc(p.a, p.a_bytes);
  const auto rsB = make_rsrc(p.b, p.b_bytes);
  const int kt0 = split * p.kt_per_split;
  const int nk = min(p.K / 64 - kt0, p.kt_per_split);
  if (nk <= 0) return;  // block-uniform

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bfr[2][2][2];

  // half-tile h (0 A0, 1 B0, 2 B1, 3 A1) of k-tile kt into ring slot kt & 1
  auto stage = [&](int h, int kt) {
    if constexpr (MFL_GB_DBG & 2) return;
    uint8_t* dst = smem + ((kt & 1) * 4 + h) * PP_HALF;
    const bool v = kt < nk;
    const int k0 = (kt0 + (v ? kt : 0)) * 64;
    if (h == 0 || h == 3) pp_stage<AT, false, BW, 128>(rsA, p.lda, m0, k0, h == 3, dst, wave, lane, v);
    else if (h == 1) pp_stage<BT, true, BW, 128>(rsB, p.ldb, n0, k0, 0, dst, wave, lane, v);
    else pp_stage<BT, true, BW, NR1>(rsB, p.ldb, n0, k0, 1, dst, wave, lane, v);
  };
  auto read_a = [&](int kt, int mi) {
    const uint8_t* h = smem + ((kt & 1) * 4 + (mi ? 3 : 0)) * PP_HALF;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) af[i][ks] = pp_frag<AT>(h, 32 * ks, wm * 64 + 16 * i, lane);
  };
  auto read_b = [&](int kt, int ni) {
    const uint8_t* h = smem + ((kt & 1) * 4 + 1 + ni) * PP_HALF;
    if (ni == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) bfr[0][j][ks] = pp_frag<BT>(h, 32 * ks, wn * 32 + 16 * j, lane);
    } else {
#pragma unroll
      for (int j = 0; j < NJ1; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          bfr[1][j][ks] = pp_frag<BT, NR1>(h, 32 * ks, wn * (BW - 32) + 16 * j, lane);
    }
  };
  auto mfma_quadrant = [&](int mi, int ni) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < (ni ? NJ1 : 2); ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc[4 * mi + i][2 * ni + j] = mfma16(af[i][ks], bfr[ni][j][ks], acc[4 * mi + i][2 * ni + j]);
  };
  // the transposing reads are inline asm: retire them and pin their registers
  auto frags_in = [&](bool a_read, int ni) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (a_read) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) asm volatile("" : "+v"(af[i][ks]));
    }
    if (ni >= 0) {
#pragma unroll
      for (int j = 0; j < (ni ? NJ1 : 2); ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) asm volatile("" : "+v"(bfr[ni][j][ks]));
    }
  };
  auto mfma_section = [&](int mi, int ni) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if constexpr (!(MFL_GB_DBG & 1)) mfma_quadrant(mi, ni);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    lds_barrier();
  };

  // prologue: the half-tiles of phases -6 .. -1, then A0(0) / B0(0) retired
  stage(0, 0);
  stage(1, 0);
  stage(2, 0);
  stage(3, 0);
  stage(0, 1);
  stage(1, 1);
  wait_vm<VM>();
  lds_barrier();
  if (wm == 1) lds_barrier();  // row 1 runs one barrier behind row 0

  for (int kt = 0; kt < nk; ++kt) {
    // phase 0: quadrant (0,0)
    read_b(kt, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(kt, 0);
    stage(2, kt + 1);
    wait_vm<VM>();
    lds_barrier();
    frags_in(true, 0);
    mfma_section(0, 0);
    // phase 1: quadrant (0,1)
    read_b(kt, 1);
    stage(3, kt + 1);
    wait_vm<VM>();
    lds_barrier();
    frags_in(false, 1);
    mfma_section(0, 1);
    // phase 2: quadrant (1,1)
    read_a(kt, 1);
    stage(0, kt + 2);
    wait_vm<VM>();
    lds_barrier();
    frags_in(true, -1);
    mfma_section(1, 1);
    // phase 3: quadrant (1,0), fragments already in registers
    stage(1, kt + 2);
    wait_vm<VM>();
    lds_barrier();
    mfma_section(1, 0);
  }
  if (wm == 0) lds_barrier();  // rebalance the barrier count
  wait_vm<0>();                // trailing out-of-range half-tiles land before the LDS is reused
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_barrier();
  if constexpr (MFL_GB_DBG & 4) {  // timing experiment: no output stage (keep the accumulators live)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  if (OUT32 && p.splits > 1 && p.ws) {
    // split-K through plain stores into this slice's slab (summed by
    // splitk_reduce_kernel): memory-side float atomics run at ~1.3 TB/s of
    // added bytes, streaming stores at ~6 (MI355X_MICROARCH 'Global float atomics')
    BigGemmArgs q = p;
    q.c32 = p.ws + (int64_t)split * p.M * p.ldc;
    q.accum = 0;
    q.splits = 1;
    big_epilogue<OUT32, BW>(q, acc, smem, m0, n0, wm, wn, wave, lane);
    return;
  }
  big_epilogue<OUT32, BW>(p, acc, smem, m0, n0, wm, wn, wave, lane);
}

template <bool AT, bool BT, bool OUT32, int BN>
__global__ __launch_bounds__(512) void gemm_pp_kernel(BigGemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  gemm_pp_body<AT, BT, OUT32, BN>(p, pp_wgid(), blockIdx.y, smem);
}

// Two independent problems of the same layout in ONE launch: workgroups
// [0, tiles0) take p0's tiles, the rest p1's; both split their reduction into
// gridDim.y slices.  For weight gradients with few output tiles (BERT's
// attention-output 768 x 768 next to its QKV 2304 x 768): alone, the small one
// needs ~28 short slices to fill the chip; together both run a handful of
// long ones, and the split-K slabs shrink with the slice count.
template <bool AT, bool BT, bool OUT32, int BN>
__global__ __launch_bounds__(512) void gemm_pp_group_kernel(BigGemmArgs p0, BigGemmArgs p1, int tiles0) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int w = pp_wgid();
  if (w < tiles0) gemm_pp_body<AT, BT, OUT32, BN>(p0, w, blockIdx.y, smem);
  else gemm_pp_body<AT, BT, OUT32, BN>(p1, w - tiles0, blockIdx.y, smem);
}

// The grouped weight gradients' two slab sets in one launch: index i < n0
// reduces into out0, the rest into out1 (the same per-element slice order as
// two splitk_reduce_kernel launches, so bitwise the same sums)
__global__ __launch_bounds__(256) void splitk_reduce2_kernel(const float4* __restrict__ ws0, int64_t n0,
                                                             float4* __restrict__ out0, const float4* __restrict__ ws1,
                                                             int64_t n1, float4* __restrict__ out1, int splits) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n0 + n1; j += stride) {
    const bool first = j < n0;
    const int64_t i = first ? j : j - n0, n = first ? n0 : n1;
    const float4* ws = first ? ws0 : ws1;
    float4 a = float4{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < splits; ++k) {
      const float4 v = ws[(int64_t)k * n + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    (first ? out0 : out1)[i] = a;
  }
}

// out (+)= sum over the split-K slabs, 16 B per lane
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float4* __restrict__ ws, int splits,
                                                            int64_t n4, float4* __restrict__ out, int accum) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = accum ? out[i] : float4{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < splits; ++k) {
      const float4 v = ws[(int64_t)k * n4 + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    out[i] = a;
  }
}

// bf16 out (+)= sum over the split-K slabs (8 outputs per lane): the output
// stage of a split long-reduction dgrad (the MLM decoder's 30,528-deep one)
// add: the bf16 term the slices' sum is added to (out itself when
// accumulating, a residual gradient, or nothing)
__global__ __launch_bounds__(256) void splitk_reduce_bf16_kernel(const float4* __restrict__ ws, int splits,
                                                                 int64_t n8, uint4* out, const uint4* add) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (add) unpack8(add[i], v);
    for (int k = 0; k < splits; ++k) {
      const float4 a = ws[(int64_t)k * 2 * n8 + 2 * i], b = ws[(int64_t)k * 2 * n8 + 2 * i + 1];
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
    out[i] = pack8(v);
  }
}

template <bool AT, bool BT, bool OUT32, int BN>
void launch_pp_t(const BigGemmArgs& p, hipStream_t s) {
  constexpr size_t kLds = 8 * (size_t)PP_HALF;  // 2 k-tiles x 4 half-tile slots = 128 KiB
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_pp_kernel<AT, BT, OUT32, BN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds);
    attr = true;
  }
  const dim3 grid((unsigned)(((p.M + GB_BM - 1) / GB_BM) * ((p.N + BN - 1) / BN)), (unsigned)p.splits);
  gemm_pp_kernel<AT, BT, OUT32, BN><<<grid, 512, kLds, s>>>(p);
}

template <bool AT, bool BT, bool OUT32, int BN>
void launch_pp_group_t(const BigGemmArgs& p0, const BigGemmArgs& p1, hipStream_t s) {
  constexpr size_t kLds = 8 * (size_t)PP_HALF;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_pp_group_kernel<AT, BT, OUT32, BN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds);
    attr = true;
  }
  const int t0 = ((p0.M + GB_BM - 1) / GB_BM) * ((p0.N + BN - 1) / BN);
  const int t1 = ((p1.M + GB_BM - 1) / GB_BM) * ((p1.N + BN - 1) / BN);
  const dim3 grid((unsigned)(t0 + t1), (unsigned)p0.splits);
  gemm_pp_group_kernel<AT, BT, OUT32, BN><<<grid, 512, kLds, s>>>(p0, p1, t0);
}

// Tile width for the ping-pong kernel: 192 when it needs fewer workgroup
// rounds x tile width (N = 768: 192 -> 256 tiles in one round; N = 2304: 2.25
// -> 3 rounds of narrower tiles), 256 otherwise (and for the fused column sum).
// Co-located learners (set_gemm_width 256, models/colocated.py) fill the CUs
// with each other's launches, so rounds do not matter and the wider tile's
// operand reuse wins: 8 BERT learners 1.336 -> 1.383M tokens/s.
int g_width_rt = 0;  // set_gemm_width (defined after the anonymous namespace)
int pp_width(const BigGemmArgs& p) {
  if (p.colsum || p.N % 192 != 0) return 256;
  if (const char* e = getenv("MFL_GB_WIDTH")) return atoi(e) == 192 ? 192 : 256;
  if (g_width_rt) return g_width_rt == 192 ? 192 : 256;
  const int64_t mt = (p.M + GB_BM - 1) / GB_BM;
  auto cost = [&](int bn) {
    const int64_t tiles = mt * ((p.N + bn - 1) / bn) * p.splits;
    return ((tiles + 255) / 256) * bn;
  };
  return cost(192) < cost(256) ? 192 : 256;
}

template <bool AT, bool BT, bool OUT32, int BK, int NST>
void launch_big_t(const BigGemmArgs& p, hipStream_t s) {
  using C = GbCfg<BK, NST>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_big_kernel<AT, BT, OUT32, BK, NST>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::LDS);
    attr = true;
  }
  const dim3 grid((unsigned)(((p.M + GB_BM - 1) / GB_BM) * ((p.N + GB_BN - 1) / GB_BN)), (unsigned)p.splits);
  gemm_big_kernel<AT, BT, OUT32, BK, NST><<<grid, 512, C::LDS, s>>>(p);
}

// pipeline variant (env MFL_GB_PIPE): 2 = the ping-pong half-tile schedule
// (default), 0 = BK 64 / 2-stage ring, one barrier per k-step, 1 = BK 32 /
// 4 stages.  Measured on the BERT shapes (scripts/gemm_sweep.sh,
// profiles/bert/gemm_sweep_pp.log): 2 is 3-12 % faster than 0 on every
// fwd / dgrad / wgrad shape (ffn2 fwd 988 -> 1037 TFLOP/s on 192 of 256 CUs);
// 1 ties 0 on forward and loses 8-25 % on dgrad / wgrad.
int gb_pipe() {
  static const int v = [] {
    const char* e = getenv("MFL_GB_PIPE");
    return e && *e ? atoi(e) : 2;
  }();
  return v;
}

// Slices actually holding k-tiles when ``nk`` k-tiles are dealt ``per`` to a
// slice: ceil(nk / ceil(nk / sp)) can be < sp (e.g. 500 tiles over 31 slices of
// 17: slice 30 would start at tile 510).  Split-K launches use this count, so
// every launched slice writes its slab.
static int used_splits(int nk, int per) { return per > 0 ? std::max(1, (nk + per - 1) / per) : 1; }

template <bool AT, bool BT, bool OUT32>
void launch_big(BigGemmArgs p, int kdim, hipStream_t s) {
  static const int dbg = [] {
    const char* v = getenv("MFL_GB_DEBUG");
    return v && *v ? atoi(v) : 0;
  }();
  p.dbg = dbg;
  const int bk = gb_pipe() == 1 ? 32 : 64;  // (the half-height kernel re-derives its own k-tiles)
  // p.kt_per_split arrives in units of GB_KQ (64) k-elements
  p.kt_per_split *= GB_KQ / bk;
  (void)kdim;
  if constexpr (!OUT32 && !AT) {
    if (gb_pipe() == 3 && p.M % 128 == 0 && p.N % GB_BN == 0 && p.K % 32 == 0) {
      p.kt_per_split = p.K / 32;
      launch_h2_t<BT>(p, s);
      return;
    }
  }
  if (gb_pipe() == 2 || gb_pipe() == 3) {
    if (pp_width(p) == 192) launch_pp_t<AT, BT, OUT32, 192>(p, s);
    else launch_pp_t<AT, BT, OUT32, 256>(p, s);
  }
  else if (bk == 32) launch_big_t<AT, BT, OUT32, 32, 4>(p, s);
  else launch_big_t<AT, BT, OUT32, 64, 2>(p, s);
}

}  // namespace

void set_gemm_width(int w) { g_width_rt = w; }

// Exact 256-multiples, or large ragged dimensions (>= 2048: the MLM decoder's
// 30,528-wide vocabulary) whose partial edge tile is a small fraction of the work.
bool gemm_big_ok(int M, int N, int K) {
  auto dim_ok = [](int d) { return d % GB_BM == 0 || (d >= 2048 && d % 8 == 0); };
  return M > 0 && N > 0 && K > 0 && dim_ok(M) && dim_ok(N) && K % GB_KQ == 0 &&
         (int64_t)M * K * 2 < (1LL << 32) && (int64_t)N * K * 2 < (1LL << 32) &&
         (int64_t)M * N * 2 < (1LL << 32);
}

void launch_gemm_big_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias,
                         const uint16_t* resid, uint16_t* act_out, int M, int N, int K, hipStream_t s,
                         int act_grad) {
  BigGemmArgs p{};
  p.a = x; p.b = w; p.M = M; p.N = N; p.K = K; p.lda = K; p.ldb = K;
  p.a_bytes = (uint32_t)((int64_t)M * K * 2); p.b_bytes = (uint32_t)((int64_t)N * K * 2);
  p.c16 = y; p.ldc = N; p.bias = bias; p.resid = resid; p.act_out = act_out;
  p.gelu_grad_out = act_out && act_grad;
  p.splits = 1; p.kt_per_split = K / GB_KQ;
  launch_big<false, false, false>(p, K, s);
}

// Split-K slices for a dgrad dX[M][K] = dY[M][N] W[N][K] whose output tiles
// cannot fill the chip while its reduction is long: the MLM decoder's
// 2,560 x 768 output (40 tiles) over the 30,528-word vocabulary ran at one
// workgroup per 6 CUs (289 us).  Same rule as the weight gradients:
// floor(256 / tiles) slices, at least 16 k-tiles each; 1 = no split.
int gemm_big_dgrad_splits(int M, int N, int K) {
  const int tiles = ((M + GB_BM - 1) / GB_BM) * ((K + GB_BN - 1) / GB_BN);
  if (tiles >= 128 || gb_pipe() != 2) return 1;
  return std::max(1, std::min(256 / std::max(1, tiles), (N / GB_KQ) / 16));
}

int64_t gemm_big_dgrad_workspace(int M, int N, int K) {
  const int sp = gemm_big_dgrad_splits(M, N, K);
  return sp > 1 ? (int64_t)sp * M * K : 0;
}

void launch_gemm_big_dgrad(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int M, int N, int K,
                           bool accumulate, hipStream_t s, float* ws, const uint16_t* resid) {
  // dX[M][K] = dY[M][N] . W[N][K]: output columns = K, reduction = N
  BigGemmArgs p{};
  p.a = dy; p.b = w; p.M = M; p.N = K; p.K = N; p.lda = N; p.ldb = K;
  p.a_bytes = (uint32_t)((int64_t)M * N * 2); p.b_bytes = (uint32_t)((int64_t)N * K * 2);
  p.ldc = K;
  const int sp = ws ? gemm_big_dgrad_splits(M, N, K) : 1;
  if (sp > 1 && K % 8 == 0) {
    // fp32 partials per slice into the slab workspace, one reduce to bf16
    p.c32 = ws; p.ws = ws; p.accum = 0;
    p.kt_per_split = (N / GB_KQ + sp - 1) / sp;
    // slices that own no k-tile would leave their slab unwritten (and the
    // reduce below would add stale workspace): launch only the slices used
    p.splits = used_splits(N / GB_KQ, p.kt_per_split);
    launch_big<false, true, true>(p, N, s);
    const int64_t n8 = (int64_t)M * K / 8;
    splitk_reduce_bf16_kernel<<<stream_grid(n8, 256, 2048), 256, 0, s>>>(
        reinterpret_cast<const float4*>(ws), p.splits, n8, reinterpret_cast<uint4*>(dx),
        accumulate ? reinterpret_cast<const uint4*>(dx) : reinterpret_cast<const uint4*>(resid));
    return;
  }
  // resid: added in the output stage (big_epilogue), the same single bf16
  // term an accumulate into a copy of it would add
  p.c16 = dx; p.accum = accumulate; p.resid = accumulate ? nullptr : resid;
  p.splits = 1; p.kt_per_split = N / GB_KQ;
  launch_big<false, true, false>(p, N, s);
}

void launch_gemm_big_dgrad_gelu(const uint16_t* dy, const uint16_t* w, uint16_t* dz, const uint16_t* z,
                                float* dbias, int M, int N, int K, hipStream_t s, int pre) {
  BigGemmArgs p{};
  p.a = dy; p.b = w; p.M = M; p.N = K; p.K = N; p.lda = N; p.ldb = K;
  p.a_bytes = (uint32_t)((int64_t)M * N * 2); p.b_bytes = (uint32_t)((int64_t)N * K * 2);
  p.c16 = dz; p.ldc = K; p.gelu_z = z; p.colsum = dbias; p.gelu_pre = pre;
  p.splits = 1; p.kt_per_split = N / GB_KQ;
  launch_big<false, true, false>(p, N, s);
}

namespace {
int wgrad_splits_env(int M, int N, int K) {
  if (const char* v = getenv("MFL_GB_SPLITS")) return std::max(1, atoi(v));
  return gemm_big_wgrad_splits(M, N, K);
}
}  // namespace

// fp32 elements of split-K slab workspace the wgrad wants (0: no split, or
// the atomics path: MFL_GB_SLABS=0 / a pipeline other than the ping-pong one)
int64_t gemm_big_wgrad_workspace(int M, int N, int K) {
  static const bool slabs = [] {
    const char* e = getenv("MFL_GB_SLABS");
    return !(e && *e == '0');
  }();
  const int sp = wgrad_splits_env(M, N, K);
  return (slabs && (gb_pipe() == 2 || gb_pipe() == 3) && sp > 1) ? (int64_t)sp * N * K : 0;
}

void launch_gemm_big_wgrad(const uint16_t* x, const uint16_t* dy, float* dw, int M, int N, int K,
                           bool accumulate, hipStream_t s, float* ws) {
  // dW[N][K] (+)= dY^T X: output rows = N, columns = K, reduction = M
  BigGemmArgs p{};
  p.a = dy; p.b = x; p.M = N; p.N = K; p.K = M; p.lda = N; p.ldb = K;
  p.a_bytes = (uint32_t)((int64_t)M * N * 2); p.b_bytes = (uint32_t)((int64_t)M * K * 2);
  p.c32 = dw; p.ldc = K; p.accum = accumulate;
  p.splits = wgrad_splits_env(M, N, K);
  p.kt_per_split = (M / GB_KQ + p.splits - 1) / p.splits;
  p.splits = used_splits(M / GB_KQ, p.kt_per_split);  // no empty slice (slab mode sums every slice)
  if (ws && p.splits > 1 && gemm_big_wgrad_workspace(M, N, K) > 0) {
    p.ws = ws;
    launch_big<true, true, true>(p, M, s);
    const int64_t n4 = (int64_t)N * K / 4;
    splitk_reduce_kernel<<<stream_grid(n4, 256, 2048), 256, 0, s>>>(
        reinterpret_cast<const float4*>(ws), p.splits, n4, reinterpret_cast<float4*>(dw), accumulate ? 1 : 0);
    return;
  }
  launch_big<true, true, true>(p, M, s);
}

// Two weight gradients with the same reduction length M in one launch
// (gemm_pp_group_kernel): dW0[N0][K0] = dY0^T X0, dW1[N1][K1] = dY1^T X1, both
// dW zero on entry.  ws: split-K slabs of splits * (N0 K0 + N1 K1) floats
// (gemm_big_wgrad2_workspace).  Falls back to two launches when the pair does
// not fit the grouped kernel (shapes off the 256 grid, other pipelines).
// run-time slice count of the grouped weight gradients (co-located BERT
// learners: their launches fill the CUs, fewer slices move fewer slab bytes;
// models/colocated.py)
static int g_wgrad2_splits_rt = 0;
void set_gemm_wgrad2_splits(int splits) { g_wgrad2_splits_rt = splits; }

int gemm_big_wgrad2_splits(int M, int N0, int K0, int N1, int K1) {
  const int tiles = (N0 / GB_BM) * (K0 / GB_BN) + (N1 / GB_BM) * (K1 / GB_BN);
  // MFL_GB_WGRAD2_SPLITS: A/B override of the grouped launch's slice count
  static const int env = [] {
    const char* v = getenv("MFL_GB_WGRAD2_SPLITS");
    return v && *v ? atoi(v) : 0;
  }();
  const int forced = env > 0 ? env : g_wgrad2_splits_rt;
  if (forced > 0) return std::max(1, std::min(forced, (M / GB_KQ) / 4));
  return std::max(1, std::min(256 / std::max(1, tiles), (M / GB_KQ) / 16));
}

bool gemm_big_wgrad2_ok(int M, int N0, int K0, int N1, int K1) {
  return (gb_pipe() == 2 || gb_pipe() == 3) && M % GB_KQ == 0 && N0 % GB_BM == 0 && K0 % GB_BN == 0 &&
         N1 % GB_BM == 0 && K1 % GB_BN == 0 && gemm_big_ok(N0, K0, M) && gemm_big_ok(N1, K1, M);
}

int64_t gemm_big_wgrad2_workspace(int M, int N0, int K0, int N1, int K1) {
  if (!gemm_big_wgrad2_ok(M, N0, K0, N1, K1)) return 0;
  const int sp = gemm_big_wgrad2_splits(M, N0, K0, N1, K1);
  return sp > 1 ? (int64_t)sp * ((int64_t)N0 * K0 + (int64_t)N1 * K1) : 0;
}

void launch_gemm_big_wgrad2(const uint16_t* x0, const uint16_t* dy0, float* dw0, int N0, int K0, const uint16_t* x1,
                            const uint16_t* dy1, float* dw1, int N1, int K1, int M, hipStream_t s, float* ws) {
  auto args = [&](const uint16_t* x, const uint16_t* dy, float* dw, int N, int K, int sp) {
    BigGemmArgs p{};
    p.a = dy; p.b = x; p.M = N; p.N = K; p.K = M; p.lda = N; p.ldb = K;
    p.a_bytes = (uint32_t)((int64_t)M * N * 2); p.b_bytes = (uint32_t)((int64_t)M * K * 2);
    p.c32 = dw; p.ldc = K; p.accum = 0;
    p.splits = sp;
    p.kt_per_split = (M / GB_KQ + sp - 1) / sp;
    return p;
  };
  const int sp0 = gemm_big_wgrad2_splits(M, N0, K0, N1, K1);
  const int sp = used_splits(M / GB_KQ, (M / GB_KQ + sp0 - 1) / sp0);
  BigGemmArgs p0 = args(x0, dy0, dw0, N0, K0, sp), p1 = args(x1, dy1, dw1, N1, K1, sp);
  if (sp > 1) {
    p0.ws = ws;
    p1.ws = ws + (int64_t)sp * N0 * K0;
  }
  launch_pp_group_t<true, true, true, 256>(p0, p1, s);
  if (sp > 1) {
    const int64_t n0 = (int64_t)N0 * K0 / 4, n1 = (int64_t)N1 * K1 / 4;
    splitk_reduce2_kernel<<<stream_grid(n0 + n1, 256, 2048), 256, 0, s>>>(
        reinterpret_cast<const float4*>(p0.ws), n0, reinterpret_cast<float4*>(dw0),
        reinterpret_cast<const float4*>(p1.ws), n1, reinterpret_cast<float4*>(dw1), sp);
  }
}

// Few output tiles, long reduction: split M so that tiles * slices fills ONE
// wave of workgroups (<= 256 = one per CU; the kernel holds 128 KiB of LDS)
// with >= 16 k-tiles per slice (attn-out: 28 slices of 9 k-tiles 66 us vs 16
// of 16 62 us -- short slices are all prologue / epilogue).  Measured (scripts/gemm_sweep.sh, BERT shapes):
// a second, partial wave of workgroups costs more than it returns (qkv 108 us
// at 216 workgroups vs 148 at 432), and power-of-two slice counts left up to
// 44 % of the CUs idle (ffn: 36 tiles x 4 = 144 workgroups) -- hence
// floor(256 / tiles) slices.  > 1 means the kernel ADDS into dw (the caller
// zeroes dw unless accumulating).
int gemm_big_wgrad_splits(int M, int N, int K) {
  const int tiles = ((N + GB_BM - 1) / GB_BM) * ((K + GB_BN - 1) / GB_BN);
  const int nk = M / GB_KQ;
  return std::max(1, std::min(256 / std::max(1, tiles), nk / 16));
}

}  // namespace mfl
