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

namespace mfl {

struct BigGemmArgs {
  const uint16_t* a;
  const uint16_t* b;
  int M, N, K;           // C[M][N] = sum_k A(m, k) * B(n, k)
  int lda, ldb;          // row pitch (elements) of the STORED operands
  uint32_t a_bytes, b_bytes;
  uint16_t* c16;         // bf16 output (forward / dgrad)
  float* c32;            // fp32 output (wgrad)
  int ldc;
  const float* bias;     // [N]
  const uint16_t* resid; // [M][ldc]
  uint16_t* act_out;     // [M][ldc] gelu(y)
  int accum;
  int splits;            // split-K slices (fp32 output only; atomics into c32)
  int kt_per_split;      // k-tiles per slice
};

namespace {

constexpr int GB_BM = 256, GB_BN = 256, GB_BK = 64;
constexpr int GB_TILE = GB_BM * GB_BK * 2;  // bytes of one operand tile (32 KiB)
constexpr int GB_STAGE = 2 * GB_TILE;       // A + B
constexpr int GB_EPI_LD = 68;               // fp32 staging row pitch (64 + 4)
constexpr size_t GB_LDS = 2 * GB_STAGE;     // 128 KiB (epilogue: 8 x 32 x 68 x 4 = 69.6 KiB)

// One operand tile (256 rows x 64 k) global -> LDS, 4 DMA instructions per wave.
template <bool T>
__device__ __forceinline__ void stage_operand(__amdgpu_buffer_rsrc_t rs, int ld, int row0, int k0,
                                              uint8_t* dst, int wave, int lane) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = wave + 8 * u;  // 1-KiB instruction index within the tile
    uint32_t off;
    if constexpr (!T) {
      // [row][k]: 8 rows of 128 B per instruction
      const int row = 8 * i + (lane >> 3);
      const int lc = (lane & 7) ^ swz_b128<128>(row);
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

template <bool T>
__device__ __forceinline__ bf16x8 frag(const uint8_t* tile, int kk, int r0, int lane) {
  if constexpr (T) return tr_frag<512>(tile, kk, r0, lane);
  else return b128_frag<128>(tile, kk, r0, lane);
}

template <bool AT, bool BT, bool OUT32>
__global__ __launch_bounds__(512) void gemm_big_kernel(BigGemmArgs p) {
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
  const int tiles_n = p.N / GB_BN;
  const int m0 = (wgid / tiles_n) * GB_BM;
  const int n0 = (wgid - (wgid / tiles_n) * tiles_n) * GB_BN;
  const auto rsA = make_rsrc(p.a, p.a_bytes);
  const auto rsB = make_rsrc(p.b, p.b_bytes);
  const int kt0 = blockIdx.y * p.kt_per_split;
  const int nk = min(p.K / GB_BK - kt0, p.kt_per_split);
  if (nk <= 0) return;  // block-uniform: an empty trailing slice

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt, int stage) {
    uint8_t* st = smem + stage * GB_STAGE;
    stage_operand<AT>(rsA, p.lda, m0, (kt0 + kt) * GB_BK, st, wave, lane);
    stage_operand<BT>(rsB, p.ldb, n0, (kt0 + kt) * GB_BK, st + GB_TILE, wave, lane);
  };
  auto compute = [&](int stage) {
    const uint8_t* As = smem + stage * GB_STAGE;
    const uint8_t* Bs = As + GB_TILE;
#pragma unroll
    for (int kk = 0; kk < GB_BK; kk += 32) {
      bf16x8 bfr[4], af[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BT>(Bs, kk, wn * 64 + 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = frag<AT>(As, kk, wm * 128 + 16 * i, lane);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  };

  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    wait_vmcnt<0>();                                   // own DMA of tile kt landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own reads of the other stage retired
    lds_barrier();  // everyone's tile kt landed; everyone done reading stage (kt+1)&1
    if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);     // in flight across the compute
    compute(kt & 1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_barrier();  // the ring is free for the epilogue staging

  if constexpr (OUT32) {
    if (p.splits > 1) {
      // split-K: fp32 atomics straight from the accumulators (16 lanes cover
      // 64 contiguous bytes of a row per instruction)
      const int fq = lane >> 4, fr = lane & 15;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = m0 + wm * 128 + 16 * i + 4 * fq + e;
            const int col = n0 + wn * 64 + 16 * j + fr;
            atomicAdd(p.c32 + (int64_t)row * p.ldc + col, acc[i][j][e]);
          }
      return;
    }
  }

  // ---- epilogue: per wave, 4 chunks of 32 rows x 64 cols through LDS --------
  float* W = reinterpret_cast<float*>(smem) + wave * (32 * GB_EPI_LD);
  const int fq = lane >> 4, fr = lane & 15;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          W[(16 * i2 + 4 * fq + e) * GB_EPI_LD + 16 * j + fr] = acc[2 * c + i2][j][e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int item = lane + 64 * u;
      const int rl = item >> 3, cg = item & 7;
      const float4 lo = *reinterpret_cast<const float4*>(W + rl * GB_EPI_LD + cg * 8);
      const float4 hi = *reinterpret_cast<const float4*>(W + rl * GB_EPI_LD + cg * 8 + 4);
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      const int row = m0 + wm * 128 + 32 * c + rl;
      const int col = n0 + wn * 64 + cg * 8;
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
          unpack8(*reinterpret_cast<const uint4*>(dst), o);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += o[k];
        }
        if (p.bias) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += p.bias[col + k];
        }
        if (p.resid) {
          float o[8];
          unpack8(*reinterpret_cast<const uint4*>(p.resid + off), o);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += o[k];
        }
        const uint4 packed = pack8(v);
        *reinterpret_cast<uint4*>(dst) = packed;
        if (p.act_out) {  // exact (erf) GELU of the stored pre-activation
          float f[8], h[8];
          unpack8(packed, f);
#pragma unroll
          for (int k = 0; k < 8; ++k) h[k] = 0.5f * f[k] * (1.f + erff(f[k] * 0.70710678f));
          *reinterpret_cast<uint4*>(p.act_out + off) = pack8(h);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // reads of this chunk done before the next overwrites W
  }
}

template <bool AT, bool BT, bool OUT32>
void launch_big(const BigGemmArgs& p, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_big_kernel<AT, BT, OUT32>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)GB_LDS);
    attr = true;
  }
  const dim3 grid((unsigned)((p.M / GB_BM) * (p.N / GB_BN)), (unsigned)p.splits);
  gemm_big_kernel<AT, BT, OUT32><<<grid, 512, GB_LDS, s>>>(p);
}

}  // namespace

bool gemm_big_ok(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 && M % GB_BM == 0 && N % GB_BN == 0 && K % GB_BK == 0 &&
         (int64_t)M * K * 2 < (1LL << 32) && (int64_t)N * K * 2 < (1LL << 32) &&
         (int64_t)M * N * 2 < (1LL << 32);
}

void launch_gemm_big_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias,
                         const uint16_t* resid, uint16_t* act_out, int M, int N, int K, hipStream_t s) {
  BigGemmArgs p{};
  p.a = x; p.b = w; p.M = M; p.N = N; p.K = K; p.lda = K; p.ldb = K;
  p.a_bytes = (uint32_t)((int64_t)M * K * 2); p.b_bytes = (uint32_t)((int64_t)N * K * 2);
  p.c16 = y; p.ldc = N; p.bias = bias; p.resid = resid; p.act_out = act_out;
  p.splits = 1; p.kt_per_split = K / GB_BK;
  launch_big<false, false, false>(p, s);
}

void launch_gemm_big_dgrad(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int M, int N, int K,
                           bool accumulate, hipStream_t s) {
  // dX[M][K] = dY[M][N] . W[N][K]: output columns = K, reduction = N
  BigGemmArgs p{};
  p.a = dy; p.b = w; p.M = M; p.N = K; p.K = N; p.lda = N; p.ldb = K;
  p.a_bytes = (uint32_t)((int64_t)M * N * 2); p.b_bytes = (uint32_t)((int64_t)N * K * 2);
  p.c16 = dx; p.ldc = K; p.accum = accumulate;
  p.splits = 1; p.kt_per_split = N / GB_BK;
  launch_big<false, true, false>(p, s);
}

void launch_gemm_big_wgrad(const uint16_t* x, const uint16_t* dy, float* dw, int M, int N, int K,
                           bool accumulate, hipStream_t s) {
  // dW[N][K] (+)= dY^T X: output rows = N, columns = K, reduction = M
  BigGemmArgs p{};
  p.a = dy; p.b = x; p.M = N; p.N = K; p.K = M; p.lda = N; p.ldb = K;
  p.a_bytes = (uint32_t)((int64_t)M * N * 2); p.b_bytes = (uint32_t)((int64_t)M * K * 2);
  p.c32 = dw; p.ldc = K; p.accum = accumulate;
  p.splits = gemm_big_wgrad_splits(M, N, K);
  p.kt_per_split = (M / GB_BK + p.splits - 1) / p.splits;
  launch_big<true, true, true>(p, s);
}

// Few output tiles, long reduction: split M so >= 256 workgroups run, each
// slice >= 8 k-tiles.  > 1 means the kernel ADDS into dw with atomics (the
// caller zeroes dw unless accumulating).
int gemm_big_wgrad_splits(int M, int N, int K) {
  const int tiles = (N / GB_BM) * (K / GB_BN);
  const int nk = M / GB_BK;
  int s = 1;
  while (tiles * s < 256 && nk / (2 * s) >= 8) s *= 2;
  return s;
}

}  // namespace mfl
