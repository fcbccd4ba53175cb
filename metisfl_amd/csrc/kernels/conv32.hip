// K6 (fp32): NHWC fp32 convolution forward / backward-data / backward-weight
// as implicit GEMMs on the gfx950 fp32 matrix cores (v_mfma_f32_32x32x2_f32).
//
// The reference trains in fp32 through Keras Conv2D layers
// (examples/keras/models/cifar_cnn.py:19-41, metisfl/models/keras/
// keras_model_ops.py:117-197: plain fit, no mixed-precision policy).  This is
// the reference-precision learner path: operands, accumulators and outputs
// are IEEE fp32, and gfx950 has no xf32/TF32 shortcut, so every product is an
// exact fp32 FMA (cdna_hip_programming.md 'FP32-input MFMA').  The bf16 family
// (conv.hip) stays as the explicit mixed-precision option.
//
// Second variant (MFL_C32_BF16X3=1, namespace mfl::c32s): same fp32 operands,
// LDS staging, fp32 accumulators and outputs, but each k-tile's fragments are
// split in registers into bf16 hi + lo and multiplied as hi*hi + hi*lo +
// lo*hi on v_mfma_f32_32x32x16_bf16 (16x the fp32 MFMA rate, 3 products):
// per-product relative error <= ~2^-17, 4e-6 measured on whole convolutions
// (exact: 3e-7).  The fp32 MFMA shares the VALU datapath, so the exact loop
// is MFMA-paced; the split loop is paced by its ~2.5 VALU per operand value
// and by the fp32 operand bytes it streams -- 1.52 -> 1.22 ms per ResNet-18
// step (profiles/r2/fp32_bf16x3_step_summary.txt).
//
// Design for CDNA4 (not a port of anything -- the reference has no kernels):
//  * fp32 MFMA runs at 1/16 of the bf16 rate (64 FLOP/clk/SIMD), so here the
//    step is COMPUTE-bound where the bf16 one is latency-bound: tiles are
//    chosen to keep every SIMD's matrix pipe fed (>= 256 workgroups, split-K
//    on the small-M CIFAR stages), not to shave launch latency.
//  * v_mfma_f32_32x32x2_f32 takes ONE fp32 per lane per operand:
//    lane l = (i = l&31, h = l>>5) supplies A[i][h] and B[h][i].  Which real
//    reduction index sits in each (MFMA, h) slot is free as long as A and B
//    agree, so a lane reads 4 consecutive k of its row with one ds_read_b128
//    and feeds them to 4 successive MFMAs: MFMA e of k-group g reduces
//    k = 8g + 4h + e.  Operands whose global layout is k-contiguous (im2col
//    rows of X / dY, the OHWI weight rows of the forward pass) are staged
//    [row][k]; operands whose layout is row-contiguous (W^T for dgrad, both
//    wgrad operands) are staged [k][row] and read with ds_read_b32 at the same
//    k index -- no transpose pass, no transposing LDS writes.
//  * Operand tiles move global -> LDS by LDS-DMA (buffer_load_dwordx4 ...
//    lds, 16 B per lane), 3-stage ring with 2 k-tiles in flight and counted
//    vmcnt waits, hardware bounds checks for padding (an out-of-range offset
//    reads zeros) -- the same staging machinery as the bf16 kernels
//    (lds_tiles.h).  [row][k] tiles are 128-B rows (32 fp32) with the
//    (row>>1)&7 XOR chunk swizzle: the 4 lane groups of a ds_read_b128
//    (rows {0-3,12-15,20-27} / {4-11,16-19,28-31} at one chunk) land on 16
//    distinct 16-B bank slots.
//  * Epilogue through LDS: the tile is written as float4 rows (coalesced), the
//    forward BN statistics (sum, sum^2 per channel) -- or, for dgrad, the
//    consumer BN-backward reductions -- are reduced in the same pass and added
//    with fp64 atomics.  Split-K slices reduce in-launch (last arriver sums
//    the write-through slabs in slice order: bitwise deterministic).
//  * Stride-2 dgrad runs parity-class decomposed (PAR), as in conv.hip.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include <type_traits>
#include <utility>

#include "kernels/common.h"
#include "kernels/conv32.h"
#include "kernels/opt_tail_dev.h"
#include "kernels/lds_tiles.h"

// Built twice (csrc/build.py): MFL_C32_BF16X3=0 -> namespace mfl::c32x (exact
// fp32 MFMA), =1 -> mfl::c32s (3-product bf16 split, see mma_tile).
#ifndef MFL_C32_BF16X3
#define MFL_C32_BF16X3 0
#endif

#if MFL_C32_BF16X3
#define MFL_C32_VARIANT c32s
#else
#define MFL_C32_VARIANT c32x
#endif

namespace mfl {
namespace MFL_C32_VARIANT {

namespace {

#ifndef MFL_C32_BK
#define MFL_C32_BK 32
#endif
constexpr int kBK = MFL_C32_BK;  // fp32 k-elements per tile (32: 128-B rows)
constexpr int kRowB = kBK * 4;       // [row][k] tiles: 256-B rows
constexpr int kRPI = 1024 / kRowB;   // rows per 1-KiB LDS-DMA instruction
constexpr int kCPR = kRowB / 16;     // 16-B chunks per row

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma_bf16x16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}


// fp32 -> bf16 (hi, lo) with a = hi + lo + e, |e| <= 2^-18 |a|: hi = RNE(a),
// a - hi is exact in fp32 (<= 16 significant bits), lo = RNE(a - hi).
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16v2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cvt_pk_bf16(f32x2 v) {  // one v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16v2));
}
// 20 VALU per 8 values: 4 cvt_pk, 8 unpack (shift / and), 4 v_pk_add_f32, 4 cvt_pk
__device__ __forceinline__ void split_hl(const f32x4& p, const f32x4& q, bf16x8& hi, bf16x8& lo) {
  const f32x2 v[4] = {{p[0], p[1]}, {p[2], p[3]}, {q[0], q[1]}, {q[2], q[3]}};
  u32x4 h, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t w = cvt_pk_bf16(v[i]);
    h[i] = w;
    l[i] = cvt_pk_bf16(v[i] - f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)});
  }
  hi = __builtin_bit_cast(bf16x8, h);
  lo = __builtin_bit_cast(bf16x8, l);
}

// One k-tile of MFMAs.  Exact mode: 32x32x2 fp32, MFMA (g, e) of lane half h
// reduces k = 8g + 4h + e.  Split mode (3-product bf16): the two 4-k fragments
// of groups 2g2 and 2g2+1 form one lane's 8 bf16 k-slots of a 32x32x16 MFMA
// (k = 16g2 + {4h + e, 8 + 4h + e}); A and B use the same slots, so the
// reduction is over the same k set and acc += Ahi Bhi + Ahi Blo + Alo Bhi.
// B operand already packed by the producer (the optimizer's weight mirror:
// dword = hi << 16 | lo, the same hi / lo split_hl computes): 8 v_perm per 8
// values instead of 20 VALU
__device__ __forceinline__ void unpack_hl(const f32x4& p, const f32x4& q, bf16x8& hi, bf16x8& lo) {
#ifdef MFL_C32_NODECODE  // timing experiment only (MFL_C32_EXTRA=-DMFL_C32_NODECODE=1 at build time):
                         // operands reinterpreted, no decode VALU, wrong products -- bounds what a
                         // decode-free operand layout would return (profiles/ANALYSIS.md, round 3)
  hi = __builtin_bit_cast(bf16x8, p);
  lo = __builtin_bit_cast(bf16x8, q);
  return;
#endif
  const uint32_t d[8] = {__float_as_uint(p[0]), __float_as_uint(p[1]), __float_as_uint(p[2]), __float_as_uint(p[3]),
                         __float_as_uint(q[0]), __float_as_uint(q[1]), __float_as_uint(q[2]), __float_as_uint(q[3])};
  u32x4 h, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = __builtin_amdgcn_perm(d[2 * i + 1], d[2 * i], 0x07060302u);  // high halves: hi(2i), hi(2i+1)
    l[i] = __builtin_amdgcn_perm(d[2 * i + 1], d[2 * i], 0x05040100u);  // low halves: lo(2i), lo(2i+1)
  }
  hi = __builtin_bit_cast(bf16x8, h);
  lo = __builtin_bit_cast(bf16x8, l);
}

// BPACK / APACK (bf16x3 only): the B / A fragments hold packed hi|lo dwords
// (the optimizer's weight mirror; activations as the fp32 BN apply wrote their
// mirror; dY as the fp32 BN backward wrote it).  Every c32s operand arrives
// packed, so the k-loop never splits.
template <int TM, int TN, bool BPACK = false, bool APACK = false, typename FA, typename FB>
__device__ __forceinline__ void mma_tile(const FA& fa, const FB& fb, f32x16 (&acc)[TM][TN]) {
#if MFL_C32_BF16X3
#pragma unroll
  for (int g2 = 0; g2 < kBK / 16; ++g2) {
    bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if constexpr (APACK) unpack_hl(fa[2 * g2][i], fa[2 * g2 + 1][i], ah[i], al[i]);
      else split_hl(fa[2 * g2][i], fa[2 * g2 + 1][i], ah[i], al[i]);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (BPACK) unpack_hl(fb[2 * g2][j], fb[2 * g2 + 1][j], bh[j], bl[j]);
      else split_hl(fb[2 * g2][j], fb[2 * g2 + 1][j], bh[j], bl[j]);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = mfma_bf16x16(al[i], bh[j], acc[i][j]);
        acc[i][j] = mfma_bf16x16(ah[i], bl[j], acc[i][j]);
        acc[i][j] = mfma_bf16x16(ah[i], bh[j], acc[i][j]);
      }
  }
#else
#pragma unroll
  for (int grp = 0; grp < kBK / 8; ++grp)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_f32(fa[grp][i][e], fb[grp][j][e], acc[i][j]);
#endif
}
// MFMA count / VALU budget per k-tile for the interleave pattern
template <int TM, int TN>
constexpr int kTileMfma = MFL_C32_BF16X3 ? 3 * (kBK / 16) * TM * TN : 4 * (kBK / 8) * TM * TN;
constexpr int kTileValu = MFL_C32_BF16X3 ? 16 : 6;
__device__ __forceinline__ int fdiv(int x, const FastDiv& f) {
  return (int)((__umulhi((uint32_t)x, f.m) >> f.sh) + ((uint32_t)x & f.id));
}

// A workgroup's coordinates in its own GEMM's grid.  The stand-alone kernels
// take them from the hardware; the paired dgrad+wgrad launch maps one
// hardware grid onto the two GEMMs' grids.
struct Blk {
  int x, y, z, gx, gy, gz;
};
// XCD-grouped block order.  The hardware deals workgroups round-robin over the
// 8 XCDs (b % 8), so the 8 tiles dispatched together -- neighbouring output
// rows that share their 3x3 halo rows -- land on 8 different L2s (measured L2
// hit rate of the bf16x3 forward: 62 %).  Within each chunk of 64 dispatched
// blocks, XCD x takes the 8 consecutive virtual tiles [8x, 8x + 8): the
// dispatch order (dgrad-before-wgrad in the paired launches, split-K slices
// 256 apart on one XCD) is kept at 64-block granularity.  (A global
// XCD-contiguous order lost that ordering: 1.22 -> 1.30 ms.)
__device__ __forceinline__ int xcd_group(int b, int n) {
  const int base = b & ~63;
  if (base + 64 > n) return b;  // ragged last chunk: hardware order
  return base + ((b & 7) << 3) + ((b >> 3) & 7);
}
__device__ __forceinline__ Blk hw_blk() {
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const int v = xcd_group(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gz);
  return Blk{v % gx, (v / gx) % gy, v / (gx * gy), gx, gy, gz};
}

// DMA offset, or past every buffer range when !ok -- bitwise, so hipcc keeps
// the address math branch-free (a ?: here became an exec-masked branch that
// split the k-loop body)
__device__ __forceinline__ uint32_t oob_or(bool ok, uint32_t off) { return off | (kOOB & (0u - (uint32_t)!ok)); }

// fp32 [row][kBK] tile: 16-B chunk ch of `row` (swizzled)
__device__ __forceinline__ int rk_off(int row, int ch) { return row * kRowB + ((ch ^ swz_b128<kRowB>(row)) << 4); }

#ifndef MFL_C32_DBG
#define MFL_C32_DBG 0  // timing experiments only: bit0 skip MFMAs, bit1 skip operand DMA
#endif
#ifndef MFL_C32_GENERIC
#define MFL_C32_GENERIC 0  // 1: every shape on the generic address path (A/B experiments)
#endif

template <int V>
using IC = std::integral_constant<int, V>;
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(IC<I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// k-loop: LDS ring of NS stages (DMA 2-3 tiles ahead) + register double
// buffer of MFMA fragments (LDS reads 1 tile ahead).  Iteration kt:
//   wait own DMA of tile kt+1, wait own fragment reads of tile kt, barrier
//   (=> every wave's tile kt+1 landed AND every wave holds tile kt's
//   fragments in registers, so stage kt%NS is free) -> issue the DMA of tile
//   kt+NS into stage kt%NS -> issue the fragment reads of tile kt+1 -> MFMAs
//   of tile kt.  The reads and the DMA address math run UNDER the MFMAs of the
//   same wave (sched_group_barrier interleave).
// The loop is unrolled by lcm(NS, 2) so that the ring stage AND the fragment
// register set of every step are compile-time constants: LDS addresses fold
// into ds_read / M0 immediates and the loop carries no per-tile VALU address
// math.  That matters more for fp32 than for bf16: the f32 MFMA shares the
// VALU datapath (measured: a VALU wave beside an MFMA wave on one SIMD runs
// no faster than both serialised, profiles/r2/mfma_valu_coissue_probe.log),
// so every VALU instruction in the loop is MFMA time lost.  DMAs past the
// last tile use out-of-range offsets (zero fill, no memory traffic).
// `issue` must be called for tiles 0, 1, 2, ... in order (it may carry
// scalar iterator state).
template <int NS, int L, typename Issue, typename Read, typename Mma>
__device__ __forceinline__ void ring_loop(int nk, Issue& issue, Read& read, Mma& mma) {
  static_assert((NS - 1) * L <= 63, "vmcnt is a 6-bit counter");
  static_for<NS>([&](auto u) { issue(decltype(u)::value, u); });
  wait_vmcnt<(NS - 1) * L>();  // tile 0
  lds_barrier();
  read(IC<0>{}, IC<0>{});
  auto step = [&](int kt, auto stc, auto setc) {
    constexpr int S = decltype(stc)::value, C = decltype(setc)::value;
    constexpr int NXT = S == NS - 1 ? 0 : S + 1;
    wait_vmcnt<(NS - 2) * L>();            // tile kt+1 landed (kt+2.. may fly)
    __builtin_amdgcn_s_waitcnt(0xC07F);    // lgkmcnt(0): tile kt's fragments in registers
    lds_barrier();
    issue(kt + NS, stc);
    read(IC<NXT>{}, IC<1 - C>{});
    mma(setc);
  };
  constexpr int P = NS % 2 == 0 ? NS : 2 * NS;
  int kt = 0;
  for (; kt + P <= nk; kt += P)
    static_for<P>([&](auto j) {
      constexpr int J = decltype(j)::value;
      step(kt + J, IC<J % NS>{}, IC<J % 2>{});
    });
  static_for<P - 1>([&](auto j) {
    constexpr int J = decltype(j)::value;
    if (kt + J < nk) step(kt + J, IC<J % NS>{}, IC<J % 2>{});
  });
  wait_vmcnt<0>();  // the trailing (zero-fill) DMAs land before smem is reused
  __builtin_amdgcn_s_waitcnt(0xC07F);
}

// Interleave pattern for one k-tile: per MFMA, one LDS read, up to V VALU,
// 2 SALU and one VMEM (LDS-DMA) instruction slot in behind it.
template <int NMFMA, int V>
__device__ __forceinline__ void interleave_mfma() {
#pragma unroll
  for (int i = 0; i < NMFMA; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    __builtin_amdgcn_sched_group_barrier(0x002, V, 0);  // VALU
    __builtin_amdgcn_sched_group_barrier(0x004, 2, 0);  // SALU
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (LDS-DMA)
  }
}

// GEMM row -> output pixel (identity, or the parity-class order of PAR dgrad)
__device__ __forceinline__ int out_pixel32(const Conv32Args& a, int row) {
  if (!a.par_mc) return row;
  const int q2 = a.g.Q >> 1, pq2 = (a.g.P >> 1) * q2;
  const int cls = row / a.par_mc;
  const int mc = row - cls * a.par_mc;
  const int n = mc / pq2;
  const int rem = mc - n * pq2;
  const int y = rem / q2, x = rem - y * q2;
  return (n * a.g.P + 2 * y + (cls >> 1)) * a.g.Q + 2 * x + (cls & 1);
}

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// Output tile [BM][BN + 4] fp32 in LDS -> y (float4 rows), + fused channel sums.
template <int BM, int BN>
__device__ __forceinline__ void tile_epilogue32(const Conv32Args& a, const Blk& b, int m0, int n0,
                                                const float* tile, float* red) {
  constexpr int TST = BN + 4;
  constexpr int CPR = BN / 4;      // float4 per row
  constexpr int RPP = 256 / CPR;   // rows per pass
  const ConvGeom& g = a.g;
  double* stats = a.bn_acc ? a.bn_acc : a.stats;
  const int t = threadIdx.x;
  const int cg = t % CPR, r0 = t / CPR;
  const int col = n0 + cg * 4;
  const bool col_ok = col < g.Ng;  // Ng % 4 == 0
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s, mu = s, is = s;
  if (a.bn_acc && col_ok) {
    mu = *reinterpret_cast<const float4*>(a.bn_mean + col);
    is = *reinterpret_cast<const float4*>(a.bn_invstd + col);
  }
  // Every global read of the output stage (the accumulated output, the
  // consumer BN's mask y and input z) is issued up front for all of this
  // thread's rows: issued row by row after each row's store they could not
  // be hoisted (the store may alias them) and each row paid a full
  // load latency.  The buffers never alias y (dX vs the BN's saved
  // activations).
  constexpr int NIT = (BM + RPP - 1) / RPP;
  float4 pre_acc[NIT], pre_y[NIT], pre_z[NIT];
  const bool rd_y = a.bn_acc && a.bn_y, rd_z = stats && a.bn_acc;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int rl = r0 + it * RPP, row = m0 + rl;
    pre_acc[it] = pre_y[it] = pre_z[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rl >= BM || row >= g.M || !col_ok) continue;
    const int64_t off = (int64_t)out_pixel32(a, row) * g.Ng + col;
    if (a.accum) pre_acc[it] = *reinterpret_cast<const float4*>(a.y + off);
    if (rd_y) pre_y[it] = *reinterpret_cast<const float4*>(a.bn_y + off);
    if (rd_z) pre_z[it] = *reinterpret_cast<const float4*>(a.bn_z + off);
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int rl = r0 + it * RPP, row = m0 + rl;
    if (rl >= BM || row >= g.M || !col_ok) continue;
    float4 v = *reinterpret_cast<const float4*>(tile + rl * TST + cg * 4);
    const int64_t off = (int64_t)out_pixel32(a, row) * g.Ng + col;
    float4* dst = reinterpret_cast<float4*>(a.y + off);
    if (a.accum) v = f4add(v, pre_acc[it]);
    if (rd_y) {
      // the consumer BN's ReLU mask applied on the way out: dX is stored as
      // g = dX [y > 0], so that BN's backward apply reads no mask
      const float4 ym = pre_y[it];
      v.x = ym.x > 0.f ? v.x : 0.f;
      v.y = ym.y > 0.f ? v.y : 0.f;
      v.z = ym.z > 0.f ? v.z : 0.f;
      v.w = ym.w > 0.f ? v.w : 0.f;
    }
    *dst = v;
    if (stats) {
      if (a.bn_acc) {
        const float4 z = pre_z[it];
        const float4 gk = v;
        s = f4add(s, gk);
        q.x += gk.x * ((z.x - mu.x) * is.x);
        q.y += gk.y * ((z.y - mu.y) * is.y);
        q.z += gk.z * ((z.z - mu.z) * is.z);
        q.w += gk.w * ((z.w - mu.w) * is.w);
      } else {
        s = f4add(s, v);
        q.x += v.x * v.x;
        q.y += v.y * v.y;
        q.z += v.z * v.z;
        q.w += v.w * v.w;
      }
    }
  }
  if (!stats) return;
  // replica of this workgroup (b % 8 = the XCD under round-robin placement)
  stats += (int64_t)((b.x + b.y * b.gx + b.z * b.gx * b.gy) % a.reps) * 2 * g.Ng;
  reinterpret_cast<float4*>(red)[2 * t] = s;
  reinterpret_cast<float4*>(red)[2 * t + 1] = q;
  __syncthreads();
  if (t < BN) {
    const int cgi = t >> 2, k = t & 3;
    double sa = 0.0, sb = 0.0;
#pragma unroll 4
    for (int r = 0; r < RPP; ++r) {
      sa += red[(r * CPR + cgi) * 8 + k];
      sb += red[(r * CPR + cgi) * 8 + 4 + k];
    }
    const int c = n0 + t;
    if (c < g.Ng) {
      atomicAdd(&stats[c], sa);
      atomicAdd(&stats[g.Ng + c], sb);
    }
  }
}

// ---------------------------------------------------------------------------
// Forward / dgrad:  Y[m][n] = sum_k A[m][k] * B[k][n]
//   fwd:   A = im2col(X) [M][R*S*C],  B[k][n] = W[n][k]   (both [row][k] tiles)
//   dgrad: A = stride-aware gather of dY [M = N*H*W][R*S*Co],
//          B[k = (r,s,co)][n = ci] = W[co][r][s][ci]      ([k][n] tile, b32 reads)
// GEN selects the generic per-element address path (channel counts that are
// not a multiple of the k-tile -- the 8-channel stem -- and the masked
// stride-2 dgrad gather); otherwise a k-tile lies inside ONE filter tap, so
// the tap (r, s) and channel offset are scalar per-tile state, each DMA row
// keeps its tap-(0,0) address and a 9-bit tap-validity mask from the
// prologue, and a DMA costs ~4 VALU (bit test, add, select) instead of ~20
// including quarter-rate integer multiplies.
template <int BM, int BN, bool DGRAD, int KS, int ST, bool PAR, int NS, bool GEN>
__device__ __forceinline__ void conv32_gemm_body(const Conv32Args& a, const Blk& blk, uint8_t* smem) {
  constexpr int A_BYTES = BM * kRowB;
  constexpr int STAGE = A_BYTES + BN * kRowB;
  constexpr int ACH = BM * kBK / 1024;  // DMA instructions per wave per k-tile (1 KiB each)
  constexpr int BCH = BN * kBK / 1024;
  constexpr int TM = BM / 64, TN = BN / 64;  // 32x32 MFMA tiles per wave
  constexpr int BRB = BN * 4;                // dgrad B row bytes
  constexpr int B_RPI = 1024 / BRB, B_CPR = BRB / 16;
  static_assert(GEN || !(DGRAD && ST > 1 && !PAR), "masked stride-2 dgrad needs the generic path");
  const ConvGeom& g = a.g;
  const auto rsA = make_rsrc(a.src, a.src_bytes);
  const auto rsB = make_rsrc(a.wgt, a.wgt_bytes);
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blk.x * BM;
  const int n0 = blk.y * BN;
  const int kbeg = blk.z * a.kchunk;
  int cls = 0, r0 = 0, s0 = 0, nr = KS, ns = KS, dh = 0, dw = 0, kc_end = g.K;
  if constexpr (PAR) {
    cls = m0 / a.par_mc;
    const int qh = cls >> 1, qw = cls & 1;
    r0 = (qh + g.pad) & 1;
    s0 = (qw + g.pad) & 1;
    nr = (KS - r0 + 1) >> 1;
    ns = (KS - s0 + 1) >> 1;
    dh = (qh + g.pad - r0) >> 1;
    dw = (qw + g.pad - s0) >> 1;
    kc_end = nr * ns * g.C;
  }
  const int kend = min(kc_end, kbeg + a.kchunk);
  const int nk = max(0, (kend - kbeg + kBK - 1) / kBK);
  const int HWC = g.H * g.W * g.C;

  // [row][k] DMA: instruction i of wave w fills rows 32i + 8w + lane/8,
  // physical chunk lane%8 <- logical chunk (k offset) a_kc (i-independent).
  const int lrow = wave * kRPI + lane / kCPR;
  const int a_kc = ((lane % kCPR) ^ swz_b128<kRowB>(lrow)) * 4;  // same for every i: rows step by 4*kRPI
  int a_nb[ACH], a_y0[ACH], a_x0[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    const int m = m0 + lrow + 4 * kRPI * i;
    const int mm = m < g.M ? m : 0;
    if constexpr (PAR) {
      const int q2 = g.Q >> 1;
      const int pq2 = (g.P >> 1) * q2;
      const int mc = mm - cls * a.par_mc;
      const int n = mc / pq2;
      const int rem = mc - n * pq2;
      const int y = rem / q2;
      a_nb[i] = n * HWC;
      a_y0[i] = y + dh;
      a_x0[i] = rem - y * q2 + dw;
    } else {
      const int n = fdiv(mm, a.dpq);
      const int rem = mm - n * g.P * g.Q;
      const int oy = fdiv(rem, a.dq);
      const int ox = rem - oy * g.Q;
      a_nb[i] = n * HWC;
      a_y0[i] = DGRAD ? oy + g.pad : oy * ST - g.pad;
      a_x0[i] = DGRAD ? ox + g.pad : ox * ST - g.pad;
    }
    if (m >= g.M) a_y0[i] = -(1 << 28);  // forces the OOB offset
  }

  // ---- fast path state (GEN == false) ----
  // per DMA row: byte address of tap (0,0) + this lane's k chunk, and the
  // validity of every tap (bit r*ns + s; fwd reads (y0 + r, x0 + s), dgrad
  // (y0 - r, x0 - s))
  int a_base[ACH];
  uint32_t a_vm[ACH];
  // B operand: fwd W[n][k] rows (per lane n, k chunk a_kc); dgrad W^T [k][n]
  int b_base[BCH];
  bool b_ok[BCH];
  // scalar per-tile iterator: tap (tr, ts) of the tile, channel offset c0
  int tr = 0, ts = 0, c0 = 0;
  if constexpr (!GEN) {
    const int sgn = DGRAD ? -1 : 1;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      a_base[i] = (int)(((uint32_t)a_nb[i] + ((uint32_t)a_y0[i] * g.W + (uint32_t)a_x0[i]) * g.C + a_kc) * 4u);
      uint32_t vm = 0;
      for (int r = 0; r < nr; ++r)
        for (int s2 = 0; s2 < ns; ++s2) {
          const int iy = a_y0[i] + sgn * r, ix = a_x0[i] + sgn * s2;
          const bool ok = (iy >= 0) & (iy < g.H) & (ix >= 0) & (ix < g.W);
          vm |= (uint32_t)ok << (r * ns + s2);
        }
      a_vm[i] = vm;
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      if constexpr (DGRAD) {
        const int row = (wave + 4 * i) * B_RPI + lane / B_CPR;  // k within the tile
        const int n = n0 + (lane % B_CPR) * 4;
        b_base[i] = (row * KS * KS * g.Ng + n) * 4;
        b_ok[i] = n < g.Ng;
      } else {
        const int n = n0 + lrow + 4 * kRPI * i;
        b_base[i] = (n * g.K + a_kc) * 4;
        b_ok[i] = n < g.Ng;
      }
    }
    const int rs0 = kbeg / g.C;  // scalar, once
    c0 = kbeg - rs0 * g.C;
    tr = rs0 / ns;
    ts = rs0 - tr * ns;
  }

  auto issue = [&](int kt, auto stc) {
    if constexpr (MFL_C32_DBG & 2) return;
    constexpr int S = decltype(stc)::value;
    uint8_t* st = smem + S * STAGE;
    const int kb = kbeg + kt * kBK;
    if constexpr (!GEN) {
      const bool kv = kb < kend;
      const int tap = kv ? tr * ns + ts : 31;  // bit 31 is never set: every row OOB
      const int sp = (tr * g.W + ts) * g.C;   // tap offset (elements)
      const int aoff = ((DGRAD ? -sp : sp) + c0) * 4;
#pragma unroll
      for (int i = 0; i < ACH; ++i) {
        const bool ok = (a_vm[i] >> tap) & 1u;
        dma16(rsA, ok ? (uint32_t)a_base[i] + (uint32_t)aoff : kOOB, st + (wave + 4 * i) * 1024);
      }
      int boff;
      if constexpr (DGRAD) {
        const int rsk = PAR ? (r0 + 2 * tr) * KS + s0 + 2 * ts : tr * KS + ts;  // kernel tap
        boff = (c0 * KS * KS + rsk) * g.Ng * 4;
      } else {
        boff = kb * 4;
      }
#pragma unroll
      for (int i = 0; i < BCH; ++i)
        dma16(rsB, (b_ok[i] & kv) ? (uint32_t)(b_base[i] + boff) : kOOB, st + A_BYTES + (wave + 4 * i) * 1024);
      // advance the scalar iterator by one k-tile (a tile never straddles a
      // tap); selects, not branches: a branch here would cut the step into
      // basic blocks the MFMA interleave cannot cross
      c0 += kBK;
      const int wrap = c0 == g.C;
      c0 = wrap ? 0 : c0;
      ts += wrap;
      const int wrap2 = ts == ns;
      ts = wrap2 ? 0 : ts;
      tr += wrap2;
      return;
    } else {
      {
        const int k = kb + a_kc;
        const int rs = fdiv(k, a.dc);
        const int c = k - rs * g.C;
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
          const uint32_t off = oob_or(ok, (uint32_t)(a_nb[i] + (iy * g.W + ix) * g.C + c) * 4u);
          dma16(rsA, off, st + (wave + 4 * i) * 1024);
        }
      }
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        uint32_t off;
        if constexpr (DGRAD) {
          const int row = (wave + 4 * i) * B_RPI + lane / B_CPR;  // k within the tile
          const int n = n0 + (lane % B_CPR) * 4;
          const int kr = kb + row;
          int rs = fdiv(kr, a.dc);
          const int ko = kr - rs * g.C;
          if (PAR) {  // class tap index -> kernel tap (r0 + 2 j_r, s0 + 2 j_s)
            const int jr = ns == 2 ? rs >> 1 : rs;
            rs = (r0 + 2 * jr) * KS + s0 + 2 * (rs - jr * ns);
          }
          off = oob_or((kr < kend) & (n < g.Ng), (uint32_t)((ko * KS * KS + rs) * g.Ng + n) * 4u);
        } else {
          const int n = n0 + lrow + 4 * kRPI * i;
          const int k = kb + a_kc;
          off = oob_or((k < kend) & (n < g.Ng), (uint32_t)(n * g.K + k) * 4u);
        }
        dma16(rsB, off, st + A_BYTES + (wave + 4 * i) * 1024);
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int li = lane & 31, lh = lane >> 5;
  // fragments of k-group grp (8 k): A as one ds_read_b128 per 32-row tile,
  // B likewise (fwd) or as 4 ds_read_b32 of the [k][n] tile (dgrad)
  auto load = [&](const uint8_t* As, const uint8_t* Bs, int grp, f32x4* af, f32x4* bfr) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * (BM / 2) + 32 * i + li;
      af[i] = *reinterpret_cast<const f32x4*>(As + rk_off(row, 2 * grp + lh));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * (BN / 2) + 32 * j + li;
      if constexpr (DGRAD) {
        const float* Bf = reinterpret_cast<const float*>(Bs);
#pragma unroll
        for (int e = 0; e < 4; ++e) bfr[j][e] = Bf[(8 * grp + 4 * lh + e) * BN + col];
      } else {
        bfr[j] = *reinterpret_cast<const f32x4*>(Bs + rk_off(col, 2 * grp + lh));
      }
    }
  };
  // every fragment of the k-tile is requested up front (TM+TN registers x4
  // per group): the reads of groups 1-3 are in flight while group 0's MFMAs
  // run, and the scheduler barrier keeps hipcc from sinking them back behind
  // the MFMAs (it otherwise re-uses one register set per group and re-exposes
  // the LDS latency before every group)
  f32x4 fa[2][kBK / 8][TM], fb[2][kBK / 8][TN];  // fragment double buffer
  auto read = [&](auto stc, auto set) {
    constexpr int S = decltype(set)::value;
    const uint8_t* As = smem + decltype(stc)::value * STAGE;
    const uint8_t* Bs = As + A_BYTES;
#pragma unroll
    for (int grp = 0; grp < kBK / 8; ++grp) load(As, Bs, grp, fa[S][grp], fb[S][grp]);
  };
  auto mma = [&](auto set) {
    constexpr int S = decltype(set)::value;
    if constexpr (MFL_C32_DBG & 1) return;
    // B = the weight mirror; A = X (fwd) or dY (dgrad), packed by its producer
    mma_tile<TM, TN, MFL_C32_BF16X3 != 0, MFL_C32_BF16X3 != 0>(fa[S], fb[S], acc);
    interleave_mfma<kTileMfma<TM, TN>, kTileValu>();
    __builtin_amdgcn_sched_barrier(0);
  };
  ring_loop<NS, ACH + BCH>(nk, issue, read, mma);
  __syncthreads();  // every wave done with the ring before smem is reused

  // ---- epilogue -----------------------------------------------------------
  constexpr int TST = BN + 4;
  float* tile = reinterpret_cast<float*>(smem);
  float* red = tile + BM * TST;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rl = wm * (BM / 2) + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * lh;
        tile[rl * TST + wn * (BN / 2) + 32 * j + li] = acc[i][j][e];
      }
  __syncthreads();
  const int splits = blk.gz;
  if (splits > 1) {
    // in-launch split-K (write-through slabs + arrival ticket; conv.hip)
    constexpr int F = BM * BN / 1024;  // float4 per thread
    constexpr int C4 = BN / 4;
    const int tile_id = blk.y * blk.gx + blk.x;
    const int ntiles = blk.gx * blk.gy;
    const int64_t zstride = (int64_t)ntiles * BM * BN * 4;
    const auto rsS = make_rsrc(a.ysplit + (int64_t)tile_id * (BM * BN), 0x7FFFFFF0u);
    const uint32_t zoff = (uint32_t)(blk.z * zstride);
#pragma unroll
    for (int u = 0; u < F; ++u) {
      const int f = t + 256 * u;
      const float4 v = *reinterpret_cast<const float4*>(tile + (f / C4) * TST + (f % C4) * 4);
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)}, rsS,
          (int)(zoff + f * 16), 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    int* flag = reinterpret_cast<int*>(red + 256 * 8);
    if (t == 0) {
      const int prev =
          __hip_atomic_fetch_add(&a.counters[tile_id], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == splits - 1;
      if (last) __hip_atomic_store(&a.counters[tile_id], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    float4 sum[F];
#pragma unroll
    for (int u = 0; u < F; ++u) sum[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    // slabs requested 4 at a time (one memory latency per 4 slices instead
    // of per slice), summed in slice order (deterministic, serial-sum bits)
    constexpr int ZB = 4;
    for (int z0 = 0; z0 < splits; z0 += ZB) {
      u32x4 sl[ZB][F];
#pragma unroll
      for (int zz = 0; zz < ZB; ++zz) {
        const int z = z0 + zz;
        if (z >= splits) break;  // uniform: only the real slices' loads issue
#pragma unroll
        for (int u = 0; u < F; ++u) {
          const int f = t + 256 * u;
          sl[zz][u] = __builtin_amdgcn_raw_buffer_load_b128(
              rsS, (int)(z != blk.z ? (uint32_t)(z * zstride + f * 16) : kOOB), 0, 16);  // own slice: LDS
        }
      }
#pragma unroll
      for (int zz = 0; zz < ZB; ++zz) {
        const int z = z0 + zz;
        if (z >= splits) break;
#pragma unroll
        for (int u = 0; u < F; ++u) {
          const int f = t + 256 * u;
          const u32x4 b = sl[zz][u];
          const float4 r = z == blk.z ? *reinterpret_cast<const float4*>(tile + (f / C4) * TST + (f % C4) * 4)
                                      : make_float4(__uint_as_float(b[0]), __uint_as_float(b[1]),
                                                    __uint_as_float(b[2]), __uint_as_float(b[3]));
          sum[u] = f4add(sum[u], r);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < F; ++u) {
      const int f = t + 256 * u;
      *reinterpret_cast<float4*>(tile + (f / C4) * TST + (f % C4) * 4) = sum[u];
    }
    __syncthreads();
  }
  tile_epilogue32<BM, BN>(a, blk, m0, n0, tile, red);
}

template <int BM, int BN, bool DGRAD, int KS, int ST, bool PAR, int NS, bool GEN>
__global__ __launch_bounds__(256, 2) void conv32_gemm_kernel(Conv32Args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  conv32_gemm_body<BM, BN, DGRAD, KS, ST, PAR, NS, GEN>(a, hw_blk(), smem);
}

// ---------------------------------------------------------------------------
// wgrad:  dW[co][j] = sum_m dY[m][co] * im2col(X)[m][j],  j = (r, s, c)
// Both operands are row-contiguous in memory: tiles [32 m][BM co] and
// [32 m][BN j], b32 fragment reads, MFMA (g, e) slot h reduces m = 8g + 4h + e.
// GEN: generic per-element pixel decomposition.  Fast path (Q divides 32 and
// the 32-pixel k-tile either divides P*Q or is a multiple of it, M % 32 == 0
// -- every ResNet-18 CIFAR layer): a k-tile's pixel m = kb + row splits into a
// scalar part (image n_s, output row oy_s: per-tile iterator) and a per-lane
// constant (row within the tile), so the im2col address of X is one add and
// its bounds test one compare per DMA.
template <int BM, int BN, int KS, int ST, int NS, bool GEN>
__device__ __forceinline__ void conv32_wgrad_body(const Conv32Args& a, const Blk& blk, uint8_t* smem,
                                                  float* __restrict__ dw, int atomic) {
  constexpr int A_BYTES = kBK * BM * 4;
  constexpr int STAGE = A_BYTES + kBK * BN * 4;
  constexpr int ARB = BM * 4, A_RPI = 1024 / ARB, A_CPR = ARB / 16;
  constexpr int BRB = BN * 4, B_RPI = 1024 / BRB, B_CPR = BRB / 16;
  constexpr int ACH = BM * kBK / 1024, BCH = BN * kBK / 1024;
  constexpr int TM = BM / 64, TN = BN / 64;
  const ConvGeom& g = a.g;  // H,W,C = X; P,Q = dY spatial; Ng = Cout; K = R*S*C; M = N*P*Q
  const auto rsA = make_rsrc(a.src, a.src_bytes);  // dY
  const auto rsB = make_rsrc(a.wgt, a.wgt_bytes);  // X
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int i0 = blk.x * BM;
  const int j0 = blk.y * BN;
  const int kbeg = blk.z * a.kchunk;
  const int kend = min(g.M, kbeg + a.kchunk);
  const int nk = max(0, (kend - kbeg + kBK - 1) / kBK);

  const int a_co = i0 + (lane % A_CPR) * 4;
  const bool a_ok = a_co < g.Ng;
  const int jcol = j0 + (lane % B_CPR) * 4;
  const bool jok = jcol < g.K;
  const int rs = fdiv(jcol, a.dc);
  const int jc = jcol - rs * g.C;
  const int jr = rs / KS, js = rs - (rs / KS) * KS;
  const int PQ = g.P * g.Q;

  // fast path: lane-constant parts of both operand addresses
  int a_base[ACH], b_base[BCH], b_iy[BCH];
  bool b_ok[BCH];
  int n_s = 0, oy_s = 0;  // scalar pixel iterator of the tile start
  if constexpr (!GEN) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int row = (wave + 4 * i) * A_RPI + lane / A_CPR;
      a_base[i] = (row * g.Ng + a_co) * 4;
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int row = (wave + 4 * i) * B_RPI + lane / B_CPR;
      const int n_l = PQ >= kBK ? 0 : row / PQ;
      const int oy_l = (row % PQ) / g.Q, ox_l = row % g.Q;
      const int iy_l = oy_l * ST - g.pad + jr, ix = ox_l * ST - g.pad + js;
      b_iy[i] = iy_l;
      b_ok[i] = jok & (ix >= 0) & (ix < g.W);
      b_base[i] = (int)((((uint32_t)n_l * g.H + (uint32_t)iy_l) * g.W + (uint32_t)ix) * g.C + jc) * 4;
    }
    n_s = kbeg / PQ;  // scalar, once
    oy_s = (kbeg - n_s * PQ) / g.Q;
  }

  auto issue = [&](int kt, auto stc) {
    if constexpr (MFL_C32_DBG & 2) return;
    uint8_t* st = smem + decltype(stc)::value * STAGE;
    const int kb = kbeg + kt * kBK;
    if constexpr (!GEN) {
      const bool kv = kb < kend;
      const int aoff = kb * g.Ng * 4;
#pragma unroll
      for (int i = 0; i < ACH; ++i)
        dma16(rsA, (a_ok & kv) ? (uint32_t)(a_base[i] + aoff) : kOOB, st + (wave + 4 * i) * 1024);
      const int oys = oy_s * ST;
      const int boff = (n_s * g.H + oys) * g.W * g.C * 4;
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const bool ok = b_ok[i] & kv & ((uint32_t)(b_iy[i] + oys) < (uint32_t)g.H);
        dma16(rsB, ok ? (uint32_t)b_base[i] + (uint32_t)boff : kOOB, st + A_BYTES + (wave + 4 * i) * 1024);
      }
      // advance 32 pixels (selects, see the gemm kernel)
      const int big = PQ >= kBK;
      const int oy_n = oy_s + (big ? kBK / g.Q : 0);
      const int wrap = oy_n == g.P;
      oy_s = wrap ? 0 : oy_n;
      n_s += big ? wrap : kBK / PQ;
      return;
    } else {
#pragma unroll
      for (int i = 0; i < ACH; ++i) {
        const int m = kb + (wave + 4 * i) * A_RPI + lane / A_CPR;
        const uint32_t off = oob_or((m < kend) & a_ok, (uint32_t)(m * g.Ng + a_co) * 4u);
        dma16(rsA, off, st + (wave + 4 * i) * 1024);
      }
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const int m = kb + (wave + 4 * i) * B_RPI + lane / B_CPR;
        const int n = fdiv(m, a.dpq);
        const int rem = m - n * PQ;
        const int oy = fdiv(rem, a.dq);
        const int ox = rem - oy * g.Q;
        const int iy = oy * ST - g.pad + jr, ix = ox * ST - g.pad + js;
        const bool ok = (m < kend) & jok & (iy >= 0) & (iy < g.H) & (ix >= 0) & (ix < g.W);
        const uint32_t off = oob_or(ok, (uint32_t)(((n * g.H + iy) * g.W + ix) * g.C + jc) * 4u);
        dma16(rsB, off, st + A_BYTES + (wave + 4 * i) * 1024);
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  const int li = lane & 31, lh = lane >> 5;
  auto load = [&](const float* As, const float* Bs, int grp, f32x4* af, f32x4* bfr) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int kr = 8 * grp + 4 * lh + e;
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i][e] = As[kr * BM + wm * (BM / 2) + 32 * i + li];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j][e] = Bs[kr * BN + wn * (BN / 2) + 32 * j + li];
    }
  };
  f32x4 fa[2][kBK / 8][TM], fb[2][kBK / 8][TN];
  auto read = [&](auto stc, auto set) {
    constexpr int S = decltype(set)::value;
    const float* As = reinterpret_cast<const float*>(smem + decltype(stc)::value * STAGE);
    const float* Bs = reinterpret_cast<const float*>(smem + decltype(stc)::value * STAGE + A_BYTES);
#pragma unroll
    for (int grp = 0; grp < kBK / 8; ++grp) load(As, Bs, grp, fa[S][grp], fb[S][grp]);
  };
  auto mma = [&](auto set) {
    constexpr int S = decltype(set)::value;
    if constexpr (MFL_C32_DBG & 1) return;
    mma_tile<TM, TN, MFL_C32_BF16X3 != 0, MFL_C32_BF16X3 != 0>(fa[S], fb[S], acc);  // A = dY, B = X (both packed)
    interleave_mfma<kTileMfma<TM, TN>, kTileValu>();
    __builtin_amdgcn_sched_barrier(0);
  };
  ring_loop<NS, ACH + BCH>(nk, issue, read, mma);

  // epilogue straight from the accumulators: each register store covers two
  // 128-B row segments (the full-rate atomic shape, MI355X_MICROARCH.md)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = j0 + wn * (BN / 2) + 32 * j + li;
      if (col >= g.K) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = i0 + wm * (BM / 2) + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * lh;
        if (co >= g.Ng) continue;
        float* p = dw + (int64_t)co * g.K + col;
        if (atomic) atomicAdd(p, acc[i][j][e]);
        else *p = acc[i][j][e];
      }
    }
}

template <int BM, int BN, int KS, int ST, int NS, bool GEN>
__global__ __launch_bounds__(256, 2) void conv32_wgrad_kernel(Conv32Args a, float* __restrict__ dw, int atomic) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  conv32_wgrad_body<BM, BN, KS, ST, NS, GEN>(a, hw_blk(), smem, dw, atomic);
}

// A layer's backward in ONE launch: blocks [0, nd) run the dgrad GEMM (with
// its fused consumer-BN reductions), the rest the wgrad GEMM.  Both read dY,
// neither waits for the other; as two launches each is a few hundred
// workgroups whose tail waves leave CUs idle and the second pays a launch
// boundary.  dgrad blocks first: it is on the critical path (the bf16
// twin measured dgrad-first / wgrad-first / alternating 502 / 551 / 508 ms).
// A downsampling block's conv1 (3x3 / stride 2) and projection shortcut
// (1x1 / stride 2) read the same x: one launch, blocks [0, n1) conv1.
template <int NS>
__global__ __launch_bounds__(256, 2) void conv32_fwd_pair_kernel(Conv32Args a1, Conv32Args a2, int n1, int g1x,
                                                                 int g1y, int g2x, int g2y, int g2z) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int b = xcd_group(blockIdx.x, gridDim.x);
  if (b < n1) {
    const Blk k{b % g1x, (b / g1x) % g1y, b / (g1x * g1y), g1x, g1y, n1 / (g1x * g1y)};
    conv32_gemm_body<64, 64, false, 3, 2, false, NS, false>(a1, k, smem);
  } else {
    const int w = b - n1;
    const Blk k{w % g2x, (w / g2x) % g2y, w / (g2x * g2y), g2x, g2y, g2z};
    conv32_gemm_body<64, 64, false, 1, 2, false, NS, false>(a2, k, smem);
  }
}

// DBM: the dgrad's pixel tile (64, or 128 -- half the W^T re-reads per
// output pixel; MFL_C32_PAIR_DBM, stride-1 pairs)
template <int KS, int ST, bool PAR, int NS, int DBM = 64>
__global__ __launch_bounds__(256, 2) void conv32_bwd_pair_kernel(Conv32Args ad, Conv32Args aw, float* __restrict__ dw,
                                                                 int atomic, int nd, int gdx, int gdy, int gwx,
                                                                 int gwy, int gwz, OptTail ot) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int b = xcd_group(blockIdx.x, gridDim.x);
  const int nconv = (int)gridDim.x - ot.nblk;
  if (b >= nconv) {  // optimizer tail (dispatched last: it fills the GEMMs' tail)
    opt_tail_body(ot, b - nconv);
    return;
  }
  if (b < nd) {
    const Blk k{b % gdx, (b / gdx) % gdy, b / (gdx * gdy), gdx, gdy, nd / (gdx * gdy)};
    conv32_gemm_body<DBM, 64, true, KS, ST, PAR, NS, false>(ad, k, smem);
  } else {
    const int w = b - nd;
    const Blk k{w % gwx, (w / gwx) % gwy, w / (gwx * gwy), gwx, gwy, gwz};
    conv32_wgrad_body<64, 64, KS, ST, NS, false>(aw, k, smem, dw, atomic);
  }
}

// ---------------------------------------------------------------------------
// host side
uint32_t range_bytes(int64_t elems) {
  const int64_t b = elems * 4;
  return b >= 0x7FFFFFF0LL ? 0x7FFFFFF0u : (uint32_t)b;
}
int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}
int cdiv(int a, int b) { return (a + b - 1) / b; }

template <typename K>
void set_lds(K* kernel, size_t lds) {
  if (lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
}

// LDS ring depth per tile shape: 64x64 workgroups run two per CU (4 stages =
// 64 KiB each), the larger tiles one per CU with the deepest ring that fits
// 160 KiB.  Measured: with 3 stages every conv ran at ~45% of the fp32 MFMA
// peak -- the k-tiles waited for their LDS-DMA (latency-bound: 2 x 16 KiB in
// flight per workgroup cannot cover ~1-2 us at 38 GB/s per CU).
#ifndef MFL_C32_NS
#define MFL_C32_NS 3
#endif
constexpr int stages_for(int bm, int bn) {
  return (156 * 1024) / ((bm + bn) * kRowB) > MFL_C32_NS ? MFL_C32_NS : (156 * 1024) / ((bm + bn) * kRowB);
}

size_t gemm_lds(int bm, int bn) {
  const size_t ring = (size_t)stages_for(bm, bn) * (bm + bn) * kRowB;
  const size_t epi = (size_t)bm * (bn + 4) * 4 + 256 * 8 * 4 + 16;
  return ring > epi ? ring : epi;
}

template <int BM, int BN, bool DG, int KS, int ST, bool PAR, bool GEN>
void launch_t2(const Conv32Args& a, dim3 grid, hipStream_t s) {
  constexpr int NS = stages_for(BM, BN);
  static bool init = false;
  const size_t lds = gemm_lds(BM, BN);
  if (!init) {
    set_lds(&conv32_gemm_kernel<BM, BN, DG, KS, ST, PAR, NS, GEN>, lds);
    init = true;
  }
  conv32_gemm_kernel<BM, BN, DG, KS, ST, PAR, NS, GEN><<<grid, 256, lds, s>>>(a);
}
// the fast address path needs every k-tile inside one filter tap
template <int BM, int BN, bool DG, int KS, int ST, bool PAR>
void launch_t(const Conv32Args& a, dim3 grid, hipStream_t s) {
  if constexpr (DG && ST > 1 && !PAR) {
    launch_t2<BM, BN, DG, KS, ST, PAR, true>(a, grid, s);
  } else {
    if (a.g.C % kBK == 0 && a.kchunk % kBK == 0 && !(MFL_C32_GENERIC))
      launch_t2<BM, BN, DG, KS, ST, PAR, false>(a, grid, s);
    else
      launch_t2<BM, BN, DG, KS, ST, PAR, true>(a, grid, s);
  }
}

template <int BM, int BN, bool DG>
void launch_geom(const Conv32Args& a, dim3 grid, hipStream_t s) {
  const ConvGeom& g = a.g;
  const bool par = a.par_mc != 0;
  if (g.R == 3 && g.stride == 1) launch_t<BM, BN, DG, 3, 1, false>(a, grid, s);
  else if (g.R == 1 && g.stride == 1) launch_t<BM, BN, DG, 1, 1, false>(a, grid, s);
  else if (g.R == 3 && g.stride == 2) {
    if (DG && par) launch_t<BM, BN, DG, 3, 2, true>(a, grid, s);
    else launch_t<BM, BN, DG, 3, 2, false>(a, grid, s);
  } else if (g.R == 1 && g.stride == 2) {
    if (DG && par) launch_t<BM, BN, DG, 1, 2, true>(a, grid, s);
    else launch_t<BM, BN, DG, 1, 2, false>(a, grid, s);
  }
}

// Plan: pick (BM, BN, split) minimising a throughput model of the fp32 matrix
// pipe.  A workgroup of a BMxBN tile over kt k-tiles keeps its CU's 4 SIMDs
// busy for BM*BN*kt*32*2 / 256 cycles; 64x64 tiles run 2 workgroups per CU.
// Costs added: the pipeline fill + epilogue per workgroup, and for split-K
// the last arriver's serial slab reads (~100 GB/s per workgroup).
struct Cand {
  int bm, bn;
};
// (128x128 needs 2 x 8 x 4 fragment registers per operand and tile row at
// kBK = 64 -- beyond the register budget of the double-buffered loop)
constexpr Cand kCands[] = {{64, 64}, {128, 64}, {64, 128}};

}  // namespace

int conv32_counter_slots(const ConvGeom& g, const ConvPlan& p) {
  return cdiv(g.M, p.bm) * cdiv(g.Ng, p.bn);
}

// Measured plans (scripts/conv32_bench.py --sweep, profiles/r2/c32_sweep_v2.log)
// for the flagship shapes -- ResNet-18 on CIFAR-10 at batch 32 -- where the
// throughput model below picks a plan >= 5% slower than the best one (it
// over-prefers 128x64 tiles for dgrad / wgrad and splits 1x1 convs that are
// latency-bound).  Keyed on the ORIGINAL convolution (dgrad geometry is role
// swapped), like a vendor library's performance database.
struct TunedPlan {
  int mode, n, h, w, c, co, r, stride, bm, bn, splits;
};
#if MFL_C32_BF16X3
// profiles/r2/c32x3_sweep.log; dgrad / wgrad stay 64x64 where that lets the
// layer's backward run as one paired launch.  Re-swept with pre-split (packed)
// operands (profiles/r2/xpack/c32x3_packed_sweep.log): stand-alone, the 32x32
// forward then prefers 64x64 tiles (15.8 vs 17.4 us) and one wgrad 1 split,
// but inside the step neither moved (forward 17.2 vs 17.35 us per call,
// profiles/r2/xpack/retune_negative/), so the table is unchanged.
constexpr TunedPlan kTuned[] = {
    {0, 32, 32, 32, 8, 64, 3, 1, 64, 64, 1},    {0, 32, 32, 32, 64, 64, 3, 1, 128, 64, 1},
    {0, 32, 32, 32, 64, 128, 3, 2, 64, 64, 1},  {0, 32, 16, 16, 128, 128, 3, 1, 64, 64, 2},
    {0, 32, 16, 16, 128, 256, 3, 2, 64, 64, 4}, {0, 32, 8, 8, 256, 256, 3, 1, 64, 64, 4},
    {0, 32, 8, 8, 256, 512, 3, 2, 64, 64, 4},   {0, 32, 4, 4, 512, 512, 3, 1, 64, 64, 8},
    {1, 32, 32, 32, 64, 64, 3, 1, 64, 64, 1},   {1, 32, 32, 32, 64, 128, 3, 2, 64, 64, 1},
    // 16x16x128 backward pair: dgrad 2 x wgrad 7 slices = 764 workgroups, one
    // wave of 3 per CU, instead of 3 x 14 = 1,272 (1.66 waves) -- whole-step
    // sweep with MFL_C32_PLANS, profiles/r4/plans/: -1.4 % per update
    // 4x4x512 dgrad 4 slices (832 workgroups with its wgrad) and 8x8x256
    // wgrad 2 (800 with its dgrad), instead of 8 / 3: neutral for one learner
    // (1.048 / 1.049 vs 1.045 / 1.050 ms), -0.7 % per update with 8 co-located
    // learners on the 2-stage pair ring (0.690 / 0.689 -> 0.685 / 0.685 ms,
    // profiles/r4/ns/tq_*.log)
    {1, 32, 32, 32, 64, 128, 1, 2, 64, 64, 1},  {1, 32, 16, 16, 128, 128, 3, 1, 64, 64, 2},
    {1, 32, 16, 16, 128, 256, 3, 2, 64, 64, 3}, {1, 32, 8, 8, 256, 256, 3, 1, 64, 64, 4},
    {1, 32, 8, 8, 256, 512, 3, 2, 64, 64, 4},   {1, 32, 4, 4, 512, 512, 3, 1, 64, 64, 4},
    {2, 32, 16, 16, 128, 128, 3, 1, 64, 64, 7}, {2, 32, 16, 16, 128, 256, 3, 2, 64, 64, 7},
    {2, 32, 8, 8, 256, 256, 3, 1, 64, 64, 2},   {2, 32, 8, 8, 256, 512, 3, 2, 64, 64, 2},
    {2, 32, 4, 4, 512, 512, 3, 1, 64, 64, 1},
};
#else
constexpr TunedPlan kTuned[] = {
    {0, 32, 8, 8, 256, 256, 3, 1, 64, 64, 4},   {0, 32, 8, 8, 256, 512, 1, 2, 64, 64, 1},
    {1, 32, 32, 32, 64, 64, 3, 1, 64, 64, 1},   {1, 32, 32, 32, 64, 128, 3, 2, 64, 64, 1},
    {1, 32, 32, 32, 64, 128, 1, 2, 64, 64, 1},  {1, 32, 8, 8, 256, 256, 3, 1, 64, 64, 4},
    {2, 32, 8, 8, 256, 256, 3, 1, 64, 64, 3},   {2, 32, 8, 8, 256, 512, 3, 2, 64, 64, 2},
    {2, 32, 4, 4, 512, 512, 3, 1, 64, 64, 2},
};
#endif
// MFL_C32_PLANS="mode,h,c,co,r,stride,splits;..." overrides the split-K
// factor of matching shapes (64x64 tiles; batch-size independent) -- for
// sweeps of whole-step plans, where a paired launch's total workgroup count
// (waves of 3 per CU) matters more than each GEMM's stand-alone optimum.
struct PlanOverride {
  int mode, h, c, co, r, stride, splits;
};
static std::vector<PlanOverride> parse_plan_overrides(const std::string& str) {
  std::vector<PlanOverride> out;
  size_t pos = 0;
  while (pos < str.size()) {
    size_t end = str.find(';', pos);
    if (end == std::string::npos) end = str.size();
    PlanOverride o{};
    if (std::sscanf(str.substr(pos, end - pos).c_str(), "%d,%d,%d,%d,%d,%d,%d", &o.mode, &o.h, &o.c, &o.co, &o.r,
                    &o.stride, &o.splits) == 7)
      out.push_back(o);
    pos = end + 1;
  }
  return out;
}
// the environment's overrides win over the regime set at run time
// (set_conv32_plan_overrides: the co-located learners' plans)
static std::vector<PlanOverride> g_rt_overrides;
static thread_local bool g_ignore_rt = false;  // plan_conv32_table: the table / model plan alone
static const std::vector<PlanOverride>& plan_overrides() {
  static const char* env = std::getenv("MFL_C32_PLANS");
  static const std::vector<PlanOverride> v = env ? parse_plan_overrides(env) : std::vector<PlanOverride>{};
  static const std::vector<PlanOverride> none;
  return env ? v : (g_ignore_rt ? none : g_rt_overrides);
}

static void tuned_plan(const ConvGeom& g, int mode, int& bm, int& bn, int& sp) {
  const bool dg = mode == 1;
  const int h = dg ? g.P : g.H, w = dg ? g.Q : g.W, c = dg ? g.Ng : g.C, co = dg ? g.C : g.Ng;
  for (const PlanOverride& o : plan_overrides())
    if (o.mode == mode && o.h == h && o.c == c && o.co == co && o.r == g.R && o.stride == g.stride) {
      bm = bn = 64;
      sp = o.splits;
      return;
    }
  for (const TunedPlan& t : kTuned)
    if (t.mode == mode && t.n == g.N && t.h == h && t.w == w && t.c == c && t.co == co && t.r == g.R &&
        t.stride == g.stride) {
      bm = t.bm;
      bn = t.bn;
      sp = t.splits;
      return;
    }
}

static ConvPlan plan_conv32_impl(const ConvGeom& g, int mode, bool allow_par, bool use_table) {
  const int rows = mode == 2 ? g.Ng : g.M;
  const int cols = mode == 2 ? g.K : g.Ng;
  int kred = mode == 2 ? g.M : g.K;
  bool par = false;
  if (allow_par && mode == 1 && g.stride == 2 && (g.P % 2 == 0) && (g.Q % 2 == 0)) {
    par = true;
    kred = ((g.R + 1) / 2) * ((g.S + 1) / 2) * g.C;  // the largest parity class
  }
  int fb = env_int("MFL_C32_BM", 0), fn = env_int("MFL_C32_BN", 0), fs = env_int("MFL_C32_SPLIT", 0);
  // CU slots one launch can count on: 256 (the whole chip) for one learner;
  // fewer when co-located learners' launches share the CUs (MFL_C32_SLOTS,
  // A/B runs).  The measured plan table assumes the whole chip.
  const int slots_env = env_int("MFL_C32_SLOTS", 256);
  if (use_table && !fb && !fn && !fs && slots_env == 256) tuned_plan(g, mode, fb, fn, fs);
  const double clk = 2.4e3;  // cycles per us
  ConvPlan best;
  double best_t = 1e30;
  const int nkt_all = cdiv(kred, kBK);
  // a forced slice count (table, MFL_C32_PLANS, MFL_C32_SPLIT) snaps to the
  // feasible count it implies: equal k-tile shares, no empty slice (an
  // infeasible request used to leave the plan without a tile)
  if (fs > 0) fs = cdiv(nkt_all, cdiv(nkt_all, std::min(fs, nkt_all)));
  for (const Cand& c : kCands) {
    if (fb && c.bm != fb) continue;
    if (fn && c.bn != fn) continue;
    if (par && ((g.N * (g.P / 2) * (g.Q / 2)) % c.bm)) continue;
    const int tiles = cdiv(rows, c.bm) * cdiv(cols, c.bn);
    const int occ = 1;  // a 64-deep ring of >= 3 stages fills most of a CU's LDS
    const int slots = slots_env * occ;
    for (int sp = 1; sp <= 64 && sp <= nkt_all; ++sp) {
      if (fs && sp != fs) continue;
      const int kt = cdiv(nkt_all, sp);
      const int s_eff = cdiv(nkt_all, kt);
      if (s_eff != sp) continue;
      if (mode != 2 && s_eff > 1 && tiles > 1024) continue;  // counter block size
      const int nwg = tiles * s_eff;
      // split mode: VALU-paced (the operand splits), ~0.6x (64x64) / ~0.47x
      // (larger wave tiles reuse each split) of the fp32-MFMA time
      const double pace = MFL_C32_BF16X3 ? (c.bm == 64 && c.bn == 64 ? 0.6 : 0.47) : 1.0;
      const double t_alone = pace * c.bm * c.bn * kt * kBK * 2 / 256.0 / clk + 1.2;
      const int full = nwg / slots, rem = nwg % slots;
      double tt = full * occ * t_alone + (rem ? (rem > slots_env ? occ : 1) * t_alone : 0.0);
      if (s_eff > 1) {
        if (mode == 2) tt += (double)tiles * s_eff * c.bm * c.bn * 4 / 1.3e6;  // atomic bytes at 1.3 TB/s
        else tt += (double)s_eff * c.bm * c.bn * 4 / 1.0e5 + 1.0;              // serial slab reduce
      }
      if (tt < best_t - 1e-9) {
        best_t = tt;
        best.bm = c.bm;
        best.bn = c.bn;
        best.splits = s_eff;
        best.kchunk = kt * kBK;
      }
    }
  }
  best.stats_rows = mode == 0 ? 1 : 0;
  best.bk = kBK;
  best.stages = stages_for(best.bm, best.bn);
  best.par_mc = par && mode == 1 ? g.N * (g.P / 2) * (g.Q / 2) : 0;
  if (best_t >= 1e30) best.kchunk = 0;  // no feasible tile
  return best;
}

ConvPlan plan_conv32_table(const ConvGeom& g, int mode) {
  g_ignore_rt = true;
  const ConvPlan p = plan_conv32(g, mode);
  g_ignore_rt = false;
  return p;
}

ConvPlan plan_conv32(const ConvGeom& g, int mode) {
  // parity-class dgrad needs class sizes that are whole tiles; otherwise the
  // masked stride-aware gather
  ConvPlan p = plan_conv32_impl(g, mode, true, true);
  if (p.kchunk == 0) p = plan_conv32_impl(g, mode, false, true);
  // a split the table / overrides force can be infeasible at another batch
  // size (the overrides are batch independent: the co-located regime's 2-way
  // 8x8x256 dgrad split has 2,048 tiles at batch 512, past the counter block
  // of an in-launch split-K reduce) -- then the throughput model decides
  if (p.kchunk == 0) p = plan_conv32_impl(g, mode, true, false);
  if (p.kchunk == 0) p = plan_conv32_impl(g, mode, false, false);
  return p;
}

static FastDiv make_fdiv(int d) {
  FastDiv f{0u, 0, 0u};
  if (d <= 1) {
    f.id = 0xFFFFFFFFu;
    return f;
  }
  int s = 0;
  while ((1LL << s) < d) ++s;
  f.m = (uint32_t)(((1ULL << (31 + s)) + (uint64_t)d - 1) / (uint64_t)d);
  f.sh = s - 1;
  return f;
}

static void fill_shifts(Conv32Args& a) {
  a.dc = make_fdiv(a.g.C);
  a.dq = make_fdiv(a.g.Q);
  a.dpq = make_fdiv(a.g.P * a.g.Q);
}

static Conv32Args gemm_args(const ConvGeom& g, bool dgrad, const ConvPlan& p, const float* src, const float* wgt,
                            float* y, float* ysplit, int* counters, double* stats, bool accum,
                            const BnBwdFusion32* bnb, int stats_reps) {
  Conv32Args a{};
  a.g = g;
  a.src = src;
  a.wgt = wgt;
  a.y = y;
  a.ysplit = ysplit;
  a.counters = counters;
  a.stats = dgrad ? nullptr : stats;
  if (bnb && bnb->acc) {
    a.bn_z = bnb->z;
    a.bn_y = bnb->y;
    a.bn_mean = bnb->mean;
    a.bn_invstd = bnb->invstd;
    a.bn_acc = bnb->acc;
  }
  a.reps = (bnb && bnb->acc) ? (bnb->reps > 0 ? bnb->reps : 1) : (stats_reps > 0 ? stats_reps : 1);
  a.src_bytes = range_bytes((int64_t)g.N * g.H * g.W * g.C);
  a.wgt_bytes = range_bytes((int64_t)g.K * g.Ng);
  a.kchunk = p.kchunk;
  a.accum = accum ? 1 : 0;
  a.par_mc = dgrad ? p.par_mc : 0;
  fill_shifts(a);
  return a;
}

void launch_conv32_gemm(const ConvGeom& g, bool dgrad, const ConvPlan& p, const float* src, const float* wgt,
                        float* y, float* ysplit, int* counters, double* stats, bool accum,
                        const BnBwdFusion32* bnb, hipStream_t s, int stats_reps) {
  const Conv32Args a = gemm_args(g, dgrad, p, src, wgt, y, ysplit, counters, stats, accum, bnb, stats_reps);
  const dim3 grid(cdiv(g.M, p.bm), cdiv(g.Ng, p.bn), p.splits);
  const int key = p.bm * 1000 + p.bn;
  switch (key) {
    case 64064: dgrad ? launch_geom<64, 64, true>(a, grid, s) : launch_geom<64, 64, false>(a, grid, s); break;
    case 128064: dgrad ? launch_geom<128, 64, true>(a, grid, s) : launch_geom<128, 64, false>(a, grid, s); break;
    default: dgrad ? launch_geom<64, 128, true>(a, grid, s) : launch_geom<64, 128, false>(a, grid, s); break;
  }
}

namespace {
bool wgrad_fast(const ConvGeom& g, int kchunk) {
  const int pq = g.P * g.Q;
  return g.Q > 0 && kBK % g.Q == 0 && (pq % kBK == 0 || kBK % pq == 0) && g.M % kBK == 0 && kchunk % kBK == 0 &&
         !(MFL_C32_GENERIC);
}

template <int BM, int BN, int KS, int ST, bool GEN>
void launch_w2(const Conv32Args& a, dim3 grid, float* dw, int atomic, hipStream_t s) {
  constexpr int NS = stages_for(BM, BN);
  static bool init = false;
  const size_t lds = (size_t)NS * kBK * (BM + BN) * 4;
  if (!init) {
    set_lds(&conv32_wgrad_kernel<BM, BN, KS, ST, NS, GEN>, lds);
    init = true;
  }
  conv32_wgrad_kernel<BM, BN, KS, ST, NS, GEN><<<grid, 256, lds, s>>>(a, dw, atomic);
}
// fast path: Q | 32, the 32-pixel k-tile divides P*Q or is a multiple of it
template <int BM, int BN, int KS, int ST>
void launch_w(const Conv32Args& a, dim3 grid, float* dw, int atomic, hipStream_t s) {
  if (wgrad_fast(a.g, a.kchunk)) launch_w2<BM, BN, KS, ST, false>(a, grid, dw, atomic, s);
  else launch_w2<BM, BN, KS, ST, true>(a, grid, dw, atomic, s);
}
template <int BM, int BN>
void launch_w_geom(const Conv32Args& a, dim3 grid, float* dw, int atomic, hipStream_t s) {
  const ConvGeom& g = a.g;
  if (g.R == 3 && g.stride == 1) launch_w<BM, BN, 3, 1>(a, grid, dw, atomic, s);
  else if (g.R == 3 && g.stride == 2) launch_w<BM, BN, 3, 2>(a, grid, dw, atomic, s);
  else if (g.R == 1 && g.stride == 1) launch_w<BM, BN, 1, 1>(a, grid, dw, atomic, s);
  else launch_w<BM, BN, 1, 2>(a, grid, dw, atomic, s);
}
}  // namespace

static Conv32Args wgrad_args(const ConvGeom& g, const ConvPlan& p, const float* x, const float* dy) {
  Conv32Args a{};
  a.g = g;
  a.src = dy;
  a.wgt = x;
  a.src_bytes = range_bytes((int64_t)g.M * g.Ng);
  a.wgt_bytes = range_bytes((int64_t)g.N * g.H * g.W * g.C);
  a.kchunk = p.kchunk;
  fill_shifts(a);
  return a;
}

void launch_conv32_wgrad(const ConvGeom& g, const ConvPlan& p, const float* x, const float* dy, float* dw,
                         bool accumulate, hipStream_t s) {
  const Conv32Args a = wgrad_args(g, p, x, dy);
  const dim3 grid(cdiv(g.Ng, p.bm), cdiv(g.K, p.bn), p.splits);
  const int atomic = (accumulate || p.splits > 1) ? 1 : 0;
  const int key = p.bm * 1000 + p.bn;
  switch (key) {
    case 64064: launch_w_geom<64, 64>(a, grid, dw, atomic, s); break;
    case 128064: launch_w_geom<128, 64>(a, grid, dw, atomic, s); break;
    default: launch_w_geom<64, 128>(a, grid, dw, atomic, s); break;
  }
}

// Pair ring depth (set_conv32_pair_ring): the throughput regime (4-8
// co-located learners, models/colocated.py) trades the third ring stage for
// a fourth resident workgroup per CU -- 0.693 / 0.696 -> 0.689 / 0.690 ms per
// update with 8 learners when every conv32 kernel ran 2 stages, while one
// learner (latency-bound) went 1.027 -> 1.071 (profiles/r4/ns/).  Only the
// bf16x3 build carries the 2-stage pair instantiations.
int g_pair_ns = 0;
void set_conv32_pair_ring(int ns) { g_pair_ns = ns; }
void set_conv32_plan_overrides(const char* spec) { g_rt_overrides = parse_plan_overrides(spec ? spec : ""); }
size_t gemm_lds_ns(int bm, int bn, int ns) {  // ring of ns stages or the gemm epilogue, whichever is larger
  return std::max((size_t)ns * (bm + bn) * kRowB, (size_t)bm * (bn + 4) * 4 + 256 * 8 * 4 + 16);
}
size_t pair_lds(int ns) {  // ring of ns 64x64 stages or the gemm epilogue, whichever is larger
  return std::max((size_t)ns * (64 + 64) * kRowB, (size_t)64 * (64 + 4) * 4 + 256 * 8 * 4 + 16);
}
bool pair_ring2() {
  return MFL_C32_BF16X3 && stages_for(64, 64) > 2 && (g_pair_ns ? g_pair_ns : env_int("MFL_C32_PAIR_NS", 0)) == 2;
}

bool launch_conv32_bwd_pair(const ConvGeom& gd, const ConvPlan& pd, const ConvGeom& gf, const ConvPlan& pw,
                            const float* dy, const float* w, float* dx, float* ysplit, int* counters, bool accum,
                            const BnBwdFusion32* bnb, const float* x, float* dw, hipStream_t s,
                            const OptTail* ot) {
  if (env_int("MFL_C32_PAIR", 1) == 0) return false;
  const bool par = pd.par_mc != 0;
  if (pd.bm != 64 || pd.bn != 64 || pw.bm != 64 || pw.bn != 64) return false;
  if (gd.C % kBK != 0 || pd.kchunk % kBK != 0 || (MFL_C32_GENERIC)) return false;  // dgrad fast path
  if (gd.stride > 1 && !par) return false;
  if (!wgrad_fast(gf, pw.kchunk)) return false;
  const Conv32Args ad = gemm_args(gd, true, pd, dy, w, dx, ysplit, counters, nullptr, accum, bnb, 1);
  const Conv32Args aw = wgrad_args(gf, pw, x, dy);
  // a 128-pixel dgrad tile (stride-1 pairs, MFL_C32_PAIR_DBM=128): half the
  // workgroups re-read the layer's W^T tile
  const int dbm = (gd.stride == 1 && gd.M % 128 == 0 && env_int("MFL_C32_PAIR_DBM", 64) == 128) ? 128 : 64;
  const int gdx = cdiv(gd.M, dbm), gdy = cdiv(gd.Ng, 64), nd = gdx * gdy * pd.splits;
  const int gwx = cdiv(gf.Ng, 64), gwy = cdiv(gf.K, 64), gwz = pw.splits;
  const OptTail tail = ot ? *ot : OptTail{};
  const int nblk = nd + gwx * gwy * gwz + tail.nblk;
  constexpr int NS = stages_for(64, 64);
  constexpr int NS2 = MFL_C32_BF16X3 && NS > 2 ? 2 : NS;
  const bool r2 = pair_ring2();
  const size_t lds = dbm == 128 ? std::max(pair_lds(r2 ? NS2 : NS), gemm_lds_ns(128, 64, r2 ? NS2 : NS))
                                : pair_lds(r2 ? NS2 : NS);
  // dw is zero on entry (the step's gradient buffer): an unsplit weight
  // gradient (ResNet-18's 512-channel stage) owns every element it writes, so
  // it stores instead of adding atomically (MFL_C32_WSTORE=0: always atomics)
  const int wg_atomic = (pw.splits > 1 || env_int("MFL_C32_WSTORE", 1) == 0) ? 1 : 0;
  auto go = [&](auto kern) {
    static_assert(NS >= 2, "ring");
    if (lds > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    kern<<<nblk, 256, lds, s>>>(ad, aw, dw, wg_atomic, nd, gdx, gdy, gwx, gwy, gwz, tail);
  };
  if (gd.R == 3 && gd.stride == 1 && dbm == 128)
    r2 ? go(conv32_bwd_pair_kernel<3, 1, false, NS2, 128>) : go(conv32_bwd_pair_kernel<3, 1, false, NS, 128>);
  else if (gd.R == 3 && gd.stride == 1) r2 ? go(conv32_bwd_pair_kernel<3, 1, false, NS2>) : go(conv32_bwd_pair_kernel<3, 1, false, NS>);
  else if (gd.R == 1 && gd.stride == 1 && dbm == 128)
    r2 ? go(conv32_bwd_pair_kernel<1, 1, false, NS2, 128>) : go(conv32_bwd_pair_kernel<1, 1, false, NS, 128>);
  else if (gd.R == 1 && gd.stride == 1) r2 ? go(conv32_bwd_pair_kernel<1, 1, false, NS2>) : go(conv32_bwd_pair_kernel<1, 1, false, NS>);
  else if (gd.R == 3 && gd.stride == 2) r2 ? go(conv32_bwd_pair_kernel<3, 2, true, NS2>) : go(conv32_bwd_pair_kernel<3, 2, true, NS>);
  else if (gd.R == 1 && gd.stride == 2) r2 ? go(conv32_bwd_pair_kernel<1, 2, true, NS2>) : go(conv32_bwd_pair_kernel<1, 2, true, NS>);
  else return false;
  return true;
}

bool launch_conv32_fwd_pair(const ConvGeom& g1, const ConvPlan& p1, const float* w1, float* y1, float* ys1,
                            int* c1, double* st1, int reps1, const ConvGeom& g2, const ConvPlan& p2,
                            const float* w2, float* y2, float* ys2, int* c2, double* st2, int reps2,
                            const float* x, hipStream_t s) {
  if (env_int("MFL_C32_PAIR", 1) == 0) return false;
  if (p1.bm != 64 || p1.bn != 64 || p2.bm != 64 || p2.bn != 64) return false;
  if (g1.R != 3 || g1.stride != 2 || g2.R != 1 || g2.stride != 2) return false;
  if (g1.C % kBK != 0 || p1.kchunk % kBK != 0 || p2.kchunk % kBK != 0 || (MFL_C32_GENERIC)) return false;
  const Conv32Args a1 = gemm_args(g1, false, p1, x, w1, y1, ys1, c1, st1, false, nullptr, reps1);
  const Conv32Args a2 = gemm_args(g2, false, p2, x, w2, y2, ys2, c2, st2, false, nullptr, reps2);
  const int g1x = cdiv(g1.M, 64), g1y = cdiv(g1.Ng, 64), n1 = g1x * g1y * p1.splits;
  const int g2x = cdiv(g2.M, 64), g2y = cdiv(g2.Ng, 64), g2z = p2.splits;
  constexpr int NS = stages_for(64, 64);
  constexpr int NS2 = MFL_C32_BF16X3 && NS > 2 ? 2 : NS;
  const bool r2 = pair_ring2();
  const size_t lds = pair_lds(r2 ? NS2 : NS);
  const int nblk = n1 + g2x * g2y * g2z;
  if (r2) conv32_fwd_pair_kernel<NS2><<<nblk, 256, lds, s>>>(a1, a2, n1, g1x, g1y, g2x, g2y, g2z);
  else conv32_fwd_pair_kernel<NS><<<nblk, 256, lds, s>>>(a1, a2, n1, g1x, g1y, g2x, g2y, g2z);
  return true;
}

}  // namespace MFL_C32_VARIANT
}  // namespace mfl
