// K6b (fp32, bf16x3 products): halo-tiled 3x3 / stride-1 convolution whose
// operand fill applies the PRODUCER's BatchNorm (+ residual, + ReLU).
//
// Why (profiles/ANALYSIS.md, round 2): the im2col conv32 kernels stream every
// operand tile through LDS-DMA once per filter tap -- ~150 MB of L2 traffic
// per 2.4-GFLOP layer -- and every BatchNorm apply is its own ~6 us launch
// (37 per step), because an LDS-DMA fill has no register pass to transform
// through.  Here a workgroup owns a spatial output tile (TH x TW pixels of
// IMGS images) and NT output channels; per 16-channel chunk it loads the
// input patch WITH its 1-pixel halo once, through registers:
//
//   v = relu?(z * sc + sh [+ residual]),   v -> bf16 hi + lo  ->  LDS
//
// and the 9 taps read shifted windows of that one LDS image.  Operand bytes
// per conv drop ~3-4x (the halo patch is read once per output-channel tile,
// not 9 times), the split of fp32 into bf16 hi / lo happens once per element
// (the k-loop has no decode VALU at all: fragments are read as ready bf16x8),
// and the BatchNorm apply launches disappear: the first output-channel tile
// of the workgroup that owns a pixel writes the activation (fp32 y + packed
// hi|lo yp) that the backward pass and later residual adds read.
//
// Products: acc += Ahi*Bhi + Ahi*Blo + Alo*Bhi on v_mfma_f32_32x32x16_bf16,
// fp32 accumulation -- the same split and product set as conv32.hip's c32s
// variant (~4e-6 relative per convolution); the transform is bit-identical to
// bn32_apply (fmaf(z, sc, sh) + residual, max 0, coefficients in fp64).
//
// Layout (per 16-channel chunk, double-buffered):
//   A: [img][py][px] patch pixels, PS bytes each: hi ch0-7 | hi ch8-15 |
//      lo ch0-7 | lo ch8-15 (+ pad).  Row / image pitches ROWB / IMGB are
//      chosen (scripts/hconv_banks.py) so every ds_read_b128 lane group of
//      every tap window hits 16 distinct 16-B bank slots.
//   B: [tap][co] 80-B rows (the same 64 B + 16 B pad): conflict-free for 32
//      consecutive output channels.
// MFMA: rows = pixels (lane li = row, lane half h = channels 8h..8h+7),
// cols = output channels; waves tile the workgroup WGM x WGN.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "kernels/common.h"
#include "kernels/hconv.h"
#include "kernels/lds_tiles.h"

namespace mfl {
namespace hc {

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16v2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t cvt_pk_bf16(f32x2 v) {  // one v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16v2));
}
// (a, b) -> hi pair (RNE) and lo pair (RNE of the exact remainder): the
// split_pack encoding of common.h, two values at a time
__device__ __forceinline__ void split2(float a, float b, uint32_t& h, uint32_t& l) {
  h = cvt_pk_bf16(f32x2{a, b});
  l = cvt_pk_bf16(f32x2{a, b} - f32x2{__uint_as_float(h << 16), __uint_as_float(h & 0xffff0000u)});
}

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

template <int TH_, int TW_, int IMGS_, int NT_, int WGM_, int WGN_, int PS_, int ROWB_, int IMGB_>
struct Cfg {
  static constexpr int TH = TH_, TW = TW_, IMGS = IMGS_, NT = NT_, WGM = WGM_, WGN = WGN_;
  static constexpr int NTHR = 64 * WGM * WGN;  // 8 waves: two per SIMD hide each other's waits
  static constexpr int MT = IMGS * TH * TW;  // output pixels per workgroup
  static constexpr int WM = MT / WGM, WN = NT / WGN;
  static constexpr int TM = WM / 32, TN = WN / 32;  // 32x32 MFMA tiles per wave
  static constexpr int CC = 16;                     // channels per k chunk
  static constexpr int KCH = 64;                    // input channels per workgroup (split-K slice)
  static constexpr int NCH = KCH / CC;              // chunks: every one's input loads issued up front
  static constexpr int PH = TH + 2, PW = TW + 2, PIX = IMGS * PH * PW;
  static constexpr int PS = PS_, ROWB = ROWB_, IMGB = IMGB_;
  static constexpr int A_BYTES = ((IMGS - 1) * IMGB + (PH - 1) * ROWB + PW * PS + 15) / 16 * 16;
  static constexpr int BPS = 80;
  static constexpr int B_BYTES = 9 * NT * BPS;
  static constexpr int STAGE = A_BYTES + B_BYTES + 64;  // + a dummy slot for padding items
  static constexpr int NA = (PIX * 4 + NTHR - 1) / NTHR;  // A float4 items per thread per chunk
  static constexpr int NB = (NT * 36 + NTHR - 1) / NTHR;  // B uint4 items per thread per chunk
  static constexpr int TST = NT + 4;                // epilogue tile row (floats)
  static constexpr int EPI = MT * TST * 4 + NTHR * 8 * 4 + 16;
  static constexpr int LDS_MAIN = 2 * STAGE > EPI ? 2 * STAGE : EPI;
  static_assert((WGM * WGN == 4 || WGM * WGN == 8) && TM >= 1 && TN >= 1 && WM % 32 == 0 && WN % 32 == 0, "wave tiling");
  static_assert(PS >= 64 && PS % 16 == 0 && ROWB % 16 == 0 && IMGB % 16 == 0, "16-B aligned fragments");
  static_assert(ROWB >= PW * PS && (IMGS == 1 || IMGB >= PH * ROWB), "patch pitches");
};

__device__ __forceinline__ f32x16 mfma_bf16x16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float4 as_f4(const u32x4& v) {
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
__device__ __forceinline__ float4 as_f4(const u32x2& v) {  // 4 bf16 -> fp32 (exact)
  return make_float4(__uint_as_float(v[0] << 16), __uint_as_float(v[0] & 0xffff0000u), __uint_as_float(v[1] << 16),
                     __uint_as_float(v[1] & 0xffff0000u));
}

// In-kernel phase stamps (profiling only, a.stamps != nullptr): lane 0 of
// wave 0 records the core clock at phase boundaries with a vector store.
template <class A>
__device__ __forceinline__ void stamp(const A& a, int k) {
  if (a.stamps && threadIdx.x == 0) {
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    a.stamps[(int64_t)b * 16 + k] = (long long)__builtin_readcyclecounter();
  }
}

// XCD-grouped workgroup order: the hardware deals workgroups round-robin
// over the 8 XCDs (id % 8); logical tile L runs on group L / ceil(n / 8), so
// consecutive spatial tiles of an image -- which share their halo rows --
// read them through ONE XCD's L2 (bijective for any n, cdna_hip_programming
// §5.5 T1).  All workgroups of a launch are co-resident (one per CU), so the
// dispatch order itself does not matter.
__device__ __forceinline__ int xcd_tile(int b, int n, bool on) {
  if (!on || n < 16) return b;
  const int q = n / 8, r = n % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// One BatchNorm replica row of the fp64 sums [reps][2][C]: (sum, sum2) of
// channel c in replica r (zeros past `reps`).
__device__ __forceinline__ void rep_load(const double* acc, int reps, int C, int r, int c, double& s0, double& s1) {
  const bool ok = acc != nullptr && r < reps;
  s0 = ok ? acc[(int64_t)r * 2 * C + c] : 0.0;
  s1 = ok ? acc[(int64_t)r * 2 * C + C + c] : 0.0;
}

// MODE 0: forward, A = FwdArgs; the operand fill applies the producer's
// BatchNorm (+ residual kind RK: 0 none, 1 fp32 tensor, 2 BN of a projection
// shortcut's pre-BN output) and ReLU.
// MODE 1: backward data, A = DgArgs; the fill applies the layer's BatchNorm
// backward (RK = 1: with the ReLU mask of the layer output), the 9 taps of
// the transposed weights are the forward's flipped (B slot 8 - tap).
// Grid: x = spatial tiles, y = output channel tiles, z = input-channel
// slices (split-K; kchunk channels each).
// BF (forward only): the bf16 option's tensors -- bf16 activations, residual,
// weights and output; the fill rounds the transformed value to bf16 once
// (the hi half only: one MFMA per product, the lo slots stay unused), the
// owner tiles write it as y, the output is rounded to bf16 and its BN sums
// are taken of the rounded values (as conv.hip's tile_epilogue).
template <class K, int MODE, int RK, bool BF, class A>
__device__ __forceinline__ void hconv_body(const A& a, int kchunk, uint8_t* smem) {
  constexpr bool DG = MODE == 1;
  static_assert(!(DG && BF), "the bf16 halo conv is forward-only");
  constexpr int EB = BF ? 2 : 4;  // activation / weight element bytes
  static_assert(K::NTHR == 512 && K::KCH == 64, "the coefficient prologue maps 8 waves onto 8 replicas x 64 channels");
  // input chunks whose loads are in flight ahead of their fill: every chunk
  // (forward, 1-2 inputs per element), or a ring of 2 (dgrad: 3 inputs)
  constexpr int PF = DG ? 2 : K::NCH;
  constexpr int NCOEF = DG ? 5 : 4;
  const int nblk = gridDim.x * gridDim.y * gridDim.z;
  const int lin = xcd_tile(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), nblk, a.xcd);
  const int bx = lin % gridDim.x, by = (lin / gridDim.x) % gridDim.y, bz = lin / (gridDim.x * gridDim.y);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int wm = wave / K::WGN, wn = wave % K::WGN;
  const int C = a.C;
  const int txn = a.W / K::TW, tyn = a.H / K::TH;
  int rem = bx;
  const int tx = rem % txn;
  rem /= txn;
  const int ty = rem % tyn;
  const int img0 = (rem / tyn) * K::IMGS;
  const int y0 = ty * K::TH, x0 = tx * K::TW;
  const int n0 = by * K::NT;
  const int kbeg = bz * kchunk;
  float* coef = reinterpret_cast<float*>(smem + K::LDS_MAIN);  // [NCOEF][kchunk]
  const auto& X = a.x;
  stamp(a, 0);

  // ---- coefficient sources, requested BEFORE the operand loads: thread t
  // holds channel cc = t % 64's sums of replica rr = t / 64 (the 8 waves
  // cover the 8 replicas) and the channel's per-channel parameters, so the
  // prologue waits only for these (counted vmcnt), never for the operands.
  const int cc = t & 63, rr = t >> 6;
  const int ch = kbeg + cc;
  double p0 = 0.0, p1 = 0.0, q0 = 0.0, q1 = 0.0;
  float g0 = 1.f, g1 = 0.f, g2 = 0.f, g3 = 0.f;  // per-channel parameters
  float e0 = 1.f, e1 = 0.f, e2 = 0.f, e3 = 0.f;  // RK == 2: the residual BN's
  if constexpr (DG) {
    rep_load(X.bn.acc, X.bn.reps, C, rr, ch, p0, p1);
    g0 = X.bn.gamma[ch];
    g1 = X.bn.mean[ch];
    g2 = X.bn.invstd[ch];
  } else {
    if (X.has_bn) {
      if (X.train) rep_load(X.bn.acc, X.bn.reps, C, rr, ch, p0, p1);
      g0 = X.bn.gamma[ch];
      g1 = X.bn.beta[ch];
      g2 = X.bn.run_mean[ch];
      g3 = X.bn.run_var[ch];
    }
    if constexpr (RK == 2) {
      if (X.train) rep_load(X.bnr.acc, X.bnr.reps, C, rr, ch, q0, q1);
      e0 = X.bnr.gamma[ch];
      e1 = X.bnr.beta[ch];
      e2 = X.bnr.run_mean[ch];
      e3 = X.bnr.run_var[ch];
    }
  }

  // ---- per-thread fill geometry (fixed over the chunks) ----
  const int q = t & 3;  // float4 within the 16-channel chunk (NTHR % 4 == 0)
  uint32_t a_off[K::NA];  // byte offset of the item's pixel + 4q channels, kOOB outside
  int a_lds[K::NA];       // LDS byte offset of the item's hi half (dummy slot: no item)
  bool a_own[K::NA];
  bool own_tile;
  if constexpr (DG) own_tile = by == 0 && (X.dzp != nullptr || X.dres != nullptr);
  else own_tile = by == 0 && (X.y != nullptr);
#pragma unroll
  for (int u = 0; u < K::NA; ++u) {
    const int i = t + K::NTHR * u;
    int p = i >> 2;
    // 80-B pixel pitch: the 4 pixels of a 16-lane ds_write_b64 group are
    // taken 2 apart (order 0 2 4 6 1 3 5 7 within each 8) so their 32-B hi /
    // lo spans cover 4 disjoint 8-bank sets (scripts/hconv_banks.py: 90 -> 28
    // extra cycles per chunk); full blocks of 8 only, so the map stays a
    // bijection on the patch
    if constexpr (K::PS == 80) {
      if (p < (K::PIX / 8) * 8) p = (p & ~7) | ((p & 3) << 1) | ((p >> 2) & 1);
    }
    const int img = p / (K::PH * K::PW);
    const int r2 = p - img * (K::PH * K::PW);
    const int py = r2 / K::PW, px = r2 - py * (K::PW);
    const int iy = y0 + py - 1, ix = x0 + px - 1;
    const bool item = i < K::PIX * 4;
    const bool in = item && (img0 + img < a.N) && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    a_off[u] = in ? (uint32_t)(((((img0 + img) * a.H + iy) * a.W + ix) * C + 4 * q) * EB) : kOOB;
    a_lds[u] = item ? img * K::IMGB + py * K::ROWB + px * K::PS + 8 * q : K::A_BYTES + K::B_BYTES + 8 * q;
    a_own[u] = own_tile && in && py >= 1 && py <= K::TH && px >= 1 && px <= K::TW;
  }
  // B items.  Forward: (co, tap, channel quad) -> one b128 of the packed
  // weight row W[n0 + co][tap][4 channels].  Dgrad: (tap, quad of 4 k =
  // layer output channels, n = ci) -> four b32 W[k .. k+3][tap][n0 + ci]
  // (each a coalesced 256-B row per wave), the transpose happens in the
  // register pass.
  uint32_t b_off[K::NB];
  int b_lds[K::NB];
#pragma unroll
  for (int u = 0; u < K::NB; ++u) {
    const int i = t + K::NTHR * u;
    const bool item = i < K::NT * 36;
    if constexpr (DG) {
      const int ci = i % K::NT, rs = i / K::NT;
      const int tap = rs >> 2, kq = rs & 3;
      b_off[u] = item ? (uint32_t)((((4 * kq) * 9 + tap) * a.Co + n0 + ci) * 4) : kOOB;
      b_lds[u] = item ? K::A_BYTES + (8 - tap) * (K::NT * K::BPS) + ci * K::BPS + 8 * kq
                      : K::A_BYTES + K::B_BYTES + 8 * kq;
    } else {
      // item -> (tap, co, channel quad) with co next-fastest: the 4 x 8-B LDS
      // writes of a 16-lane group land on 4 different rows; with tap
      // next-fastest (dbg & 8, the first layout) they were 5,120 B apart --
      // one bank group, a 4-way conflict on every weight write
      // (scripts/hconv_banks.py: 736 -> 0 extra cycles per chunk)
      int co, tap, bq;
      if (a.dbg & 8) {
        co = i / 36;
        const int r = i - co * 36;
        tap = r >> 2;
        bq = r & 3;
      } else {
        // rows taken 2 apart within each 8 (0 2 4 6 1 3 5 7): the 80-B row
        // pitch then puts a group's 4 rows on disjoint banks (0 extra cycles)
        bq = i & 3;
        const int k = (i >> 2) % K::NT;
        co = (k & ~7) | ((k & 3) << 1) | ((k >> 2) & 1);
        tap = (i >> 2) / K::NT;
      }
      b_off[u] = item ? (uint32_t)((((n0 + co) * 9 + tap) * C + 4 * bq) * EB) : kOOB;
      b_lds[u] = item ? K::A_BYTES + tap * (K::NT * K::BPS) + co * K::BPS + 8 * bq
                      : K::A_BYTES + K::B_BYTES + 8 * bq;
    }
  }
  const uint32_t in_bytes = (uint32_t)((int64_t)a.N * a.H * a.W * C * EB);
  const float* src0;
  const float* src1;
  const float* src2 = nullptr;
  if constexpr (DG) {
    src0 = X.dy;
    src1 = X.z;
    src2 = X.ymask;
  } else {
    src0 = X.z;
    src1 = RK == 1 ? X.res : X.zr;
  }
  const auto rs0 = make_rsrc(src0, in_bytes);
  const auto rs1 = make_rsrc(src1, in_bytes);
  const auto rs2 = make_rsrc(src2, in_bytes);
  const auto rsW = make_rsrc(a.wp, (uint32_t)((int64_t)a.Co * 9 * C * EB));
  constexpr bool IN1 = DG || RK != 0;  // second input per element
  constexpr bool IN2 = DG && RK == 1;  // third (dgrad ReLU mask)

  // Operand registers: a ring of PF chunks of the input patch (the
  // producer's output comes from the Infinity Cache / HBM, ~2 us: its latency
  // is paid once, under the coefficient prologue); the weights (L2-resident)
  // stream one chunk ahead through a single register set.
  using AV = std::conditional_t<BF, u32x2, u32x4>;  // 4 channels of one pixel
  AV az[PF][K::NA], ar[PF][K::NA];
  u32x4 am[PF][K::NA];
  AV bw[K::NB];
  auto ld4 = [&](__amdgpu_buffer_rsrc_t r, uint32_t off) -> AV {
    if constexpr (BF) return __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
    else return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  };
  auto load_a = [&](auto kc) {
    constexpr int k = decltype(kc)::value, S = k % PF;
    if (a.dbg & 4) return;
    const uint32_t cb = (uint32_t)((kbeg + k * K::CC) * EB);
#pragma unroll
    for (int u = 0; u < K::NA; ++u) {
      const uint32_t off = a_off[u] == kOOB ? kOOB : a_off[u] + cb;
      az[S][u] = ld4(rs0, off);
      if constexpr (IN1) ar[S][u] = ld4(rs1, off);
      if constexpr (IN2) am[S][u] = __builtin_amdgcn_raw_buffer_load_b128(rs2, (int)off, 0, 0);
    }
  };
  auto load_b = [&](int k) {
    if (a.dbg & 4) return;
    if constexpr (DG) {
      const uint32_t kb = (uint32_t)((kbeg + k * K::CC) * 9 * a.Co * 4);  // first k row of the chunk
      const uint32_t kst = (uint32_t)(9 * a.Co * 4);                       // next k
#pragma unroll
      for (int u = 0; u < K::NB; ++u) {
        const uint32_t off = b_off[u] == kOOB ? kOOB : b_off[u] + kb;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          bw[u][e] = __builtin_amdgcn_raw_buffer_load_b32(rsW, (int)(off == kOOB ? kOOB : off + e * kst), 0, 0);
      }
    } else {
      const uint32_t cb = (uint32_t)((kbeg + k * K::CC) * EB);
#pragma unroll
      for (int u = 0; u < K::NB; ++u) {
        const uint32_t off = b_off[u] == kOOB ? kOOB : b_off[u] + cb;
        bw[u] = ld4(rsW, off);
      }
    }
  };
  // The fill of a chunk as NA + NB independent work units (unit u < NA: one
  // float4 of the input patch -> transform -> bf16 hi + lo -> LDS and, for
  // owner tiles, the transform's global outputs; unit NA + v: one packed
  // weight float4 -> hi / lo -> LDS).  The units of chunk k+1 are spread over
  // the taps of chunk k's MFMAs (their VALU / LDS writes issue under the
  // matrix pipe).
  struct Coef4 {
    float4 c0, c1, c2, c3, c4;
  };
  auto coef4 = [&](int k) {
    const int cl = k * K::CC + 4 * q;  // channel within the slice
    Coef4 c;
    c.c0 = *reinterpret_cast<const float4*>(coef + cl);
    c.c1 = *reinterpret_cast<const float4*>(coef + kchunk + cl);
    c.c2 = c.c0;
    c.c3 = c.c1;
    c.c4 = c.c0;
    if constexpr (DG || RK == 2) {
      c.c2 = *reinterpret_cast<const float4*>(coef + 2 * kchunk + cl);
      c.c3 = *reinterpret_cast<const float4*>(coef + 3 * kchunk + cl);
    }
    if constexpr (DG) c.c4 = *reinterpret_cast<const float4*>(coef + 4 * kchunk + cl);
    return c;
  };
  auto store_unit = [&](auto kc, auto uc, uint8_t* stage, const Coef4& cf) {
    constexpr int k = decltype(kc)::value, U = decltype(uc)::value, S = k % PF;
    if constexpr (U < K::NA) {
      constexpr int u = U;
      const bool oob = a_off[u] == kOOB;  // padding: zero after the transform
      float4 v, gd;
      if constexpr (DG) {
        // bn32_bwd_apply's arithmetic (explicit fma: the same bits):
        // dz = k1 (g - mg - ((z - mu) is) mx)
        gd = as_f4(az[S][u]);
        if constexpr (IN2) {
          const float4 ym = as_f4(am[S][u]);
          gd.x = ym.x > 0.f ? gd.x : 0.f;
          gd.y = ym.y > 0.f ? gd.y : 0.f;
          gd.z = ym.z > 0.f ? gd.z : 0.f;
          gd.w = ym.w > 0.f ? gd.w : 0.f;
        }
        const float4 zv = as_f4(ar[S][u]);
        const float4 &k1 = cf.c0, &mg = cf.c1, &mx = cf.c2, &mu = cf.c3, &is = cf.c4;
        v.x = k1.x * fmaf(-((zv.x - mu.x) * is.x), mx.x, gd.x - mg.x);
        v.y = k1.y * fmaf(-((zv.y - mu.y) * is.y), mx.y, gd.y - mg.y);
        v.z = k1.z * fmaf(-((zv.z - mu.z) * is.z), mx.z, gd.z - mg.z);
        v.w = k1.w * fmaf(-((zv.w - mu.w) * is.w), mx.w, gd.w - mg.w);
      } else {
        const float4 zv = as_f4(az[S][u]);
        v = make_float4(fmaf(zv.x, cf.c0.x, cf.c1.x), fmaf(zv.y, cf.c0.y, cf.c1.y),
                        fmaf(zv.z, cf.c0.z, cf.c1.z), fmaf(zv.w, cf.c0.w, cf.c1.w));
        if constexpr (RK == 1) {
          const float4 r = as_f4(ar[S][u]);
          v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
        } else if constexpr (RK == 2) {
          const float4 r = as_f4(ar[S][u]);
          v.x += fmaf(r.x, cf.c2.x, cf.c3.x);
          v.y += fmaf(r.y, cf.c2.y, cf.c3.y);
          v.z += fmaf(r.z, cf.c2.z, cf.c3.z);
          v.w += fmaf(r.w, cf.c2.w, cf.c3.w);
        }
        const float lo = X.relu ? 0.f : -__builtin_inff();
        v.x = fmaxf(v.x, lo); v.y = fmaxf(v.y, lo); v.z = fmaxf(v.z, lo); v.w = fmaxf(v.w, lo);
      }
      v.x = oob ? 0.f : v.x; v.y = oob ? 0.f : v.y; v.z = oob ? 0.f : v.z; v.w = oob ? 0.f : v.w;
      uint8_t* d = stage + a_lds[u];
      if constexpr (BF) {
        const uint32_t h01 = cvt_pk_bf16(f32x2{v.x, v.y}), h23 = cvt_pk_bf16(f32x2{v.z, v.w});
        *reinterpret_cast<uint2*>(d) = make_uint2(h01, h23);
        if (a_own[u]) {
          const uint32_t go = a_off[u] + (uint32_t)((kbeg + k * K::CC) * EB);
          *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(X.y) + go) = make_uint2(h01, h23);
        }
        return;
      }
      uint32_t h01, l01, h23, l23;
      split2(v.x, v.y, h01, l01);
      split2(v.z, v.w, h23, l23);
      *reinterpret_cast<uint2*>(d) = make_uint2(h01, h23);
      *reinterpret_cast<uint2*>(d + 32) = make_uint2(l01, l23);
      if (a_own[u]) {
        const uint32_t go = a_off[u] + (uint32_t)((kbeg + k * K::CC) * 4);  // pixel + chunk + 4q channels
        const uint4 pk = make_uint4((h01 << 16) | (l01 & 0xffffu), (h01 & 0xffff0000u) | (l01 >> 16),
                                    (h23 << 16) | (l23 & 0xffffu), (h23 & 0xffff0000u) | (l23 >> 16));
        if constexpr (DG) {
          if (X.dres) *reinterpret_cast<float4*>(reinterpret_cast<uint8_t*>(X.dres) + go) = gd;
          if (X.dzp) *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(X.dzp) + go) = pk;
        } else {
          *reinterpret_cast<float4*>(reinterpret_cast<uint8_t*>(X.y) + go) = v;
          if (X.yp) *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(X.yp) + go) = pk;
        }
      }
    } else if constexpr (BF) {
      constexpr int u = U - K::NA;
      *reinterpret_cast<uint2*>(stage + b_lds[u]) = make_uint2(bw[u][0], bw[u][1]);
    } else {
      constexpr int u = U - K::NA;
      const u32x4 d = bw[u];
      const uint32_t h01 = __builtin_amdgcn_perm(d[1], d[0], 0x07060302u);
      const uint32_t h23 = __builtin_amdgcn_perm(d[3], d[2], 0x07060302u);
      const uint32_t l01 = __builtin_amdgcn_perm(d[1], d[0], 0x05040100u);
      const uint32_t l23 = __builtin_amdgcn_perm(d[3], d[2], 0x05040100u);
      uint8_t* p = stage + b_lds[u];
      *reinterpret_cast<uint2*>(p) = make_uint2(h01, h23);
      *reinterpret_cast<uint2*>(p + 32) = make_uint2(l01, l23);
    }
  };
  constexpr int NU = K::NA + K::NB;
  // LDS-only barrier: the owner-write global stores and the operand loads
  // stay in flight (__syncthreads would drain vmcnt)
  auto bar = [&]() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes / reads done
    lds_barrier();
  };

  static_for<PF>([&](auto kc) { load_a(kc); });
  load_b(0);

  // ---- coefficients of this slice's input channels: replica partials ->
  // LDS (stage 1, free until chunk 1's fill) -> wave 0 sums them in replica
  // order (bit-identical to bn32's rep_sums) -> coef[][]
  double* part = reinterpret_cast<double*>(smem + K::STAGE);  // [2 sources][8][2][64]
  part[(rr * 2 + 0) * 64 + cc] = p0;
  part[(rr * 2 + 1) * 64 + cc] = p1;
  if constexpr (!DG && RK == 2) {
    part[1024 + (rr * 2 + 0) * 64 + cc] = q0;
    part[1024 + (rr * 2 + 1) * 64 + cc] = q1;
  }
  bar();
  if (wave == 0) {
    const int c = cc;
    auto sums = [&](int base, double& s0, double& s1) {
      s0 = 0.0;
      s1 = 0.0;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        s0 += part[base + (r * 2 + 0) * 64 + c];
        s1 += part[base + (r * 2 + 1) * 64 + c];
      }
    };
    const double inv_m = 1.0 / (double)X.M;
    const bool publish = bx == 0 && by == 0;
    if constexpr (DG) {
      double s, qq;
      sums(0, s, qq);
      coef[c] = g0 * g2;                    // gamma * invstd
      coef[kchunk + c] = (float)(s * inv_m);  // mean g
      coef[2 * kchunk + c] = (float)(qq * inv_m);  // mean g * xhat
      coef[3 * kchunk + c] = g1;            // mean
      coef[4 * kchunk + c] = g2;            // invstd
      if (publish) {
        if (X.bn.dgamma) X.bn.dgamma[ch] = (float)qq;
        if (X.bn.dbeta) X.bn.dbeta[ch] = (float)s;
      }
    } else {
      // bn32_apply's fp64 coefficient math; publishes the batch statistics
      // and running averages once per channel
      auto coefs = [&](const BnSrc& b, int base, float gm, float bt, float rm, float rv, float& sc, float& sh) {
        double mu, var;
        if (X.train) {
          double s0, s1;
          sums(base, s0, s1);
          mu = s0 * inv_m;
          var = s1 * inv_m - mu * mu;
          if (var < 0.0) var = 0.0;
        } else {
          mu = rm;
          var = rv;
        }
        const double isd = 1.0 / sqrt(var + (double)b.eps);
        sc = (float)((double)gm * isd);
        sh = (float)((double)bt - mu * (double)gm * isd);
        if (X.train && publish) {
          b.mean[ch] = (float)mu;
          b.invstd[ch] = (float)isd;
          if (b.run_mean) {
            const int M = X.M;
            const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
            b.run_mean[ch] = fmaf(1.f - b.momentum, rm, b.momentum * (float)mu);  // = bn32_apply's bits
            b.run_var[ch] = fmaf(1.f - b.momentum, rv, b.momentum * (float)unb);
          }
        }
      };
      float sc = 1.f, sh = 0.f;
      if (X.has_bn) coefs(X.bn, 0, g0, g1, g2, g3, sc, sh);
      coef[c] = sc;
      coef[kchunk + c] = sh;
      if constexpr (RK == 2) {
        float s2, h2;
        coefs(X.bnr, 1024, e0, e1, e2, e3, s2, h2);
        coef[2 * kchunk + c] = s2;
        coef[3 * kchunk + c] = h2;
      }
    }
  }
  bar();  // coefficients visible; the operand loads are still in flight

  // ---- fragment addresses (tap (0,0), hi half; lo at +32) ----
  int fa_off[K::TM], fb_off[K::TN];
#pragma unroll
  for (int i = 0; i < K::TM; ++i) {
    const int m = wm * K::WM + 32 * i + li;
    const int img = m / (K::TH * K::TW);
    const int r2 = m - img * (K::TH * K::TW);
    const int y = r2 / K::TW, x = r2 - y * K::TW;
    fa_off[i] = img * K::IMGB + y * K::ROWB + x * K::PS + 16 * lh;
  }
#pragma unroll
  for (int j = 0; j < K::TN; ++j) fb_off[j] = K::A_BYTES + (wn * K::WN + 32 * j + li) * K::BPS + 16 * lh;

  f32x16 acc[K::TM][K::TN];
#pragma unroll
  for (int i = 0; i < K::TM; ++i)
#pragma unroll
    for (int j = 0; j < K::TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // 9 taps, fragments read two taps ahead (three register sets): the MFMAs
  // of tap t wait only for the reads issued before tap t-1's; sched_barrier
  // keeps hipcc from sinking the reads back behind the MFMAs
  auto compute = [&](const uint8_t* st, auto&& side) {
    bf16x8 ah[3][K::TM], al[3][K::TM], bh[3][K::TN], bl[3][K::TN];
    auto rd = [&](auto tapc) {
      constexpr int TAP = decltype(tapc)::value, S = TAP % 3;
      constexpr int AO = (TAP / 3) * K::ROWB + (TAP % 3) * K::PS;
      constexpr int BO = TAP * K::NT * K::BPS;
#pragma unroll
      for (int i = 0; i < K::TM; ++i) {
        ah[S][i] = *reinterpret_cast<const bf16x8*>(st + fa_off[i] + AO);
        if constexpr (!BF) al[S][i] = *reinterpret_cast<const bf16x8*>(st + fa_off[i] + AO + 32);
      }
#pragma unroll
      for (int j = 0; j < K::TN; ++j) {
        bh[S][j] = *reinterpret_cast<const bf16x8*>(st + fb_off[j] + BO);
        if constexpr (!BF) bl[S][j] = *reinterpret_cast<const bf16x8*>(st + fb_off[j] + BO + 32);
      }
    };
    rd(IC<0>{});
    rd(IC<1>{});
    static_for<9>([&](auto tapc) {
      constexpr int TAP = decltype(tapc)::value, S = TAP % 3;
      if constexpr (TAP + 2 < 9) {
        if (!(a.dbg & 2)) rd(IC<TAP + 2>{});
      }
      __builtin_amdgcn_sched_barrier(0);
      if (!(a.dbg & 1)) {
#pragma unroll
        for (int i = 0; i < K::TM; ++i)
#pragma unroll
          for (int j = 0; j < K::TN; ++j) {
            if constexpr (!BF) {
              acc[i][j] = mfma_bf16x16(al[S][i], bh[S][j], acc[i][j]);
              acc[i][j] = mfma_bf16x16(ah[S][i], bl[S][j], acc[i][j]);
            }
            acc[i][j] = mfma_bf16x16(ah[S][i], bh[S][j], acc[i][j]);
          }
      }
      side(tapc);  // fill units of the next chunk, behind this tap's MFMAs
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  stamp(a, 1);
  {
    const Coef4 cf = coef4(0);
    static_for<NU>([&](auto uc) { store_unit(IC<0>{}, uc, smem, cf); });
  }
  if constexpr (PF < K::NCH) load_a(IC<PF>{});  // chunk 0's registers are free
  load_b(1);
  bar();
  stamp(a, 2);
  static_for<K::NCH>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    uint8_t* cur = smem + (k & 1) * K::STAGE;
    uint8_t* nxt = smem + ((k + 1) & 1) * K::STAGE;
    if constexpr (k + 1 < K::NCH) {
      const Coef4 cf = coef4(k + 1);
      // unit u of chunk k+1 rides behind tap (u * 9 / NU)
      compute(cur, [&](auto tapc) {
        constexpr int TAP = decltype(tapc)::value;
        static_for<NU>([&](auto uc) {
          constexpr int U = decltype(uc)::value;
          if constexpr (U * 9 / NU == TAP) store_unit(IC<k + 1>{}, uc, nxt, cf);
        });
      });
      if constexpr (k + 1 + PF < K::NCH) load_a(IC<k + 1 + PF>{});
      if constexpr (k + 2 < K::NCH) load_b(k + 2);
    } else {
      compute(cur, [](auto) {});
    }
    if constexpr (k == 0) stamp(a, 3);
    bar();
    if constexpr (k == 0) stamp(a, 4);
  });
  __syncthreads();
  stamp(a, 5);

  // ---- epilogue: tile through LDS, split-K reduce, output (+ reductions) ----
  float* tile = reinterpret_cast<float*>(smem);
  float* red = tile + K::MT * K::TST;
#pragma unroll
  for (int i = 0; i < K::TM; ++i)
#pragma unroll
    for (int j = 0; j < K::TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rl = wm * K::WM + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * lh;
        tile[rl * K::TST + wn * K::WN + 32 * j + li] = acc[i][j][e];
      }
  __syncthreads();
  const int splits = gridDim.z;
  constexpr int C4 = K::NT / 4;
  constexpr int F = K::MT * K::NT / (4 * K::NTHR);  // float4 per thread
  static_assert(K::MT * K::NT % (4 * K::NTHR) == 0, "epilogue vectors");
  if (splits > 1) {
    // in-launch split-K (conv32.hip): write-through slabs + arrival ticket,
    // the last arriver sums the slices in slice order (deterministic)
    const int tile_id = by * gridDim.x + bx;
    const int ntiles = gridDim.x * gridDim.y;
    const int64_t zstride = (int64_t)ntiles * K::MT * K::NT * 4;
    const auto rsS = make_rsrc(a.slab + (int64_t)tile_id * (K::MT * K::NT), 0x7FFFFFF0u);
    const uint32_t zoff = (uint32_t)(bz * zstride);
#pragma unroll
    for (int u = 0; u < F; ++u) {
      const int f = t + K::NTHR * u;
      const float4 v = *reinterpret_cast<const float4*>(tile + (f / C4) * K::TST + (f % C4) * 4);
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)}, rsS,
          (int)(zoff + f * 16), 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(red + K::NTHR * 8);
    if (t == 0) {
      const int prev = __hip_atomic_fetch_add(&a.counters[tile_id], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == splits - 1;
      if (last) __hip_atomic_store(&a.counters[tile_id], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    float4 sum[F];
#pragma unroll
    for (int u = 0; u < F; ++u) sum[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    // every other slice's slab is requested at once (one memory latency,
    // not splits - 1 in series: 2-4 us of the 8-slice 4x4x512 stage), then
    // summed in slice order (deterministic, the same bits as a serial sum)
    constexpr int MAXS = 8;  // plan_fwd: at most 8 slices
    u32x4 sl[MAXS][F];
#pragma unroll
    for (int z = 0; z < MAXS; ++z) {
      if (z >= splits) break;  // uniform: only the real slices' loads issue
#pragma unroll
      for (int u = 0; u < F; ++u) {
        const int f = t + K::NTHR * u;
        sl[z][u] = __builtin_amdgcn_raw_buffer_load_b128(
            rsS, (int)(z != bz ? (uint32_t)(z * zstride + f * 16) : kOOB), 0, 16);  // own slice: LDS below
      }
    }
#pragma unroll
    for (int z = 0; z < MAXS; ++z) {
      if (z >= splits) break;
#pragma unroll
      for (int u = 0; u < F; ++u) {
        const int f = t + K::NTHR * u;
        const float4 r = z == bz ? *reinterpret_cast<const float4*>(tile + (f / C4) * K::TST + (f % C4) * 4)
                                 : as_f4(sl[z][u]);
        sum[u] = make_float4(sum[u].x + r.x, sum[u].y + r.y, sum[u].z + r.z, sum[u].w + r.w);
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < F; ++u) {
      const int f = t + K::NTHR * u;
      *reinterpret_cast<float4*>(tile + (f / C4) * K::TST + (f % C4) * 4) = sum[u];
    }
    __syncthreads();
  }
  stamp(a, 6);
  // output rows: float4 per thread per pass, + the per-channel reductions
  // (forward: this conv's BN statistics; dgrad: the consumer BN backward's)
  constexpr int RPP = K::NTHR / C4;
  const int cg = t % C4, r0 = t / C4;
  const int col = n0 + cg * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), sq = s, mu = s, is = s;
  bool red_on;
  if constexpr (DG) {
    red_on = a.bnb.acc != nullptr;
    if (red_on) {
      mu = *reinterpret_cast<const float4*>(a.bnb.mean + col);
      is = *reinterpret_cast<const float4*>(a.bnb.invstd + col);
    }
  } else {
    red_on = a.stats != nullptr;
  }
  for (int rl = r0; rl < K::MT; rl += RPP) {
    const int img = rl / (K::TH * K::TW);
    const int r2 = rl - img * (K::TH * K::TW);
    const int y = r2 / K::TW, x = r2 - y * K::TW;
    if (img0 + img >= a.N) continue;
    float4 v = *reinterpret_cast<const float4*>(tile + rl * K::TST + cg * 4);
    const int64_t off = (((int64_t)(img0 + img) * a.H + y0 + y) * a.W + x0 + x) * a.Co + col;
    if constexpr (BF) {
      const uint32_t p01 = cvt_pk_bf16(f32x2{v.x, v.y}), p23 = cvt_pk_bf16(f32x2{v.z, v.w});
      *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(a.out) + off) = make_uint2(p01, p23);
      v = as_f4(u32x2{p01, p23});  // the statistics of the stored (rounded) output
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      sq.x += v.x * v.x; sq.y += v.y * v.y; sq.z += v.z * v.z; sq.w += v.w * v.w;
      continue;
    }
    float4* dst = reinterpret_cast<float4*>(a.out + off);
    if constexpr (DG) {
      if (a.accumulate) {
        const float4 o = *dst;
        v = make_float4(v.x + o.x, v.y + o.y, v.z + o.z, v.w + o.w);
      }
      *dst = v;
      if (red_on) {
        // tile_epilogue32's consumer-BN reductions: g = dx [* (y > 0)]
        const float4 z = *reinterpret_cast<const float4*>(a.bnb.z + off);
        float4 gk = v;
        if (a.bnb.y) {
          const float4 ym = *reinterpret_cast<const float4*>(a.bnb.y + off);
          gk.x = ym.x > 0.f ? gk.x : 0.f;
          gk.y = ym.y > 0.f ? gk.y : 0.f;
          gk.z = ym.z > 0.f ? gk.z : 0.f;
          gk.w = ym.w > 0.f ? gk.w : 0.f;
        }
        s.x += gk.x; s.y += gk.y; s.z += gk.z; s.w += gk.w;
        sq.x += gk.x * ((z.x - mu.x) * is.x);
        sq.y += gk.y * ((z.y - mu.y) * is.y);
        sq.z += gk.z * ((z.z - mu.z) * is.z);
        sq.w += gk.w * ((z.w - mu.w) * is.w);
      }
    } else {
      *dst = v;
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      sq.x += v.x * v.x; sq.y += v.y * v.y; sq.z += v.z * v.z; sq.w += v.w * v.w;
    }
  }
  stamp(a, 7);
  if (!red_on) return;
  double* stats;
  if constexpr (DG) stats = a.bnb.acc + (int64_t)((bx + by * gridDim.x) % a.bnb.reps) * 2 * a.Co;
  else stats = a.stats + (int64_t)((bx + by * gridDim.x) % a.reps) * 2 * a.Co;
  reinterpret_cast<float4*>(red)[2 * t] = s;
  reinterpret_cast<float4*>(red)[2 * t + 1] = sq;
  __syncthreads();
  if (t < K::NT) {
    const int cgi = t >> 2, kk = t & 3;
    double sa = 0.0, sb = 0.0;
    for (int r = 0; r < RPP; ++r) {
      sa += red[(r * C4 + cgi) * 8 + kk];
      sb += red[(r * C4 + cgi) * 8 + 4 + kk];
    }
    atomicAdd(&stats[n0 + t], sa);
    atomicAdd(&stats[a.Co + n0 + t], sb);
  }
  stamp(a, 8);
}

template <class K, int RK, bool BF>
__global__ __launch_bounds__(K::NTHR, 1) void hconv_fwd_kernel(FwdArgs a, int kchunk) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  hconv_body<K, 0, RK, BF>(a, kchunk, smem);
}

template <class K, int MASK>
__global__ __launch_bounds__(K::NTHR, 1) void hconv_dgrad_kernel(DgArgs a, int kchunk) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  hconv_body<K, 1, MASK, false>(a, kchunk, smem);
}

// Stage configurations for the CIFAR ResNet-18 shapes at any batch (3x3, s1):
// Every stage: 128 output pixels x 64 output channels per workgroup, 8 waves
// as 4 (pixels) x 2 (channels) of 32x32 MFMA tiles, 64 input channels per
// workgroup (split-K over the rest):
// S1 32x32x64: 8x16-pixel tiles; S2 16x16x128: 8x16, 2 slices;
// S3 8x8x256: 2 images, 4 slices; S4 4x4x512: 8 images, 8 slices
// (pitches from scripts/hconv_banks.py: conflict-free A reads for every tap)
using S1 = Cfg<8, 16, 1, 64, 4, 2, 80, 1536, 15360>;
using S2 = Cfg<8, 16, 1, 64, 4, 2, 80, 1536, 15360>;
using S3 = Cfg<8, 8, 2, 64, 4, 2, 64, 784, 7936>;
using S4 = Cfg<4, 4, 8, 64, 4, 2, 64, 528, 3328>;

struct Plan {
  int stage;  // 0: unsupported
  int splits;
  int kchunk;
  dim3 grid;
  int mt, nt;
};

Plan plan_fwd(int N, int H, int W, int C, int Co) {
  Plan p{0, 1, C, dim3(1, 1, 1), 0, 0};
  if (H != W || C != Co) return p;
  auto fill = [&](int st, int th, int tw, int imgs, int nt, int splits) {
    if (N % imgs || H % th || W % tw || Co % nt || C % (splits * 32)) return;
    p.stage = st;
    p.splits = splits;
    p.kchunk = C / splits;
    p.grid = dim3((N / imgs) * (H / th) * (W / tw), Co / nt, splits);
    p.mt = imgs * th * tw;
    p.nt = nt;
  };
  if (H == 32 && C == 64) fill(1, 8, 16, 1, 64, 1);
  else if (H == 16 && C == 128) fill(2, 8, 16, 1, 64, 2);
  else if (H == 8 && C == 256) fill(3, 8, 8, 2, 64, 4);
  else if (H == 4 && C == 512) fill(4, 4, 4, 8, 64, 8);
  if (p.stage && p.splits > 1 && p.grid.x * p.grid.y > 1024) p.stage = 0;  // split-K arrival counter block
  if (p.stage && p.kchunk != 64) p.stage = 0;               // Cfg::KCH
  return p;
}

template <class Kern, class Args>
void launch(Kern* kern, const Args& a, const Plan& p, size_t lds, int nthr, hipStream_t s) {
  static bool init = false;  // one per kernel instantiation
  if (!init) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    init = true;
  }
  kern<<<p.grid, nthr, lds, s>>>(a, p.kchunk);
}

template <class K>
size_t lds_of(const Plan& p) {
  return (size_t)K::LDS_MAIN + 5 * (size_t)p.kchunk * sizeof(float);  // + coef [5][kchunk]
}

template <class K, bool BF>
void go_rk(const FwdArgs& a, const Plan& p, hipStream_t s) {
  const size_t lds = lds_of<K>(p);
  if (a.x.zr) launch(&hconv_fwd_kernel<K, 2, BF>, a, p, lds, K::NTHR, s);
  else if (a.x.res) launch(&hconv_fwd_kernel<K, 1, BF>, a, p, lds, K::NTHR, s);
  else launch(&hconv_fwd_kernel<K, 0, BF>, a, p, lds, K::NTHR, s);
}

template <class K>
void go_rk(const FwdArgs& a, const Plan& p, hipStream_t s) {
  if (a.bf16) go_rk<K, true>(a, p, s);
  else go_rk<K, false>(a, p, s);
}

template <class K>
void go_dg(const DgArgs& a, const Plan& p, hipStream_t s) {
  const size_t lds = lds_of<K>(p);
  if (a.x.ymask) launch(&hconv_dgrad_kernel<K, 1>, a, p, lds, K::NTHR, s);
  else launch(&hconv_dgrad_kernel<K, 0>, a, p, lds, K::NTHR, s);
}

}  // namespace

int64_t hconv_fwd_workspace(int N, int H, int W, int C, int Co) {
  const Plan p = plan_fwd(N, H, W, C, Co);
  if (!p.stage) return -1;
  if (p.splits <= 1) return 0;
  return 1024 + (int64_t)p.splits * p.grid.x * p.grid.y * p.mt * p.nt;
}

void launch_hconv_fwd(const FwdArgs& a, hipStream_t s) {
  const Plan p = plan_fwd(a.N, a.H, a.W, a.C, a.Co);
  switch (p.stage) {
    case 1: go_rk<S1>(a, p, s); break;
    case 2: go_rk<S2>(a, p, s); break;
    case 3: go_rk<S3>(a, p, s); break;
    case 4: go_rk<S4>(a, p, s); break;
    default: break;  // the binding checked support
  }
}

void launch_hconv_dgrad(const DgArgs& a, hipStream_t s) {
  const Plan p = plan_fwd(a.N, a.H, a.W, a.C, a.Co);  // C == Co: the forward's tiling
  switch (p.stage) {
    case 1: go_dg<S1>(a, p, s); break;
    case 2: go_dg<S2>(a, p, s); break;
    case 3: go_dg<S3>(a, p, s); break;
    case 4: go_dg<S4>(a, p, s); break;
    default: break;
  }
}

}  // namespace hc
}  // namespace mfl
