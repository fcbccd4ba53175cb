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

// BatchNorm coefficients of channel c (bn32.hip bn32_apply_body, same fp64
// math): scale / shift, publishing the batch statistics and running averages
// when `publish`.
__device__ __forceinline__ void bn_coef(const BnSrc& b, int C, int c, int M, bool train, bool publish, float& sc,
                                        float& sh) {
  double mu, var;
  if (train) {
    double a[8], q[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      a[r] = r < b.reps ? b.acc[(int64_t)r * 2 * C + c] : 0.0;
      q[r] = r < b.reps ? b.acc[(int64_t)r * 2 * C + C + c] : 0.0;
    }
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      s0 += a[r];
      s1 += q[r];
    }
    const double inv_m = 1.0 / (double)M;
    mu = s0 * inv_m;
    var = s1 * inv_m - mu * mu;
    if (var < 0.0) var = 0.0;
  } else {
    mu = b.run_mean[c];
    var = b.run_var[c];
  }
  const double isd = 1.0 / sqrt(var + (double)b.eps);
  sc = (float)((double)b.gamma[c] * isd);
  sh = (float)((double)b.beta[c] - mu * (double)b.gamma[c] * isd);
  if (train && publish) {
    b.mean[c] = (float)mu;
    b.invstd[c] = (float)isd;
    if (b.run_mean) {
      const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
      b.run_mean[c] = (1.f - b.momentum) * b.run_mean[c] + b.momentum * (float)mu;
      b.run_var[c] = (1.f - b.momentum) * b.run_var[c] + b.momentum * (float)unb;
    }
  }
}

__device__ __forceinline__ f32x16 mfma_bf16x16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float4 as_f4(const u32x4& v) {
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}

// In-kernel phase stamps (profiling only, a.stamps != nullptr): lane 0 of
// wave 0 records the core clock at phase boundaries with a vector store.
__device__ __forceinline__ void stamp(const FwdArgs& a, int k) {
  if (a.stamps && threadIdx.x == 0) {
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    a.stamps[(int64_t)b * 16 + k] = (long long)__builtin_readcyclecounter();
  }
}

// RK: residual kind of the input transform (0 none, 1 fp32 tensor, 2 BN of a
// projection shortcut's pre-BN output).  Grid: x = spatial tiles, y = output
// channel tiles, z = input-channel slices (split-K; kchunk channels each).
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

template <class K, int RK>
__global__ __launch_bounds__(K::NTHR, 1) void hconv_fwd_kernel(FwdArgs a, int kchunk) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
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
  float* coef = reinterpret_cast<float*>(smem + K::LDS_MAIN);  // [4][kchunk]: sc, sh, sc2, sh2
  const FwdXform& X = a.x;
  stamp(a, 0);

  // ---- per-thread fill geometry (fixed over the chunks) ----
  const int q = t & 3;  // float4 within the 16-channel chunk (NTHR % 4 == 0)
  uint32_t a_off[K::NA];  // byte offset of the item's pixel + 4q channels, kOOB outside
  int a_lds[K::NA];       // LDS byte offset of the item's hi half (-1: no item)
  bool a_own[K::NA];
  const bool own_tile = by == 0 && (X.y != nullptr);
#pragma unroll
  for (int u = 0; u < K::NA; ++u) {
    const int i = t + K::NTHR * u;
    const int p = i >> 2;
    const int img = p / (K::PH * K::PW);
    const int r2 = p - img * (K::PH * K::PW);
    const int py = r2 / K::PW, px = r2 - py * (K::PW);
    const int iy = y0 + py - 1, ix = x0 + px - 1;
    const bool item = i < K::PIX * 4;
    const bool in = item && (img0 + img < a.N) && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    a_off[u] = in ? (uint32_t)(((((img0 + img) * a.H + iy) * a.W + ix) * C + 4 * q) * 4) : kOOB;
    a_lds[u] = item ? img * K::IMGB + py * K::ROWB + px * K::PS + 8 * q : K::A_BYTES + K::B_BYTES + 8 * q;
    a_own[u] = own_tile && in && py >= 1 && py <= K::TH && px >= 1 && px <= K::TW;
  }
  uint32_t b_off[K::NB];
  int b_lds[K::NB];
#pragma unroll
  for (int u = 0; u < K::NB; ++u) {
    const int i = t + K::NTHR * u;
    const int co = i / 36, r = i - co * 36;
    const int tap = r >> 2, bq = r & 3;
    const bool item = i < K::NT * 36;
    b_off[u] = item ? (uint32_t)((((n0 + co) * 9 + tap) * C + 4 * bq) * 4) : kOOB;
    b_lds[u] = item ? K::A_BYTES + tap * (K::NT * K::BPS) + co * K::BPS + 8 * bq : K::A_BYTES + K::B_BYTES + 8 * bq;
  }
  const uint32_t in_bytes = (uint32_t)((int64_t)a.N * a.H * a.W * C * 4);
  const auto rsZ = make_rsrc(X.z, in_bytes);
  const auto rsR = make_rsrc(RK == 1 ? X.res : X.zr, in_bytes);
  const auto rsW = make_rsrc(a.wp, (uint32_t)((int64_t)a.Co * 9 * C * 4));

  // The input patch of EVERY chunk is requested at kernel start (its latency
  // -- the producer's output comes from the Infinity Cache / HBM, ~2 us -- is
  // paid once, under the BatchNorm coefficient prologue); the weights (L2-
  // resident) stream one chunk ahead through a single register set.
  u32x4 az[K::NCH][K::NA], ar[K::NCH][K::NA], bw[K::NB];
  auto load_a = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    if (a.dbg & 4) return;
    const uint32_t cb = (uint32_t)((kbeg + k * K::CC) * 4);
#pragma unroll
    for (int u = 0; u < K::NA; ++u) {
      const uint32_t off = a_off[u] == kOOB ? kOOB : a_off[u] + cb;
      az[k][u] = __builtin_amdgcn_raw_buffer_load_b128(rsZ, (int)off, 0, 0);
      if constexpr (RK != 0) ar[k][u] = __builtin_amdgcn_raw_buffer_load_b128(rsR, (int)off, 0, 0);
    }
  };
  auto load_b = [&](int k) {
    if (a.dbg & 4) return;
    const uint32_t cb = (uint32_t)((kbeg + k * K::CC) * 4);
#pragma unroll
    for (int u = 0; u < K::NB; ++u) {
      const uint32_t off = b_off[u] == kOOB ? kOOB : b_off[u] + cb;
      bw[u] = __builtin_amdgcn_raw_buffer_load_b128(rsW, (int)off, 0, 0);
    }
  };
  // The fill of a chunk as NA + NB independent work units (unit u < NA: one
  // float4 of the input patch -> BN / residual / ReLU -> bf16 hi + lo -> LDS
  // and, for owner tiles, y / yp; unit NA + v: one packed weight float4 ->
  // hi / lo -> LDS).  The units of chunk k+1 are spread over the taps of
  // chunk k's MFMAs (their VALU / LDS writes issue under the matrix pipe).
  struct Coef4 {
    float4 sc, sh, s2, h2;
  };
  auto coef4 = [&](int k) {
    const int cl = k * K::CC + 4 * q;  // channel within the slice
    Coef4 c;
    c.sc = *reinterpret_cast<const float4*>(coef + cl);
    c.sh = *reinterpret_cast<const float4*>(coef + kchunk + cl);
    c.s2 = c.sc;
    c.h2 = c.sh;
    if constexpr (RK == 2) {
      c.s2 = *reinterpret_cast<const float4*>(coef + 2 * kchunk + cl);
      c.h2 = *reinterpret_cast<const float4*>(coef + 3 * kchunk + cl);
    }
    return c;
  };
  auto store_unit = [&](auto kc, auto uc, uint8_t* stage, const Coef4& cf) {
    constexpr int k = decltype(kc)::value, U = decltype(uc)::value;
    if constexpr (U < K::NA) {
      constexpr int u = U;
      const float4 zv = as_f4(az[k][u]);
      float4 v = make_float4(fmaf(zv.x, cf.sc.x, cf.sh.x), fmaf(zv.y, cf.sc.y, cf.sh.y),
                             fmaf(zv.z, cf.sc.z, cf.sh.z), fmaf(zv.w, cf.sc.w, cf.sh.w));
      if constexpr (RK == 1) {
        const float4 r = as_f4(ar[k][u]);
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
      } else if constexpr (RK == 2) {
        const float4 r = as_f4(ar[k][u]);
        v.x += fmaf(r.x, cf.s2.x, cf.h2.x);
        v.y += fmaf(r.y, cf.s2.y, cf.h2.y);
        v.z += fmaf(r.z, cf.s2.z, cf.h2.z);
        v.w += fmaf(r.w, cf.s2.w, cf.h2.w);
      }
      const float lo = X.relu ? 0.f : -__builtin_inff();
      v.x = fmaxf(v.x, lo); v.y = fmaxf(v.y, lo); v.z = fmaxf(v.z, lo); v.w = fmaxf(v.w, lo);
      const bool oob = a_off[u] == kOOB;  // padding is post-activation zero
      v.x = oob ? 0.f : v.x; v.y = oob ? 0.f : v.y; v.z = oob ? 0.f : v.z; v.w = oob ? 0.f : v.w;
      uint32_t h01, l01, h23, l23;
      split2(v.x, v.y, h01, l01);
      split2(v.z, v.w, h23, l23);
      uint8_t* d = stage + a_lds[u];
      *reinterpret_cast<uint2*>(d) = make_uint2(h01, h23);
      *reinterpret_cast<uint2*>(d + 32) = make_uint2(l01, l23);
      if (a_own[u]) {
        const uint32_t go = a_off[u] + (uint32_t)((kbeg + k * K::CC) * 4);  // pixel + chunk + 4q channels
        *reinterpret_cast<float4*>(reinterpret_cast<uint8_t*>(X.y) + go) = v;
        if (X.yp)
          *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(X.yp) + go) =
              make_uint4((h01 << 16) | (l01 & 0xffffu), (h01 & 0xffff0000u) | (l01 >> 16),
                         (h23 << 16) | (l23 & 0xffffu), (h23 & 0xffff0000u) | (l23 >> 16));
      }
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
  auto store = [&](auto kc, uint8_t* stage) {
    const Coef4 cf = coef4(decltype(kc)::value);
    static_for<NU>([&](auto uc) { store_unit(kc, uc, stage, cf); });
  };

  static_for<K::NCH>([&](auto kc) { load_a(kc); });
  load_b(0);
  // ---- coefficients of this slice's input channels ----
  {
    const bool publish = X.train && bx == 0 && by == 0;
    for (int c = t; c < kchunk; c += K::NTHR) {
      float sc = 1.f, sh = 0.f;
      if (X.has_bn) bn_coef(X.bn, C, kbeg + c, X.M, X.train, publish, sc, sh);
      coef[c] = sc;
      coef[kchunk + c] = sh;
      if constexpr (RK == 2) {
        float s2, h2;
        bn_coef(X.bnr, C, kbeg + c, X.M, X.train, publish, s2, h2);
        coef[2 * kchunk + c] = s2;
        coef[3 * kchunk + c] = h2;
      }
    }
  }

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
        al[S][i] = *reinterpret_cast<const bf16x8*>(st + fa_off[i] + AO + 32);
      }
#pragma unroll
      for (int j = 0; j < K::TN; ++j) {
        bh[S][j] = *reinterpret_cast<const bf16x8*>(st + fb_off[j] + BO);
        bl[S][j] = *reinterpret_cast<const bf16x8*>(st + fb_off[j] + BO + 32);
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
            acc[i][j] = mfma_bf16x16(al[S][i], bh[S][j], acc[i][j]);
            acc[i][j] = mfma_bf16x16(ah[S][i], bl[S][j], acc[i][j]);
            acc[i][j] = mfma_bf16x16(ah[S][i], bh[S][j], acc[i][j]);
          }
      }
      side(tapc);  // fill units of the next chunk, behind this tap's MFMAs
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  // LDS-only barrier: the owner-write global stores and the next chunk's
  // loads stay in flight (__syncthreads would drain vmcnt)
  auto bar = [&]() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes / reads done
    lds_barrier();
  };

  __syncthreads();  // coefficients visible
  stamp(a, 1);
  store(IC<0>{}, smem);
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

  // ---- epilogue: tile through LDS, split-K reduce, output + BN sums ----
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
    for (int z = 0; z < splits; ++z) {
#pragma unroll
      for (int u = 0; u < F; ++u) {
        const int f = t + K::NTHR * u;
        float4 r;
        if (z == bz) {
          r = *reinterpret_cast<const float4*>(tile + (f / C4) * K::TST + (f % C4) * 4);
        } else {
          r = as_f4(__builtin_amdgcn_raw_buffer_load_b128(rsS, (int)(z * zstride + f * 16), 0, 16));
        }
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
  // output rows: float4 per thread per pass
  constexpr int RPP = K::NTHR / C4;
  const int cg = t % C4, r0 = t / C4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), sq = s;
  for (int rl = r0; rl < K::MT; rl += RPP) {
    const int img = rl / (K::TH * K::TW);
    const int r2 = rl - img * (K::TH * K::TW);
    const int y = r2 / K::TW, x = r2 - y * K::TW;
    if (img0 + img >= a.N) continue;
    const float4 v = *reinterpret_cast<const float4*>(tile + rl * K::TST + cg * 4);
    const int64_t pix = ((int64_t)(img0 + img) * a.H + y0 + y) * a.W + x0 + x;
    *reinterpret_cast<float4*>(a.out + pix * a.Co + n0 + cg * 4) = v;
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    sq.x += v.x * v.x; sq.y += v.y * v.y; sq.z += v.z * v.z; sq.w += v.w * v.w;
  }
  stamp(a, 7);
  if (!a.stats) return;
  double* stats = a.stats + (int64_t)((bx + by * gridDim.x) % a.reps) * 2 * a.Co;
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
  if (p.stage && p.grid.x * p.grid.y > 1024) p.stage = 0;  // counter block
  if (p.stage && p.kchunk != 64) p.stage = 0;               // Cfg::KCH
  return p;
}

template <class K, int RK>
void go(const FwdArgs& a, const Plan& p, hipStream_t s) {
  const size_t lds = (size_t)K::LDS_MAIN + 4 * (size_t)p.kchunk * sizeof(float);
  static bool init = false;
  if (!init) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&hconv_fwd_kernel<K, RK>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    init = true;
  }
  hconv_fwd_kernel<K, RK><<<p.grid, K::NTHR, lds, s>>>(a, p.kchunk);
}

template <class K>
void go_rk(const FwdArgs& a, const Plan& p, hipStream_t s) {
  if (a.x.zr) go<K, 2>(a, p, s);
  else if (a.x.res) go<K, 1>(a, p, s);
  else go<K, 0>(a, p, s);
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

}  // namespace hc
}  // namespace mfl
