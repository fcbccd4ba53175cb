// K6 throughput-regime backward convolutions (fp32 operands, bf16 matrix
// pipe): weight gradient and input gradient of a 3x3 / stride-1 layer for the
// co-located regime (models/colocated.py: several learners' launches share
// the GPU, so each launch is judged by MFMA work per operand byte and per
// LDS instruction, not by its latency).
//
// The reference hands this loop to Keras (metisfl/models/keras/
// keras_model_ops.py:156-164, fp32 Conv2D training); conv32.hip is the
// latency-regime implementation of the same products.
//
// ---- the pair-expanded formulation ---------------------------------------
// Every fp32 operand arrives packed: dword = hi << 16 | lo with a = hi + lo +
// O(2^-18 |a|) (common.h split_pack).  Read as bf16, a packed row of n values
// IS a row of 2n bf16 values [lo0 hi0 lo1 hi1 ...].  With that view:
//
//  * weight gradient: dW'[(co,h1)][(j,h2)] = sum_m dY'[m][(co,h1)] X'[m][(j,h2)]
//    is a plain bf16 GEMM over the pixel index m on the raw packed operands,
//    and dW[co][j] = sum of the 2x2 block (lo.lo + lo.hi + hi.lo + hi.hi:
//    every cross product, the lo.lo one included).  Both operands are
//    m-major in memory, so both MFMA fragments come from ds_read_b64_tr_b16
//    transposing reads of LDS images filled by LDS-DMA: no decode VALU, no
//    b32 fragment reads (conv32.hip reads these with 8 ds_read_b32 + 8 v_perm
//    per fragment).
//  * input gradient: dX'[m][(ci,h)] = sum_{(tap,co,slot)} dY'[m][(tap,co,slot)]
//    W'[(tap,co,slot)][(ci,h)] where W'[(k,lo)][.] = W'[(k,hi)][.] = the
//    halves of W[co][tap][ci]: the A fragment is the raw packed dY row
//    (ds_read_b128, slots lo/hi interleaved) and the B fragment a transposing
//    read of the natural OHWI weight rows in which rows k and k are read twice
//    (lanes 4q+p of a 16-lane group give row q's address: rows co, co, co+1,
//    co+1).  dX[m][ci] = dX'[m][(ci,lo)] + dX'[m][(ci,hi)].
//
// 4 bf16 products per fp32 product (33 % more matrix work than conv32's 3
// hi/lo products), in exchange for zero decode VALU, one ds_read per 4 bytes
// of operand instead of one per 4 bytes + a v_perm, and 4 x 4 = 16 bytes of
// operand per expanded k-slot pair -- the same MFMA rate per operand byte as
// a bf16 GEMM of twice the size.  Accuracy: every product's relative error is
// that of the hi + lo representation of its two factors (~2^-17), i.e. the
// bf16x3 bound without its dropped lo.lo term.
//
// ---- staging ----------------------------------------------------------------
// 512-thread workgroups (WM x WN waves of TM x TN 32x32 MFMA tiles, 2 waves
// per SIMD, one workgroup per CU), k-tiles of 32 (pixels for wgrad, channels
// of one tap for dgrad), an NS-stage LDS ring filled by LDS-DMA (16 B per
// lane, hardware bounds checks zero-fill the padding) with counted vmcnt
// waits, one barrier per k-tile.  Sizing (measured, round 5): at 128 x 128
// expanded tiles and 3 x 16 KiB stages the kernels ran at 16-35 % of the
// MFMA rate -- the operand stream needs ~64 B/clk/CU at full rate and two
// 16 KiB tiles in flight cover ~0.3 us of LDS-DMA latency, not the ~1 us it
// takes under load.  So: 256 x 256 (or 128 x 512) expanded tiles (24-40
// B/clk/CU at full rate), 32-40 KiB stages, 2-3 of them in flight.
// Transposing reads use 4-row blocks whose 16-B chunks are XOR-swizzled by
// 4 * (row & 3) (the DMA source address carries the swizzle; LDS stays
// lane-linear), which puts a 32-lane half's 4 rows x 64 B on 16 distinct bank
// slots.  Workgroups are dealt XCD-contiguously (consecutive virtual tiles on
// one XCD's L2): a wgrad split's tiles all read the same dY rows and nearly
// the same X rows, neighbouring dgrad pixel tiles share their halo rows.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "kernels/common.h"
#include "kernels/lds_tiles.h"
#include "kernels/tconv.h"

namespace mfl {
namespace tc {

namespace {

template <int V>
using IC = std::integral_constant<int, V>;
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(IC<I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)p;
}

// ds_read_b64_tr_b16 through inline asm (the builtin makes hipcc drain every
// LDS-DMA in flight first, lds_tiles.h).  A read address is kept per 64-KiB
// LDS window (base + 65536 w), so every ring-stage offset is an immediate.
template <int OFF, int NW>
__device__ __forceinline__ v4s tr_read(const uint32_t (&addr)[NW]) {
  static_assert(OFF >= 0 && (OFF >> 16) < NW, "LDS offset beyond the address windows");
  v4s r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr[OFF >> 16]), "n"(OFF & 0xFFFF));
  return r;
}
template <int OFF, int NW>
__device__ __forceinline__ bf16x8 read_b128(const uint32_t (&addr)[NW]) {
  static_assert(OFF >= 0 && (OFF >> 16) < NW, "LDS offset beyond the address windows");
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr[OFF >> 16]), "n"(OFF & 0xFFFF));
  return r;
}
template <int NW>
__device__ __forceinline__ void windows(uint32_t a, uint32_t (&w)[NW]) {
#pragma unroll
  for (int k = 0; k < NW; ++k) w[k] = a + 65536u * k;
}
// Bijective XCD-contiguous deal: the hardware hands block b to XCD b % 8;
// virtual tile v runs on XCD v / ceil-share (cdna_hip_programming.md T1).
__device__ __forceinline__ int xcd_remap(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}
__device__ __forceinline__ bf16x8 cat8(const v4s& a, const v4s& b) {
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
#ifndef MFL_TC_SETPRIO
#define MFL_TC_SETPRIO 1
#endif
constexpr bool kSetPrio = MFL_TC_SETPRIO != 0;  // s_setprio(1) around each MFMA cluster (T5)

template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void pin(bf16x8 (&f)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
}

// ============================================================================
// weight gradient
// ============================================================================
struct WgArgs {
  Geom g;
  const uint32_t* x;
  const uint32_t* dy;
  float* dw;
  uint32_t x_bytes, dy_bytes;
  int mchunk;  // pixels per split (multiple of 32)
  int tiles_i, tiles_j;
  int lgQ, lgPQ;
  int store;  // one split: plain stores into dw (caller: dw is zero / overwritten)
};

// BM: expanded dW rows (2 x output channels), BN: expanded columns (2 x
// (r, s, c) entries; a column tile may span several taps when C < BN / 2).
template <int BM, int BN, int WM, int WN, int NS, int OCC>
__global__ __launch_bounds__(64 * WM * WN, 1) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void wgrad_kernel(WgArgs args) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // by value: lambdas capturing the kernel argument by reference made hipcc
  // copy the whole struct to scratch
  const WgArgs a = args;
  constexpr int NWV = WM * WN, NT = 64 * NWV;
  constexpr int ARB = BM * 2, BRB = BN * 2;  // LDS row bytes (packed dwords)
  constexpr int A_BYTES = 32 * ARB, B_BYTES = 32 * BRB, STAGE = A_BYTES + B_BYTES;
  constexpr int AI = A_BYTES / 1024 / NWV, BI = B_BYTES / 1024 / NWV, L = AI + BI;
  constexpr int A_CPR = ARB / 16, B_CPR = BRB / 16;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int RPS = 2 * (TM + TN);  // LDS reads per 16-pixel substep
  static_assert(A_CPR % 16 == 0 && B_CPR % 16 == 0, "row starts must be bank-window aligned");
  constexpr int NWIN = (NS * STAGE + 65535) / 65536;
  static_assert(AI * NWV * 1024 == A_BYTES && BI * NWV * 1024 == B_BYTES, "DMA split over the waves");
  static_assert(A_CPR >= 16 && B_CPR >= 16, "rows too short for the transposing-read swizzle");
  static_assert(RPS <= 15, "lgkmcnt is 4 bits");
  static_assert((NS - 2) * L <= 63, "vmcnt is 6 bits");
  // geometry as scalars (a Geom captured by the lambdas went to scratch)
  const int gN = a.g.N, gH = a.g.H, gW = a.g.W, gC = a.g.C, gCo = a.g.Co, gKS = a.g.KS, gST = a.g.ST,
            gpad = a.g.pad, gP = a.g.P, gQ = a.g.Q;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int ntile = a.tiles_i * a.tiles_j;
  const int v = xcd_remap(blockIdx.x, gridDim.x);
  const int split = v / ntile;
  const int tile = v - split * ntile;
  const int ti = tile % a.tiles_i, tj = tile / a.tiles_i;
  const int co0 = ti * (BM / 2);
  const int j0 = tj * (BN / 2);
  const int K = gKS * gKS * gC;
  const int M = gN * gP * gQ;
  const int mbeg = split * a.mchunk;
  const int mend = min(M, mbeg + a.mchunk);
  const int nk = max(0, (mend - mbeg) >> 5);
  const auto rsA = make_rsrc(a.dy, a.dy_bytes);
  const auto rsB = make_rsrc(a.x, a.x_bytes);

  // ---- DMA lane constants (the XOR swizzle lives in the source address) ----
  uint32_t a_off[AI];
  int b_row[BI], b_fr[BI], b_fs[BI];
  uint32_t b_coff[BI];
  // a lane's 16-B LDS chunk (lane-linear DMA image; rows may straddle
  // instructions: 768-B rows at C = 64)
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int ci = (wave * AI + i) * 64 + lane;
    const int row = ci / A_CPR;
    const int logc = (ci % A_CPR) ^ (4 * (row & 3));
    a_off[i] = (uint32_t)((row * gCo + co0 + logc * 4) * 4);
  }
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int ci = (wave * BI + i) * 64 + lane;
    const int row = ci / B_CPR;
    const int logc = (ci % B_CPR) ^ (4 * (row & 3));
    const int j = j0 + logc * 4;  // real (r, s, c) of this lane's 4 dwords
    const int tp = j / gC, c = j - tp * gC;
    b_row[i] = row;
    b_fr[i] = tp / gKS - gpad;
    b_fs[i] = tp - (tp / gKS) * gKS - gpad;
    b_coff[i] = (uint32_t)(c * 4);
  }
  const int pqm = (1 << a.lgPQ) - 1, qm = (1 << a.lgQ) - 1;

  auto issue = [&](int kt, auto stc) __attribute__((always_inline)) {
    constexpr int S = decltype(stc)::value;
    uint8_t* st = smem + S * STAGE;
    const int kb = mbeg + kt * 32;
    const bool kv = kb < mend;
    const uint32_t aoff = (uint32_t)kb * (uint32_t)gCo * 4u;
#pragma unroll
    for (int i = 0; i < AI; ++i) dma16(rsA, kv ? a_off[i] + aoff : kOOB, st + (wave * AI + i) * 1024);
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int m = kb + b_row[i];
      const int n = m >> a.lgPQ;
      const int rem = m & pqm;
      const int oy = rem >> a.lgQ, ox = rem & qm;
      const int iy = oy * gST + b_fr[i], ix = ox * gST + b_fs[i];
      const bool ok = kv & (iy >= 0) & (iy < gH) & (ix >= 0) & (ix < gW);
      const uint32_t off = (uint32_t)(((n * gH + iy) * gW + ix) * gC) * 4u + b_coff[i];
      dma16(rsB, ok ? off : kOOB, st + A_BYTES + (wave * BI + i) * 1024);
    }
  };

  // ---- fragment read addresses: block row q = lane>>2 & 3, piece p = lane & 3
  const int g4 = lane >> 4, hh = g4 >> 1, q = (lane >> 2) & 3, p = lane & 3;
  const uint32_t base = lds_addr(smem);
  uint32_t ar[TM][NWIN], br[TN][NWIN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int col = wm * (BM / WM) + 32 * i + 16 * (g4 & 1) + 4 * p;
    windows(base + (8 * hh + q) * ARB + ((((col >> 3) ^ (4 * q))) << 4) + ((col & 4) << 1), ar[i]);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * (BN / WN) + 32 * j + 16 * (g4 & 1) + 4 * p;
    windows(base + A_BYTES + (8 * hh + q) * BRB + ((((col >> 3) ^ (4 * q))) << 4) + ((col & 4) << 1), br[j]);
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  bf16x8 fa[2][TM], fb[2][TN];
  // reads of 16-pixel substep KS of ring stage S into fragment set F
  auto read = [&](auto sc, auto ksc, auto fc) __attribute__((always_inline)) {
    constexpr int S = decltype(sc)::value, KS = decltype(ksc)::value, F = decltype(fc)::value;
#pragma unroll
    for (int i = 0; i < TM; ++i)
      fa[F][i] = cat8(tr_read<S * STAGE + 16 * KS * ARB>(ar[i]), tr_read<S * STAGE + (16 * KS + 4) * ARB>(ar[i]));
#pragma unroll
    for (int j = 0; j < TN; ++j)
      fb[F][j] = cat8(tr_read<S * STAGE + 16 * KS * BRB>(br[j]), tr_read<S * STAGE + (16 * KS + 4) * BRB>(br[j]));
  };
  auto mma = [&](auto fc) __attribute__((always_inline)) {
    constexpr int F = decltype(fc)::value;
    if constexpr (kSetPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(fa[F][i], fb[F][j], acc[i][j]);
    if constexpr (kSetPrio) __builtin_amdgcn_s_setprio(0);
  };

  // ---- k-loop: NS-stage ring, one barrier per 32-pixel tile ----------------
  sfor<NS - 1>([&](auto u) __attribute__((always_inline)) { issue(decltype(u)::value, u); });
  auto step = [&](int kt, auto sc) __attribute__((always_inline)) {
    constexpr int S = decltype(sc)::value;
    constexpr int NXT = (S + NS - 1) % NS;
    wait_vmcnt<(NS - 2) * L>();  // own DMAs of tile kt landed
    lds_barrier();               // everyone's landed; everyone done with tile kt-1
    issue(kt + NS - 1, IC<NXT>{});
    read(sc, IC<0>{}, IC<0>{});
    read(sc, IC<1>{}, IC<1>{});
    lgkm_wait<RPS>();
    pin(fa[0]);
    pin(fb[0]);
    mma(IC<0>{});
    lgkm_wait<0>();
    pin(fa[1]);
    pin(fb[1]);
    mma(IC<1>{});
  };
  int kt = 0;
  for (; kt + NS <= nk; kt += NS) sfor<NS>([&](auto j) __attribute__((always_inline)) { step(kt + decltype(j)::value, j); });
  sfor<NS - 1>([&](auto j) __attribute__((always_inline)) {
    if (kt + decltype(j)::value < nk) step(kt + decltype(j)::value, j);
  });
  wait_vmcnt<0>();

  // ---- epilogue: 2x2 fold (rows = regs e, e+1; columns = lanes l, l^1) ----
  const int odd = lane & 1;
  const int colr = (lane & 31) >> 1;
  float* dw = a.dw;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float v8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v8[u] = acc[i][j][2 * u] + acc[i][j][2 * u + 1];
        v8[u] += __shfl_xor(v8[u], 1, 64);
      }
      const int jj = j0 + wn * (BN / WN / 2) + 16 * j + colr;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int tt = u + 4 * odd;
        // bitwise select (a ?: here became a dynamically indexed scratch array)
        const uint32_t msk = 0u - (uint32_t)odd;
        const float val = __uint_as_float((__float_as_uint(v8[u]) & ~msk) | (__float_as_uint(v8[u + 4]) & msk));
        const int co = co0 + wm * (BM / WM / 2) + 16 * i + (tt & 1) + 4 * (tt >> 1) + 2 * (lane >> 5);
        float* dst = dw + (int64_t)co * K + jj;
        if (a.store)
          *dst = val;
        else
          atomicAdd(dst, val);
      }
    }
}

// ============================================================================
// input gradient
// ============================================================================
struct DgArgs {
  Geom g;
  const uint32_t* dy;
  const uint32_t* w;
  float* dx;
  uint32_t dy_bytes, w_bytes;
  int accum;
  Bnb bnb;
  float* ws;
  int* counters;
  int tiles_m, tiles_n, splits, ktps;  // k-tiles per split
  int lgW, lgHW;
};

// BM: dX pixels, BN: expanded input-channel columns (2 x ci).
template <int BM, int BN, int WM, int WN, int NS, int OCC>
__global__ __launch_bounds__(64 * WM * WN, 1) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void dgrad_kernel(DgArgs args) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const DgArgs a = args;
  constexpr int NWV = WM * WN, NT = 64 * NWV;
  constexpr int ARB = 128;     // 32 packed channels of one tap
  constexpr int BRB = BN * 2;  // W rows: BN / 2 packed input channels
  constexpr int A_BYTES = BM * ARB, B_BYTES = 32 * BRB, STAGE = A_BYTES + B_BYTES;
  constexpr int AI = A_BYTES / 1024 / NWV, BI = B_BYTES / 1024 / NWV, L = AI + BI;
  constexpr int B_RPI = 1024 / BRB, B_CPR = BRB / 16;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int RPS = TM + 2 * TN;  // LDS reads per 8-channel substep
  constexpr int NWIN = (NS * STAGE + 65535) / 65536;
  static_assert(AI * NWV * 1024 == A_BYTES && BI * NWV * 1024 == B_BYTES, "DMA split over the waves");
  static_assert(B_CPR >= 16, "rows too short for the transposing-read swizzle");
  static_assert(RPS <= 15, "lgkmcnt is 4 bits");
  static_assert((NS - 2) * L <= 63, "vmcnt is 6 bits");
  // geometry as scalars (a Geom captured by the lambdas went to scratch)
  const int gN = a.g.N, gH = a.g.H, gW = a.g.W, gC = a.g.C, gCo = a.g.Co, gKS = a.g.KS, gST = a.g.ST,
            gpad = a.g.pad, gP = a.g.P, gQ = a.g.Q;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int ntile = a.tiles_m * a.tiles_n;
  const int v = xcd_remap(blockIdx.x, gridDim.x);
  // virtual order: pixel tiles fastest (neighbours share halo rows), then
  // channel tiles, then split-K slices
  const int split = v / ntile;
  const int tile = v - split * ntile;
  const int tm = tile % a.tiles_m, tn = tile / a.tiles_m;
  const int m0 = tm * BM;
  const int ci0 = tn * (BN / 2);
  const int KK = gKS * gKS;
  const int CC = gCo >> 5;  // 32-channel chunks per tap
  const int nkt = KK * CC;
  const int kt0 = split * a.ktps;
  const int nk = max(0, min(nkt, kt0 + a.ktps) - kt0);
  const int M = gN * gH * gW;
  const auto rsA = make_rsrc(a.dy, a.dy_bytes);
  const auto rsB = make_rsrc(a.w, a.w_bytes);

  // A DMA (dY rows of the tap-shifted pixels): 8 rows of 128 B per instruction
  uint32_t a_base[AI], a_vm[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = (wave * AI + i) * 8 + (lane >> 3);
    const int logc = (lane & 7) ^ ((row >> 1) & 7);
    const int m = m0 + row;
    const int mm = m < M ? m : 0;
    const int n = mm >> a.lgHW;
    const int rem = mm & ((1 << a.lgHW) - 1);
    const int y = rem >> a.lgW, x = rem & ((1 << a.lgW) - 1);
    // dY pixel of tap (r, s): (y + pad - r, x + pad - s) (stride 1)
    a_base[i] = (uint32_t)((((n * gP + y + gpad) * gQ + x + gpad) * gCo + logc * 4) * 4);
    uint32_t vm = 0;
    for (int r = 0; r < gKS; ++r)
      for (int s = 0; s < gKS; ++s) {
        const int yy = y + gpad - r, xx = x + gpad - s;
        const bool ok = (m < M) & (yy >= 0) & (yy < gP) & (xx >= 0) & (xx < gQ);
        vm |= (uint32_t)ok << (r * gKS + s);
      }
    a_vm[i] = vm;
  }
  uint32_t b_off[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int row = (wave * BI + i) * B_RPI + lane / B_CPR;  // output channel within the k-tile
    const int logc = (lane % B_CPR) ^ (4 * (row & 3));
    b_off[i] = (uint32_t)(((row * KK) * gC + ci0 + logc * 4) * 4);
  }
  // scalar k-tile iterator, taps fastest: consecutive tiles read tap-shifted,
  // mostly overlapping dY rows of the same channel chunk (L1 / L2 hits)
  int kcc = kt0 / KK, ktap = kt0 - (kt0 / KK) * KK;

  auto issue = [&](int kt, auto stc) __attribute__((always_inline)) {
    constexpr int S = decltype(stc)::value;
    uint8_t* st = smem + S * STAGE;
    const bool kv = kt < nk;
    const int tp = kv ? ktap : 31;  // bit 31 never set: every row out of range
    const int fr = ktap / gKS, fs = ktap - fr * gKS;
    const uint32_t sh = (uint32_t)(((fr * gQ + fs) * gCo - kcc * 32) * 4);  // subtracted
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const bool ok = (a_vm[i] >> tp) & 1u;
      dma16(rsA, ok ? a_base[i] - sh : kOOB, st + (wave * AI + i) * 1024);
    }
    const uint32_t boff = (uint32_t)(((kcc * 32 * KK + ktap) * gC) * 4);
#pragma unroll
    for (int i = 0; i < BI; ++i) dma16(rsB, kv ? b_off[i] + boff : kOOB, st + A_BYTES + (wave * BI + i) * 1024);
    ktap += 1;
    const int wrap = ktap == KK;
    ktap = wrap ? 0 : ktap;
    kcc += wrap;
  };

  const int g4 = lane >> 4, hh = lane >> 5, q = (lane >> 2) & 3, p = lane & 3;
  const uint32_t base = lds_addr(smem);
  // A (b128 row reads): row = pixel, chunk 2 ks + hh of the 128-B row
  uint32_t ar[TM][4][NWIN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = wm * (BM / WM) + 32 * i + (lane & 31);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) windows(base + row * ARB + (((2 * ks + hh) ^ ((row >> 1) & 7)) << 4), ar[i][ks]);
  }
  // B (transposing reads, rows co, co, co+1, co+1 of each 4-row block)
  uint32_t br[TN][2][NWIN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * (BN / WN) + 32 * j + 16 * (g4 & 1) + 4 * p;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 4 * hh + 2 * h + (q >> 1);
      windows(base + A_BYTES + row * BRB + ((((col >> 3) ^ (4 * (row & 3)))) << 4) + ((col & 4) << 1), br[j][h]);
    }
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  bf16x8 fa[2][TM], fb[2][TN];
  auto read = [&](auto sc, auto ksc, auto fc) __attribute__((always_inline)) {
    constexpr int S = decltype(sc)::value, KS = decltype(ksc)::value, F = decltype(fc)::value;
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[F][i] = read_b128<S * STAGE>(ar[i][KS]);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      fb[F][j] = cat8(tr_read<S * STAGE + 8 * KS * BRB>(br[j][0]), tr_read<S * STAGE + 8 * KS * BRB>(br[j][1]));
  };
  auto mma = [&](auto fc) __attribute__((always_inline)) {
    constexpr int F = decltype(fc)::value;
    if constexpr (kSetPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(fa[F][i], fb[F][j], acc[i][j]);
    if constexpr (kSetPrio) __builtin_amdgcn_s_setprio(0);
  };

  sfor<NS - 1>([&](auto u) __attribute__((always_inline)) { issue(decltype(u)::value, u); });
  auto step = [&](int kt, auto sc) __attribute__((always_inline)) {
    constexpr int S = decltype(sc)::value;
    constexpr int NXT = (S + NS - 1) % NS;
    wait_vmcnt<(NS - 2) * L>();
    lds_barrier();
    issue(kt + NS - 1, IC<NXT>{});
    read(sc, IC<0>{}, IC<0>{});
    read(sc, IC<1>{}, IC<1>{});
    lgkm_wait<RPS>();
    pin(fa[0]);
    pin(fb[0]);
    mma(IC<0>{});
    read(sc, IC<2>{}, IC<0>{});
    lgkm_wait<RPS>();
    pin(fa[1]);
    pin(fb[1]);
    mma(IC<1>{});
    read(sc, IC<3>{}, IC<1>{});
    lgkm_wait<RPS>();
    pin(fa[0]);
    pin(fb[0]);
    mma(IC<0>{});
    lgkm_wait<0>();
    pin(fa[1]);
    pin(fb[1]);
    mma(IC<1>{});
  };
  int kt = 0;
  for (; kt + NS <= nk; kt += NS) sfor<NS>([&](auto j) __attribute__((always_inline)) { step(kt + decltype(j)::value, j); });
  sfor<NS - 1>([&](auto j) __attribute__((always_inline)) {
    if (kt + decltype(j)::value < nk) step(kt + decltype(j)::value, j);
  });
  wait_vmcnt<0>();
  __syncthreads();  // ring no longer read: the epilogue reuses smem

  // ---- fold column pairs (lanes l, l^1) into an fp32 tile [BM][BN/2 + 4] ----
  constexpr int TW = BN / 2, TST = TW + 4;
  float* tilep = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float vv = acc[i][j][e];
        vv += __shfl_xor(vv, 1, 64);
        if (!(lane & 1)) {
          const int rl = wm * (BM / WM) + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * hh;
          tilep[rl * TST + wn * (BN / WN / 2) + 16 * j + ((lane & 31) >> 1)] = vv;
        }
      }
  __syncthreads();

  // ---- split-K: write-through slabs + arrival ticket, last arriver sums ----
  constexpr int F4 = BM * TW / (4 * NT);  // float4 per thread
  constexpr int C4 = TW / 4;
  static_assert(F4 * 4 * NT == BM * TW, "tile / thread count");
  if (a.splits > 1) {
    const int64_t zstride = (int64_t)ntile * BM * TW;
    const auto rsS = make_rsrc(a.ws + (int64_t)tile * BM * TW, 0x7FFFFFF0u);
#pragma unroll
    for (int u = 0; u < F4; ++u) {
      const int f = t + NT * u;
      const float4 vv = *reinterpret_cast<const float4*>(tilep + (f / C4) * TST + (f % C4) * 4);
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{__float_as_uint(vv.x), __float_as_uint(vv.y), __float_as_uint(vv.z), __float_as_uint(vv.w)}, rsS,
          (int)((uint32_t)(split * zstride * 4) + f * 16), 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(tilep + BM * TST);
    if (t == 0) {
      const int prev = __hip_atomic_fetch_add(&a.counters[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == a.splits - 1;
      if (last) __hip_atomic_store(&a.counters[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    float4 sum[F4];
#pragma unroll
    for (int u = 0; u < F4; ++u) sum[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int z = 0; z < a.splits; ++z) {  // slice order: deterministic
#pragma unroll
      for (int u = 0; u < F4; ++u) {
        const int f = t + NT * u;
        float4 r;
        if (z == split) {
          r = *reinterpret_cast<const float4*>(tilep + (f / C4) * TST + (f % C4) * 4);
        } else {
          const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rsS, (int)((uint32_t)(z * zstride * 4) + f * 16), 0, 16);
          r = make_float4(__uint_as_float(b[0]), __uint_as_float(b[1]), __uint_as_float(b[2]), __uint_as_float(b[3]));
        }
        sum[u].x += r.x;
        sum[u].y += r.y;
        sum[u].z += r.z;
        sum[u].w += r.w;
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < F4; ++u) {
      const int f = t + NT * u;
      *reinterpret_cast<float4*>(tilep + (f / C4) * TST + (f % C4) * 4) = sum[u];
    }
    __syncthreads();
  }

  // ---- store (+ accumulate, + consumer-BN mask and backward sums) ----------
  constexpr int RPP = NT / C4;  // rows per pass
  const int cg = t % C4, r0 = t / C4;
  const int col = ci0 + cg * 4;
  const bool fuse = a.bnb.acc != nullptr;
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1, mu = s1, is = s1;
  if (fuse) {
    mu = *reinterpret_cast<const float4*>(a.bnb.mean + col);
    is = *reinterpret_cast<const float4*>(a.bnb.invstd + col);
  }
  for (int rl = r0; rl < BM; rl += RPP) {
    const int m = m0 + rl;
    if (m >= M) break;
    float4 vv = *reinterpret_cast<const float4*>(tilep + rl * TST + cg * 4);
    const int64_t off = (int64_t)m * gC + col;
    float4* dst = reinterpret_cast<float4*>(a.dx + off);
    if (a.accum) {
      const float4 o = *dst;
      vv.x += o.x;
      vv.y += o.y;
      vv.z += o.z;
      vv.w += o.w;
    }
    if (fuse) {
      if (a.bnb.y) {
        const float4 ym = *reinterpret_cast<const float4*>(a.bnb.y + off);
        vv.x = ym.x > 0.f ? vv.x : 0.f;
        vv.y = ym.y > 0.f ? vv.y : 0.f;
        vv.z = ym.z > 0.f ? vv.z : 0.f;
        vv.w = ym.w > 0.f ? vv.w : 0.f;
      }
      const float4 z = *reinterpret_cast<const float4*>(a.bnb.z + off);
      s1.x += vv.x;
      s1.y += vv.y;
      s1.z += vv.z;
      s1.w += vv.w;
      s2.x += vv.x * ((z.x - mu.x) * is.x);
      s2.y += vv.y * ((z.y - mu.y) * is.y);
      s2.z += vv.z * ((z.z - mu.z) * is.z);
      s2.w += vv.w * ((z.w - mu.w) * is.w);
    }
    *dst = vv;
  }
  if (!fuse) return;
  __syncthreads();
  float* red = tilep;
  reinterpret_cast<float4*>(red)[2 * t] = s1;
  reinterpret_cast<float4*>(red)[2 * t + 1] = s2;
  __syncthreads();
  if (t < TW) {
    const int cgi = t >> 2, k = t & 3;
    double sa = 0.0, sb = 0.0;
    for (int r = 0; r < RPP; ++r) {
      sa += red[(r * C4 + cgi) * 8 + k];
      sb += red[(r * C4 + cgi) * 8 + 4 + k];
    }
    double* acc2 = a.bnb.acc + (int64_t)(blockIdx.x % a.bnb.reps) * 2 * gC;
    atomicAdd(&acc2[ci0 + t], sa);
    atomicAdd(&acc2[gC + ci0 + t], sb);
  }
}

int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}
bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

template <typename K>
void lds_attr(K* kern, size_t lds) {
  if (lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

// ---- tile configurations ----------------------------------------------------
// Instantiated variants; the planners below pick one per shape, the
// MFL_TC_WG_CFG / MFL_TC_DG_CFG overrides (index) exist for sweeps
// (scripts/tconv_check.cpp).  OCC: waves per SIMD the register budget keeps.
template <int BM, int BN, int WM, int WN, int NS, int OCC>
void run_wg(const WgArgs& a, int nwg, hipStream_t s) {
  constexpr int STAGE = 32 * BM * 2 + 32 * BN * 2;
  constexpr size_t lds = (size_t)NS * STAGE;
  static bool attr = false;
  if (!attr) {
    lds_attr(&wgrad_kernel<BM, BN, WM, WN, NS, OCC>, lds);
    attr = true;
  }
  hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, NS, OCC>), dim3(nwg), dim3(64 * WM * WN), lds, s, a);
}
template <int BM, int BN, int WM, int WN, int NS, int OCC>
void run_dg(const DgArgs& a, int nwg, hipStream_t s) {
  constexpr int STAGE = BM * 128 + 32 * BN * 2;
  constexpr size_t lds = std::max((size_t)NS * STAGE, (size_t)(BM * (BN / 2 + 4) * 4 + 16));
  static bool attr = false;
  if (!attr) {
    lds_attr(&dgrad_kernel<BM, BN, WM, WN, NS, OCC>, lds);
    attr = true;
  }
  hipLaunchKernelGGL((dgrad_kernel<BM, BN, WM, WN, NS, OCC>), dim3(nwg), dim3(64 * WM * WN), lds, s, a);
}
struct CfgEntry {
  int bm, bn, wm, wn, ns;
  void (*wg)(const WgArgs&, int, hipStream_t);
  void (*dg)(const DgArgs&, int, hipStream_t);
};
const CfgEntry kWgCfg[] = {
    {128, 128, 2, 2, 3, run_wg<128, 128, 2, 2, 3, 2>, nullptr},
    {128, 384, 2, 4, 3, run_wg<128, 384, 2, 4, 3, 1>, nullptr},
    {256, 256, 2, 4, 3, run_wg<256, 256, 2, 4, 3, 1>, nullptr},
    {128, 256, 2, 2, 3, run_wg<128, 256, 2, 2, 3, 2>, nullptr},
    {256, 128, 2, 2, 3, run_wg<256, 128, 2, 2, 3, 2>, nullptr},
    {128, 128, 2, 2, 4, run_wg<128, 128, 2, 2, 4, 2>, nullptr},
    {256, 256, 2, 4, 4, run_wg<256, 256, 2, 4, 4, 1>, nullptr},
    {128, 384, 2, 4, 4, run_wg<128, 384, 2, 4, 4, 1>, nullptr},
};
const CfgEntry kDgCfg[] = {
    {128, 128, 2, 2, 3, nullptr, run_dg<128, 128, 2, 2, 3, 2>},
    {256, 128, 4, 2, 3, nullptr, run_dg<256, 128, 4, 2, 3, 1>},
    {256, 256, 4, 2, 3, nullptr, run_dg<256, 256, 4, 2, 3, 1>},
    {128, 256, 2, 2, 3, nullptr, run_dg<128, 256, 2, 2, 3, 1>},
    {128, 128, 2, 2, 4, nullptr, run_dg<128, 128, 2, 2, 4, 2>},
    {256, 128, 4, 2, 4, nullptr, run_dg<256, 128, 4, 2, 4, 1>},
};
constexpr int kNWg = sizeof(kWgCfg) / sizeof(kWgCfg[0]);
constexpr int kNDg = sizeof(kDgCfg) / sizeof(kDgCfg[0]);

bool wg_fits(const Geom& g, const CfgEntry& c) {
  return (2 * g.Co) % c.bm == 0 && (2 * g.KS * g.KS * g.C) % c.bn == 0;
}
bool dg_fits(const Geom& g, const CfgEntry& c) { return (2 * g.C) % c.bn == 0; }

// Plans measured in the co-located regime (8 learners' launches over 4
// streams, scripts/tconv_check.cpp, profiles/r5/tconv/): 128 x 128 tiles,
// ~256 workgroups per wgrad launch and ~128 per dgrad launch (at batch 32:
// wgrad 28 / 7 / 1 / 1 splits, dgrad 1 / 1 / 2 / 4 over the four stages);
// the 4-stage ring for the 8x8 / 4x4 weight gradients.
int wg_pick(const Geom& g, int cfg) {
  if (cfg < 0) cfg = env_int("MFL_TC_WG_CFG", -1);
  if (cfg >= 0 && cfg < kNWg && wg_fits(g, kWgCfg[cfg])) return cfg;
  return g.Co <= 128 ? 0 : 5;
}
int dg_pick(const Geom& g, int cfg) {
  if (cfg < 0) cfg = env_int("MFL_TC_DG_CFG", -1);
  if (cfg >= 0 && cfg < kNDg && dg_fits(g, kDgCfg[cfg])) return cfg;
  return 0;
}

}  // namespace

int num_wgrad_cfgs() { return kNWg; }
int num_dgrad_cfgs() { return kNDg; }
bool wgrad_cfg_fits(const Geom& g, int cfg) { return cfg >= 0 && cfg < kNWg && wg_fits(g, kWgCfg[cfg]); }
bool dgrad_cfg_fits(const Geom& g, int cfg) { return cfg >= 0 && cfg < kNDg && dg_fits(g, kDgCfg[cfg]); }

bool wgrad_ok(const Geom& g) {
  return g.KS == 3 && g.ST == 1 && g.pad == 1 && g.C % 64 == 0 && g.Co % 64 == 0 && pow2(g.P) && pow2(g.Q) &&
         (int64_t)g.N * g.P * g.Q % 32 == 0;
}
bool dgrad_ok(const Geom& g) {
  return g.KS == 3 && g.ST == 1 && g.pad == 1 && g.C % 64 == 0 && g.Co % 32 == 0 && pow2(g.H) && pow2(g.W) &&
         g.H == g.P && g.W == g.Q;
}

int wgrad_default_splits(const Geom& g, int cfg) {
  const CfgEntry& c = kWgCfg[wg_pick(g, cfg)];
  const int M = g.N * g.P * g.Q;
  const int ntile = (2 * g.Co / c.bm) * (2 * g.KS * g.KS * g.C / c.bn);
  const int target = env_int("MFL_TC_WG_TARGET", 256);
  int sp = std::max(1, target / ntile);
  sp = std::min(sp, std::max(1, M / 32 / 8));  // >= 8 k-tiles per split
  return sp;
}

void launch_wgrad(const Geom& g, const uint32_t* xp, const uint32_t* dyp, float* dw, int splits, hipStream_t s,
                  int cfg) {
  const CfgEntry& c = kWgCfg[wg_pick(g, cfg)];
  WgArgs a{};
  a.g = g;
  a.x = xp;
  a.dy = dyp;
  a.dw = dw;
  a.x_bytes = (uint32_t)((int64_t)g.N * g.H * g.W * g.C * 4);
  const int M = g.N * g.P * g.Q;
  a.dy_bytes = (uint32_t)((int64_t)M * g.Co * 4);
  a.tiles_i = 2 * g.Co / c.bm;
  a.tiles_j = 2 * g.KS * g.KS * g.C / c.bn;
  if (splits <= 0) splits = wgrad_default_splits(g, cfg);
  const int ktiles = M / 32;
  const int per = (ktiles + splits - 1) / splits;
  splits = (ktiles + per - 1) / per;
  a.mchunk = per * 32;
  a.lgQ = ilog2(g.Q);
  a.lgPQ = ilog2(g.P * g.Q);
  a.store = 0;
  c.wg(a, a.tiles_i * a.tiles_j * splits, s);
}

int dgrad_default_splits(const Geom& g, int cfg) {
  const CfgEntry& c = kDgCfg[dg_pick(g, cfg)];
  const int M = g.N * g.H * g.W;
  const int ntile = ((M + c.bm - 1) / c.bm) * (2 * g.C / c.bn);
  const int nkt = g.KS * g.KS * (g.Co / 32);
  const int target = env_int("MFL_TC_DG_TARGET", 128);
  int sp = std::max(1, target / std::max(1, ntile));
  sp = std::min(sp, std::max(1, nkt / 9));  // >= ~9 k-tiles per split
  return sp;
}
int64_t dgrad_workspace(const Geom& g, int splits, int cfg) {
  if (splits <= 1) return 0;
  const CfgEntry& c = kDgCfg[dg_pick(g, cfg)];
  const int M = g.N * g.H * g.W;
  const int ntile = ((M + c.bm - 1) / c.bm) * (2 * g.C / c.bn);
  return (int64_t)splits * ntile * c.bm * (c.bn / 2);
}
int dgrad_counters(const Geom& g, int cfg) {
  const CfgEntry& c = kDgCfg[dg_pick(g, cfg)];
  const int M = g.N * g.H * g.W;
  return ((M + c.bm - 1) / c.bm) * (2 * g.C / c.bn);
}

void launch_dgrad(const Geom& g, const uint32_t* dyp, const uint32_t* wp, float* dx, bool accum, const Bnb* bnb,
                  float* ws, int* counters, int splits, hipStream_t s, int cfg) {
  const CfgEntry& c = kDgCfg[dg_pick(g, cfg)];
  DgArgs a{};
  a.g = g;
  a.dy = dyp;
  a.w = wp;
  a.dx = dx;
  const int M = g.N * g.H * g.W;
  a.dy_bytes = (uint32_t)((int64_t)g.N * g.P * g.Q * g.Co * 4);
  a.w_bytes = (uint32_t)((int64_t)g.Co * g.KS * g.KS * g.C * 4);
  a.accum = accum ? 1 : 0;
  if (bnb) a.bnb = *bnb;
  a.ws = ws;
  a.counters = counters;
  a.tiles_m = (M + c.bm - 1) / c.bm;
  a.tiles_n = 2 * g.C / c.bn;
  const int nkt = g.KS * g.KS * (g.Co / 32);
  if (splits <= 0) splits = dgrad_default_splits(g, cfg);
  if (!ws || !counters) splits = 1;
  const int per = (nkt + splits - 1) / splits;
  a.splits = (nkt + per - 1) / per;
  a.ktps = per;
  a.lgW = ilog2(g.W);
  a.lgHW = ilog2(g.H * g.W);
  c.dg(a, a.tiles_m * a.tiles_n * a.splits, s);
}

}  // namespace tc
}  // namespace mfl
