// Kernels of the controller's device aggregation backend (engine/device_agg.h).
//
// Every model lives in ONE packed device buffer (variables 256-B aligned), so a
// whole-model rule is one launch over a tile table: tile t covers up to
// kTileBytes of one variable and carries that variable's dtype.  A workgroup
// handles one tile with 16-B vector loads per lane (4 x fp32, 2 x fp64, ...),
// which is what an HBM-bound multi-tensor op wants (cdna_hip_programming.md
// Guideline 13); ~2,700 tiles for a 43 MB model fill the 256 CUs many times.
//
// Arithmetic is the host rule's, term by term (aggregation.cc): the scaled
// term is converted back to T before the add, in learner order, and no FMA
// contraction is allowed -- the device result is byte-identical to the host.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine/device_agg_kernels.h"

#pragma clang fp contract(off)

namespace mfl {
namespace devagg {
namespace {

template <typename T>
struct alignas(16) Vec {
  T v[16 / sizeof(T)];
};

template <typename T>
__device__ __forceinline__ T wrap_add(T a, T b) {
  return (T)(a + b);
}
template <typename T>
__device__ __forceinline__ T wrap_sub(T a, T b) {
  return (T)(a - b);
}
template <typename T>
__device__ __forceinline__ T term(T x, double w) {
  return (T)((double)x * w);
}

template <typename T>
__device__ void wsum_tile(char* __restrict__ out, const WSumArgs& a, uint64_t off, uint32_t n,
                          int accumulate) {
  constexpr int V = 16 / sizeof(T);
  T* o = reinterpret_cast<T*>(out + off);
  const uint32_t nv = n / V;
  for (uint32_t i = threadIdx.x; i < nv; i += blockDim.x) {
    Vec<T> acc;
    if (accumulate) {
      acc = reinterpret_cast<const Vec<T>*>(o)[i];
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) acc.v[j] = (T)0;
    }
    for (int k = 0; k < a.count; ++k) {
      const Vec<T> x = reinterpret_cast<const Vec<T>*>(a.x[k] + off)[i];
      const double w = a.w[k];
#pragma unroll
      for (int j = 0; j < V; ++j) acc.v[j] = wrap_add<T>(acc.v[j], term<T>(x.v[j], w));
    }
    reinterpret_cast<Vec<T>*>(o)[i] = acc;
  }
  for (uint32_t i = nv * V + threadIdx.x; i < n; i += blockDim.x) {
    T acc = accumulate ? o[i] : (T)0;
    for (int k = 0; k < a.count; ++k)
      acc = wrap_add<T>(acc, term<T>(reinterpret_cast<const T*>(a.x[k] + off)[i], a.w[k]));
    o[i] = acc;
  }
}

template <typename T>
__device__ __forceinline__ T roll1(T y, T x, double w, int op) {
  switch (op) {
    case ROLL_ADD: return wrap_add<T>(y, term<T>(x, w));
    case ROLL_SUB: return wrap_sub<T>(y, term<T>(x, w));
    case ROLL_MUL: return (T)((double)x * w);
    case ROLL_DIV: return (T)((double)x / w);
    default: return x;  // ROLL_COPY
  }
}

// y = roll(y, x, w): ADD / SUB merge x into y; MUL / DIV / COPY write
// y = f(x) (x may alias y).
template <typename T>
__device__ void roll_tile(char* y_, const char* x_, double w, int op, uint64_t off, uint32_t n) {
  constexpr int V = 16 / sizeof(T);
  T* y = reinterpret_cast<T*>(y_ + off);
  const T* x = reinterpret_cast<const T*>(x_ + off);
  const uint32_t nv = n / V;
  for (uint32_t i = threadIdx.x; i < nv; i += blockDim.x) {
    const Vec<T> xv = reinterpret_cast<const Vec<T>*>(x)[i];
    Vec<T> yv = xv;
    if (op == ROLL_ADD || op == ROLL_SUB) yv = reinterpret_cast<const Vec<T>*>(y)[i];
#pragma unroll
    for (int j = 0; j < V; ++j) yv.v[j] = roll1<T>(yv.v[j], xv.v[j], w, op);
    reinterpret_cast<Vec<T>*>(y)[i] = yv;
  }
  for (uint32_t i = nv * V + threadIdx.x; i < n; i += blockDim.x) y[i] = roll1<T>(y[i], x[i], w, op);
}

#define DEVAGG_DTYPE_SWITCH(dt, FN, ...)     \
  switch (dt) {                              \
    case 0: FN<int8_t>(__VA_ARGS__); break;  \
    case 1: FN<int16_t>(__VA_ARGS__); break; \
    case 2: FN<int32_t>(__VA_ARGS__); break; \
    case 3: FN<int64_t>(__VA_ARGS__); break; \
    case 4: FN<uint8_t>(__VA_ARGS__); break; \
    case 5: FN<uint16_t>(__VA_ARGS__); break;\
    case 6: FN<uint32_t>(__VA_ARGS__); break;\
    case 7: FN<uint64_t>(__VA_ARGS__); break;\
    case 8: FN<float>(__VA_ARGS__); break;   \
    case 9: FN<double>(__VA_ARGS__); break;  \
    default: break;                          \
  }

__global__ __launch_bounds__(256) void wsum_kernel(char* out, const Tile* __restrict__ tiles,
                                                   WSumArgs a, int accumulate) {
  const Tile t = tiles[blockIdx.x];
  DEVAGG_DTYPE_SWITCH(t.dtype, wsum_tile, out, a, t.off, t.n, accumulate);
}

__global__ __launch_bounds__(256) void roll_kernel(char* y, const char* x, const Tile* __restrict__ tiles,
                                                   double w, int op) {
  const Tile t = tiles[blockIdx.x];
  DEVAGG_DTYPE_SWITCH(t.dtype, roll_tile, y, x, w, op, t.off, t.n);
}

__device__ __forceinline__ uint64_t mulmod_shoup(uint64_t a, uint64_t w, uint64_t wp, uint64_t q) {
  const uint64_t hi = __umul64hi(a, wp);
  const uint64_t r = a * w - hi * q;
  return r >= q ? r - q : r;
}

// out[j] (+)= SUM_i w_i * ct_i[j] mod q, limb = (j / N) % L.
__global__ __launch_bounds__(256) void pwa_kernel(PwaArgs a, const uint64_t* __restrict__ wtab,
                                                  const uint64_t* __restrict__ q, uint64_t* out,
                                                  uint32_t L, uint32_t N, uint64_t total,
                                                  int accumulate) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += stride) {
    const uint32_t limb = (uint32_t)((j / N) % L);
    const uint64_t qq = q[limb];
    uint64_t acc = accumulate ? out[j] : 0;
    for (int i = 0; i < a.count; ++i) {
      const uint64_t* w = wtab + ((uint64_t)(a.first + i) * L + limb) * 2;
      acc += mulmod_shoup(a.ct[i][j], w[0], w[1], qq);
      acc = acc >= qq ? acc - qq : acc;
    }
    out[j] = acc;
  }
}

}  // namespace

int launch_wsum(char* out, const Tile* tiles, int ntiles, const WSumArgs& a, bool accumulate,
                hipStream_t s) {
  if (ntiles <= 0) return 0;
  hipLaunchKernelGGL(wsum_kernel, dim3(ntiles), dim3(256), 0, s, out, tiles, a, accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

int launch_roll(char* y, const char* x, const Tile* tiles, int ntiles, double w, int op,
                hipStream_t s) {
  if (ntiles <= 0) return 0;
  hipLaunchKernelGGL(roll_kernel, dim3(ntiles), dim3(256), 0, s, y, x, tiles, w, op);
  return (int)hipGetLastError();
}

int launch_pwa(const PwaArgs& a, const uint64_t* wtab, const uint64_t* q, uint64_t* out, uint32_t L,
               uint32_t N, uint64_t total, bool accumulate, hipStream_t s) {
  if (total == 0) return 0;
  uint64_t g = (total + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(pwa_kernel, dim3((unsigned)g), dim3(256), 0, s, a, wtab, q, out, L, N, total,
                     accumulate ? 1 : 0);
  return (int)hipGetLastError();
}

}  // namespace devagg
}  // namespace mfl
