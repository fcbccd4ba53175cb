// K1 / K2 / K8 / K9: device-side model aggregation kernels.
//
// * weighted_sum  (K1)  out = SUM_k (T)((double)x_k * w_k), accumulated in T
//   in learner order.  This is bit-for-bit the arithmetic of the reference's
//   FedAvg (metisfl/controller/aggregation/federated_average.cc:14-37): every
//   scaled term is converted back to the tensor's own type before the add, so
//   integer tensors truncate per term (gtest federated_average_test.cc:106-110)
//   and fp32 tensors round per term.  One launch covers every variable of the
//   model because the engine stores each model as one flat byte buffer.
// * merge / scale (K2)  the rolling-average primitives of
//   federated_rolling_average_base.cc:18-171 (l -/+= (T)(r*w); t = (T)(t*/z)).
// * count_zeros   (K8)  per-variable zero counts for TensorQuantifier
//   (proto_tensor_serde.h:35-50, controller.cc:952-1004), one launch over a
//   tile table.
// * ckks_pwa      (K9)  private weighted average over RNS-CKKS ciphertexts:
//   per limb modular scalar-multiply + add with Shoup precomputation
//   (replaces ckks_scheme.cc:164-206 EvalMult/EvalAdd).
#include "kernels/common.h"
#include "kernels/launchers.h"

// Bit-exactness with the host reference requires separate multiply and add
// roundings: no FMA contraction of `acc + x * w` (it changes fp64 results).
#pragma clang fp contract(off)

namespace mfl {

template <typename T>
struct Wrap {  // wrapping add/sub for integer types (std::plus<T> + narrowing)
  __device__ static T add(T a, T b) { return (T)(a + b); }
  __device__ static T sub(T a, T b) { return (T)(a - b); }
};

template <typename T>
__device__ __forceinline__ T scale_term(T x, double w) {
  return (T)((double)x * w);
}

template <typename T>
__global__ __launch_bounds__(256) void weighted_sum_kernel(T* __restrict__ out, AggInputs in,
                                                           int64_t n, int accumulate) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    T acc = accumulate ? out[i] : (T)0;
    for (int k = 0; k < in.count; ++k) {
      const T x = reinterpret_cast<const T*>(in.ptr[k])[i];
      acc = Wrap<T>::add(acc, scale_term<T>(x, in.w[k]));
    }
    out[i] = acc;
  }
}

template <typename T>
static void ws_launch(void* out, const AggInputs& in, int64_t n, bool acc, hipStream_t s) {
  weighted_sum_kernel<T><<<stream_grid(n, 256, 4096), 256, 0, s>>>(reinterpret_cast<T*>(out), in, n,
                                                                    acc ? 1 : 0);
}

#define MFL_DTYPE_SWITCH(dtype, FN, ...)                 \
  switch (dtype) {                                       \
    case 0: FN<int8_t>(__VA_ARGS__); break;              \
    case 1: FN<int16_t>(__VA_ARGS__); break;             \
    case 2: FN<int32_t>(__VA_ARGS__); break;             \
    case 3: FN<int64_t>(__VA_ARGS__); break;             \
    case 4: FN<uint8_t>(__VA_ARGS__); break;             \
    case 5: FN<uint16_t>(__VA_ARGS__); break;            \
    case 6: FN<uint32_t>(__VA_ARGS__); break;            \
    case 7: FN<uint64_t>(__VA_ARGS__); break;            \
    case 8: FN<float>(__VA_ARGS__); break;               \
    case 9: FN<double>(__VA_ARGS__); break;              \
    default: break;                                      \
  }

void launch_weighted_sum(int dtype, void* out, const AggInputs& in, int64_t n, bool accumulate,
                         hipStream_t s) {
  MFL_DTYPE_SWITCH(dtype, ws_launch, out, in, n, accumulate, s);
}

// mode (encoded in a,b): y = y*? ... we expose the four reference ops:
//   a == 0 : MERGE  y = y + (T)(x*b)         (b may be negative -> subtraction form below)
// The host wrapper maps MergeTensors(ADD/SUB) and ScaleTensors(MUL/DIV).
template <typename T>
__global__ __launch_bounds__(256) void rolling_kernel(T* __restrict__ y, const T* __restrict__ x,
                                                      double w, int op, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    switch (op) {
      case 0: y[i] = Wrap<T>::add(y[i], scale_term<T>(x[i], w)); break;   // MERGE ADD
      case 1: y[i] = Wrap<T>::sub(y[i], scale_term<T>(x[i], w)); break;   // MERGE SUB
      case 2: y[i] = (T)((double)y[i] * w); break;                       // SCALE MUL
      case 3: y[i] = (T)((double)y[i] / w); break;                       // SCALE DIV
    }
  }
}

template <typename T>
static void roll_launch(void* y, const void* x, double w, int op, int64_t n, hipStream_t s) {
  rolling_kernel<T><<<stream_grid(n, 256, 4096), 256, 0, s>>>(reinterpret_cast<T*>(y),
                                                               reinterpret_cast<const T*>(x), w, op, n);
}

// a selects the op (0 add,1 sub,2 mul,3 div), b is the scaling factor.
void launch_axpby(int dtype, void* y, const void* x, double a, double b, int64_t n, hipStream_t s) {
  MFL_DTYPE_SWITCH(dtype, roll_launch, y, x, b, (int)a, n, s);
}

template <typename T>
__global__ __launch_bounds__(256) void count_zeros_kernel(const T* __restrict__ x,
                                                          const int64_t* __restrict__ tseg,
                                                          const int64_t* __restrict__ tbeg,
                                                          const int64_t* __restrict__ tend,
                                                          unsigned long long* __restrict__ counts) {
  const int t = blockIdx.x;
  const int64_t b = tbeg[t], e = tend[t];
  unsigned long long c = 0;
  for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x) c += (x[i] == (T)0);
  c = wave_sum(c);
  __shared__ unsigned long long red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long tot = red[0] + red[1] + red[2] + red[3];
    if (tot) atomicAdd(&counts[tseg[t]], tot);
  }
}

template <typename T>
static void cz_launch(const void* x, const int64_t* ts, const int64_t* tb, const int64_t* te,
                      int ntiles, unsigned long long* counts, hipStream_t s) {
  count_zeros_kernel<T><<<ntiles, 256, 0, s>>>(reinterpret_cast<const T*>(x), ts, tb, te, counts);
}

void launch_count_zeros(int dtype, const void* x, const int64_t* tile_seg, const int64_t* tile_beg,
                        const int64_t* tile_end, int ntiles, unsigned long long* counts,
                        hipStream_t s) {
  if (ntiles <= 0) return;
  MFL_DTYPE_SWITCH(dtype, cz_launch, x, tile_seg, tile_beg, tile_end, ntiles, counts, s);
}

// ---------------------------------------------------------------------------
// K9: RNS-CKKS private weighted average.
// cts[i] points at learner i's ciphertext limbs laid out [nct][2 polys][nlimbs][N];
// wq[(i*nlimbs + j)*2 + {0,1}] = {w_ij, shoup(w_ij)} with w_ij = round(w_i*Delta_w) mod q_j.
__device__ __forceinline__ uint64_t mulmod_shoup(uint64_t a, uint64_t w, uint64_t wp, uint64_t q) {
  const uint64_t hi = __umul64hi(a, wp);
  uint64_t r = a * w - hi * q;
  return r >= q ? r - q : r;
}

__global__ __launch_bounds__(256) void ckks_pwa_kernel(const uint64_t* const* __restrict__ cts,
                                                       const uint64_t* __restrict__ wq, int L,
                                                       uint64_t* __restrict__ out,
                                                       const uint64_t* __restrict__ moduli,
                                                       int nlimbs, int64_t ncoef, int64_t total) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int limb = (int)((i / ncoef) % nlimbs);
    const uint64_t q = moduli[limb];
    uint64_t acc = 0;
    for (int l = 0; l < L; ++l) {
      const uint64_t a = cts[l][i];
      const uint64_t* w = wq + ((int64_t)l * nlimbs + limb) * 2;
      acc += mulmod_shoup(a, w[0], w[1], q);
      acc = acc >= q ? acc - q : acc;
    }
    out[i] = acc;
  }
}

void launch_ckks_pwa(const uint64_t* const* cts, const uint64_t* wq, int nlearners, uint64_t* out,
                     const uint64_t* moduli, int nlimbs, int64_t coeffs_per_limb, int64_t nct,
                     hipStream_t s) {
  const int64_t total = nct * 2 * nlimbs * coeffs_per_limb;
  ckks_pwa_kernel<<<stream_grid(total, 256, 4096), 256, 0, s>>>(cts, wq, nlearners, out, moduli,
                                                                 nlimbs, coeffs_per_limb, total);
}

}  // namespace mfl
