// K10 / K11: RNS-CKKS encryption and decryption on the GPU.
//
// The reference encrypts each learner's model with Palisade on the CPU
// (metisfl/encryption/palisade/ckks_scheme.cc:109-162 Encrypt, :208-251
// Decrypt; OpenMP over 4096-slot chunks) -- for an 11.2M-parameter ResNet-18
// that is ~2.7k ciphertexts, tens of seconds per learner per round on a host.
// Here the whole model is encrypted / decrypted in a handful of launches,
// batched over every ciphertext at once, producing exactly the host scheme's
// byte layout (he/ckks.h: [nct][c0,c1][limb][N] u64 in NTT form, same
// twiddles, same keys), so device and host ciphertexts interoperate.
//
// Pipeline (one workgroup per ciphertext chunk or per (chunk, poly, limb) row):
//   encrypt: ckks_encode_sample  -- HEAAN special inverse FFT of the 4096
//              real slots in LDS (fp64 complex, 64 KiB), scale by Delta and
//              round, draw u (ternary) and e0 / e1 (discrete Gaussian,
//              sigma 3.2) from a counter-based hash (K11), write the three
//              RNS polynomials u, m + e0, e1 (coefficient form)
//            ckks_ntt_fwd        -- negacyclic Cooley-Tukey NTT per row in LDS
//              (bit-reversed psi powers, Shoup multiplications)
//            ckks_pk_combine     -- c0 = b*u + (m+e0), c1 = a*u + e1 (NTT form)
//   decrypt: ckks_dec_prep       -- m = c0 + c1*s (NTT form)
//            ckks_ntt_inv        -- Gentleman-Sande inverse NTT, times N^-1
//            ckks_crt_decode     -- Garner CRT to a centred fp64 value per
//              coefficient, / scale, special FFT back to the slots
//   secure all-reduce helpers: ckks_scale (ct *= round(w*2^30) mod q) and
//            ckks_reduce (x mod q after an int64 sum all-reduce of <= 16
//            pre-scaled ciphertexts: every residue is < 2^60, so the sum of
//            16 stays below 2^64).
// Randomness: ChaCha20 (RFC 8439, common/chacha20.h) in counter mode under a
// secret 256-bit key drawn from the OS entropy pool for every encryption:
// ciphertext c is stream (nonce c, domain "encr"), coefficient k reads block
// k, so every (c, k) samples independently.  One 64-byte block gives u
// (ternary, 64-bit uniform mod 3: bias < 2^-62) and e0 / e1 (Box-Muller of
// two 53-bit uniforms, sigma 3.2 clipped at 6 sigma).
#include "kernels/ckks.h"
#include "kernels/common.h"
// after the HIP headers: chacha20.h marks its functions __host__ __device__
#include "common/chacha20.h"

namespace mfl {
namespace {

__device__ __forceinline__ uint64_t mulsh(uint64_t a, uint64_t w, uint64_t wp, uint64_t q) {
  const uint64_t hi = __umul64hi(a, wp);
  uint64_t r = a * w - hi * q;
  return r >= q ? r - q : r;
}
__device__ __forceinline__ uint64_t addmod(uint64_t a, uint64_t b, uint64_t q) {
  const uint64_t s = a + b;
  return s >= q ? s - q : s;
}
__device__ __forceinline__ uint64_t submod(uint64_t a, uint64_t b, uint64_t q) {
  return a >= b ? a - b : a + q - b;
}
// signed int64 -> [0, q)
__device__ __forceinline__ uint64_t smod(int64_t x, uint64_t q) {
  int64_t r = x % (int64_t)q;
  return (uint64_t)(r < 0 ? r + (int64_t)q : r);
}
// K11: the noise of coefficient k of ciphertext c
__device__ __forceinline__ void sample_noise(const CkksKey& key, int64_t c, int k, int64_t& u, int64_t& e0,
                                             int64_t& e1) {
  const uint32_t nonce[3] = {(uint32_t)c, (uint32_t)((uint64_t)c >> 32), kChaEncrypt};
  uint32_t w[16];
  chacha20_block(key.w, (uint32_t)k, nonce, w);
  u = chacha_ternary(chacha_u64(w));
  const double u1 = chacha_unit_open0(chacha_u64(w + 2)), u2 = chacha_unit(chacha_u64(w + 4));
  const double r = 3.2 * sqrt(-2.0 * log(u1));
  double g0 = r * cospi(2.0 * u2), g1 = r * sinpi(2.0 * u2);
  g0 = fmin(19.2, fmax(-19.2, g0));
  g1 = fmin(19.2, fmax(-19.2, g1));
  e0 = llrint(g0);
  e1 = llrint(g1);
}
__device__ __forceinline__ int log2u(uint32_t x) { return 31 - __clz(x); }
__device__ __forceinline__ uint32_t bitrev(uint32_t x, int bits) { return __brev(x) >> (32 - bits); }

struct cplx {
  double re, im;
};
__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(512) void ckks_encode_sample_kernel(CkksTables T, const float* __restrict__ x,
                                                                 int64_t n, double delta, CkksKey key,
                                                                 uint64_t* __restrict__ ct,
                                                                 uint64_t* __restrict__ u_out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  cplx* v = reinterpret_cast<cplx*>(smem);
  const int S = T.S, N = T.N, L = T.L;
  const uint32_t M = 2u * (uint32_t)N;
  const int64_t c = blockIdx.x;
  const int64_t off = c * S;
  for (int i = threadIdx.x; i < S; i += blockDim.x)
    v[i] = {off + i < n ? (double)x[off + i] : 0.0, 0.0};
  // special inverse FFT (he/ckks.cc CKKS::encode): len = S .. 2
  for (int len = S; len >= 2; len >>= 1) {
    __syncthreads();
    const int lenh = len >> 1, lsh = log2u(lenh);
    const uint32_t lenq = (uint32_t)len << 2, gap = M / lenq;
    for (int b = threadIdx.x; b < (S >> 1); b += blockDim.x) {
      const int blk = b >> lsh, j = b & (lenh - 1);
      const int i = blk * len;
      const uint32_t idx = (lenq - (T.rot[j] & (lenq - 1))) * gap;
      const cplx a = v[i + j], bb = v[i + j + lenh];
      const cplx w = {T.ksi_re[idx], T.ksi_im[idx]};
      v[i + j] = {a.re + bb.re, a.im + bb.im};
      v[i + j + lenh] = cmul({a.re - bb.re, a.im - bb.im}, w);
    }
  }
  __syncthreads();
  const int sbits = log2u((uint32_t)S);
  const double inv_s = 1.0 / (double)S;
  uint64_t* c0 = ct + c * 2 * (int64_t)L * N;
  uint64_t* c1 = c0 + (int64_t)L * N;
  uint64_t* uo = u_out + c * (int64_t)L * N;
  for (int k = threadIdx.x; k < N; k += blockDim.x) {
    const cplx z = v[bitrev((uint32_t)(k < S ? k : k - S), sbits)];
    const double coeff = (k < S ? z.re : z.im) * inv_s;
    const int64_t m = (int64_t)round(coeff * delta);
    int64_t u, e0, e1;
    sample_noise(key, c, k, u, e0, e1);
    for (int l = 0; l < L; ++l) {
      const uint64_t q = T.q[l];
      c0[(int64_t)l * N + k] = addmod(smod(m, q), smod(e0, q), q);
      c1[(int64_t)l * N + k] = smod(e1, q);
      uo[(int64_t)l * N + k] = smod(u, q);
    }
  }
}

// rows [nrows][N], row r in limb r % L
__global__ __launch_bounds__(512) void ckks_ntt_fwd_kernel(CkksTables T, uint64_t* __restrict__ rows) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t* a = reinterpret_cast<uint64_t*>(smem);
  const int N = T.N;
  const int l = (int)(blockIdx.x % (unsigned)T.L);
  const uint64_t q = T.q[l];
  const uint64_t* W = T.psi + (int64_t)l * N;
  const uint64_t* Wp = T.psi_sh + (int64_t)l * N;
  uint64_t* g = rows + (int64_t)blockIdx.x * N;
  for (int i = threadIdx.x; i < N; i += blockDim.x) a[i] = g[i];
  int t = N;
  for (int m = 1; m < N; m <<= 1) {
    t >>= 1;
    const int tsh = log2u((uint32_t)t);
    __syncthreads();
    for (int b = threadIdx.x; b < (N >> 1); b += blockDim.x) {
      const int i = b >> tsh;
      const int j = 2 * i * t + (b & (t - 1));
      const uint64_t U = a[j];
      const uint64_t V = mulsh(a[j + t], W[m + i], Wp[m + i], q);
      a[j] = addmod(U, V, q);
      a[j + t] = submod(U, V, q);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < N; i += blockDim.x) g[i] = a[i];
}

__global__ __launch_bounds__(512) void ckks_ntt_inv_kernel(CkksTables T, uint64_t* __restrict__ rows) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint64_t* a = reinterpret_cast<uint64_t*>(smem);
  const int N = T.N;
  const int l = (int)(blockIdx.x % (unsigned)T.L);
  const uint64_t q = T.q[l];
  const uint64_t* W = T.ipsi + (int64_t)l * N;
  const uint64_t* Wp = T.ipsi_sh + (int64_t)l * N;
  uint64_t* g = rows + (int64_t)blockIdx.x * N;
  for (int i = threadIdx.x; i < N; i += blockDim.x) a[i] = g[i];
  int t = 1;
  for (int m = N; m > 1; m >>= 1) {
    const int h = m >> 1, tsh = log2u((uint32_t)t);
    __syncthreads();
    for (int b = threadIdx.x; b < (N >> 1); b += blockDim.x) {
      const int i = b >> tsh;
      const int j = 2 * i * t + (b & (t - 1));
      const uint64_t U = a[j], V = a[j + t];
      a[j] = addmod(U, V, q);
      a[j + t] = mulsh(submod(U, V, q), W[h + i], Wp[h + i], q);
    }
    t <<= 1;
  }
  __syncthreads();
  const uint64_t ni = T.ninv[l], nis = T.ninv_sh[l];
  for (int i = threadIdx.x; i < N; i += blockDim.x) g[i] = mulsh(a[i], ni, nis, q);
}

// c0 = b*u + c0, c1 = a*u + c1 over [nct][2][L][N] with u [nct][L][N]
__global__ __launch_bounds__(256) void ckks_pk_combine_kernel(CkksTables T, uint64_t* __restrict__ ct,
                                                              const uint64_t* __restrict__ u, int64_t nct) {
  const int64_t LN = (int64_t)T.L * T.N;
  const int64_t total = nct * LN;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i / LN, r = i - c * LN;
    const int l = (int)(r / T.N);
    const uint64_t q = T.q[l];
    const uint64_t uu = u[i];
    uint64_t* c0 = ct + c * 2 * LN + r;
    uint64_t* c1 = c0 + LN;
    *c0 = addmod(mulsh(uu, T.pk_b[r], T.pk_b_sh[r], q), *c0, q);
    *c1 = addmod(mulsh(uu, T.pk_a[r], T.pk_a_sh[r], q), *c1, q);
  }
}

// m[c][l][k] = c0 + c1 * s
__global__ __launch_bounds__(256) void ckks_dec_prep_kernel(CkksTables T, const uint64_t* __restrict__ ct,
                                                            uint64_t* __restrict__ m, int64_t nct) {
  const int64_t LN = (int64_t)T.L * T.N;
  const int64_t total = nct * LN;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i / LN, r = i - c * LN;
    const int l = (int)(r / T.N);
    const uint64_t q = T.q[l];
    const uint64_t* c0 = ct + c * 2 * LN + r;
    m[i] = addmod(*c0, mulsh(c0[LN], T.sk[r], T.sk_sh[r], q), q);
  }
}

// Garner mixed-radix digits -> centred fp64 (he/ckks.cc Crt::centred; the sign
// is read off the top digit, exact for |x| < Q/2 - Q/q_top)
__device__ __forceinline__ double crt_centred(const CkksTables& T, const uint64_t* res, int64_t stride) {
  uint64_t v[kCkksMaxLimbs];
  const int L = T.L;
  for (int j = 0; j < L; ++j) {
    const uint64_t qj = T.q[j];
    uint64_t t = res[(int64_t)j * stride];
    for (int i = 0; i < j; ++i) {
      const uint64_t vi = mulsh(v[i], 1, T.one_sh[j], qj);  // v_i mod q_j
      const uint64_t* g = T.garner + ((int64_t)i * kCkksMaxLimbs + j) * 2;
      t = mulsh(submod(t, vi, qj), g[0], g[1], qj);
    }
    v[j] = t;
  }
  const uint64_t qt = T.q[L - 1];
  double acc = v[L - 1] > (qt >> 1) ? -(double)(qt - v[L - 1]) : (double)v[L - 1];
  for (int j = L - 2; j >= 0; --j) acc = acc * (double)T.q[j] + (double)v[j];
  return acc;
}

__global__ __launch_bounds__(512) void ckks_crt_decode_kernel(CkksTables T, const uint64_t* __restrict__ m,
                                                              double inv_scale, float* __restrict__ out,
                                                              double* __restrict__ out64, int64_t n) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  cplx* v = reinterpret_cast<cplx*>(smem);
  const int S = T.S, N = T.N;
  const uint32_t M = 2u * (uint32_t)N;
  const int64_t c = blockIdx.x;
  const uint64_t* mc = m + c * (int64_t)T.L * N;
  const int sbits = log2u((uint32_t)S);
  for (int i = threadIdx.x; i < S; i += blockDim.x) {
    const double re = crt_centred(T, mc + i, N) * inv_scale;
    const double im = crt_centred(T, mc + i + S, N) * inv_scale;
    v[bitrev((uint32_t)i, sbits)] = {re, im};
  }
  for (int len = 2; len <= S; len <<= 1) {
    __syncthreads();
    const int lenh = len >> 1, lsh = log2u(lenh);
    const uint32_t lenq = (uint32_t)len << 2, gap = M / lenq;
    for (int b = threadIdx.x; b < (S >> 1); b += blockDim.x) {
      const int blk = b >> lsh, j = b & (lenh - 1);
      const int i = blk * len;
      const uint32_t idx = (T.rot[j] & (lenq - 1)) * gap;
      const cplx u = v[i + j];
      const cplx w = cmul(v[i + j + lenh], {T.ksi_re[idx], T.ksi_im[idx]});
      v[i + j] = {u.re + w.re, u.im + w.im};
      v[i + j + lenh] = {u.re - w.re, u.im - w.im};
    }
  }
  __syncthreads();
  const int64_t off = c * S;
  for (int i = threadIdx.x; i < S; i += blockDim.x)
    if (off + i < n) {
      if (out64) out64[off + i] = v[i].re;
      else out[off + i] = (float)v[i].re;
    }
}

// x[c][p][l][k] = x * w_l mod q_l  (w = round(weight * 2^30) mod q_l, Shoup)
__global__ __launch_bounds__(256) void ckks_scale_kernel(CkksTables T, uint64_t* __restrict__ x,
                                                         const uint64_t* __restrict__ wq, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)((i / T.N) % T.L);
    x[i] = mulsh(x[i], wq[2 * l], wq[2 * l + 1], T.q[l]);
  }
}

// x mod q_l for any x < 2^64 (Shoup with w = 1: one conditional subtraction)
__global__ __launch_bounds__(256) void ckks_reduce_kernel(CkksTables T, uint64_t* __restrict__ x, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)((i / T.N) % T.L);
    x[i] = mulsh(x[i], 1, T.one_sh[l], T.q[l]);
  }
}

}  // namespace

void launch_ckks_encrypt(const CkksTables& T, const float* x, int64_t n, int64_t nct, double delta,
                         const CkksKey& key, uint64_t* ct, uint64_t* u_scratch, hipStream_t s) {
  const size_t lds = (size_t)T.N * 8;  // S complex doubles == N u64
  ckks_encode_sample_kernel<<<(unsigned)nct, 512, lds, s>>>(T, x, n, delta, key, ct, u_scratch);
  ckks_ntt_fwd_kernel<<<(unsigned)(nct * 2 * T.L), 512, lds, s>>>(T, ct);
  ckks_ntt_fwd_kernel<<<(unsigned)(nct * T.L), 512, lds, s>>>(T, u_scratch);
  ckks_pk_combine_kernel<<<stream_grid(nct * T.L * T.N, 256, 8192), 256, 0, s>>>(T, ct, u_scratch, nct);
}

void launch_ckks_decrypt(const CkksTables& T, const uint64_t* ct, int64_t nct, double inv_scale,
                         uint64_t* m_scratch, float* out, double* out64, int64_t n, hipStream_t s) {
  const size_t lds = (size_t)T.N * 8;
  ckks_dec_prep_kernel<<<stream_grid(nct * T.L * T.N, 256, 8192), 256, 0, s>>>(T, ct, m_scratch, nct);
  ckks_ntt_inv_kernel<<<(unsigned)(nct * T.L), 512, lds, s>>>(T, m_scratch);
  ckks_crt_decode_kernel<<<(unsigned)nct, 512, lds, s>>>(T, m_scratch, inv_scale, out, out64, n);
}

void launch_ckks_ntt(const CkksTables& T, uint64_t* rows, int64_t nrows, bool inverse, hipStream_t s) {
  const size_t lds = (size_t)T.N * 8;
  if (inverse) ckks_ntt_inv_kernel<<<(unsigned)nrows, 512, lds, s>>>(T, rows);
  else ckks_ntt_fwd_kernel<<<(unsigned)nrows, 512, lds, s>>>(T, rows);
}

void launch_ckks_scale(const CkksTables& T, uint64_t* x, const uint64_t* wq, int64_t total, hipStream_t s) {
  ckks_scale_kernel<<<stream_grid(total, 256, 8192), 256, 0, s>>>(T, x, wq, total);
}

void launch_ckks_reduce(const CkksTables& T, uint64_t* x, int64_t total, hipStream_t s) {
  ckks_reduce_kernel<<<stream_grid(total, 256, 8192), 256, 0, s>>>(T, x, total);
}

namespace {
__global__ void chacha_blocks_kernel(CkksKey key, uint32_t counter0, uint32_t n0, uint32_t n1, uint32_t n2,
                                     int nblocks, uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nblocks) return;
  const uint32_t nonce[3] = {n0, n1, n2};
  uint32_t w[16];
  chacha20_block(key.w, counter0 + (uint32_t)i, nonce, w);
  for (int j = 0; j < 16; ++j) out[(int64_t)i * 16 + j] = w[j];
}
__global__ void noise_dump_kernel(CkksKey key, int64_t c, int n, int64_t* __restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  int64_t u, e0, e1;
  sample_noise(key, c, k, u, e0, e1);
  out[k] = u;
  out[n + k] = e0;
  out[2 * (int64_t)n + k] = e1;
}
}  // namespace

void launch_chacha_blocks(const CkksKey& key, uint32_t counter0, const uint32_t nonce[3], int nblocks, uint32_t* out,
                          hipStream_t s) {
  chacha_blocks_kernel<<<(nblocks + 255) / 256, 256, 0, s>>>(key, counter0, nonce[0], nonce[1], nonce[2], nblocks,
                                                             out);
}
void launch_ckks_noise_dump(const CkksKey& key, int64_t c, int n, int64_t* out, hipStream_t s) {
  noise_dump_kernel<<<(n + 255) / 256, 256, 0, s>>>(key, c, n, out);
}

}  // namespace mfl
