// Device tables + launchers of the RNS-CKKS encrypt / decrypt kernels (ckks.hip).
// All pointers are device memory uploaded once per key set by
// metisfl_amd/encryption/device.py from CKKS::device_tables (he/ckks.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfl {

constexpr int kCkksMaxLimbs = 4;

struct CkksTables {
  int N, S, L;                 // ring dimension, slots (= N/2), RNS limbs (<= kCkksMaxLimbs)
  const uint64_t* q;           // [L]
  const uint64_t* one_sh;      // [L] floor(2^64 / q_l): Shoup companion of 1 (reduction)
  const uint64_t* psi;         // [L][N] bit-reversed psi powers
  const uint64_t* psi_sh;      // [L][N]
  const uint64_t* ipsi;        // [L][N] bit-reversed psi^-1 powers
  const uint64_t* ipsi_sh;     // [L][N]
  const uint64_t* ninv;        // [L] N^-1 mod q_l
  const uint64_t* ninv_sh;     // [L]
  const uint64_t* pk_b;        // [L][N] public key (NTT form) -- nullptr if not loaded
  const uint64_t* pk_b_sh;
  const uint64_t* pk_a;
  const uint64_t* pk_a_sh;
  const uint64_t* sk;          // [L][N] secret key (NTT form) -- nullptr if not loaded
  const uint64_t* sk_sh;
  const uint64_t* garner;      // [kCkksMaxLimbs][kCkksMaxLimbs][2] q_i^-1 mod q_j, Shoup
  const uint32_t* rot;         // [S] 5^j mod 2N
  const double* ksi_re;        // [2N + 1] cos(2 pi k / 2N)
  const double* ksi_im;        // [2N + 1] sin(2 pi k / 2N)
};

// 256-bit ChaCha20 key of one encryption (secret; fresh per call)
struct CkksKey {
  uint32_t w[8];
};

// x: fp32 [n] -> ct: u64 [nct][2][L][N] (nct = ceil(n / S)); u_scratch: u64 [nct][L][N]
void launch_ckks_encrypt(const CkksTables& T, const float* x, int64_t n, int64_t nct, double delta,
                         const CkksKey& key, uint64_t* ct, uint64_t* u_scratch, hipStream_t s);
// tests: RFC 8439 blocks counter0.. on the device; the (u, e0, e1) noise of
// ciphertext c's first n coefficients -> out [3][n]
void launch_chacha_blocks(const CkksKey& key, uint32_t counter0, const uint32_t nonce[3], int nblocks, uint32_t* out,
                          hipStream_t s);
void launch_ckks_noise_dump(const CkksKey& key, int64_t c, int n, int64_t* out, hipStream_t s);
// ct [nct][2][L][N] -> out fp32 [n] (or fp64 into out64 when non-null); m_scratch: u64 [nct][L][N]
void launch_ckks_decrypt(const CkksTables& T, const uint64_t* ct, int64_t nct, double inv_scale,
                         uint64_t* m_scratch, float* out, double* out64, int64_t n, hipStream_t s);
// in-place NTT of nrows rows (row r in limb r % L)
void launch_ckks_ntt(const CkksTables& T, uint64_t* rows, int64_t nrows, bool inverse, hipStream_t s);
// x[.][.][l][.] *= w_l (mod q_l); wq [L][2] = {w_l, shoup(w_l)}
void launch_ckks_scale(const CkksTables& T, uint64_t* x, const uint64_t* wq, int64_t total, hipStream_t s);
// x mod q_l, for the int64 sum all-reduce of pre-scaled ciphertexts
void launch_ckks_reduce(const CkksTables& T, uint64_t* x, int64_t total, hipStream_t s);

}  // namespace mfl
