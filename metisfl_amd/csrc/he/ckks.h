// RNS-CKKS approximate homomorphic encryption for private weighted averaging.
//
// Replaces the Palisade-backed CKKS of the reference
// (metisfl/encryption/palisade/ckks_scheme.{h,cc}, he_scheme.h:20-43), which is
// not available here.  Scope = what federated PWA needs:
//   keygen -> encode/encrypt (learners) -> sum_i w_i * ct_i (controller,
//   plaintext-scalar weights, no ct x ct multiplication) -> decrypt/decode.
//
// Parameters: ring dimension N = 2 * batch_size (batch_size slots), three NTT
// primes q_j = 1 (mod 2N): one 60-bit base prime and two `scaling_bits`-bit
// primes (the reference's multDepth = 2 chain); Delta = 2^scaling_bits.
// Weighted averaging multiplies by round(w * 2^30) per limb and raises the
// ciphertext scale to Delta * 2^30 -- no rescaling, so PWA is a pure
// element-wise modular FMA (the HIP kernel K9, kernels/aggregate.hip, runs the
// same arithmetic on device).  Ciphertexts are stored in NTT form.
//
// Serialized ciphertext (own format; Palisade's is not reproducible):
//   "MCK1" | u32 N | u32 nlimbs | u32 nct | f64 log2(scale) | u64 moduli[nlimbs]
//   | nct x { c0[nlimbs][N], c1[nlimbs][N] }  (u64, little endian)
// Security note: secrets are ternary, errors discrete Gaussian (sigma 3.2),
// log2(Q) ~ 60 + 2*scaling_bits <= 218 at N = 8192 (128-bit HE-standard bound);
// randomness comes from std::random_device-seeded mt19937_64 (not a CSPRNG).
#pragma once
#include <cstdint>
#include <random>
#include <string>
#include <string_view>
#include <vector>

namespace mfl {

class CKKS {
 public:
  CKKS(uint32_t batch_size, uint32_t scaling_bits);

  // Files: <dir>/cryptocontext.txt, key-public.txt, key-private.txt, key-eval-mult.txt
  void gen_crypto_context_and_keys(const std::string& dir);
  struct Files {
    std::string crypto_context_file, public_key_file, private_key_file, eval_mult_key_file;
  };
  Files files() const { return files_; }
  void load_context(const std::string& file);
  void load_public_key(const std::string& file);
  void load_private_key(const std::string& file);
  void load_context_and_keys(const std::string& ctx, const std::string& pk, const std::string& sk);

  std::string encrypt(const std::vector<double>& values);
  std::string weighted_average(const std::vector<std::string_view>& cts,
                               const std::vector<double>& weights) const;
  std::vector<double> decrypt(std::string_view ct, size_t n) const;

  // Encoding without encryption (tests): coefficient vector of one chunk.
  std::vector<double> encode_decode_roundtrip(const std::vector<double>& v) const;

  uint32_t ring_dim() const { return N_; }
  uint32_t slots() const { return slots_; }
  const std::vector<uint64_t>& moduli() const { return q_; }
  static constexpr int kWeightBits = 30;

  // Read-only views for the device (HIP) encrypt / decrypt path
  // (kernels/ckks.hip): NTT twiddles in bit-reversed order with their Shoup
  // companions, N^-1, keys in NTT form [limb][N], canonical-embedding tables.
  bool has_public_key() const { return has_pk_; }
  bool has_private_key() const { return has_sk_; }
  uint32_t scaling_bits() const { return bits_; }
  const std::vector<std::vector<uint64_t>>& psi_rev() const { return psi_rev_; }
  const std::vector<std::vector<uint64_t>>& psi_rev_shoup() const { return psi_rev_sh_; }
  const std::vector<std::vector<uint64_t>>& ipsi_rev() const { return ipsi_rev_; }
  const std::vector<std::vector<uint64_t>>& ipsi_rev_shoup() const { return ipsi_rev_sh_; }
  const std::vector<uint64_t>& n_inv() const { return ninv_; }
  const std::vector<uint64_t>& n_inv_shoup() const { return ninv_sh_; }
  const std::vector<uint64_t>& pk_b() const { return pk_b_; }
  const std::vector<uint64_t>& pk_a() const { return pk_a_; }
  const std::vector<uint64_t>& sk() const { return sk_; }
  const std::vector<uint64_t>& rot() const { return rot_; }
  const std::vector<double>& ksi_re() const { return ksi_re_; }
  const std::vector<double>& ksi_im() const { return ksi_im_; }

 private:
  void setup_primes();
  void precompute();
  void ntt(uint64_t* a, int limb) const;
  void intt(uint64_t* a, int limb) const;
  void encode(const double* z, size_t n, std::vector<double>& coeffs) const;
  void decode(const std::vector<long double>& coeffs, double scale, double* out, size_t n) const;
  void sample_ternary(std::vector<int64_t>& v);
  void sample_gauss(std::vector<int64_t>& v);
  uint64_t reduce_signed(long double x, int limb) const;

  uint32_t batch_, bits_, N_, slots_;
  std::vector<uint64_t> q_;
  std::vector<std::vector<uint64_t>> psi_rev_, psi_rev_sh_, ipsi_rev_, ipsi_rev_sh_;
  std::vector<uint64_t> ninv_, ninv_sh_;
  std::vector<uint64_t> pk_b_, pk_a_, sk_;  // [limb][N] NTT form
  bool has_pk_ = false, has_sk_ = false;
  Files files_;
  std::mt19937_64 rng_;
  // canonical-embedding FFT tables
  std::vector<uint64_t> rot_;
  std::vector<double> ksi_re_, ksi_im_;
};

}  // namespace mfl
