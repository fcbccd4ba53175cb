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
// randomness is ChaCha20 (RFC 8439, common/chacha20.h) keyed from getrandom():
// a context generator for key generation, and a fresh 256-bit key per
// encryption with one counter-mode stream per ciphertext.
#pragma once
#include <cstdint>
#include <random>
#include <string>
#include <string_view>
#include <vector>

namespace mfl {

// Host CSPRNG: ChaCha20 in counter mode.  Default-constructed: a 256-bit key
// from the kernel entropy pool (getrandom); or an explicit (key, stream,
// domain) for the per-ciphertext encryption streams.
class ChaCha20Rng {
 public:
  ChaCha20Rng();
  ChaCha20Rng(const uint32_t key[8], uint64_t stream, uint32_t domain);
  uint64_t next_u64();
  uint64_t below(uint64_t q);     // uniform in [0, q), rejection sampled
  int ternary();                  // uniform in {-1, 0, 1}
  double gauss(double sigma);     // Box-Muller
  void derive_key(uint32_t out[8]);  // 256 fresh bits for a sub-stream key
  static void os_random(void* buf, size_t n);

 private:
  void refill();
  uint32_t key_[8];
  uint32_t nonce_[3];
  uint32_t ctr_ = 0;
  uint32_t buf_[16];
  int pos_ = 16;
  bool has_spare_ = false;
  double spare_ = 0.0;
};

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

 public:
  // statistical tests of the samplers (tests/test_ckks_rng.py)
  std::vector<int64_t> debug_sample(int kind, size_t n);

 private:
  uint64_t reduce_signed(long double x, int limb) const;

  uint32_t batch_, bits_, N_, slots_;
  std::vector<uint64_t> q_;
  std::vector<std::vector<uint64_t>> psi_rev_, psi_rev_sh_, ipsi_rev_, ipsi_rev_sh_;
  std::vector<uint64_t> ninv_, ninv_sh_;
  std::vector<uint64_t> pk_b_, pk_a_, sk_;  // [limb][N] NTT form
  bool has_pk_ = false, has_sk_ = false;
  Files files_;
  ChaCha20Rng rng_;
  // canonical-embedding FFT tables
  std::vector<uint64_t> rot_;
  std::vector<double> ksi_re_, ksi_im_;
};

}  // namespace mfl
